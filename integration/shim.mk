# integration/shim.mk -- link the reference's own bam-somaticsniper sources
# (compiled in place from /root/reference, never copied) with the batching
# shim glf_somatic_shim.c and libsniper_amd.so: the drop-in a maintainer of
# the reference would build.  Output: integration/_build/bam-somaticsniper-amd
# (git-ignored; travels to the GPU box).  Needs /root/reference, so it is
# built in the build container by __graft_entry__.build().
#
#   make -f integration/shim.mk

REF      ?= /root/reference
SCRATCH  ?= /tmp/ss_ref_build
OUT      ?= $(CURDIR)/integration/_build
CC       ?= gcc
CFLAGS   := -O3 -DNDEBUG -ffp-contract=off -w
SAMDIR   := $(SCRATCH)/samtools-0.1.6
SNIPER   := $(REF)/src/lib/sniper
SNIPSRC  := sniper_maqcns.c somatic_sniper.c allele_util.c dqstats.c \
            output_format.c output_classic.c output_vcf.c output_bed.c sniper_pileup.c
INC      := -I$(SAMDIR) -I$(REF)/src/lib -I$(SNIPER) -I$(SCRATCH)/ver -I$(CURDIR)/include
LIBDIR   := $(CURDIR)/somatic-sniper_amd
WRAP     := -Wl,--wrap=glf_somatic -Wl,--wrap=bam_sspileup_file -Wl,--wrap=makeSoloPrior

all: $(OUT)/bam-somaticsniper-amd

$(SCRATCH)/libbam.a $(SCRATCH)/ver/version.h:
	$(MAKE) -f $(CURDIR)/oracle/ref.mk $@

$(OUT)/bam-somaticsniper-amd: $(CURDIR)/integration/glf_somatic_shim.c $(SCRATCH)/libbam.a \
                              $(SCRATCH)/ver/version.h $(LIBDIR)/libsniper_amd.so
	mkdir -p $(OUT)/obj
	$(CC) $(CFLAGS) $(INC) -c $(REF)/src/exe/bam-somaticsniper/main.c -o $(OUT)/obj/main.o
	for f in $(SNIPSRC); do $(CC) $(CFLAGS) $(INC) -c $(SNIPER)/$$f -o $(OUT)/obj/$${f%.c}.o || exit 1; done
	$(CC) $(CFLAGS) -Wall $(INC) -c $(CURDIR)/integration/glf_somatic_shim.c -o $(OUT)/obj/shim.o
	$(CC) -o $@ $(OUT)/obj/main.o $(addprefix $(OUT)/obj/,$(SNIPSRC:.c=.o)) $(OUT)/obj/shim.o \
	  $(SCRATCH)/libbam.a $(WRAP) -L$(LIBDIR) -lsniper_amd -Wl,-rpath,'$$ORIGIN/../../somatic-sniper_amd' \
	  -lz -lm

clean:
	rm -rf $(OUT)

.PHONY: all clean
