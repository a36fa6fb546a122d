# oracle/ref.mk -- build the REAL reference scorer from /root/reference sources.
#
# TEST INFRASTRUCTURE ONLY (see oracle/README.md).  Nothing here is shipped or
# measured as the product.  Outputs go to oracle/_ref/ only (git-ignored; the
# binaries travel to the GPU box like our own .so files).  Sources are read in
# place under $(REF); the vendored samtools 0.1.6 tarball is unpacked into a
# scratch directory OUTSIDE the repository ($(SCRATCH)), so no reference source
# ever lands in the repo or in a gpurun snapshot.
#
# We do not run the reference's own build system (CMake / samtools Makefile):
# the handful of translation units the scorer needs are compiled directly.
#
#   make -f oracle/ref.mk            # -> oracle/_ref/bam-somaticsniper, oracle/_ref/ref_harness

REF      ?= /root/reference
SCRATCH  ?= /tmp/ss_ref_build
OUT      ?= $(CURDIR)/oracle/_ref
CC       ?= gcc
# Same flags as the reference Release build (cmake/ProjectHelper: -O3 -DNDEBUG),
# contraction pinned off so libm/x87 table building is reproducible.
CFLAGS   := -O3 -DNDEBUG -ffp-contract=off -w
SAMDIR   := $(SCRATCH)/samtools-0.1.6
SNIPER   := $(REF)/src/lib/sniper
# samtools objects the scorer + CLI need (bam_pileup.c is deliberately absent:
# sniper_pileup.c provides the bam_plbuf_* symbols).
SAMSRC   := bgzf.c kstring.c bam_aux.c bam.c bam_import.c sam.c bam_index.c \
            faidx.c razf.c knetfile.c glf.c
SNIPSRC  := sniper_maqcns.c somatic_sniper.c allele_util.c dqstats.c \
            output_format.c output_classic.c output_vcf.c output_bed.c sniper_pileup.c
HARNESS  := $(CURDIR)/oracle/ref_harness.c
SYNTH    := $(CURDIR)/somatic-sniper_amd/csrc/ss_synth.c

all: $(OUT)/bam-somaticsniper $(OUT)/ref_harness $(OUT)/bam-somaticsniper-dump

$(SAMDIR)/.unpacked: $(REF)/vendor/samtools-0.1.6.tar.gz
	mkdir -p $(SCRATCH)
	tar xzf $< -C $(SCRATCH)
	touch $@

$(SCRATCH)/libbam.a: $(SAMDIR)/.unpacked
	cd $(SAMDIR) && for f in $(SAMSRC); do \
	  $(CC) $(CFLAGS) -D_FILE_OFFSET_BITS=64 -D_USE_KNETFILE -c $$f -o $${f%.c}.o || exit 1; done
	cd $(SAMDIR) && ar cr $@ $(SAMSRC:.c=.o)

$(SCRATCH)/ver/version.h: $(REF)/version/version.h.in
	mkdir -p $(SCRATCH)/ver
	sed 's/@FULL_VERSION@/oracle/;s/@COMMIT_HASH@/ref/;s/@CMAKE_BUILD_TYPE@//' $< > $@

INC := -I$(SAMDIR) -I$(REF)/src/lib -I$(SNIPER) -I$(SCRATCH)/ver

$(OUT)/bam-somaticsniper: $(SCRATCH)/libbam.a $(SCRATCH)/ver/version.h
	mkdir -p $(OUT)
	$(CC) $(CFLAGS) $(INC) -o $@ $(REF)/src/exe/bam-somaticsniper/main.c \
	  $(addprefix $(SNIPER)/,$(SNIPSRC)) $(SCRATCH)/libbam.a -lz -lm

$(OUT)/ref_harness: $(SCRATCH)/libbam.a $(HARNESS) $(SYNTH)
	mkdir -p $(OUT)
	$(CC) $(CFLAGS) $(INC) -I$(CURDIR)/somatic-sniper_amd/csrc -I$(CURDIR)/include \
	  -o $@ $(HARNESS) $(SYNTH) $(addprefix $(SNIPER)/,$(SNIPSRC)) $(SCRATCH)/libbam.a -lz -lm

# the reference CLI with a glf_somatic wrapper that dumps every site it is
# handed (pileup parity test of the native CLI, tests/test_cli_native.py)
$(OUT)/bam-somaticsniper-dump: $(SCRATCH)/libbam.a $(SCRATCH)/ver/version.h $(CURDIR)/oracle/pileup_dump_shim.c
	mkdir -p $(OUT)/dumpobj
	$(CC) $(CFLAGS) $(INC) -c $(REF)/src/exe/bam-somaticsniper/main.c -o $(OUT)/dumpobj/main.o
	$(CC) $(CFLAGS) $(INC) -I$(CURDIR)/include -c $(CURDIR)/oracle/pileup_dump_shim.c -o $(OUT)/dumpobj/shim.o
	$(CC) $(CFLAGS) $(INC) -o $@ $(OUT)/dumpobj/main.o $(OUT)/dumpobj/shim.o \
	  $(addprefix $(SNIPER)/,$(SNIPSRC)) $(SCRATCH)/libbam.a -Wl,--wrap=glf_somatic -lz -lm

clean:
	rm -rf $(OUT)

.PHONY: all clean
