"""Synthetic tumor/normal BAM pairs + FASTA for end-to-end CLI tests.

Writes BAM (BGZF-compressed, coordinate-sorted, SAM spec v1) directly with
zlib: no samtools needed.  The reads exercise what the pileup walker and the
scorer care about: deletions, insertions, soft clips,
reference skips (BAM_CREF_SKIP), reverse strand, duplicate / QC-fail flags
(masked by BAM_DEF_MASK), mapQ 0..60 and 255, baseQ 0..93, '=' / N / IUPAC
read bases, lowercase and N reference bases, reads running past the contig
end, several contigs (first-read-drop quirk), a contig covered in one BAM only,
germline and somatic variants.
"""
import gzip
import struct
import zlib

import numpy as np

SEQ_CODES = "=ACMGRSVTWYHKDBN"
CIGAR_OPS = "MIDNSHP=X"


def reg2bin(beg, end):
    end -= 1
    if beg >> 14 == end >> 14:
        return ((1 << 15) - 1) // 7 + (beg >> 14)
    if beg >> 17 == end >> 17:
        return ((1 << 12) - 1) // 7 + (beg >> 17)
    if beg >> 20 == end >> 20:
        return ((1 << 9) - 1) // 7 + (beg >> 20)
    if beg >> 23 == end >> 23:
        return ((1 << 6) - 1) // 7 + (beg >> 23)
    if beg >> 26 == end >> 26:
        return ((1 << 3) - 1) // 7 + (beg >> 26)
    return 0


def bgzf_blocks(data: bytes):
    out = bytearray()
    for i in range(0, len(data), 0xff00):
        chunk = data[i:i + 0xff00]
        c = zlib.compressobj(6, zlib.DEFLATED, -15)
        comp = c.compress(chunk) + c.flush()
        bsize = 18 + len(comp) + 8 - 1
        out += struct.pack("<4BI2BH2BHH", 0x1f, 0x8b, 8, 4, 0, 0, 0xff, 6, ord("B"), ord("C"), 2, bsize)
        out += comp
        out += struct.pack("<II", zlib.crc32(chunk) & 0xffffffff, len(chunk))
    # EOF marker block
    out += bytes.fromhex("1f8b08040000000000ff0600424302001b0003000000000000000000")
    return bytes(out)


def encode_record(tid, pos, name, mapq, flag, cigar, seq, qual):
    """cigar: list of (op_char, len); seq: str over SEQ_CODES; qual: list of ints."""
    ref_len = sum(n for op, n in cigar if op in "MDN")
    bin_ = reg2bin(pos, pos + max(ref_len, 1))
    nm = name.encode() + b"\0"
    cig = b"".join(struct.pack("<I", n << 4 | CIGAR_OPS.index(op)) for op, n in cigar)
    codes = [SEQ_CODES.index(c) for c in seq]
    if len(codes) % 2:
        codes.append(0)
    packed = bytes((codes[i] << 4) | codes[i + 1] for i in range(0, len(codes), 2))
    body = struct.pack("<iiIIiiii", tid, pos, bin_ << 16 | mapq << 8 | len(nm),
                       flag << 16 | len(cigar), len(seq), -1, -1, 0)
    body += nm + cig + packed + bytes(qual)
    return struct.pack("<i", len(body)) + body


def write_bam(path, contigs, records, disorder=None):
    text = "@HD\tVN:1.0\tSO:coordinate\n" + "".join(
        f"@SQ\tSN:{n}\tLN:{len(s)}\n" for n, s in contigs)
    hdr = b"BAM\1" + struct.pack("<i", len(text)) + text.encode() + struct.pack("<i", len(contigs))
    for n, s in contigs:
        nb = n.encode() + b"\0"
        hdr += struct.pack("<i", len(nb)) + nb + struct.pack("<i", len(s))
    recs = sorted(records, key=lambda r: (r[0] if r[0] >= 0 else 1 << 30, r[1]))   # unmapped (tid -1) last
    if disorder is not None:
        # positions out of order within a contig (the reference checks only the
        # contig order): some records move a few places back in the file
        for i in disorder.choice(len(recs), max(1, len(recs) // 40), replace=False):
            j = max(0, int(i) - int(disorder.integers(1, 12)))
            if recs[j][0] == recs[i][0]:
                recs.insert(j, recs.pop(int(i)))
    data = hdr + b"".join(encode_record(*r) for r in recs)
    with open(path, "wb") as f:
        f.write(bgzf_blocks(data))


def write_fasta(path, contigs, width=60):
    with open(path, "w") as f:
        for n, s in contigs:
            f.write(f">{n}\n")
            for i in range(0, len(s), width):
                f.write(s[i:i + width] + "\n")


def make_pair(outdir, seed=1, lengths=(3000, 2200, 1500, 800), depth_t=30, depth_n=24,
              read_len=(40, 100), exotic=True, names=None, empty_normal=False, unmapped=False,
              odd_cigars=False, unsorted=False):
    """Returns paths (fasta, tumor_bam, normal_bam).

    names: contig names (default chr1..); the reference looks them up in the
    FASTA index with fai_fetch's region parser, so ':' and ',' in a name
    matter.  empty_normal: a normal BAM with a header and no reads.
    unmapped: add flag-0x4 reads, placed next to a mate and at the tail
    (tid -1), to both samples.  odd_cigars: also reads with no reference
    span (all soft clip / insertion), leading deletions, H and P ops, '=' / 'X'
    ops (samtools 0.1.6 moves neither coordinate for them) and long reference
    skips.  unsorted: positions out of order within a contig."""
    rng = np.random.default_rng(seed)
    contigs = []
    for ci, L in enumerate(lengths):
        s = list(rng.choice(list("ACGT"), L))
        if exotic:
            for i in rng.choice(L, max(1, L // 200), replace=False):
                s[i] = "N"
            lo = int(rng.integers(0, L - 50))
            for i in range(lo, lo + 40):          # a soft-masked stretch
                s[i] = s[i].lower()
            for i in rng.choice(L, 3, replace=False):
                s[i] = str(rng.choice(list("MRWSYKn")))
        contigs.append((names[ci] if names else f"chr{ci + 1}", "".join(s)))
    # variants: germline (both samples) and somatic (tumor only)
    variants = {}
    for ci, (_, s) in enumerate(contigs):
        for i in rng.choice(len(s), max(2, len(s) // 150), replace=False):
            alt = str(rng.choice([b for b in "ACGT" if b != s[i].upper()]))
            variants[(ci, int(i))] = (alt, "germ" if rng.random() < 0.4 else "som")

    def reads_for(sample, depth):
        recs = []
        skip_contig = 2 if sample == "n" else None   # contig covered by the tumor only
        k = 0
        for ci, (_, s) in enumerate(contigs):
            if ci == skip_contig:
                continue
            L = len(s)
            mean_len = (read_len[0] + read_len[1]) / 2
            nreads = int(L * depth / mean_len)
            starts = np.sort(rng.integers(-20, L - 10, nreads))
            for st in starts:
                st = int(max(0, st))
                rl = int(rng.integers(read_len[0], read_len[1] + 1))
                cigar, qpos_ref = [], []
                # build a cigar
                r = rng.random()
                if exotic and r < 0.06:
                    a = int(rng.integers(5, rl - 5)); d = int(rng.integers(1, 4))
                    cigar = [("M", a), ("D", d), ("M", rl - a)]
                elif exotic and r < 0.10:
                    a = int(rng.integers(5, rl - 8)); ins = int(rng.integers(1, 4))
                    cigar = [("M", a), ("I", ins), ("M", rl - a - ins)]
                elif exotic and r < 0.13:
                    sc = int(rng.integers(1, 8))
                    cigar = [("S", sc), ("M", rl - sc)]
                elif exotic and r < 0.15:
                    a = int(rng.integers(5, rl - 5)); gap = int(rng.integers(5, 40))
                    cigar = [("M", a), ("N", gap), ("M", rl - a)]
                elif odd_cigars and r < 0.25:
                    a = int(rng.integers(5, rl - 10)); b = int(rng.integers(1, 5))
                    cigar = [[("S", rl)], [("I", 3), ("S", rl - 3)], [("D", 3), ("M", rl)],
                             [("H", 5), ("M", a), ("P", 2), ("I", b), ("M", rl - a - b), ("H", 4)],
                             [("M", a), ("=", b), ("M", rl - a - b)], [("M", a), ("X", b), ("D", 2), ("M", rl - a - b)],
                             [("S", 4), ("M", a), ("N", 300), ("M", rl - a - 4)],
                             [("M", a), ("D", 2), ("N", 7), ("I", b), ("M", rl - a - b)]][int(rng.integers(0, 8))]
                else:
                    cigar = [("M", rl)]
                # read bases following the cigar
                seq = []
                rp = st
                for op, n in cigar:
                    if op == "M":
                        for _ in range(n):
                            rb = s[rp].upper() if rp < L else "A"
                            b = rb if rb in "ACGT" else str(rng.choice(list("ACGT")))
                            v = variants.get((ci, rp))
                            if v and (v[1] == "germ" and rng.random() < 0.5 or
                                      v[1] == "som" and sample == "t" and rng.random() < 0.4):
                                b = v[0]
                            x = rng.random()
                            if x < 0.01:
                                b = str(rng.choice(list("ACGT")))
                            elif exotic and x < 0.013:
                                b = "N"
                            elif exotic and x < 0.015:
                                b = "="
                            elif exotic and x < 0.017:
                                b = str(rng.choice(list("MRWSYKVHDB")))
                            seq.append(b)
                            rp += 1
                    elif op in "IS=X":
                        seq += list(rng.choice(list("ACGT"), n))
                    elif op in "DN":
                        rp += n
                q = rng.integers(2, 42, len(seq))
                if exotic:
                    m = rng.random(len(seq))
                    q[m < 0.02] = 0
                    q[(m >= 0.02) & (m < 0.04)] = 1
                    q[(m >= 0.04) & (m < 0.05)] = rng.integers(64, 94, int(((m >= 0.04) & (m < 0.05)).sum()))
                mq = 60 if rng.random() < 0.85 else int(rng.integers(0, 61))
                if exotic and rng.random() < 0.01:
                    mq = 255
                flag = 0x10 if rng.random() < 0.5 else 0
                if exotic and rng.random() < 0.02:
                    flag |= 0x400
                if exotic and rng.random() < 0.01:
                    flag |= 0x200
                recs.append((ci, st, f"{sample}{k}", mq, flag, cigar, "".join(seq), [int(x) for x in q]))
                k += 1
                if unmapped and rng.random() < 0.03:       # unmapped mate placed at this read
                    useq = "".join(rng.choice(list("ACGT"), 50))
                    recs.append((ci, st, f"{sample}{k}u", 0, 0x4 | 0x1, [], useq, [30] * 50))
                    k += 1
        if unmapped:
            for j in range(25):
                useq = "".join(rng.choice(list("ACGTN"), 60))
                recs.append((-1, -1, f"{sample}un{j}", 0, 0x4, [], useq, [20] * 60))
        return recs

    import os
    fa = os.path.join(outdir, "ref.fa")
    tb = os.path.join(outdir, "tumor.bam")
    nb = os.path.join(outdir, "normal.bam")
    write_fasta(fa, contigs)
    write_bam(tb, contigs, reads_for("t", depth_t), rng if unsorted else None)
    write_bam(nb, contigs, [] if empty_normal else reads_for("n", depth_n), rng if unsorted else None)
    return fa, tb, nb


if __name__ == "__main__":
    import sys
    print(make_pair(sys.argv[1] if len(sys.argv) > 1 else "."))
