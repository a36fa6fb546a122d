#!/usr/bin/env python3
"""Vectorised synthetic tumor/normal BAM pair for end-to-end CLI timing.

Fixed-length reads (100M, fixed-width names) let numpy assemble every BAM
record at once.  Coverage is Poisson along one or more contigs; bases follow
the reference except for a 1% error rate and germline / somatic sites.
    python tools/bamsim.py OUTDIR --length 5000000 --depth-t 60 --depth-n 30
"""
import argparse
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from bamgen import bgzf_blocks, reg2bin, write_fasta  # noqa: E402

CODE = {"A": 1, "C": 2, "G": 4, "T": 8}


def make_bam(path, contigs, refs, depth, rng, seed_tag, read_len=100, vaf_tab=None):
    recs = []
    for ci, (name, seq) in enumerate(contigs):
        print(f"[bamsim] {os.path.basename(path)}: contig {ci + 1}/{len(contigs)}", file=sys.stderr, flush=True)
        L = len(seq)
        n = int(L * depth / read_len)
        pos = np.sort(rng.integers(0, max(1, L - read_len), n)).astype(np.int32)
        idx = pos[:, None] + np.arange(read_len)[None, :]
        bases = refs[ci][idx].copy()                                  # nt16 codes
        if vaf_tab is not None:
            vsite, valt, vfrac = vaf_tab[ci]
            hit = np.isin(idx, vsite)
            if hit.any():
                sel = np.searchsorted(vsite, idx[hit])
                take = rng.random(hit.sum()) < vfrac[sel]
                b = bases[hit]
                b[take] = valt[sel][take]
                bases[hit] = b
        err = rng.random(bases.shape) < 0.01
        bases[err] = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, err.sum())]
        qual = rng.integers(2, 42, bases.shape).astype(np.uint8)
        mapq = np.where(rng.random(n) < 0.9, 60, rng.integers(0, 61, n)).astype(np.uint32)
        flag = np.where(rng.random(n) < 0.5, 16, 0).astype(np.uint32)
        l_name = 12                                                   # "t%010d\0"
        block = 32 + l_name + 4 + read_len // 2 + read_len
        rec = np.zeros((n, 4 + block), np.uint8)
        hdr = np.zeros((n, 9), np.int32)
        hdr[:, 0] = block
        hdr[:, 1] = ci
        hdr[:, 2] = pos
        bins = np.array([reg2bin(int(p), int(p) + read_len) for p in pos[:: max(1, n // 4096)]], np.int64)
        binv = np.vectorize(lambda p: reg2bin(int(p), int(p) + read_len))(pos) if n < 200000 else \
            (4681 + (pos >> 14)).astype(np.int64)
        del bins
        hdr[:, 3] = ((binv << 16) | (mapq << 8) | l_name).astype(np.int64).astype(np.int32)
        hdr[:, 4] = ((flag << 16) | 1).astype(np.int64).astype(np.int32)
        hdr[:, 5] = read_len
        hdr[:, 6] = -1
        hdr[:, 7] = -1
        hdr[:, 8] = 0
        rec[:, :36] = hdr.view(np.uint8).reshape(n, 36)
        names = np.char.add(seed_tag, np.char.zfill(np.arange(n).astype(str), 10))
        rec[:, 36:36 + 11] = np.frombuffer("".join(names).encode(), np.uint8).reshape(n, 11)
        o = 36 + l_name
        rec[:, o:o + 4] = np.frombuffer(np.uint32(read_len << 4).tobytes(), np.uint8)
        o += 4
        rec[:, o:o + read_len // 2] = (bases[:, 0::2] << 4) | bases[:, 1::2]
        o += read_len // 2
        rec[:, o:o + read_len] = qual
        recs.append(rec.reshape(-1))
    text = "@HD\tVN:1.0\tSO:coordinate\n" + "".join(f"@SQ\tSN:{n}\tLN:{len(s)}\n" for n, s in contigs)
    h = b"BAM\1" + np.int32(len(text)).tobytes() + text.encode() + np.int32(len(contigs)).tobytes()
    for n, s in contigs:
        nb = n.encode() + b"\0"
        h += np.int32(len(nb)).tobytes() + nb + np.int32(len(s)).tobytes()
    data = h + b"".join(r.tobytes() for r in recs)
    with open(path, "wb") as f:
        f.write(bgzf_blocks(data))
    return sum(len(r) for r in recs) // (recs[0].size // max(1, 1)) if recs else 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("outdir")
    ap.add_argument("--length", type=int, default=2_000_000)
    ap.add_argument("--contigs", type=int, default=2)
    ap.add_argument("--depth-t", type=float, default=60)
    ap.add_argument("--depth-n", type=float, default=30)
    ap.add_argument("--seed", type=int, default=5)
    a = ap.parse_args()
    os.makedirs(a.outdir, exist_ok=True)
    rng = np.random.default_rng(a.seed)
    contigs, refs, vt, vn = [], [], [], []
    per = a.length // a.contigs
    for c in range(a.contigs):
        r = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, per)]
        refs.append(r)
        contigs.append((f"chr{c + 1}", "".join("ACGT"[int(x).bit_length() - 1] for x in r[:0]) or None))
        s = np.array(list("ACGT"))[np.log2(r).astype(int)]
        contigs[-1] = (f"chr{c + 1}", "".join(s.tolist()))
        nv = per // 1000
        site = np.sort(rng.choice(per, nv, replace=False))
        alt = np.array([1, 2, 4, 8], np.uint8)[rng.integers(0, 4, nv)]
        som = rng.random(nv) < 0.3
        vt.append((site, alt, np.where(som, 0.4, 0.5)))
        vn.append((site, alt, np.where(som, 0.0, 0.5)))
    write_fasta(os.path.join(a.outdir, "ref.fa"), contigs)
    make_bam(os.path.join(a.outdir, "tumor.bam"), contigs, refs, a.depth_t, rng, "t", vaf_tab=vt)
    make_bam(os.path.join(a.outdir, "normal.bam"), contigs, refs, a.depth_n, rng, "n", vaf_tab=vn)
    print(f"{a.outdir}: {a.length} bp, {a.contigs} contigs, depth {a.depth_t}/{a.depth_n}")


if __name__ == "__main__":
    main()
