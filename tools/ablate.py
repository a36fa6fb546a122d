#!/usr/bin/env python3
"""Out-of-tree timing ablations of the main kernel (never shipped).

Writes a copy of somatic-sniper_amd/csrc/ss_kernels.hip with the named phases
of ss_score_main replaced by cheap stand-ins, for `make variant` and
tools/ab.sh; the scores of such a build are meaningless (ab.sh with
AB_NOPARITY=1).  The shipped source carries no switches for this.

  python tools/ablate.py OUT.hip nonet norec nofold nofin nodecide
  make -C somatic-sniper_amd variant V=abl KSRC=build/exp_abl.hip

Phases (round 3's SS_AB_* switches):
  nonet     no bitonic network (keys stay unsorted)
  norec     no fold records written to LDS
  nofold    no ordered fold (es / fs from the group counts)
  nofin     no likelihoods / glf2cns (fields from the fold sums)
  nodecide  no site decision (score = tumor cns word)
  nominor   only the largest base group's chain per sample (the other three skipped)
            (the kernel's own round-5 early exit is left in: it runs only without glf and
            only in shallow batches, so a 60x/30x timing run never takes it)
  noload    reads synthesised in registers instead of loaded (key build without memory)
  fdep      the long chains' float accumulations split in two interleaved chains (odd / even
            records, summed at the end of each 4-record step): half the serial f64 depth,
            the same instructions plus two adds -- how much the fold waits on its own latency
and of ss_score_group (the C5 path):
  gnosort   no in-lane network (ln_levels)
  gnomerge  no cross-lane merge levels (gp_level)
  gnorec    no fold records written to the arena
  gnofold   no ordered fold in finish_sub (sums from the counts)
  gnofin    no likelihoods in finish_sub (p from the sums)
  gfdep     fdep for finish_sub's chains
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "somatic-sniper_amd", "csrc", "ss_kernels.hip")

EDITS = {
    "nonet": [("        ln_levels<LN_R, 2>(v);\n        ln_records(", "        ln_records(")],
    "norec": [("        ln_records(v, 4u * nch, L, lane);\n", "")],
    "nofold": [("            ln_fold(L, lane, k ? tot_a : 0u, k ? acc.cnt_b : acc.cnt_a, fk, es, fs, c);\n",
                "            for (int b = 0; b < 4; ++b) { es[b] = fs[b] = (float)(acc.cnt_a >> b); "
                "c[b] = (acc.cnt_a >> (8 * b)) & 0xffu; }\n")],
    "nofin": [("            ln_finish(es, fs, c, smpN ? nn : nt, k ? acc.rms_b : acc.rms_a, a.m, l03, l47, l89, cn, mq);\n",
               "            l03 = __float_as_uint(es[0]); l47 = __float_as_uint(fs[1]); l89 = c[2]; "
               "cn = 0x11000000u; mq = c[3];\n")],
    "nodecide": [("    if (ok) decide_site(kernarg_args(), qtab, s, refc | ref16 << 8, L.res[lane][0], L.res[lane][1]);\n",
                  "    if (ok) a.score[s] = (int)L.res[lane][0].cns;\n")],
    "nominor": [("    if (!__ballot(max(max(no[0], no[1]), no[2]) > 6u)) {\n",
                 "    if (true) {\n        es[0] = es[1] = es[2] = es[3] = e; fs[0] = fs[1] = fs[2] = fs[3] = f;\n        return;\n"),
                ("        ln_chain(L, lane, st[b], isbig ? 0u : c[b], fk, eb, fb);\n",
                 "        eb = fb = 0.0f;\n")],
    "noload": [("    if (in.tail) {                   /* wave-uniform: word loads, none past the lane's reads */\n",
                "    if (true) {\n#pragma unroll\n        for (int t = 0; t < 4; ++t) "
                "x[t] = ((in.na + 4u * c + (uint32_t)t) * 0x9E3779B1u) & 0x001f3f3fu;\n        return;\n    }\n"
                "    if (in.tail) {                   /* wave-uniform: word loads, none past the lane's reads */\n")],
    "fdep": [("        if (TAIL) w8 = (uint32_t)j < m ? w8 : 8u * LN_FK_ZERO;\n        W += inc << sh;\n"
              "        t[j] = *reinterpret_cast<const double *>(fkb + w8);\n    }\n"
              "#pragma unroll\n    for (int j = 0; j < 4; ++j) {\n        const uint32_t q = (R >> (24 - 8 * j)) & 63u;\n"
              "        e = (float)((double)e + t[j] * (double)q);\n        f = (float)((double)f + t[j]);\n    }\n",
              "        if (TAIL) w8 = (uint32_t)j < m ? w8 : 8u * LN_FK_ZERO;\n        W += inc << sh;\n"
              "        t[j] = *reinterpret_cast<const double *>(fkb + w8);\n    }\n"
              "    float e2 = 0.0f, f2 = 0.0f;\n#pragma unroll\n    for (int j = 0; j < 4; ++j) {\n"
              "        const uint32_t q = (R >> (24 - 8 * j)) & 63u;\n        if (j & 1) { e2 = (float)((double)e2 + t[j] * (double)q); "
              "f2 = (float)((double)f2 + t[j]); }\n        else { e = (float)((double)e + t[j] * (double)q); "
              "f = (float)((double)f + t[j]); }\n    }\n    e += e2;\n    f += f2;\n")],
    "gfdep": [("        if (TAIL) w8 = j < m ? w8 : 8u * GP_FK_ZERO;\n        W += 8u << sh;\n"
               "        t[j] = *reinterpret_cast<const double *>(fkb + w8);\n    }\n"
               "#pragma unroll\n    for (int j = 0; j < 4; ++j) {\n        const uint32_t q = (R >> (24 - 8 * j)) & 63u;\n"
               "        e = (float)((double)e + t[j] * (double)q);\n        f = (float)((double)f + t[j]);\n    }\n",
               "        if (TAIL) w8 = j < m ? w8 : 8u * GP_FK_ZERO;\n        W += 8u << sh;\n"
               "        t[j] = *reinterpret_cast<const double *>(fkb + w8);\n    }\n"
               "    float e2 = 0.0f, f2 = 0.0f;\n#pragma unroll\n    for (int j = 0; j < 4; ++j) {\n"
               "        const uint32_t q = (R >> (24 - 8 * j)) & 63u;\n        if (j & 1) { e2 = (float)((double)e2 + t[j] * (double)q); "
               "f2 = (float)((double)f2 + t[j]); }\n        else { e = (float)((double)e + t[j] * (double)q); "
               "f = (float)((double)f + t[j]); }\n    }\n    e += e2;\n    f += f2;\n")],
    "gnosort": [("            ln_levels<LN_R, 2>(v);\n            if (__ballot(act && uP >= 2u))",
                 "            if (__ballot(act && uP >= 2u))")],
    "gnomerge": [("            if (__ballot(act && uP >= 2u)) { if (act && uP >= 2u) gp_level<2>(v, j, pb, uU); }\n"
                  "            if (__ballot(act && uP >= 4u)) { if (act && uP >= 4u) gp_level<4>(v, j, pb, uU); }\n"
                  "            if (__ballot(act && uP >= 8u)) { if (act && uP >= 8u) gp_level<8>(v, j, pb, uU); }\n"
                  "            if (__ballot(act && uP >= 16u)) { if (act && uP >= 16u) gp_level<16>(v, j, pb, uU); }\n", "")],
    "gnorec": [("                    *reinterpret_cast<uint4 *>(gbuf + ubase + 4u * (uint32_t)i) =\n"
                "                        make_uint4(ln_rec_dword(v, i), ln_rec_dword(v, i + 1), ln_rec_dword(v, i + 2),\n"
                "                                   ln_rec_dword(v, i + 3));\n",
                "                    asm volatile(\"\" :: \"v\"(ubase));\n")],
    "gnofold": [("        fold_sample(recs, m3.rec_n & 0x1ffffu, cnt, fk, es, fs);\n",
                 "        for (int b = 0; b < 4; ++b) es[b] = fs[b] = (float)cnt[b] + (float)(m3.rec_n >> b);\n")],
    "gnofin": [("    geno_p5(0u, es, fs, c, tot, a.m, p);\n    geno_p5(1u, es, fs, c, tot, a.m, p + 5);\n",
                "    for (int t = 0; t < 10; ++t) p[t] = es[t & 3] + (float)c[t & 3];\n")],
}


def main():
    if len(sys.argv) < 3:
        sys.exit(__doc__)
    out, phases = sys.argv[1], sys.argv[2:]
    s = open(SRC).read()
    for ph in phases:
        if ph not in EDITS:
            sys.exit(f"unknown phase {ph}; known: {', '.join(EDITS)}")
        for old, new in EDITS[ph]:
            if s.count(old) != 1:
                sys.exit(f"{ph}: the kernel source no longer has exactly one {old.strip()[:60]!r}")
            s = s.replace(old, new)
    open(out, "w").write(s)


if __name__ == "__main__":
    main()
