#!/usr/bin/env python3
"""Diagnosis build (not shipped): libsniper_amd + CLI with round 4's device
memory source -- the stream-ordered pool (hipMallocAsync / hipFreeAsync on the
context's streams, no idle-block cache) -- but with this tree's table
fingerprint guard, so a run that loses calls the way round 4's CLI did now
says which table region no longer matches and when (creation or a later
ss_ctx_check).  Variants (VARIANTS below) test one hypothesis each; every variant prints
[diag] lines (blocks taken, each host batch's outcome, destroys) on stderr.
Output: somatic-sniper_amd/build/diag_<variant>/{libsniper_amd.so,
bam-somaticsniper}.  Run here (hipcc): python tools/diag_pool.py pool ...; then on the GPU box:
  REPRO_NATIVE=somatic-sniper_amd/build/diag_pool/bam-somaticsniper python tools/repro_groups.py 25
"""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "somatic-sniper_amd")


def patched_capi(variant):
    s = open(os.path.join(PKG, "csrc", "ss_capi.hip")).read()
    subs = [
        # allocation: the device's default pool, ordered on the caller's stream; no idle-cache reuse
        ("        size_t best = g_idle.size();\n",
         "        size_t best = g_idle.size();\n        if (1) {} else\n"),
        ("        if (hipMalloc(&b.base, need + 2 * SS_GUARD) != hipSuccess) {",
         "        if (hipMallocAsync(&b.base, need + 2 * SS_GUARD, s) != hipSuccess) {"),
        # release: hipFreeAsync on the context's stream at once (round 4's dev_free)
        ("            if (idle_now) {\n                std::lock_guard<std::mutex> g(g_mem_mu);\n"
         "                g_idle.push_back(b);\n            } else {",
         "            if (1) {\n                hipFreeAsync(b.base, c->hstream);\n            } else {"),
        # destroy: every block back to the pool on the context's stream, then synchronize it
        ("        for (auto *list : {c->blocks, c->retired})\n            for (const dev_blk &b : *list) g_idle.push_back(b);\n",
         "        for (auto *list : {c->blocks, c->retired})\n            for (const dev_blk &b : *list) hipFreeAsync(b.base, c->hstream);\n"
         "        if (c->hstream) hipStreamSynchronize(c->hstream);\n"),
    ]
    subs += [
        # diagnosis prints: every block a context takes, and each host batch's outcome
        ("    c->blocks->push_back(b);\n",
         "    c->blocks->push_back(b);\n    fprintf(stderr, \"[diag] ctx %p alloc %p %zu\\n\", (void *)c, b.base, need);\n"),
        ("    memcpy(o->score, h + o_sc, 4 * n);\n",
         "    memcpy(o->score, h + o_sc, 4 * n);\n"
         "    { long long hist[3] = {0, 0, 0}, sum = 0; uint32_t nc0; memcpy(&nc0, h + o_cnt, 4);\n"
         "      for (uint64_t i = 0; i < n; ++i) { const int v = o->score[i]; hist[v == -1 ? 0 : (v == 255 ? 1 : 2)]++; sum += v; }\n"
         "      fprintf(stderr, \"[diag] ctx %p batch n %llu nt %llu nn %llu stage %p tab %p ncalls %u rc %d score -1:%lld 255:%lld other:%lld sum %lld\\n\",\n"
         "              (void *)c, (unsigned long long)n, (unsigned long long)nt, (unsigned long long)nn, c->d_stage,\n"
         "              (void *)c->d_tab, nc0, rc, hist[0], hist[1], hist[2], sum); }\n"),
        ("extern \"C\" void ss_ctx_destroy(ss_ctx_t *c)\n{\n    if (!c) return;\n",
         "extern \"C\" void ss_ctx_destroy(ss_ctx_t *c)\n{\n    if (!c) return;\n"
         "    fprintf(stderr, \"[diag] ctx %p destroy\\n\", (void *)c);\n"),
    ]
    subs += VARIANTS[variant]
    for a, b in subs:
        assert s.count(a) == 1, a
        s = s.replace(a, b)
    return s


VARIANTS = {
    "pool": [],
    # the host path's staging area from hipMalloc / hipFree, everything else from the pool
    "pool_stage_malloc": [
        ("        if (hipMallocAsync(&b.base, need + 2 * SS_GUARD, s) != hipSuccess) {",
         "        if ((p == &c->d_stage ? hipMalloc(&b.base, need + 2 * SS_GUARD) : "
         "hipMallocAsync(&b.base, need + 2 * SS_GUARD, s)) != hipSuccess) {"),
        ("                hipFreeAsync(b.base, c->hstream);\n",
         "                if (&p == &c->d_stage) { hipStreamSynchronize(c->hstream); hipFree(b.base); }\n"
         "                else hipFreeAsync(b.base, c->hstream);\n"),
        ("            for (const dev_blk &b : *list) hipFreeAsync(b.base, c->hstream);\n",
         "            for (const dev_blk &b : *list) { if (blk_user(b) == c->d_stage) { hipStreamSynchronize(c->hstream); hipFree(b.base); } else hipFreeAsync(b.base, c->hstream); }\n"),
    ],
    # every pool allocation waited for on the host before the pointer is used
    "pool_sync": [
        ("        if (hipMallocAsync(&b.base, need + 2 * SS_GUARD, s) != hipSuccess) {",
         "        if (hipMallocAsync(&b.base, need + 2 * SS_GUARD, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {"),
    ],
    # a destroyed context keeps its stream (no hipStreamDestroy)
    "pool_keepstream": [
        ("    if (c->hstream) hipStreamDestroy(c->hstream);\n", "    /* stream kept (diagnosis) */\n"),
    ],
}


def main():
    for v in (sys.argv[1:] or ["pool"]):
        build(v)


def build(variant):
    OUT = os.path.join(PKG, "build", "diag_" + variant)
    os.makedirs(OUT, exist_ok=True)
    src = os.path.join(OUT, "ss_capi_pool.hip")
    open(src, "w").write(patched_capi(variant))
    hip = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-fPIC", "-std=c++17", "-ffp-contract=off",
           "-fno-fast-math", "-fno-gpu-flush-denormals-to-zero", "-I" + os.path.join(ROOT, "include"),
           "-I" + os.path.join(PKG, "csrc")]
    subprocess.run(hip + ["-c", src, "-o", os.path.join(OUT, "ss_capi.o")], check=True)
    b = os.path.join(PKG, "build")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-o",
                    os.path.join(OUT, "libsniper_amd.so"), os.path.join(b, "ss_tables.o"),
                    os.path.join(b, "ss_synth.o"), os.path.join(b, "ss_kernels.o"), os.path.join(OUT, "ss_capi.o"),
                    "-lpthread", "-lm"], check=True)
    cli = [os.path.join("cli", f) for f in ("sniper_cli.c", "dual_pileup.c", "column_pileup.c", "bam_reader.c",
                                            "bgzf_reader.c", "fasta_index.c", "sniper_output.c", "bam_index.c")]
    subprocess.run(["gcc", "-O2", "-I../include", "-Icli", "-o", os.path.join(OUT, "bam-somaticsniper")] + cli +
                   ["-L" + OUT, "-lsniper_amd", "-Wl,-rpath,$ORIGIN", "-lz", "-lpthread", "-ldl", "-lm"],
                   cwd=PKG, check=True)
    print("built", OUT)


if __name__ == "__main__":
    main()
