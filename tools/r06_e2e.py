#!/usr/bin/env python3
"""End-to-end timing of the drop-in CLI: the reference
CLI against the native one on a synthetic BAM pair (tools/bamsim.py), outputs
compared byte for byte, with a host-side split.

Runs (classic output):
  reference           oracle/_ref/bam-somaticsniper (1 thread)
  stream              native, SS_CONTIG_GROUPS=1 (one streaming walk, no index use)
  stream_pileup       the same with SS_PILEUP_ONLY=1 (no scoring)
  groups4 / groups8   native with the BAM indexes, 4 / 8 contig ranges
  groups4_pileup      4 ranges, SS_PILEUP_ONLY=1
  inflate             zcat of both BAMs, one core each, sequential (DEFLATE work)
Each run's wall time and CPU time (user + sys of the child) are recorded.
The split: inflate = zcat CPU; column build = pileup-only CPU - inflate CPU;
scoring wait = full wall - pileup-only wall (GPU scoring and the writers on
the critical path).

    python3 tools/r06_e2e.py OUT_JSON [--length 50000000] [--depth-t 60] [--depth-n 30] [--contigs 8]
"""
import argparse
import json
import os
import resource
import shutil
import subprocess
import sys
import tempfile
import threading
import time

R = os.environ.get("GRAFT_REPO_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(name, cmd, cwd, env=None, timeout=1000):
    """wall and child CPU seconds of one command; progress every 30 s"""
    stop = threading.Event()

    def tick():
        t = 0
        while not stop.wait(30):
            t += 30
            print(f"[e2e] {name} running {t} s", flush=True)
    th = threading.Thread(target=tick, daemon=True)
    th.start()
    r0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t0 = time.perf_counter()
    e = dict(os.environ)
    e.update(env or {})
    p = subprocess.run(cmd, cwd=cwd, env=e, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True,
                       timeout=timeout)
    wall = time.perf_counter() - t0
    r1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    stop.set()
    if p.returncode != 0:
        raise SystemExit(f"{name} failed ({p.returncode}): {p.stderr[-2000:]}")
    cpu = (r1.ru_utime - r0.ru_utime) + (r1.ru_stime - r0.ru_stime)
    print(f"[e2e] {name}: wall {wall:.2f} s, cpu {cpu:.2f} s", flush=True)
    return {"wall_s": round(wall, 3), "cpu_s": round(cpu, 3)}, p.stderr


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("--length", type=int, default=50_000_000)
    ap.add_argument("--depth-t", type=float, default=60)
    ap.add_argument("--depth-n", type=float, default=30)
    ap.add_argument("--contigs", type=int, default=8)
    ap.add_argument("--no-reference", action="store_true")
    a = ap.parse_args()
    w = tempfile.mkdtemp(prefix="ss_e2e6_", dir="/tmp")
    res = {"genome_bp": a.length, "contigs": a.contigs, "depth": f"{a.depth_t:g}/{a.depth_n:g}", "format": "classic",
           "host_cpus_visible": os.cpu_count()}
    try:
        t, _ = run("generate", [sys.executable, os.path.join(R, "tools/bamsim.py"), w, "--length", str(a.length),
                                "--depth-t", str(a.depth_t), "--depth-n", str(a.depth_n), "--contigs",
                                str(a.contigs)], w, timeout=1000)
        res["generate"] = t
        res["bam_bytes"] = {f: os.path.getsize(os.path.join(w, f)) for f in ("tumor.bam", "normal.bam")}
        nat = os.path.join(R, "somatic-sniper_amd/bam-somaticsniper")
        idx = os.path.join(R, "somatic-sniper_amd/ss-index")
        args = ["-f", "ref.fa", "tumor.bam", "normal.bam"]
        runs = {}
        if not a.no_reference:
            runs["reference"], _ = run("reference", [os.path.join(R, "oracle/_ref/bam-somaticsniper"), *args, "ref.out"],
                                       w, timeout=1100)
        runs["stream"], err = run("stream", [nat, *args, "stream.out"], w, {"SS_CONTIG_GROUPS": "1", "SS_TIMING": "1"})
        res["stream_timing_stamps"] = [x for x in err.splitlines() if x.startswith("[timing]")][-8:]
        runs["stream_pileup"], _ = run("stream_pileup", [nat, *args, "stream_po.out"], w,
                                       {"SS_CONTIG_GROUPS": "1", "SS_PILEUP_ONLY": "1"})
        t, _ = run("index", [idx, "tumor.bam"], w)
        t2, _ = run("index", [idx, "normal.bam"], w)
        res["index_both"] = {"wall_s": round(t["wall_s"] + t2["wall_s"], 3)}
        runs["groups4"], err = run("groups4", [nat, *args, "g4.out"], w,
                                   {"SS_CONTIG_GROUPS": "4", "SS_BGZF_THREADS": "2", "SS_TIMING": "1"})
        res["groups4_timing_stamps"] = [x for x in err.splitlines() if "scorer ready" in x or "done" in x][-6:]
        runs["groups4_pileup"], _ = run("groups4_pileup", [nat, *args, "g4_po.out"], w,
                                        {"SS_CONTIG_GROUPS": "4", "SS_BGZF_THREADS": "2", "SS_PILEUP_ONLY": "1"})
        runs["groups8"], _ = run("groups8", [nat, *args, "g8.out"], w,
                                 {"SS_CONTIG_GROUPS": "8", "SS_BGZF_THREADS": "2", "SS_PILEUP_WORKERS": "2"})
        inf = {"wall_s": 0.0, "cpu_s": 0.0}
        for f in ("tumor.bam", "normal.bam"):
            t, _ = run("inflate " + f, ["bash", "-c", f"zcat {f} > /dev/null"], w)
            inf = {k: round(inf[k] + t[k], 3) for k in inf}
        runs["inflate_zcat"] = inf
        res["runs"] = runs
        outs = ["stream.out", "g4.out", "g8.out"]
        base = "ref.out" if not a.no_reference else "stream.out"
        res["outputs_identical"] = all(open(os.path.join(w, base), "rb").read() == open(os.path.join(w, o), "rb").read()
                                       for o in outs)
        res["emitted_lines"] = sum(1 for _ in open(os.path.join(w, base)))
        sp = runs["stream_pileup"]
        res["split_stream"] = {
            "inflate_cpu_s": inf["cpu_s"],
            "column_build_cpu_s": round(sp["cpu_s"] - inf["cpu_s"], 3),
            "scoring_wait_wall_s": round(runs["stream"]["wall_s"] - sp["wall_s"], 3),
            "note": "inflate = zcat CPU of both BAMs; column build = pileup-only CPU minus inflate; scoring wait = "
                    "full minus pileup-only wall time (GPU scoring, D2H, writers on the critical path)"}
        res["split_groups4"] = {"scoring_wait_wall_s": round(runs["groups4"]["wall_s"] - runs["groups4_pileup"]["wall_s"], 3)}
        if "reference" in runs:
            ref = runs["reference"]["wall_s"]
            res["speedup_vs_reference"] = {k: round(ref / runs[k]["wall_s"], 2) for k in ("stream", "groups4", "groups8")}
            res["reference_positions_per_s"] = round(a.length / ref, 1)
        res["native_positions_per_s"] = {k: round(a.length / runs[k]["wall_s"], 1) for k in ("stream", "groups4", "groups8")}
    finally:
        shutil.rmtree(w, ignore_errors=True)
    with open(a.out, "w") as f:
        f.write(json.dumps(res) + "\n")
    print(json.dumps(res))


if __name__ == "__main__":
    main()
