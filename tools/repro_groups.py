#!/usr/bin/env python3
"""Repeat the native CLI's contig-group + shared-device run on the 60x/30x
synthetic pair (tests/conftest.py seed 2) and compare each output with the
reference CLI's; on a mismatch keep the output and the per-batch log
(SS_DEBUG_BATCHES=1) under gpurun_out/repro/.  Diagnosis tool (GPU box)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bamgen  # noqa: E402

NATIVE = os.path.join(ROOT, os.environ.get("REPRO_NATIVE", "somatic-sniper_amd/bam-somaticsniper"))
REF_CLI = os.path.join(ROOT, "oracle", "_ref", "bam-somaticsniper")
INDEX = os.path.join(ROOT, "somatic-sniper_amd", "ss-index")
OUT = os.path.join(ROOT, "gpurun_out", os.environ.get("REPRO_OUT", "repro"))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    os.makedirs(OUT, exist_ok=True)
    d = "/tmp/repro_pair2"
    shutil.rmtree(d, ignore_errors=True)
    os.makedirs(d)
    bamgen.make_pair(d, seed=2, depth_t=60, depth_n=30)
    for b in ("tumor.bam", "normal.bam"):
        assert subprocess.run([INDEX, b], cwd=d, capture_output=True).returncode == 0
    args = ["-F", "vcf", "-Q", "0", "-f", "ref.fa", "tumor.bam", "normal.bam"]
    assert subprocess.run([REF_CLI] + args + ["ref.out"], cwd=d, capture_output=True).returncode == 0
    strip = lambda s: "".join(l for l in s.splitlines(True) if not l.startswith("##fileDate"))
    ref = strip(open(os.path.join(d, "ref.out")).read())
    env = dict(os.environ, SS_CONTIG_GROUPS="2", SS_DEVICES="0,0", SS_DEVICES_SHARED="1", SS_DEBUG_BATCHES="1")
    for kv in sys.argv[2:]:                      # extra VAR=value settings
        k, v = kv.split("=", 1)
        env[k] = v
    bad = 0
    for r in range(reps):
        p = subprocess.run([NATIVE] + args + ["nat.out"], cwd=d, capture_output=True, text=True, env=env,
                           timeout=120)
        nat = strip(open(os.path.join(d, "nat.out")).read())
        ok = p.returncode == 0 and nat == ref
        if not ok:
            bad += 1
            open(os.path.join(OUT, f"bad{r}.out"), "w").write(nat)
            open(os.path.join(OUT, f"bad{r}.err"), "w").write(p.stderr)
        elif r == 0 or os.environ.get("REPRO_KEEP_ALL") == "1":
            open(os.path.join(OUT, f"good{r}.err"), "w").write(p.stderr)
        print(f"run {r}: {'ok' if ok else 'MISMATCH'} rc={p.returncode} lines nat={nat.count(chr(10))} "
              f"ref={ref.count(chr(10))}", flush=True)
    print("mismatches", bad, "of", reps)


if __name__ == "__main__":
    main()
