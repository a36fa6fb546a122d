#!/usr/bin/env python3
"""bench.py -- pileup sites/sec of the MI355X somatic scorer (BASELINE.json metric).

Workload c4 (default; BASELINE.json configs[3]): the 24 GRCh38 primary contigs
as a synthetic genome (one pileup site per position, 60xT/30xN Poisson depths,
SURVEY.md 8(d)), contigs assigned to ranks by sharding.shard_contigs.  Sites
are keyed by (contig, position): synth shard = contig index.  One STEP = every
rank scores its share of the genome once (ss_score_batch_device per launch of
up to --chunk sites: main + group + deep kernels).  By default the genome is
divided by 8 / N (--c4-scale auto): every GPU holds one eighth of GRCh38
(3.86e8 sites, about 143 GB of packed reads in HBM), so N = 8 scores the whole
3.09e9-site genome of configs[3] in one step and N = 1, 2, 4 the same
per-GPU share (weak scaling: per-GPU work fixed).  A secondary line,
"strong_scaling", times the genome / 16 at every N (total work fixed).
Workload shard: --sites sites per rank per step (weak scaling; the C2/C3/C5
depth runs).  Inputs are generated on the device before timing; the timed
region contains only scoring.

Multi-GPU: one process per GPU (torch.distributed, RCCL backend only for the
barrier and the max-over-ranks timing reduction).  Each rank scores its own
contigs -- no collective on the data path.  value = sites scored by all ranks
/ max rank time.  Launched either
by torch.distributed.run (RANK/WORLD_SIZE/LOCAL_RANK in the environment) or
directly as ``bench.py --gpus N``: the parent then starts N fresh rank
processes itself before anything touches the GPU, stays GPU-free, and relays
rank 0's line.

Extra fields, all measured by rank 0 after the timed region at EVERY N (so
each line of a 1/2/4/8-GPU scaling run carries them): "roofline" (the kernel
with the most time, HIP events over the timed region's launches, algorithmic
bytes 4 B/read + 16 B/site per launch; "traffic" and "valu" from rocprofv3
--pmc passes over a child scoring rank 0's own first launches of this N),
"cpu_baseline" (the real reference glf_somatic compiled from source,
oracle/_ref/ref_harness, 1 core, on a bounded sample of the same synthetic
workload -- about the same CPU time at any depth --, also used as a parity
spot check), "cpu_baseline_all_cores" (the same on every core we may use, one
process per core) and "host_fed" (ss_score_batch_host, the PCIe-inclusive
path a BAM-driven caller uses, on pageable and page-locked host arrays of the
same workload; never `value`).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# BASELINE.json "metric", verbatim
METRIC = "pileup sites/sec at 60\u00d7T/30\u00d7N; 1\u21928 GPU scaling; achieved HBM GB/s vs roofline"


def cpu_baseline(lt, ln, sample, seed, gpu_scores_prefix, shard=0):
    """Time the reference's glf_somatic (compiled from /root/reference) on `sample`
    sites of synth shard `shard` (rank 0's first contig); falls back to the CPU
    port when the binary is absent."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    scores_path = os.path.join("/tmp", f"ss_cpu_scores_{os.getpid()}.bin")
    if os.path.exists(harness):
        out = subprocess.run([harness, "synth", str(lt), str(ln), str(sample), "--seed", str(seed),
                              "--shard", str(shard), "--scores", scores_path],
                             check=True, capture_output=True, text=True).stdout
        r = json.loads(out.strip().splitlines()[-1])
        kind, value = "reference", r["sites_per_s"]
        cpu_scores = np.fromfile(scores_path, np.int32)
        os.unlink(scores_path)
        desc = (f"{sample} synthetic sites ({lt}xT/{ln}xN, synth shard {shard} from site 0: the first positions of "
                f"rank 0's first contig of the c4 workload / of rank 0's batch 0 of the shard workload), reference "
                f"glf_somatic only (pileups prebuilt, BAM decode excluded), 1 thread")
    else:
        from __graft_entry__ import load_package
        from oracle import binding as ob
        pkg = load_package()
        h = pkg.synth_batch_host(pkg.Synth.default(lt, ln, seed=seed, shard=shard), 0, sample)
        o = ob.Oracle()
        t0 = time.perf_counter()
        cpu_scores, _, _ = o.score_batch(h.ref, h.off_tumor, h.off_normal, h.reads_tumor,
                                         h.reads_normal, want_glf=False)
        dt = time.perf_counter() - t0
        kind, value = "port", sample / dt
        desc = f"{sample} synthetic sites ({lt}xT/{ln}xN), CPU restatement oracle, 1 thread"
    parity = None
    if gpu_scores_prefix is not None and len(gpu_scores_prefix) >= sample:
        parity = bool((gpu_scores_prefix[:sample] == cpu_scores).all())
    return {"value": round(value, 1), "unit": "sites/s", "cores": 1, "kind": kind, "cpu_model": cpu_model(),
            "sample": desc, "parity_vs_gpu": parity}


def cpu_baseline_all_cores(lt, ln, seed, per_proc=500_000):
    """The reference glf_somatic on every host core we may use: one harness
    process per core, each on its own synthetic shard (same distribution),
    run concurrently; sites of all processes / the longest process's scoring
    time.  None without the compiled reference."""
    harness = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(harness):
        return None
    cores, cores_source = host_cores()
    procs = [subprocess.Popen([harness, "synth", str(lt), str(ln), str(per_proc), "--seed", str(seed),
                               "--shard", str(100 + k)], stdout=subprocess.PIPE, text=True)
             for k in range(cores)]
    secs = []
    for p in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            return None
        secs.append(json.loads(out.strip().splitlines()[-1])["seconds"])
    return {"value": round(cores * per_proc / max(secs), 1), "unit": "sites/s", "cores": cores,
            "kind": "reference", "cpu_model": cpu_model(), "cores_source": cores_source,
            "host_cpus": os.cpu_count(),
            "sample": f"{cores} concurrent processes x {per_proc} synthetic sites ({lt}xT/{ln}xN, own shard each), "
                      f"reference glf_somatic only, total sites / longest process time"}


def host_fed(ctx, pkg, args, dev, reps=3):
    """The PCIe-inclusive rate of ss_score_batch_host (host arrays -> H2D ->
    kernels -> D2H -> calls sorted), the entry point a BAM-driven caller of
    bam_sspileup_file -> glf_somatic uses (sniper_pileup.c:226-266).  The
    batch is the first --host-fed-sites sites of synth shard 0 at the bench's
    depths (fewer where that many would pass 2^31 reads), generated on the
    device and copied to host memory once; then timed from pageable numpy
    arrays (staged by the library) and from ss_host_alloc (page-locked)
    arrays.  Best of `reps` calls each; the
    scores are checked against the device path on the same sites."""
    import torch
    # at most 2^31 expected reads per sample: u32 read offsets with Poisson headroom
    n = min(args.host_fed_sites, (1 << 31) // int(max(args.lt, args.ln, 1)))
    d = ctx.synth_device(pkg.Synth.default(args.lt, args.ln, seed=args.seed, shard=0), 0, n, device=dev)
    dev_score = torch.empty(n, dtype=torch.int32, device=dev)
    ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"],
                     score=dev_score)
    torch.cuda.synchronize(dev)
    nt, nn = d["n_reads"]
    hb = pkg.Batch(d["ref"].cpu().numpy(), d["off_tumor"].cpu().numpy().view(np.uint32),
                   d["off_normal"].cpu().numpy().view(np.uint32),
                   d["reads_tumor"][:nt].cpu().numpy().view(np.uint32),
                   d["reads_normal"][:nn].cpu().numpy().view(np.uint32))
    want = dev_score.cpu().numpy()
    del d, dev_score
    torch.cuda.empty_cache()
    in_bytes = hb.ref.nbytes + hb.off_tumor.nbytes + hb.off_normal.nbytes + hb.reads_tumor.nbytes + \
        hb.reads_normal.nbytes
    out = {"unit": "sites/s", "sites_per_call": n, "input_bytes_per_call": in_bytes,
           "output_bytes_per_call": 4 * n, "parity_vs_device_path": True}
    for kind, b in (("pageable", hb), ("pinned", hb.pinned())):
        got = ctx.score_batch(b)[0]                    # warm-up: staging areas, first launch
        out["parity_vs_device_path"] &= bool((got == want).all())
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            ctx.score_batch(b)
            ts.append(time.perf_counter() - t0)
        out[kind] = {"value": round(n / min(ts), 1), "mean": round(n / float(np.mean(ts)), 1),
                     "h2d_GBps": round(in_bytes / min(ts) / 1e9, 2), "ms_per_call": round(min(ts) * 1e3, 3)}
    out["note"] = ("PCIe-inclusive (H2D of the packed batch, kernels, D2H of the scores and calls), one call at a "
                   "time on one context; `value` is the HBM-resident rate")
    return out


# tuning / diagnostic switches of earlier builds: refused so that no timed run
# can be mistaken for one made with them (the shipped library reads none)
REFUSED_ENV = ("SS_DIAG", "SS_MAIN_GRID", "SS_WIDE_GRID")


def library_id(pkg):
    """Path (relative to the repo) and content hash of the scoring library used."""
    import hashlib
    path = pkg.library_path()
    with open(path, "rb") as f:
        digest = hashlib.sha256(f.read()).hexdigest()[:16]
    return {"path": os.path.relpath(path, ROOT), "sha256_16": digest}


def free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n: int, argv=None, script=None) -> int:
    """Start n rank processes of this script (RANK/WORLD_SIZE/LOCAL_RANK set), one
    per GPU, and wait for them.  Called before the parent imports torch or touches
    a device: every rank is a fresh process that initialises only its own GPU.
    If one rank fails the others are stopped (by PID) and its exit code returned."""
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR=os.environ.get("MASTER_ADDR", "127.0.0.1"),
                   MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, script or os.path.abspath(__file__)]
                                      + list(sys.argv[1:] if argv is None else argv), env=env))
    rc = 0
    live = list(procs)
    while live:
        time.sleep(0.2)
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c
                for q in live:
                    q.terminate()
    for p in procs:
        p.wait()
    return rc


def host_cores():
    """CPUs this process may use: the cgroup CPU quota when one is set (a GPU box
    grants a share of a larger host), else the affinity mask (nproc)."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, -(-int(quota) // int(period))), "cgroup cpu.max quota"
    except (OSError, ValueError):
        pass
    try:
        return len(os.sched_getaffinity(0)), "sched_getaffinity (nproc)"
    except AttributeError:
        return os.cpu_count() or 1, "os.cpu_count"


# PMC passes bench.py runs on itself (rank 0, N=1): one rocprofv3 process per
# pass (counters of different blocks / slot budgets never share a pass).
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",),
              ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
               "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_BUSY_CYCLES", "GRBM_GUI_ACTIVE"))


def pmc_child(args):
    """--pmc-child: the bench's own launches (rank 0's of an --pmc-world-GPU
    run: its first --pmc-batches c4 launches, or the shard workload's batch 0),
    scored --pmc-launches passes, nothing else (run under rocprofv3 by
    live_counters)."""
    import torch
    from __graft_entry__ import load_package
    pkg = load_package()
    dev = torch.device("cuda", 0)
    ctx = pkg.Context(pkg.Params.default(), device=0)
    if args.workload == "shard":
        args.batches = 1
    batches = make_batches(ctx, pkg, args, 0, args.pmc_world, dev, limit=args.pmc_batches)
    scores = [torch.empty(max(1, d["n_sites"]), dtype=torch.int32, device=dev) for d in batches]
    for _ in range(args.pmc_launches):
        for d, sc in zip(batches, scores):
            ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"],
                             score=sc)
    torch.cuda.synchronize(dev)
    ctx.check()
    ctx.close()


def _launch_groups(rows, names):
    """rocprofv3 records of the kernels `names` (a launch's dispatches of its
    kernel class in launch order, the last name closing a launch: the triage
    kernel, then the main kernel) grouped per launch, in dispatch order:
    [(dispatch ids, records)]"""
    by_id = {}
    for name, did, rec in rows:
        by_id.setdefault(did, (name, []))[1].append(rec)
    groups, cur_ids, cur = [], [], []
    for did in sorted(by_id):
        name, recs = by_id[did]
        cur_ids.append(did)
        cur.extend(recs)
        if name == names[-1]:
            groups.append((cur_ids, cur))
            cur_ids, cur = [], []
    return groups


def live_counters(args, kernel="ss_score_main"):
    """rocprofv3 --pmc passes over a child that scores the bench's own batch
    (same sites, depths, seed): per-launch means of `kernel`'s counters ('a+b':
    a kernel class of several kernels, summed per launch), the first launch
    dropped (cold tables).  None when rocprofv3 is missing or a pass fails --
    the timed result never depends on it."""
    import csv
    import re
    import shutil
    import tempfile
    names = kernel.split("+")
    kpat = re.compile("(" + "|".join(re.escape(k) for k in names) + r")[<(]")
    exe = shutil.which("rocprofv3") or ("/opt/rocm/bin/rocprofv3" if os.path.exists("/opt/rocm/bin/rocprofv3") else None)
    if exe is None:
        return None
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE")}
    env["TMPDIR"] = "/tmp"
    if env.get("SNIPER_AMD_LIB"):                  # the child runs in /tmp: the library the bench loaded
        env["SNIPER_AMD_LIB"] = os.path.abspath(env["SNIPER_AMD_LIB"])
    vals = {}
    # the counter passes, then one --kernel-trace pass over the same child: the
    # dispatches' own durations next to the bench's HIP-event times (the
    # rocprofv3 --stats average includes each batch's cold first launch)
    for counters in PMC_PASSES + (None,):
        out = tempfile.mkdtemp(prefix="ss_pmc_", dir="/tmp")
        try:
            mode = ["--kernel-trace", "--stats"] if counters is None else ["--pmc", *counters]
            cmd = [exe, *mode, "--output-format", "csv", "-d", out, "-o", "run", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", "--workload", args.workload,
                   *(["--c4-scale", str(args.c4_scale)] if args.c4_scale is not None else []),
                   "--chunk", str(args.chunk), "--sites", str(args.sites),
                   "--lt", str(args.lt), "--ln", str(args.ln), "--seed", str(args.seed),
                   "--pmc-launches", str(args.pmc_launches), "--pmc-batches", str(args.pmc_batches),
                   "--pmc-world", str(args.pmc_world)]
            # own process group: a pass that overruns is killed with its python child
            proc = subprocess.Popen(cmd, cwd="/tmp", env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                    text=True, start_new_session=True)
            try:
                _, err = proc.communicate(timeout=150)
            except subprocess.TimeoutExpired:
                import signal
                os.killpg(proc.pid, signal.SIGKILL)
                proc.communicate()
                raise
            r = subprocess.CompletedProcess(cmd, proc.returncode, "", err)
            path = None
            want = "run_kernel_trace.csv" if counters is None else "run_counter_collection.csv"
            for dp, _, fs in os.walk(out):
                if want in fs:
                    path = os.path.join(dp, want)
            if counters is None and r.returncode == 0 and path is not None:
                rows = []
                with open(path) as f:
                    for row in csv.DictReader(f):
                        mk = kpat.search(row["Kernel_Name"])
                        if mk:
                            rows.append((mk.group(1), int(row["Dispatch_Id"]),
                                         float(row["End_Timestamp"]) - float(row["Start_Timestamp"])))
                durs = [sum(g) for _, g in _launch_groups(rows, names)]
                n_pass = len(durs) // max(1, args.pmc_launches)
                warm = durs[n_pass:] or durs
                vals["_kt"] = {"all_dispatches_ms": round(float(np.mean(durs)) / 1e6, 4) if durs else None,
                               "warm_dispatches_ms": round(float(np.mean(warm)) / 1e6, 4) if warm else None,
                               "dispatches": len(durs), "cold_dropped": n_pass}
                continue
            if counters is None:            # the trace is a side figure: its failure drops only it
                print(f"bench: kernel-trace pass failed (rc {r.returncode}): {r.stderr[-300:]}", file=sys.stderr)
                continue
            if r.returncode != 0 or path is None:
                print(f"bench: PMC pass {counters} failed (rc {r.returncode}): {r.stderr[-500:]}", file=sys.stderr)
                return None
            rows = []
            with open(path) as f:
                for row in csv.DictReader(f):
                    mk = kpat.search(row["Kernel_Name"])
                    if mk:
                        rows.append((mk.group(1), int(row["Dispatch_Id"]),
                                     (row["Counter_Name"], float(row["Counter_Value"]),
                                      float(row["End_Timestamp"]) - float(row["Start_Timestamp"]))))
            dispatch_ns = {did: dns for _, did, (_, _, dns) in rows}
            grbm = {}
            for _, did, (cn, cv, _) in rows:
                if cn == "GRBM_GUI_ACTIVE":
                    grbm[did] = grbm.get(did, 0.0) + cv
            per = {}
            for gi, (ids, recs) in enumerate(_launch_groups(rows, names)):
                d = per.setdefault(gi, {})
                for cn, cv, _ in recs:
                    d[cn] = d.get(cn, 0.0) + cv
                # the launch's duration in this same profiled pass (ns): its dispatches' durations summed
                d["_dur_ns"] = float(sum(dispatch_ns[i] for i in ids))
                # the clock from the launch's longest dispatch (a short one's busy count
                # includes its dispatch overhead beyond its own duration)
                big = max(ids, key=lambda i: dispatch_ns[i])
                d["_clock_pair"] = (grbm.get(big, 0.0), dispatch_ns[big])
            # one pass = one launch per batch; the first pass (cold tables) is dropped
            n_pass = len(per) // max(1, args.pmc_launches)
            ds = sorted(per)[n_pass:] or sorted(per)
            for c in counters:
                vals[c] = float(np.mean([per[k].get(c, 0.0) for k in ds]))
            if "GRBM_GUI_ACTIVE" in counters:
                # busy cycles per XCD / duration, both of the same profiled dispatches
                vals["_clock_ghz"] = float(np.mean([per[k]["_clock_pair"][0] / 8.0 / per[k]["_clock_pair"][1]
                                                    for k in ds if per[k]["_clock_pair"][1] > 0]))
                vals["_dur_ms_profiled"] = float(np.mean([per[k]["_dur_ns"] for k in ds])) / 1e6
            vals["_sites_per_launch"] = sites_per_launch(args)
        except (OSError, subprocess.SubprocessError, KeyError, ValueError) as e:
            print(f"bench: PMC pass {counters} failed: {e}", file=sys.stderr)
            return None
        finally:
            shutil.rmtree(out, ignore_errors=True)
    return vals


def sites_per_launch(args) -> float:
    """Mean sites per launch of the PMC child's workload (rank 0's of --pmc-world GPUs)."""
    if args.workload == "shard":
        return float(args.sites)
    launches = c4_launches(args.c4_scale, args.pmc_world, 0, args.chunk)[:args.pmc_batches]
    return sum(n for pieces in launches for _, _, n in pieces) / len(launches)


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def depth_scaled(n: int, lt: float, ln: float) -> int:
    """A CPU-baseline sample of about the same CPU time at any depth: the
    reference's glf_somatic costs about linearly in the reads per site, and n
    is the sample size at 60xT/30xN (89.1 non-deleted reads per site)."""
    return max(10_000, int(n * 89.1 / max(1.0, lt + ln)))


C4_GPUS = 8   # BASELINE.json configs[3]: the 3.2 Gb genome over 8 GPUs


def c4_auto_scale(world: int) -> int:
    """--c4-scale auto: the genome divided so that every GPU holds one eighth of
    it (8 / N), i.e. exactly configs[3]'s per-GPU share; 1 at N >= 8."""
    return max(1, -(-C4_GPUS // world))


def site_bytes(lt: float, ln: float) -> float:
    """HBM bytes one resident site takes: its packed reads (4 B each; the
    generator's mean non-deleted depth is 0.99 (lt + ln), below this bound),
    two u32 offsets, the ref byte and the i32 score."""
    return 4.0 * (lt + ln) + 4 + 4 + 1 + 4


# a context's own device memory (ss_capi.hip): the model tables (SS_TAB_BYTES)
# and, at full-grid batches, the group kernel's fold-record buffers (n_CU x 12
# waves x SS_GRP_REC_BYTES; allocated at the first batch that needs them)
CTX_BYTES = 34_092_416 + 256 * 12 * (131072 + 128)


def c4_rank_bytes(scale: int, world: int, lt: float, ln: float, chunk: int):
    """Planned resident HBM bytes of each rank's C4 share: its sites, plus the
    working set of its largest launch (the context's deep lists, 8 B per site,
    and the generator's depth arrays, 8 B per site) and the context itself."""
    _, sizes, plan = c4_layout(scale, world)
    out = []
    for p in plan:
        n = sum(sizes[t] for t in p)
        out.append(n * site_bytes(lt, ln) + 16.0 * min(chunk, n) + CTX_BYTES)
    return out


def c4_layout(scale: int, world: int):
    """Config C4 (BASELINE.json configs[3]): the 24 GRCh38 primary contigs, one
    synthetic site per position, the genome divided by `scale`; contigs are
    assigned to ranks by sharding.shard_contigs.  Returns (names, sites per
    contig, plan)."""
    import importlib
    sh = importlib.import_module("somatic_sniper_amd.sharding")
    names = [n for n, _ in sh.GRCH38_PRIMARY]
    sizes = [-(-length // scale) for _, length in sh.GRCH38_PRIMARY]
    return names, sizes, sh.shard_contigs(sizes, world)


def c4_launches(scale: int, world: int, rank: int, chunk: int):
    """The rank's contigs back to back (ascending tid), cut into launches of at
    most `chunk` sites: a launch may hold the end of one contig and the start
    of the next (sites are independent; fewer, fuller launches).  Each launch
    is a list of (tid, first position, sites) pieces."""
    _, sizes, plan = c4_layout(scale, world)
    launches, cur, room = [], [], chunk
    for tid in plan[rank]:
        first = 0
        while first < sizes[tid]:
            n = min(room, sizes[tid] - first)
            cur.append((tid, first, n))
            first += n
            room -= n
            if room == 0:
                launches.append(cur)
                cur, room = [], chunk
    if cur:
        launches.append(cur)
    return launches


def make_batches(ctx, pkg, args, rank, world, dev, limit=None, scale=None):
    """The rank's HBM-resident synthetic input, generated on the device.
    c4: the launches of c4_launches (genome / `scale`, default --c4-scale),
    keyed by (contig, position) -- synth shard = contig index, site =
    position --, the first `limit` of them when given.  shard: --batches
    batches of --sites sites of synth shard = rank."""
    out = []
    if args.workload == "c4":
        launches = c4_launches(args.c4_scale if scale is None else scale, world, rank, args.chunk)
        for pieces in launches[:limit]:
            d = synth_pieces(ctx, pkg, args, pieces, dev)
            d.update(tid=pieces[0][0], first=pieces[0][1], pieces=pieces)
            out.append(d)
    else:
        S = args.sites
        for b in range(args.batches):
            syn = pkg.Synth.default(args.lt, args.ln, seed=args.seed, shard=rank)
            d = ctx.synth_device(syn, b * S, S, device=dev)
            d.update(tid=rank, first=b * S)
            out.append(d)
    return out


def i32(x: int) -> int:
    """The int32 with the bits of the u32 x."""
    return x - (1 << 32) if x >= 1 << 31 else x


def synth_pieces(ctx, pkg, args, pieces, dev):
    """One HBM batch made of synthetic pieces (synth shard = contig, sites
    [first, first + n)), generated on the device piece by piece straight into
    the batch's arrays; each piece's read offsets are then moved up by the
    reads of the pieces before it."""
    import ctypes as C
    import torch
    S = sum(n for _, _, n in pieces)
    ref = torch.empty(S, dtype=torch.uint8, device=dev)
    ot = torch.empty(S + 1, dtype=torch.int32, device=dev)
    on = torch.empty(S + 1, dtype=torch.int32, device=dev)
    lib = ctx.lib
    tot = []
    so = 0
    torch.cuda.synchronize(dev)
    for tid, first, n in pieces:                  # pass 1: ref, piece-local offsets, read counts
        syn = pkg.Synth.default(args.lt, args.ln, seed=args.seed, shard=tid)
        nt, nn = C.c_uint64(), C.c_uint64()
        rc = lib.ss_synth_batch_device(ctx.h, C.byref(syn), first, n, ref.data_ptr() + so,
                                       ot.data_ptr() + 4 * so, on.data_ptr() + 4 * so, None, None,
                                       C.byref(nt), C.byref(nn))
        if rc:
            raise pkg.SniperError(rc, "ss_synth_batch_device")
        tot.append((nt.value, nn.value))
        so += n
    T, N = sum(t for t, _ in tot), sum(u for _, u in tot)
    if T >= 1 << 32 or N >= 1 << 32:
        sys.exit("bench.py: a launch holds >= 2^32 reads of one sample (u32 offsets); lower --chunk")
    rt = torch.empty(max(1, T), dtype=torch.int32, device=dev)
    rn = torch.empty(max(1, N), dtype=torch.int32, device=dev)
    so = bt = bn = 0
    for (tid, first, n), (nt, nn) in zip(pieces, tot):   # pass 2: reads; then rebase the offsets
        syn = pkg.Synth.default(args.lt, args.ln, seed=args.seed, shard=tid)
        rc = lib.ss_synth_batch_device(ctx.h, C.byref(syn), first, n, ref.data_ptr() + so,
                                       ot.data_ptr() + 4 * so, on.data_ptr() + 4 * so,
                                       rt.data_ptr() + 4 * bt, rn.data_ptr() + 4 * bn, None, None)
        if rc:
            raise pkg.SniperError(rc, "ss_synth_batch_device")
        if bt:
            ot[so:so + n] += i32(bt)              # u32 offsets held in int32 tensors: wrap-around add
        if bn:
            on[so:so + n] += i32(bn)
        so += n
        bt += nt
        bn += nn
    ot[S] = i32(T)
    on[S] = i32(N)
    torch.cuda.synchronize(dev)
    return {"ref": ref, "off_tumor": ot, "off_normal": on, "reads_tumor": rt, "reads_normal": rn,
            "n_reads": (T, N), "n_sites": S}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=("c4", "shard"), default="c4",
                    help="c4: GRCh38 contig-sharded genome (BASELINE config C4; strong scaling, total work fixed); "
                         "shard: --sites synthetic sites per rank (weak scaling; the C2/C3/C5 depth runs)")
    ap.add_argument("--c4-scale", type=int, default=None,
                    help="C4 genome sites divided by this (default: 8 / N, one eighth of the genome per GPU; "
                         "N = 8 runs the whole 3.09e9-site genome of BASELINE configs[3])")
    ap.add_argument("--chunk", type=int, default=1 << 26,
                    help="c4: most sites per launch (contig pieces packed back to back)")
    ap.add_argument("--sites", type=int, default=1 << 26, help="shard: sites per batch (per step, per GPU)")
    ap.add_argument("--batches", type=int, default=2, help="shard: distinct resident batches cycled per rank")
    ap.add_argument("--strong-scale", type=int, default=16,
                    help="c4: genome divisor of the secondary strong-scaling line (total work fixed at every N)")
    ap.add_argument("--strong-steps", type=int, default=10, help="c4: timed steps of that line (0 = skip it)")
    ap.add_argument("--lt", type=float, default=60.0)
    ap.add_argument("--ln", type=float, default=30.0)
    ap.add_argument("--seed", type=int, default=0x5EED5A1DC0FFEE01)
    ap.add_argument("--cpu-sample", type=int, default=None,
                    help="sites of the 1-core reference baseline (default: 2M at 60x/30x, scaled by depth)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--backend", default="nccl",
                    help="process-group backend for N>1 (nccl = RCCL; gloo rehearses N ranks on one GPU)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the live rocprofv3 counter passes")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-launches", type=int, default=3, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-batches", type=int, default=2, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--no-host-fed", action="store_true", help="skip the host-fed (PCIe-inclusive) sub-line")
    ap.add_argument("--host-fed-sites", type=int, default=1 << 22,
                    help="sites per ss_score_batch_host call of the host-fed sub-line")
    args = ap.parse_args()
    if args.pmc_child:
        return pmc_child(args)

    bad = [k for k in REFUSED_ENV if os.environ.get(k)]
    if bad:
        sys.exit(f"bench.py: refusing to time with tuning/diagnostic variables set: {', '.join(bad)}")
    if args.gpus < 1:
        sys.exit("bench.py: --gpus must be >= 1")
    if (args.c4_scale is not None and args.c4_scale < 1) or args.chunk < 1 or args.strong_scale < 1:
        sys.exit("bench.py: --c4-scale, --strong-scale and --chunk must be >= 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            sys.exit(spawn_ranks(args.gpus))      # parent: no torch, no GPU
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if args.backend != "nccl":
        local %= max(1, ndev)                       # rehearsal: ranks share the visible GPUs
    elif local >= ndev:
        sys.exit(f"bench.py: rank {rank} needs cuda:{local} but {ndev} device(s) are visible")
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from __graft_entry__ import load_package
    import importlib
    pkg = load_package()
    sharding = importlib.import_module("somatic_sniper_amd.sharding")
    ctx = pkg.Context(pkg.Params.default(), device=local)
    pinned = pkg.model_check()["pinned"]
    c4 = args.workload == "c4"
    auto_scale = c4 and args.c4_scale is None
    planned = None
    if c4:
        # every rank resolves the same scale (same world, same device model)
        _, hbm_total = torch.cuda.mem_get_info(dev)
        budget = 0.85 * hbm_total
        if auto_scale:
            args.c4_scale = c4_auto_scale(world)
            while max(c4_rank_bytes(args.c4_scale, world, args.lt, args.ln, args.chunk)) > budget:
                args.c4_scale += 1          # a smaller device than MI355X's 288 GB
        planned = max(c4_rank_bytes(args.c4_scale, world, args.lt, args.ln, args.chunk))
        if planned > budget:
            sys.exit(f"bench.py: --c4-scale {args.c4_scale} needs {planned / 1e9:.1f} GB of HBM per rank, "
                     f"more than 85% of the device's {hbm_total / 1e9:.1f} GB")

    # ---- resident synthetic input (this rank's contigs / shard) ----
    batches = make_batches(ctx, pkg, args, rank, world, dev)
    torch.cuda.synchronize(dev)
    if batches and max(max(d["n_reads"]) for d in batches) >= 1 << 32:
        sys.exit("bench.py: a batch holds >= 2^32 reads of one sample (u32 offsets); lower --chunk / --sites")
    reads = [sum(d["n_reads"]) for d in batches]
    bytes_of = [4 * r + 16 * d["n_sites"] for r, d in zip(reads, batches)]
    score = [torch.empty(max(1, d["n_sites"]), dtype=torch.int32, device=dev) for d in batches]
    cap = max(1024, max([d["n_sites"] for d in batches] + [0]) // 256)
    calls = torch.zeros(cap * 28, dtype=torch.uint8, device=dev)
    ncalls = torch.zeros(1, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    # a step: c4 scores every batch of the rank (its share of the genome, once);
    # shard scores one batch, cycling through the resident ones
    per_step = list(range(len(batches))) if c4 else None

    def launch(k):
        d = batches[k]
        ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"],
                         score=score[k], calls=calls, calls_cap=cap, n_calls=ncalls, stream=stream)

    def step(i):
        ks = per_step if c4 else [i % len(batches)]
        for k in ks:
            launch(k)
        return ks

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize(dev)
    ctx.check()

    # ---- timed region ----
    ctx.set_kernel_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    used = []
    for i in range(args.steps):
        used.extend(step(i))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    ctx.set_kernel_timing(False)
    ctx.check()
    elapsed = t1 - t0
    # per-kernel HIP-event durations of the logged launches (the first 4096);
    # the roofline is quoted for the kernel with the most time
    klog = {k: ctx.kernel_time_log(k) for k in ("main", "wide", "deep")}
    ksum = {k: float(np.sum(v)) for k, v in klog.items()}
    kmean = {k: float(np.mean(v)) if len(v) else 0.0 for k, v in klog.items()}
    dom = max(ksum, key=ksum.get)
    kms = klog[dom]
    logged = used[: len(kms)]
    sites_step_rank = sum(batches[k]["n_sites"] for k in (per_step if c4 else [0]))
    sites_rank = sum(batches[k]["n_sites"] for k in used)
    rank_elapsed = elapsed
    elapsed, total_sites, _ = sharding.aggregate(elapsed, sites_rank, world)
    prop = torch.cuda.get_device_properties(dev)
    me = {"rank": rank, "device": local, "pci_bus_id": getattr(prop, "pci_bus_id", None),
          "ms_per_step": round(rank_elapsed / args.steps * 1e3, 4), "sites": sites_rank,
          "sites_per_step": sites_step_rank, "launches_per_step": len(per_step) if c4 else 1,
          "hbm_peak_allocated_bytes": torch.cuda.max_memory_allocated(dev)}
    if c4:
        names, sizes, plan = c4_layout(args.c4_scale, world)
        me["contigs"] = [names[t] for t in plan[rank]]

    # GPU scores the CPU baseline is checked against: the first sites of this
    # rank's first launch (c4: its first contig from position 0, synth shard =
    # that contig; shard: batch 0, synth shard = rank)
    sample = depth_scaled(2_000_000, args.lt, args.ln) if args.cpu_sample is None else args.cpu_sample
    pre, cpu_shard = None, 0
    if batches and batches[0]["first"] == 0:
        d0 = batches[0]
        n0 = d0["pieces"][0][2] if c4 else d0["n_sites"]       # the first contig's sites in that launch
        sample = min(sample, n0)
        pre = score[0][:sample].cpu().numpy()
        cpu_shard = d0["tid"]
    reads_all = float(np.sum(reads))
    sites_all = sum(d["n_sites"] for d in batches)
    n_batches = len(batches)
    # free the resident batches before the next line / the counter passes
    del batches, score
    torch.cuda.synchronize(dev)
    torch.cuda.empty_cache()

    # ---- secondary strong-scaling line (c4 only): genome / --strong-scale at every N ----
    strong = None
    if c4 and args.strong_steps > 0:
        sb = make_batches(ctx, pkg, args, rank, world, dev, scale=args.strong_scale)
        ss = [torch.empty(max(1, d["n_sites"]), dtype=torch.int32, device=dev) for d in sb]

        def strong_step():
            for d, sc in zip(sb, ss):
                ctx.score_device(d["ref"], d["off_tumor"], d["off_normal"], d["reads_tumor"], d["reads_normal"],
                                 score=sc, calls=calls, calls_cap=cap, n_calls=ncalls, stream=stream)
        strong_step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        w0 = time.perf_counter()
        for _ in range(args.strong_steps):
            strong_step()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        s_sites = sum(d["n_sites"] for d in sb) * args.strong_steps
        s_el, s_tot, s_rate = sharding.aggregate(time.perf_counter() - w0, s_sites, world)
        ctx.check()
        _, s_sizes, _ = c4_layout(args.strong_scale, world)
        strong = {"value": round(s_rate, 1), "unit": "sites/s", "scaling": "strong", "c4_scale": args.strong_scale,
                  "genome_sites_per_step": sum(s_sizes), "steps": args.strong_steps,
                  "ms_per_step": round(s_el / args.strong_steps * 1e3, 4),
                  "workload": f"C4 / {args.strong_scale} (total work fixed at every N), "
                              f"{args.lt:g}xT/{args.ln:g}xN, contig-sharded"}
        del sb, ss
        torch.cuda.synchronize(dev)
        torch.cuda.empty_cache()

    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, me)
    else:
        ranks = [me]
    if rank == 0:
        print(f"bench: ranks {[(r['rank'], r['device'], r['pci_bus_id']) for r in ranks]}", file=sys.stderr)

    avg_kernel_ms = float(np.mean(kms)) if len(kms) else None
    alg_bytes = float(np.mean([bytes_of[k] for k in logged])) if logged else None
    achieved = alg_bytes / (avg_kernel_ms * 1e-3) / 1e9 if avg_kernel_ms and alg_bytes else None
    mean_reads = reads_all / max(1, sites_all)
    if c4:
        genome_sites = sum(sizes)
        whole = "the whole genome (BASELINE configs[3])" if args.c4_scale == 1 else f"/ {args.c4_scale}"
        config = {"workload": f"C4: synthetic GRCh38 (24 primary contigs, one site per position) {whole}, "
                              f"{args.lt:g}xT/{args.ln:g}xN Poisson depth, contig-sharded over {world} GPU(s)",
                  "genome_sites_per_step": genome_sites, "c4_scale": args.c4_scale,
                  "c4_scale_mode": ("auto: 8 / N, one eighth of GRCh38 per GPU (per-GPU work fixed)"
                                    if auto_scale else "fixed (--c4-scale)"),
                  "planned_hbm_bytes_per_rank": round(planned),
                  "sharding": "sharding.shard_contigs (LPT + local search on the contig lengths)",
                  "plan_imbalance": round(sharding.plan_imbalance(sizes, plan), 5),
                  "contigs_per_rank": [len(p) for p in plan],
                  "max_sites_per_launch": args.chunk}
        assert sum(r["sites_per_step"] for r in ranks) == genome_sites, "a contig scored twice or not at all"
    else:
        config = {"workload": f"synthetic shard per GPU, {args.lt:g}xT/{args.ln:g}xN Poisson depth",
                  "sites_per_step_per_gpu": args.sites, "resident_batches": n_batches}
    config.update({"mean_reads_per_site": round(mean_reads, 2),
                   "parallelism": f"{'contig' if c4 else 'region'}-sharded x{world}, no collectives",
                   "model_tables_pinned": pinned, "library": library_id(pkg)})
    result = {
        "metric": METRIC,
        "value": round(total_sites / elapsed, 1),
        "unit": "sites/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong" if c4 and not auto_scale else "weak",
        "vs_baseline": None,
        "dtype": "f32+f64 (u32 packed reads)",
        "data": "synthetic (device-generated counter-based pileups, Poisson depth)",
        "config": config,
        "ranks": ranks,
        "roofline": {
            "bound": "hbm",
            # the main class: the triage kernel (run when no glf records are
            # requested), the deep triage (blocks past 128 reads per sample) and the
            # main kernel, summed per launch
            "kernel": {"main": "ss_score_triage+ss_score_triage_deep+ss_score_main", "wide": "ss_score_group",
                       "deep": "ss_score_deep"}[dom],
            "achieved": round(achieved, 2) if achieved else None,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5) if achieved else None,
            "traffic": None,
            "algorithmic_bytes_per_launch": alg_bytes,
            "avg_kernel_ms": round(avg_kernel_ms, 4) if avg_kernel_ms else None,
            "avg_ms_by_kernel": {k: round(v, 4) for k, v in kmean.items()},
            "launches_timed": len(kms),
        },
    }
    if strong:
        result["strong_scaling"] = strong
    if rank == 0 and not args.no_pmc:
        # live counters of the dominant kernel on this same workload (separate
        # rocprofv3 passes after the timed region, over a child scoring rank 0's
        # own first launches of this N; MI355X_MICROARCH.md: FETCH_SIZE reports
        # half the streamed read bytes on gfx950 and is doubled, both KiB; SQ_*
        # wave counters, GRBM_GUI_ACTIVE = busy cycles summed over 8 XCDs)
        args.pmc_world = world
        pc = live_counters(args, result["roofline"]["kernel"])
        if pc:
            rd, wr = 2.0 * pc["FETCH_SIZE"] * 1024.0, pc["WRITE_SIZE"] * 1024.0
            rf = result["roofline"]
            rf["traffic"] = rd + wr
            # the counter child scores the first --pmc-batches launches (full
            # 2^26-site launches at C4): compare with their own algorithmic bytes
            alg_pmc = float(np.mean(bytes_of[:args.pmc_batches])) if c4 else alg_bytes
            rf["traffic_over_algorithmic"] = round((rd + wr) / alg_pmc, 4)
            rf["traffic_bytes_per_site"] = {"read": round(rd / pc["_sites_per_launch"], 2),
                                            "write": round(wr / pc["_sites_per_launch"], 2),
                                            "algorithmic": round(alg_pmc / pc["_sites_per_launch"], 2)}
            cyc = pc["GRBM_GUI_ACTIVE"] / 8.0                       # kernel cycles
            simds = 4 * torch.cuda.get_device_properties(dev).multi_processor_count
            site_n = pc["_sites_per_launch"]
            rf["valu"] = {
                "insts_per_site": round(pc["SQ_INSTS_VALU"] / site_n, 1),
                "salu_per_site": round(pc["SQ_INSTS_SALU"] / site_n, 1),
                "lds_per_site": round(pc["SQ_INSTS_LDS"] / site_n, 1),
                "issue_frac_lower_bound": round(2.0 * pc["SQ_INSTS_VALU"] / (cyc * simds), 4) if cyc else None,
                "issue_frac_assumes": "2 SIMD cycles per wave64 VALU instruction (the multi-wave rate of v_fma_f32 "
                                      "in MI355X_MICROARCH.md); f64, DPP and transcendental instructions take "
                                      "longer, so the true VALU busy share is higher",
                "wave_cycles_split": {k: round(pc[c] / pc["SQ_WAVE_CYCLES"], 3) for k, c in
                                      (("issue", "SQ_ACTIVE_INST_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"),
                                       ("waitcnt", "SQ_WAIT_ANY"))} if pc["SQ_WAVE_CYCLES"] else None,
                "clock_ghz_profiled": round(pc["_clock_ghz"], 3) if pc.get("_clock_ghz") else None,
                "kernel_ms_profiled": round(pc["_dur_ms_profiled"], 4) if pc.get("_dur_ms_profiled") else None,
                "clock_source": "GRBM_GUI_ACTIVE / 8 over the same dispatches' durations in the same profiled "
                                "pass (End - Start timestamps of rocprofv3's counter records); of each launch's "
                                "longest dispatch (the triage kernel when it runs)",
                "source": "rocprofv3 --pmc, separate passes over a child scoring rank 0's own launches of this N: "
                          "per-launch means of the second pass",
            }
            rf["pmc_launch_world"] = world
            if pc.get("_kt"):
                # `frac` uses the HIP-event mean of the timed
                # launches (the same launches as `value`); rocprofv3's trace of
                # the counter child's launches is quoted beside it
                rf["kernel_ms_rocprof_trace"] = dict(pc["_kt"], hip_events_ms=rf["avg_kernel_ms"],
                                                     source="rocprofv3 --kernel-trace over the counter child "
                                                            "(its first launch per batch is cold and dropped "
                                                            "from warm_dispatches_ms)")
    if rank == 0 and not args.no_host_fed:
        result["host_fed"] = host_fed(ctx, pkg, args, dev)
    if rank == 0 and not args.no_cpu:
        result["cpu_baseline"] = cpu_baseline(args.lt, args.ln, sample, args.seed, pre, shard=cpu_shard)
        allc = cpu_baseline_all_cores(args.lt, args.ln, args.seed,
                                      per_proc=depth_scaled(500_000, args.lt, args.ln))
        if allc:
            result["cpu_baseline_all_cores"] = allc
    if rank == 0:
        print(json.dumps(result), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
