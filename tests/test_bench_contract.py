"""bench.py's JSON line (the driver's contract) on a small run of the real path."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRCH38_NAMES = [("chr%s" % c, 0) for c in list(range(1, 23)) + ["X", "Y"]]
GRCH38 = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973, 145138636, 138394717,
          133797422, 135086622, 133275309, 114364328, 107043718, 101991189, 90338345, 83257441, 80373285,
          58617616, 64444167, 46709983, 50818468, 156040895, 57227415]


@pytest.mark.gpu
def test_bench_json_contract():
    """Default workload (C4, contig-sharded GRCh38, here / 4096): the driver's
    fields, strong scaling (a fixed --c4-scale), the roofline of the timed
    launches, the strong-scaling line and the 1-core reference baseline with
    its parity spot check."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--c4-scale", "4096", "--steps", "2",
                        "--warmup", "1", "--cpu-sample", "20000", "--strong-scale", "8192", "--strong-steps", "2",
                        "--host-fed-sites", "262144"],
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline", "strong_scaling"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["value"] > 1e8 and r["higher_is_better"] is True
    assert r["scaling"] == "strong" and r["unit"] == "sites/s" and r["config"]["workload"].startswith("C4")
    genome = r["config"]["genome_sites_per_step"]
    assert genome == sum(-(-length // 4096) for length in GRCH38)
    assert r["ranks"][0]["sites"] == 2 * genome and len(r["ranks"][0]["contigs"]) == 24
    assert abs(r["value"] - 2 * genome / (r["ms_per_step"] * 2e-3)) / r["value"] < 1e-3
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    assert rf["launches_timed"] == 2 * r["ranks"][0]["launches_per_step"]
    import shutil
    if shutil.which("rocprofv3") or os.path.exists("/opt/rocm/bin/rocprofv3"):
        # live PMC passes: HBM traffic of the timed kernel and its VALU issue share
        assert rf["traffic"] and 0.5 < rf["traffic_over_algorithmic"] < 3.0, rf
        v = rf["valu"]
        assert v["insts_per_site"] > 50 and 0 < v["issue_frac_lower_bound"] < 1.0, v
        # the clock from the profiled pass's own cycles and durations (never above MI355X's 2.4 GHz)
        assert 0.5 < v["clock_ghz_profiled"] <= 2.45 and v["kernel_ms_profiled"] > 0, v
        # the rocprofv3 kernel trace of the same launches beside the HIP-event mean
        kt = rf["kernel_ms_rocprof_trace"]
        assert kt["dispatches"] > 0 and kt["warm_dispatches_ms"] > 0 and kt["hip_events_ms"] == rf["avg_kernel_ms"]
    cb = r["cpu_baseline"]
    assert cb["cores"] == 1 and cb["value"] > 0 and cb["parity_vs_gpu"] is True
    hf = r["host_fed"]                      # PCIe-inclusive ss_score_batch_host, never `value`
    assert hf["parity_vs_device_path"] is True and hf["pinned"]["value"] > 1e6 and hf["pageable"]["value"] > 1e6
    assert 0 < hf["pinned"]["h2d_GBps"] < 200 and hf["pinned"]["value"] < r["value"]
    st = r["strong_scaling"]
    assert st["scaling"] == "strong" and st["value"] > 1e8 and st["c4_scale"] == 8192
    assert st["genome_sites_per_step"] == sum(-(-length // 8192) for length in GRCH38)
    assert r["config"]["planned_hbm_bytes_per_rank"] >= r["ranks"][0]["hbm_peak_allocated_bytes"] * 0.5


@pytest.mark.gpu
def test_bench_shard_workload_depth_baseline():
    """--workload shard (the C2/C3/C5 depth runs): weak scaling, and the CPU
    baseline is taken at the run's own depth with its parity spot check."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "shard", "--lt", "500",
                        "--ln", "500", "--sites", "65536", "--steps", "2", "--warmup", "1", "--no-pmc",
                        "--cpu-sample", "3000"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["scaling"] == "weak" and r["config"]["sites_per_step_per_gpu"] == 65536
    # 500x/500x: the deep triage decides almost every site
    assert r["roofline"]["kernel"] == "ss_score_triage+ss_score_triage_deep+ss_score_main"
    cb = r["cpu_baseline"]
    assert "500.0xT/500.0xN" in cb["sample"] and cb["parity_vs_gpu"] is True


# ---------------------------------------------------------------- CPU: launcher
def _bench():
    sys.path.insert(0, ROOT)
    from __graft_entry__ import load_package
    load_package()                     # registers somatic_sniper_amd (sharding) for bench.c4_layout
    import bench
    return bench


def test_gpus_flag_spawns_ranks(tmp_path):
    """bench.py --gpus N without a launcher starts N rank processes with
    RANK/WORLD_SIZE/LOCAL_RANK set (the parent itself stays GPU-free)."""
    child = tmp_path / "child.py"
    child.write_text("import os, sys\n"
                     "open(os.path.join(sys.argv[1], 'r' + os.environ['RANK']), 'w').write("
                     "' '.join(os.environ[k] for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR')))\n")
    env_keep = {k: os.environ.pop(k) for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK") if k in os.environ}
    try:
        rc = _bench().spawn_ranks(3, argv=[str(tmp_path)], script=str(child))
    finally:
        os.environ.update(env_keep)
    assert rc == 0
    got = sorted((tmp_path / f"r{r}").read_text() for r in range(3))
    assert got == [f"{r} 3 {r} 127.0.0.1" for r in range(3)]


def test_failing_rank_stops_the_others(tmp_path):
    child = tmp_path / "child.py"
    child.write_text("import os, sys, time\n"
                     "if os.environ['RANK'] == '1': sys.exit(7)\n"
                     "time.sleep(60)\n")
    import time
    t0 = time.time()
    rc = _bench().spawn_ranks(2, argv=[], script=str(child))
    assert rc == 7 and time.time() - t0 < 30


def test_gpus_must_match_launcher_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "WORLD_SIZE=2" in p.stderr


def test_tuning_variables_refused():
    env = dict(os.environ, SS_MAIN_GRID="16")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")], env=env,
                       capture_output=True, text=True, timeout=60)
    assert p.returncode != 0 and "SS_MAIN_GRID" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("gpus", [2, 8])
def test_bench_c4_ranks_self_spawned_gloo(gpus):
    """--gpus N launched directly, C4 workload: N ranks (sharing the box's one
    GPU under gloo), each scoring the contigs sharding.shard_contigs gives it;
    every contig is scored exactly once, and the whole genome's sites over the
    max rank time is the value.  Every N's line carries the north star's
    fields: the reference CPU baseline (rank 0, with its parity check), the
    PMC traffic of rank 0's own launches of this N, and the host-fed rate."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "gloo",
                        "--c4-scale", "8192", "--steps", "2", "--warmup", "1", "--strong-scale", "16384",
                        "--strong-steps", "2", "--cpu-sample", "20000", "--host-fed-sites", "65536"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["n_gpus"] == gpus and len(r["ranks"]) == gpus and r["scaling"] == "strong"
    assert sorted(x["rank"] for x in r["ranks"]) == list(range(gpus))
    contigs = [c for x in r["ranks"] for c in x["contigs"]]
    assert sorted(contigs) == sorted(n for n, _ in GRCH38_NAMES) and len(set(contigs)) == 24
    genome = r["config"]["genome_sites_per_step"]
    assert sum(x["sites_per_step"] for x in r["ranks"]) == genome
    assert r["value"] > 0 and r["strong_scaling"]["value"] > 0
    cb = r["cpu_baseline"]
    assert cb["cores"] == 1 and cb["value"] > 0 and cb["parity_vs_gpu"] is True and "cpu_baseline_all_cores" in r
    assert r["host_fed"]["parity_vs_device_path"] is True
    import shutil
    if shutil.which("rocprofv3") or os.path.exists("/opt/rocm/bin/rocprofv3"):
        rf = r["roofline"]
        assert rf["traffic"] and 0.5 < rf["traffic_over_algorithmic"] < 3.0 and rf["pmc_launch_world"] == gpus, rf
    worst = max(x["ms_per_step"] for x in r["ranks"])
    assert abs(r["ms_per_step"] - worst) < 1e-3 + 1e-6 * worst
    assert abs(r["value"] - genome * 2 / (worst * 2 * 1e-3)) / r["value"] < 1e-3
    assert r["config"]["plan_imbalance"] < (1.01 if gpus == 8 else 1.001)


@pytest.mark.gpu
def test_c4_packed_launch_equals_its_pieces(pkg):
    """bench.synth_pieces: contig pieces generated back to back in one HBM
    batch (offsets rebased per piece) hold exactly the sites of each piece
    (host generator, synth shard = contig), and score like them."""
    import numpy as np
    import torch
    b = _bench()
    dev = torch.device("cuda", 0)
    args = type("A", (), dict(lt=60.0, ln=30.0, seed=0x5EED5A1DC0FFEE01))()
    pieces = [(3, 1000, 700), (4, 0, 1234), (7, 55, 3)]
    with pkg.Context(pkg.Params.default(), device=0) as ctx:
        d = b.synth_pieces(ctx, pkg, args, pieces, dev)
        host = [pkg.synth_batch_host(pkg.Synth.default(60, 30, seed=args.seed, shard=t), f, n) for t, f, n in pieces]
        ref = np.concatenate([h.ref for h in host])
        rt = np.concatenate([h.reads_tumor for h in host])
        rn = np.concatenate([h.reads_normal for h in host])
        ot = np.concatenate([[0]] + [h.off_tumor[1:] + sum(int(x.off_tumor[-1]) for x in host[:i])
                                     for i, h in enumerate(host)]).astype(np.uint32)
        on = np.concatenate([[0]] + [h.off_normal[1:] + sum(int(x.off_normal[-1]) for x in host[:i])
                                     for i, h in enumerate(host)]).astype(np.uint32)
        assert (d["ref"].cpu().numpy() == ref).all()
        assert (d["off_tumor"].cpu().numpy().view(np.uint32) == ot).all()
        assert (d["off_normal"].cpu().numpy().view(np.uint32) == on).all()
        assert (d["reads_tumor"].cpu().numpy().view(np.uint32)[: len(rt)] == rt).all()
        assert (d["reads_normal"].cpu().numpy().view(np.uint32)[: len(rn)] == rn).all()
        s, _, _ = ctx.score_batch(pkg.Batch(ref, ot, on, rt, rn))
        parts = np.concatenate([ctx.score_batch(h)[0] for h in host])
        assert (s == parts).all()


def test_c4_layout_partitions_the_genome():
    """CPU: the C4 plan covers every GRCh38 contig exactly once at 1..8 ranks,
    sized by --c4-scale, and balances the 8-GPU split to within 1% (greedy LPT
    alone leaves the largest rank 3.6% over the mean)."""
    b = _bench()
    for world in (1, 2, 3, 4, 8):
        names, sizes, plan = b.c4_layout(16, world)
        assert sorted(t for p in plan for t in p) == list(range(24))
        assert sizes == [-(-length // 16) for length in GRCH38]
        loads = [sum(sizes[t] for t in p) for p in plan]
        assert max(loads) / (sum(loads) / world) < (1.01 if world == 8 else 1.001)
    import importlib
    sh = importlib.import_module("somatic_sniper_amd.sharding")
    assert sh.plan_imbalance(GRCH38, sh.shard_contigs(GRCH38, 8, restarts=0)) < 1.04


def test_c4_default_sizing_fits_hbm():
    """CPU: --c4-scale auto gives every GPU one eighth of GRCh38 (8 / N), so
    N = 8 is the whole 3.09e9-site genome of BASELINE configs[3]; the planned
    resident bytes per rank (reads, offsets, ref, scores, the largest launch's
    working set) fit 85% of one MI355X's 288 GB at every N, and the per-GPU
    share stays within 1% of the 8-GPU one."""
    b = _bench()
    hbm = 288e9
    assert [b.c4_auto_scale(w) for w in (1, 2, 4, 8, 16)] == [8, 4, 2, 1, 1]
    per8 = max(b.c4_rank_bytes(1, 8, 60.0, 30.0, 1 << 26))
    assert 1.3e11 < per8 < 0.85 * hbm, per8            # about 143 GB per GPU
    _, sizes, plan = b.c4_layout(1, 8)
    assert sum(sizes) == sum(GRCH38)
    for world in (1, 2, 4):
        per = max(b.c4_rank_bytes(b.c4_auto_scale(world), world, 60.0, 30.0, 1 << 26))
        assert per < 0.85 * hbm and abs(per / per8 - 1) < 0.01, (world, per, per8)
    # a site's bytes bound the generator's mean non-deleted depth (0.99 (lt + ln))
    assert b.site_bytes(60, 30) >= 4 * 89.1 + 13
