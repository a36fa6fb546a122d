"""bench.py's JSON line (the driver's contract) on a small run of the real path."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_contract():
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--sites", "262144", "--steps", "2",
                        "--warmup", "1", "--cpu-sample", "20000"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in r, k
    assert r["n_gpus"] == 1 and r["steps"] == 2 and r["value"] > 1e8 and r["higher_is_better"] is True
    assert r["scaling"] == "weak" and r["unit"] == "sites/s" and "workload" in r["config"]
    rf = r["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and 0 < rf["frac"] < 1
    assert abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-3
    import shutil
    if shutil.which("rocprofv3") or os.path.exists("/opt/rocm/bin/rocprofv3"):
        # live PMC passes: HBM traffic of the timed kernel and its VALU issue share
        assert rf["traffic"] and 0.5 < rf["traffic_over_algorithmic"] < 3.0, rf
        v = rf["valu"]
        assert v["insts_per_site"] > 50 and 0 < v["issue_frac"] < 1.0, v
    cb = r["cpu_baseline"]
    assert cb["cores"] == 1 and cb["value"] > 0 and cb["parity_vs_gpu"] is True


# ---------------------------------------------------------------- CPU: launcher
def _bench():
    sys.path.insert(0, ROOT)
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
def test_bench_gpus2_self_spawned_gloo():
    """--gpus 2 launched directly: two ranks (sharing the box's one GPU under
    gloo), each scoring its own shard; whole-job sites over the max rank time."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--backend", "gloo",
                        "--sites", "262144", "--steps", "2", "--warmup", "1"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["n_gpus"] == 2 and len(r["ranks"]) == 2
    assert sorted(x["rank"] for x in r["ranks"]) == [0, 1]
    assert r["value"] > 0 and "cpu_baseline" not in r
    worst = max(x["ms_per_step"] for x in r["ranks"])
    assert abs(r["ms_per_step"] - worst) < 1e-3 + 1e-6 * worst
    assert abs(r["value"] - 2 * 262144 * 2 / (worst * 2 * 1e-3)) / r["value"] < 1e-3
