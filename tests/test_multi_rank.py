"""Multi-process (gloo, world_size 2, CPU) checks of the genome sharding: each
rank scores only its own region with no data-path collective, the per-rank
results are exactly the corresponding slices of a single-process run, and the
bench aggregation takes the max time and the summed sites over ranks.
The scorer here is the CPU oracle (the GPU path is covered by -m gpu tests)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from __graft_entry__ import load_package
    import importlib
    pkg = load_package()
    sharding = importlib.import_module("somatic_sniper_amd.sharding")
    from oracle import binding as ob
    n = 3000
    first, last = sharding.shard_range(n, world, rank)
    b = pkg.synth_batch_host(pkg.Synth.default(60, 30, p_somatic=0.02), first, last - first)
    score, calls, _ = ob.Oracle().score_batch(b.ref, b.off_tumor, b.off_normal, b.reads_tumor,
                                              b.reads_normal, want_glf=False)
    np.save(os.path.join(out_dir, f"score{rank}.npy"), score)
    elapsed = 1.0 + rank            # rank 1 is the slow one
    t, sites, rate = sharding.aggregate(elapsed, last - first, world)
    np.save(os.path.join(out_dir, f"agg{rank}.npy"), np.array([t, sites, rate]))
    plan = sharding.shard_contigs([50, 40, 30, 20, 10, 5], world)
    np.save(os.path.join(out_dir, f"plan{rank}.npy"), np.array([len(x) for x in plan]))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_gloo(tmp_path, pkg):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    from oracle import binding as ob
    b = pkg.synth_batch_host(pkg.Synth.default(60, 30, p_somatic=0.02), 0, 3000)
    full, _, _ = ob.Oracle().score_batch(b.ref, b.off_tumor, b.off_normal, b.reads_tumor,
                                         b.reads_normal, want_glf=False)
    parts = np.concatenate([np.load(tmp_path / f"score{r}.npy") for r in range(world)])
    assert (parts == full).all()
    for r in range(world):
        t, sites, rate = np.load(tmp_path / f"agg{r}.npy")
        assert t == 2.0 and sites == 3000 and rate == 1500.0


def test_shard_contigs_partition():
    import importlib
    from __graft_entry__ import load_package
    load_package()
    sh = importlib.import_module("somatic_sniper_amd.sharding")
    lengths = [248956422, 242193529, 198295559, 190214555, 181538259, 170805979, 159345973,
               145138636, 138394717, 133797422, 135086622, 133275309, 114364328, 107043718,
               101991189, 90338345, 83257441, 80373285, 58617616, 64444167, 46709983, 50818468,
               156040895, 57227415]
    for world in (1, 2, 4, 8):
        plan = sh.shard_contigs(lengths, world)
        flat = sorted(t for p in plan for t in p)
        assert flat == list(range(len(lengths)))
        loads = [sum(lengths[t] for t in p) for p in plan]
        assert max(loads) <= sum(lengths) / world + max(lengths)
        assert all(p == sorted(p) for p in plan)
    assert sh.shard_range(10, 3, 0) == (0, 4) and sh.shard_range(10, 3, 2) == (7, 10)
