"""Genome sharding across GPUs (one process per GPU, no data-path collectives).

Sites are independent (glf_somatic keeps no state across sites except the cached
contig string, somatic_sniper.c:112-117), so a run is split into genome regions
and every rank scores its own regions end to end.  The only cross-rank traffic is
the barrier and the max-over-ranks timing reduction of the benchmark, and the
host-side concatenation of per-rank outputs in (tid, pos) order.

* ``shard_contigs``  assignment of whole contigs to ranks (SURVEY.md section
  8(e)): greedy longest-processing-time first, then a local search (single
  moves and pairwise swaps that lower the sum of squared rank loads) from the
  LPT start and from seeded random starts, keeping the plan with the smallest
  maximum load.  Deterministic for a given (lengths, world).  On GRCh38's 24
  primary contigs the largest rank holds 1.0040x the mean at 8 ranks (LPT
  alone: 1.0363x), 1.00017x at 4 and 1.0000001x at 2.  Assemblies with more than
  ``LOCAL_SEARCH_MAX`` contigs (alts, decoys, scaffolds) get LPT alone: the
  search's n x n move matrices would cost far more than they gain there, and
  with thousands of small contigs LPT is already within one contig of the mean.
* ``GRCH38_PRIMARY``  (name, length) of GRCh38 chr1..22, X, Y -- config C4's
  genome (BASELINE.json configs[3]).
* ``shard_range``    contiguous equal split of a site range (synthetic shards).
* ``aggregate``      whole-job throughput from per-rank (elapsed, sites) with the
  bench contract: time = max over ranks, sites = sum over ranks.
"""
from __future__ import annotations

import heapq


GRCH38_PRIMARY = (
    ("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
    ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
    ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
    ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
    ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
    ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415),
)


def _lpt(lengths, world: int):
    heap = [(0, r) for r in range(world)]
    heapq.heapify(heap)
    a = [0] * len(lengths)
    for tid in sorted(range(len(lengths)), key=lambda t: (-int(lengths[t]), t)):
        load, r = heapq.heappop(heap)
        a[tid] = r
        heapq.heappush(heap, (load + int(lengths[tid]), r))
    return a


LOCAL_SEARCH_MAX = 256


def _descend(x, a, world: int):
    """Steepest descent on the sum of squared rank loads over single moves
    (contig t to rank r) and pairwise swaps (contigs t, u of different
    ranks); returns the local optimum (assignment, loads).  At most 4 n
    improving steps (each strictly lowers the objective, so it ends anyway;
    the cap bounds the time)."""
    import numpy as np
    n = len(x)
    a = np.array(a, dtype=np.int64)
    loads = np.bincount(a, weights=x, minlength=world)
    idx = np.arange(n)
    for _ in range(4 * n + 4):
        own = loads[a]
        dm = (own[:, None] - x[:, None]) ** 2 + (loads[None, :] + x[:, None]) ** 2 \
            - own[:, None] ** 2 - loads[None, :] ** 2
        dm[idx, a] = 0.0
        d = x[:, None] - x[None, :]
        ds = (own[:, None] - d) ** 2 + (own[None, :] + d) ** 2 - own[:, None] ** 2 - own[None, :] ** 2
        ds[a[:, None] == a[None, :]] = 0.0
        i = np.unravel_index(int(np.argmin(dm)), dm.shape)
        j = np.unravel_index(int(np.argmin(ds)), ds.shape)
        if min(dm[i], ds[j]) >= -1e-12:
            return a, loads
        if dm[i] <= ds[j]:
            t, r = i
            loads[a[t]] -= x[t]
            loads[r] += x[t]
            a[t] = r
        else:
            t, u = j
            o, r = a[t], a[u]
            loads[o] += x[u] - x[t]
            loads[r] += x[t] - x[u]
            a[t], a[u] = r, o
    return a, loads


def shard_contigs(lengths, world: int, restarts: int = 200, seed: int = 12345):
    """Assign contig indices to ``world`` ranks: greedy LPT by length, improved
    by local search from the LPT start and ``restarts`` seeded random starts;
    the plan with the smallest maximum load wins (ties: the first found).

    Returns a list (per rank) of contig indices in ascending contig order, so a
    rank's output is already in (tid, pos) order and the global output is the
    merge of the per-rank streams by tid.  ``restarts=0`` is LPT + descent.
    """
    import numpy as np
    if world < 1:
        raise ValueError("world must be >= 1")
    if len(lengths) == 0:
        return [[] for _ in range(world)]
    x = np.asarray([float(v) for v in lengths], dtype=np.float64)
    x = x / max(x.max(), 1.0)
    if len(x) > LOCAL_SEARCH_MAX:               # large assemblies: LPT only
        plan = [[] for _ in range(world)]
        for tid, r in enumerate(_lpt(lengths, world)):
            plan[r].append(tid)
        return [sorted(p) for p in plan]
    a, loads = _descend(x, _lpt(lengths, world), world)
    best = (float(loads.max()), a.copy())
    rng = np.random.default_rng(seed)
    for _ in range(restarts if world > 1 else 0):
        a, loads = _descend(x, rng.integers(0, world, len(x)), world)
        if float(loads.max()) < best[0] - 1e-12:
            best = (float(loads.max()), a.copy())
    plan = [[] for _ in range(world)]
    for tid, r in enumerate(best[1]):
        plan[int(r)].append(tid)
    return [sorted(p) for p in plan]


def plan_imbalance(lengths, plan):
    """max rank load / mean rank load of a plan (1.0 = perfectly balanced)."""
    loads = [sum(int(lengths[t]) for t in p) for p in plan]
    mean = sum(loads) / max(1, len(loads))
    return max(loads) / mean if mean else 1.0


def shard_range(n_sites: int, world: int, rank: int):
    """[first, last) of rank's contiguous share of n_sites."""
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    base, extra = divmod(n_sites, world)
    first = rank * base + min(rank, extra)
    return first, first + base + (1 if rank < extra else 0)


def aggregate(elapsed_s: float, sites: float, world: int):
    """(max elapsed, total sites, sites/s) across ranks of the default process
    group; a single process when world == 1."""
    if world <= 1:
        return elapsed_s, float(sites), float(sites) / elapsed_s
    import torch
    import torch.distributed as dist
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([elapsed_s], dtype=torch.float64, device=dev)
    s = torch.tensor([float(sites)], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    return float(t.item()), float(s.item()), float(s.item()) / float(t.item())
