"""Genome sharding across GPUs (one process per GPU, no data-path collectives).

Sites are independent (glf_somatic keeps no state across sites except the cached
contig string, somatic_sniper.c:112-117), so a run is split into genome regions
and every rank scores its own regions end to end.  The only cross-rank traffic is
the barrier and the max-over-ranks timing reduction of the benchmark, and the
host-side concatenation of per-rank outputs in (tid, pos) order.

* ``shard_contigs``  longest-processing-time assignment of contigs to ranks
  (SURVEY.md section 8(e)), deterministic for a given (lengths, world).
* ``shard_range``    contiguous equal split of a site range (synthetic shards).
* ``aggregate``      whole-job throughput from per-rank (elapsed, sites) with the
  bench contract: time = max over ranks, sites = sum over ranks.
"""
from __future__ import annotations

import heapq


def shard_contigs(lengths, world: int):
    """Assign contig indices to ``world`` ranks, greedy LPT by length.

    Returns a list (per rank) of contig indices in ascending contig order, so a
    rank's output is already in (tid, pos) order and the global output is the
    merge of the per-rank streams by tid.
    """
    if world < 1:
        raise ValueError("world must be >= 1")
    heap = [(0, r) for r in range(world)]
    heapq.heapify(heap)
    plan = [[] for _ in range(world)]
    for tid in sorted(range(len(lengths)), key=lambda t: (-int(lengths[t]), t)):
        load, r = heapq.heappop(heap)
        plan[r].append(tid)
        heapq.heappush(heap, (load + int(lengths[tid]), r))
    return [sorted(p) for p in plan]


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
