"""Document sharding across ranks and the path's single collective (gather to rank 0).

Documents are independent replicas (each merge-tree ``Client`` is self-contained,
packages/dds/merge-tree/src/client.ts:42-83), so the replay shards by document with no
collective on the data path: rank r of W owns the global documents [r*D, (r+1)*D) and
generates / ingests exactly those.  After the replay, rank 0 gathers a fixed-size record per
document — the 8-byte device digest and the status — with one
``dist.gather``: RCCL over xGMI on the GPU box (backend "nccl", CUDA tensors), gloo on CPU.
"""
from __future__ import annotations

import numpy as np


def shard(rank: int, docs_per_rank: int) -> int:
    """Global index of this rank's first document."""
    return rank * docs_per_rank


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def zipf_sizes(n_docs: int, n_min: int, n_max: int, s: float = 1.1, seed: int = 0x5A1F) -> np.ndarray:
    """Config 4 document sizes (ops per document) for the global document space: the document
    of Zipf rank r (1-based) gets max(n_min, floor(n_max * r**-s)) ops, and ranks are a seeded
    permutation of the document ids (documents sorted by splitmix64(seed ^ id)), so the few
    large documents are scattered over the id space."""
    ids = np.arange(n_docs, dtype=np.uint64)
    order = np.argsort(_splitmix64(ids ^ np.uint64(seed)), kind="stable")
    rank = np.empty(n_docs, np.float64)
    rank[order] = np.arange(1, n_docs + 1, dtype=np.float64)
    return np.maximum(n_min, np.floor(n_max * rank ** -s)).astype(np.int32)


def lpt(costs, world: int):
    """Greedy longest-processing-time assignment of documents to ranks: documents
    in decreasing cost go to the least-loaded rank (ties: lowest rank).  Returns (per-rank arrays of
    global document ids, each in decreasing cost — the order a rank launches them in — and the
    per-rank loads).  Cost = ops per document (per-op cost grows only with tree depth)."""
    import heapq

    costs = np.asarray(costs)
    order = np.argsort(-costs, kind="stable")
    heap = [(0, r) for r in range(world)]
    parts = [[] for _ in range(world)]
    for d in order:
        load, r = heapq.heappop(heap)
        parts[r].append(int(d))
        heapq.heappush(heap, (load + int(costs[d]), r))
    loads = [int(costs[p].sum()) if p else 0 for p in parts]
    return [np.array(p, np.int64) for p in parts], loads


def gather_results(digests, statuses, world: int, rank: int, snapshot_digests=None, counts=None):
    """Gather per-document (digest, status[, SnapshotV1 digest]) to rank 0.

    digests: int64 tensor [D] (uint64 digests viewed as int64), statuses: int tensor [D],
    snapshot_digests: optional int64 tensor [D] (mt_batch_snapshot_digests), all on the
    backend's device.  Returns (digests uint64 [W*D], statuses int32 [W*D][, snapshot digests
    uint64 [W*D]]) in rank order on rank 0 (the global document order for contiguous shards),
    None on the other ranks.  counts: per-rank document counts when they differ (LPT shards):
    every rank pads to the largest and rank 0 trims each part back."""
    import torch
    import torch.distributed as dist

    cols = [digests.to(torch.int64), statuses.to(torch.int64)]
    if snapshot_digests is not None:
        cols.append(snapshot_digests.to(torch.int64))
    rec = torch.stack(cols, 1).contiguous()
    if world > 1 and dist.get_backend() == "gloo":
        rec = rec.cpu()  # gloo gathers host tensors
    if counts is not None and max(counts) > rec.shape[0]:
        rec = torch.cat([rec, rec.new_zeros((max(counts) - rec.shape[0], rec.shape[1]))], 0)
    if world == 1 and not dist.is_initialized():
        parts = [rec]
    else:  # through the process group (also a one-rank RCCL group: the collective runs)
        parts = [torch.empty_like(rec) for _ in range(world)] if rank == 0 else None
        dist.gather(rec, parts, dst=0)
    if rank != 0:
        return None
    if counts is not None:
        parts = [q[: counts[r]] for r, q in enumerate(parts)]
    allr = torch.cat(parts, 0).cpu().numpy()
    out = (allr[:, 0].copy().view(np.uint64), allr[:, 1].astype(np.int32))
    if snapshot_digests is not None:
        out += (allr[:, 2].copy().view(np.uint64),)
    return out


def gather_bytes(buf, world: int, rank: int):
    """Gather each rank's byte buffer (a 1-D uint8 tensor of any length; SnapshotV1 summaries) to
    rank 0: one all_gather of the lengths, then one dist.gather of the buffers padded to the
    longest (RCCL on the GPU box, gloo on CPU).  Returns the per-rank buffers (trimmed) on rank 0,
    None elsewhere."""
    import torch
    import torch.distributed as dist

    if world == 1 and not dist.is_initialized():
        return [buf]
    n = torch.tensor([buf.numel()], dtype=torch.int64, device=buf.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n)
    sizes = [int(x.item()) for x in sizes]
    m = max(1, max(sizes))
    pad = torch.zeros(m, dtype=torch.uint8, device=buf.device)
    pad[: buf.numel()] = buf
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == 0 else None
    dist.gather(pad, parts, dst=0)
    if rank != 0:
        return None
    return [q[: sizes[r]] for r, q in enumerate(parts)]
