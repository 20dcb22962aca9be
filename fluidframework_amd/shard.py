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


def gather_results(digests, statuses, world: int, rank: int, snapshot_digests=None):
    """Gather per-document (digest, status[, SnapshotV1 digest]) to rank 0.

    digests: int64 tensor [D] (uint64 digests viewed as int64), statuses: int tensor [D],
    snapshot_digests: optional int64 tensor [D] (mt_batch_snapshot_digests), all on the
    backend's device.  Returns (digests uint64 [W*D], statuses int32 [W*D][, snapshot digests
    uint64 [W*D]]) in global document order on rank 0, None on the other ranks."""
    import torch
    import torch.distributed as dist

    cols = [digests.to(torch.int64), statuses.to(torch.int64)]
    if snapshot_digests is not None:
        cols.append(snapshot_digests.to(torch.int64))
    rec = torch.stack(cols, 1).contiguous()
    if world == 1:
        parts = [rec]
    else:
        parts = [torch.empty_like(rec) for _ in range(world)] if rank == 0 else None
        dist.gather(rec, parts, dst=0)
    if rank != 0:
        return None
    allr = torch.cat(parts, 0).cpu().numpy()
    out = (allr[:, 0].copy().view(np.uint64), allr[:, 1].astype(np.int32))
    if snapshot_digests is not None:
        out += (allr[:, 2].copy().view(np.uint64),)
    return out
