"""The multi-GPU path with the HIP engine in every rank (world_size 2 on the box's one MI355X, the
gather over gloo): each rank generates and replays its shard of the global document space on the
GPU (the same calls bench.py makes per rank), digests and statuses are gathered to rank 0 by
fluidframework_amd/shard.py, and the union equals one process replaying every document and the
oracle on the downloaded logs.  RCCL itself needs one GPU per rank, which the round's one-GPU box
does not have; the gather code is the same for both backends (tensors on the device for "nccl")."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle_ffi as O
import fluidframework_amd as fa
from fluidframework_amd import shard

pytestmark = pytest.mark.gpu

WORLD, DOCS, OPS = 2, 96, 1500
GEN = dict(pct_insert=55, pct_remove=35, seed=0x5EED)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank(rank, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    with fa.ReplayBatch(DOCS) as b:
        b.generate(fa.gen_params(OPS, **GEN), shard.shard(rank, DOCS))
        b.run()
        dig = torch.from_numpy(b.device_digests().view(np.int64))
        st = torch.from_numpy(b.counters()["status"].astype(np.int64))
    res = shard.gather_results(dig, st, WORLD, rank)
    if rank == 0:
        np.savez(out_path, dig=np.asarray(res[0]), st=np.asarray(res[1]))
    else:
        assert res is None
    dist.destroy_process_group()


def test_hip_ranks_gather_equals_single_process(tmp_path):
    out = tmp_path / "gathered.npz"
    mp.spawn(_rank, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    with fa.ReplayBatch(WORLD * DOCS) as b:
        b.generate(fa.gen_params(OPS, **GEN), 0)
        ops, off, text, props = b.download_log()
        b.run()
        one = b.device_digests()
        host = np.array([b.doc(d).digest() for d in range(WORLD * DOCS)], np.uint64)
    assert (got["st"] == 0).all()
    assert (got["dig"].view(np.uint64) == one).all()
    assert len(set(one.tolist())) == WORLD * DOCS  # the shards are disjoint documents
    _, dig, st = O.replay_batch(ops, off, text, props, O.gen_tables(), O.gen_client_names(8))
    assert (st == 0).all() and (dig == host).all()
