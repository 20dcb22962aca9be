"""The multi-GPU path with the HIP engine in every rank (world_size 2 on the box's one MI355X, the
gather over gloo): each rank generates and replays its shard of the global document space on the
GPU (the same calls bench.py makes per rank), digests and statuses are gathered to rank 0 by
fluidframework_amd/shard.py, and the union equals one process replaying every document and the
oracle on the downloaded logs.  RCCL needs one GPU per rank, which the one-GPU box does not have for
two ranks: the RCCL test runs the same gathers through a one-rank "nccl" process group, so the
collectives execute in RCCL on the device tensors."""
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


def _rccl_rank(rank, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    with fa.ReplayBatch(DOCS) as b:
        b.generate(fa.gen_params(OPS, **GEN), 0)
        b.run()
        dig_np = b.device_digests()
        dig = torch.from_numpy(dig_np.view(np.int64)).cuda()
        st = torch.from_numpy(b.counters()["status"].astype(np.int64)).cuda()
        snap = b.doc(0).snapshot_v1()["header"].encode()
    res = shard.gather_results(dig, st, 1, 0)
    blobs = shard.gather_bytes(torch.tensor(list(snap), dtype=torch.uint8, device="cuda"), 1, 0)
    np.savez(out_path, dig=np.asarray(res[0]), st=np.asarray(res[1]), local=dig_np,
             blob=blobs[0].cpu().numpy(), snap=np.frombuffer(snap, np.uint8))
    dist.destroy_process_group()


def test_rccl_gathers_one_rank_group(tmp_path):
    """shard.gather_results / gather_bytes through a one-rank "nccl" (RCCL) process group on the
    device: the gathered digests, statuses and bytes equal the local ones."""
    out = tmp_path / "rccl.npz"
    mp.spawn(_rccl_rank, args=(_free_port(), str(out)), nprocs=1, join=True)
    got = np.load(out)
    assert (got["st"] == 0).all()
    assert (got["dig"].view(np.uint64) == got["local"]).all()
    assert got["blob"].tobytes() == got["snap"].tobytes()
