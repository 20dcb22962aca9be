"""world_size-2 rehearsal of the multi-GPU path on CPU (gloo): each rank replays its shard of
the global document space and rank 0 gathers the per-document digests; the union must equal
one process replaying every document.  The per-rank engine here is the oracle (the test
checker) since there is no GPU; the sharding and gather code is the product's
(fluidframework_amd/shard.py, also used by bench.py over RCCL)."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

import oracle_ffi as O
from fluidframework_amd import shard
from snapdigest import bytes_digest

WORLD, DOCS, OPS = 2, 6, 300


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _replay(first, n):
    p = O.gen_params(OPS, pct_insert=55, pct_remove=35, seed=0x5EED)
    ops, text, props, off = O.gen_batch(p, n, first_doc=first)
    t, names = O.gen_tables(), O.gen_client_names(8)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names, n_threads=1)
    snap = np.array([bytes_digest("".join(O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names)
                                          .snapshot_v1().values()).encode("utf-8")) for d in range(n)], np.uint64)
    return dig, st, snap


def _rank(rank, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    dig, st, snap = _replay(shard.shard(rank, DOCS), DOCS)
    res = shard.gather_results(torch.from_numpy(dig.view(np.int64)), torch.from_numpy(st), WORLD, rank,
                               torch.from_numpy(snap.view(np.int64)))
    if rank == 0:
        np.savez(out_path, dig=res[0], st=res[1], snap=res[2])
    else:
        assert res is None
    dist.destroy_process_group()


def test_gather_over_gloo_equals_single_process(tmp_path):
    out = tmp_path / "gathered.npz"
    mp.spawn(_rank, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    dig, st, snap = _replay(0, WORLD * DOCS)
    assert (got["st"] == st).all() and (st == 0).all()
    assert (got["dig"] == dig).all()
    assert (got["snap"] == snap).all()
    assert len(set(got["dig"].tolist())) == WORLD * DOCS  # documents differ: the shards are disjoint


def test_shard_ranges_partition_the_document_space():
    firsts = [shard.shard(r, 1000) for r in range(8)]
    assert firsts == [r * 1000 for r in range(8)]


def test_zipf_sizes_are_deterministic_and_bounded():
    z = shard.zipf_sizes(5000, 1000, 200000, 1.1)
    assert (z == shard.zipf_sizes(5000, 1000, 200000, 1.1)).all()
    assert z.max() == 200000 and z.min() == 1000
    top = np.sort(z)[::-1]
    assert top[1] == int(200000 * 2 ** -1.1) and top[9] == int(200000 * 10 ** -1.1)
    assert np.argmax(z) != 0  # ranks are permuted over the document ids


def test_lpt_assigns_every_document_once_and_balances():
    costs = shard.zipf_sizes(4000, 100, 50000, 1.1)
    parts, loads = shard.lpt(costs, 8)
    allp = np.concatenate(parts)
    assert sorted(allp.tolist()) == list(range(4000))
    assert loads == [int(costs[q].sum()) for q in parts]
    assert max(loads) - min(loads) <= costs.max()  # greedy LPT bound
    for q in parts:
        assert (np.diff(costs[q]) <= 0).all()  # each rank launches its largest documents first


def _rank_uneven(rank, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    sizes = shard.zipf_sizes(11, 50, 900, 1.1)
    parts, _ = shard.lpt(sizes, WORLD)
    mine = parts[rank]
    dig = (mine.astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)).view(np.int64)
    res = shard.gather_results(torch.from_numpy(dig), torch.from_numpy(np.zeros(len(mine), np.int32)), WORLD, rank,
                               counts=[len(q) for q in parts])
    if rank == 0:
        np.savez(out_path, dig=res[0], ids=np.concatenate(parts))
    dist.destroy_process_group()


def test_gather_with_uneven_lpt_shards(tmp_path):
    out = tmp_path / "uneven.npz"
    mp.spawn(_rank_uneven, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    assert len(got["dig"]) == 11
    with np.errstate(over="ignore"):
        assert (got["dig"] == got["ids"].astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)).all()


def _rank_summaries(rank, port, out_path):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    p = O.gen_params(OPS, pct_insert=55, pct_remove=35, seed=0x5EED)
    first = shard.shard(rank, DOCS)
    ops, text, props, off = O.gen_batch(p, DOCS, first_doc=first)
    t, names = O.gen_tables(), O.gen_client_names(8)
    # this rank's SnapshotV1 summaries, back to back (the layout of the GPU snapshot buffer)
    blob = "".join("".join(O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names).snapshot_v1().values())
                   for d in range(DOCS)).encode("utf-8")
    blob = blob[: len(blob) - 37 * rank]  # uneven sizes across ranks
    got = shard.gather_bytes(torch.frombuffer(bytearray(blob), dtype=torch.uint8), WORLD, rank)
    if rank == 0:
        np.savez(out_path, *[g.numpy() for g in got])
    else:
        assert got is None
    dist.destroy_process_group()


def test_summaries_gather_over_gloo(tmp_path):
    """SnapshotV1 summaries (variable-size byte buffers) reach rank 0 intact, in rank order."""
    out = tmp_path / "summaries.npz"
    mp.spawn(_rank_summaries, args=(_free_port(), str(out)), nprocs=WORLD, join=True)
    got = np.load(out)
    p = O.gen_params(OPS, pct_insert=55, pct_remove=35, seed=0x5EED)
    t, names = O.gen_tables(), O.gen_client_names(8)
    for r in range(WORLD):
        ops, text, props, off = O.gen_batch(p, DOCS, first_doc=shard.shard(r, DOCS))
        want = "".join("".join(O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names).snapshot_v1()
                               .values()) for d in range(DOCS)).encode("utf-8")
        want = want[: len(want) - 37 * r]
        assert got[f"arr_{r}"].tobytes() == want


def test_bench_gpus_flag_spawns_ranks():
    """`bench.py --gpus 2` with no outer launcher starts two rank processes itself (RANK /
    WORLD_SIZE / MASTER_* set, Popen, never exec); --launch-check runs the rank layout and the
    gather to rank 0 over gloo without a replay, so the CPU suite can see n_gpus and the gather."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["MT_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_gathered"] == 2
    assert line["digests_gathered"] == 8 and line["digests_in_order"]


def test_bench_rejects_world_size_mismatch():
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MT_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "4", "--launch-check"], env=env,
                       capture_output=True, text=True, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr
