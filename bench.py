#!/usr/bin/env python3
"""Benchmark: sequenced merge-tree ops/sec of the MI355X batch replay engine.

One step = one replay (mt_replay_kernel) of every document of this rank's batch, starting
from empty documents, with the synthetic op logs already resident in HBM.  Workload
(BASELINE.json configs[1]): 4,096 docs x 2,000 text-only insert/removeRange ops per GPU,
8 writer clients, refSeq lag <= 32; `--config 3` selects configs[2]'s op mix
(65,536 docs x 10k ops, 10% annotate) scaled per GPU with --docs/--ops.

Multi-GPU: one process per GPU (torchrun); documents shard across ranks with no data-path
collective (weak scaling); after the timed steps rank 0 gathers per-document results with
RCCL (torch.distributed "nccl").  rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md: 8.0 TB/s spec)

CONFIGS = {
    2: dict(docs=4096, ops=2000, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40,
            workload="configs[1]: 4,096 docs x 2k text-only insert/removeRange ops, 8 clients, refSeq lag<=32"),
    3: dict(docs=8192, ops=10000, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35,
            workload="configs[2] mix: docs x 10k ops, 10% annotate, minSeq advance/zamboni, 8 clients"),
    4: dict(docs=16384, ops=200000, ops_min=1000, zipf_s=1.1, n_clients=8, max_lag=32, pct_insert=70, pct_remove=20,
            workload="configs[3]: Zipf(s=1.1) document sizes by rank over [1k, 200k] ops (70/20/10 mix), "
                     "16,384 docs per GPU, LPT-balanced across GPUs, largest documents through the LDS ladder "
                     "and the HBM spill class"),
    5: dict(docs=131072, ops=2000, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35, snapshot=True,
            workload="configs[4]: 1M docs over 8 GPUs (131,072 per GPU) x 2k ops (10% annotate), full replay + "
                     "SnapshotV1 of every doc on the GPU in each step, digests gathered to rank 0"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=2, choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="documents per GPU (default: config)")
    ap.add_argument("--ops", type=int, default=0, help="ops per document (default: config)")
    ap.add_argument("--seed", type=int, default=0xDEADBEEF)
    ap.add_argument("--cpu-sample-docs", type=int, default=0, help="oracle baseline sample (default: auto)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--snapshot", action="store_true", help="serialize SnapshotV1 of every doc in each step")
    return ap.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MT_BENCH_BACKEND=gloo rehearses the multi-rank path with ranks sharing GPUs (RCCL needs
    # one rank per device); the real runs use "nccl" (= RCCL) with one process per GPU
    backend = os.environ.get("MT_BENCH_BACKEND", "nccl")
    dev = local_rank % max(1, torch.cuda.device_count())
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(dev)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    torch.cuda.init()

    import __graft_entry__ as g

    # the library is built in-tree beforehand (build()); ranks never compile concurrently
    if not g.LIB.exists():
        if rank == 0:
            g.build_lib()
        if world > 1:
            dist.barrier()
    import fluidframework_amd as fa

    cfg = dict(CONFIGS[args.config])
    n_docs = args.docs or cfg["docs"]
    n_ops = args.ops or cfg["ops"]
    p = fa.gen_params(n_ops, n_clients=cfg["n_clients"], max_lag=cfg["max_lag"], pct_insert=cfg["pct_insert"],
                      pct_remove=cfg["pct_remove"], seed=args.seed)
    from fluidframework_amd import shard

    sizes = None
    if "zipf_s" in cfg:  # config 4: Zipf sizes over the global documents, LPT across ranks
        all_sizes = shard.zipf_sizes(n_docs * world, cfg["ops_min"], n_ops, cfg["zipf_s"])
        parts, loads = shard.lpt(all_sizes, world)
        my_docs = parts[rank]
        sizes = all_sizes[my_docs]
        counts = [len(q) for q in parts]
        total_ops_step = int(all_sizes.sum())
        n_docs = len(my_docs)
    else:
        doc_first = shard.shard(rank, n_docs)  # disjoint shard of the global document space
        counts = None
        total_ops_step = n_ops * n_docs * world

    b = fa.ReplayBatch(n_docs)
    t0 = time.time()
    if sizes is not None:
        b.generate_docs(p, my_docs, sizes)
    else:
        b.generate(p, doc_first)  # synthesize this rank's logs on the GPU (untimed)
    gen_s = time.time() - t0
    log(rank, f"generated {n_docs} docs, {int(b.stats()['n_ops'])} ops in {gen_s:.1f} s")
    stream = torch.cuda.current_stream().cuda_stream

    with_snap = args.snapshot or cfg.get("snapshot", False)
    for i in range(args.warmup):
        b.run(stream)
        if with_snap:
            b.snapshots()
        log(rank, f"warmup {i}: {b.stats()['kernel_ms']:.1f} ms kernel")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms, first_ms, first_ops, snap_ms, snap_bytes = [], [], [], [], 0
    for i in range(args.steps):
        b.run(stream)
        kernel_ms.append(b.stats()["kernel_ms"])
        # the dominant kernel: the launch that applied the most ops (launch 0 in uniform batches)
        l0 = max(b.launches(), key=lambda li: li["ops"])
        first_ms.append(l0["ms"])
        first_ops.append(l0["ops"])
        dom_class = l0["seg_class"]
        if with_snap:  # SnapshotV1 of every document, part of the step
            sn = b.snapshots()
            snap_ms.append(sn["device_ms"])
            snap_bytes = sn["bytes"]
        log(rank, f"step {i}: {kernel_ms[-1]:.1f} ms kernel" + (f", {snap_ms[-1]:.1f} ms snapshot" if with_snap else ""))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = elapsed
    if world > 1:
        t = torch.tensor([elapsed], device="cuda" if backend == "nccl" else "cpu", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())

    st = b.stats()
    statuses = b.statuses()
    import numpy as np

    cnt = b.counters()
    capacity = {f: [int(np.percentile(cnt[f], q)) for q in (50, 99, 100)]
                for f in ("max_slots", "max_unsettled", "max_blocks", "max_heap")}
    ops_done = st["ops_applied"]
    # gather the per-document device digests and statuses to rank 0 over RCCL (untimed)
    dig_t = torch.empty(n_docs, dtype=torch.int64, device="cuda")
    b.device_digests(dig_t)
    st_t = torch.from_numpy(statuses.astype("int64")).cuda()
    torch.cuda.synchronize()
    tg = time.perf_counter()
    snap_t = None
    if with_snap:  # per-document digest of the GPU SnapshotV1 bytes, gathered with the rest
        snap_t = torch.empty(n_docs, dtype=torch.int64, device="cuda")
        b.snapshot_digests(snap_t)
        torch.cuda.synchronize()
        tg = time.perf_counter()
    gathered = shard.gather_results(dig_t, st_t, world, rank, snap_t, counts)
    torch.cuda.synchronize()
    gather_ms = 1e3 * (time.perf_counter() - tg)
    all_ok, digest_xor, snap_xor = 0, None, None
    if rank == 0:
        all_dig, all_st = gathered[:2]
        all_ok = int((all_st == 0).all())
        digest_xor = f"{int(np.bitwise_xor.reduce(all_dig)):016x}"
        if with_snap:
            snap_xor = f"{int(np.bitwise_xor.reduce(gathered[2])):016x}"
    total_ops = total_ops_step * args.steps
    value = total_ops / t_max
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    alg_bytes = b.algorithmic_bytes()
    # roofline of the dominant kernel (launch 0, mt_replay_kernel_<class>): the algorithmic bytes
    # of the ops it applied (DESIGN.md "Roofline": per-op share of the batch's algorithmic bytes)
    # over its average launch duration (hipEvents on the run stream)
    avg_first_ms = sum(first_ms) / len(first_ms)
    first_bytes = alg_bytes * (sum(first_ops) / len(first_ops)) / max(1, ops_done)
    achieved_gbs = first_bytes / (avg_first_ms * 1e-3) / 1e9

    traffic, traffic_src = pmc_traffic(args.config, n_docs, n_ops, f"mt_replay_kernel_{dom_class}")
    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu:
        cpu, parity = cpu_baseline(b, fa, n_docs, args)
    snapshot = None
    if with_snap:
        avg_snap = sum(snap_ms) / len(snap_ms)
        snapshot = {"bytes_per_step": int(snap_bytes), "avg_device_ms": round(avg_snap, 3),
                    "GB_per_s": round(snap_bytes / (avg_snap * 1e-3) / 1e9, 3), "kernel": "mt_snapshot_kernel"}
        if rank == 0:  # spot check: GPU blobs == host serializer on a sample
            sample = range(0, n_docs, max(1, n_docs // 64))
            snapshot["host_match"] = sum(b.doc(d).snapshot_v1(device=True) == b.doc(d).snapshot_v1() for d in sample)
            snapshot["checked"] = len(sample)

    if rank == 0:
        line = {
            "metric": "sequenced merge-tree ops/sec",
            "value": round(value, 1),
            "unit": "ops/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * t_max / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (GPU-generated conflict-farm logs, include/mt_gen.h)",
            "config": {"workload": cfg["workload"], "docs_per_gpu": n_docs,
                       "ops_per_doc": n_ops if sizes is None else {"min": int(sizes.min()), "max": int(sizes.max()),
                                                                  "lpt_loads": loads},
                       "clients": cfg["n_clients"], "max_lag": cfg["max_lag"],
                       "op_mix": [cfg["pct_insert"], cfg["pct_remove"], 100 - cfg["pct_insert"] - cfg["pct_remove"]],
                       "parallelism": f"doc-sharded x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": f"mt_replay_kernel_{dom_class}", "avg_launch_ms": round(avg_first_ms, 3),
                         "algorithmic_bytes_per_launch": int(first_bytes),
                         "ops_per_launch": int(sum(first_ops) / len(first_ops))},
            "replay_ms_per_step": round(avg_kernel_ms, 3),
            "launches": b.launches(),
            "cpu_baseline": cpu,
            "parity": parity,
            "snapshot": snapshot,
            "docs_ok": all_ok,
            "digests_gathered": len(gathered[0]) if rank == 0 else None,
            "digest_xor": digest_xor,
            "snapshot_digest_xor": snap_xor,
            "ops_applied_per_step": int(ops_done),
            "lds_bytes_per_doc": st["lds_bytes"],
            "launches_per_step": st["launches"],
            "capacity_p50_p99_max": capacity,
            "gen_s": round(gen_s, 2),
            "gather_ms": round(gather_ms, 3),
        }
        print(json.dumps(line), flush=True)
    b.close()
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(config, n_docs, n_ops, kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes of this same configuration (tools/pmc_traffic.py; scripts/gpu_check.sh pmcf pmcw).
    The counters cannot be read from inside this process, so the profile of the current kernel
    build is committed under profiles/ and quoted here; None when no matching profile exists."""
    path = ROOT / "profiles" / f"pmc_traffic_config{config}.json"
    try:
        prof = json.loads(path.read_text())
    except (OSError, ValueError):
        return None, None
    if prof.get("docs") != n_docs or prof.get("ops") != n_ops or kernel not in prof.get("kernels", {}):
        return None, None
    return int(prof["kernels"][kernel]["traffic_bytes"]), str(path.relative_to(ROOT))


def log(rank, msg):
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_baseline(b, fa, n_docs, args):
    """Oracle (CPU restatement, tests-only code) on a bounded sample of the same logs,
    timed on this host's cores; its per-doc digests double as a parity spot check.
    Sample: the first documents of this rank's batch up to ~8.2M ops (config 2's size)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np

    import oracle_ffi as O

    ops, off, text, props = b.download_log()
    if args.cpu_sample_docs:
        sample = min(args.cpu_sample_docs, n_docs)
    else:
        sample = int(np.searchsorted(off, 4096 * 2000, side="left"))
        sample = min(n_docs, max(16, sample))
    end = off[sample]
    sops = ops[:end].copy()
    soff = off[: sample + 1].copy()
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    tables, names = O.gen_tables(), O.gen_client_names(8)
    secs, dig, st = O.replay_batch(sops, soff, text, props, tables, names, n_threads=threads)
    gpu_dig = np.array([b.doc(d).digest() for d in range(sample)], np.uint64)
    match = int((gpu_dig == dig).sum())
    cpu = {"value": round(int(end) / secs, 1), "unit": "ops/s", "cores": threads, "kind": "port",
           "sample": f"first {sample} docs ({int(end)} ops) of the same log, oracle/ C restatement, {threads} threads",
           "seconds": round(secs, 3)}
    parity = {"docs_checked": sample, "digest_match": match, "oracle_status_ok": int((st == 0).sum())}
    return cpu, parity


if __name__ == "__main__":
    main()
