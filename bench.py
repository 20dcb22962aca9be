#!/usr/bin/env python3
"""Benchmark: sequenced merge-tree ops/sec of the MI355X batch replay engine.

One step = one replay (mt_replay_kernel, every capacity-class launch) of every document of this
rank's batch from empty documents, with the synthetic op logs already resident in HBM, then the
per-document device digests (mt_digest_kernel) and their gather to rank 0 — SURVEY.md §8(d):
"wall-clock from ingested logs in HBM to final state plus digests on rank 0".

Default workload = the north-star headline, BASELINE.json configs[2]: 65,536 documents x 10,000
ops per GPU (insert 55 / remove 35 / annotate 10, 8 writer clients, refSeq lag <= 32, minSeq
advancing with zamboni).  `--config 2` = configs[1] (4,096 docs x 2k text-only ops),
`--config 4` = configs[3] (Zipf sizes), `--config 5` = configs[4] (+ SnapshotV1 of every document).

Multi-GPU: one process per GPU (torchrun); documents shard across ranks with no data-path
collective (weak scaling); rank 0 gathers per-document results with RCCL (torch.distributed
"nccl").  rank 0 prints ONE JSON line.
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
N_CUS, CLOCK_GHZ = 256, 2.4  # MI355X_MICROARCH.md: 256 CUs, ~2.4 GHz shader clock

CONFIGS = {
    2: dict(docs=4096, ops=2000, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40,
            workload="configs[1]: 4,096 docs x 2k text-only insert/removeRange ops, 8 clients, refSeq lag<=32"),
    3: dict(docs=65536, ops=10000, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35,
            workload="configs[2]: 65,536 docs x 10k ops per GPU, insert 55 / remove 35 / annotate 10, "
                     "minSeq advance + zamboni, 8 clients, refSeq lag<=32"),
    4: dict(docs=16384, ops=2000000, ops_min=1000, zipf_s=1.1, n_clients=8, max_lag=32, pct_insert=50, pct_remove=15,
            workload="configs[3]: Zipf(s=1.1) document sizes by rank over [1k, 2M] ops (insert 50 / remove 15 / "
                     "annotate 35: props keep segments apart, so the largest documents reach ~10^6 segments), "
                     "16,384 docs per GPU, LPT-balanced across GPUs; the largest documents run the LDS ladder, "
                     "then the HBM class (2M slots)"),
    5: dict(docs=131072, ops=2000, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35, snapshot=True,
            workload="configs[4]: 1M docs over 8 GPUs (131,072 per GPU) x 2k ops (10% annotate), full replay + "
                     "SnapshotV1 of every doc on the GPU in each step, digests gathered to rank 0"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, default=3, choices=sorted(CONFIGS))
    ap.add_argument("--docs", type=int, default=0, help="documents per GPU (default: config)")
    ap.add_argument("--ops", type=int, default=0, help="ops per document (default: config)")
    ap.add_argument("--seed", type=int, default=0xDEADBEEF)
    ap.add_argument("--cpu-sample-docs", type=int, default=0, help="oracle baseline sample (default: auto)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (default: every usable core)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--seg-cap", type=int, default=0, help="first capacity class (default: from the op count)")
    ap.add_argument("--snapshot", action="store_true", help="serialize SnapshotV1 of every doc in each step")
    ap.add_argument("--launch-check", action="store_true",
                    help="rank layout + gather to rank 0 only, no replay (tests the --gpus N launcher on CPU)")
    ap.add_argument("--writers", action="store_true",
                    help="replay every document as one of its writers (local ops + acks, the local-client path)")
    return ap.parse_args()


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def spawn_ranks(n: int) -> int:
    """`bench.py --gpus N` without an outer launcher: start N rank processes of this same command
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set, as torch.distributed.run
    would), before this process touches the GPU (it never does: children are started with Popen,
    never exec).  Rank 0 writes the JSON line to the inherited stdout.  Returns 0 when every rank
    succeeded, else the first failing rank's exit status (the other ranks are then stopped)."""
    import subprocess

    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve())] + sys.argv[1:], env=env))
    rc = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            code = p.poll()
            if code is None:
                continue
            pending.remove(p)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"[bench] rank {procs.index(p)} exited with status {code}; stopping the others",
                      file=sys.stderr, flush=True)
                for q in pending:
                    q.terminate()
        time.sleep(0.05)
    return rc


def launch_check(world, rank, backend):
    """--launch-check: the rank layout and the gather to rank 0 without a replay (the CPU suite's
    test of `--gpus N`): every rank contributes a digest per document of a 4-document shard and rank
    0 prints {"launch_check": ..., "n_gpus", "ranks_gathered", "digests_gathered"}."""
    import numpy as np
    import torch
    import torch.distributed as dist

    from fluidframework_amd import shard

    if world > 1:
        dist.init_process_group(backend)
    dig = torch.arange(4, dtype=torch.int64) + 4 * rank
    st = torch.zeros(4, dtype=torch.int64)
    g = shard.gather_results(dig, st, world, rank)
    ranks_gathered = dist.get_world_size() if dist.is_initialized() else 1
    if rank == 0:
        print(json.dumps({"launch_check": True, "n_gpus": world, "ranks_gathered": ranks_gathered,
                          "digests_gathered": int(len(g[0])),
                          "digests_in_order": bool((g[0].astype(np.int64) == np.arange(4 * world)).all())}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one rank per GPU)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # MT_BENCH_BACKEND=gloo rehearses the multi-rank path with ranks sharing GPUs (RCCL needs
    # one rank per device); the real runs use "nccl" (= RCCL) with one process per GPU
    backend = os.environ.get("MT_BENCH_BACKEND", "nccl")
    if args.launch_check:
        launch_check(world, rank, backend)
        return
    import torch
    import torch.distributed as dist

    if world > 1 and backend == "nccl" and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} RCCL ranks need {world} GPUs, {torch.cuda.device_count()} visible")
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

    import numpy as np

    b = fa.ReplayBatch(n_docs, seg_cap=args.seg_cap)
    t0 = time.time()
    if sizes is not None:
        b.generate_docs(p, my_docs, sizes)
    else:
        b.generate(p, doc_first)  # synthesize this rank's logs on the GPU (untimed)
    gen_s = time.time() - t0
    log(rank, f"generated {n_docs} docs, {int(b.stats()['n_ops'])} ops in {gen_s:.1f} s")
    writer_log = None
    if args.writers:
        # writer replicas of the same logs: document d is replayed as its writer 1 + d % C
        # (oplog.writer_records: local copies of its ops + its own messages as acks) on
        # mt_writer_kernel_<SEG>; the metric still counts the sequenced ops of the log
        from fluidframework_amd import oplog
        from fluidframework_amd.mtreplay import GEN_KEYS, GEN_VALUES, gen_client_names

        t0 = time.time()
        ops, off, text, props = b.download_log()
        b.close()
        wof = 1 + np.arange(n_docs) % cfg["n_clients"]
        wops, woff = oplog.writer_records(ops, off, wof)
        base = gen_client_names(cfg["n_clients"])
        b = fa.ReplayBatch(n_docs, seg_cap=args.seg_cap)
        b.set_tables(GEN_KEYS, GEN_VALUES)
        for d in range(n_docs):
            nm = list(base)
            nm[0], nm[int(wof[d])] = nm[int(wof[d])], nm[0]
            b.set_clients(nm, d)
        b.ingest(wops, woff, text, props)
        n_local = len(wops) - len(ops)
        writer_log = (wops, woff, text, props, wof, base)
        log(rank, f"writer logs: {len(wops)} records ({n_local} local ops) in {time.time() - t0:.1f} s")
    stream = torch.cuda.current_stream().cuda_stream

    with_snap = args.snapshot or cfg.get("snapshot", False)

    dig_t = torch.empty(n_docs, dtype=torch.int64, device="cuda")
    snap_t = torch.empty(n_docs, dtype=torch.int64, device="cuda") if with_snap else None

    def step():
        """replay + digests (+ SnapshotV1) of this rank's documents, gathered to rank 0"""
        b.run(stream)
        sn = b.snapshots() if with_snap else None
        b.device_digests(dig_t)
        if with_snap:
            b.snapshot_digests(snap_t)
        st_t = torch.from_numpy(b.counters()["status"].astype(np.int64)).to(dig_t.device)
        return sn, shard.gather_results(dig_t, st_t, world, rank, snap_t, counts)

    for i in range(args.warmup):
        step()
        log(rank, f"warmup {i}: {b.stats()['kernel_ms']:.1f} ms kernel")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms, first_ms, first_ops, snap_ms, snap_bytes = [], [], [], [], 0
    cls_span, cls_ops, cls_launches = [], [], []
    gathered = None
    for i in range(args.steps):
        sn, gathered = step()
        kernel_ms.append(b.stats()["kernel_ms"])
        # the dominant kernel: the launch that took the longest (config 4: the giant-class launch of
        # the Zipf tail, not the class that applied the most ops)
        lis = b.launches()
        l0 = max(lis, key=lambda li: li["ms"])
        first_ms.append(l0["ms"])
        first_ops.append(l0["ops"])
        dom_class = l0["seg_class"]
        # the launches of that class share the chip (config 3: the two halves' launches run
        # concurrently): their ops over the span from the first one's start to the last one's end
        dom = [li for li in lis if li["seg_class"] == dom_class]
        cls_span.append(max(li["start_ms"] + li["ms"] for li in dom) - min(li["start_ms"] for li in dom))
        cls_ops.append(sum(li["ops"] for li in dom))
        cls_launches.append(len(dom))
        if with_snap:
            snap_ms.append(sn["device_ms"])
            snap_bytes = sn["bytes"]
        log(rank, f"step {i}: {kernel_ms[-1]:.1f} ms kernel" + (f", {snap_ms[-1]:.1f} ms snapshot" if with_snap else ""))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t_max = elapsed
    st = b.stats()
    ops_done = int(st["ops_applied"])  # ops applied per step on this rank (same every step)
    if args.writers:  # the metric counts the log's sequenced messages, not the writers' local copies
        ops_done -= n_local
    ops_all = ops_done
    alg_bytes = b.algorithmic_bytes()
    alg_all = alg_bytes
    if world > 1:
        dev = "cuda" if backend == "nccl" else "cpu"
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_max = float(t.item())
        o = torch.tensor([ops_done], device=dev, dtype=torch.int64)
        dist.all_reduce(o, op=dist.ReduceOp.SUM)
        ops_all = int(o.item())
        a = torch.tensor([alg_bytes], device=dev, dtype=torch.float64)
        dist.all_reduce(a, op=dist.ReduceOp.SUM)
        alg_all = float(a.item())
    ranks_gathered = dist.get_world_size() if dist.is_initialized() else 1
    summaries = None
    if with_snap:  # the SnapshotV1 bytes themselves to rank 0 (after the timed steps)
        summaries = gather_summaries(b, torch, dist, world, rank, backend)

    cnt = b.counters()
    capacity = {f: [int(np.percentile(cnt[f], q)) for q in (50, 99, 100)]
                for f in ("max_slots", "max_unsettled", "max_blocks", "max_heap")}
    all_ok, not_ok, digest_xor, snap_xor = 0, None, None, None
    if rank == 0:
        all_dig, all_st = gathered[:2]
        all_ok = int((all_st == 0).all())
        not_ok = int((all_st != 0).sum())
        digest_xor = f"{int(np.bitwise_xor.reduce(all_dig)):016x}"
        if with_snap:
            snap_xor = f"{int(np.bitwise_xor.reduce(gathered[2])):016x}"
    # throughput counts the ops actually applied (a document that stopped early counts only its
    # applied ops); requested_ops_per_step is reported beside it
    value = ops_all * args.steps / t_max
    avg_kernel_ms = sum(kernel_ms) / len(kernel_ms)
    # roofline of the dominant kernel (the longest launch, mt_replay_kernel_<class>): the algorithmic bytes
    # of the ops it applied (DESIGN.md "Roofline": per-op share of the batch's algorithmic bytes)
    # over its average launch duration (hipEvents on the launch's stream)
    avg_first_ms = sum(first_ms) / len(first_ms)
    ops_per_launch = sum(first_ops) / len(first_ops)
    alg_per_op = alg_bytes / max(1, ops_done)
    first_bytes = alg_per_op * ops_per_launch
    achieved_gbs = first_bytes / (avg_first_ms * 1e-3) / 1e9
    # the class window: every launch of the dominant class (they run concurrently) over their span
    avg_cls_span = sum(cls_span) / len(cls_span)
    avg_cls_ops = sum(cls_ops) / len(cls_ops)
    class_gbs = alg_per_op * avg_cls_ops / (avg_cls_span * 1e-3) / 1e9
    # the whole step: every rank's algorithmic bytes over the max-over-ranks step time
    step_gbs = alg_all * args.steps / t_max / 1e9
    kname = f"mt_{'writer' if args.writers else 'replay'}_kernel_{dom_class}"
    traffic, traffic_src = pmc_traffic(args.config, n_docs, n_ops, kname, ops_per_launch)
    # issue / LDS utilisation over the chip time the class's concurrent launches share
    lds = lds_busy(args.config, n_ops, kname, avg_cls_span, avg_cls_ops)
    issue = issue_util(args.config, n_ops, kname, avg_cls_span, avg_cls_ops)
    cpu = None
    parity = None
    if rank == 0 and not args.no_cpu:
        cpu, parity = cpu_baseline(b, fa, n_docs, args, writer_log)
    snapshot = None
    if with_snap:
        avg_snap = sum(snap_ms) / len(snap_ms)
        snapshot = {"bytes_per_step": int(snap_bytes), "avg_device_ms": round(avg_snap, 3),
                    "GB_per_s": round(snap_bytes / (avg_snap * 1e-3) / 1e9, 3), "kernel": "mt_snapshot_kernel",
                    "summaries_gathered": summaries}
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
            "config": {"workload": ("writer replicas (local ops + acks) of " if args.writers else "") + cfg["workload"],
                       "docs_per_gpu": n_docs,
                       "ops_per_doc": n_ops if sizes is None else {"min": int(sizes.min()), "max": int(sizes.max()),
                                                                  "lpt_loads": loads},
                       "clients": cfg["n_clients"], "max_lag": cfg["max_lag"],
                       "op_mix": [cfg["pct_insert"], cfg["pct_remove"], 100 - cfg["pct_insert"] - cfg["pct_remove"]],
                       "parallelism": f"doc-sharded x{world}",
                       "step": "replay + device digests" + (" + GPU SnapshotV1" if with_snap else "") +
                               " + gather to rank 0"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbs, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved_gbs / HBM_PEAK_GBS, 6), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "traffic_per": "launch (PMC HBM bytes per op of this kernel x ops_per_launch)",
                         "kernel": kname, "avg_launch_ms": round(avg_first_ms, 3),
                         "algorithmic_bytes_per_launch": int(first_bytes),
                         "algorithmic_bytes_per_op": round(alg_per_op, 2),
                         "algorithmic_bytes_formula": "32 B/op record + 2 B/inserted code unit + 8 B/prop record "
                                                      "+ 32 B/final table entry (DESIGN.md §5)",
                         "ops_per_launch": int(ops_per_launch),
                         "class_window": {"launches": round(sum(cls_launches) / len(cls_launches), 2),
                                          "span_ms": round(avg_cls_span, 3), "ops": int(avg_cls_ops),
                                          "achieved": round(class_gbs, 3),
                                          "frac": round(class_gbs / HBM_PEAK_GBS, 6)},
                         "step": {"achieved": round(step_gbs, 3), "frac": round(step_gbs / HBM_PEAK_GBS, 6),
                                  "algorithmic_bytes_per_step": int(alg_all)},
                         "utilisation_window": "issue_frac / lds_busy: the class window's ops over its span x the chip",
                         "lds_busy": lds,
                         "issue_frac": issue["frac"] if issue else None,
                         "issue": issue},
            "replay_ms_per_step": round(avg_kernel_ms, 3),
            "launches": b.launches(),
            "cpu_baseline": cpu,
            "parity": parity,
            "snapshot": snapshot,
            "docs_ok": all_ok,
            # writer replicas can stop where the reference's would (a remote insert beside the
            # replica's own unacked removes: the #1213 family, "MergeTree insert failed");
            # parity.digest_match compares statuses too
            "docs_not_ok": not_ok,
            "digests_gathered": len(gathered[0]) if rank == 0 else None,
            "ranks_gathered": ranks_gathered,
            "digest_xor": digest_xor,
            "snapshot_digest_xor": snap_xor,
            "ops_applied_per_step": ops_all,
            "requested_ops_per_step": int(total_ops_step),
            "lds_bytes_per_doc": st["lds_bytes"],
            "launches_per_step": st["launches"],
            "capacity_p50_p99_max": capacity,
            "gen_s": round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    b.close()
    if world > 1:
        dist.destroy_process_group()


def pmc_traffic(config, n_docs, n_ops, kernel, ops_per_launch):
    """HBM bytes of one launch of `kernel` from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE passes
    of this same configuration (tools/pmc_counters.py -> profiles/pmc_counters_config<N>.json,
    scripts/gpu_check.sh pmcf<N> / pmcw<N>): (2 x FETCH_SIZE + WRITE_SIZE) x 1024 per the guide's
    gfx950 correction.  The profile sums every launch of the kernel in one step (config 3: two
    concurrent launches of the dominant class), so its bytes per op times this run's ops per launch
    is the per-launch figure that pairs with algorithmic_bytes_per_launch.  The counters cannot be
    read from inside this process, so the profile of the current kernel build is committed under
    profiles/ and quoted here; None when no profile of this configuration and kernel exists."""
    path = ROOT / "profiles" / f"pmc_counters_config{config}.json"
    try:
        prof = json.loads(path.read_text())
    except (OSError, ValueError):
        return None, None
    k = prof.get("kernels", {}).get(kernel)
    if prof.get("docs") != n_docs or prof.get("ops") != n_ops or not k or "hbm_bytes" not in k or not k.get("ops"):
        return None, None
    return int(k["hbm_bytes"] / k["ops"] * ops_per_launch), str(path.relative_to(ROOT))


def log(rank, msg):
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def usable_cores():
    """Cores this process may run on: the affinity set, capped by a cgroup CPU quota (the GPU
    box gives each job a share of a larger machine; os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(float(quota) / float(period))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(b, fa, n_docs, args, writer=None):
    """Oracle (CPU restatement, tests-only code) on a bounded sample of the same logs, timed on
    every usable host core (one pthread per core); its per-doc digests and statuses double as a
    parity check of every sampled document.  Sample: the first documents of this rank's batch up to
    ~8.2M ops.  writer = (records, offsets, text, props, writer_of, client names) of --writers: the
    oracle replays the same writer replicas (one sub-batch per writer id, its client table)."""
    sys.path.insert(0, str(ROOT / "tests"))
    import numpy as np

    import oracle_ffi as O

    if args.cpu_sample_docs:
        sample = min(args.cpu_sample_docs, n_docs)
    else:
        csum = np.cumsum(b.counters()["ops_done"].astype(np.int64))
        sample = int(np.searchsorted(csum, 4096 * 2000, side="left")) + 1
        sample = min(n_docs, max(16, sample))
    threads = args.cpu_threads or usable_cores()
    tables = O.gen_tables()
    if writer is None:
        sops, soff, text, props = b.download_log(0, sample)
        secs, dig, st = O.replay_batch(sops, soff, text, props, tables, O.gen_client_names(8), n_threads=threads)
        n_ops = int(soff[-1])
    else:
        wops, woff, text, props, wof, base = writer
        dig, st = np.zeros(sample, np.uint64), np.zeros(sample, np.int32)
        secs, n_ops = 0.0, 0
        for w in sorted(set(int(x) for x in wof[:sample])):
            idx = np.nonzero(wof[:sample] == w)[0]
            parts = [wops[woff[d]:woff[d + 1]] for d in idx]
            soff = np.concatenate([[0], np.cumsum([len(x) for x in parts])]).astype(np.int64)
            nm = list(base)
            nm[0], nm[w] = nm[w], nm[0]
            s, dg, sg = O.replay_batch(np.concatenate(parts), soff, text, props, tables, nm, n_threads=threads)
            secs += s
            dig[idx], st[idx] = dg, sg
            n_ops += int(soff[-1])
    gpu_dig = np.array([b.doc(d).digest() for d in range(sample)], np.uint64)
    gpu_st = b.counters()["status"][:sample]
    match = int(((gpu_dig == dig) & (gpu_st == st)).sum())
    cpu = {"value": round(n_ops / secs, 1), "unit": "ops/s", "cores": threads, "kind": "port",
           "sample": f"first {sample} docs ({n_ops} ops) of the same log, oracle/ C restatement, {threads} threads "
                     f"(usable cores; os.cpu_count()={os.cpu_count()}), CPU: {cpu_model()}",
           "seconds": round(secs, 3)}
    parity = {"docs_checked": sample, "digest_match": match, "oracle_status_ok": int((st == 0).sum())}
    if writer is not None:  # records: local copies + sequenced messages
        cpu["sample"] = "writer replicas: " + cpu["sample"].replace(" ops)", " records)")
    return cpu, parity


def gather_summaries(b, torch, dist, world, rank, backend):
    """SnapshotV1 summaries of every document to rank 0 (digests *and summaries*):
    each rank's GPU SnapshotV1 buffer (mt_batch_snapshot_copy, device to device) is padded to the
    largest and gathered with one dist.gather over RCCL; rank 0 re-checks the received bytes of
    its own shard against the local buffer.  Returns {bytes, ranks} on rank 0."""
    import numpy as np

    from fluidframework_amd import shard

    off, meta = b.snapshot_index()
    n = int(off[-1])
    dev = "cuda" if backend == "nccl" or world == 1 else "cpu"
    buf = torch.empty(max(1, n), dtype=torch.uint8, device="cuda")
    b.snapshot_copy(buf)
    recv = shard.gather_bytes(buf[:n] if dev == "cuda" else buf[:n].cpu(), world, rank)
    if rank != 0:
        return None
    ok = bool(torch.equal(recv[0].to(buf.device), buf[:n]))
    return {"bytes": int(sum(int(r.numel()) for r in recv)), "ranks": len(recv), "rank0_roundtrip_equal": ok}


INSTR_COUNTERS = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH",
                  "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR")


def issue_util(config, n_ops, kernel, avg_ms, ops_per_launch):
    """What bounds the dominant kernel when neither HBM nor LDS does: its instruction issue.
    frac = instructions per op (the committed rocprofv3 SQ_INSTS_* passes of this configuration,
    profiles/pmc_counters_config<N>.json) x the ops the class's concurrent launches applied / (their
    span measured live here x 256 CUs x 4 SIMDs x ~2.4 GHz), i.e. instructions per SIMD-cycle against
    one per cycle.
    One wave alone issues at most one instruction per ~4 cycles (MI355X_MICROARCH.md, 'vector-
    instruction ISSUE cost'), so `wave_frac` = 4 x instructions / SQ_WAVE_CYCLES-derived cycles per
    op is how much of its own issue ceiling a document's wave uses; `wait_share` = SQ_WAIT_ANY /
    SQ_WAVE_CYCLES, the share of wave time parked on s_waitcnt (memory latency)."""
    path = ROOT / "profiles" / f"pmc_counters_config{config}.json"
    try:
        prof = json.loads(path.read_text())
    except (OSError, ValueError):
        return None
    k = prof.get("kernels", {}).get(kernel)
    if not k or prof.get("ops") != n_ops:
        return None
    per = k.get("per_op") or {}
    if any(c not in per for c in INSTR_COUNTERS):
        return None
    inst = sum(per[c] for c in INSTR_COUNTERS)
    simd_cycles = avg_ms * 1e-3 * CLOCK_GHZ * 1e9 * N_CUS * 4
    out = {"frac": round(inst * ops_per_launch / simd_cycles, 6), "instructions_per_op": round(inst, 1),
           "source": str(path.relative_to(ROOT))}
    wc = per.get("SQ_WAVE_CYCLES")
    if wc:  # SQ_WAVE_CYCLES counts in units of 4 cycles (quad-cycles) per wave
        out["wave_cycles_per_op"] = round(4 * wc, 1)
        out["wave_frac"] = round(4.0 * inst / (4.0 * wc), 4)  # 4 cycles per instruction / 4 cycles per quad
        if per.get("SQ_WAIT_ANY"):
            out["wait_share"] = round(per["SQ_WAIT_ANY"] / wc, 4)
    return out


def lds_busy(config, n_ops, kernel, avg_ms, ops_per_launch):
    """How busy the dominant kernel keeps the LDS arrays, from the committed rocprofv3 counter passes
    of this same configuration (tools/pmc_counters.py -> profiles/pmc_counters_config<N>.json):
    SQ_LDS_IDX_ACTIVE (LDS-array cycles, bank-conflict cycles included) per op x the ops of one
    launch, over the launch time measured live here x 256 CUs x ~2.4 GHz.  A utilisation, not bytes
    moved; the bank-conflict share is SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
    (MI355X_MICROARCH.md: BANK_CONFLICT = extra cycles, IDX_ACTIVE = all LDS-array cycles).
    None without a matching profile."""
    path = ROOT / "profiles" / f"pmc_counters_config{config}.json"
    try:
        prof = json.loads(path.read_text())
    except (OSError, ValueError):
        return None
    k = prof.get("kernels", {}).get(kernel)
    if not k or prof.get("ops") != n_ops:
        return None
    per = k.get("per_op") or {}
    act, conf = per.get("SQ_LDS_IDX_ACTIVE"), per.get("SQ_LDS_BANK_CONFLICT")
    if not act:
        return None
    cu_cycles = avg_ms * 1e-3 * CLOCK_GHZ * 1e9 * N_CUS
    return {"frac": round(act * ops_per_launch / cu_cycles, 6), "lds_cycles_per_op": act,
            "bank_conflict_cycles_per_op": conf,
            "bank_conflict_share": round(conf / act, 4) if conf is not None else None,
            "source": str(path.relative_to(ROOT)), "counters_per_op": per}


if __name__ == "__main__":
    main()
