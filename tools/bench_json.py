#!/usr/bin/env python3
"""JSON op-log ingest on the MI355X: GPU parser (mt_json_gpu.hip) vs the host parser (mt_pack_json).

Workload: synthetic logs of a BASELINE config shape (generated on the GPU, include/mt_gen.h),
exported as ISequencedDocumentMessage JSON arrays (oplog.records_to_json), copied to HBM once.
Timed: K x (mt_batch_ingest_json_gpu from the HBM-resident JSON, then the replay), and the host
parser (mt_pack_json on every usable core + mt_batch_ingest_packed) on the same documents.
Parity: every document's device digest after GPU ingest == after host ingest.  Prints one JSON
line (profiles/r02_json_ingest_*.json)."""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--docs", type=int, default=2048)
    ap.add_argument("--ops", type=int, default=2000)
    ap.add_argument("--mix", default="60,40", help="pct_insert,pct_remove (rest annotate)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--threads", type=int, default=0)
    args = ap.parse_args()
    import __graft_entry__ as g

    g.build_lib()
    import fluidframework_amd as fa
    from fluidframework_amd import oplog
    from fluidframework_amd.mtreplay import GEN_KEYS, GEN_VALUES, gen_client_names

    pi, pr = (int(x) for x in args.mix.split(","))
    p = fa.gen_params(args.ops, n_clients=8, max_lag=32, pct_insert=pi, pct_remove=pr, seed=0xDEADBEEF)
    t0 = time.time()
    with fa.ReplayBatch(args.docs) as b:
        b.generate(p, 0)
        ops, off, text, props = b.download_log()
    texts = oplog.records_to_json(ops, off, text, props, GEN_KEYS, GEN_VALUES, gen_client_names(8))
    buf, doff = fa.json_concat(texts)
    n_ops = int(off[-1])
    print(f"[json] {args.docs} docs, {n_ops} ops, {len(buf) / 1e6:.1f} MB of JSON in {time.time() - t0:.1f} s",
          flush=True)
    hip = C.CDLL("libamdhip64.so.7")
    ptr = C.c_void_p()
    assert hip.hipMalloc(C.byref(ptr), C.c_size_t(len(buf) + 64)) == 0
    assert hip.hipMemset(ptr, 0, C.c_size_t(len(buf) + 64)) == 0
    assert hip.hipMemcpy(ptr, buf, C.c_size_t(len(buf)), 1) == 0
    gpu = []
    with fa.ReplayBatch(args.docs) as bg:
        for k in range(args.steps + 1):
            t = time.perf_counter()
            st = bg.ingest_json_gpu(buf, doff, d_json=ptr)
            t_ing = time.perf_counter() - t
            t = time.perf_counter()
            bg.run()
            t_run = time.perf_counter() - t
            if k:  # the first is the warmup
                gpu.append((t_ing, t_run, st))
            print(f"[json] step {k}: GPU ingest {1e3 * t_ing:.1f} ms (scan {st['ms_scan']:.2f} count "
                  f"{st['ms_count']:.2f} clients {st['ms_clients']:.2f} write {st['ms_write']:.2f} props "
                  f"{st['ms_props']:.2f} host merge {st['ms_host']:.2f}), replay {1e3 * t_run:.1f} ms", flush=True)
        dig_g = np.array([bg.doc(d).digest() for d in range(args.docs)], np.uint64)
        st_g = bg.counters()["status"].copy()
    hip.hipFree(ptr)
    sys.path.insert(0, str(ROOT))
    from bench import usable_cores

    threads = args.threads or usable_cores()
    host = []
    with fa.ReplayBatch(args.docs) as bh:
        for k in range(2):
            t = time.perf_counter()
            pj = fa.PackedJson(texts, n_threads=threads)
            t_parse = time.perf_counter() - t
            t = time.perf_counter()
            assert fa.lib().mt_batch_ingest_packed(bh.h, pj.h) == 0
            t_ing = time.perf_counter() - t
            pj.close()
            host.append((t_parse, t_ing))
        bh.run()
        dig_h = np.array([bh.doc(d).digest() for d in range(args.docs)], np.uint64)
        st_h = bh.counters()["status"].copy()
    ing = sum(x[0] for x in gpu) / len(gpu)
    run = sum(x[1] for x in gpu) / len(gpu)
    st = gpu[-1][2]
    dev_ms = st["ms_scan"] + st["ms_count"] + st["ms_clients"] + st["ms_write"] + st["ms_props"]
    hp, hi = host[-1]
    line = {
        "metric": "JSON op-log ingest ops/s", "unit": "ops/s",
        "value": round(n_ops / ing, 1),
        "workload": f"{args.docs} docs x {args.ops} ops (insert {pi} / remove {pr} / annotate {100 - pi - pr}), "
                    f"8 clients, ISequencedDocumentMessage JSON ({len(buf)} bytes) resident in HBM",
        "gpu_ingest_ms": round(1e3 * ing, 3),
        "gpu_device_ms": {k: round(st[k], 3) for k in ("ms_scan", "ms_count", "ms_clients", "ms_write", "ms_props")},
        "gpu_host_merge_ms": round(st["ms_host"], 3),
        "parse_GB_per_s_device": round(len(buf) / (dev_ms * 1e-3) / 1e9, 2),
        "scan_roofline": {"bound": "hbm", "achieved": round(len(buf) / (st["ms_scan"] * 1e-3) / 1e9, 2),
                          "peak": HBM_PEAK_GBS, "unit": "GB/s",
                          "frac": round(len(buf) / (st["ms_scan"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5),
                          "kernel": "jg_scan_kernel", "bytes": len(buf)},
        "replay_ms": round(1e3 * run, 3),
        "ingest_plus_replay_ops_per_s": round(n_ops / (ing + run), 1),
        "host_baseline": {"parse_ms": round(1e3 * hp, 3), "ingest_ms": round(1e3 * hi, 3),
                          "value": round(n_ops / (hp + hi), 1), "unit": "ops/s", "threads": threads,
                          "kind": "mt_pack_json (product host parser) + mt_batch_ingest_packed"},
        "parity": {"docs": args.docs, "digest_match": int(((dig_g == dig_h) & (st_g == st_h)).sum()),
                   "status_ok": int((st_g == 0).sum())},
    }
    print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
