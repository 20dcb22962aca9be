"""Full-batch parity of the headline workload: every document of bench.py's config 3 (65,536
docs x 10k ops, the bench's generator parameters and seed) replayed on the GPU and by the oracle
(tests/oracle_ffi.py, test infrastructure: the checker, never the thing measured), chunk by chunk
so host memory stays bounded.  Per document: the GPU's state digest (mt_doc_digest) and status
against the oracle's; over the batch: the XOR of the GPU device digests, which must equal the
bench line's digest_xor.  python tools/full_parity.py [docs] [chunk] [out.json]"""
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ffi as O  # noqa: E402

import bench  # noqa: E402  (CONFIGS, usable_cores: the bench's own workload definition)
import fluidframework_amd as fa  # noqa: E402

cfg = bench.CONFIGS[3]
n_docs = int(sys.argv[1]) if len(sys.argv) > 1 else cfg["docs"]
chunk = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
out = sys.argv[3] if len(sys.argv) > 3 else None
p = fa.gen_params(cfg["ops"], n_clients=cfg["n_clients"], max_lag=cfg["max_lag"], pct_insert=cfg["pct_insert"],
                  pct_remove=cfg["pct_remove"], seed=0xDEADBEEF)
threads = bench.usable_cores()
tables, names = O.gen_tables(), O.gen_client_names(cfg["n_clients"])
res = {"config": 3, "docs": n_docs, "ops_per_doc": cfg["ops"], "chunk": chunk, "oracle_threads": threads,
       "digest_match": 0, "status_match": 0, "oracle_status_ok": 0, "ops": 0, "mismatches": []}
xor_dev = 0
t0 = time.time()
for first in range(0, n_docs, chunk):
    n = min(chunk, n_docs - first)
    with fa.ReplayBatch(n) as b:
        b.generate(p, first)
        b.run()
        dev = b.device_digests()
        st = b.counters()["status"].astype(np.int32)
        gdig = np.array([b.doc(d).digest() for d in range(n)], np.uint64)
        ops, off, text, props = b.download_log()
    _, odig, ost = O.replay_batch(ops, off, text, props, tables, names, n_threads=threads)
    ok = gdig == odig
    res["digest_match"] += int(ok.sum())
    res["status_match"] += int((st == ost).sum())
    res["oracle_status_ok"] += int((ost == 0).sum())
    res["ops"] += int(off[-1])
    res["mismatches"] += [first + int(i) for i in np.nonzero(~ok)[0][:8]]
    xor_dev ^= int(np.bitwise_xor.reduce(dev))
    print(f"docs [{first}, {first + n}): {int(ok.sum())}/{n} digests equal, {time.time() - t0:.0f} s", flush=True)
res["device_digest_xor"] = f"{xor_dev:016x}"
res["seconds"] = round(time.time() - t0, 1)
print(json.dumps(res))
if out:
    Path(out).write_text(json.dumps(res, indent=1) + "\n")
