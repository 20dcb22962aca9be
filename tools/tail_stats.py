"""Which documents leave the first launch, why, and how far they got (capacity planning aid).

Runs a bench configuration with max_retries=0 so every document keeps the first launch's
result, then prints the cap_kind histogram and ops_done percentiles of those that stopped."""
import argparse
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402
import fluidframework_amd as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", type=int, default=2)
ap.add_argument("--docs", type=int, default=0)
ap.add_argument("--ops", type=int, default=0)
a = ap.parse_args()
cfg = bench.CONFIGS[a.config]
n_docs, n_ops = a.docs or cfg["docs"], a.ops or cfg["ops"]
p = fa.gen_params(n_ops, n_clients=cfg["n_clients"], max_lag=cfg["max_lag"], pct_insert=cfg["pct_insert"],
                  pct_remove=cfg["pct_remove"], seed=0xDEADBEEF)
for retries in (6, -1):
    with fa.ReplayBatch(n_docs, max_retries=retries) as b:
        b.generate(p, 0)
        b.run()
        st = b.stats()
        c = b.counters()
        for li in b.launches():
            print("  launch", li)
        stopped = c.status == fa.MT_CAPACITY
        print(f"max_retries={retries}: kernel {st['kernel_ms']:.2f} ms launches {st['launches']} "
              f"class {st['lds_class']} stopped {int(stopped.sum())}")
        if stopped.any():
            kinds, cnt = np.unique(c.cap_kind[stopped], return_counts=True)
            print("  cap_kind:", dict(zip(kinds.tolist(), cnt.tolist())))
            print("  ops_done p0/p10/p50/p90/p100:", np.percentile(c.ops_done[stopped], [0, 10, 50, 90, 100]).astype(int).tolist())
            print("  max_slots of stopped:", np.percentile(c.max_slots[stopped], [0, 50, 100]).astype(int).tolist())
