"""Debugging aid: replay oracle-generated logs on the GPU and print the run counters of every
document that did not finish OK (status, cap_kind, ops_done, fail_op, launch, capacities)."""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import oracle_ffi as O  # noqa: E402
import fluidframework_amd as fa  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--ops", type=int, default=2000)
ap.add_argument("--docs", type=int, default=48)
ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xC0FFEE)
ap.add_argument("--seg-cap", type=int, default=0)
a = ap.parse_args()
p = O.gen_params(a.ops, seed=a.seed)
ops, text, props, off = O.gen_batch(p, a.docs)
t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
with fa.ReplayBatch(a.docs, seg_cap=a.seg_cap) as b:
    b.set_tables([O.lib().mto_gen_key_name(k).decode() for k in range(4)],
                 [O.lib().mto_gen_value_json(v).decode() for v in range(22)])
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    print("stats", b.stats())
    c = b.counters()
    for d in range(a.docs):
        if c["status"][d] != 0:
            print("doc", d, {k: int(c[k][d]) for k in c.dtype.names})
