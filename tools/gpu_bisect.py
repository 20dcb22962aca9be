"""Debugging aid: find the first op where the GPU replay diverges from the oracle.

Replays a generated batch on the GPU, picks the first document whose state digest differs,
then replays every prefix of that document's log (one prefix per GPU document) and reports
the first diverging op with both segment tables.  Uses the oracle as the checker.
"""
import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]

import numpy as np  # noqa: E402

import oracle_ffi as O  # noqa: E402
import fluidframework_amd as fa  # noqa: E402

KEYS = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
VALUES = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]


def gpu_batch(ops_list, text, props, names):
    off = np.zeros(len(ops_list) + 1, np.int64)
    for i, o in enumerate(ops_list):
        off[i + 1] = off[i] + len(o)
    ops = np.concatenate(ops_list)
    b = fa.ReplayBatch(len(ops_list))
    b.set_tables(KEYS, VALUES)
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    return b


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ops", type=int, default=2000)
    ap.add_argument("--docs", type=int, default=48)
    ap.add_argument("--ins", type=int, default=60)
    ap.add_argument("--rem", type=int, default=40)
    ap.add_argument("--seed", type=lambda x: int(x, 0), default=0xC0FFEE)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--lag", type=int, default=32)
    a = ap.parse_args()
    p = O.gen_params(a.ops, n_clients=a.clients, max_lag=a.lag, pct_insert=a.ins, pct_remove=a.rem, seed=a.seed)
    ops, text, props, off = O.gen_batch(p, a.docs)
    t, names = O.gen_tables(), O.gen_client_names(a.clients)
    _, dig, st = O.replay_batch(ops, off, text, props, t, names)
    b = gpu_batch([ops[off[d]:off[d + 1]] for d in range(a.docs)], text, props, names)
    print("stats", b.stats())
    bad = [d for d in range(a.docs) if b.doc(d).status != st[d] or b.doc(d).digest() != int(dig[d])]
    print(f"mismatching docs: {len(bad)}/{a.docs}: {bad[:20]}")
    print("gpu statuses", np.bincount(b.statuses(), minlength=8), "oracle", np.bincount(st, minlength=8))
    if not bad:
        return
    d = bad[0]
    dops = ops[off[d]:off[d + 1]]
    n = len(dops)
    b.close()
    pb = gpu_batch([dops[:k].copy() for k in range(1, n + 1)], text, props, names)
    def differs(k):
        od = O.replay_doc(dops[:k].copy(), text, props, t, names)
        gv = pb.doc(k - 1)
        return gv.status != od.status or (od.status == 0 and gv.digest() != od.digest())

    if not differs(n):
        print("full prefix matches?!")
        return
    lo, hi = 0, n  # differs(hi) is True; differs(lo) assumed False (empty doc)
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if differs(mid):
            hi = mid
        else:
            lo = mid
    first = hi
    print(f"doc {d}: first divergence after op index {first - 1}")
    for i in range(max(0, first - 4), first):
        print("  op", i, dops[i])
    od_prev = O.replay_doc(dops[:first - 1].copy(), text, props, t, names) if first > 1 else None
    od = O.replay_doc(dops[:first].copy(), text, props, t, names)
    print("---- oracle before:\n", od_prev.dump() if od_prev else "(empty)")
    print("---- GPU before:\n", pb.doc(first - 2).dump() if first > 1 else "(empty)")
    print("---- oracle after:\n", od.dump(), od.shape())
    print("---- GPU after:\n", pb.doc(first - 1).dump(), pb.doc(first - 1).shape())


if __name__ == "__main__":
    main()
