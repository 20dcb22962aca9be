"""Parity diagnosis of a generated batch: replays it on the GPU and reports every document whose
digest differs from the oracle's, with where its text / shape first differ and the launches it ran.
python tools/diag_parity.py [n_ops] [n_docs] [seed] [pct_insert] [pct_remove]  (env toggles apply)"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ffi as O  # noqa: E402

import fluidframework_amd as fa  # noqa: E402

n_ops = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
n_docs = int(sys.argv[2]) if len(sys.argv) > 2 else 48
seed = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0xC0FFEE
pi = int(sys.argv[4]) if len(sys.argv) > 4 else 60
pr = int(sys.argv[5]) if len(sys.argv) > 5 else 40
p = O.gen_params(n_ops, pct_insert=pi, pct_remove=pr, seed=seed)
ops, text, props, off = O.gen_batch(p, n_docs)
t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
_, dig, st = O.replay_batch(ops, off, text, props, t, names)
keys = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
vals = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]
with fa.ReplayBatch(n_docs) as b:
    b.set_tables(keys, vals)
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    print("env MT_TEXT_QUEUE=%s stats %s" % (os.environ.get("MT_TEXT_QUEUE"), json.dumps(b.stats())[:600]))
    bad = [d for d in range(n_docs) if b.doc(d).digest() != int(dig[d])]
    print("mismatching docs:", bad)
    for d in bad[:3]:
        dv = b.doc(d)
        od = O.replay_doc(ops[off[d]:off[d + 1]].copy(), text, props, t, names)
        gt, ot = dv.get_text(), od.text()
        i = next((k for k in range(min(len(gt), len(ot))) if gt[k] != ot[k]), min(len(gt), len(ot)))
        c = {k: [int(x) & 0xFFFFFFFF for x in b.counters()[k]] for k in fa.mtreplay.DOC_COUNTERS}
        ck = int(c["cap_kind"][d])
        if ck >= 100:
            print("  debug: entry dst %d word %#x (src %d len %d) ep|n|idx %#x info %#x addr %d" % (
                c["min_seq"][d] & 0xFFFFFFFF, c["cur_seq"][d] & 0xFFFFFFFF, c["cur_seq"][d] & 0x1FFFFFF,
                ((c["cur_seq"][d] & 0xFFFFFFFF) >> 25) + 1, c["max_blocks"][d] & 0xFFFFFFFF,
                c["max_heap"][d] & 0xFFFFFFFF, c["max_unsettled"][d]))
        print(f"doc {d}: cap_kind {ck} status {dv.status}/{od.status} text len {len(gt)}/{len(ot)} first diff at {i}: "
              f"gpu {gt[max(0, i - 20):i + 20]!r} cpu {ot[max(0, i - 20):i + 20]!r}")
        gs, os_ = dv.shape(), od.shape()
        print(f"  shape equal: {gs == os_}; gpu {str(gs)[:300]}")
        print(f"  cpu {str(os_)[:300]}")
