"""One large generated document through the ladder (test_giant_document_beyond_65k_segments' log):
launches, status and digest vs the oracle.  python tools/diag_giant.py [n_ops] [seed]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))
import oracle_ffi as O  # noqa: E402

import fluidframework_amd as fa  # noqa: E402

n_ops = int(sys.argv[1]) if len(sys.argv) > 1 else 360000
seed = int(sys.argv[2], 0) if len(sys.argv) > 2 else 4096
p = O.gen_params(n_ops, pct_insert=50, pct_remove=15, seed=seed)
ops, text, props, off = O.gen_batch(p, 1)
t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
_, dig, st = O.replay_batch(ops, off, text, props, t, names)
with fa.ReplayBatch(1) as b:
    b.set_tables([O.lib().mto_gen_key_name(k).decode() for k in range(4)],
                 [O.lib().mto_gen_value_json(v).decode() for v in range(22)])
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    for li in b.launches():
        print({k: li[k] for k in ("seg_class", "n_docs", "resumed", "ms", "ops") if k in li})
    c = b.counters()
    print("status", b.doc(0).status, "oracle", st[0], "cap_kind", int(c["cap_kind"][0]), "digest ok",
          b.doc(0).digest() == int(dig[0]))
    od = O.replay_doc(ops.copy(), text, props, t, names)
    gt, ot = b.doc(0).get_text(), od.text()
    i = next((k for k in range(min(len(gt), len(ot))) if gt[k] != ot[k]), min(len(gt), len(ot)))
    print("text len", len(gt), len(ot), "first diff", i, repr(gt[max(0, i - 10):i + 10]), repr(ot[max(0, i - 10):i + 10]))
    print("shape equal", b.doc(0).shape() == od.shape())
