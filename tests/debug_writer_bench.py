"""Debugging aid (run on the GPU box): writer replicas of bench-config logs whose GPU status is not
OK, with the failing record index and the oracle's status for the same document.
usage: python tests/debug_writer_bench.py [config n_docs]"""
import collections
import sys
from pathlib import Path

sys.path[:0] = [str(Path(__file__).resolve().parents[1]), str(Path(__file__).resolve().parent)]

import numpy as np  # noqa: E402
import oracle_ffi as O  # noqa: E402
import fluidframework_amd as fa  # noqa: E402
from fluidframework_amd import oplog  # noqa: E402
from fluidframework_amd.mtreplay import GEN_KEYS, GEN_VALUES  # noqa: E402

sys.argv += [] if len(sys.argv) > 1 else ["2", "512"]
cfgn, N = int(sys.argv[1]), int(sys.argv[2])
mix = {2: (2000, 60, 40), 3: (10000, 55, 35)}[cfgn]
p = O.gen_params(mix[0], n_clients=8, max_lag=32, pct_insert=mix[1], pct_remove=mix[2], seed=0xDEADBEEF)
ops, text, props, off = O.gen_batch(p, N)
names = O.gen_client_names(p.n_clients)
wof = 1 + np.arange(N) % 8
wops, woff = oplog.writer_records(ops, off, wof)
t = O.gen_tables()
with fa.ReplayBatch(N) as b:
    b.set_tables(GEN_KEYS, GEN_VALUES)
    nms = []
    for d in range(N):
        nm = list(names)
        w = int(wof[d])
        nm[0], nm[w] = nm[w], nm[0]
        nms.append(nm)
        b.set_clients(nm, d)
    b.ingest(wops, woff, text, props)
    b.run()
    cnt = b.counters()
    bad = np.nonzero(cnt["status"] != 0)[0]
    print(f"{len(bad)} of {N} documents not OK:",
          collections.Counter(fa.status_string(int(s)) for s in cnt["status"][bad]))
    for d in bad[:8]:
        r = wops[woff[d]:woff[d + 1]]
        fo = int(cnt["fail_op"][d])
        od = O.replay_doc(r.copy(), text, props, t, nms[d])
        print(f"doc {d}: GPU {fa.status_string(int(cnt['status'][d]))} cap_kind {int(cnt['cap_kind'][d])} at record {fo}"
              f" of {len(r)}: {r[fo] if 0 <= fo < len(r) else None}; oracle {od.status} {od.error}")
        lo = max(0, fo - 6)
        for i in range(lo, min(len(r), fo + 2)):
            print("   ", i, r[i])
