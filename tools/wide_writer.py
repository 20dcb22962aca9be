"""Which writer replica of the config-2 writer bench escalates, and what its log looks like
(diagnostic for the writer config-2 tail)."""
import sys
import numpy as np
import fluidframework_amd as fa
from fluidframework_amd import oplog
from fluidframework_amd.mtreplay import GEN_KEYS, GEN_VALUES, gen_client_names

p = fa.gen_params(2000, n_clients=8, max_lag=32, pct_insert=60, pct_remove=40, seed=0xDEADBEEF)
D = 4096
b = fa.ReplayBatch(D)
b.generate(p, 0)
ops, off, text, props = b.download_log()
b.close()
wof = 1 + np.arange(D) % 8
wops, woff = oplog.writer_records(ops, off, wof)
base = gen_client_names(8)
b = fa.ReplayBatch(D)
b.set_tables(GEN_KEYS, GEN_VALUES)
for d in range(D):
    nm = list(base)
    nm[0], nm[int(wof[d])] = nm[int(wof[d])], nm[0]
    b.set_clients(nm, d)
b.ingest(wops, woff, text, props)
b.run()
c = b.counters()
print(b.launches())
names = c.dtype.names
order = np.argsort(-c["max_unsettled"])[:5]
for d in order:
    print(d, {n: int(c[n][d]) for n in names})
d = int(order[0])
r = wops[woff[d]:woff[d + 1]]
print("first records of", d)
for k in range(min(80, len(r))):
    print(k, r[k])
