"""Per-phase cycles of the lane-parallel SnapshotV1 kernels (a -DMT_SNAP_PROF library, e.g.
FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_snapprof.so): config-5 shaped documents are
replayed and serialized; prints mean cycles per document per phase of the sizing and the writing
kernel (tile loads / flags, record loop, segment framing, text, placement).
usage: python tools/snap_phases.py [docs] [ops]"""
import sys

import numpy as np

sys.path.insert(0, '.')
import fluidframework_amd as fa  # noqa: E402
from fluidframework_amd.mtreplay import SNAP_META  # noqa: E402

docs = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
ops = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
p = fa.gen_params(ops, n_clients=8, max_lag=32, pct_insert=55, pct_remove=35, seed=0x5EED)
with fa.ReplayBatch(docs) as b:
    b.generate(p)
    b.run()
    r = b.snapshots()
    _, meta = b.snapshot_index()
    names = ("tile", "records", "frame", "text", "place")
    ok = meta[:, 0] > 0
    print(f"docs {docs} ops {ops}: {r['bytes']} bytes in {r['device_ms']:.2f} ms "
          f"({r['bytes'] / r['device_ms'] / 1e6:.2f} GB/s), {int(ok.sum())} on the GPU")
    for pas, lo in (("size", SNAP_META - 5), ("write", SNAP_META - 10)):
        m = meta[ok, lo:lo + 5].astype(np.float64).mean(axis=0) * 64
        print(pas, " ".join(f"{n}={v:,.0f}" for n, v in zip(names, m)), f"total={m.sum():,.0f} cycles/doc")
