"""Replay the 150/200-client farms of tests/test_gpu_parity.py with seg_cap=64 (checkpoint /
resume through every class), printing each launch (MT_DEBUG_LAUNCHES) and the result."""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT), str(ROOT / "tests")]
os.environ["MT_DEBUG_LAUNCHES"] = "1"
import test_gpu_parity as T  # noqa: E402
import fluidframework_amd as fa  # noqa: E402

docs = [T._many_client_farm(150, 2500, seed=11), T._many_client_farm(200, 1500, seed=12, lag=60, hot=6)]
oracle = T.oracle_docs_from_messages(docs)
for cap in (0, 64):
    with fa.ReplayBatch(len(docs), seg_cap=cap) as b:
        b.ingest_messages(docs)
        print(f"seg_cap {cap}: run", flush=True)
        b.run()
        print([(li["seg_class"], li["n_docs"], round(li["ms"], 2)) for li in b.launches()], flush=True)
        for i in range(len(docs)):
            print(i, b.doc(i).status, b.doc(i).digest() == oracle[i].digest(), flush=True)
