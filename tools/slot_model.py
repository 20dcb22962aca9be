"""Per-document features of generated logs vs the slots the replay needed (capacity planning).

Writes gpurun_out/slot_model.npz: for several op mixes and sizes, per document: ops, inserts,
removes, annotates, inserted code units, inserted '\\n', removed units (pos2 - pos1), and the
device's max_slots / max_blocks / max_heap / max_unsettled high-water marks."""
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fluidframework_amd as fa  # noqa: E402

CASES = [  # (n_ops, docs, pct_insert, pct_remove)
    (2000, 4096, 60, 40), (2000, 2048, 55, 35), (10000, 512, 55, 35), (5000, 512, 70, 20), (1000, 2048, 60, 40),
]
rows = []
for n_ops, docs, pi, pr in CASES:
    with fa.ReplayBatch(docs) as b:
        b.generate(fa.gen_params(n_ops, pct_insert=pi, pct_remove=pr, seed=0xDEADBEEF))
        b.run()
        c = b.counters()
        ops, off, text, props = b.download_log()
        for d in range(docs):
            o = ops[off[d]:off[d + 1]]
            ins = (o["tc"] & 0xF) == 0
            rem = (o["tc"] & 0xF) == 1
            ann = (o["tc"] & 0xF) == 2
            units = int(o["payload_len"][ins].sum())
            nl = sum(int((text[x["payload"]:x["payload"] + x["payload_len"]] == 10).sum()) for x in o[ins])
            removed = int((o["pos2"][rem] - o["pos1"][rem]).sum())
            rows.append((n_ops, pi, pr, int(ins.sum()), int(rem.sum()), int(ann.sum()), units, nl, removed,
                         c.max_slots[d], c.max_blocks[d], c.max_heap[d], c.max_unsettled[d]))
    print(f"case {n_ops} {docs} {pi}/{pr}: done", flush=True)
np.savez("gpurun_out/slot_model.npz", rows=np.array(rows, np.int64))
