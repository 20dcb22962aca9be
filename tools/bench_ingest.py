"""Native JSON ingest throughput (mt_pack_json) on this host's cores.

Generates config-2 shaped logs on the GPU (or takes --docs/--ops), renders them as
ISequencedDocumentMessage JSON (one messages.json array per document), then times
mt_pack_json (parse + pack) at several thread counts and the full host->device
mt_batch_ingest_packed.  Prints one JSON line."""
import argparse
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import fluidframework_amd as fa  # noqa: E402
from fluidframework_amd.mtreplay import PackedJson  # noqa: E402

KEYS = ["bold", "italic", "color", "size"]
VALS = [None, True, "red", "green", "blue"] + list(range(8, 25))
NAMES = ["readonly"] + [chr(ord("A") + i) for i in range(26)]


def render(ops, off, text, props, d):
    out = []
    for o in ops[off[d]:off[d + 1]]:
        t = int(o["tc"]) & 0xF
        if t == 0:
            c = {"type": 0, "pos1": int(o["pos1"]),
                 "seg": text[o["payload"]:o["payload"] + o["payload_len"]].tobytes().decode("utf-16-le")}
        elif t == 1:
            c = {"type": 1, "pos1": int(o["pos1"]), "pos2": int(o["pos2"])}
        else:
            pr = props[o["payload"]:o["payload"] + o["payload_len"]]
            c = {"type": 2, "pos1": int(o["pos1"]), "pos2": int(o["pos2"]),
                 "props": {KEYS[int(q["key"])]: VALS[int(q["value"])] for q in pr}}
        out.append({"clientId": NAMES[int(o["tc"]) >> 4], "sequenceNumber": int(o["seq"]),
                    "referenceSequenceNumber": int(o["ref_seq"]), "minimumSequenceNumber": int(o["msn"]),
                    "type": "op", "contents": c})
    return json.dumps(out).encode()


ap = argparse.ArgumentParser()
ap.add_argument("--docs", type=int, default=512)
ap.add_argument("--ops", type=int, default=2000)
ap.add_argument("--threads", default="1,4,8,16")
a = ap.parse_args()
with fa.ReplayBatch(a.docs) as b:
    b.generate(fa.gen_params(a.ops, pct_insert=55, pct_remove=35, seed=7))
    ops, off, text, props = b.download_log()
    t0 = time.time()
    docs = [render(ops, off, text, props, d) for d in range(a.docs)]
    print(f"[ingest] rendered {a.docs} docs in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    nbytes = sum(len(x) for x in docs)
    res = {"metric": "JSON op-log ingest (parse + pack)", "docs": a.docs, "ops_per_doc": a.ops,
           "json_bytes": nbytes, "host_cores": os.cpu_count(), "runs": []}
    for nt in [int(x) for x in a.threads.split(",")]:
        best = 1e9
        for _ in range(3):
            t0 = time.perf_counter()
            PackedJson(docs, n_threads=nt).close()
            best = min(best, time.perf_counter() - t0)
        res["runs"].append({"threads": nt, "seconds": round(best, 4), "ops_per_s": round(a.docs * a.ops / best, 1),
                            "MB_per_s": round(nbytes / best / 1e6, 1)})
        print(f"[ingest] {nt} threads: {best:.3f} s", file=sys.stderr, flush=True)
    t0 = time.perf_counter()
    b.ingest_json(docs, n_threads=16)
    res["ingest_to_device_s"] = round(time.perf_counter() - t0, 4)
    b.run()
    res["replay_ok"] = int(b.stats()["docs_failed"] == 0)
    print(json.dumps(res))
