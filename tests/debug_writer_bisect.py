"""Debugging aid (run on the GPU box): the first event of a writer replica's stream after which the
GPU replay differs from the oracle's.  Every prefix of the stream is one GPU document; the oracle
replays the same prefixes.  usage: python tests/debug_writer_bisect.py [seed n_clients steps rewrite writer]"""
import json
import sys
from pathlib import Path

sys.path[:0] = [str(Path(__file__).resolve().parents[1]), str(Path(__file__).resolve().parent)]

import oracle_ffi as O  # noqa: E402
import fluidframework_amd as fa  # noqa: E402
from writer_sim import farm  # noqa: E402


def oracle_replica(name, events, initial):
    d = O.Doc()
    if initial:
        d.insert_local(0, json.dumps(initial))
    d.start_collab(name)
    for m in events:
        if m.get("type") == "regenerate":
            d.regenerate(m["contents"])
        elif m["sequenceNumber"] == -1:
            d.local_op(m["contents"])
        elif d.apply_msg(json.dumps(m)) != 0:
            break
    return d


def main():
    a = [int(x) for x in sys.argv[1:]] if len(sys.argv) > 1 else [1, 3, 400, 0, 0]
    seed, n_clients, steps, rewrite, wi = a
    initial = ""  # a message stream carries no pre-collaboration text
    f = farm(n_clients, steps, seed, initial=initial, rewrite=rewrite)
    name = f.names[wi]
    ev = f.events[name]
    print(f"writer {name}: {len(ev)} events; oracle status {f.docs[name].status} {f.docs[name].error}")
    docs = [ev[:L] for L in range(1, len(ev) + 1)]
    with fa.ReplayBatch(len(docs)) as b:
        b.ingest_messages(docs, observer=name)
        b.run()
        prev = None
        for L in range(1, len(ev) + 1):
            od = oracle_replica(name, ev[:L], initial)
            dv = b.doc(L - 1)
            same = dv.status == od.status and (od.status != 0 or dv.digest() == od.digest())
            if not same:
                print(f"first difference after event {L - 1}: {json.dumps(ev[L - 1])}")
                print(f"GPU status {fa.status_string(dv.status)}  oracle status {od.status} {od.error}")
                if prev is not None:
                    print("---- oracle before:\n" + prev.dump())
                    print("---- GPU before:\n" + b.doc(L - 2).dump())
                print("---- oracle after:\n" + od.dump())
                if dv.status == 0:
                    print("---- GPU after:\n" + dv.dump())
                return
            prev = od
        print("no difference")


if __name__ == "__main__":
    main()
