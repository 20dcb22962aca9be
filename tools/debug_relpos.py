import sys, json
sys.path.insert(0, 'tests'); sys.path.insert(0, '.')
import combine_logs as C, oracle_ffi as O
import fluidframework_amd as fa
docs = []
for seed, cut, chunk in ((11, 150, 10000),):
    msgs = C.relpos_farm(350, seed=seed, live_ids_only=True)
    a = O.Doc(); a.start_collab("readonly")
    for m in msgs[:cut]: a.apply_msg(json.dumps(m))
    docs.append({"snapshot": a.snapshot_v1(chunk), "messages": msgs[cut:]})
with fa.ReplayBatch(len(docs)) as b:
    b.ingest_json([json.dumps(d) for d in docs])
    b.run()
    c = b.counters()
    print({k: c[k].tolist() for k in c.dtype.names})
    print(b.launches())
    sops, soff, text, props = b.download_log(0, 1)
    fo = int(c["ops_done"][0])
    for i in range(max(0, fo - 3), min(len(sops), fo + 3)):
        print(i, sops[i])
