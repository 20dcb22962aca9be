"""Follow-on worker check on one batch shape: launch table + digest mismatches vs the oracle.
usage: MT_FOLLOW_WORKERS=<n> python tools/follow_debug.py [n_docs] [ops] [seed]"""
import sys
sys.path.insert(0, "tests")
sys.path.insert(0, ".")
import oracle_ffi as O
import fluidframework_amd as fa

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
ops_n = int(sys.argv[2]) if len(sys.argv) > 2 else 1500
seed = int(sys.argv[3], 0) if len(sys.argv) > 3 else 0xBADC0DE
p = O.gen_params(ops_n, pct_insert=55, pct_remove=35, seed=seed)
ops, text, props, off = O.gen_batch(p, n)
t, names = O.gen_tables(), O.gen_client_names(p.n_clients)
_, dig, st = O.replay_batch(ops, off, text, props, t, names)
keys = [O.lib().mto_gen_key_name(k).decode() for k in range(4)]
vals = [O.lib().mto_gen_value_json(v).decode() for v in range(22)]
with fa.ReplayBatch(n) as b:
    b.set_tables(keys, vals)
    b.set_clients(names)
    b.ingest(ops, off, text, props)
    b.run()
    for li in b.launches():
        print(li, flush=True)
    bad = [d for d in range(n) if b.doc(d).digest() != int(dig[d]) or b.doc(d).status != st[d]]
    print("mismatches", len(bad), bad[:10], flush=True)
    sys.exit(1 if bad else 0)
