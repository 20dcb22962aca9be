"""Per-phase cycles of the HBM class (giant documents) with the MT_PROF library:
FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python tools/hbm_phases.py [ops] [docs]
Documents start directly in the HBM class (seg_cap), config-4 op mix (insert 50 / remove 15 /
annotate 35); the library prints mean cycles per document per phase (MT_PROF lines on stderr)."""
import sys
import time

sys.path.insert(0, '.')
import fluidframework_amd as fa

ops = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
docs = int(sys.argv[2]) if len(sys.argv) > 2 else 8
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 2097152
p = fa.gen_params(ops, pct_insert=50, pct_remove=15, seed=0xDEADBEEF)
with fa.ReplayBatch(docs, seg_cap=cap) as b:
    t0 = time.time()
    b.generate(p, 0)
    print(f"generated {docs} x {ops} in {time.time() - t0:.1f} s", flush=True)
    b.run()
    st = b.stats()
    print("kernel_ms", round(st["kernel_ms"], 1), "us/op", round(1e3 * st["kernel_ms"] / ops, 2),
          [(l["seg_class"], l["n_docs"], round(l["ms"], 1), l["ops"]) for l in b.launches()],
          "max_slots", int(b.counters()["max_slots"].max()), flush=True)
