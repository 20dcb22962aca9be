"""Experiment: LDS ladder vs starting every document in the HBM class (tables in global
memory, no LDS residency cap) for the config-2 and config-3 shapes."""
import sys; sys.path.insert(0, '.')
import fluidframework_amd as fa
for (n, ops, pi, pr) in [(4096, 2000, 60, 40), (8192, 10000, 55, 35)]:
    for cap in (0, 60000):
        with fa.ReplayBatch(n, seg_cap=cap) as b:
            b.generate(fa.gen_params(ops, pct_insert=pi, pct_remove=pr, seed=0xDEADBEEF))
            b.run(); b.run()
            st = b.stats()
            print(n, ops, cap, round(st['kernel_ms'], 1), [(l['seg_class'], l['n_docs'], round(l['ms'], 1)) for l in b.launches()], flush=True)
