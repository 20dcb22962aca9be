import sys; sys.path.insert(0, '.')
import fluidframework_amd as fa
for (n, ops, pi, pr) in [(32768, 2000, 55, 35), (8192, 10000, 55, 35)]:
    for cap in ([0, 320, 384, 512] if ops == 2000 else [0, 1280, 1664]):
        with fa.ReplayBatch(n, seg_cap=cap) as b:
            b.generate(fa.gen_params(ops, pct_insert=pi, pct_remove=pr, seed=0xDEADBEEF))
            b.run(); b.run()
            st = b.stats()
            print(n, ops, cap, round(st['kernel_ms'], 1), st['launches'], flush=True)
