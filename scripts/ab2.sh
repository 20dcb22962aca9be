#!/bin/bash
# A/B of library variants on the config-3 slice (8,192 docs): for each round, each variant in turn
# (`base` = fluidframework_amd/libmtreplay.so, else libmtreplay_<name>.so); digests must agree
set -u
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    lib=fluidframework_amd/libmtreplay.so; [ "$v" = base ] || lib=fluidframework_amd/libmtreplay_$v.so
    timeout -k 10 300 env FLUIDFRAMEWORK_AMD_LIB=$lib python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu > gpurun_out/ab_${v}_$r.log 2>&1
    rc=$?
    echo "== $v round $r rc=$rc $(grep -o '"value": [0-9.]*\|"digest_xor": "[0-9a-f]*"' gpurun_out/ab_${v}_$r.log | tr '\n' ' ')"
    [ $rc -eq 0 ] || { tail -20 gpurun_out/ab_${v}_$r.log; exit $rc; }
  done
done
