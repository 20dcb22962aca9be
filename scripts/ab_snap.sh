#!/bin/bash
# A/B of library variants on the config-5 slice (32,768 docs): SnapshotV1 GB/s per variant
set -u
mkdir -p gpurun_out
for v in "$@"; do
  lib=fluidframework_amd/libmtreplay.so; [ "$v" = base ] || lib=fluidframework_amd/libmtreplay_$v.so
  timeout -k 10 300 env FLUIDFRAMEWORK_AMD_LIB=$lib python -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/absnap_$v.log 2>&1
  rc=$?
  echo "== $v rc=$rc $(grep -o '"GB_per_s": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|"host_match": [0-9]*' gpurun_out/absnap_$v.log | tr '\n' ' ')"
  [ $rc -eq 0 ] || { tail -20 gpurun_out/absnap_$v.log; exit $rc; }
done
