#!/bin/bash
# A/B: parity suite on the current build, then config 2 / config 3 (8,192 docs) for the current
# and the baseline library (fluidframework_amd/libmtreplay_base.so)
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|passed\|failed' gpurun_out/$name.log | sort | uniq -c | tr '\n' ' '; echo; [ $rc -eq 0 ] || { tail -30 gpurun_out/$name.log; exit $rc; }; }
step tests 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step c2_new 300 python -u bench.py --steps 3 --warmup 1 --no-cpu
step c2_base 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_base.so python -u bench.py --steps 3 --warmup 1 --no-cpu
step c3_new 300 python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 1 --no-cpu
step c3_base 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_base.so python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 1 --no-cpu
