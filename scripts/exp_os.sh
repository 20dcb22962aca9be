#!/bin/bash
# code-size experiment: -O3 vs -Os replay kernels on configs 2 and 3 (8192 docs), then one
# icache PMC pass
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/$name.log | tr '\n' ' '; echo; [ $rc -eq 0 ] || exit $rc; }
step c2_o3 300 python -u bench.py --steps 3 --warmup 1 --no-cpu
step c2_os 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_os.so python -u bench.py --steps 3 --warmup 1 --no-cpu
step c3_o3 300 python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 1 --no-cpu
step c3_os 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_os.so python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 1 --no-cpu
step pmc_ic 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d gpurun_out/pmc_ic -o run -- python3 -u bench.py --docs 1024 --steps 1 --warmup 0 --no-cpu
