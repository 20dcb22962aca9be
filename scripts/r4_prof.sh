#!/bin/bash
# round-4 measurements: the headline bench, its kernel stats, phase profile and PMC passes, and the
# SnapshotV1 kernels' stats (each GPU step under its own time limit; stop at the first failure)
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name: $*"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|"GB_per_s": [0-9.]*\|"host_match": [0-9]*\|[0-9]* passed\|[0-9]* failed' gpurun_out/$name.log | sort | uniq -c | tr '\n' ' '; echo; if [ $rc -ne 0 ]; then tail -30 gpurun_out/$name.log; exit $rc; fi; }
B3="bench.py --config 3 --steps 1 --warmup 0 --no-cpu"
for s in "$@"; do
  case $s in
    c3) step c3 600 python -u bench.py --steps 3 --warmup 1 ;;
    prof3) step prof3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    phases3) step phases3 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    pmcA3) step pmcA3 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA3 -o run -- python3 -u $B3 ;;
    pmcB3) step pmcB3 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB3 -o run -- python3 -u $B3 ;;
    pmcf3) step pmcf3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf3 -o run -- python3 -u $B3 ;;
    pmcw3) step pmcw3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3 -o run -- python3 -u $B3 ;;
    bench3one) step bench3one 300 python -u $B3 ;;
    prof5) step prof5 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    pmcA5) step pmcA5 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA5 -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    pmcB5) step pmcB5 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB5 -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    pmcw5) step pmcw5 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw5 -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    prof5f) step prof5f 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5f -o run -- python3 -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    pmcA5f) step pmcA5f 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA5f -o run -- python3 -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu ;;
    pmcB5f) step pmcB5f 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB5f -o run -- python3 -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu ;;
    pmcw5f) step pmcw5f 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw5f -o run -- python3 -u bench.py --config 5 --steps 1 --warmup 0 --no-cpu ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
