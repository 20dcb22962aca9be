#!/bin/bash
# round-5 GPU steps (each under its own time limit; stop at the first failure):
#   tests            the -m gpu suite
#   parity           tests/test_gpu_parity.py only
#   c2 / c3s / c3    bench config 2 / config-3 slice (8,192 docs) / config 3 (default lib)
#   c3s_q0 / c3s_z0 / c3s_q0z0  the config-3 slice with the deferred text queue off (MT_TEXT_QUEUE=0),
#                    the zamboni prefetch off (MT_ZAMBONI_PREFETCH=0), both off
#   c3s_base / c2_base  the same with fluidframework_amd/libmtreplay_base.so (the previous tree)
#   c3s_a / c2_a     the same with fluidframework_amd/libmtreplay_r5a.so (an A/B reference build)
#   phases3 / phases3f  MT_PROF phase + drain profile of the config-3 slice / full config 3 (libmtreplay_prof.so)
#   c4               bench config 4 (Zipf sizes, the giant class), one step
#   prof3            rocprofv3 kernel stats of the headline bench
set -u
mkdir -p gpurun_out
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1
  local rc=$?
  echo "== $name rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|"GB_per_s": [0-9.]*\|"host_match": [0-9]*\|"launches_per_step": [0-9]*\|[0-9]* passed\|[0-9]* failed' gpurun_out/$name.log | sort | uniq -c | tr '\n' ' ')"
  if [ $rc -ne 0 ]; then tail -40 gpurun_out/$name.log; exit $rc; fi
}
BASE=fluidframework_amd/libmtreplay_base.so
PROF=fluidframework_amd/libmtreplay_prof.so
C3S="bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu"
C2="bench.py --config 2 --steps 3 --warmup 1 --no-cpu"
B3="bench.py --config 3 --steps 1 --warmup 0 --no-cpu"
B3S="bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu"
PT="-x -v --timeout 200 --timeout-method thread -p no:cacheprovider"
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu $PT ;;
    parity) step parity 600 python -u -m pytest tests/test_gpu_parity.py -m gpu $PT ;;
    gjson) step gjson 400 python -u -m pytest tests/test_gpu_json.py -m gpu $PT ;;
    shard) step shard 300 python -u -m pytest tests/test_gpu_shard.py -m gpu $PT ;;
    writer) step writer 600 python -u -m pytest tests/test_gpu_writer.py -m gpu $PT ;;
    smoke) step smoke 300 python -u __graft_entry__.py smoke ;;
    c2) step c2 300 python -u $C2 ;;
    c2_base) step c2_base 300 env FLUIDFRAMEWORK_AMD_LIB=$BASE python -u $C2 ;;
    c3s) step c3s 400 python -u $C3S ;;
    c3s_q0) step c3s_q0 400 env MT_TEXT_QUEUE=0 python -u $C3S ;;
    c3s_base) step c3s_base 400 env FLUIDFRAMEWORK_AMD_LIB=$BASE python -u $C3S ;;
    c3s_a) step c3s_a 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5a.so python -u $C3S ;;
    c2_a) step c2_a 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5a.so python -u $C2 ;;
    c3s_ilp) step c3s_ilp 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_ilp.so python -u $C3S ;;
    c2_ilp) step c2_ilp 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_ilp.so python -u $C2 ;;
    giant) step giant 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "giant or million or hbm_class or 16_bit or escalation" -x -v -s --timeout 600 --timeout-method thread -p no:cacheprovider ;;
    grate) step grate 400 python -u tools/hbm_phases.py 100000 8 2000000 ;;
    grate_a) step grate_a 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5a.so python -u tools/hbm_phases.py 100000 8 2000000 ;;
    c3s_z0) step c3s_z0 400 env MT_ZAMBONI_PREFETCH=0 python -u $C3S ;;
    c3s_q0z0) step c3s_q0z0 400 env MT_TEXT_QUEUE=0 MT_ZAMBONI_PREFETCH=0 python -u $C3S ;;
    c3) step c3 600 python -u bench.py --steps 3 --warmup 1 ;;
    phases3f) step phases3f 600 env FLUIDFRAMEWORK_AMD_LIB=$PROF python -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    c3fs[1-4]*) n=${s#c3fs}; step $s 400 env MT_FIRST_SPLIT=${n%%_*} python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    c5) step c5 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    c5fs1) step c5fs1 400 env MT_FIRST_SPLIT=1 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    pcap) step pcap 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -k "beyond_64_keys" $PT ;;
    c3lpt[01]*) v=${s#c3lpt}; step $s 400 env MT_LPT=${v%%_*} python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    snap) step snap 600 python -u -m pytest tests/test_gpu_snapshot.py tests/test_gpu_snapshot_load.py -m gpu $PT ;;
    c5b) step c5b 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5b.so python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    c5_*) step $s 400 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    c5b_*) step $s 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5b.so python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    prof5n) step prof5n 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5n -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    prof5b) step prof5b 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5b.so rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5b -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    pmcA5n) step pmcA5n 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA5n -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    pmcB5n) step pmcB5n 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB5n -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    pmcw5n) step pmcw5n 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw5n -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 1 --warmup 0 --no-cpu ;;
    c3n_*) step $s 400 python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    c3b_*) step $s 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_r5b.so python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    c3ht) step c3ht 400 env MT_HOST_TIMING=1 python -u bench.py --config 3 --steps 1 --warmup 1 --no-cpu ;;
    c3sf*) v=${s#c3sf}; step $s 400 env MT_SPLIT_FRAC=0.${v%%_*} python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    c3prio*) step $s 400 env MT_CHAIN_PRIO=1 python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    fullpar) step fullpar 1100 python -u tools/full_parity.py 65536 8192 gpurun_out/full_parity_config3.json ;;
    pmcA4) step pmcA4 500 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA4 -o run -- python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu ;;
    pmcB4) step pmcB4 500 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB4 -o run -- python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu ;;
    pmcf4) step pmcf4 500 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf4 -o run -- python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu ;;
    pmcw4) step pmcw4 500 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw4 -o run -- python3 -u bench.py --config 4 --steps 1 --warmup 0 --no-cpu ;;
    c3v_*) v=${s#c3v_}; step $s 400 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_${v%%_*}.so python -u bench.py --config 3 --steps 2 --warmup 1 --no-cpu ;;
    rehearse2) step rehearse2 600 env MT_BENCH_BACKEND=gloo python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 2 --warmup 1 --docs 32768 --no-cpu ;;
    c2w) step c2w 400 python -u bench.py --config 2 --writers --steps 3 --warmup 1 ;;
    c2f) step c2f 300 python -u bench.py --config 2 --steps 3 --warmup 1 ;;
    c4) step c4 1000 python -u bench.py --config 4 --steps 1 --warmup 0 ;;
    phases3) step phases3 400 env FLUIDFRAMEWORK_AMD_LIB=$PROF python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    pmcA3) step pmcA3 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA3 -o run -- python3 -u $B3 ;;
    pmcB3) step pmcB3 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB3 -o run -- python3 -u $B3 ;;
    pmcf3) step pmcf3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf3 -o run -- python3 -u $B3 ;;
    pmcw3) step pmcw3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3 -o run -- python3 -u $B3 ;;
    b3s1) step b3s1 300 python -u $B3S ;;
    b3c1) step b3c1 300 python -u $B3S --seg-cap 2046 ;;
    pmcf3s) step pmcf3s 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf3s -o run -- python3 -u $B3S ;;
    pmcw3s) step pmcw3s 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3s -o run -- python3 -u $B3S ;;
    pmcf3c) step pmcf3c 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf3c -o run -- python3 -u $B3S --seg-cap 2046 ;;
    pmcw3c) step pmcw3c 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3c -o run -- python3 -u $B3S --seg-cap 2046 ;;
    bench3one) step bench3one 300 python -u $B3 ;;
    driver) step driver 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof3) step prof3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
