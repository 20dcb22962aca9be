#!/bin/bash
# Run GPU steps on the gpurun box; stop at the first crash-type exit (fault/abort/timeout).
set -u
mkdir -p gpurun_out
run() {
  local name=$1 limit=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "fatal exit in $name; stopping"; exit $rc; fi
  return 0
}
for step in "$@"; do
  case "$step" in
    tests) run tests 900 python -u -m pytest tests -m gpu -x -v -s --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    smoke) run smoke 300 python -u __graft_entry__.py smoke ;;
    bench) run bench 900 python -u bench.py --steps 3 --warmup 1 ;;
    benchfinal) run benchfinal 600 python -u bench.py --steps 20 --warmup 5 ;;
    bench2) run bench2 600 python -u bench.py --config 2 --steps 3 --warmup 1 ;;
    bench3) run bench3 900 python -u bench.py --config 3 --docs 2048 --steps 2 --warmup 1 ;;
    gianttests) run gianttests 600 python -u -m pytest tests/test_gpu_parity.py -k "giant or 16_bit or wide_collab or hbm_class or escalation" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider ;;
    giant1m) run giant1m 600 python -u -m pytest tests/test_gpu_parity.py -k "million_segments" -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider ;;
    hbmphases) run hbmphases 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python -u tools/hbm_phases.py 100000 8 ;;
    hbmrate) run hbmrate 600 python -u tools/hbm_phases.py 100000 8 ;;
    hbmrate_base) run hbmrate_base 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_base.so python -u tools/hbm_phases.py 100000 8 ;;
    hbmrate_rangeonly) run hbmrate_rangeonly 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_rangeonly.so python -u tools/hbm_phases.py 100000 8 ;;
    pmcGA) run pmcGA 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmcGA -o run -- python3 -u tools/hbm_phases.py 100000 8 ;;
    pmcGB) run pmcGB 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcGB -o run -- python3 -u tools/hbm_phases.py 100000 8 ;;
    b3s) run b3s 600 python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    jsontests) run jsontests 600 python -u -m pytest tests/test_gpu_json.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    b3s_base) run b3s_base 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_base.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    b3s_lazy) run b3s_lazy 600 python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    b3s_eager) run b3s_eager 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_eagercold.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    f3s_lazy) run f3s_lazy 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f3s_lazy -o run -- python3 -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    f3s_eager) run f3s_eager 180 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_eagercold.so rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/f3s_eager -o run -- python3 -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    hbmrate_nocache) run hbmrate_nocache 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_nocache.so python -u tools/hbm_phases.py 100000 8 ;;
    bisect) run bisect 600 python -u tools/gpu_bisect.py ;;
    bisect3) run bisect3 600 python -u tools/gpu_bisect.py --ops 1500 --docs 32 --ins 55 --rem 35 --seed 0xBADC0DE ;;
    b3s_notext) run b3s_notext 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_notext.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    b3s_var) run b3s_var 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_var.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    b3full) run b3full 600 python -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    b3full_var) run b3full_var 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_var.so python -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    c2) run c2 600 python -u bench.py --config 2 --steps 5 --warmup 2 ;;
    earlytest) run earlytest 300 python -u -m pytest tests/test_gpu_parity.py -k "early_escalation or several_classes or escalation" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    c2w) run c2w 600 python -u bench.py --config 2 --writers --steps 3 --warmup 1 ;;
    c2wnsp) run c2wnsp 600 env MT_EARLY_SETPRIO=0 python -u bench.py --config 2 --writers --steps 3 --warmup 1 --no-cpu ;;
    c2wne) run c2wne 600 env MT_EARLY_ESCALATION=0 python -u bench.py --config 2 --writers --steps 3 --warmup 1 --no-cpu ;;
    c5ne) run c5ne 900 env MT_EARLY_ESCALATION=0 python -u bench.py --config 5 --steps 3 --warmup 1 --no-cpu ;;
    c5) run c5 900 python -u bench.py --config 5 --steps 3 --warmup 1 ;;
    fullpar) run fullpar 900 python -u tools/full_parity.py 65536 8192 gpurun_out/full_parity_config3.json ;;
    c4) run c4 900 python -u bench.py --config 4 --steps 1 --warmup 0 ;;
    b3s_old) run b3s_old 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_old.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    giantrate) run giantrate 600 python -u tools/hbm_phases.py 100000 8 2000000 ;;
    giantrate_nopf) run giantrate_nopf 600 env MT_GIANT_PREFETCH=0 python -u tools/hbm_phases.py 100000 8 2000000 ;;
    l2giant) run l2giant 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/l2giant -o run -- python3 -u tools/hbm_phases.py 100000 8 2000000 ;;
    l2giant_nopf) run l2giant_nopf 300 env MT_GIANT_PREFETCH=0 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/l2giant_nopf -o run -- python3 -u tools/hbm_phases.py 100000 8 2000000 ;;
    ptests) run ptests 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_snapshot.py -k "any_size or combining or markers or kats or escalation" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    prof) run prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    phases) run phases 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python -u bench.py --steps 1 --warmup 0 --no-cpu ;;
    phases3) run phases3 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    docs256) run docs256 600 python -u bench.py --docs 256 --steps 2 --warmup 1 --no-cpu ;;
    docs1024) run docs1024 600 python -u bench.py --docs 1024 --steps 2 --warmup 1 --no-cpu ;;
    pmc1) run pmc1 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d gpurun_out/pmc1 -o run -- python3 -u bench.py --docs 1024 --steps 1 --warmup 0 --no-cpu ;;
    pmc2) run pmc2 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc2 -o run -- python3 -u bench.py --docs 1024 --steps 1 --warmup 0 --no-cpu ;;
    pmcf) run pmcf 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu ;;
    pmcw) run pmcw 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw -o run -- python3 -u bench.py --steps 1 --warmup 0 --no-cpu ;;
    full3) run full3 900 python -u bench.py --config 3 --docs 65536 --steps 1 --warmup 0 --no-cpu ;;
    full3p) run full3p 900 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_prof.so python -u bench.py --config 3 --docs 8192 --steps 1 --warmup 0 --no-cpu ;;
    snaptests) run snaptests 300 python -u -m pytest tests/test_gpu_snapshot.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    benchsnap) run benchsnap 600 python -u bench.py --snapshot --steps 3 --warmup 1 --no-cpu ;;
    bench5) run bench5 900 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    profsnap) run profsnap 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profsnap -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    benchw2) run benchw2 600 python -u bench.py --config 2 --writers --steps 3 --warmup 1 ;;
    benchw3) run benchw3 900 python -u bench.py --config 3 --docs 8192 --writers --steps 2 --warmup 1 ;;
    bench2o) run bench2o 600 python -u bench.py --config 2 --steps 3 --warmup 1 --no-cpu ;;
    bench3s_wpe4) run bench3s_wpe4 900 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_wpe4.so python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    bench3s) run bench3s 900 python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    writertests) run writertests 600 python -u -m pytest tests/test_gpu_writer.py tests/test_node_host.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    bench4s) run bench4s 600 python -u bench.py --config 4 --docs 4096 --ops 20000 --steps 1 --warmup 0 --no-cpu ;;
    bench4) run bench4 1100 python -u bench.py --config 4 --steps 1 --warmup 0 ;;
    loadtests) run loadtests 300 python -u -m pytest tests/test_gpu_snapshot_load.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    cap848) run cap848 600 python -u bench.py --steps 1 --warmup 0 --no-cpu --seg-cap 848 ;;
    cap456) run cap456 600 python -u bench.py --steps 1 --warmup 0 --no-cpu --seg-cap 456 ;;
    cap280) run cap280 600 python -u bench.py --steps 1 --warmup 0 --no-cpu --seg-cap 280 ;;
    cap628) run cap628 600 python -u bench.py --steps 1 --warmup 0 --no-cpu --seg-cap 628 ;;
    listpmc) run listpmc 120 rocprofv3 -L ;;
    pmcA3) run pmcA3 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcB3) run pmcB3 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcC3) run pmcC3 300 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_ATOMIC_BANDWIDTH --output-format csv -d gpurun_out/pmcC3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcC2) run pmcC2 200 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_LDS_LOAD_BANDWIDTH SQ_INSTS_LDS_STORE_BANDWIDTH SQ_INSTS_LDS_ATOMIC_BANDWIDTH --output-format csv -d gpurun_out/pmcC2 -o run -- python3 -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu ;;
    pmcD3) run pmcD3 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_TCC_READ_REQ_LATENCY TCP_TCP_LATENCY TCC_HIT TCC_MISS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d gpurun_out/pmcD3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcf3) run pmcf3 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcw3) run pmcw3 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw3 -o run -- python3 -u bench.py --config 3 --steps 1 --warmup 0 --no-cpu ;;
    pmcA2) run pmcA2 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmcA2 -o run -- python3 -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu ;;
    pmcB2) run pmcB2 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d gpurun_out/pmcB2 -o run -- python3 -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu ;;
    pmcf2) run pmcf2 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf2 -o run -- python3 -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu ;;
    pmcw2) run pmcw2 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw2 -o run -- python3 -u bench.py --config 2 --steps 1 --warmup 0 --no-cpu ;;
    jsontests) run jsontests 300 python -u -m pytest tests/test_gpu_json.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    benchjson) run benchjson 600 python -u tools/bench_json.py ;;
    benchjson3) run benchjson3 600 python -u tools/bench_json.py --docs 512 --ops 10000 --mix 55,35 ;;
    prof3) run prof3 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof3 -o run -- python3 -u bench.py --steps 3 --warmup 1 --no-cpu ;;
    *) echo "unknown step $step" ;;
  esac
done
