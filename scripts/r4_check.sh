#!/bin/bash
# round-4 GPU check: the -m gpu suite, then config 2 and a config-3 slice (8,192 documents)
set -u
mkdir -p gpurun_out
step() { local name=$1 lim=$2; shift 2; echo "== $name: $*"; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "== $name rc=$rc"; grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|"GB_per_s": [0-9.]*\|"host_match": [0-9]*\|[0-9]* passed\|[0-9]* failed' gpurun_out/$name.log | sort | uniq -c | tr '\n' ' '; echo; if [ $rc -ne 0 ]; then tail -40 gpurun_out/$name.log; exit $rc; fi; }
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ;;
    c2) step c2 300 python -u bench.py --steps 3 --warmup 1 --no-cpu --config 2 ;;
    c3s) step c3s 400 python -u bench.py --config 3 --docs 8192 --steps 2 --warmup 1 --no-cpu ;;
    c3) step c3 600 python -u bench.py --steps 3 --warmup 1 ;;
    snap) step snap 300 python -u -m pytest tests/test_gpu_snapshot.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider ;;
    c5) step c5 600 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    c5serial) step c5serial 600 env MT_SNAP_SERIAL=1 python -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    c5s) step c5s 600 python -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    c5srec) step c5srec 600 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_recloop.so python -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu ;;
    snapphases) step snapphases 300 env FLUIDFRAMEWORK_AMD_LIB=fluidframework_amd/libmtreplay_snapprof.so python -u tools/snap_phases.py 8192 2000 ;;
    default) step default 600 python -u bench.py ;;
    c5full) step c5full 900 python -u bench.py --config 5 --steps 2 --warmup 1 --no-cpu ;;
    giant) step giant 600 python -u -m pytest tests/test_gpu_parity.py -k "giant or 16_bit or wide_collab or hbm_class or escalation or million" -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider ;;
    *) echo "unknown $s"; exit 2 ;;
  esac
done
