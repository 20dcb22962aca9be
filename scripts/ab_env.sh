#!/bin/bash
# A/B of an environment toggle: ab_env.sh ROUNDS CONFIGS VAR; each round runs each config with VAR=0 then VAR=1
# (configs: c2 = config 2, c3s = config-3 slice of 8,192 documents, c3 = config 3); digests must agree
set -u
mkdir -p gpurun_out
rounds=$1; configs=$2; var=$3
for r in $(seq 1 $rounds); do
  for c in $configs; do
    case $c in
      c2) args="--config 2 --steps 3 --warmup 1" ;;
      c3s) args="--config 3 --docs 8192 --steps 2 --warmup 1" ;;
      c3) args="--config 3 --steps 3 --warmup 1" ;;
    esac
    for v in 0 1; do
      log=gpurun_out/abenv_${c}_${v}_$r.log
      timeout -k 10 400 env $var=$v python -u bench.py $args --no-cpu > $log 2>&1
      rc=$?
      echo "== $c $var=$v round $r rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"digest_xor": "[0-9a-f]*"\|"launches": [0-9]*' $log | tr '\n' ' ')"
      [ $rc -eq 0 ] || { tail -20 $log; exit $rc; }
    done
  done
done
