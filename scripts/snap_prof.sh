#!/bin/bash
# kernel statistics of the config-5 slice (32,768 documents): replay + SnapshotV1 kernels
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/snapprof -o run -- python3 -u bench.py --config 5 --docs 32768 --steps 2 --warmup 1 --no-cpu > gpurun_out/snapprof.log 2>&1
rc=$?; echo "rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/snapprof.log; exit $rc; }
f=$(find gpurun_out/snapprof -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/snap_kernel_stats.csv
grep -i "snapshot\|digest" gpurun_out/snap_kernel_stats.csv | cut -d, -f1-4
