#!/bin/bash
# rocprof kernel stats of the configs[4] prompt loop (10 steps), raw traces pruned on the box.
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_s3
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_s3 -o run -- python3 bench.py \
  --config 4 --steps 1 --warmup 0 --sampling-steps 10 --no-cpu-baseline --no-profile > gpurun_out/prof_s3.log 2>&1
rc=$?
find gpurun_out/prof_s3 -name "*.csv" ! -name "*kernel_stats.csv" -delete
exit $rc
