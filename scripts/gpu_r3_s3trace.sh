#!/bin/bash
# Timeline of the configs[4] prompt loop (10 steps): per-step wall split into our HIP kernels and the
# stock-torch towers (TESTR, CLIP-H), traces pruned on the box.
export TMPDIR=/tmp
mkdir -p gpurun_out
rm -rf gpurun_out/prof_s3t
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_s3t -o run -- python3 bench.py \
  --config 4 --steps 1 --warmup 0 --sampling-steps 10 --no-cpu-baseline --no-profile > gpurun_out/prof_s3t.log 2>&1
rc=$?
f=$(ls gpurun_out/prof_s3t/*kernel_trace.csv gpurun_out/prof_s3t/*/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 tools/stage3_split.py "$f" > gpurun_out/prof_s3t/split.txt 2>&1
find gpurun_out/prof_s3t -name "*.csv" -delete
cat gpurun_out/prof_s3t/split.txt
exit $rc
