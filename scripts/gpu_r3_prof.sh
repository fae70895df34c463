#!/bin/bash
# Round-3 rocprof evidence: B=1 kernel stats + PMC traffic (scripts/gpu_profile.sh), B=16 kernel stats;
# the raw traces are pruned on the box (gpurun copies back <= 64 MiB), the summaries stay.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r03* gpurun_out/pmc_r03*
B=1 TAG=r03b1 bash scripts/gpu_profile.sh || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r03b16 -o run --output-format csv -- python3 bench.py --steps 1 \
  --warmup 1 --batch 16 --no-cpu-baseline --no-profile --no-stage3-probe > gpurun_out/prof_r03b16.log 2>&1 || exit $?
tail -1 gpurun_out/prof_r03b16.log | cut -c1-200
for d in gpurun_out/prof_r03b1 gpurun_out/prof_r03b16; do
  f=$(ls $d/*kernel_trace.csv $d/*/*kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/trace_step.py "$f" step_update $d/step_timeline.txt > $d/step_summary.txt 2>&1
done
find gpurun_out/prof_r03* gpurun_out/pmc_r03* -name '*.csv' ! -name '*kernel_stats.csv' -delete
find gpurun_out/prof_r03* gpurun_out/pmc_r03* -name '*.db' -delete
du -sh gpurun_out
