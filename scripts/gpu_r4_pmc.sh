#!/bin/bash
# Round-4 rocprof evidence: kernel stats + PMC summaries for configs[1] (B=1), configs[2] micro-batch (B=64),
# fp8 B=1; the large raw traces are reduced on the box (step summary) and deleted (64 MiB pull cap).
set -o pipefail
for spec in "1 0 r04b1" "64 0 r04b64" "1 1 r04b1_fp8"; do
  set -- $spec
  B=$1 FP8=$2 TAG=$3 bash scripts/gpu_profile.sh || exit 1
  python3 tools/trace_step.py gpurun_out/prof_$3/run_kernel_trace.csv > gpurun_out/step_summary_$3.txt 2>&1
  python3 tools/step_span.py gpurun_out/prof_$3/run_kernel_trace.csv >> gpurun_out/step_summary_$3.txt 2>&1
  rm -f gpurun_out/prof_$3/run_kernel_trace.csv
  rm -rf gpurun_out/pmc_$3_fetch gpurun_out/pmc_$3_write gpurun_out/pmc_$3_mfma
done
du -sh gpurun_out
