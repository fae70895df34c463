#!/bin/bash
# After restricting the pipelined loop to 8-wave / shallow tiles: kernel tests, B=1/16/64 bench lines, PMC (B=1 bf16, fp8).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
T=${TAG:-b1fix2}
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_${T}_kern.log 2>&1; rc=$?; tail -2 gpurun_out/r4_${T}_kern.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r4_${T}_bench.log 2>&1 || exit 1
B="--no-cpu-baseline --no-profile --no-stage3-probe"
timeout -k 10 300 python -u bench.py --batch 16 --tiles 16 --steps 2 --warmup 1 $B > gpurun_out/r4_${T}_b16.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --batch 64 --tiles 64 --steps 1 --warmup 1 $B > gpurun_out/r4_${T}_b64.log 2>&1 || exit 1
for b in bench b16 b64; do echo "$b $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/r4_${T}_$b.log | head -2 | tr '\n' ' ')"; done
for spec in "1 0 r04b1" "1 1 r04b1_fp8"; do
  set -- $spec
  B=$1 FP8=$2 TAG=$3 bash scripts/gpu_profile.sh || exit 1
  python3 tools/trace_step.py gpurun_out/prof_$3/run_kernel_trace.csv > gpurun_out/step_summary_$3.txt 2>&1
  python3 tools/step_span.py gpurun_out/prof_$3/run_kernel_trace.csv >> gpurun_out/step_summary_$3.txt 2>&1
  rm -f gpurun_out/prof_$3/run_kernel_trace.csv
  rm -rf gpurun_out/pmc_$3_fetch gpurun_out/pmc_$3_write gpurun_out/pmc_$3_mfma
done
