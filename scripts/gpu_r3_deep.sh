#!/bin/bash
# B=1 A/B: deep-ring 64-row tiles (TAIR_DEEP) x split-K worker targets (TAIR_TGT_CONV/LIN).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for cfg in ${CFGS:-"0 400 240" "1 400 240" "1 256 256" "0 256 256" "1 320 200"}; do
  set -- $cfg
  TAIR_DEEP=$1 TAIR_TGT_CONV=$2 TAIR_TGT_LIN=$3 timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/deep_$1_$2_$3.log 2>&1 || exit $?
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/deep_$1_$2_$3.log').read().strip().splitlines()[-1]); print('deep/conv/lin', '$cfg', r['breakdown_ms']['per_denoise_step_per_micro_batch'], 'ms/step', r['value'])"
done
