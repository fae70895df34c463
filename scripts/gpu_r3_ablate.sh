#!/bin/bash
# Timing-only ablations at B=1 (TAIR_ABLATE: skip launches of a kernel class; outputs are garbage):
# what each fusion could buy at most.  0 = baseline.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for m in ${MASKS:-0 4 8 256 2 268}; do
  TAIR_ABLATE=$m timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/abl_$m.log 2>&1 || exit $?
  python3 -c "import json,sys; r=json.loads(open('gpurun_out/abl_$m.log').read().strip().splitlines()[-1]); print('ablate', $m, r['breakdown_ms']['per_denoise_step_per_micro_batch'], 'ms/step', r['value'])"
done
