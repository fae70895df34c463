#!/bin/bash
# XCD tile-order A/B at B=1 and B=16 (TAIR_XCD: 0 auto, 1 m-fastest, 2 n-fastest, 3 auto + bytes rule).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for x in 0 3 2 1; do
  TAIR_XCD=$x timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/xcd_$x.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/xcd_$x.log').read().strip().splitlines()[-1]); print('xcd', $x, 'b1', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
done
for x in 0 3; do
  TAIR_XCD=$x timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/xcd16_$x.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/xcd16_$x.log').read().strip().splitlines()[-1]); print('xcd', $x, 'b16', r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
done
