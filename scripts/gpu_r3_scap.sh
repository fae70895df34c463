#!/bin/bash
# B=1 A/B: cap on the small-grid split count (in-kernel combine covers <= 3 slices).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for c in 16 3 4 6 8; do
  TAIR_SPLIT_CAP=$c timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/scap_$c.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/scap_$c.log').read().strip().splitlines()[-1]); print('cap', $c, r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
done
