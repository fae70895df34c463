#!/bin/bash
# In-kernel split-K combine with batched slab reads: GEMM kernel tests, then the B=1 step at
# TAIR_INK_SMAX = 3 / 4 / 6 / 8 / 16 (largest split count combined in-kernel).
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "gemm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/inkb_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/inkb_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for v in 3 16 8 4 6 3 16; do
  TAIR_INK_SMAX=$v timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/inkb_b1_$v.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/inkb_b1_$v.log').read().strip().splitlines()[-1]); print('ink', $v, r['breakdown_ms']['per_denoise_step_per_micro_batch'], r['value'])"
done
