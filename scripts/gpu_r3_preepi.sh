#!/bin/bash
# Epilogue operands of 64x64 tiles loaded before the main loop (TAIR_PRE_EPI): kernel tests, probe and
# bench A/B at B=16 and B=1.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
TAIR_PRE_EPI=1 timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider -k "gemm or conv" > gpurun_out/r3_pre_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r3_pre_tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for pe in 0 1; do
  TAIR_PRE_EPI=$pe timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --shapes proj64,qkv64,ff1_64,proj32,qkv32 --tiles "0x0" > gpurun_out/r3_pre_probe_$pe.log 2>&1 || exit $?
  echo "pre_epi=$pe"; grep shape gpurun_out/r3_pre_probe_$pe.log
done
for pe in 0 1; do
  TAIR_PRE_EPI=$pe timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_pre_b1_$pe.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/r3_pre_b1_$pe.log').read().strip().splitlines()[-1]); print('b1 pre', $pe, r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
  TAIR_PRE_EPI=$pe timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/r3_pre_b16_$pe.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/r3_pre_b16_$pe.log').read().strip().splitlines()[-1]); print('b16 pre', $pe, r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
done
