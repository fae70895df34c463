#!/bin/bash
# 4 vs 5 waves/SIMD launch bound on the 2-stage 64x64 tiles (5: 96 VGPRs, 160 B/lane scratch):
# short-K probe + B=16 bench each, then the GEMM kernel tests on the faster one is left to a later call.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in W4 W5 W4 W5; do
  cp tair_amd/libtair_$v.so.bin tair_amd/libtair_cldm.so
  timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --shapes proj64,qkv64,ff1_64,proj32,qkv32,ff2_64 --tiles "0x0" > gpurun_out/w5_probe_$v.log 2>&1 || exit $?
  echo "== $v"; grep shape gpurun_out/w5_probe_$v.log | cut -c1-120
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/w5_b16_$v.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/w5_b16_$v.log').read().strip().splitlines()[-1]); print('b16', '$v', r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
done
cp tair_amd/libtair_W4.so.bin tair_amd/libtair_cldm.so
