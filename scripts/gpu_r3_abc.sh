#!/bin/bash
# Library variants A (items in flight 2 beside small tiles), B (1 everywhere), C (B + 4 waves/SIMD
# launch bound on 64x64 tiles): probe + B=1 / B=16 bench each.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in A B C; do
  cp tair_amd/libtair_$v.so.bin tair_amd/libtair_cldm.so
  timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --shapes proj64,qkv64,ff1_64,proj32,qkv32,ff2_64 --tiles "0x0" > gpurun_out/abc_probe_$v.log 2>&1 || exit $?
  echo "== $v"; grep shape gpurun_out/abc_probe_$v.log | cut -c1-120
  timeout -k 10 200 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/abc_b1_$v.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/abc_b1_$v.log').read().strip().splitlines()[-1]); print('b1', '$v', r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
  timeout -k 10 300 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-stage3-probe --no-profile > gpurun_out/abc_b16_$v.log 2>&1 || exit $?
  python3 -c "import json; r=json.loads(open('gpurun_out/abc_b16_$v.log').read().strip().splitlines()[-1]); print('b16', '$v', r['breakdown_ms']['per_denoise_step_per_micro_batch'])"
done
