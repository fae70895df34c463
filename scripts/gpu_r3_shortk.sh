#!/bin/bash
# Short-K batched linears (B=16): the planner vs 2-stage 128-row tiles (a2:...), with/without epilogue.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --shapes proj64,qkv64,ff1_64,ff2_64,ff1_32,proj32,qkv32,proj16 \
  --tiles "0x0,e2:0x0,a2:64x64,a2:128x128,a2:128x256,e2:a2:128x128,128x128,128x256" > gpurun_out/r3_shortk_b16.log 2>&1 || exit $?
cat gpurun_out/r3_shortk_b16.log
