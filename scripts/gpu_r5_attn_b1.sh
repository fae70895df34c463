#!/bin/bash
# Round-5: B=1 attention plan sweep on the final kernel (bare v_exp_f32 softmax), two passes.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --batch 1 > gpurun_out/attn_b1_sweep1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/attn_bench.py --batch 1 > gpurun_out/attn_b1_sweep2.log 2>&1 || exit 1
