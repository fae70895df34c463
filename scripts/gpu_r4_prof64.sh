#!/bin/bash
# rocprofv3 kernel stats of the B=64 denoise step, bf16 vs fp8 (bench.py --profile-only: 2 graph steps + 1 eager)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for v in bf16 fp8; do
  X=""; [ $v = fp8 ] && X="--fp8"
  echo "== $v ($(date +%T))"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64_$v -o run --output-format csv -- \
    python3 bench.py --profile-only --sampling-steps 2 --batch 64 $X > gpurun_out/prof64_$v.log 2>&1 || exit 1
done
