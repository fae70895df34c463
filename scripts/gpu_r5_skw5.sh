#!/bin/bash
# Round-5: wide short-K plans 256x128 + 128x256 (TAIR_SK_WIDE=5, 256x160 left out: it moved the B=64 sampler
# parity) vs none (libtair_cldm_skw0.so): B=64 parity, GEMM tests, configs[2] paired.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step p64_skw5 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cldm_gpu.py || exit 1
step cfg2_skw5 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=skw0 step cfg2_skw0 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
