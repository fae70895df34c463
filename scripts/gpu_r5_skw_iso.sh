#!/bin/bash
# Round-5: which wide short-K tile shape moves the B=64 sampler parity (TAIR_SK_WIDE bit variants:
# skw1 256x128, skw2 256x160, skw4 128x256). A failed assertion (rc 1) goes on to the next variant; any other
# non-zero status stops the script.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
for v in skw1 skw2 skw4; do
  TAIR_LIB_VARIANT=$v timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_cldm_gpu.py -k "batch64" > gpurun_out/p64_$v.log 2>&1
  rc=$?; echo "$v rc=$rc"; tail -1 gpurun_out/p64_$v.log
  [ $rc -le 1 ] || exit $rc
  grep -h "sampler_b64_4steps" gpurun_out/parity.jsonl | tail -1
done
