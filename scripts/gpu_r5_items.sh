#!/bin/bash
# Round-5 epilogue anatomy: per-item stamps of thread 0 (stamps2 variant) for B=1 linears / convs.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-600; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
TAIR_LIB_VARIANT=stamps2 step items 300 python -u tools/b1_stamps.py \
  --shapes lin64proj,lin32proj,lin16proj,lin8proj,lin16ff2,conv64,conv16 --variants plan,e1:plan || exit 1
