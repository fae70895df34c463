#!/bin/bash
# Kernel-argument placement A/B (HIP_FORCE_DEV_KERNARG): phase stamps of B=1 GEMM launches and the B=1 bench step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n ${TAILN:-3} "gpurun_out/$name.log" | cut -c1-500; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
SH=lin64proj,lin16proj,conv64,conv16
TAILN=5 TAIR_LIB_VARIANT=stamps step stamps_kdef 200 python -u tools/b1_stamps.py --shapes $SH --variants plan || exit 1
TAILN=5 HIP_FORCE_DEV_KERNARG=1 TAIR_LIB_VARIANT=stamps step stamps_kdev 200 python -u tools/b1_stamps.py --shapes $SH --variants plan || exit 1
TAILN=5 HIP_FORCE_DEV_KERNARG=0 TAIR_LIB_VARIANT=stamps step stamps_khost 200 python -u tools/b1_stamps.py --shapes $SH --variants plan || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_kdef 300 $B || exit 1
HIP_FORCE_DEV_KERNARG=1 step bench_kdev 300 $B || exit 1
HIP_FORCE_DEV_KERNARG=0 step bench_khost 300 $B || exit 1
step pytest_fwd 600 python -u -m pytest tests/test_cldm_gpu.py -x -q -k "forward_parity or no_control or restoration_50" --timeout 300 --timeout-method thread -p no:cacheprovider || exit 1
