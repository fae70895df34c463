#!/bin/bash
# Halo-tile conv kernel: kernel tests, forward parity, then A/B (TAIR_HALO=0 vs default) at B=1 and B=64.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -3 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step r4_halo_kern 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -k "conv3" -x -v --timeout 120 --timeout-method thread -p no:cacheprovider || exit 1
step r4_halo_fwd 400 python -u -m pytest tests/test_cldm_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider || exit 1
B64="--batch 64 --tiles 64 --steps 1 --warmup 1 --no-cpu-baseline --no-profile --no-stage3-probe"
step r4_halo_b64_on 300 python -u bench.py $B64 || exit 1
TAIR_HALO=0 step r4_halo_b64_off 300 python -u bench.py $B64 || exit 1
B1="--steps 3 --warmup 1 --no-cpu-baseline --no-profile --no-stage3-probe"
step r4_halo_b1_on 300 python -u bench.py $B1 || exit 1
TAIR_HALO=0 step r4_halo_b1_off 300 python -u bench.py $B1 || exit 1
