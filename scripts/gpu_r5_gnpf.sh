#!/bin/bash
# Round-5: GroupNorm apply with the next two rows loaded before the current two are applied (TAIR_GN_PREFETCH)
# vs libtair_cldm_gnpf0.so: kernel tests, apply bandwidth (interleaved), configs[2] and B=1.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -1 "gpurun_out/$name.log" | cut -c1-160; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step gtests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gn or group or norm" || exit 1
for r in 1 2; do
  step gn_pf$r 200 python -u tools/gn_probe.py --batch 64 || exit 1
  TAIR_LIB_VARIANT=gnpf0 step gn_base$r 200 python -u tools/gn_probe.py --batch 64 || exit 1
done
step cfg2_pf 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=gnpf0 step cfg2_base 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step b1_pf 300 $B || exit 1
TAIR_LIB_VARIANT=gnpf0 step b1_base 300 $B || exit 1
