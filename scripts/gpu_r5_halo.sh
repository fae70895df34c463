#!/bin/bash
# Round-5: nine-tap unrolled halo conv loop vs the round-4 loop (oldloop variant): kernel tests of the halo
# tiles, conv_probe at B=64 (forced 256x160 halo, with / without epilogue), configs[2] bench with each.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -4 "gpurun_out/$name.log" | cut -c1-200; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step ktests 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "halo or conv" || exit 1
for v in new oldloop; do
  if [ $v = new ]; then unset TAIR_LIB_VARIANT; else export TAIR_LIB_VARIANT=oldloop; fi
  for sh in 64,320,320 32,640,640 16,1280,1280; do
    step cp_${v}_${sh//,/_} 200 python -u tools/conv_probe.py --batch 64 --force 256x160/1/9 --only $sh --tag $v || exit 1
    step cpne_${v}_${sh//,/_} 200 python -u tools/conv_probe.py --batch 64 --force 256x160/1/9 --only $sh --no-epilogue --tag $v || exit 1
  done
done
unset TAIR_LIB_VARIANT
step cfg2_new 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
TAIR_LIB_VARIANT=oldloop step cfg2_old 600 python -u bench.py --config 2 --no-cpu-baseline --no-stage3-probe --no-profile || exit 1
