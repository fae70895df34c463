#!/bin/bash
# Round-5 B=1 A/B: halo vs tile kernel durations under rocprof, deep-ring / epilogue-U variants in the graph
# probe, and the B=1 bench step with each variant (TAIR_B1_DEEP, TAIR_LIB_VARIANT).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-400; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
step b1prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/b1prof -o run --output-format csv -- \
  python3 -u tools/b1_probe.py --shapes conv64,conv16 --variants plan,e2:plan,halo256x64/s5,e2:halo256x64/s5,halo256x128/s10 --n 20 --reps 2 || exit 1
V=plan,e2:plan,d4:64x64/s1,d5:64x64/s1,d6:64x64/s1,d8:64x64/s1,d4:64x128/s1,d5:64x128/s1,d6:64x128/s1,64x64/s2/sem,d5:64x64/s2/sem
S=lin64proj,lin64qkv,lin64ff2,lin32proj,lin32ff2,lin16proj,lin16ff2,lin8proj,conv64,conv32,conv16,conv8
step probe_base 300 python -u tools/b1_probe.py --shapes $S --variants $V || exit 1
TAIR_LIB_VARIANT=u2 step probe_u2 300 python -u tools/b1_probe.py --shapes $S --variants plan,d5:64x64/s1 || exit 1
TAIR_LIB_VARIANT=u4 step probe_u4 300 python -u tools/b1_probe.py --shapes $S --variants plan,d5:64x64/s1 || exit 1
B="python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-stage3-probe --no-profile"
step bench_base 300 $B || exit 1
TAIR_B1_DEEP=1 step bench_deep 300 $B || exit 1
TAIR_LIB_VARIANT=u2 step bench_u2 300 $B || exit 1
TAIR_B1_DEEP=1 TAIR_LIB_VARIANT=u2 step bench_deep_u2 300 $B || exit 1
TAIR_LIB_VARIANT=u4 step bench_u4 300 $B || exit 1
step probe_warm 300 python -u tools/b1_probe.py --warm --shapes lin64proj,lin32proj,lin16proj,lin8proj,lin16ff2,conv64,conv32,conv16,conv8 --variants plan,e2:plan || exit 1
