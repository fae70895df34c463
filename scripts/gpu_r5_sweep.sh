#!/bin/bash
# Round-5: split-count sweep under the cooperative combine (graph probe), then the B=1 rocprof + PMC profile.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
step() { local name=$1 lim=$2; shift 2; echo "== $name ($(date +%T))"; timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -2 "gpurun_out/$name.log" | cut -c1-300; return $rc; }
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
S=lin64proj,lin64qkv,lin64ff2,lin32proj,lin32qkv,lin32ff2,lin16proj,lin16qkv,lin16ff2,lin8proj,conv64,conv64cat,conv32,conv32in,conv16,conv16in,conv8,conv8cat,down32,down16,down8,up64,up32,up16
V=plan,64x64/s1,64x64/s2/sem,64x64/s3/sem,64x64/s4/sem,64x64/s6/sem,64x64/s8/sem,64x128/s2/sem,64x128/s4/sem,64x128/s8/sem,64x128/s16/sem
step sweep_coop 600 python -u tools/b1_probe.py --shapes $S --variants $V --reps 3 || exit 1
B=1 TAG=r05b1 timeout -k 10 1000 bash scripts/gpu_profile.sh || exit 1
