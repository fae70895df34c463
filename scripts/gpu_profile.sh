#!/bin/bash
# rocprofv3 evidence for profiles/: kernel-trace stats of the default bench, then one PMC pass per
# counter group (FETCH_SIZE | WRITE_SIZE | MFMA busy + GRBM_GUI_ACTIVE) over a short profiled
# run (bench.py --profile-only --sampling-steps 2: two graph-replayed denoise steps, no VAE decode,
# + one eager profiled step; bench.PMC_STEPS = 3 denoise steps per pass).
# Output: gpurun_out/prof_<tag>/ (stats) and gpurun_out/pmc_<tag>_{fetch,write,mfma}/ (counters).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
B=${B:-1}
FP8=${FP8:-0}
XF=""
SUF=""
if [ "$FP8" = "1" ]; then XF="--fp8"; SUF="_fp8"; fi
TAG=${TAG:-b$B$SUF}
export PYTHONUNBUFFERED=1
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
# the source hash of the library these passes measure (bench.py withholds traffic from a summary of other code)
python -c "from tair_amd import build; print(build.library_hash())" > gpurun_out/prof_$TAG.srchash || exit 1
echo "== stats ($(date +%T))"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --batch $B $XF --no-cpu-baseline --no-profile --no-stage3-probe > gpurun_out/prof_$TAG.log 2>&1 || exit 1
tail -2 gpurun_out/prof_$TAG.log
PROF="python3 bench.py --profile-only --sampling-steps 2 --batch $B $XF"
echo "== pmc fetch ($(date +%T))"
TAIR_PROFILE_CSV=gpurun_out/launches_$TAG.csv timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_${TAG}_fetch \
  -o run --output-format csv -- $PROF > gpurun_out/pmc_${TAG}_fetch.log 2>&1 || exit 1
echo "== pmc write ($(date +%T))"
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_${TAG}_write -o run --output-format csv -- $PROF \
  > gpurun_out/pmc_${TAG}_write.log 2>&1 || exit 1
echo "== pmc mfma ($(date +%T))"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_${TAG}_mfma -o run \
  --output-format csv -- $PROF > gpurun_out/pmc_${TAG}_mfma.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/pmc_summary_$TAG.json gpurun_out/pmc_${TAG}_fetch gpurun_out/pmc_${TAG}_write \
  gpurun_out/pmc_${TAG}_mfma --launches gpurun_out/launches_$TAG.csv --steps 3 > gpurun_out/pmc_summary_$TAG.txt 2>&1
echo "== done ($(date +%T))"
