#!/bin/bash
# PMC counters of the halo conv (B=64, 64x64 level, C=320) vs the 128x320 implicit-GEMM tile kernel.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
for v in halo tile; do
  F=""; [ $v = tile ] && F="--force 128x320/1/3"
  [ $v = halo ] && F="--force 256x160/1/9"
  timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/pmcconv_$v -o run --output-format csv -- \
    python3 tools/conv_probe.py --batch 64 --only 64,320,320 --reps 5 $F > gpurun_out/pmcconv_$v.log 2>&1 || exit 1
done
