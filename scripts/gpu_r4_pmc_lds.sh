#!/bin/bash
# LDS-side PMC counters of the halo conv (B=64, 64x64 level, C=320): command / data FIFO full, LDS waits.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C1 -d gpurun_out/pmclds_halo -o run --output-format csv -- \
  python3 tools/conv_probe.py --batch 64 --only 64,320,320 --reps 5 --force 256x160/1/9 > gpurun_out/pmclds_halo.log 2>&1 || exit 1
# pass 2: where the issue cycles go (one counter set per run)
C2="SQ_WAVE_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_WAIT_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C2 -d gpurun_out/pmcissue_halo -o run --output-format csv -- \
  python3 tools/conv_probe.py --batch 64 --only 64,320,320 --reps 5 --force 256x160/1/9 > gpurun_out/pmcissue_halo.log 2>&1 || exit 1
find gpurun_out/pmclds_halo gpurun_out/pmcissue_halo -name "*.csv" | head
