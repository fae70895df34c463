#!/bin/bash
# HBM traffic + MFMA busy per kernel: one rocprofv3 --pmc pass per counter group (counters cannot be
# split over passes), each over 2 eager sampler steps + one eager profiled step at B=1.
source "$(dirname "$0")/gpu_tests.sh"
TAG=${TAG:-r01}
CMD="python3 bench.py --profile-only --eager --sampling-steps 2 --batch ${PMC_BATCH:-1}"
run pmc_fetch 240 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- $CMD
run pmc_write 240 timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- $CMD
run pmc_mfma 240 timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_mfma -o m -- $CMD
python3 tools/pmc_summary.py gpurun_out/pmc_summary_b${PMC_BATCH:-1}.json gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma > gpurun_out/pmc_summary_b${PMC_BATCH:-1}.txt
head -40 gpurun_out/pmc_summary_b${PMC_BATCH:-1}.txt
rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_mfma
cp gpurun_out/pmc_summary_b${PMC_BATCH:-1}.json profiles/ 2>/dev/null
run bench 600 python bench.py --steps 3 --warmup 1 --no-cpu-baseline
