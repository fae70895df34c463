#!/bin/bash
# GPU parity tests (or the files given in TESTS) then a short B=1 bench; stops after a crash/timeout.
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
TESTS=${TESTS:-"tests/test_cldm_gpu.py tests/test_golden_gpu.py"}
TAG=${TAG:-r3}
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread $TESTS > gpurun_out/${TAG}_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/${TAG}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
if [ -n "$NO_BENCH" ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/${TAG}_bench.log 2>&1
brc=$?
echo "bench rc=$brc"; tail -1 gpurun_out/${TAG}_bench.log | cut -c1-400
exit $brc
