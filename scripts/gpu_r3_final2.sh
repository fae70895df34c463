#!/bin/bash
# Round-3 checkpoint after the batched in-kernel combine: the whole GPU suite, smoke(), the default bench line (driver command), configs[2]
# and configs[4].  Stops at the first GPU failure.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 1000 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/r3_final2_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r3_final2_pytest.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_final2_smoke.log 2>&1 || exit $?
tail -1 gpurun_out/r3_final2_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/r3_final2_bench.log 2>&1 || exit $?
tail -1 gpurun_out/r3_final2_bench.log | cut -c1-250
timeout -k 10 600 python -u bench.py --config 2 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3_final2_cfg2.log 2>&1 || exit $?
tail -1 gpurun_out/r3_final2_cfg2.log | cut -c1-250
timeout -k 10 600 python -u bench.py --config 4 --steps 1 --warmup 1 --no-cpu-baseline --no-profile > gpurun_out/r3_final2_cfg4.log 2>&1 || exit $?
tail -1 gpurun_out/r3_final2_cfg4.log | cut -c1-250
