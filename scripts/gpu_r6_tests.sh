#!/bin/bash
# Round 6: run the given GPU test files / ids (TESTS, all failures reported: no -x), then optional bench lines.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
python -c "from tair_amd import _lib; _lib.lib()" || exit 1
timeout -k 10 ${LIM:-900} python -u -m pytest ${TESTS} ${K:+-k "$K"} -v -m gpu --timeout 600 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/${NAME:-r6_tests}.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/${NAME:-r6_tests}.log | tail -60
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for b in ${BENCH-}; do
  timeout -k 10 600 python -u bench.py --steps ${STEPS:-3} --warmup 1 --batch $b ${BENCH_FLAGS-} > gpurun_out/${NAME:-r6}_bench_b$b.log 2>&1 || exit 1
  tail -2 gpurun_out/${NAME:-r6}_bench_b$b.log
done
