#!/bin/bash
# Round-3 profiling pass (B=1 and batched GEMM evidence); each GPU step under its own time limit,
# stopping at the first crash / timeout.
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() { echo "== $1 ($(date +%T))"; }
ok() { local rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop: rc=$rc"; exit $rc; fi; }
step tests
timeout -k 10 400 python -u -m pytest -v --timeout 300 --timeout-method thread \
  "tests/test_cldm_gpu.py::test_custom_op_registered" "tests/test_cldm_gpu.py::test_sample_cfg_vs_oracle" \
  > gpurun_out/r3p_tests.log 2>&1; ok $?; tail -2 gpurun_out/r3p_tests.log
step bench
TAIR_PROFILE_CSV=gpurun_out/r3p_b1_launches.csv timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 \
  --no-cpu-baseline > gpurun_out/r3p_bench_b1.log 2>&1; ok $?; tail -1 gpurun_out/r3p_bench_b1.log | cut -c1-300
step trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3p_trace -o run --output-format csv -- \
  python3 bench.py --steps 1 --warmup 1 --sampling-steps 12 --no-profile --no-cpu-baseline --no-stage3-probe \
  > gpurun_out/r3p_trace.log 2>&1; ok $?
f=$(ls gpurun_out/r3p_trace/*/*kernel_trace.csv 2>/dev/null | head -1)
[ -n "$f" ] && python3 tools/trace_step.py "$f" step_update gpurun_out/r3p_step_timeline.txt > gpurun_out/r3p_step.txt 2>&1
cat gpurun_out/r3p_step.txt | head -20
step probe16
timeout -k 10 300 python3 tools/gemm_probe.py --batch 16 --reps 10 --tiles "0x0,e1:0x0,e2:0x0" \
  > gpurun_out/r3p_probe_b16.log 2>&1; ok $?
step probe1
timeout -k 10 300 python3 tools/gemm_probe.py --batch 1 --reps 10 --tiles "0x0,e1:0x0,e2:0x0" \
  > gpurun_out/r3p_probe_b1.log 2>&1; ok $?
step done
