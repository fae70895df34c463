export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -f gpurun_out/parity.jsonl
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_kernels_gpu.py tests/test_vae_gpu.py tests/test_cldm_gpu.py tests/test_golden_gpu.py > gpurun_out/r3e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3e_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python3 tools/gemm_probe.py --batch 16 --reps 10 --tiles "0x0,e2:0x0" > gpurun_out/r3e_probe_b16.log 2>&1 || exit $?
timeout -k 10 200 python3 tools/gemm_probe.py --batch 1 --reps 10 --tiles "0x0,e2:0x0" > gpurun_out/r3e_probe_b1.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-stage3-probe > gpurun_out/r3e_bench_b1.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --batch 16 --tiles 64 --no-cpu-baseline --no-profile > gpurun_out/r3e_bench_b16.log 2>&1 || exit $?
echo done
