export TMPDIR=/tmp; mkdir -p gpurun_out/r03l
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_determinism.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03l/tests.log 2>&1 || exit 1
R=3 BENCH_ARGS="--precision bf16 --warmup 100" timeout -k 10 400 bash tools/ab_libs.sh gpurun_out/r03l/ab ab_old/b0.so ab_old/b2_c1persist.so || exit 1
