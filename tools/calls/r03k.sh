export TMPDIR=/tmp; mkdir -p gpurun_out/r03k
timeout -k 10 120 python tools/warm_probe.py bf16 > gpurun_out/r03k/warm_bf16.log 2>&1 || exit 1
timeout -k 10 120 python tools/warm_probe.py x6 > gpurun_out/r03k/warm_x6.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 > gpurun_out/r03k/bench_w5.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 200 > gpurun_out/r03k/bench_w200.json 2>/dev/null || exit 1
