export TMPDIR=/tmp; mkdir -p gpurun_out/r03j
R=3 BENCH_ARGS="--precision bf16" timeout -k 10 400 bash tools/ab_libs.sh gpurun_out/r03j/ab_bf16 ab_old/b0.so ab_old/b1_nst5.so || exit 1
timeout -k 10 200 python tools/twostream_eval.py --precision bf16 > gpurun_out/r03j/twostream_bf16.log 2>&1 || exit 1
timeout -k 10 200 python tools/twostream_eval.py --precision x6 > gpurun_out/r03j/twostream_x6.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --size 2048 --batch 8 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/r03j/bench_2048_x6.json 2> gpurun_out/r03j/bench_2048_x6.err || exit 1
timeout -k 10 400 python bench.py --size 2048 --batch 8 --steps 5 --warmup 2 --precision bf16 --no-cpu-baseline > gpurun_out/r03j/bench_2048_bf16.json 2> gpurun_out/r03j/bench_2048_bf16.err || exit 1
NAME=r03j_train timeout -k 10 500 bash tools/prof_train.sh || exit 1
