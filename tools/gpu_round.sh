set -u
mkdir -p gpurun_out/r02g
O=gpurun_out/r02g
timeout -k 10 200 python -u -m pytest tests/test_gpu_determinism.py -q --timeout 150 --timeout-method thread > $O/det.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --mode train --batch 32 --steps 10 --warmup 3 --cpu-budget 12 > $O/bench_train.json 2> $O/bench_train.err || exit 1
TAG=r02g_x6 PREC=x6 timeout -k 10 600 bash tools/profile_round.sh > $O/prof_x6.log 2>&1 || exit 1
TAG=r02g_bf16 PREC=bf16 timeout -k 10 600 bash tools/profile_round.sh > $O/prof_bf16.log 2>&1 || exit 1
