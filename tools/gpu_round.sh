# Round-end GPU record (run from the repo root on the box): determinism, the default bench, the
# B=32 train bench, and the x6 / bf16 kernel-trace + PMC profiles, all under gpurun_out/$TAG.
set -u
TAG=${TAG:?TAG}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_determinism.py -q --timeout 150 --timeout-method thread > $O/det.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --mode train --batch 32 --steps 20 --warmup 5 --cpu-budget 12 > $O/bench_train.json 2> $O/bench_train.err || exit 1
timeout -k 10 300 python bench.py --mode kodak > $O/bench_kodak.json 2> $O/bench_kodak.err || exit 1
TAG=${TAG}_x6 PREC=x6 timeout -k 10 600 bash tools/profile_round.sh > $O/prof_x6.log 2>&1 || exit 1
TAG=${TAG}_bf16 PREC=bf16 timeout -k 10 600 bash tools/profile_round.sh > $O/prof_bf16.log 2>&1 || exit 1
