# Round-end record, part A (run from the repo root on the box): GPU suite, determinism, the
# default bench, the B=32 train bench, Kodak-G9 and the 2048² benches, under gpurun_out/$TAG.
set -u
TAG=${TAG:?TAG}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -20 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_determinism.py -q --timeout 150 --timeout-method thread > $O/det.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python bench.py --mode train --batch 32 --steps 20 --warmup 5 --cpu-budget 12 > $O/bench_train.json 2> $O/bench_train.err || exit 1
timeout -k 10 300 python bench.py --mode kodak > $O/bench_kodak.json 2> $O/bench_kodak.err || exit 1
timeout -k 10 300 python bench.py --size 2048 --batch 8 --no-cpu-baseline --no-bf16-leg > $O/bench_2048_x6.json 2> $O/bench_2048_x6.err || exit 1
timeout -k 10 300 python bench.py --size 2048 --batch 8 --no-cpu-baseline --no-bf16-leg --precision bf16 > $O/bench_2048_bf16.json 2> $O/bench_2048_bf16.err || exit 1
for f in bench bench_train bench_kodak bench_2048_x6 bench_2048_bf16; do python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['unit'], d.get('ms_per_step'))"; done
