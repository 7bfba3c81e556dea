# multi-rank rehearsal on the box's one GPU: bench.py --gpus 2 starts its own 2 ranks (gloo)
set -u
O=gpurun_out/${TAG:-r03q}
mkdir -p $O
export ICLR17_DIST_BACKEND=gloo
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_2rank_gloo_1gpu.json 2> $O/bench_2rank.err || { tail -5 $O/bench_2rank.err; exit 1; }
timeout -k 10 300 python bench.py --gpus 2 --mode train --batch 16 --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_train_2rank_gloo_1gpu.json 2> $O/bench_train_2rank.err || { tail -5 $O/bench_train_2rank.err; exit 1; }
for f in bench_2rank_gloo_1gpu bench_train_2rank_gloo_1gpu; do python -c "import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['n_gpus'], d['value'], d.get('rank_devices'), d.get('dist_backend'), d['config'].get('parallelism'))"; done
