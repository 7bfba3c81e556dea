# training conv3 (x6 noise, B=32, 48-column tiles): pre-split weights (ICLR17_TRAIN_W6=1, default) vs the per-k-step split (=0)
set -u
O=gpurun_out/ab_w6n; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dp_overlap.py tests/test_gpu_rccl.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in 0 1; do
ICLR17_TRAIN_W6=$v timeout -k 10 200 python bench.py --mode train --batch 32 --no-cpu-baseline --steps 30 --warmup 10 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('TRAIN_W6='+sys.argv[2], 'train B=32 ms', d['ms_per_step'], d['value'])" $O/t_${v}_$r.json $v
done; done
cd /tmp && for v in 0 1; do
ICLR17_TRAIN_W6=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run -- python $GRAFT_REPO_ROOT/bench.py --mode train --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof_$v.log; exit 1; }
done
