# training step: weight gradients on a side stream (ICLR17_WGRAD_STREAM=1) vs one stream
set -u
O=gpurun_out/ab_train; mkdir -p $O; export TMPDIR=/tmp
ICLR17_WGRAD_STREAM=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_dp_overlap.py -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do
for v in 0 2; do
ICLR17_WGRAD_STREAM=$v timeout -k 10 200 python bench.py --mode train --batch 32 --steps 30 --warmup 5 --no-cpu-baseline > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print("small" if sys.argv[2]=="2" else "one  ", d['value'], d['ms_per_step'])" $O/t_${v}_$r.json $v
done; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "encoder or forward or codec or kodak" > $O/tests_eval.log 2>&1 || { tail -30 $O/tests_eval.log; exit 1; }
tail -1 $O/tests_eval.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d['bf16_mode']; print('bf16', b['value'], {k: v['ms'] for k, v in b['layers'].items()})" $O/bench.json
