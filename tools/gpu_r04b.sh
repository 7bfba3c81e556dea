# x6k engine: parity test, then eval bench A/B (16x16x32 x6 engine vs x6k) on one box
set -u
O=gpurun_out/r04b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "x6k" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/x6k_tests.log 2>&1 || { tail -40 $O/x6k_tests.log; exit 1; }
tail -3 $O/x6k_tests.log
for r in 1 2; do
ICLR17_X6K=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg > $O/bench_old_$r.json 2> $O/bench_old_$r.err || { tail $O/bench_old_$r.err; exit 1; }
ICLR17_X6K=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg > $O/bench_new_$r.json 2> $O/bench_new_$r.err || { tail $O/bench_new_$r.err; exit 1; }
for v in old new; do python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], {k: v['ms'] for k, v in d['layers'].items()})" $O/bench_${v}_$r.json $v; done
done
