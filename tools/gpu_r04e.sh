set -u
O=gpurun_out/r04e; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "x6k or encoder" -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ONLY=deconv1_old,deconv1_x6k,deconv1_x6k_int timeout -k 10 120 python tools/x6k_time.py > $O/time.log 2>&1 || { cat $O/time.log; exit 1; }
cat $O/time.log
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d['bf16_mode']; print('bf16', b['value'], {k: v['ms'] for k, v in b['layers'].items()})" $O/bench.json
TAG=r04e_train timeout -k 10 900 bash tools/prof_train_pmc.sh > $O/prof_train.log 2>&1 || { tail -20 $O/prof_train.log; exit 1; }
tail -15 $O/prof_train.log
