# Round-4 final-build record, part A: GPU suite (+ parity maxima), default bench, train bench, Kodak (1 rank,
# 2 gloo ranks), encdec x6/bf16, x6 and bf16 trace + PMC profiles, PMC at 8 × 2048², training PMC.
# Everything lands in gpurun_out/r04z*; copy into profiles/ with tools/collect_r04.sh.
set -u
O=gpurun_out/r04z; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
step() { echo "== $(date +%T) $1"; }
step tests
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step bench
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d['bf16_mode']; print('bf16', b['value'], {k: v['ms'] for k, v in b['layers'].items()})" $O/bench.json
step train
timeout -k 10 300 python bench.py --mode train --batch 32 > $O/bench_train.json 2> $O/bench_train.err || { tail $O/bench_train.err; exit 1; }
grep '^{' $O/bench_train.json | tail -1 | cut -c1-400
step kodak
timeout -k 10 200 python bench.py --mode kodak > $O/kodak.json 2> $O/kodak.err || { tail $O/kodak.err; exit 1; }
ICLR17_DIST_BACKEND=gloo timeout -k 10 200 python bench.py --mode kodak --gpus 2 > $O/kodak_2rank.json 2> $O/kodak_2rank.err || { tail $O/kodak_2rank.err; exit 1; }
step encdec
timeout -k 10 200 python bench.py --mode encdec > $O/encdec_x6.json 2> $O/encdec_x6.err || { tail $O/encdec_x6.err; exit 1; }
timeout -k 10 200 python bench.py --mode encdec --precision bf16 > $O/encdec_bf16.json 2> $O/encdec_bf16.err || { tail $O/encdec_bf16.err; exit 1; }
step done
