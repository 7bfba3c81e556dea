# round-4 checkpoint: the full GPU suite, the default bench, Kodak (1 rank and 2 gloo ranks), encdec
set -u
O=gpurun_out/r04d; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d['bf16_mode']; print('bf16', b['value'], {k: v['ms'] for k, v in b['layers'].items()})" $O/bench.json
timeout -k 10 200 python bench.py --mode kodak > $O/kodak.json 2> $O/kodak.err || { tail $O/kodak.err; exit 1; }
ICLR17_DIST_BACKEND=gloo timeout -k 10 200 python bench.py --mode kodak --gpus 2 > $O/kodak_2rank.json 2> $O/kodak_2rank.err || { tail $O/kodak_2rank.err; exit 1; }
timeout -k 10 200 python bench.py --mode encdec > $O/encdec_x6.json 2> $O/encdec_x6.err || { tail $O/encdec_x6.err; exit 1; }
timeout -k 10 200 python bench.py --mode encdec --precision bf16 > $O/encdec_bf16.json 2> $O/encdec_bf16.err || { tail $O/encdec_bf16.err; exit 1; }
for f in kodak kodak_2rank encdec_x6 encdec_bf16; do grep '^{' $O/$f.json | tail -1 | cut -c1-700; done
for B in 128 256; do
timeout -k 10 300 python bench.py --no-cpu-baseline --batch $B > $O/bench_b$B.json 2> $O/bench_b$B.err || { tail $O/bench_b$B.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('B', sys.argv[2], 'x6', d['value'], 'bf16', d['bf16_mode']['value'], {k: v['ms'] for k, v in d['bf16_mode']['layers'].items()})" $O/bench_b$B.json $B
done
