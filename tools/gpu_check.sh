# GPU suite + bit-identity SHAs of the default library against build/ab_head (if present) + bench
set -u
mkdir -p gpurun_out/chk
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/chk/tests.log 2>&1
rc=$?; tail -3 gpurun_out/chk/tests.log; [ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/chk/tests.log | head -20; exit 1; }
timeout -k 10 120 python tools/bf16_layer_sha.py 2>/dev/null | tail -1 | sed 's/^/lib  /'
[ -d build/ab_head ] && { ICLR17_LIB=build/ab_head/libiclr17.so timeout -k 10 120 python tools/bf16_layer_sha.py 2>/dev/null | tail -1 | sed 's/^/head /'; }
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > gpurun_out/chk/bench.json 2> gpurun_out/chk/bench.err || { tail -5 gpurun_out/chk/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/chk/bench.json')); print('x6', d['value'], {k: v['ms'] for k, v in d['layers'].items()}); b=d.get('bf16_mode') or {}; print('bf16', b.get('value'), {k: v['ms'] for k, v in b.get('layers', {}).items()})"
