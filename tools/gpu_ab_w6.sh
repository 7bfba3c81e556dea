# x6 conv3 with pre-split weights (default, ICLR17_W6=1) vs split in the loop (ICLR17_W6=0):
# GPU parity suite (operating points, encoder/codec identity), bit-identity, bench A/B
set -u
O=gpurun_out/ab_w6; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 120 python tools/w6_sha.py > $O/sha.log 2>&1 || { tail $O/sha.log; exit 1; }
cat $O/sha.log | grep -v amdgpu
for r in 1 2 3; do for v in 0 1; do
ICLR17_W6=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg --steps 40 --warmup 20 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('W6', sys.argv[2], 'x6', d['value'], 'conv3', d['layers']['conv3_quant_rate']['ms'])" $O/b_${v}_$r.json $v
done; done
