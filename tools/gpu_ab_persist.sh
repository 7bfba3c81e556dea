set -u
O=gpurun_out/ab_persist; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "bf16 or x6k or fold" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B=64 timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_p1.log 2>&1 || { tail $O/sha_p1.log; exit 1; }
B=64 ICLR17_BF_PERSIST=0 timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_p0.log 2>&1 || { tail $O/sha_p0.log; exit 1; }
if diff <(grep "^{" $O/sha_p0.log) <(grep "^{" $O/sha_p1.log) > /dev/null; then echo "bf16 layer outputs bit-identical (persistent vs per-tile deconv)"; else echo "DIFFERENT"; fi
for r in 1 2 3; do for v in 0 1; do
ICLR17_BF_PERSIST=$v timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 --steps 40 --warmup 100 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('persist' if sys.argv[2] == '1' else 'tiles  ', d['value'], d['layers']['deconv2_igdn2']['ms'], d['layers']['deconv2_igdn2']['frac'])" $O/b_${v}_$r.json $v
done; done
