# bf16 conv3: ŷ stored through an LDS tile (ICLR17_BF_C3ST=1, default build) vs the accumulator-layout
# stores (build/c3st0): bf16 tests, bit-identity of every layer output, bench A/B, conv3 stamps
set -u
O=gpurun_out/ab_c3st; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_bf16.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
B=64 timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_1.log 2>&1 || { tail $O/sha_1.log; exit 1; }
B=64 ICLR17_LIB=build/c3st0/libiclr17.so timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_0.log 2>&1 || { tail $O/sha_0.log; exit 1; }
if diff <(grep "^{" $O/sha_0.log) <(grep "^{" $O/sha_1.log) > /dev/null; then echo "bf16 layer outputs bit-identical (LDS-tile vs direct conv3 stores)"; else echo "DIFFERENT"; fi
ICLR17_LIB=build/st/libiclr17.so timeout -k 10 120 python tools/k5_stamps.py conv3 > $O/st_conv3.log 2>&1 || { cat $O/st_conv3.log; exit 1; }
grep -v amdgpu.ids $O/st_conv3.log
for r in 1 2 3; do for v in 0 1; do
if [ $v = 0 ]; then L=build/c3st0/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 --steps 40 --warmup 100 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lds-tile' if sys.argv[2] == '1' else 'direct  ', d['value'], d['layers']['conv3_quant_rate']['ms'], d['layers']['deconv2_igdn2']['ms'])" $O/b_${v}_$r.json $v
done; done
