# conv3 quantiser epilogues with the element_bits fallback out of the lookup stream, the XCD-aware
# column-block map (default build; build/noxcd without the map) vs HEAD (build/head): GPU suite, bf16 layer bit-identity, x6/bf16 bench A/B, conv3 stamps
set -u
O=gpurun_out/ab_rtab; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
timeout -k 10 700 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
B=64 timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_new.log 2>&1 || { tail $O/sha_new.log; exit 1; }
B=64 ICLR17_LIB=build/head/libiclr17.so timeout -k 10 200 python tools/bf16_layer_sha.py > $O/sha_head.log 2>&1 || { tail $O/sha_head.log; exit 1; }
if diff <(grep "^{" $O/sha_head.log) <(grep "^{" $O/sha_new.log) > /dev/null; then echo "bf16 layer outputs bit-identical (new vs HEAD)"; else echo "DIFFERENT"; fi
ICLR17_LIB=build/st/libiclr17.so timeout -k 10 120 python tools/k5_stamps.py conv3 > $O/st_conv3.log 2>&1 || { cat $O/st_conv3.log; exit 1; }
grep -v amdgpu.ids $O/st_conv3.log | head -7
for r in 1 2 3; do for v in head noxcd new; do
if [ $v = head ]; then L=build/head/libiclr17.so; elif [ $v = noxcd ]; then L=build/noxcd/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 20 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); b=d['bf16_mode']; print(sys.argv[2], 'x6', d['value'], d['layers']['conv3_quant_rate']['ms'], 'bf16', b['value'], b['layers']['conv3_quant_rate']['ms'])" $O/b_${v}_$r.json $v
done; done
for r in 1 2; do for v in head new; do
if [ $v = head ]; then L=build/head/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --mode train --no-cpu-baseline --steps 30 --warmup 10 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'train ms', d['ms_per_step'], d['value'])" $O/t_${v}_$r.json $v
done; done
timeout -k 10 300 python tools/streams_eval.py --steps 40 --rounds 3 > $O/streams.log 2>&1 || { tail $O/streams.log; exit 1; }
grep -v amdgpu.ids $O/streams.log
for r in 1 2; do for v in 1 2; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 --warmup 20 --streams $v --bf16-streams $v > $O/s_${v}_$r.json 2> $O/s_${v}_$r.err || { tail $O/s_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('streams', sys.argv[2], 'x6', d['value'], 'bf16', d['bf16_mode']['value'])" $O/s_${v}_$r.json $v
done; done
