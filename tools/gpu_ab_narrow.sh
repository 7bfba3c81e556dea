# training conv3 (noise, x6) on 48-column tiles at B=32 (default) vs 96-column tiles (build/nonarrow)
set -u
O=gpurun_out/ab_narrow; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dp_overlap.py tests/test_gpu_rccl.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in wide narrow; do
if [ $v = wide ]; then L=build/nonarrow/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --mode train --batch 32 --no-cpu-baseline --steps 30 --warmup 10 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'train B=32 ms', d['ms_per_step'], d['value'])" $O/t_${v}_$r.json $v
done; done
