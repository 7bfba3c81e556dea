# k9 x6 weight gradient with the window built in-kernel (default) vs the materialised split
# im2col (build/k9dma): backward tests, bit-identity of dW (tools/k9_sha.py), train A/B
set -u
O=gpurun_out/ab_k9; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_fullsize.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python tools/k9_sha.py > $O/sha_new.log 2>&1 || { tail $O/sha_new.log; exit 1; }
ICLR17_LIB=build/k9dma/libiclr17.so timeout -k 10 120 python tools/k9_sha.py > $O/sha_dma.log 2>&1 || { tail $O/sha_dma.log; exit 1; }
if diff <(grep "^{" $O/sha_dma.log) <(grep "^{" $O/sha_new.log) > /dev/null; then echo "k9 x6 dW bit-identical (in-kernel window vs im2col)"; else echo "DIFFERENT"; cat $O/sha_dma.log $O/sha_new.log; fi
for r in 1 2 3; do for v in dma new; do
if [ $v = dma ]; then L=build/k9dma/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --mode train --batch 32 --no-cpu-baseline --steps 30 --warmup 10 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'train B=32 ms', d['ms_per_step'], d['value'])" $O/t_${v}_$r.json $v
done; done
