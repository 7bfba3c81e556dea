# narrow training conv3 (x6 noise, B=32): XCD-contiguous work order (build/xcd1, -DICLR17_C3N_XCD=1) vs dispatch order (default)
set -u
O=gpurun_out/ab_c3xcd; mkdir -p $O; export TMPDIR=/tmp
ICLR17_LIB=build/xcd1/libiclr17.so timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_dp_overlap.py tests/test_gpu_rccl.py -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in xcd0 xcd1; do
if [ $v = xcd1 ]; then L=build/xcd1/libiclr17.so; else L=iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 200 python bench.py --mode train --batch 32 --no-cpu-baseline --steps 30 --warmup 10 > $O/t_${v}_$r.json 2> $O/t_${v}_$r.err || { tail $O/t_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'train B=32 ms', d['ms_per_step'], d['value'])" $O/t_${v}_$r.json $v
done; done
cd /tmp && for v in xcd0 xcd1; do
if [ $v = xcd1 ]; then L=$GRAFT_REPO_ROOT/build/xcd1/libiclr17.so; else L=$GRAFT_REPO_ROOT/iclr_17_compression_amd/libiclr17.so; fi
ICLR17_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_$v -o run -- python $GRAFT_REPO_ROOT/bench.py --mode train --batch 32 --no-cpu-baseline --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$O/prof_$v.log 2>&1 || { tail $GRAFT_REPO_ROOT/$O/prof_$v.log; exit 1; }
done
