set -u
O=gpurun_out/ab_fold; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "fold or encoder or forward or codec" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2 3; do for v in 0 1; do
ICLR17_FOLD_BITS=$v timeout -k 10 200 python bench.py --no-cpu-baseline --steps 40 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('fold' if sys.argv[2] == '1' else 'sep ', 'x6', d['value'], 'bf16', d['bf16_mode']['value'], d['layers']['bits_reduce']['ms'], d['bf16_mode']['layers']['bits_reduce']['ms'])" $O/b_${v}_$r.json $v
done; done
