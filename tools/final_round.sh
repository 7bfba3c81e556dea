set -o pipefail
O=gpurun_out/final
P=${P:-r05g}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread > $O/${P}_gpu_tests.log 2>&1 || { echo tests-failed; tail -5 $O/${P}_gpu_tests.log; exit 1; }
tail -2 $O/${P}_gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log | tail -1 > $O/${P}_bench.json
timeout -k 10 300 python bench.py --mode train --batch 32 > $O/bench_train.log 2>&1 || exit 1
grep '^{' $O/bench_train.log | tail -1 > $O/${P}_bench_train.json
timeout -k 10 300 python bench.py --mode kodak > $O/bench_kodak.log 2>&1 || exit 1
grep '^{' $O/bench_kodak.log | tail -1 > $O/${P}_bench_kodak_g9.json
timeout -k 10 300 python bench.py --mode encdec > $O/bench_encdec.log 2>&1 || exit 1
grep '^{' $O/bench_encdec.log | tail -1 > $O/${P}_encdec_h3.json
echo done
