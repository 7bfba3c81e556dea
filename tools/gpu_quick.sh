#!/bin/bash
# quick GPU iteration: gpu tests (optionally a subset) + eval bench + train bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -x -p no:cacheprovider > gpurun_out/quick_tests.log 2>&1
rc=$?; tail -5 gpurun_out/quick_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit 1; fi
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/quick_tests.log | head -20; }
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/quick_bench.log 2>&1 || exit 1
tail -1 gpurun_out/quick_bench.log
timeout -k 10 300 python bench.py --mode train --batch 32 --steps 10 --warmup 3 > gpurun_out/quick_train.log 2>&1 || exit 1
tail -1 gpurun_out/quick_train.log
