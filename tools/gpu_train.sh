#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 300 python bench.py --mode train --batch 32 --steps 10 --warmup 3 > gpurun_out/bench_train.log 2>&1 || { echo "bench train failed"; tail -30 gpurun_out/bench_train.log; exit 1; }
tail -2 gpurun_out/bench_train.log
timeout -k 10 300 python -m iclr_17_compression_amd.train --synthetic --config tools/configs/smoke_train.json --max-steps 40 > gpurun_out/train_driver.log 2>&1 || { echo "driver failed"; tail -30 gpurun_out/train_driver.log; exit 1; }
tail -5 gpurun_out/train_driver.log
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_train -o run --output-format csv -- python $R/bench.py --mode train --batch 32 --steps 5 --warmup 2 > $R/gpurun_out/prof_train.log 2>&1
echo "prof rc=$?"
