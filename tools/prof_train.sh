#!/bin/bash
# rocprofv3 kernel stats of the train bench (B=32), summarised per step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/prof
export TMPDIR=/tmp
cd /tmp
rm -rf $R/gpurun_out/prof/${NAME:-train}
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof/${NAME:-train} -o run --output-format csv -- \
  python $R/bench.py --no-cpu-baseline --mode ${MODE:-train} --batch ${BATCH:-32} --steps 5 --warmup 2 > $R/gpurun_out/prof/${NAME:-train}.log 2>&1
