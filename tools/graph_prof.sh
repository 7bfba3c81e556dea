set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/graphprof
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/g -o t -- python $R/bench.py --no-cpu-baseline --no-bf16-leg --graph --steps 20 --warmup 3 > $O/g.log 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/e -o t -- python $R/bench.py --no-cpu-baseline --no-bf16-leg --steps 20 --warmup 3 > $O/e.log 2>&1 || exit 1
