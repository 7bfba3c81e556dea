# Round-4 final-build record, part B (profiles): GPU suite (+ parity maxima), default bench, train bench, Kodak (1 rank,
# 2 gloo ranks), encdec x6/bf16, x6 and bf16 trace + PMC profiles, PMC at 8 × 2048², training PMC.
# Everything lands in gpurun_out/r04z*; copy into profiles/ with tools/collect_r04.sh.
set -u
O=gpurun_out/r04z; mkdir -p $O; export TMPDIR=/tmp
export ICLR17_PARITY_OUT=$O
step() { echo "== $(date +%T) $1"; }
step prof_x6
TAG=r04_x6 PREC=x6 timeout -k 10 900 bash tools/profile_round.sh > $O/prof_x6.log 2>&1 || { tail -20 $O/prof_x6.log; exit 1; }
step prof_bf16
TAG=r04_bf16 PREC=bf16 timeout -k 10 900 bash tools/profile_round.sh > $O/prof_bf16.log 2>&1 || { tail -20 $O/prof_bf16.log; exit 1; }
step prof_2048
TAG=r04_2048_x6 PREC=x6 PMC_NSB="192 2048 8" BENCH_ARGS="--size 2048 --batch 8" timeout -k 10 900 bash tools/profile_round.sh > $O/prof_2048_x6.log 2>&1 || { tail -20 $O/prof_2048_x6.log; exit 1; }
TAG=r04_2048_bf16 PREC=bf16 PMC_NSB="192 2048 8" BENCH_ARGS="--size 2048 --batch 8" timeout -k 10 900 bash tools/profile_round.sh > $O/prof_2048_bf16.log 2>&1 || { tail -20 $O/prof_2048_bf16.log; exit 1; }
step bench_2048
timeout -k 10 300 python bench.py --size 2048 --batch 8 > $O/bench_2048.json 2> $O/bench_2048.err || { tail $O/bench_2048.err; exit 1; }
step prof_train
TAG=r04_train timeout -k 10 900 bash tools/prof_train_pmc.sh > $O/prof_train.log 2>&1 || { tail -20 $O/prof_train.log; exit 1; }
step done
