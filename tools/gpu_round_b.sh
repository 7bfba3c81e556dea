# Round-end record, part B: x6 and bf16 kernel-trace + PMC profiles of the default bench
set -u
TAG=${TAG:?TAG}
O=gpurun_out/$TAG
mkdir -p $O
TAG=${TAG}_x6 PREC=x6 timeout -k 10 500 bash tools/profile_round.sh > $O/prof_x6.log 2>&1 || { tail -5 $O/prof_x6.log; exit 1; }
TAG=${TAG}_bf16 PREC=bf16 timeout -k 10 500 bash tools/profile_round.sh > $O/prof_bf16.log 2>&1 || { tail -5 $O/prof_bf16.log; exit 1; }
ls gpurun_out/${TAG}_x6 gpurun_out/${TAG}_bf16
