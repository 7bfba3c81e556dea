#!/bin/bash
# Copy the round-4 final-build record (tools/gpu_r04_final_{a,b}.sh outputs) into profiles/.
set -u
S=gpurun_out/r04z; P=profiles
j() { grep '^{' "$1" | tail -1 > "$2"; }
j $S/bench_final.json $P/r04_bench.json
j $S/bench_train32.json $P/r04_bench_train.json
j $S/bench_train.json $P/r04_bench_train_b64.json
j $S/kodak.json $P/r04_bench_kodak_g9.json
j $S/kodak_2rank.json $P/r04_bench_kodak_g9_2rank_gloo_1gpu.json
j $S/encdec_x6.json $P/r04_encdec_x6.json
j $S/encdec_bf16.json $P/r04_encdec_bf16.json
[ -f $S/bench_2048_final.json ] && j $S/bench_2048_final.json $P/r04_bench_2048.json
for f in $S/parity_*.json; do cp "$f" $P/r04_$(basename "$f"); done
tail -3 $S/gpu_tests.log > $P/r04_gpu_tests.log
for t in r04_x6 r04_bf16 r04_2048_x6 r04_2048_bf16; do
  [ -d gpurun_out/$t ] || continue
  cp gpurun_out/$t/${t}_traffic.json gpurun_out/$t/${t}_kernel_stats.csv gpurun_out/$t/${t}_bench_under_trace.json $P/
done
if [ -d gpurun_out/r04_train ]; then
  cp gpurun_out/r04_train/r04_train_train_kernels.json $P/
  cp "$(find gpurun_out/r04_train/trace -name '*kernel_stats.csv' | head -1)" $P/r04_train_b32_kernel_stats.csv
  [ -s gpurun_out/r04_train/r04_train_bench_under_trace.json ] && cp gpurun_out/r04_train/r04_train_bench_under_trace.json $P/
fi
ls -la $P | grep r04_
