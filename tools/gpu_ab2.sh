# bf16 A/B: bit-identity SHAs per variant, then interleaved layer timings
set -u
mkdir -p gpurun_out/ab
export TMPDIR=/tmp
for n in $VARIANTS; do
  ICLR17_LIB=build/ab_$n/libiclr17.so timeout -k 10 120 python tools/bf16_layer_sha.py > gpurun_out/ab/sha_$n.txt 2>&1 || { tail -5 gpurun_out/ab/sha_$n.txt; exit 1; }
  echo "$n $(tail -1 gpurun_out/ab/sha_$n.txt)"
done
ROUNDS=${ROUNDS:-3} AB_OUT=${AB_OUT:-r2} bash tools/bf16_ab.sh run > /dev/null || exit 1
cat gpurun_out/ab/${AB_OUT:-r2}.txt
