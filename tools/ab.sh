#!/bin/bash
# A/B two compile-time variants of the library on one box: VARIANTS="name:-DFLAG name2:" ; times
# each with tools/time_layers.py, interleaved ROUNDS times.
set -u
mkdir -p gpurun_out/ab
for v in $VARIANTS; do
  n=${v%%:*}; f=${v#*:}; f=${f//,/ }; d=/tmp/ab_$n; mkdir -p $d
  for s in $(sed -n 's/^SRCS = //p' iclr_17_compression_amd/csrc/Makefile); do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -munsafe-fp-atomics $f -c iclr_17_compression_amd/csrc/$s -o $d/${s%.hip}.o || exit 1
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libiclr17.so $d/*.o || exit 1
done
for r in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    n=${v%%:*}
    TAG=$n X6_TIME_ONLY=1 ICLR17_LIB=/tmp/ab_$n/libiclr17.so timeout -k 10 120 python ${TOOL:-tools/time_layers.py} --tag $n 2>/dev/null \
      | tee -a gpurun_out/ab/results.txt
    [ ${PIPESTATUS[0]} -eq 0 ] || { echo "variant $n failed" | tee -a gpurun_out/ab/results.txt; exit 1; }
  done
done
