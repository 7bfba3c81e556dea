#!/bin/bash
# A/B compile-time variants of engine_bf16.hip on one box.
#   build (here, CPU):  VARIANTS="name:-DFLAG name2:" tools/bf16_ab.sh build
#   run (GPU box):      VARIANTS="name name2" ROUNDS=3 tools/bf16_ab.sh run
# Variants relink libiclr17.so with the shipped objects of the other sources into
# build/ab_<name>/ (git-ignored, travels with the snapshot); tools/bf16_time.py times them
# interleaved.
set -u
C=iclr_17_compression_amd/csrc
if [ "${1:-}" = build ]; then
  for v in $VARIANTS; do
    n=${v%%:*}; f=${v#*:}; f=${f//,/ }; d=build/ab_$n; mkdir -p $d
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -munsafe-fp-atomics $f -c $C/engine_bf16.hip -o $d/engine_bf16.o || exit 1
    objs=$(ls $C/*.o | grep -v engine_bf16.o)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libiclr17.so $objs $d/engine_bf16.o || exit 1
    rm -f $d/engine_bf16.o
  done
  exit 0
fi
mkdir -p gpurun_out/ab
for r in $(seq ${ROUNDS:-2}); do
  for n in $VARIANTS; do
    n=${n%%:*}
    ICLR17_LIB=build/ab_$n/libiclr17.so timeout -k 10 120 python tools/bf16_time.py --tag $n \
      2>/dev/null | tee -a gpurun_out/ab/${AB_OUT:-bf16_ab}.txt
    [ ${PIPESTATUS[0]} -eq 0 ] || { echo "variant $n failed" | tee -a gpurun_out/ab/${AB_OUT:-bf16_ab}.txt; exit 1; }
  done
done
