#!/bin/bash
# Diagnostic: build ablation variants of the library (-DICLR17_ABL=mask) and time conv2+GDN
# and deconv2+IGDN (+conv1+GDN1) with each (separate processes). Runs on the GPU box.
set -u
R=$(pwd)
mkdir -p gpurun_out/abl
for m in ${MASKS:-0 8 16 32 48}; do
  d=/tmp/abl$m; mkdir -p $d
  for f in $(sed -n 's/^SRCS = //p' iclr_17_compression_amd/csrc/Makefile); do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -DICLR17_ABL=$m \
      -munsafe-fp-atomics -c iclr_17_compression_amd/csrc/$f -o $d/${f%.hip}.o || exit 1
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libiclr17.so $d/*.o || exit 1
  ICLR17_LIB=$d/libiclr17.so timeout -k 10 120 python tools/time_layers.py --tag abl$m >> gpurun_out/abl/results.txt 2>&1 || exit 1
done
cat gpurun_out/abl/results.txt
