#!/bin/bash
# Builds compile-time library variants (VARIANTS="name:-DFLAG,-DFLAG2 name2:") on the box and runs
# one command per variant with ICLR17_LIB pointing at it, ROUNDS times, interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/var
for v in $VARIANTS; do
  n=${v%%:*}; f=${v#*:}; f=${f//,/ }; d=/tmp/var_$n; mkdir -p $d
  for s in $(sed -n 's/^SRCS = //p' iclr_17_compression_amd/csrc/Makefile); do
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
      -munsafe-fp-atomics $f -c iclr_17_compression_amd/csrc/$s -o $d/${s%.hip}.o || exit 1
  done
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $d/libiclr17.so $d/*.o || exit 1
done
for r in $(seq ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    n=${v%%:*}
    echo "== $n $r" | tee -a gpurun_out/var/out.txt
    ICLR17_LIB=/tmp/var_$n/libiclr17.so timeout -k 10 300 $CMD 2>&1 | grep -v amdgpu.ids | tee -a gpurun_out/var/out.txt
    [ ${PIPESTATUS[0]} -eq 0 ] || exit 1
  done
done
