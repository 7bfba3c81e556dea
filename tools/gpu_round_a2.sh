set -u
mkdir -p gpurun_out/ab
VARIANTS="p0 p1" ROUNDS=3 bash tools/gpu_ab2.sh > gpurun_out/ab/pair.txt 2>&1 || { tail -5 gpurun_out/ab/pair.txt; exit 1; }
tail -6 gpurun_out/ab/pair.txt
bash tools/gpu_round_a.sh
