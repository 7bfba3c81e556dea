# round-4 final build, all in one call: part A (suite, benches, Kodak, encdec), part B (profiles),
# part C (the default bench line with this build's PMC traffic, C3 at B=32)
set -u
bash tools/gpu_r04_final_a.sh && bash tools/gpu_r04_final_b.sh && bash tools/gpu_r04_final_c.sh
