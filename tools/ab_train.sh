set -u
mkdir -p gpurun_out/abt
for r in 1 2 3; do
  for v in new old; do
    d=.; [ $v = old ] && d=ab_old
    timeout -k 10 300 python $d/bench.py --no-cpu-baseline --mode train --batch 32 --steps 10 --warmup 3 > gpurun_out/abt/$v$r.log 2>&1 || exit 1
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/abt/$v$r.log $v | tee -a gpurun_out/abt/ab.txt
  done
done
