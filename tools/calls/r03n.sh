export TMPDIR=/tmp; mkdir -p gpurun_out/r03n
for r in 1 2 3; do
  for cm in 0 1; do
    ICLR17_D3_CM=$cm timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg --warmup 30 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cm=$cm', d['value'], {k: v['ms'] for k, v in d['layers'].items()})" >> gpurun_out/r03n/ab.log || exit 1
  done
done
