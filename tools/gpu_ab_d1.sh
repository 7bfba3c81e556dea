set -u
O=gpurun_out/ab_d1; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
for v in old new; do
if [ $v = old ]; then export ICLR17_D1_OLD=1; else export ICLR17_D1_OLD=0; fi
timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg --steps 40 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['layers']['deconv1_igdn1']['ms'], d['layers']['deconv2_igdn2']['ms'])" $O/b_${v}_$r.json $v
done; done
