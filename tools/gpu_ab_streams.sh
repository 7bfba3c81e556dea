# bf16 throughput mode: eager vs hipGraph, one stream vs the batch split over two HIP streams
# (layer-interleaved SplitStep); x6 the same with two streams
set -u
O=gpurun_out/ab_streams2; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do for v in e1 e2 g1 g2; do
case $v in e1) A="--bf16-streams 1";; e2) A="--bf16-streams 2";; g1) A="--bf16-streams 1 --graph";; g2) A="--bf16-streams 2 --graph";; esac
timeout -k 10 200 python bench.py --no-cpu-baseline --precision bf16 --steps 40 --warmup 100 $A > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || { tail $O/b_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'bf16', d['value'], d['config']['launch'])" $O/b_${v}_$r.json $v
done; done
for r in 1 2; do for v in g1 g2; do
case $v in g1) A="--streams 1 --graph";; g2) A="--streams 2 --graph";; esac
timeout -k 10 200 python bench.py --no-cpu-baseline --no-bf16-leg --steps 30 --warmup 20 $A > $O/x_${v}_$r.json 2> $O/x_${v}_$r.err || { tail $O/x_${v}_$r.err; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'x6', d['value'], d['config']['launch'])" $O/x_${v}_$r.json $v
done; done
