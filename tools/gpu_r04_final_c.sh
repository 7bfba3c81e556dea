# round-4 final build: the default bench line (PMC traffic of this build picked up) and C3 at B=32
set -u
O=gpurun_out/r04z; mkdir -p $O; export TMPDIR=/tmp
# this build's PMC summaries (part B, if it ran in this call) where bench.py looks for them
for t in r04_x6 r04_bf16 r04_2048_x6 r04_2048_bf16; do
  [ -f gpurun_out/$t/${t}_traffic.json ] && cp gpurun_out/$t/${t}_traffic.json profiles/
done
timeout -k 10 300 python bench.py > $O/bench_final.json 2> $O/bench_final.err || { tail $O/bench_final.err; exit 1; }
timeout -k 10 300 python bench.py --mode train --batch 32 > $O/bench_train32.json 2> $O/bench_train32.err || { tail $O/bench_train32.err; exit 1; }
timeout -k 10 300 python bench.py --size 2048 --batch 8 > $O/bench_2048_final.json 2> $O/bench_2048_final.err || { tail $O/bench_2048_final.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open("gpurun_out/r04z/bench_final.json").read().strip().splitlines()[-1])
r=d["roofline"]; b=d["bf16_mode"]["roofline"]
print("x6", d["value"], r["frac"], r.get("frac_from_profile"), r.get("traffic"), r.get("traffic_source"))
print("bf16", d["bf16_mode"]["value"], b["frac"], b.get("frac_from_profile"), b.get("traffic"))
t=json.loads(open("gpurun_out/r04z/bench_train32.json").read().strip().splitlines()[-1])
print("train32", t["value"], t["ms_per_step"], t["roofline"]["frac"])
PY
