set -u
O=gpurun_out/r04f; mkdir -p $O; export TMPDIR=/tmp
TAG=r04f_bf16 PREC=bf16 timeout -k 10 900 bash tools/profile_round.sh > $O/prof_bf16.log 2>&1 || { tail -20 $O/prof_bf16.log; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/r04f_bf16/r04f_bf16_traffic.json"))
for k,v in d["layers"].items(): print(k, {kk: v.get(kk) for kk in ("mean_ms","frac","traffic_bytes","mfma_busy") if kk in v})
PY
