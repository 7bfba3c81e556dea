"""Summarise tools/pmc.sh output into per-layer HBM traffic per launch → profiles/<tag>_traffic.json.

FETCH_SIZE / WRITE_SIZE are rocprofv3's KB counters, averaged over the dispatches of each kernel.
gfx950 counts half the bytes of wide (16 B/lane) streaming reads in FETCH_SIZE (MI355X_MICROARCH.md
§HBM), so read bytes = 2 × FETCH_SIZE × 1024; write bytes = WRITE_SIZE × 1024.

    python tools/pmc_summary.py gpurun_out/pmc r02_fwd_x6_b64 [x6|fp32]
"""
import csv
import glob
import json
import os
import re
import subprocess
import sys

# bench.py layer name → kernel (B=64 eval at 256², N=192: each name is unique in that run)
LAYER_KERNELS = {
    "fp32": {
        "conv1_gdn1": r"conv1_gdn_kernel<192, 0, false>",
        "conv2_gdn2": r"engine_kernel<192, 192, 192, 1, 4, 0, false, false>",
        "conv3_quant_rate": r"engine_kernel<192, 192, 64, 1, 4, 2, false, false>",
        "deconv1_igdn1": r"engine_kernel<192, 192, 192, 1, 4, 1, false, false>",
        "deconv2_igdn2": r"engine_kernel<192, 192, 192, 1, 4, 1, true, false>",
        "deconv3_clamp": r"engine_kernel<192, 48, 48, 4, 1, 3, false, false>",
    },
    "x6": {
        "conv1_gdn1": r"conv1_x6_kernel<192, 0>",
        "conv2_gdn2": r"engine_kernel<192, 192, 192, 1, 4, 0, false, true>",
        "conv3_quant_rate": r"engine_kernel<192, 192, 96, 2, 2, 2, false, true>",
        "deconv1_igdn1": r"engine_kernel<192, 192, 192, 1, 4, 1, false, true>",
        "deconv2_igdn2": r"engine_kernel_occ2<192, 192, 192, 1, 4, 1, true, true>",
        "deconv3_clamp": r"deconv3_x6_kernel<192>",
    },
}


def norm(name: str) -> str:
    name = re.sub(r"\s+", " ", name)
    name = name.replace("(bool)1", "true").replace("(bool)0", "false")
    return name


def main() -> None:
    src, tag = sys.argv[1], sys.argv[2]
    prec = sys.argv[3] if len(sys.argv) > 3 else "x6"
    per = {}   # kernel → counter → [values]
    for f in sorted(glob.glob(os.path.join(src, "p*", "pmc_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = norm(row["Kernel_Name"])
            per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    kernels = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}
    layers = {}
    for layer, pat in LAYER_KERNELS[prec].items():
        hits = [k for k in kernels if pat in k]
        if len(hits) != 1:
            continue
        c = kernels[hits[0]]
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        rd, wr = 2.0 * c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
        layers[layer] = {"kernel": hits[0], "read_bytes": rd, "write_bytes": wr,
                         "traffic_bytes": rd + wr,
                         **{k: v for k, v in c.items() if k not in ("FETCH_SIZE", "WRITE_SIZE")}}
    try:
        rev = subprocess.check_output(["git", "rev-parse", "--short", "HEAD"], text=True).strip()
    except Exception:  # noqa: BLE001 — no git on the box snapshot
        rev = "unknown"
    out = {"note": "rocprofv3 --pmc, separate passes (tools/pmc.sh) of bench.py; mean per dispatch. "
                   "read_bytes = 2 x FETCH_SIZE (gfx950 half-count of wide reads), write_bytes = WRITE_SIZE.",
           "build": rev, "precision": prec, "layers": layers, "kernels": kernels}
    path = os.path.join("profiles", f"{tag}_traffic.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path, {k: round(v["traffic_bytes"] / 2**20, 1) for k, v in layers.items()}, "MiB/launch")


if __name__ == "__main__":
    main()
