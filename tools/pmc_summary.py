"""Summarise a tools/profile_round.sh output directory into <dir>/<tag>_traffic.json: per
bench.py layer, the kernel that ran it, its mean duration from the kernel trace and its HBM
traffic per launch from the PMC passes, stamped with the SHA-256 of the library that ran.

FETCH_SIZE / WRITE_SIZE are rocprofv3's KB counters, averaged over the dispatches of each layer.
gfx950 counts half the bytes of wide (16 B/lane) streaming reads in FETCH_SIZE (MI355X_MICROARCH.md
§HBM), so read bytes = 2 × FETCH_SIZE × 1024; write bytes = WRITE_SIZE × 1024.

Layers are told apart by kernel name and, where two layers run the same instantiation (the x6
and fp32 deconv1 / deconv2, one engine_kernel each), by grid size: deconv1 runs on the 16×16
latent grid, deconv2 on the 32×32 one, so deconv1 is the smaller of the two grids.

    python tools/pmc_summary.py gpurun_out/<tag> <tag> <precision> [N S B]
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# bench.py layer → (kernel-name pattern, grid rank among that name's distinct grid sizes or None)
# engine_kernel names are matched as prefixes: the trailing template arguments (the W6 flag)
# differ by instantiation
LAYER_KERNELS = {
    "fp32": {
        "conv1_gdn1": (r"conv1_gdn_kernel<192, 0, false>", None),
        "conv2_gdn2": (r"engine_kernel<192, 192, 192, 1, 4, 0, false", None),
        "conv3_quant_rate": (r"engine_kernel<192, 192, 96, 2, 2, 2, false", None),
        "deconv1_igdn1": (r"engine_kernel<192, 192, 192, 1, 4, 1, false", 0),
        "deconv2_igdn2": (r"engine_kernel<192, 192, 192, 1, 4, 1, false", 1),
        "deconv3_clamp": (r"engine_kernel<192, 48, 48, 4, 1, 3, false", None),
    },
    "x6": {
        "conv1_gdn1": (r"conv1_x6_kernel<192, 0>", None),
        "conv2_gdn2": (r"engine_kernel<192, 192, 192, 1, 4, 0, true", None),
        "conv3_quant_rate": (r"engine_kernel<192, 192, 96, 2, 2, 2, true", None),   # also the W6 form
        "deconv1_igdn1": (r"engine_kernel<192, 192, 192, 1, 4, 1, true", 0),
        "deconv2_igdn2": (r"engine_kernel<192, 192, 192, 1, 4, 1, true", 1),
        "deconv3_clamp": (r"deconv3_x6_kernel<192>", None),
    },
    "h3": {   # h3k_kernel<MODE, TH, CO, CI, EPI, INT_OK, COT, SEP, ICM>
        "conv1_gdn1": (r"h3k_kernel<3, 16, 192, 3, 0, false, 192, false, 0>", None),
        "conv2_gdn2": (r"h3k_kernel<2, 16, 192, 192, 0, false, 192, false, 8>", None),
        "conv3_quant_rate": (r"h3k_kernel<2, 8, 192, 192, 2, false, 64, true, 8>", None),
        "deconv1_igdn1": (r"h3k_kernel<1, 16, 192, 192, 1, true, 192, false, 16>", None),
        "deconv2_igdn2": (r"h3k_kernel<1, 16, 192, 192, 1, false, 192, false, 16>", None),
        "deconv3_clamp": (r"deconv3_x6_kernel<192, true>", None),
    },
    "bf16": {
        "conv1_gdn1": (r"conv1p_bf16_kernel<192, true>", None),
        "conv2_gdn2": (r"k5_bf16_kernel<0, 16, 192, 192, 192, 0>", None),
        "conv3_quant_rate": (r"k5_bf16_kernel<0, 8, 96, 192, 192, 2>", None),
        "deconv1_igdn1": (r"k5_bf16_kernel<1, ", 0),   # 8-row tiles at 256², 16-row at 2048²
        "deconv2_igdn2": (r"k5_bf16_kernel<1, ", 1),
        "deconv3_clamp": (r"deconv3_bf16_kernel<192>", None),
    },
}


def norm(name: str) -> str:
    name = re.sub(r"\s+", " ", name)
    return name.replace("(bool)1", "true").replace("(bool)0", "false")


def lib_sha(path=None) -> str:
    path = path or os.environ.get("ICLR17_LIB",
                                  os.path.join(REPO, "iclr_17_compression_amd", "libiclr17.so"))
    return hashlib.sha256(open(path, "rb").read()).hexdigest()[:16]


def assign(rows, prec):
    """rows: dicts with name, grid → {layer: [row, ...]} by LAYER_KERNELS."""
    out = {}
    for layer, (pat, rank) in LAYER_KERNELS[prec].items():
        hits = [r for r in rows if pat in r["name"]]
        if rank is not None:
            grids = sorted({r["grid"] for r in hits})
            if len(grids) < 2:
                continue
            hits = [r for r in hits if r["grid"] == grids[rank]]
        if hits and len({r["name"] for r in hits}) == 1:
            out[layer] = hits
    return out


def main() -> None:
    src, tag, prec = sys.argv[1], sys.argv[2], sys.argv[3]
    N, S, B = (int(v) for v in sys.argv[4:7]) if len(sys.argv) >= 7 else (192, 256, 64)
    # PMC: one row per (dispatch, counter)
    disp = {}
    for f in sorted(glob.glob(os.path.join(src, "p*", "pmc_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            key = (f, row["Dispatch_Id"])
            d = disp.setdefault(key, {"name": norm(row["Kernel_Name"]), "grid": int(row["Grid_Size"]),
                                      "c": {}})
            d["c"][row["Counter_Name"]] = float(row["Counter_Value"])
    pmc = assign(list(disp.values()), prec)
    # kernel trace: one row per dispatch
    trace = []
    for f in glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            grid = (int(row["Grid_Size"]) if "Grid_Size" in row else
                    int(row["Grid_Size_X"]) * int(row["Grid_Size_Y"]) * int(row["Grid_Size_Z"]))
            trace.append({"name": norm(row["Kernel_Name"]), "grid": grid,
                          "ns": int(row["End_Timestamp"]) - int(row["Start_Timestamp"])})
    tr = assign(trace, prec)
    layers = {}
    for layer in LAYER_KERNELS[prec]:
        e = {}
        if layer in tr:
            ns = sorted(r["ns"] for r in tr[layer])
            e.update(kernel=tr[layer][0]["name"], grid=tr[layer][0]["grid"], dispatches=len(ns),
                     mean_ms=sum(ns) / len(ns) / 1e6, median_ms=ns[len(ns) // 2] / 1e6)
        if layer in pmc:
            cs = {}
            for r in pmc[layer]:
                for c, v in r["c"].items():
                    cs.setdefault(c, []).append(v)
            c = {k: sum(v) / len(v) for k, v in cs.items()}
            e.setdefault("kernel", pmc[layer][0]["name"])
            e.setdefault("grid", pmc[layer][0]["grid"])
            if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
                rd, wr = 2.0 * c["FETCH_SIZE"] * 1024.0, c["WRITE_SIZE"] * 1024.0
                e.update(read_bytes=rd, write_bytes=wr, traffic_bytes=rd + wr)
            e["counters"] = {k: v for k, v in c.items() if k not in ("FETCH_SIZE", "WRITE_SIZE")}
        if e:
            layers[layer] = e
    out = {"note": "tools/profile_round.sh: rocprofv3 --kernel-trace --stats run and separate --pmc "
                   "passes of bench.py; per-layer mean per dispatch. read_bytes = 2 x FETCH_SIZE "
                   "(gfx950 half-count of wide reads), write_bytes = WRITE_SIZE.",
           "lib_sha256": lib_sha(), "precision": prec, "workload": {"N": N, "S": S, "B": B},
           "layers": layers}
    path = os.path.join(src, f"{tag}_traffic.json")   # copied into profiles/ when committed
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    print(path, {k: (round(v.get("traffic_bytes", 0) / 2**20, 1), round(v.get("mean_ms", 0), 4))
                 for k, v in layers.items()}, "MiB/launch, ms")


if __name__ == "__main__":
    main()
