"""Per-kernel table of a tools/prof_train_pmc.sh run: calls per training step, trace mean and
share of the step, HBM traffic per call (2 × FETCH_SIZE + WRITE_SIZE, KB counters; the gfx950
half-count of wide reads, MI355X_MICROARCH.md §HBM), MFMA busy fraction and wait shares.

    python tools/train_pmc_table.py gpurun_out/<tag> <tag>   → <dir>/<tag>_train_kernels.json
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name: str) -> str:
    """Kernel name without its trailing argument list (an anonymous namespace stays)."""
    name = name.strip()
    if name.endswith(")"):
        depth = 0
        for i in range(len(name) - 1, -1, -1):
            depth += {")": 1, "(": -1}.get(name[i], 0)
            if depth == 0:
                name = name[:i]
                break
    name = re.sub(r"^void ", "", name)
    return name.replace("(anonymous namespace)::", "")[:160]


def main() -> None:
    src, tag = sys.argv[1], sys.argv[2]
    steps = int(os.environ.get("TRACE_STEPS", "13"))   # 10 timed + 3 warm-up
    trace = glob.glob(f"{src}/trace/**/*kernel_trace.csv", recursive=True)
    dur = defaultdict(list)
    for f in trace:
        for row in csv.DictReader(open(f)):
            dur[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    total = sum(sum(v) for v in dur.values())
    cnt = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{src}/p*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            cnt[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
    rows = []
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        c = {n: sum(x) / len(x) for n, x in cnt.get(k, {}).items()}
        r = {"kernel": k, "calls_per_step": round(len(v) / steps, 2), "mean_ms": round(sum(v) / len(v), 5),
             "share": round(sum(v) / total, 4)}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            r["traffic_bytes_per_call"] = round(2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024)
        if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            # GRBM_GUI_ACTIVE sums the 8 XCDs; 32 CUs × 4 SIMDs per XCD
            simd_cycles = c["GRBM_GUI_ACTIVE"] / 8 * 1024
            r["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / simd_cycles, 3)
            r["clock_ghz"] = round(c["GRBM_GUI_ACTIVE"] / 8 / (r["mean_ms"] * 1e6), 2)
        if c.get("SQ_WAVE_CYCLES"):
            r["wait_any"] = round(c.get("SQ_WAIT_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
            r["wait_inst_any"] = round(c.get("SQ_WAIT_INST_ANY", 0) / c["SQ_WAVE_CYCLES"], 3)
        if c.get("SQ_INSTS_MFMA"):
            r["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0) / c["SQ_INSTS_MFMA"], 2)
        if c.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict"] = round(c.get("SQ_LDS_BANK_CONFLICT", 0) / c["SQ_LDS_IDX_ACTIVE"], 3)
        rows.append(r)
    lib = os.path.join(REPO, "iclr_17_compression_amd", "libiclr17.so")
    out = {"lib_sha256": hashlib.sha256(open(lib, "rb").read()).hexdigest()[:16],
           "workload": "bench.py --mode train --batch 32 (B=32 256², N=192, h3 forward + x6 backward)",
           "traced_steps": steps, "step_ms_under_trace": round(total / steps, 4), "kernels": rows}
    json.dump(out, open(os.path.join(src, f"{tag}_train_kernels.json"), "w"), indent=1)
    print(f"{len(rows)} kernels, {total / steps:.3f} ms per step under trace")
    for r in rows[:12]:
        print(f"{r['share']:.3f} {r['mean_ms']:.4f} ms x{r['calls_per_step']} {r.get('mfma_busy')} {r.get('clock_ghz')} {r['kernel'][:90]}")


if __name__ == "__main__":
    main()
