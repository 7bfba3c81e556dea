"""Per-kernel PMC table from a tools/prof_bf16.sh (or pmc.sh) output directory: averages each
counter over the dispatches of each kernel and prints derived ratios.

    python tools/pmc_table.py gpurun_out/<tag> [kernel-substring ...]
"""
import csv
import glob
import os
import re
import sys


def load(src):
    per = {}
    for f in sorted(glob.glob(os.path.join(src, "p*", "pmc_counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            k = re.sub(r"\s+", " ", row["Kernel_Name"])
            per.setdefault(k, {}).setdefault(row["Counter_Name"], []).append(float(row["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main():
    src = sys.argv[1]
    pats = sys.argv[2:]
    ks = load(src)
    for k, c in sorted(ks.items()):
        if pats and not any(p in k for p in pats):
            continue
        if "SQ_WAVE_CYCLES" not in c and "SQ_INSTS_MFMA" not in c:
            continue
        print(k[:110])
        w = c.get("SQ_WAVE_CYCLES", 0) or 1
        line = []
        for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if n in c:
                line.append(f"{n[3:]} {c[n] / w:.2f}")
        if "SQ_INSTS_MFMA" in c:
            line.append(f"MFMA {c['SQ_INSTS_MFMA']:.3e} VALU {c.get('SQ_INSTS_VALU', 0):.3e} "
                        f"LDS {c.get('SQ_INSTS_LDS', 0):.3e}")
        if "SQ_LDS_IDX_ACTIVE" in c:
            line.append(f"LDS conflict {c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_LDS_IDX_ACTIVE'], 1):.3f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and "GRBM_GUI_ACTIVE" in c:
            # MFMA busy per SIMD over the kernel's GUI-active cycles (per XCD: / 8)
            line.append(f"MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (c['GRBM_GUI_ACTIVE'] / 8):.3f}")
        if "FETCH_SIZE" in c:
            line.append(f"read {2 * c['FETCH_SIZE'] * 1024 / 1e6:.1f} MB")
        if "WRITE_SIZE" in c:
            line.append(f"write {c['WRITE_SIZE'] * 1024 / 1e6:.1f} MB")
        print("   " + " | ".join(line))


if __name__ == "__main__":
    main()
