"""Summarise tools/gpu_c3_pmc.sh: per conv3 kernel variant and run, mean per dispatch of the
collected counters and the derived MFMA busy, VALU per MFMA, wait share and L2 hit rate."""
import collections
import sqlite3
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c3_pmc"
KEYS = ("engine_kernel<192, 192, 48", "engine_kernel<192, 192, 96")
for run in ("p1", "p2", "t1_0", "t1_1", "t2_0", "t2_1"):
    c = sqlite3.connect(f"{root}/{run}/run_results.db")
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for name, disp, d, cn, cv in c.execute(
            "select name, dispatch_id, duration, counter_name, counter_value from pmc_events"):
        if not any(k in name for k in KEYS):
            continue
        key = name.split("(")[0].replace("void iclr17::", "")
        acc[key][cn].append(cv)
        dur[key][disp] = d
    for key, cs in acc.items():
        m = {cn: sum(v) / len(v) for cn, v in cs.items()}
        # counter values are summed per dispatch already (one row per dispatch and counter)
        n = len(dur[key])
        ms = sum(dur[key].values()) / n / 1e6
        out = [f"{run:5s} {key:55s} n={n:3d} {ms:.4f} ms"]
        g = m.get("GRBM_GUI_ACTIVE")
        if g:
            out.append(f"clk {g / 8 / (ms * 1e-3) / 1e9:.2f} GHz")
        if "TCC_HIT_sum" in m:
            h, mi = m["TCC_HIT_sum"], m["TCC_MISS_sum"]
            out.append(f"L2 hit {h / (h + mi):.3f} (miss {mi * 128 / 1e6:.0f} MB@128B)")
        if "SQ_INSTS_MFMA" in m:
            out.append(f"mfma_busy {m['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
            out.append(f"valu/mfma {m['SQ_INSTS_VALU'] / m['SQ_INSTS_MFMA']:.2f}")
            out.append(f"lds/mfma {m['SQ_INSTS_LDS'] / m['SQ_INSTS_MFMA']:.2f}")
            out.append(f"wait_any {m['SQ_WAIT_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
            out.append(f"wait_inst {m['SQ_WAIT_INST_ANY'] / m['SQ_WAVE_CYCLES']:.3f}")
            out.append(f"waves/SIMD {m['SQ_WAVE_CYCLES'] / (g / 8 * 1024):.2f}")
        print("  ".join(out))
