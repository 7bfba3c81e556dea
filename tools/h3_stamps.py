"""Per-phase cycle counts of the h3 engine's kernels from a stamped diagnostic build (s_memtime
at kernel entry, end of prologue, end of main loop, end of epilogue pass 0, end; wave 0 of each
workgroup; tools/stamp_build.py builds it). Diagnostic tool:
ICLR17_LIB=build/diag/lib_st.so ONLY=<h3_time runs> python tools/h3_stamps.py"""
import ctypes
import os
import runpy
import sys

import numpy as np
import torch

os.environ.setdefault("REPS", "3")
sys.argv = ["h3_time.py"]
g = runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "h3_time.py"))
from iclr_17_compression_amd import _lib  # noqa: E402

lib = _lib.load()
for k in os.environ["ONLY"].split(","):
    g["runs"][k]()
    torch.cuda.synchronize()
    scratch = np.zeros((4096, 16), dtype=np.uint64)   # clears the stamps (read, then zeroed)
    lib.diag_stamps(ctypes.c_void_p(scratch.ctypes.data), ctypes.c_long(scratch.nbytes))
    g["runs"][k]()
    torch.cuda.synchronize()
    buf = np.zeros((4096, 16), dtype=np.uint64)
    lib.diag_stamps(ctypes.c_void_p(buf.ctypes.data), ctypes.c_long(buf.nbytes))
    st = buf.astype(np.int64)
    used = st[:, 8] > 0
    st = st[used]
    d = np.diff(st[:, :9], axis=1)
    names = ["prologue", "main", "γ wait", "contract0", "out0", "γ2 wait", "contract1", "out1"]
    wall_ns = (st[:, 10] - st[:, 9]) * 10.0   # s_memrealtime: 100 MHz
    clk = (st[:, 8] - st[:, 0]) / wall_ns
    t0 = st[:, 9].min()
    span_us = (st[:, 10].max() - t0) / 100.0
    print(f"{k}: {used.sum()} WGs, span {span_us:.1f} us, WG mean {wall_ns.mean() / 1000:.2f} us, "
          f"clock {np.median(clk):.2f} GHz; cycles per WG (median): " +
          ", ".join(f"{n} {np.median(d[:, i]):.0f}" for i, n in enumerate(names)))
    starts = np.sort((st[:, 9] - t0) / 100.0)
    print("   start-time quantiles (us):", np.round(np.quantile(starts, [0, .25, .5, .75, 1]), 1))
