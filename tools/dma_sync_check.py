"""Static check of the built libiclr17.so: no workgroup barrier may be reached while one of the
wave's own LDS-DMA loads (global_load_lds) can still be in flight, unless the kernel is one of the
counted-wait kernels listed below.

Why: a bare __syncthreads() lowers to `s_waitcnt lgkmcnt(0); s_barrier` — the workgroup release
fence does not wait for vmcnt, and the compiler adds a vmcnt wait only when it proves this wave's
own later LDS reads may alias the DMA. Another wave can then read an LDS stage whose DMA has not
landed. Kernels publish DMA data with dma_barrier() (common.h: vmcnt(0) + barrier), or, in the
bf16 k5 engine, with counted vmcnt(F·K) waits over uniform per-wave DMA groups (by design they keep
F groups in flight across the barrier and never read them before the next counted wait).

The check extracts every gfx950 code object from the library's .hip_fatbin section, disassembles
it with llvm-objdump, builds each kernel's control-flow graph and runs a forward may-analysis of
"an LDS-DMA of this wave may be outstanding" (set by global_load_lds / buffer_load … lds, cleared
by s_waitcnt vmcnt(0)) to a fixed point. Usage: python tools/dma_sync_check.py [lib.so]
"""
from __future__ import annotations

import os
import re
import struct
import subprocess
import sys
import tempfile

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
OBJCOPY = "/opt/rocm/lib/llvm/bin/llvm-objcopy"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
# kernels whose DMA groups are retired by counted vmcnt(N) waits by design (engine_bf16.hip)
COUNTED_WAIT_KERNELS = ("k5_bf16_kernel",)


def code_objects(lib: str) -> list[bytes]:
    with tempfile.TemporaryDirectory() as td:
        fb = os.path.join(td, "fatbin")
        subprocess.run([OBJCOPY, "-O", "binary", "--only-section=.hip_fatbin", lib, fb], check=True)
        data = open(fb, "rb").read()
    out, pos = [], 0
    while True:
        i = data.find(MAGIC, pos)
        if i < 0:
            return out
        (cnt,) = struct.unpack_from("<Q", data, i + 24)
        p = i + 32
        for _ in range(cnt):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            p += 24
            triple = data[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                out.append(data[i + off:i + off + size])
        pos = i + 1


INS = re.compile(r"^\s+(\S+)(.*?)//\s*([0-9A-Fa-f]+):")
SYM = re.compile(r"^[0-9a-f]+ <(\S+)>:")
TGT = re.compile(r"<(\S+)\+0x([0-9a-f]+)>")


def kernels(co: bytes) -> dict[str, list[tuple[int, str, str]]]:
    with tempfile.NamedTemporaryFile(suffix=".elf") as f:
        f.write(co)
        f.flush()
        txt = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], check=True,
                             capture_output=True, text=True).stdout
    ks: dict[str, list] = {}
    cur = None
    base = 0
    for ln in txt.splitlines():
        m = SYM.match(ln)
        if m:
            cur = m.group(1)
            ks[cur] = []
            base = int(ln.split()[0], 16)
            continue
        m = INS.match(ln)
        if m and cur:
            ks[cur].append((int(m.group(3), 16) - base, m.group(1), ln))
    return ks


def is_dma(op: str, line: str) -> bool:
    return op.startswith("global_load_lds") or (op.startswith("buffer_load") and " lds" in line)


def clears(op: str, line: str) -> bool:
    return op == "s_waitcnt" and "vmcnt(0)" in line


def unguarded_barriers(body) -> list[int]:
    """Offsets of s_barrier instructions reachable with a possibly outstanding LDS-DMA."""
    idx = {off: i for i, (off, _, _) in enumerate(body)}
    n = len(body)
    succ: list[list[int]] = []
    for i, (off, op, ln) in enumerate(body):
        s = []
        if op.startswith("s_branch") or op.startswith("s_cbranch"):
            m = TGT.search(ln)
            if m and int(m.group(2), 16) in idx:
                s.append(idx[int(m.group(2), 16)])
            if op.startswith("s_cbranch") and i + 1 < n:
                s.append(i + 1)
        elif op == "s_endpgm" or op.startswith("s_setpc") or op.startswith("s_trap"):
            pass
        elif i + 1 < n:
            s.append(i + 1)
        succ.append(s)
    state_in = [False] * n
    reached = [False] * n
    work = [0]
    reached[0] = True
    while work:
        i = work.pop()
        st = state_in[i]
        off, op, ln = body[i]
        out = True if is_dma(op, ln) else (False if clears(op, ln) else st)
        for j in succ[i]:
            if not reached[j] or (out and not state_in[j]):
                reached[j] = True
                state_in[j] = state_in[j] or out
                work.append(j)
    return [body[i][0] for i in range(n) if body[i][1] == "s_barrier" and state_in[i]]


def check(lib: str) -> tuple[list[str], int]:
    bad, nk = [], 0
    for co in code_objects(lib):
        for name, body in kernels(co).items():
            if not any(is_dma(op, ln) for _, op, ln in body):
                continue
            nk += 1
            if any(k in name for k in COUNTED_WAIT_KERNELS):
                continue
            offs = unguarded_barriers(body)
            if offs:
                bad.append(f"{name}: s_barrier at +{', +'.join(hex(o) for o in offs)}")
    return bad, nk


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iclr_17_compression_amd", "libiclr17.so")
    bad, nk = check(lib)
    print(f"{nk} kernels issue LDS-DMA; {len(bad)} reach a barrier with a DMA possibly in flight")
    for b in bad:
        print("  " + b)
    sys.exit(1 if bad else 0)
