"""Static check of the built libiclr17.so: every workgroup barrier that a wave can reach with one of
its own LDS-DMA loads (global_load_lds) still in flight must be covered by a proof that the data
read after the barrier has landed.

Why: a bare __syncthreads() lowers to `s_waitcnt lgkmcnt(0); s_barrier` — the workgroup release
fence does not wait for vmcnt, and the compiler adds a vmcnt wait only when it proves this wave's
own later LDS reads may alias the DMA. Another wave can then read an LDS stage whose DMA has not
landed. Kernels publish DMA data in one of two ways, and each is checked on the binary:

(A) dma_barrier() / vm_barrier() (common.h: vmcnt(0) + barrier). Check: a forward may-analysis of
    "an LDS-DMA of this wave may be outstanding" (set by global_load_lds / buffer_load … lds,
    cleared by s_waitcnt vmcnt(0)) over the kernel's control-flow graph finds no barrier reached
    with the flag set.
(B) counted waits (engine_bf16.hip k5_bf16_kernel): in every step of the main loop every wave
    issues exactly K DMA instructions, and `s_waitcnt vmcnt(F·K); s_barrier` retires everything
    but the last F steps' groups; the data read after the barrier was issued F+1 steps earlier
    (the weights of step g+F+1 go out in step g; the next chunk's patch pieces in steps
    0 .. S−F−1; engine_bf16.hip:319-331, 440-453). Check: a second analysis tracks, at every
    instruction, the VMEM instructions (all of them: vmcnt counts loads and stores, in order)
    issued in the current and the previous barrier intervals, and an upper bound p on the
    outstanding ones (+1 per VMEM instruction, min(p, n) at s_waitcnt vmcnt(n)). At every barrier
    reached with p > 0 it derives K (the previous interval's count), F = p / K, and the number R
    of most recent intervals that may still hold an outstanding instruction (those newer than the
    newest p). It requires, on every path: the intervals of the loop have the same count K
    (uniform groups), p is a multiple of K, and R ≤ F — so the group issued F+1 intervals before
    the reads, the one they consume, has landed. The prologue's barrier (the first, after an
    interval of any count) needs p ≤ its count, R = 1: its last F·K instructions are the step-F
    group and F−1 padding groups (engine_bf16.hip:415-431), so the patch and the weights of
    steps 0 .. F−1, issued before them, have landed.

The check extracts every gfx950 code object from the library's .hip_fatbin section, disassembles
it with llvm-objdump and runs both analyses to a fixed point. Usage:
python tools/dma_sync_check.py [lib.so]
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
# kernels exempt from both analyses (none: every LDS-DMA kernel is checked)
COUNTED_WAIT_KERNELS: tuple = ()


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


def successors(body) -> list[list[int]]:
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
    return succ


VMCNT = re.compile(r"vmcnt\((\d+)\)")
HIST = 6        # barrier intervals tracked
CAP = 255       # counts saturate here (= unknown)
MAXSTATES = 24  # per instruction, before widening


def is_vmem(op: str) -> bool:
    return op.startswith(("global_", "buffer_", "scratch_", "flat_"))


SREG = re.compile(r"^s\[(\d+):(\d+)\]$|^s(\d+)$")


def _regs(tok: str):
    """SGPR numbers (or 'vcc') named by an operand token, or None for anything else."""
    tok = tok.strip().rstrip(",")
    if tok in ("vcc", "vcc_lo", "vcc_hi"):
        return {"vcc"}
    m = SREG.match(tok)
    if not m:
        return None
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _consts_after(consts: frozenset, op: str, ln: str) -> frozenset:
    """Wave-uniform condition tracking for the compiler's branch-select idioms
    (`s_mov_b64 sX, -1|0` … `s_and(n2)_b64 vcc, exec, sX` … `s_cbranch_vcc(n)z`), so that the
    per-path DMA counts of an if / else-if / else chain are those of feasible paths only.
    Values: 'ones' / 'zero' / 'nzx' (non-zero under exec) for SGPR pairs; for vcc 'nz' / 'zero',
    or ('and' | 'andn2', sX) while unknown (the branch on it then decides sX)."""
    text = ln.split("//")[0].strip()
    parts = text.split(None, 1)
    ops = [t.strip() for t in parts[1].split(",")] if len(parts) > 1 else []
    d = dict(consts)
    if op == "s_mov_b64" and len(ops) == 2 and ops[1] in ("-1", "0"):
        _kill(d, ops[0])
        d[ops[0]] = "ones" if ops[1] == "-1" else "zero"
        return frozenset(d.items())
    if op in ("s_and_b64", "s_andn2_b64") and len(ops) == 3 and ops[0] == "vcc" and ops[1] == "exec":
        v = d.get(ops[2])
        d.pop("vcc", None)
        if op == "s_and_b64":
            d["vcc"] = {"ones": "nz", "nzx": "nz", "zero": "zero"}.get(v, ("and", ops[2]))
        else:
            d["vcc"] = {"ones": "zero", "zero": "nz"}.get(v, ("andn2", ops[2]))
        return frozenset(d.items())
    if ops and (op.startswith("s_") or op.startswith("v_cmp") or op.startswith("v_readfirstlane")
                or op.startswith("v_readlane")):
        _kill(d, ops[0])
    return frozenset(d.items())


def _kill(d: dict, dest: str) -> None:
    w = _regs(dest)
    if not w:
        return
    for k in list(d):
        kr = _regs(k)
        if kr and kr & w:
            del d[k]
        elif isinstance(d.get(k), tuple) and (_regs(d[k][1]) or set()) & w:
            del d[k]   # vcc derived from a register now overwritten


def _branch_edges(consts: frozenset, op: str, nxt: list) -> list:
    """Successors of s_cbranch_vcc(n)z with the knowledge each edge implies: [(j, consts)]."""
    d = dict(consts)
    v = d.get("vcc")
    if len(nxt) != 2 or v is None:
        return [(j, consts) for j in nxt]
    taken_if_nz = op == "s_cbranch_vccnz"
    if v in ("nz", "zero"):
        return [(nxt[0] if (v == "nz") == taken_if_nz else nxt[1], consts)]
    kind, reg = v
    out = []
    for j, vcc_nz in ((nxt[0], taken_if_nz), (nxt[1], not taken_if_nz)):
        e = dict(d)
        e["vcc"] = "nz" if vcc_nz else "zero"
        if kind == "and":
            e[reg] = "nzx" if vcc_nz else "zero"
        elif not vcc_nz:            # exec & ~reg == 0: reg covers exec
            e[reg] = "ones"
        out.append((j, frozenset(e.items())))
    return out


def counted_barriers(body):
    """Per s_barrier offset, the set of (interval counts newest first, outstanding bound p, VMEM
    instructions since the last LDS-DMA) with which it can be reached (analysis (B) of the
    module docstring), over the feasible paths of the branch-select idioms (_consts_after)."""
    succ = successors(body)
    n = len(body)
    states: list[set] = [set() for _ in range(n)]
    start = ((0,) * HIST, 0, CAP, frozenset())
    states[0].add(start)
    work = [(0, start)]
    at_barrier: dict[int, set] = {}
    while work:
        i, (hist, p, since, consts) = work.pop()
        off, op, ln = body[i]
        if is_vmem(op):
            hist = (min(hist[0] + 1, CAP),) + hist[1:]
            p = min(p + 1, CAP)
            since = 0 if is_dma(op, ln) else min(since + 1, CAP)
        elif op == "s_waitcnt":
            m = VMCNT.search(ln)
            if m:
                p = min(p, int(m.group(1)))
        elif op == "s_barrier":
            at_barrier.setdefault(off, set()).add((hist, p, since))
            # nothing of this wave outstanding (p = 0, e.g. after vm_barrier's vmcnt(0)): the
            # intervals before are settled, and the next one starts like the kernel's first
            hist = (0,) * HIST if p == 0 else (0,) + hist[:-1]
        consts = _consts_after(consts, op, ln)
        if op in ("s_cbranch_vccnz", "s_cbranch_vccz"):
            edges = _branch_edges(consts, op, succ[i])
        elif op in ("s_cbranch_execnz", "s_cbranch_execz") and len(succ[i]) == 2:
            # exec is never empty here (full 64-lane waves, wave-uniform control flow); the
            # compiler uses these as the taken / not-taken ends of its uniform block layout
            edges = [(succ[i][0] if op == "s_cbranch_execnz" else succ[i][1], consts)]
        else:
            edges = [(j, consts) for j in succ[i]]
        for j, cj in edges:
            st = (hist, p, since, cj)
            if st in states[j]:
                continue
            if len(states[j]) >= MAXSTATES:
                # widening (a loop without a barrier that issues VMEM: its count is unknown):
                # join every state of this point into one, differing counts → CAP, p → max
                allst = states[j] | {st}
                hs = [h for h, _, _, _ in allst]
                st = (tuple(hs[0][k] if all(h[k] == hs[0][k] for h in hs) else CAP
                            for k in range(HIST)), max(q for _, q, _, _ in allst),
                      min(q for _, _, q, _ in allst),
                      frozenset.intersection(*[c for _, _, _, c in allst]))
                if st in states[j]:
                    continue
                states[j] = {st}
            else:
                states[j].add(st)
            work.append((j, st))
    return at_barrier


def window_intervals(hist, p) -> int:
    """How many of the most recent intervals may hold one of the newest p VMEM instructions."""
    if p == 0:
        return 0
    newer = 0
    for i, c in enumerate(hist):
        if c >= CAP:
            return i + 1      # the rest lies in the prologue's interval (see counted_violations)
        if newer + c >= p:
            return i + 1
        newer += c
    return HIST + 1


def counted_violations(body) -> tuple[list[str], set]:
    """Analysis (B): the counted-wait proof at every barrier reached with p > 0. K = the count of
    the interval the barrier closes (a step's group), F = p / K; walking back from it, the
    intervals the newest p instructions may reach must each hold exactly K, except where the
    window reaches the prologue's interval (unknown count: its trailing F·K instructions are the
    step-F group and F−1 padding groups by construction). Returns the violations and the
    (K, F) pairs proved."""
    bad, kf = [], set()
    for off, sts in sorted(counted_barriers(body).items()):
        for hist, p, since in sts:
            if p <= since:
                continue   # the newest p VMEM instructions hold no LDS-DMA
            K = hist[0]
            if K >= CAP or all(c == 0 for c in hist[1:]):
                # the prologue's own barrier: the newest p are its padding tail
                if K < CAP and p > K:
                    bad.append(f"+{hex(off)}: prologue barrier with p={p} > its {K} instructions")
                continue
            if K == 0 or p % K:
                bad.append(f"+{hex(off)}: vmcnt bound {p} vs a closing group of {K} ({hist})")
                continue
            F = p // K
            covered = 0
            for i in range(HIST):
                if covered >= p:
                    break
                if hist[i] >= CAP or all(c == 0 for c in hist[i + 1:]):
                    break          # into the prologue's tail (the kernel's first interval)
                if hist[i] != K:
                    bad.append(f"+{hex(off)}: non-uniform groups {hist} (K={K}, p={p})")
                    break
                covered += K
            else:
                if covered < p:
                    bad.append(f"+{hex(off)}: window of {p} beyond the tracked history {hist}")
                    continue
            if window_intervals(hist, p) > F:
                bad.append(f"+{hex(off)}: {window_intervals(hist, p)} intervals may be outstanding, F={F}")
            kf.add((K, F))
    return bad, kf


def check(lib: str, report: dict | None = None) -> tuple[list[str], int]:
    bad, nk = [], 0
    for co in code_objects(lib):
        for name, body in kernels(co).items():
            if not any(is_dma(op, ln) for _, op, ln in body):
                continue
            nk += 1
            if any(k in name for k in COUNTED_WAIT_KERNELS):
                continue
            offs = unguarded_barriers(body)
            if not offs:
                continue
            # (B): the barriers reached with a DMA in flight must carry the counted-wait proof
            vb, kf = counted_violations(body)
            if vb or not kf:
                bad.append(f"{name}: s_barrier at +{', +'.join(hex(o) for o in offs)} with an LDS-DMA "
                           f"in flight; counted-wait proof: {'; '.join(vb) or 'no counted barrier'}")
            elif report is not None:
                report[name] = sorted(kf)
    return bad, nk


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "iclr_17_compression_amd", "libiclr17.so")
    rep: dict = {}
    bad, nk = check(lib, rep)
    print(f"{nk} kernels issue LDS-DMA; {len(rep)} publish by counted waits (proved: (K, F) = groups "
          f"per step, groups in flight); {len(bad)} reach a barrier with a DMA unproven")
    for k, v in sorted(rep.items()):
        print(f"  counted: {k} {v}")
    for b in bad:
        print("  " + b)
    sys.exit(1 if bad else 0)
