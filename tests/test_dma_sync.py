"""Static synchronisation check of the built library (CPU): in every kernel that stages operands
by LDS-DMA, no workgroup barrier is reachable while one of the wave's own DMAs may still be in
flight (tools/dma_sync_check.py: CFG may-analysis over the disassembled gfx950 code objects),
unless the counted-wait proof holds there (analysis (B): uniform per-step DMA groups under
vmcnt(F·K), the consumed group F+1 steps old) — no kernel is exempt.
A bare __syncthreads() does not wait for vmcnt; conv1_gdn_kernel's main loop once compiled to
`s_waitcnt lgkmcnt(0); s_barrier` with the next weight stage in flight and read a stale stage in
about one run in twenty."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "iclr_17_compression_amd", "libiclr17.so")
sys.path.insert(0, os.path.join(REPO, "tools"))
import dma_sync_check  # noqa: E402


@pytest.mark.skipif(not os.path.exists(dma_sync_check.OBJDUMP), reason="no llvm-objdump")
def test_no_barrier_with_lds_dma_in_flight():
    assert os.path.exists(LIB), "build the library first (__graft_entry__.build())"
    rep = {}
    bad, nk = dma_sync_check.check(LIB, rep)
    assert nk >= 20, nk   # the engine, conv1, deconv3, wgrad, bf16 kernels all use LDS-DMA
    assert not bad, bad
    assert dma_sync_check.COUNTED_WAIT_KERNELS == ()   # nothing exempt
    # every bf16 k5 engine instantiation carries the counted-wait proof (analysis (B))
    assert len([k for k in rep if "k5_bf16_kernel" in k]) == 8, sorted(rep)


def _body(lines):
    """(offset, mnemonic, text) triples in the disassembler's form, 4 bytes apart."""
    out = []
    for i, t in enumerate(lines):
        out.append((4 * i, t.split()[0], "\t" + t + " // " + format(4 * i, "x") + ":"))
    return out


def _loop(groups, wait):
    """A prologue of 5 DMAs, then barrier-closed steps issuing groups[i] DMAs each."""
    lines = ["global_load_lds_dwordx4 v[0:1], off"] * 5 + [f"s_waitcnt vmcnt({wait})", "s_barrier"]
    for g in groups:
        lines += ["global_load_lds_dwordx4 v[0:1], off"] * g + [f"s_waitcnt vmcnt({wait})", "s_barrier"]
    return _body(lines + ["s_waitcnt vmcnt(0)", "s_barrier", "s_endpgm"])


def test_counted_wait_proof_on_synthetic_schedules():
    """The counted-wait analysis (B) accepts uniform K-instruction groups under vmcnt(F·K) and
    rejects a step that issues a different count (an older group may then still be in flight)."""
    bad, kf = dma_sync_check.counted_violations(_loop([2] * 6, 4))
    assert not bad and kf == {(2, 2)}
    bad, _ = dma_sync_check.counted_violations(_loop([2, 2, 1, 2, 2, 2], 4))
    assert bad
    bad, _ = dma_sync_check.counted_violations(_loop([2] * 6, 3))   # not a multiple of K
    assert bad
    # the dma_barrier form needs no proof: vmcnt(0) before every barrier
    assert not dma_sync_check.unguarded_barriers(_loop([2] * 3, 0))


def test_branch_select_paths_are_feasible_only():
    """An if / else-if / else DMA chain in the compiler's select idiom issues one DMA per path;
    without the constant tracking the analysis would count infeasible 0- and 2-DMA paths."""
    step = ["global_load_lds_dwordx4 v[0:1], off",
            "s_and_b64 vcc, exec, s[24:25]", "s_mov_b64 s[90:91], -1",
            "s_cbranch_vccnz BR1",
            "s_mov_b64 s[90:91], 0", "global_load_lds_dwordx4 v[0:1], off",
            "s_andn2_b64 vcc, exec, s[90:91]", "s_cbranch_vccnz BR2",
            "global_load_lds_dwordx4 v[0:1], off", "s_waitcnt vmcnt(4)", "s_barrier"]
    lines = ["global_load_lds_dwordx4 v[0:1], off"] * 5 + ["s_waitcnt vmcnt(4)", "s_barrier"]
    for _ in range(5):
        lines += step
    body = _body(lines + ["s_waitcnt vmcnt(0)", "s_barrier", "s_endpgm"])
    # resolve the two forward branches of each step (to the andn2 and to the wait)
    fixed = []
    for off, op, ln in body:
        if "BR1" in ln:
            tgt = next(o for o, p2, l2 in body if o > off and "s_andn2_b64" in l2)
            ln = ln.replace("BR1", f"<k+0x{tgt:x}>")
        if "BR2" in ln:
            tgt = next(o for o, p2, l2 in body if o > off and "s_waitcnt vmcnt(4)" in l2)
            ln = ln.replace("BR2", f"<k+0x{tgt:x}>")
        fixed.append((off, op, ln))
    bad, kf = dma_sync_check.counted_violations(fixed)
    assert not bad and kf == {(2, 2)}, (bad, kf)
