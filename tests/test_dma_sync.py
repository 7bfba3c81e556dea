"""Static synchronisation check of the built library (CPU): in every kernel that stages operands
by LDS-DMA, no workgroup barrier is reachable while one of the wave's own DMAs may still be in
flight (tools/dma_sync_check.py: CFG may-analysis over the disassembled gfx950 code objects).
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
    bad, nk = dma_sync_check.check(LIB)
    assert nk >= 20, nk   # the engine, conv1, deconv3, wgrad, bf16 kernels all use LDS-DMA
    assert not bad, bad
