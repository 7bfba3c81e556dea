"""ORACLE — CPU restatement of the entropy coder (csrc/rans.hip). TEST INFRASTRUCTURE ONLY.

Only ``tests/`` may import this module, as the checker. The reference has no entropy coder: it
only ESTIMATES the rate from the factorised model (model.py:71-78, models/bitEstimator.py:20-42).
This restates the build's coder in plain Python integers so that the GPU
bitstream can be checked word for word. The probability model is pinned to the reference
through ``codec_ref.bit_estimator`` (itself pinned by the G2 golden). The coder format has no
reference counterpart: parity unpinned by the reference; the pins are round-trip exactness and
word-for-word agreement with this restatement.

Format (shared with rans.hip):
  symbols per channel c: v ∈ [−K, K] → v + K, escape 2K + 1 (then v + 32768 as a uniform
  16-bit symbol); frequencies f_i = 1 + ⌊p_i·(2^16 − (2K + 2))⌋ in fp32, the most probable
  symbol absorbing the remainder; interleaved rANS with 64 states in [2^16, 2^32) (state l
  owns symbols l, l + 64, …), 16-bit words, every state starting from 2^16; streams = (image,
  channel group), symbols in (channel, row, column) order (see encode_stream for the word
  order).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

from . import codec_ref

PROB_SCALE = 1 << 16
L = 1 << 16
LANES = 64        # interleaved rANS states per stream (one wave on the GPU)


def boundary_cdf(p: Dict[str, torch.Tensor], N: int, K: int) -> np.ndarray:
    """F_c(j − K − ½) for j = 0 .. 2K + 1, float32 [N, 2K + 2] (codec_ref.bit_estimator)."""
    v = torch.arange(2 * K + 2, dtype=torch.float32) - K - 0.5
    x = v.view(1, 1, 1, -1).expand(1, N, 1, 2 * K + 2).contiguous()
    return codec_ref.bit_estimator(x, p)[0, :, 0, :].numpy().astype(np.float32)


def tables_from_cdf(cdf: np.ndarray, K: int) -> np.ndarray:
    """rans.hip tables_kernel: int64 [N, 2K + 3] cumulative frequencies."""
    N = cdf.shape[0]
    NS = 2 * K + 2
    spread = np.float32(PROB_SCALE - NS)
    cum = np.zeros((N, NS + 1), dtype=np.int64)
    for c in range(N):
        s = cdf[c]
        freq = []
        pmax, imax = np.float32(-1.0), 0
        for i in range(NS):
            if i < NS - 1:
                p = np.float32(s[i + 1] - s[i])
            else:
                p = np.float32(s[0] + np.float32(np.float32(1.0) - s[2 * K + 1]))
            p = max(p, np.float32(0.0))
            freq.append(1 + int(np.floor(np.float32(p * spread))))
            if p > pmax:
                pmax, imax = p, i
        freq[imax] += PROB_SCALE - sum(freq)
        cum[c, 1:] = np.cumsum(freq)
    return cum


def _symbols(values: Sequence[int], K: int) -> List[Tuple[int, int]]:
    """(symbol, escape payload or −1) per value."""
    out = []
    for v in values:
        v = int(v)
        if not -32767 <= v <= 32767:
            raise ValueError("value out of the 16-bit escape range")
        out.append((v + K, -1) if -K <= v <= K else (2 * K + 1, v + 32768))
    return out


def encode_stream(values: Sequence[int], chans: Sequence[int], cum: np.ndarray, K: int,
                  W: int = LANES) -> List[int]:
    """One stream's words (decoder order). Lane l of W owns symbols l, l + W, …; blocks of W
    symbols are encoded last to first, escape payloads (sub-round B) before the symbols
    (sub-round A); each (block, sub-round)'s renormalisation words form one group in lane
    order; the stream is the W final states (high word first) then the groups in reverse of
    the order they were written."""
    syms = _symbols(values, K)
    n = len(syms)
    x = [L] * W
    groups: List[List[int]] = []
    for blk in reversed(range((n + W - 1) // W)):
        lanes = [l for l in range(W) if blk * W + l < n]
        gb = []
        for l in lanes:
            sym, pay = syms[blk * W + l]
            if pay >= 0:   # uniform 16-bit payload (freq 1): always one word out
                gb.append(x[l] & 0xFFFF)
                x[l] = ((x[l] >> 16) << 16) + pay
        groups.append(gb)
        ga = []
        for l in lanes:
            sym, _ = syms[blk * W + l]
            c = chans[blk * W + l]
            start, f = int(cum[c, sym]), int(cum[c, sym + 1] - cum[c, sym])
            if x[l] >= (f << 16):
                ga.append(x[l] & 0xFFFF)
                x[l] >>= 16
            x[l] = ((x[l] // f) << 16) + (x[l] % f) + start
        groups.append(ga)
    words = [w for l in range(W) for w in (x[l] >> 16, x[l] & 0xFFFF)]
    for g in reversed(groups):
        words += g
    return words


def decode_stream(words: Sequence[int], chans: Sequence[int], cum: np.ndarray, K: int,
                  W: int = LANES) -> List[int]:
    if len(words) < 2 * W:
        raise ValueError("stream ran past its words")
    x = [(int(words[2 * l]) << 16) | int(words[2 * l + 1]) for l in range(W)]
    pos = 2 * W

    def nxt() -> int:
        nonlocal pos
        if pos >= len(words):
            raise ValueError("stream ran past its words")
        w = int(words[pos])
        pos += 1
        return w

    NS = 2 * K + 2
    n = len(chans)
    vals = [0] * n
    for blk in range((n + W - 1) // W):
        lanes = [l for l in range(W) if blk * W + l < n]
        esc = []
        for l in lanes:
            c = chans[blk * W + l]
            slot = x[l] & 0xFFFF
            sym = int(np.searchsorted(cum[c], slot, side="right")) - 1
            start, f = int(cum[c, sym]), int(cum[c, sym + 1] - cum[c, sym])
            x[l] = f * (x[l] >> 16) + slot - start
            vals[blk * W + l] = sym - K
            if sym == NS - 1:
                esc.append(l)
        for l in lanes:            # sub-round A
            if x[l] < L:
                x[l] = (x[l] << 16) | nxt()
        for l in esc:              # sub-round B
            vals[blk * W + l] = (x[l] & 0xFFFF) - 32768
            x[l] >>= 16
            x[l] = (x[l] << 16) | nxt()
    if any(v != L for v in x) or pos != len(words):
        raise ValueError("stream did not end in the initial state")
    return vals


def _stream_order(B: int, h: int, w: int, N: int, P: int):
    cpg = N // P
    for b in range(B):
        for g in range(P):
            idx = [(b, y, x, g * cpg + cl) for cl in range(cpg) for y in range(h) for x in range(w)]
            yield idx


def encode(y_nhwc: np.ndarray, cum: np.ndarray, K: int, P: int) -> Tuple[np.ndarray, np.ndarray]:
    """ŷ NHWC integer-valued → (uint16 words, int64 offsets [B·P + 1]) as rans.hip lays them out."""
    B, h, w, N = y_nhwc.shape
    streams = []
    for idx in _stream_order(B, h, w, N, P):
        vals = [int(y_nhwc[i]) for i in idx]
        streams.append(encode_stream(vals, [i[3] for i in idx], cum, K))
    offsets = np.concatenate([[0], np.cumsum([len(s) for s in streams])]).astype(np.int64)
    words = np.array([wd for s in streams for wd in s], dtype=np.uint16)
    return words, offsets


def decode(words: np.ndarray, offsets: np.ndarray, cum: np.ndarray, K: int, B: int, h: int,
           w: int, N: int, P: int) -> np.ndarray:
    y = np.zeros((B, h, w, N), dtype=np.float32)
    for s, idx in enumerate(_stream_order(B, h, w, N, P)):
        vals = decode_stream(words[offsets[s]:offsets[s + 1]], [i[3] for i in idx], cum, K)
        for i, v in zip(idx, vals):
            y[i] = v
    return y


def ideal_bits(y_nhwc: np.ndarray, cum: np.ndarray, K: int) -> float:
    """Σ −log2(f/2^16) of the symbols (+16 per escape payload): the coder's own entropy."""
    NS = 2 * K + 2
    v = y_nhwc.astype(np.int64)
    sym = np.where(np.abs(v) <= K, v + K, NS - 1)
    c = np.broadcast_to(np.arange(y_nhwc.shape[-1]), v.shape)
    f = (cum[c, sym + 1] - cum[c, sym]).astype(np.float64)
    return float((-np.log2(f / PROB_SCALE)).sum() + 16.0 * (sym == NS - 1).sum())
