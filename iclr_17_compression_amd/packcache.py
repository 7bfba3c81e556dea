"""Derived-layout caches of module parameters (packed weights, effective GDN params, rate
tables). Keyed by (storage pointer, version counter) of every source tensor, so an in-place
optimizer step or load_state_dict invalidates the entry; ``invalidate()`` forces a repack."""
from __future__ import annotations

from typing import Callable, Dict, Sequence, Tuple

import torch


class PackCache:
    def __init__(self) -> None:
        self._d: Dict[str, Tuple[tuple, object]] = {}

    def get(self, key: str, sources: Sequence[torch.Tensor], build: Callable[[], object],
            force: bool = False):
        sig = tuple((t.data_ptr(), t._version, str(t.device)) for t in sources)
        hit = self._d.get(key)
        if not force and hit is not None and hit[0] == sig:
            return hit[1]
        val = build()
        self._d[key] = (sig, val)
        return val

    def invalidate(self) -> None:
        self._d.clear()
