"""The reference's ``models`` package surface (models/__init__.py:1-9) for the hot path:
GDN, BitEstimator, Analysis_net_17, Synthesis_net_17 (+ Bitparm, LowerBound).

The legacy 4-layer nets (Analysis_net, Synthesis_net, *_prior_net) the reference re-exports
reference undefined globals there and are not instantiable, and ms_ssim/ssim
are evaluation metrics outside this round's kernel scope."""
from .GDN import GDN, LowerBound
from .bitEstimator import BitEstimator, Bitparm
from .analysis_17 import Analysis_net_17
from .synthesis_17 import Synthesis_net_17

__all__ = ["GDN", "LowerBound", "BitEstimator", "Bitparm", "Analysis_net_17", "Synthesis_net_17"]
