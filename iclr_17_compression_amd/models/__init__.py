"""The reference's ``models`` package surface (models/__init__.py:1-9) for the hot path:
GDN, BitEstimator, Analysis_net_17, Synthesis_net_17 (+ Bitparm, LowerBound) and the
evaluation metrics ms_ssim / ssim (models/__init__.py:7, on the GPU kernels).

The legacy 4-layer nets (Analysis_net, Synthesis_net, *_prior_net) the reference re-exports
reference undefined globals there and are not instantiable."""
from .GDN import GDN, LowerBound
from .bitEstimator import BitEstimator, Bitparm
from .ms_ssim_torch import ms_ssim, ssim
from .analysis_17 import Analysis_net_17
from .synthesis_17 import Synthesis_net_17

__all__ = ["GDN", "LowerBound", "BitEstimator", "Bitparm", "Analysis_net_17", "Synthesis_net_17",
           "ms_ssim", "ssim"]
