"""iclr_17_compression_amd — MI355X-native (gfx950) Ballé-2017 codec hot path.

Drop-in for the reference's model.py / models/ surface (Yuval-H/iclr_17_compression):

    from iclr_17_compression_amd.model import ImageCompressor, save_model, load_model
    from iclr_17_compression_amd.models import GDN, BitEstimator, Analysis_net_17, Synthesis_net_17

All compute runs in libiclr17.so (hand-written HIP kernels, C ABI in include/iclr17.h).
"""
__version__ = "0.1.0"
