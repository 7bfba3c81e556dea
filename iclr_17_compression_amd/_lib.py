"""ctypes binding of libiclr17.so (C ABI declared in include/iclr17.h).

The library is the ONLY compute path of this package: there is no PyTorch or CPU fallback.
Loading fails loudly (ImportError-style RuntimeError) when the shared object is missing; every
op fails loudly on non-GPU tensors.

torch is imported first on purpose: torch ships its own libamdhip64.so (same SONAME as the
system ROCm's), so importing it first makes libiclr17.so bind to the HIP runtime that owns
torch's streams and allocations instead of loading a second runtime into the process.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ICLR17_LIB", os.path.join(_HERE, "libiclr17.so"))

ICLR17_QUANT_ROUND = 0
ICLR17_QUANT_NOISE = 1
ICLR17_LAYOUT_NCHW = 0
ICLR17_LAYOUT_NHWC = 1
ICLR17_W_CONV1 = 0
ICLR17_W_CONV5 = 1
ICLR17_W_DECONV5 = 2
ICLR17_W_DECONV9 = 3
ICLR17_W_CONV1_X6 = 4
ICLR17_PACK_GDN = 16
ICLR17_PACK_RATE = 17
ICLR17_PACK_SPLIT = 18
ICLR17_BF_CONV5 = 32
ICLR17_BF_DECONV5 = 33
ICLR17_H3K_CONV5 = 42
ICLR17_H3K_DECONV5 = 43
ICLR17_H3K_CONV1 = 44
ICLR17_PACK_H3K = 19
ICLR17_PACK_SPLIT_H3 = 20
ICLR17_PACK_H3_MAXJ = 16

_P = ctypes.c_void_p
_I = ctypes.c_int
_I64 = ctypes.c_int64
_D = ctypes.c_double
_F = ctypes.c_float
_SZ = ctypes.c_size_t

# name: (restype, argtypes) — one line per entry point of include/iclr17.h
SIGNATURES = {
    "iclr17_version": (_I, []),
    "iclr17_last_error": (_I, [ctypes.c_char_p, _SZ]),
    "iclr17_packed_weight_size": (_SZ, [_I, _I]),
    "iclr17_pack_weight": (_I, [_I, _P, _P, _I, _P]),
    "iclr17_pack_gdn": (_I, [_P, _P, _P, _P, _P, _I, _F, _F, _F, _P]),
    "iclr17_pack_rate": (_I, [_P] * 12 + [_I, _P]),
    "iclr17_pack_batch": (_I, [_P, _I, _P, _P]),
    "iclr17_analysis_conv1_gdn": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv2_gdn": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv3_quant_rate": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_rate_partials_per_image": (_I, [_I, _I, _I]),
    "iclr17_conv3_x6_partials_per_image": (_I, [_I, _I, _I, _I, _I]),
    "iclr17_synthesis_deconv_igdn": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_synthesis_deconv3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P]),
    "iclr17_synthesis_deconv3_x6": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P]),
    "iclr17_synthesis_deconv3_x6_cm": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P]),
    "iclr17_synthesis_deconv3_x6_cm_bits": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I,
                                                 _P, _I, _P, _P, _D, _P]),
    "iclr17_synthesis_deconv3_bf16_bits": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I,
                                                _P, _I, _P, _P, _D, _P]),
    "iclr17_output_partials_per_image": (_I, [_I, _I]),
    "iclr17_split_planes": (_I, [_P, ctypes.c_long, _P, _P]),
    "iclr17_split_packed": (_I, [_P, _I, _I, _I, _P, _P]),
    "iclr17_analysis_conv1_gdn_x6": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv1x6_gdn": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv2_gdn_x6": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv3_quant_rate_x6": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P,
                                                 _P, _P, _P, _P]),
    "iclr17_analysis_conv3_quant_rate_x6w": (_I, [_P, _I, _I, _I, _I, _P, _P, _I, _P, _P, _P, _P,
                                                  _P, _P, _P, _P]),
    "iclr17_synthesis_deconv_igdn_x6": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                             _P]),
    "iclr17_synthesis_deconv_igdn_x6_cm": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                                _P]),
    "iclr17_reduce_partials": (_I, [_P, _I, _I, _P, _P, _D, _P]),
    "iclr17_resized_crop_batch": (_I, [_P, _P, _I, _I, _I, _P, _P, _P, _P]),
    "iclr17_adam_step": (_I, [_P, _I, ctypes.c_long, _D, _D, _D, _D, ctypes.c_long, _F, _P]),
    "iclr17_entropy_tables": (_I, [_P, _I, _I, _P, _P]),
    "iclr17_rans_capacity": (ctypes.c_long, [_I, _I, _I, _I]),
    "iclr17_rans_encode": (_I, [_P, _I, _I, _I, _I, _I, _P, _I, _P, ctypes.c_long, _P, _P, _P]),
    "iclr17_rans_offsets": (_I, [_P, _I, _P, _P]),
    "iclr17_rans_pack": (_I, [_P, ctypes.c_long, _P, _I, _P, _P]),
    "iclr17_rans_decode": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _I, _P, _P, _P]),
    "iclr17_ms_ssim_workspace_size": (_SZ, [_I, _I, _I]),
    "iclr17_ms_ssim": (_I, [_P, _P, _I, _I, _I, _F, _P, _SZ, _P, _P]),
    "iclr17_ssim_workspace_size": (_SZ, [_I, _I, _I]),
    "iclr17_ssim": (_I, [_P, _P, _I, _I, _I, _F, _P, _SZ, _P, _P, _P]),
    "iclr17_gdn": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P]),
    "iclr17_gdn_bwd": (_I, [_P, _P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_bitest_bwd_chunks": (_I, [_I64, _I]),
    "iclr17_bit_estimator_bwd": (_I, [_P, _P, _I64, _I, _I64, _P, _P, _P, _P]),
    "iclr17_bitparm_bwd": (_I, [_P, _P, _I64, _I, _I64, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_bit_estimator": (_I, [_P, _I64, _I, _I64, _P, _P, _P]),
    "iclr17_bitparm": (_I, [_P, _I64, _I, _I64, _P, _P, _P, _P, _P]),
    "iclr17_rate_bits": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_rate_bits_partials": (_I, [_I, _I, _I]),
    "iclr17_grad_recon": (_I, [_P, _P, _P, _P, _I64, _P, _P]),
    "iclr17_bwd_deconv3_igdn": (_I, [_P, _I, _I, _I, _I] + [_P] * 14),
    "iclr17_bwd_deconv_igdn": (_I, [_P, _P, _I, _I, _I, _I] + [_P] * 13),
    "iclr17_bwd_deconv_rate": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P, _P, _F, _P, _P, _P, _P]),
    "iclr17_rate_bwd_partials": (_I, [_I, _I]),
    "iclr17_bwd_conv_gdn": (_I, [_P, _P, _I, _I, _I, _I] + [_P] * 13),
    "iclr17_bwd_tiles": (_I, [_I, _I, _I]),
    "iclr17_sum_rows": (_I, [_P, _I, _I, _P, _P, _P]),
    "iclr17_sum_rows2": (_I, [_P, _P, _I, _I, _P, _P, _P, _P]),
    "iclr17_sum_rows_workspace_size": (_SZ, [_I]),
    "iclr17_wgrad_workspace_size": (_SZ, [_I, _I, _I, _I, _I, _I]),
    "iclr17_wgrad_k5": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_wgrad_k5_x6": (_I, [_P, _P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_wgrad_k9_x6": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_wgrad_k9": (_I, [_P, _P, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_gdn_wgrad_workspace_size": (_SZ, [ctypes.c_long, _I]),
    "iclr17_gdn_wgrad": (_I, [_P, _P, ctypes.c_long, _I, _P, _P, _P]),
    "iclr17_gdn_wgrad_x6_workspace_size": (_SZ, [ctypes.c_long, _I]),
    "iclr17_gdn_wgrad_x6": (_I, [_P, _P, ctypes.c_long, _I, _P, _P, _P]),
    "iclr17_gdn_param_chain": (_I, [_P, _P, _P, _P, _I, _F, _F, _P, _P, _P]),
    "iclr17_bias_grad_nhwc": (_I, [_P, ctypes.c_long, _I, _P, _P, _P]),
    "iclr17_bias_grad_nchw": (_I, [_P, _I, _I, ctypes.c_long, _P, _P, _P]),
    "iclr17_rate_param_grad": (_I, [_P, _I, _I] + [_P] * 7 + [_P] * 11 + [_P]),
    # h3 form, k5 layers on the 32x32x16 f16 MFMA (csrc/engine_h3.hip)
    "iclr17_h3k_weight_size": (_SZ, [_I, _I]),
    "iclr17_pack_h3k": (_I, [_I, _P, _P, _I, _P]),
    "iclr17_h3_planes": (_I, [_P, ctypes.c_long, _P, _P, _P]),
    "iclr17_h3_planes_cm": (_I, [_P, _I, _I, _I, _I, _I, _P, _P, _P]),
    "iclr17_split_packed_h3_size": (_SZ, [_I, _I, _I]),
    "iclr17_split_packed_h3": (_I, [_P, _I, _I, _I, _P, _P]),
    "iclr17_pack_h3_batch": (_I, [_P, _I, _P]),
    "iclr17_analysis_conv1_gdn_h3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "iclr17_analysis_conv2_gdn_h3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "iclr17_conv3_h3_partials_per_image": (_I, [_I, _I, _I, _I, _I]),
    "iclr17_analysis_conv3_quant_rate_h3": (_I, [_P, _I, _I, _I, _I, _P, _I, _P, _P, _P, _P, _P,
                                                 _P, _I, _P, _P, _P]),
    "iclr17_synthesis_deconv3_h3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _I,
                                         _P, _P, _D, _P, _P]),
    "iclr17_synthesis_deconv_igdn_h3": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P,
                                             _I, _I, _P, _P]),
    # bf16 throughput mode (csrc/engine_bf16.hip)
    "iclr17_bf16_weight_size": (_SZ, [_I, _I]),
    "iclr17_pack_bf16": (_I, [_I, _P, _P, _I, _P]),
    "iclr17_round_packed": (_I, [_P, _I, _I, _I, _P, _P]),
    "iclr17_to_bf16": (_I, [_P, ctypes.c_long, _P, _P]),
    "iclr17_analysis_conv1_gdn_bf16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "iclr17_analysis_conv2_gdn_bf16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "iclr17_bf16_rate_partials_per_image": (_I, [_I, _I, _I]),
    "iclr17_rate_table_size": (_SZ, [_I]),
    "iclr17_rate_table": (_I, [_P, _I, _P, _P]),
    "iclr17_analysis_conv3_quant_rate_bf16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _P]),
    "iclr17_synthesis_deconv_igdn_bf16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "iclr17_synthesis_deconv3_bf16": (_I, [_P, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P]),
}


class Iclr17Error(RuntimeError):
    pass


_lock = threading.Lock()
_lib = None


def load() -> ctypes.CDLL:
    """Load libiclr17.so once; raise if it is missing (no fallback exists)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise Iclr17Error(
                f"iclr17: HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` or `make -C "
                "iclr_17_compression_amd/csrc` (there is no CPU fallback)")
        lib = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def last_error() -> str:
    buf = ctypes.create_string_buffer(512)
    load().iclr17_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def call(name: str, *args) -> int:
    """Invoke an entry point; non-zero return → Iclr17Error with the library's message."""
    rc = getattr(load(), name)(*args)
    if rc != 0:
        raise Iclr17Error(last_error() or f"{name} failed with code {rc}")
    return rc


def query(name: str, *args):
    return getattr(load(), name)(*args)
