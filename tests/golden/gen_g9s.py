"""G8s / G9s: the REFERENCE's own disagreement with itself across CPU summation orders.

The reference computes in fp32 on whatever conv kernels torch picks on the host. Its ŷ = round(y)
and its bpp / PSNR / MS-SSIM therefore depend on the summation order of those kernels: an
element of y that lies within fp32 accumulation noise of k + ½ rounds either way. This script
measures that floor on the G8 / G9 operating points (24 Kodak-synth images, weights trained to
λ = 0.01·255²) by running the reference (model.py:46-80, imported from /root/reference exactly as
gen_goldens.py does) under several summation orders of its own:

    default      oneDNN (AVX-512 kernels on this host) — the order the G8 / G9 fixtures hold
    mkldnn_off   torch.backends.mkldnn.flags(enabled=False): ATen's native conv (im2col + MKL
                 sgemm for conv2d, slow_conv_transpose2d for the deconvs)
    onednn_avx2  oneDNN restricted to AVX2 kernels (child process, ONEDNN_MAX_CPU_ISA=AVX2)
    native_avx2  ATen's native conv with MKL restricted to AVX2 (child process,
                 MKL_ENABLE_INSTRUCTIONS=AVX2, mkldnn off)
    fp64         the same modules in float64 (the exact-arithmetic value the fp32 orders
                 approximate; reported, not one of the reference's fp32 orders)

and writes, per image and per order, the latent flip count against the default order and the
raw relative Δbpp, ΔPSNR and ΔMS-SSIM, plus the distance of every flipped y from its rounding
boundary, and per fp32 order the number of latents it rounds differently from the float64 run. Only these numbers are committed (tests/golden/g9s_*.json); they are data, not
reference source. tests/test_gpu_operating_point.py holds the GPU to this floor.

    python tests/golden/gen_g9s.py [--sets g8,g9] [--orders ...]
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_goldens as gg  # noqa: E402  (import_reference, run_reference_eval, KODAK_PORTRAIT)

from iclr_17_compression_amd import synth  # noqa: E402

SETS = {"g8": ("g8_kodak24_synth_n128_trained.json", "g8s_reference_orders_n128.json"),
        "g9": ("g9_kodak24_synth_n192_trained.json", "g9s_reference_orders_n192.json")}
CHILD_ENV = {"onednn_avx2": {"ONEDNN_MAX_CPU_ISA": "AVX2"},
             "native_avx2": {"MKL_ENABLE_INSTRUCTIONS": "AVX2"}}
MKLDNN_OFF = ("mkldnn_off", "native_avx2")
ORDERS = ("default", "mkldnn_off", "onednn_avx2", "native_avx2", "fp64")


def run_order(set_name: str, order: str, ref_root: str) -> dict:
    """Per image: ŷ (int8), y, bpp, PSNR, MS-SSIM of the reference under `order` (this process)."""
    fixture = SETS[set_name][0]
    meta = json.load(open(os.path.join(HERE, fixture)))
    ref_model, ref_models = gg.import_reference(ref_root)
    sd = gg.trained_weights(meta["weights"])
    net = ref_model.ImageCompressor(out_channel_N=meta["N"])
    net.load_state_dict(sd)
    dt = torch.float64 if order == "fp64" else torch.float32
    net = net.to(dt).eval()
    out = {"y_hat": [], "y": [], "bpp": [], "psnr": [], "ms_ssim": []}
    ctx = torch.backends.mkldnn.flags(enabled=order not in MKLDNN_OFF)
    with ctx:
        for row in meta["images"]:
            x = torch.from_numpy(synth.to_unit_float(synth.smooth_image_u8(
                meta["image_seed_base"] + row["index"], row["height"], row["width"])))[None].to(dt)
            clipped, y_hat, bpp, recon, y = gg.run_reference_eval(net, x)
            mse = torch.mean((clipped - x).pow(2))
            psnr = 10 * (torch.log(1.0 / mse) / np.log(10))
            msssim = ref_models.ms_ssim(clipped.float(), x.float(), data_range=1.0,
                                        size_average=True)
            out["y_hat"].append(y_hat.numpy().astype(np.int8))
            out["y"].append(y.numpy().astype(np.float64))
            for k, v in (("bpp", bpp), ("psnr", psnr), ("ms_ssim", msssim)):
                out[k].append(float(v.item()))
            print(f"{set_name} {order} image {row['index']}: bpp {out['bpp'][-1]:.8f} "
                  f"psnr {out['psnr'][-1]:.6f}", file=sys.stderr, flush=True)
    return out


def child(set_name: str, order: str, ref_root: str, path: str):
    r = run_order(set_name, order, ref_root)
    np.savez(path, **{f"{k}_{i}": v for k in ("y_hat", "y") for i, v in enumerate(r[k])},
             **{k: np.array(r[k]) for k in ("bpp", "psnr", "ms_ssim")})


def load_child(path: str, n: int) -> dict:
    d = np.load(path, allow_pickle=False)
    return {"y_hat": [d[f"y_hat_{i}"] for i in range(n)], "y": [d[f"y_{i}"] for i in range(n)],
            **{k: list(d[k]) for k in ("bpp", "psnr", "ms_ssim")}}


def summarise(set_name: str, runs: dict) -> dict:
    fixture, _ = SETS[set_name]
    meta = json.load(open(os.path.join(HERE, fixture)))
    base = runs["default"]
    rows = []
    for i, row in enumerate(meta["images"]):
        # the default order must be the fixture's own numbers
        assert base["bpp"][i] == row["bpp"] and base["psnr"][i] == row["psnr"], (i, base["bpp"][i], row["bpp"])
        r = {"index": row["index"], "orders": {}}
        for o, run in runs.items():
            if o == "default":
                continue
            diff = run["y_hat"][i] != base["y_hat"][i]
            yb = base["y"][i][diff]
            r["orders"][o] = {
                "latent_flips": int(diff.sum()),
                "flip_dist_to_half_max": float(np.abs(yb - (np.floor(yb) + 0.5)).max()) if diff.any() else None,
                "max_abs_dy": float(np.abs(run["y"][i] - base["y"][i]).max()),
                "rel_dbpp": abs(run["bpp"][i] - base["bpp"][i]) / abs(base["bpp"][i]),
                "rel_dpsnr": abs(run["psnr"][i] - base["psnr"][i]) / abs(base["psnr"][i]),
                "rel_dms_ssim": abs(run["ms_ssim"][i] - base["ms_ssim"][i]) / abs(base["ms_ssim"][i]),
            }
        fp32 = [v for o, v in r["orders"].items() if o != "fp64"]
        r["fp32_spread"] = {k: max(v[k] for v in fp32) for k in
                            ("latent_flips", "rel_dbpp", "rel_dpsnr", "rel_dms_ssim", "max_abs_dy")}
        rows.append(r)
    total = {o: sum(r["orders"][o]["latent_flips"] for r in rows) for o in rows[0]["orders"]}
    fp32_orders = [o for o in rows[0]["orders"] if o != "fp64"]
    # each fp32 order's latents rounded differently from the float64 run (the exact value the
    # orders approximate): how many latents the reference itself rounds "wrong", order by order
    wrong = ({o: int(sum(int((runs[o]["y_hat"][i] != runs["fp64"]["y_hat"][i]).sum())
                         for i in range(len(rows)))) for o in ["default"] + fp32_orders}
             if "fp64" in runs else {})
    return {
        "note": ("the reference (model.py:46-80) under several CPU summation orders of its own, "
                 "each compared with the default (oneDNN) order the fixture holds; generated by "
                 "tests/golden/gen_g9s.py"),
        "fixture": fixture, "N": meta["N"], "orders": list(runs),
        "latents_per_set": int(sum(v.size for v in base["y_hat"])),
        "total_flips_vs_default": total,
        "total_wrong_vs_fp64": wrong,
        "max_wrong_vs_fp64_fp32": max(wrong.values()) if wrong else None,
        "max_images_with_flips_fp32": max(sum(1 for r in rows if r["orders"][o]["latent_flips"])
                                          for o in fp32_orders),
        "set_spread_fp32": {k: max(r["fp32_spread"][k] for r in rows) for k in
                            ("latent_flips", "rel_dbpp", "rel_dpsnr", "rel_dms_ssim", "max_abs_dy")},
        "images": rows,
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reference", default="/root/reference")
    ap.add_argument("--sets", default="g9,g8")
    ap.add_argument("--orders", default=",".join(ORDERS))
    ap.add_argument("--child", default="")
    ap.add_argument("--child-set", default="")
    ap.add_argument("--child-out", default="")
    args = ap.parse_args()
    torch.set_num_threads(os.cpu_count() or 1)
    if args.child:
        child(args.child_set, args.child, args.reference, args.child_out)
        return
    orders = args.orders.split(",")
    assert orders[0] == "default"
    for s in args.sets.split(","):
        runs = {}
        n = len(json.load(open(os.path.join(HERE, SETS[s][0])))["images"])
        for o in orders:
            if o in CHILD_ENV:
                with tempfile.TemporaryDirectory() as td:
                    path = os.path.join(td, "run.npz")
                    env = {**os.environ, **CHILD_ENV[o]}
                    subprocess.run([sys.executable, os.path.abspath(__file__), "--reference",
                                    args.reference, "--child", o, "--child-set", s,
                                    "--child-out", path], env=env, check=True)
                    runs[o] = load_child(path, n)
            else:
                runs[o] = run_order(s, o, args.reference)
        res = summarise(s, runs)
        with open(os.path.join(HERE, SETS[s][1]), "w") as f:
            json.dump(res, f, indent=1)
        print(s, json.dumps({k: res[k] for k in ("total_flips_vs_default", "set_spread_fp32",
                                                  "max_images_with_flips_fp32")}))


if __name__ == "__main__":
    main()
