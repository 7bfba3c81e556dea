"""Host logic of bench.py (no GPU): the roofline's HBM traffic is taken only from a PMC summary of
the library build that runs (tools/profile_round.sh stamps the SHA-256 of libiclr17.so), for the
same precision and workload; anything else gives traffic = null with the reason. And the CPU
baseline's thread count."""
import json
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def _write(tmp_path, name, sha, prec="x6", workload=None, layer="deconv2_igdn2"):
    d = tmp_path / "profiles"
    d.mkdir(exist_ok=True)
    (d / name).write_text(json.dumps({
        "lib_sha256": sha, "precision": prec,
        "workload": workload or {"N": 192, "S": 256, "B": 64},
        "layers": {layer: {"kernel": "k", "traffic_bytes": 123.0, "mean_ms": 0.1}}}))


def test_traffic_only_from_this_build(tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    sha = bench.lib_sha()
    _write(tmp_path, "r01_traffic.json", "0" * 16)
    t, why, ms = bench.pmc_traffic("deconv2_igdn2", 192, 256, 64, "x6")
    assert t is None and ms is None and sha in why and "r01_traffic.json" in why
    _write(tmp_path, "r02_traffic.json", sha)
    t, src, ms = bench.pmc_traffic("deconv2_igdn2", 192, 256, 64, "x6")
    assert t == 123.0 and ms == 0.1 and "r02_traffic.json" in src
    # another precision, workload or layer of the same build does not count
    assert bench.pmc_traffic("deconv2_igdn2", 192, 256, 64, "bf16")[0] is None
    assert bench.pmc_traffic("deconv2_igdn2", 192, 256, 32, "x6")[0] is None
    assert bench.pmc_traffic("conv2_gdn2", 192, 256, 64, "x6")[0] is None


def test_cpu_threads(monkeypatch):
    aff = len(os.sched_getaffinity(0))
    monkeypatch.delenv("OMP_NUM_THREADS", raising=False)
    assert bench.cpu_threads() == (aff, aff)
    monkeypatch.setenv("OMP_NUM_THREADS", "1")
    assert bench.cpu_threads() == (1, aff)


@pytest.mark.parametrize("prec,kernel_peak", [("bf16", bench.BF16_MFMA_PEAK_TFLOPS),
                                              ("x6", bench.X6_PEAK_TFLOPS)])
def test_roofline_object(prec, kernel_peak, tmp_path, monkeypatch):
    monkeypatch.setattr(bench, "REPO", str(tmp_path))   # no PMC summaries
    ms = {k: 0.1 for k in bench.LAYERS}
    ms["deconv2_igdn2"] = 0.2
    dom, layers, roof = bench.roofline(ms, prec, 192, 256, 64)
    assert dom == "deconv2_igdn2" and roof["peak"] == round(kernel_peak, 1)
    flops = bench.layer_flops(192, 256, 256)["deconv2_igdn2"] * 64
    assert roof["achieved"] == pytest.approx(flops / 0.2e-3 / 1e12, rel=1e-3)
    assert roof["frac"] == pytest.approx(roof["achieved"] / kernel_peak, rel=1e-3)
    assert roof["traffic"] is None and roof["traffic_null_reason"]
    assert roof["duration"].startswith("hip_events")
    assert roof["frac_of_bf16_dense_peak"] == pytest.approx(roof["achieved"] / bench.BF16_MFMA_PEAK_TFLOPS, rel=1e-3)
    assert "frac_from_profile" not in roof


def test_chain_roofline(tmp_path, monkeypatch):
    """per-layer T_roof = max(F / P_peak, bytes / 8 TB/s) and the chain's
    Σ T_roof / Σ T; in the bf16 mode activations are 2 bytes, which makes conv1 and deconv3
    HBM-bound; at measured times equal to T_roof the chain fraction is 1."""
    monkeypatch.setattr(bench, "REPO", str(tmp_path))
    N, S, B = 192, 256, 64
    fl = bench.layer_flops(N, S, S)
    for prec, act, peak in (("x6", 4, bench.X6_PEAK_TFLOPS), ("bf16", 2, bench.BF16_MFMA_PEAK_TFLOPS)):
        by = bench.layer_bytes(N, S, S, act)
        roof_ms = {k: max(fl[k] * B / (peak * 1e12), by[k] * B / (bench.HBM_PEAK_GBS * 1e9)) * 1e3
                   if fl[k] else 0.01 for k in bench.LAYERS}
        _, layers, roof = bench.roofline(roof_ms, prec, N, S, B)
        assert roof["chain_roofline_frac"] == pytest.approx(1.0, rel=1e-3)
        _, layers2, roof2 = bench.roofline({k: 2 * v for k, v in roof_ms.items()}, prec, N, S, B)
        assert roof2["chain_roofline_frac"] == pytest.approx(0.5, rel=1e-3)
        bounds = {k: v.get("roof_bound") for k, v in layers.items() if fl[k]}
        if prec == "x6":
            assert set(bounds.values()) == {"mfma"}
        else:
            assert bounds["conv1_gdn1"] == "hbm" and bounds["deconv3_clamp"] == "hbm"
            assert bounds["conv2_gdn2"] == "mfma" and bounds["deconv2_igdn2"] == "mfma"


def _run_bench(args, env_extra, timeout=240):
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra)
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return subprocess.run([sys.executable, os.path.join(repo, "bench.py"), *args], env=env,
                          capture_output=True, text=True, timeout=timeout)


@pytest.mark.parametrize("n", [1, 2])
def test_launcher_spawns_ranks(n):
    """`python bench.py --gpus N` without torchrun starts N ranks itself (here over gloo, no GPU:
    --dry-run runs the launch, rendezvous, barrier and max-over-ranks only)."""
    r = _run_bench(["--gpus", str(n), "--dry-run"], {"ICLR17_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["global_batch"] == 64 * n and d["scaling"] == "weak"
    assert len(d["rank_devices"]) == n
    assert d["dist_backend"] == ("gloo" if n > 1 else None)


def test_dry_run_default_backend_without_gpu():
    """--dry-run with the default backend (RCCL) on a host without a GPU falls back to gloo, as
    its help promises, instead of failing in init_process_group("nccl", device_id=cpu)."""
    import torch
    if torch.cuda.device_count():
        pytest.skip("host has a GPU: the default backend is RCCL there")
    r = _run_bench(["--gpus", "2", "--dry-run"], {"ICLR17_DIST_BACKEND": "nccl"})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["n_gpus"] == 2 and d["dist_backend"] == "gloo"


def test_launcher_strong_scaling_and_errors():
    r = _run_bench(["--gpus", "2", "--dry-run", "--global-batch", "64"], {"ICLR17_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert d["batch_per_gpu"] == 32 and d["global_batch"] == 64 and d["scaling"] == "strong"
    # an odd global batch over 2 ranks, and more GPUs than the host has (RCCL), both fail loudly
    assert _run_bench(["--gpus", "2", "--dry-run", "--global-batch", "63"],
                      {"ICLR17_DIST_BACKEND": "gloo"}).returncode != 0
    assert _run_bench(["--gpus", "4096"], {}).returncode != 0
    # under torchrun, --gpus must equal WORLD_SIZE
    r = _run_bench(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0",
                                                  "ICLR17_DIST_BACKEND": "gloo"})
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_kodak_rank_images_partition():
    """C2 at N GPUs: every Kodak image on exactly one rank, landscape and portrait batches apart,
    at most 3 images per rank at 8 ranks."""
    for w in range(1, 9):
        seen = []
        for r in range(w):
            land, port = bench.kodak_rank_images(r, w)
            assert not set(land) & set(bench.KODAK_PORTRAIT)
            assert set(port) <= set(bench.KODAK_PORTRAIT)
            seen += land + port
            if w == 8:
                assert len(land) + len(port) == 3
        assert sorted(seen) == list(range(24))


def _kodak_worker(r, w, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(w))
    dist.init_process_group("gloo", rank=r, world_size=w)
    try:
        land, port_ = bench.kodak_rank_images(r, w)
        rows = {i: [0.25 + i, 30.0 - i / 7, 0.9 + i / 1000, float(i % 3)] for i in land + port_}
        t = bench.kodak_table(rows, 4, "cpu")
        import numpy as np
        expect = np.array([[0.25 + i, 30.0 - i / 7, 0.9 + i / 1000, float(i % 3)] for i in range(24)])
        q.put((r, bool(np.array_equal(t, expect))))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((r, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("w", [2, 8])
def test_kodak_sharded_table_gloo(w):
    """The sharded Kodak path's per-image table (bench.kodak_table) over gloo ranks: every rank
    ends with the full 24-row table, bit for bit what one rank would hold."""
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_kodak_worker, args=(r, w, port, q)) for r in range(w)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(w))
    for p in ps:
        p.join(timeout=60)
    assert all(v is True for v in res.values()), res
