"""The multi-process paths (world_size 2 and 8, gloo on CPU): batch sharding, the per-image gather,
bucketed gradient averaging and max-over-ranks timing — the same functions the RCCL runs use."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from iclr_17_compression_amd import dist as idist


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(r, w, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(r), WORLD_SIZE=str(w))
    dist.init_process_group("gloo", rank=r, world_size=w)
    try:
        # sharding covers the batch exactly once, in order
        x = torch.arange(7 * 3, dtype=torch.float32).view(7, 3)
        mine = idist.shard_batch(x)
        full = idist.gather_rows(mine * 2, 7)
        assert torch.equal(full, x * 2)
        # bucketed gradient averaging == mean of the per-rank gradients
        torch.manual_seed(0)
        params = [torch.nn.Parameter(torch.zeros(s)) for s in (5, 300, 7, 1000, 3)]
        for i, p in enumerate(params):
            p.grad = torch.full(p.shape, float(r + 1) * (i + 1))
        idist.allreduce_grads(params, bucket_mb=0.002)
        for i, p in enumerate(params):
            expect = (i + 1) * (1 + w) / 2.0
            assert torch.allclose(p.grad, torch.full(p.shape, expect))
        assert idist.max_over_ranks(float(r), "cpu") == float(w - 1)
        # the overlapped reducer: groups launched as a backward would (decoder first), one
        # parameter left for finish(), a bucket size that splits groups
        ps = [torch.nn.Parameter(torch.zeros(s)) for s in (40, 3000, 9, 700, 5)]
        for i, p in enumerate(ps):
            p.grad = torch.full(p.shape, float(r + 1) * (i + 2)) + torch.arange(p.numel()) * r
        red = idist.GradAllReducer(ps, bucket_mb=0.005)
        assert red.active
        red.launch(ps[2:4], [p.grad for p in ps[2:4]])
        red.launch(ps[0:2], [p.grad for p in ps[0:2]])
        red.launch(ps[2:3], [ps[2].grad])   # already in flight: not reduced twice
        red.finish()
        for i, p in enumerate(ps):
            expect = (i + 2) * (1 + w) / 2.0 + torch.arange(p.numel()) * (w - 1) / 2.0
            assert torch.allclose(p.grad, expect), i
        assert not red.pending and not red.launched
        q.put((r, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        q.put((r, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("w", [2, 8])   # 8: the rank count of BASELINE C4 / the 8-GPU bench
def test_multi_rank_gloo(w):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, w, port, q)) for r in range(w)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(w))
    for p in ps:
        p.join(timeout=60)
    assert res == {r: "ok" for r in range(w)}, res


def test_shard_range_balanced():
    for n in (0, 1, 7, 64, 65):
        for w in (1, 2, 3, 8):
            spans = [idist.shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [hi - lo for lo, hi in spans]
            assert max(sizes) - min(sizes) <= 1


def test_buckets_respect_size_and_order():
    ps = [torch.zeros(n) for n in (10, 20, 30, 5, 1000, 1)]
    bs = idist.bucketize(ps, 25 * 4)
    assert [p for b in bs for p in b] == ps
    assert all(sum(p.numel() for p in b) <= 25 or len(b) == 1 for b in bs)
