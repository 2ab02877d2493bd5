"""Data-parallel logic on CPU with torch.distributed gloo, world_size 2 (no GPU):
gradient buckets (reverse layer order, launched during backward), averaging, parameter
broadcast; and the SyncBN statistics recipe (all-reduced per-channel sums) reproducing
single-process batch norm on the concatenated batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dorknet_amd.parallel import DataParallel, plan_buckets
from oracle import ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class FakeLayer:
    """Stands in for a layer: backward() writes rank-dependent gradients in place."""

    def __init__(self, name, shapes, idx):
        self.layer_name = name
        self.idx = idx
        self.learned_params = {k: torch.full(s, float(idx)) for k, s in shapes.items()}
        self.grads = {k: torch.zeros(s) for k, s in shapes.items()}
        self.non_learned_params = None

    def backward(self, dy):
        r = dist.get_rank()
        for k, g in self.grads.items():
            g.copy_(torch.arange(g.numel(), dtype=torch.float32).view(g.shape) * (r + 1) + self.idx)
        return dy


class FakeLoss:
    def backward(self):
        return None


class FakeNet:
    def __init__(self):
        self.layers = [FakeLayer("l%d" % i, {"weights": (i + 1, 50), "bias": (i + 1,)}, i) for i in range(6)]
        self.loss_layer = FakeLoss()
        self._steps = [(l,) for l in self.layers]


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        net = FakeNet()
        if rank == 1:  # diverge, then broadcast from rank 0
            for l in net.layers:
                l.learned_params["weights"].add_(100.0)
        dp = DataParallel(net, bucket_bytes=1000, device=torch.device("cpu"))
        dp.broadcast_parameters(0)
        for i, l in enumerate(net.layers):
            assert torch.all(l.learned_params["weights"] == float(i))
        order = []
        orig = dp._launch
        dp._launch = lambda lo, hi: (order.append(lo), orig(lo, hi))
        dp.backward()
        # buckets are contiguous ranges laid out in reverse layer order -> launched lo ascending
        assert order == sorted(order) and len(order) == len(dp.buckets) > 1
        for l in net.layers:
            for k, g in l.grads.items():
                base = torch.arange(g.numel(), dtype=torch.float32).view(g.shape)
                want = base * (1 + 2) / 2.0 + l.idx          # mean over ranks of base*(r+1)+idx
                assert torch.allclose(g, want), (l.layer_name, k)
                assert g.data_ptr() >= dp.flat.data_ptr()    # gradients live in the flat buffer
        # SyncBN recipe: per-rank fp64 sums all-reduced == full-batch statistics
        rng = np.random.default_rng(0)
        full = (2.0 + 3.0 * rng.standard_normal((8, 4, 3, 3))).astype(np.float64)
        mine = full[rank * 4:(rank + 1) * 4]
        sums = torch.tensor(np.concatenate([mine.sum(axis=(0, 2, 3)), (mine ** 2).sum(axis=(0, 2, 3))]))
        dist.all_reduce(sums)
        count = mine.shape[0] * 9 * world
        mean = sums[:4].numpy() / count
        var = sums[4:].numpy() / count - mean ** 2
        assert np.allclose(mean, full.mean(axis=(0, 2, 3))) and np.allclose(var, full.var(axis=(0, 2, 3)))
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
        raise


def test_data_parallel_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert results == {0: "ok", 1: "ok"}, results


def test_bucket_plan_reverse_order():
    numels = [10, 300, 20, 500, 40]
    owners = [0, 1, 1, 2, 3]
    b = plan_buckets(numels, owners, bucket_bytes=4 * 400)
    assert [sorted(x[0]) for x in b] == [[3, 4], [0, 1, 2]]
    assert [x[1] for x in b] == [2, 0]      # ready once backward has passed top-level layer 2, then 0


def test_syncbn_backward_recipe_matches_full_batch():
    """dgamma/dbeta from *local* sums (then averaged like every other gradient) and the dx
    coefficients from *global* sums reproduce single-process BN backward on the
    concatenated batch, given the reference's per-rank 1/N_local loss scaling."""
    rng = np.random.default_rng(1)
    world, n = 2, 3
    X = 1.0 + rng.standard_normal((world * n, 5, 4, 4))
    G = rng.standard_normal((world * n, 5, 4, 4))        # dL/dy of the *full* batch loss
    g = (1 + 0.1 * rng.standard_normal((1, 5, 1, 1)))
    b = 0.1 * rng.standard_normal((1, 5, 1, 1))
    Y, cache, _, _ = ref.bn_forward_train(X, g, b, None, None)
    dX_full, dg_full, db_full = ref.bn_backward(G, g, cache)
    mean = X.mean(axis=(0, 2, 3), keepdims=True)
    std = np.sqrt(X.var(axis=(0, 2, 3), keepdims=True) + 1e-5)
    M = X.shape[0] * 16
    dg_avg, db_avg = 0, 0
    sums_g = [0, 0]
    for r in range(world):  # per-rank upstream grads carry 1/n instead of 1/(world*n): x world
        xr, gr = X[r * n:(r + 1) * n], world * G[r * n:(r + 1) * n]
        xh = (xr - mean) / std
        sums_g[0] += gr.sum(axis=(0, 2, 3), keepdims=True)
        sums_g[1] += (gr * xh).sum(axis=(0, 2, 3), keepdims=True)
        dg_avg = dg_avg + (gr * xh).sum(axis=(0, 2, 3), keepdims=True) / world
        db_avg = db_avg + gr.sum(axis=(0, 2, 3), keepdims=True) / world
    for r in range(world):
        xr, gr = X[r * n:(r + 1) * n], world * G[r * n:(r + 1) * n]
        xh = (xr - mean) / std
        dxr = g / std * (gr - sums_g[0] / M - xh * sums_g[1] / M)
        assert np.allclose(dxr / world, dX_full[r * n:(r + 1) * n])
    assert np.allclose(dg_avg, dg_full) and np.allclose(db_avg, db_full)
