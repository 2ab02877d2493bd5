"""The real data-parallel path (dorknet_amd.parallel.DataParallel + BatchNormLayer SyncBN) on
the GPU (BASELINE config 4's code path at a size one box runs).

* world 1 over RCCL: SyncBN (per-channel sums all-reduced between the partial and finalize
  stages) equals local BN up to the fp64 fold order; the default DataParallel leaves the skip
  projections' gradients out of the buckets (SGDMomentum never applies them,
  optimisers/SGDMomentum.py:7-14);
* stream ordering: every bucket's all-reduce sees the gradients the main stream
  writes (BatchNorm dgamma/dbeta) even when the main stream lags far behind;
* world 2 over gloo, both ranks on cuda:0, freshly spawned: one ResNet-18-depsep training step
  with SyncBN, each rank on half the batch, equals the oracle (fp64 restatement of the
  reference) on the concatenated batch within SURVEY.md 8c's 1e-4 normwise -- the reference's
  per-rank 1/N_local loss gradient (layers/losses.py:34) averaged over ranks is the full-batch
  gradient, and SyncBN normalises with whole-batch statistics (layers/batch_norm.py:67-68).
"""
import os
import socket

import numpy as np
import pytest
import torch

from tests._convert import all_layers, network_to_oracle, rel_err, slack_bound

pytestmark = pytest.mark.gpu

SEED_W, SEED_X = 21, 22


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _grads(net):
    return {(l.layer_name, k): l.grads[k].detach().float().cpu().numpy()
            for l in all_layers(net.layers) for k in sorted(l.grads or {})}


def _excess(got, want64, want32, tol=1e-4):
    got = np.asarray(got, dtype=np.float64)
    err = np.linalg.norm((got - want64).ravel())
    bound = slack_bound(want64, want32, tol)
    return 0.0 if err == 0 else err / max(bound, 1e-300)


def _rccl_world1():
    import torch.distributed as dist
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _port(), rank=0, world_size=1)


def test_syncbn_world1_matches_local_bn():
    import torch.distributed as dist
    from dorknet_amd.parallel import DataParallel
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    _rccl_world1()
    try:
        X, _, onehot = synthetic_batch(4, seed=SEED_X)
        res = {}
        for mode in ("local", "sync"):
            np.random.seed(SEED_W)
            net = ResNet18("r18")
            net.to_gpu()
            dp = DataParallel(net, batch_norm=mode, bucket_bytes=1 << 20)
            loss, P = net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
            dp.backward()
            torch.cuda.synchronize()
            res[mode] = (float(loss), P.cpu().numpy(), _grads(net),
                         {l.layer_name: l.non_learned_params["running_std"].cpu().numpy()
                          for l in all_layers(net.layers) if getattr(l, "non_learned_params", None)})
            skip_ptrs = [l.skip_projection.grads["weights"].data_ptr() for l in net.layers
                         if getattr(l, "skip_projection", None) is not None]
            lo, hi = dp.flat.data_ptr(), dp.flat.data_ptr() + 4 * dp.flat.numel()
            assert len(skip_ptrs) == 3 and not any(lo <= p < hi for p in skip_ptrs)
        (l0, p0, g0, s0), (l1, p1, g1, s1) = res["local"], res["sync"]
        assert abs(l0 - l1) <= 1e-6 * abs(l0)
        assert rel_err(p1, p0) <= 1e-6
        for k in g0:
            assert np.linalg.norm(g1[k] - g0[k]) <= 1e-5 * np.linalg.norm(g0[k]) + 1e-12, k
        for k in s0:
            assert rel_err(s1[k], s0[k]) <= 1e-6, k
    finally:
        dist.destroy_process_group()


def test_bucket_allreduce_waits_for_main_stream(monkeypatch):
    """Every bucket handed to the collective must already hold the gradients written on the
    main stream.  The main stream is held back (a device-side spin) right before each BatchNorm
    writes dgamma/dbeta; the collective is wrapped to snapshot what it is given, on the stream
    it is issued from; the buffer starts as NaN.  World size 1 averages nothing, so every
    snapshot must equal the final gradients."""
    import torch.distributed as dist
    from dorknet_amd import _hip
    from dorknet_amd.parallel import DataParallel
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    _rccl_world1()
    try:
        X, _, onehot = synthetic_batch(2, seed=SEED_X)
        np.random.seed(SEED_W)
        net = ResNet18("r18")
        net.to_gpu()
        dp = DataParallel(net, bucket_bytes=256 << 10)
        net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
        dp.flat.fill_(float("nan"))
        orig_bn = _hip.lib.dk_bn_bwd_from_partials_f32

        def slow_bn(*args):
            torch.cuda._sleep(20_000_000)  # ~10 ms of spinning on the current (main) stream
            return orig_bn(*args)
        monkeypatch.setattr(_hip.lib, "dk_bn_bwd_from_partials_f32", slow_bn)
        snaps = []
        real = dist.all_reduce

        def spy(t, *a, **k):
            snaps.append((t, t.clone()))
            return real(t, *a, **k)
        monkeypatch.setattr(dist, "all_reduce", spy)
        dp.backward()
        torch.cuda.synchronize()
        assert len(snaps) == len(dp.buckets) > 3
        for t, snap in snaps:
            assert not torch.isnan(snap).any()
            assert torch.equal(snap, t)
    finally:
        dist.destroy_process_group()


def test_bucket_allreduce_waits_for_branch_stream(monkeypatch):
    """with side-stream weight gradients off (DORKNET_ASYNC_WGRAD=0), the skip
    projections' backward -- weight gradient included -- runs on the branch stream
    (residual_block.py), and update_skip_projections=True puts those gradients in the buckets.
    The branch stream is held back (a device-side spin) right before each skip projection's
    weight gradient; every bucket the collective is given, snapshotted on the stream it is issued
    from, must already hold the final gradients (the buffer starts as NaN)."""
    import torch.distributed as dist
    from dorknet_amd import _hip
    from dorknet_amd.parallel import DataParallel
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    monkeypatch.setenv("DORKNET_ASYNC_WGRAD", "0")
    monkeypatch.setenv("DORKNET_BRANCH_STREAM", "1")
    _rccl_world1()
    try:
        X, _, onehot = synthetic_batch(2, seed=SEED_X)
        np.random.seed(SEED_W)
        net = ResNet18("r18")
        net.to_gpu()
        dp = DataParallel(net, bucket_bytes=256 << 10, update_skip_projections=True)
        net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
        dp.flat.fill_(float("nan"))
        orig = _hip.lib.dk_pwconv_wgrad_f32
        calls = []

        def slow_wgrad(*args):
            calls.append(torch.cuda.current_stream() == _hip.branch_stream())
            torch.cuda._sleep(20_000_000)  # ~10 ms of spinning on the current (branch) stream
            return orig(*args)
        monkeypatch.setattr(_hip.lib, "dk_pwconv_wgrad_f32", slow_wgrad)
        snaps = []
        real = dist.all_reduce

        def spy(t, *a, **k):
            snaps.append((t, t.clone()))
            return real(t, *a, **k)
        monkeypatch.setattr(dist, "all_reduce", spy)
        dp.backward()
        torch.cuda.synchronize()
        # the three skip projections' weight gradients ran on the branch stream
        assert calls == [True, True, True], calls
        assert len(snaps) == len(dp.buckets) > 3
        for t, snap in snaps:
            assert not torch.isnan(snap).any()
            assert torch.equal(snap, t)
    finally:
        dist.destroy_process_group()


def test_bucket_launch_order_rccl_world1():
    """RCCL world 1: the order in which gradient buckets go to the collective against the order in
    which layers finish backward.  Each bucket is launched as soon as every leaf layer it covers
    has been through backward -- so inside a residual block, before the block's first layer is
    done -- and the buckets go out in flat-buffer order (reverse layer order)."""
    import torch.distributed as dist
    from dorknet_amd.layers._chain import backward_progress
    from dorknet_amd.parallel import DataParallel
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    _rccl_world1()
    try:
        X, _, onehot = synthetic_batch(2, seed=SEED_X)
        np.random.seed(SEED_W)
        net = ResNet18("r18")
        net.to_gpu()
        dp = DataParallel(net, bucket_bytes=64 << 10)
        net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
        events = []  # ("done", layer names) / ("launch", lo)
        orig = dp._launch

        def launch(lo, hi):
            events.append(("launch", lo))
            orig(lo, hi)
        dp._launch = launch
        with backward_progress(lambda layers: events.append(("done", tuple(l.layer_name for l in layers)))):
            dp.backward()
        torch.cuda.synchronize()
        launches = [e[1] for e in events if e[0] == "launch"]
        assert launches == sorted(launches) and len(launches) == len(dp.buckets) > 8
        # a bucket launched before the first layer of res8's chain finished backward holds only
        # gradients of layers already reported done
        first_res8 = next(i for i, e in enumerate(events) if e[0] == "done" and e[1][0] == "res8_dw1_dw")
        early = [i for i, e in enumerate(events) if e[0] == "launch" and i < first_res8]
        assert early, "no bucket went out while res8's backward was still running"
        done_before = set()
        for i, e in enumerate(events):
            if e[0] == "done":
                done_before.update(e[1])
        names = {id(l): l.layer_name for l in all_layers(net.layers)}
        for bi, (lo, hi, _, owners) in enumerate(dp.buckets):
            li = next(i for i, e in enumerate(events) if e == ("launch", lo))
            seen = set()
            for e in events[:li]:
                if e[0] == "done":
                    seen.update(e[1])
            assert {names[o] for o in owners} <= seen, (bi, {names[o] for o in owners} - seen)
    finally:
        dist.destroy_process_group()


def _gloo_rank(rank, world, port, outdir, q, env=None):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ.update(env or {})
        import torch.distributed as dist
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from dorknet_amd.parallel import DataParallel
        from examples.resnet18_depsep import ResNet18, synthetic_batch
        X, _, onehot = synthetic_batch(2 * world, seed=SEED_X)
        np.random.seed(SEED_W)
        net = ResNet18("r18")
        net.to_gpu()
        dp = DataParallel(net, batch_norm="sync", bucket_bytes=512 << 10, update_skip_projections=True)
        sl = slice(2 * rank, 2 * rank + 2)
        loss, _ = net.forward(torch.as_tensor(X[sl], device="cuda"), torch.as_tensor(onehot[sl], device="cuda"))
        dp.backward()
        torch.cuda.synchronize()
        g = _grads(net)
        out = {"loss": np.array(float(loss))}
        for (name, k), v in g.items():
            out["g|{}|{}".format(name, k)] = v
        for l in all_layers(net.layers):
            nlp = getattr(l, "non_learned_params", None)
            if nlp and nlp.get("running_std") is not None:
                out["rs|" + l.layer_name] = nlp["running_std"].cpu().numpy()
        np.savez(os.path.join(outdir, "rank%d.npz" % rank), **out)
        dist.destroy_process_group()
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("env", [{}, {"DORKNET_ASYNC_WGRAD": "0", "DORKNET_BRANCH_STREAM": "1"}],
                         ids=["default", "sync_wgrad_branch"])
def test_data_parallel_gloo_world2_equals_full_batch(tmp_path, env):
    """`sync_wgrad_branch`: weight gradients on the issuing stream, skip projections on
    the branch stream, their gradients all-reduced (update_skip_projections=True)."""
    import torch.multiprocessing as mp
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_gloo_rank, args=(r, world, port, str(tmp_path), q, env)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        results = dict(q.get(timeout=100) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
    assert results == {0: "ok", 1: "ok"}, results
    ranks = [dict(np.load(tmp_path / ("rank%d.npz" % r))) for r in range(world)]
    # the oracle on the concatenated batch (same initial weights: same numpy seed)
    X, _, onehot = synthetic_batch(2 * world, seed=SEED_X)
    np.random.seed(SEED_W)
    net = ResNet18("r18")
    onet = network_to_oracle(net)
    o32 = network_to_oracle(net, np.float32)
    oloss, _ = onet.forward(X.astype(np.float64), onehot.astype(np.float64))
    onet.backward()
    o32.forward(X, onehot)
    o32.backward()
    loss_dp = np.mean([float(r["loss"]) for r in ranks])
    assert abs(loss_dp - oloss) <= 1e-4 * abs(oloss), (loss_dp, oloss)
    worst = []
    for ol, o3 in zip(all_layers(onet.layers), all_layers(o32.layers)):
        for k in (ol.grads or {}):
            key = "g|{}|{}".format(ol.layer_name, k)
            assert np.array_equal(ranks[0][key], ranks[1][key]), key  # the average is the same on every rank
            worst.append((_excess(ranks[0][key], np.asarray(ol.grads[k], np.float64), o3.grads[k]),
                          ol.layer_name, k))
        nlp = getattr(ol, "non_learned_params", None)
        if nlp and nlp.get("running_std") is not None:
            assert rel_err(ranks[0]["rs|" + ol.layer_name].ravel(), np.ravel(nlp["running_std"])) <= 1e-4
    worst.sort(reverse=True)
    assert worst[0][0] <= 1.0, worst[:5]
