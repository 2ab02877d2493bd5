"""Weight gradients on the side stream (dorknet_amd._hip.weight_grad_stream) and the skip
projections on the branch stream (dorknet_amd._hip.on_branch): the network
backward with DORKNET_ASYNC_WGRAD=1 must give bit-identical gradients to the single-stream
run (same kernels, only their stream changes), and the data-parallel backward, whose
RCCL buckets are issued from the side stream, must deliver them through the flat buffer
(RCCL, world size 1 on the one GPU: the average is the identity)."""
import socket

import numpy as np
import pytest
import torch

from tests._convert import all_layers

pytestmark = pytest.mark.gpu


def _grads(net):
    return [l.grads[k].detach().clone() for l in all_layers(net.layers) for k in sorted(l.grads or {})]


def _step(net, X, onehot, dp=None):
    net.forward(torch.as_tensor(X, device="cuda"), torch.as_tensor(onehot, device="cuda"))
    (dp or net).backward()
    return _grads(net)


def test_async_weight_grads_bitwise(monkeypatch):
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    X, _, onehot = synthetic_batch(4, seed=7)
    np.random.seed(9)
    net = ResNet18("r18")
    net.to_gpu()
    runs = []
    for flag in ("1", "0", "1"):
        monkeypatch.setenv("DORKNET_ASYNC_WGRAD", flag)
        runs.append(_step(net, X, onehot))
    torch.cuda.synchronize()
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert torch.equal(a, b)


def test_branch_stream_bitwise(monkeypatch):
    """The residual blocks' skip projections on the branch stream (forward and input gradient,
    DORKNET_BRANCH_STREAM=1) give the same gradients bit for bit as the single-stream run, at a
    batch where the skip kernels overlap the chain, with and without side-stream weight gradients."""
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    X, _, onehot = synthetic_batch(16, seed=11)
    np.random.seed(12)
    net = ResNet18("r18")
    net.to_gpu()
    runs = []
    for branch, wgrad in (("1", "1"), ("0", "1"), ("1", "0"), ("0", "0"), ("1", "1")):
        monkeypatch.setenv("DORKNET_BRANCH_STREAM", branch)
        monkeypatch.setenv("DORKNET_ASYNC_WGRAD", wgrad)
        runs.append(_step(net, X, onehot))
    torch.cuda.synchronize()
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert torch.equal(a, b)


def test_wgrad_reduce_side_stream_bitwise(monkeypatch):
    """The fused backward entry points' weight-gradient reduces deferred to the side stream
    (dk_wgrad_reduce_defer / _flush, DORKNET_WGRAD_REDUCE_SIDE=1, the default) give the same
    gradients bit for bit as reducing in the entry point, with the branch stream on and off."""
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    X, _, onehot = synthetic_batch(16, seed=13)
    np.random.seed(14)
    net = ResNet18("r18")
    net.to_gpu()
    runs = []
    for side, branch in (("1", "1"), ("0", "1"), ("1", "0"), ("0", "0"), ("1", "1")):
        monkeypatch.setenv("DORKNET_WGRAD_REDUCE_SIDE", side)
        monkeypatch.setenv("DORKNET_BRANCH_STREAM", branch)
        runs.append(_step(net, X, onehot))
    torch.cuda.synchronize()
    for other in runs[1:]:
        for a, b in zip(runs[0], other):
            assert torch.equal(a, b)


def test_stream_helpers_match_torch():
    """_hip.cur_stream / use_stream (torch's C layer directly) agree with torch.cuda.current_stream /
    torch.cuda.stream: the stream is switched inside the block and restored after it, nested too."""
    from dorknet_amd._hip import cur_stream, stream_handle, use_stream
    main = torch.cuda.current_stream()
    assert cur_stream() == main
    a, b = torch.cuda.Stream(), torch.cuda.Stream()
    with use_stream(a):
        assert torch.cuda.current_stream() == a and cur_stream() == a and stream_handle() == a.cuda_stream
        with use_stream(b):
            assert torch.cuda.current_stream() == b
        assert torch.cuda.current_stream() == a
    assert torch.cuda.current_stream() == main and stream_handle() == main.cuda_stream


def test_wgrad_reduce_defer_protocol():
    """A flush with none recorded is refused, an unknown mode is refused, and mode -1 drops the
    recorded ones."""
    from dorknet_amd._hip import HipError, lib
    lib.dk_wgrad_reduce_defer(-1)
    assert lib.dk_wgrad_reduce_pending() == 0
    with pytest.raises(HipError):
        lib.dk_wgrad_reduce_flush(0)
    with pytest.raises(HipError):
        lib.dk_wgrad_reduce_defer(2)
    lib.dk_wgrad_reduce_defer(0)


@pytest.mark.parametrize("every", ["1", "4", "64"])
def test_wgrad_reduce_batched_flush_bitwise(monkeypatch, every):
    """Recorded reduces launched in batches (dorknet_amd._hip.FLUSH_EVERY: one cross-stream wait per
    batch) give the same gradients bit for bit as one flush per layer."""
    from dorknet_amd import _hip
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._hip import lib
    X, _, onehot = synthetic_batch(8, seed=15)
    np.random.seed(16)
    net = ResNet18("r18")
    net.to_gpu()
    monkeypatch.setattr(_hip, "FLUSH_EVERY", 1)
    ref = _step(net, X, onehot)
    monkeypatch.setattr(_hip, "FLUSH_EVERY", min(60, int(every)))
    got = _step(net, X, onehot)
    torch.cuda.synchronize()
    assert lib.dk_wgrad_reduce_pending() == 0
    for a, b in zip(ref, got):
        assert torch.equal(a, b)


def test_data_parallel_rccl_world1():
    import torch.distributed as dist
    from dorknet_amd.parallel import DataParallel
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % port, rank=0, world_size=1)
    try:
        X, _, onehot = synthetic_batch(4, seed=8)
        np.random.seed(10)
        net = ResNet18("r18")
        net.to_gpu()
        ref = _step(net, X, onehot)
        dp = DataParallel(net, bucket_bytes=1 << 20, update_skip_projections=True)
        got = _step(net, X, onehot, dp)
        torch.cuda.synchronize()
        for a, b in zip(ref, got):
            assert torch.equal(a, b)
        assert all(l.grads[k].data_ptr() >= dp.flat.data_ptr() for l in all_layers(net.layers)
                   for k in (l.grads or {}))
        # bucket launches against layer order: every bucket once, in bucket order (the buckets
        # cover the layers in reverse, the order the backward finishes them), and issued while the
        # backward still runs -- not all after it (sub-layer readiness inside residual blocks)
        order = [b for b, _ in dp.launch_log]
        reported = [n for _, n in dp.launch_log]
        assert sorted(order) == list(range(len(dp.buckets)))
        assert order == sorted(order)
        assert reported == sorted(reported)
        assert len(dp.buckets) > 2 and reported[0] < reported[-1]
    finally:
        dist.destroy_process_group()
