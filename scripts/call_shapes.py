"""Every C-ABI call of one training step in issue order: entry point, its integer arguments (the
shape), HIP-event time on the launch stream and the fraction of its own roofline bound
(perfmodel).  The step runs single-stream (DORKNET_ASYNC_WGRAD=0) so that no call's time
includes a concurrent weight gradient.
    python scripts/call_shapes.py [--config 3|5] [--min-us 20]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min-us", type=float, default=20.0)
    ap.add_argument("--batch", type=int, default=0, help="default: 256 (config 3), 512 (config 5)")
    ap.add_argument("--config", type=int, choices=[3, 5], default=3)
    a = ap.parse_args()
    os.environ["DORKNET_ASYNC_WGRAD"] = "0"
    a.batch = a.batch or (256 if a.config == 3 else 512)
    from bench import Instrument
    from dorknet_amd import perfmodel
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    torch.cuda.set_device(0)
    np.random.seed(0)
    if a.config == 3:
        net = ResNet18("r")
        net.to_gpu()
        X, _, onehot = synthetic_batch(a.batch, seed=1000)
        X, onehot = as_device(X), as_device(onehot)

        def fb():
            net.forward(X, onehot)
            net.backward()
    else:
        from examples.mobilenet_stack import MobileNetStack, synthetic_input
        net = MobileNetStack("m")
        net.to_gpu()
        X = synthetic_input(a.batch, seed=0)
        dY = torch.randn((a.batch, 512, 7, 7), device="cuda").to(torch.bfloat16)
        dY = dY.contiguous(memory_format=torch.channels_last)

        def fb():
            net.forward(X, None)
            net.backward(dY)
    sgd = SGDMomentum(net, 0.05 * a.batch / 200.0, 0.9)

    def step():
        fb()
        sgd.update_weights()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    with Instrument(perfmodel.MODEL.keys()) as ins:
        step()
    torch.cuda.synchronize()
    rows = []
    for n, calls in ins.calls.items():
        for e0, e1, args in calls:
            rows.append((e0, n, args, e0.elapsed_time(e1)))
    # issue order: by the start event's time relative to the first event recorded
    first = min(rows, key=lambda r: 0)[0]
    rows.sort(key=lambda r: first.elapsed_time(r[0]))
    tot = 0.0
    for _, n, args, ms in rows:
        us = 1e3 * ms
        tot += us
        if us < a.min_us:
            continue
        f, b = perfmodel.work(n, args)
        frac = perfmodel.bound_time_s(f, b, n) / (ms / 1e3) if ms > 0 else 0.0
        ints = [x for x in args if isinstance(x, int) and abs(x) < 1 << 20]
        print(f"{us:8.1f} us  frac {frac:5.3f}  {'mfma' if perfmodel.is_mfma_bound(f, b, n) else 'hbm '}  "
              f"{n:34s} {ints[:10]}", flush=True)
    print(f"total {tot:.1f} us over {len(rows)} calls")


if __name__ == "__main__":
    main()
