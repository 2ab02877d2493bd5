"""Host-side enqueue cost of one ResNet-18-depsep training step vs its GPU time: if the host
takes as long to issue a step as the GPU takes to run it, the step is launch-bound.

    python scripts/host_overhead.py [--steps 20] [--config 3|5] [--profile]
--profile: the same steps under cProfile, the top functions by own time (where the issue time goes).
"""
import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--config", type=int, choices=[3, 5], default=3)
    ap.add_argument("--profile", action="store_true")
    args = ap.parse_args()
    args.batch = args.batch or (256 if args.config == 3 else 512)
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    torch.cuda.set_device(0)
    np.random.seed(0)
    if args.config == 3:
        net = ResNet18("r")
        net.to_gpu()
        X, _, onehot = synthetic_batch(args.batch, seed=1000)
        X, onehot = as_device(X), as_device(onehot)

        def fb():
            net.forward(X, onehot)
            net.backward()
    else:
        from examples.mobilenet_stack import MobileNetStack, synthetic_input
        net = MobileNetStack("m")
        net.to_gpu()
        X = synthetic_input(args.batch, seed=0)
        dY = torch.randn((args.batch, 512, 7, 7), device="cuda").to(torch.bfloat16)
        dY = dY.contiguous(memory_format=torch.channels_last)

        def fb():
            net.forward(X, None)
            net.backward(dY)
    sgd = SGDMomentum(net, 0.05 * args.batch / 200.0, 0.9)

    def step():
        fb()
        sgd.update_weights()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    # host enqueue time with the GPU far behind (queue filling): time per step() call
    host = []
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = time.perf_counter()
        step()
        host.append(time.perf_counter() - a)
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    # host time with an idle GPU: sync, then issue one step
    solo = []
    for _ in range(5):
        torch.cuda.synchronize()
        a = time.perf_counter()
        step()
        solo.append(time.perf_counter() - a)
    torch.cuda.synchronize()
    print(f"host issue per step {1e3 * np.median(host):.2f} ms (min {1e3 * min(host):.2f}); "
          f"wall per step {1e3 * t_all / args.steps:.2f} ms; issue total {1e3 * t_issue / args.steps:.2f} ms/step; "
          f"solo issue {1e3 * np.median(solo):.2f} ms", flush=True)
    if args.profile:
        import cProfile
        import pstats
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        pr.disable()
        st = pstats.Stats(pr)
        st.sort_stats("tottime").print_stats(35)


if __name__ == "__main__":
    main()
