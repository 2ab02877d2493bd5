"""Host-side enqueue cost of one ResNet-18-depsep training step vs its GPU time: if the host
takes as long to issue a step as the GPU takes to run it, the step is launch-bound.

    python scripts/host_overhead.py [--steps 20]
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
    ap.add_argument("--batch", type=int, default=256)
    args = ap.parse_args()
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    torch.cuda.set_device(0)
    np.random.seed(0)
    net = ResNet18("r")
    net.to_gpu()
    sgd = SGDMomentum(net, 0.05 * args.batch / 200.0, 0.9)
    X, _, onehot = synthetic_batch(args.batch, seed=1000)
    X, onehot = as_device(X), as_device(onehot)

    def step():
        net.forward(X, onehot)
        net.backward()
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


if __name__ == "__main__":
    main()
