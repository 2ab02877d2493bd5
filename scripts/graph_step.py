"""ResNet-18-depsep training step (bs=256) replayed as a captured HIP graph vs eager launches.

    python scripts/graph_step.py [--steps 20]
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

    def timed(fn, n):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
    torch.cuda.current_stream().wait_stream(s)
    eager = timed(step, args.steps)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    graph = timed(g.replay, args.steps)
    eager2 = timed(step, args.steps)
    print(f"eager {eager:.3f} ms/step, graph {graph:.3f} ms/step, eager again {eager2:.3f} ms/step "
          f"({args.batch / graph * 1e3:.0f} img/s graph)", flush=True)


if __name__ == "__main__":
    main()
