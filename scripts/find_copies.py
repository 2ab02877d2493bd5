"""Where the torch-side copies and fills of a ResNet-18-depsep training step come from: one step
under torch.profiler (with Python stacks), the aten copy / fill / zero ops listed with the
innermost dorknet_amd frames.  python scripts/find_copies.py"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from dorknet_amd._tensor import as_device
    from dorknet_amd.optimisers.SGDMomentum import SGDMomentum
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    torch.cuda.set_device(0)
    np.random.seed(0)
    net = ResNet18("r")
    net.to_gpu()
    sgd = SGDMomentum(net, 0.05 * 256 / 200.0, 0.9)
    X, _, onehot = synthetic_batch(256, seed=1000)
    X, onehot = as_device(X), as_device(onehot)

    def step():
        net.forward(X, onehot)
        net.backward()
        sgd.update_weights()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    hits = collections.Counter()
    for ev in prof.events():
        name = ev.name
        if not any(k in name for k in ("copy_", "fill_", "zero_", "aten::clone", "aten::contiguous", "aten::cat",
                                       "aten::to", "aten::_to_copy", "aten::zeros", "aten::full")):
            continue
        frames = [f for f in (ev.stack or []) if "dorknet_amd" in f or "examples" in f or "bench" in f]
        hits[(name, str(ev.input_shapes)[:80], " <- ".join(frames[:3]))] += 1
    for (name, shapes, where), n in hits.most_common(60):
        print(f"{n:3d}  {name:22s} {shapes:80s} {where}")


if __name__ == "__main__":
    main()
