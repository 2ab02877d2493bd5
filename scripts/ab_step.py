"""A/B timing of the ResNet-18-depsep training step (bs=256) under C-ABI tuning knobs.

    python scripts/ab_step.py --knob 2:0 --knob 2:1 --knob 2:2     # dk_debug_set_gemm_config(kind, cfg)
Each setting is timed `--rounds` times interleaved (median ms per step reported).
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
    ap.add_argument("--knob", action="append", default=[], help="kind:cfg for dk_debug_set_gemm_config")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--batch", type=int, default=0, help="default: 256 (config 3), 512 (config 5)")
    ap.add_argument("--config", type=int, choices=[3, 5], default=3)
    args = ap.parse_args()
    args.batch = args.batch or (256 if args.config == 3 else 512)
    from examples.resnet18_depsep import ResNet18, synthetic_batch
    from dorknet_amd._tensor import as_device
    from dorknet_amd._hip import lib
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

    # kind:cfg (dk_debug_set_gemm_config) or env:NAME=VALUE (read per call by the layers)
    knobs = [tuple(k.split(":", 1)) if k.startswith("env:") else tuple(int(v) for v in k.split(":"))
             for k in args.knob] or [(2, -1)]
    res = {k: [] for k in knobs}
    for _ in range(args.rounds):
        for k in knobs:
            if k[0] == "env":
                name, val = k[1].split("=", 1)
                prev = os.environ.get(name)
                os.environ[name] = val
            else:
                lib.dk_debug_set_gemm_config(*k)
            for _ in range(2):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            res[k].append(1e3 * (time.perf_counter() - t0) / args.steps)
            if k[0] != "env":
                lib.dk_debug_set_gemm_config(k[0], -1)
            elif prev is None:  # the next setting runs without this one
                os.environ.pop(name)
            else:
                os.environ[name] = prev
    for k, v in res.items():
        print(f"knob {k[0]}:{k[1]:>3}  {np.median(v):7.3f} ms/step  ({', '.join(f'{x:.3f}' for x in v)})  "
              f"{args.batch / np.median(v) * 1e3:9.1f} img/s", flush=True)


if __name__ == "__main__":
    main()
