"""Diagnostic: conv0's weight gradient with and without the lattice hand-over at a small image size."""
import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from examples.resnet18_depsep import ResNet18, synthetic_batch
from dorknet_amd._tensor import as_device
for size in (97, 65, 225):
    res = {}
    for lat in ("1", "0"):
        os.environ["DORKNET_LATTICE"] = lat
        np.random.seed(0)
        net = ResNet18("r"); net.to_gpu()
        X, _, onehot = synthetic_batch(4 if size < 225 else 2, seed=2, size=size)
        net.forward(as_device(X), as_device(onehot)); net.backward(); torch.cuda.synchronize()
        res[lat] = {k: v.clone() for k, v in net.layers[0].grads.items()}
        g = res[lat]["weights"]
        print(size, "lattice", lat, "nan", bool(torch.isnan(g).any()), "norm", float(g.norm()), flush=True)
    a, b = res["1"]["weights"], res["0"]["weights"]
    print(size, "rel diff", float((a - b).norm() / b.norm()), flush=True)
