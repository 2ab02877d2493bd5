"""Diagnostic: ReLU masks of the batch-2 ResNet forward, narrow stem vs implicit GEMM."""
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
import torch
from tests._convert import all_layers
from examples.resnet18_depsep import ResNet18, synthetic_batch
from tests.test_gpu_network import dev
masks = {}
for narrow in ["0", "1"]:
    os.environ["DORKNET_NARROW"] = narrow
    np.random.seed(0)
    net = ResNet18("r18"); net.to_gpu()
    X, _, onehot = synthetic_batch(2, seed=1)
    net.forward(dev(X), dev(onehot))
    net.backward()
    torch.cuda.synchronize()
    m = {}
    for l in all_layers(net.layers):
        if getattr(l, "_mean", None) is not None and isinstance(getattr(l, "X", None), torch.Tensor):
            C = l.X.shape[1]
            sh = (1, C, 1, 1)
            ga = torch.as_tensor(l.learned_params["gamma"]).reshape(sh).to(l.X.device).float()
            be = torch.as_tensor(l.learned_params["beta"]).reshape(sh).to(l.X.device).float()
            y = ga * ((l.X - l._mean.reshape(sh)) * l._invstd.reshape(sh)) + be
            m[l.layer_name] = (y > 0).cpu()
    masks[narrow] = m
for k, a in masks["0"].items():
    b = masks["1"].get(k)
    if b is not None and a.shape == b.shape:
        n = int((a != b).sum())
        if n:
            print(f"{k}: {n} mask flips of {a.numel()}")
print("done", len(masks["0"]))
