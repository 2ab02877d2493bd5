"""Diagnostic: batch-2 ResNet training steps vs the oracle for several input seeds and both stem paths."""
import os, sys, numpy as np
sys.path.insert(0, os.getcwd())
from tests.test_gpu_network import _compare_step
from tests._convert import network_to_oracle
from examples.resnet18_depsep import ResNet18, synthetic_batch
for seed in [1, 2, 3, 4, 5, 6]:
    for narrow in ["1", "0"]:
        os.environ["DORKNET_NARROW"] = narrow
        np.random.seed(0)
        net = ResNet18("r18"); onet = network_to_oracle(net); o32 = network_to_oracle(net, np.float32)
        net.to_gpu()
        X, _, onehot = synthetic_batch(2, seed=seed)
        try:
            _compare_step(net, onet, o32, X, onehot, lr=0.05 * 2 / 200.0)
            print("seed", seed, "narrow", narrow, "PASS", flush=True)
        except AssertionError as e:
            print("seed", seed, "narrow", narrow, "FAIL", str(e)[:200], flush=True)
