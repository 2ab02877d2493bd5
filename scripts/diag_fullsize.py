"""Diagnostics for tests/test_gpu_fullsize.py: error breakdown (per image, per channel, every
gradient) of the res1 chain at several batch sizes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from tests.test_gpu_fullsize import _perturb_bn, _run
from tests._convert import rel_err

def main():
    from examples.resnet18_depsep import ResNet18
    for N in [int(a) for a in sys.argv[1:]] or [16, 256]:
        np.random.seed(31)
        layers = ResNet18("r18").layers[4:7]
        rng = np.random.default_rng(32)
        _perturb_bn(layers, rng)
        X = (0.5 + 2.0 * rng.standard_normal((N, 64, 56, 56), dtype=np.float32))
        dY = rng.standard_normal((N, 64, 56, 56), dtype=np.float32)
        (Yg, dXg, gg), (Yt, dXt, gt), _, twin, net = _run(layers, X, dY, input_grad=True)
        print("N", N, "Y", rel_err(Yg, Yt), "dX", rel_err(dXg, dXt), flush=True)
        per_img = [rel_err(dXg[i], dXt[i]) for i in range(N)]
        print("  dX per image: min %.2e max %.2e argmax %d" % (min(per_img), max(per_img), int(np.argmax(per_img))))
        per_ch = [rel_err(dXg[:, c], dXt[:, c]) for c in range(64)]
        print("  dX per channel: min %.2e max %.2e argmax %d" % (min(per_ch), max(per_ch), int(np.argmax(per_ch))))
        d = np.abs(dXg - dXt)
        i = np.unravel_index(np.argmax(d), d.shape)
        print("  worst element", i, dXg[i], dXt[i], "scale", np.abs(dXt).mean())
        for (name, k), w in sorted(gt.items()):
            g = gg[(name, k)].reshape(w.shape)
            print("  %-24s %-8s rel %.3e  |w| %.3e" % (name, k, rel_err(g, w), np.linalg.norm(w)))
        # twin in fp32 (same maths, fp32 arithmetic) for the conditioning of dX
        import tests._torch_twin as T
        old = T._np
        T._np = lambda v: np.asarray(v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else v, dtype=np.float32)
        try:
            from tests._torch_twin import TorchTwin
            tw32 = TorchTwin.__new__(TorchTwin)
            tw32.__init__(layers)
            Y32, dX32, g32 = tw32.run(X, dY, input_grad=True)
        finally:
            T._np = old
        print("  torch fp32 twin: Y %.3e dX %.3e" % (rel_err(Y32, Yt), rel_err(dX32, dXt)))
        for (name, k), w in sorted(gt.items()):
            print("  fp32 %-24s %-8s rel %.3e" % (name, k, rel_err(g32[(name, k)].reshape(w.shape), w)))

main()
