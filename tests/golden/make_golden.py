"""Generate the committed golden fixtures (tests/golden/*.npz) from the oracle.

The reference ships no fixtures and running it was denied, so the
fixtures are produced by the oracle (oracle/ref.py, oracle/net.py) -- itself pinned
against torch CPU and analytic known answers (tests/test_oracle.py) -- with fixed seeds.
Each case stores fp32 inputs / parameters, the fp64 oracle outputs ("<name>_f64") and
the reference-faithful fp32 oracle outputs ("<name>_f32").

    python tests/golden/make_golden.py          # rewrites tests/golden/*.npz
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import net as O  # noqa: E402
from oracle import ref  # noqa: E402


def _both(fn, *arrays):
    """Run fn on fp64 and fp32 copies of the arrays; returns (out64, out32)."""
    a64 = [None if a is None else np.asarray(a, np.float64) for a in arrays]
    a32 = [None if a is None else np.asarray(a, np.float32) for a in arrays]
    return fn(*a64), fn(*a32)


def case_conv(name, N, C, H, W, K, R, S, st, pd, bias, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, C, H, W)).astype(np.float32)
    Wt = (0.1 * rng.standard_normal((K, C, R, S))).astype(np.float32)
    b = rng.standard_normal(K).astype(np.float32) if bias else None
    OH = int((H + 2 * pd - R) / st + 1)
    OW = int((W + 2 * pd - S) / st + 1)
    dY = rng.standard_normal((N, K, OH, OW)).astype(np.float32)

    def run(X, Wt, b, dY):
        Y, cache = ref.conv_forward(X, Wt, b, st, pd)
        dX, dW, db = ref.conv_backward(dY, Wt, cache, st, pd, bias, 1e-4)
        return {"Y": Y, "dX": dX, "dW": dW, **({"db": db} if bias else {})}

    o64, o32 = _both(run, X, Wt, b, dY)
    meta = dict(kind="conv", stride=st, padding=pd, bias=int(bias), l2=1e-4)
    return name, dict(X=X, W=Wt, dY=dY, **({"b": b} if bias else {})), o64, o32, meta


def case_dw(name, N, C, H, R, st, pd, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, C, H, H)).astype(np.float32)
    Wt = (0.3 * rng.standard_normal((C, R, R))).astype(np.float32)
    OH = int((H + 2 * pd - R) / st + 1)
    dY = rng.standard_normal((N, C, OH, OH)).astype(np.float32)

    def run(X, Wt, dY):
        Y, cache = ref.depthwise_forward(X, Wt, None, st, pd)
        dX, dW, _ = ref.depthwise_backward(dY, Wt, cache, st, pd, False)
        return {"Y": Y, "dX": dX, "dW": dW}

    o64, o32 = _both(run, X, Wt, dY)
    return name, dict(X=X, W=Wt, dY=dY), o64, o32, dict(kind="dw", stride=st, padding=pd, bias=0, l2=0.0)


def case_pw(name, N, C, H, K, st, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((N, C, H, H)).astype(np.float32)
    Wt = (0.1 * rng.standard_normal((K, C))).astype(np.float32)
    OH = -(-H // st)
    dY = rng.standard_normal((N, K, OH, OH)).astype(np.float32)

    def run(X, Wt, dY):
        Y, cache = ref.pointwise_forward(X, Wt, None, st)
        dX, dW, _ = ref.pointwise_backward(dY, Wt, cache, st, False, 1e-4)
        return {"Y": Y, "dX": dX, "dW": dW}

    o64, o32 = _both(run, X, Wt, dY)
    return name, dict(X=X, W=Wt, dY=dY), o64, o32, dict(kind="pw", stride=st, bias=0, l2=1e-4)


def case_dense(name, B, IN, OUT, seed):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((B, IN)).astype(np.float32)
    Wt = (0.1 * rng.standard_normal((IN, OUT))).astype(np.float32)
    b = rng.standard_normal(OUT).astype(np.float32)
    dY = rng.standard_normal((B, OUT)).astype(np.float32)

    def run(X, Wt, b, dY):
        Y = ref.dense_forward(X, Wt, b)
        dX, dW, db = ref.dense_backward(dY, X, Wt, True, 1e-4)
        return {"Y": Y, "dX": dX, "dW": dW, "db": db}

    o64, o32 = _both(run, X, Wt, b, dY)
    return name, dict(X=X, W=Wt, b=b, dY=dY), o64, o32, dict(kind="dense", bias=1, l2=1e-4)


def case_bn(name, shape, seed):
    rng = np.random.default_rng(seed)
    C = shape[1]
    pshape = (1, C, 1, 1) if len(shape) == 4 else (C,)
    g = (1 + 0.2 * rng.standard_normal(pshape)).astype(np.float32)
    b = (0.3 * rng.standard_normal(pshape)).astype(np.float32)
    X1 = (1.5 + 2.0 * rng.standard_normal(shape)).astype(np.float32)
    X2 = (-0.5 + 1.0 * rng.standard_normal(shape)).astype(np.float32)
    dY = rng.standard_normal(shape).astype(np.float32)
    Xt = rng.standard_normal(shape).astype(np.float32)

    def run(g, b, X1, X2, dY, Xt):
        bn = O.OBatchNorm("bn", g, b)
        Y1 = bn.forward(X1)
        Y2 = bn.forward(X2)
        dX2 = bn.backward(dY)
        Yt = bn.forward(Xt, test_mode=True)
        return {"Y1": Y1, "Y2": Y2, "dX2": dX2, "dgamma": bn.grads["gamma"], "dbeta": bn.grads["beta"],
                "running_mean": bn.non_learned_params["running_mean"],
                "running_std": bn.non_learned_params["running_std"], "Ytest": Yt}

    o64, o32 = _both(run, g, b, X1, X2, dY, Xt)
    return name, dict(gamma=g, beta=b, X1=X1, X2=X2, dY=dY, Xt=Xt), o64, o32, dict(kind="bn")


def case_head(name, seed):
    rng = np.random.default_rng(seed)
    A = rng.standard_normal((3, 16, 5, 5)).astype(np.float32)
    logits = rng.standard_normal((4, 12)).astype(np.float32)
    y = np.eye(12, dtype=np.float32)[rng.integers(0, 12, 4)]

    def run(A, logits, y):
        out, mask = ref.relu_forward(A)
        loss, P = ref.softmax_xent_forward(logits, y)
        return {"relu": out, "mask": mask, "gap": ref.gap_forward(A), "P": P,
                "loss": np.array(loss), "dlogits": ref.softmax_xent_backward(P, y)}

    o64, o32 = _both(run, A, logits, y)
    return name, dict(A=A, logits=logits, y=y), o64, o32, dict(kind="head")


CASES = [
    lambda: case_conv("conv_conv0like_s2", 2, 3, 17, 17, 8, 5, 5, 2, 1, False, 10),
    lambda: case_conv("conv_3x3_bias", 2, 16, 9, 11, 16, 3, 3, 1, 1, True, 11),
    lambda: case_conv("conv_4x4_s2", 2, 8, 14, 14, 16, 4, 4, 2, 1, False, 12),
    lambda: case_dw("dw_3x3_s1", 2, 16, 9, 3, 1, 1, 13),
    lambda: case_dw("dw_3x3_s2", 2, 32, 14, 3, 2, 1, 14),
    lambda: case_pw("pw_s2", 2, 16, 12, 32, 2, 15),
    lambda: case_pw("pw_s1", 2, 32, 7, 64, 1, 16),
    lambda: case_dense("dense", 4, 64, 20, 17),
    lambda: case_bn("bn_4d", (3, 8, 5, 7), 18),
    lambda: case_bn("bn_2d", (6, 12), 19),
    lambda: case_head("head", 20),
]


def save(name, inputs, o64, o32, meta):
    arrays = {("in_" + k): v for k, v in inputs.items()}
    arrays.update({k + "_f64": np.asarray(v, np.float64) for k, v in o64.items()})
    arrays.update({k + "_f32": np.asarray(v, np.float32) for k, v in o32.items()})
    for k, v in meta.items():
        arrays["meta_" + k] = np.asarray(v)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **arrays)


def main():
    for make in CASES:
        save(*make())
    print("wrote", len(CASES), "fixtures to", HERE)


if __name__ == "__main__":
    main()
