"""Where the stride-2 join forward's y differs from the join pass (tests/test_gpu_join_fwd.py case
stats=True, abn=True, bbn=False, C=64, N=2, H=13, W=11): prints the mismatching (n, h, w, c) positions.
DORKNET_HIP_LIB selects the library."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dorknet_amd._hip import LIB_PATH, lib, stream_handle  # noqa: E402


def nhwc(a):
    return torch.as_tensor(np.ascontiguousarray(a, dtype=np.float32), device="cuda").contiguous(
        memory_format=torch.channels_last)


def case(stride, C, N, H, W, stats):
    rng = np.random.RandomState(C + N + H + 3 * stride + 5)
    a = nhwc(rng.randn(N, C, H, W) * 1.5)
    b = nhwc(rng.randn(N, C, H, W))
    pa = [torch.as_tensor(v.astype(np.float32), device="cuda") for v in
          (rng.randn(C) * 0.3, rng.rand(C) + 0.5, 1 + 0.3 * rng.randn(C), 0.2 * rng.randn(C))]
    w = torch.as_tensor((rng.randn(C, 3, 3) * 0.3).astype(np.float32), device="cuda")
    OH, OW = (H - 1) // stride + 1, (W - 1) // stride + 1
    st = stream_handle()
    aa = (*(t.data_ptr() for t in pa), 0)
    ba = (0, 0, 0, 0, 0)
    rows = lib.dk_dwconv_fwd_stats_rows(N, OH, OW, C, stride)
    y0 = nhwc(np.zeros((N, C, H, W)))
    lib.dk_bn_add_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, a.numel(), C, 1, y0.data_ptr(), 0, st)
    ybuf = torch.full((N * C * H * W + 4096,), 12345.0, device="cuda")
    y1 = ybuf[:N * C * H * W].view(N, H, W, C)
    o1 = torch.full((N, C, OH, OW), float("nan"), device="cuda").contiguous(memory_format=torch.channels_last)
    p1 = torch.full((rows, 2, C), float("nan"), dtype=torch.float64, device="cuda") if stats else None
    rc = lib.dk_dwconv_fwd_join_f32(a.data_ptr(), *aa, b.data_ptr(), *ba, ybuf.data_ptr(), 0, N, H, W, C,
                                    w.data_ptr(), stride, 0, o1.data_ptr(), OH, OW, p1.data_ptr() if stats else 0, st)
    torch.cuda.synchronize()
    y0h = y0.permute(0, 2, 3, 1).cpu().numpy()
    y1h = y1.cpu().numpy()
    bad = np.argwhere(y0h != y1h)
    print("stride %d C %d N %d H %d W %d stats %d rc %d: %d of %d differ" % (stride, C, N, H, W, stats, rc, len(bad),
                                                                           y0h.size), flush=True)
    if len(bad):
        hs = sorted(set(int(v) for v in bad[:, 1]))
        ws = sorted(set(int(v) for v in bad[:, 2]))
        cs = sorted(set(int(v) for v in bad[:, 3]))
        print("  rows", hs, "cols", ws, "channels", cs[:16], "... (%d)" % len(cs))
        for i in bad[:6]:
            i = tuple(int(v) for v in i)
            print("  ", i, y0h[i], y1h[i])


if __name__ == "__main__":
    print("lib", LIB_PATH)
    for stats in (1, 0):
        case(2, 64, 2, 13, 11, stats)
        case(2, 256, 2, 7, 7, stats)
        case(2, 128, 3, 9, 16, stats)
