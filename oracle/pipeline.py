"""TEST INFRASTRUCTURE ONLY -- the checker for the device-side input pipeline.  Imported by
tests/ only; the product path (dorknet_amd/data_loading) never calls it.

numpy restatement of the reference's per-image preprocessing and mixup:

- preprocess(im): data_loading/image_preprocessor.py:16-39 -- cv2.resize (INTER_LINEAR), crop
  ("random": offsets drawn per image, row then column, np.random.randint(0, max_offset);
  "center": int((size - crop) / 2)), astype(float32), transpose(2, 0, 1), - 128.0.  The
  augmenter call (:33-34) discards its result in the reference, so augmentation has no effect
  and is not restated.
- resize_bilinear(im, OW, OH): cv2's INTER_LINEAR geometry (source coordinate
  (float)((o + 0.5) * scale - 0.5) computed in double, floor, clamps to [0, L - 1] with zero
  weight at the edges), interpolated in fp32 (every operation rounded to fp32, the same order as
  dorknet_amd/csrc/input_pipeline.hip), rounded to nearest-even, saturated to uint8.  cv2 itself
  interpolates uint8 in 11-bit fixed point and is not installed here: agreement with cv2 is
  parity unpinned; this restatement pins the GPU kernel bit for bit.
- mixup(X, Xm, p): data_loading/image_data_loader.py:101-111 -- p * X_m + (1 - p) * X and the
  mirror, numpy semantics (a Python float times a float32 array stays float32).
"""
from __future__ import annotations

import numpy as np


def _coords(O, L):
    s = np.float64(L) / np.float64(O)
    v = ((np.arange(O, dtype=np.float64) + 0.5) * s - 0.5).astype(np.float32)
    k = np.floor(v).astype(np.int64)
    f = (v - k.astype(np.float32)).astype(np.float32)
    lo = k < 0
    k[lo], f[lo] = 0, 0
    hi = k >= L - 1
    k[hi], f[hi] = L - 1, 0
    return k, np.minimum(k + 1, L - 1), f


def resize_bilinear(im, OW, OH):
    """im: uint8 (H, W, C) -> uint8 (OH, OW, C)."""
    H, W = im.shape[:2]
    y0, y1, fy = _coords(OH, H)
    x0, x1, fx = _coords(OW, W)
    one = np.float32(1.0)
    gy, gx = (one - fy).astype(np.float32), (one - fx).astype(np.float32)
    f = im.astype(np.float32)
    p00, p01 = f[y0][:, x0], f[y0][:, x1]
    p10, p11 = f[y1][:, x0], f[y1][:, x1]
    gx3, fx3 = gx[None, :, None], fx[None, :, None]
    gy3, fy3 = gy[:, None, None], fy[:, None, None]
    top = (gx3 * p00).astype(np.float32) + (fx3 * p01).astype(np.float32)
    bot = (gx3 * p10).astype(np.float32) + (fx3 * p11).astype(np.float32)
    v = (gy3 * top.astype(np.float32)).astype(np.float32) + (fy3 * bot.astype(np.float32)).astype(np.float32)
    return np.clip(np.rint(v.astype(np.float32)), 0, 255).astype(np.uint8)


def crop_offsets(shape, image_size, crop_mode, rng=np.random):
    """(row, col) offsets for one image of `shape` (image_preprocessor.py:18-31)."""
    if crop_mode == "random":
        return rng.randint(0, int(shape[0] - image_size[0])), rng.randint(0, int(shape[1] - image_size[1]))
    if crop_mode == "center":
        return int((shape[0] - image_size[0]) / 2), int((shape[1] - image_size[1]) / 2)
    return 0, 0


def preprocess(im, image_size, crop_mode=None, precrop_size=None, offsets=None):
    """One uint8 HWC image -> float32 CHW, image_preprocessor.py:16-39 (offsets given)."""
    if precrop_size is None:
        precrop_size = (int(image_size[0] * 1.25), int(image_size[1] * 1.25))
    if crop_mode in ("random", "center"):
        im = resize_bilinear(im, precrop_size[0], precrop_size[1])
        r, c = offsets
        im = im[r:r + image_size[0], c:c + image_size[1], :]
    else:
        im = resize_bilinear(im, image_size[0], image_size[1])
    out = im.astype(np.float32).transpose(2, 0, 1)
    out -= 128.0
    return out


def mixup(X, Xm, p):
    return p * Xm + (1 - p) * X, p * X + (1 - p) * Xm
