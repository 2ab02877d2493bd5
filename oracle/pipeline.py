"""TEST INFRASTRUCTURE ONLY -- the checker for the device-side input pipeline.  Imported by
tests/ only; the product path (dorknet_amd/data_loading) never calls it.

numpy restatement of the reference's per-image preprocessing and mixup:

- preprocess(im): data_loading/image_preprocessor.py:16-39 -- cv2.resize (INTER_LINEAR), crop
  ("random": offsets drawn per image, row then column, np.random.randint(0, max_offset);
  "center": int((size - crop) / 2)), astype(float32), transpose(2, 0, 1), - 128.0.  The
  augmenter call (:33-34) discards its result in the reference, so augmentation has no effect
  and is not restated.
- resize_bilinear(im, OW, OH): cv2.resize INTER_LINEAR for uint8 as OpenCV 4.3 (the reference's
  pin, requirements.txt: opencv-python==4.3.0.36) computes it in imgproc/src/resize.cpp's generic
  path: the geometry above, 11-bit fixed-point weights (INTER_RESIZE_COEF_BITS), an integer
  horizontal pass and the FixedPtCast vertical rounding, INTER_AREA for an exact 2x downscale.
  cv2 is not installed here, so agreement with cv2 itself is parity unpinned (OpenCV's x86 SIMD
  vertical pass can differ in the last bit); this restatement pins the GPU kernel bit for bit.
- mixup(X, Xm, p): data_loading/image_data_loader.py:101-111 -- p * X_m + (1 - p) * X and the
  mirror, numpy semantics (a Python float times a float32 array stays float32).
"""
from __future__ import annotations

import numpy as np


def _axis(O, L, is_x):
    """cv::resize INTER_LINEAR coordinates and 11-bit weights (imgproc/src/resize.cpp, OpenCV 4.3):
    scale = 1 / (O / L); f = float((o + 0.5) * scale - 0.5); s = floor(f); f -= s.  x axis: s < 0 ->
    (0, 0); s >= L - 1 -> (L - 1, 0); outputs at or past the first s + 1 >= L take src[s] * 2048.
    y axis: no weight clamping, the two rows clipped to [0, L - 1].  Weights cvRound((1 - f) * 2048),
    cvRound(f * 2048) (round half to even)."""
    scale = 1.0 / (O / L)
    f = ((np.arange(O, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    s = np.floor(f).astype(np.int64)
    f = (f - s.astype(np.float32)).astype(np.float32)
    if is_x:
        lo = s < 0
        s[lo], f[lo] = 0, 0
        edge = s + 1 >= L
        hi = s >= L - 1
        s[hi], f[hi] = L - 1, 0
    a0 = np.rint((np.float32(1) - f) * np.float32(2048)).astype(np.int64)
    a1 = np.rint(f * np.float32(2048)).astype(np.int64)
    if is_x:
        a0[edge], a1[edge] = 2048, 0
    return np.clip(s, 0, L - 1), np.clip(s + 1, 0, L - 1), a0, a1


def resize_bilinear(im, OW, OH):
    """cv2.resize(im, (OW, OH)) with INTER_LINEAR for uint8 (H, W, C) -> uint8 (OH, OW, C): OpenCV's
    fixed-point path -- integer horizontal pass S = src[x0] * a0 + src[x1] * a1, vertical
    FixedPtCast (S0 * b0 + S1 * b1 + 2^21) >> 22 saturated; an exact 2x downscale of both axes is
    INTER_AREA ((a + b + c + d + 2) >> 2); the same size is a copy."""
    H, W = im.shape[:2]
    if (OH, OW) == (H, W):
        return im.copy()
    sy, sx = 1.0 / (OH / H), 1.0 / (OW / W)
    eps = np.finfo(np.float64).eps
    if abs(sx - round(sx)) < eps and abs(sy - round(sy)) < eps and round(sx) == 2 and round(sy) == 2:
        v = im.astype(np.int64)
        t = v[0:2 * OH:2, 0:2 * OW:2] + v[0:2 * OH:2, 1:2 * OW:2] + v[1:2 * OH:2, 0:2 * OW:2] + v[1:2 * OH:2, 1:2 * OW:2]
        return ((t + 2) >> 2).astype(np.uint8)
    y0, y1, b0, b1 = _axis(OH, H, False)
    x0, x1, a0, a1 = _axis(OW, W, True)
    v = im.astype(np.int64)
    A0, A1 = a0[None, :, None], a1[None, :, None]
    S0 = v[y0][:, x0] * A0 + v[y0][:, x1] * A1
    S1 = v[y1][:, x0] * A0 + v[y1][:, x1] * A1
    out = (S0 * b0[:, None, None] + S1 * b1[:, None, None] + (1 << 21)) >> 22
    return np.clip(out, 0, 255).astype(np.uint8)


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
