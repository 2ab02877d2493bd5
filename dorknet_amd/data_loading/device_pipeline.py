"""Device-side input pipeline (SURVEY.md section 8 f, row 4).

Reference: ``ImagePreprocessor`` (data_loading/image_preprocessor.py:4-39) turns one decoded
uint8 HWC image into the float32 CHW array the network eats -- cv2.resize (INTER_LINEAR) to the
pre-crop size, a random or centred crop, ``astype(float32).transpose(2, 0, 1) - 128`` -- and
``ImageDataLoader.load_batch`` (data_loading/image_data_loader.py:88-117) stacks a batch of
them on the host (a thread pool over cv2) and optionally mixes two batches up.

Here the batch is one uint8 NHWC tensor on the GPU (decoded images of one size, e.g. straight
from the decoder); resize, crop, cast, layout change and the -128 shift run as HIP kernels
(dorknet_amd/csrc/input_pipeline.hip) and the result is the reference's X_batch layout, fp32
NCHW, already in HBM -- 4x fewer bytes over PCIe than shipping the fp32 batch.

- ``DeviceImagePreprocessor(image_size, crop_mode=None, precrop_size=None, image_augmenter=None)``:
  the reference constructor; ``preprocess_batch(images)`` is ``np.stack([preprocess_image(im)
  for im in images])``.  Crop offsets are drawn exactly as the reference draws them
  (np.random.randint per image, row then column).  The reference calls the augmenter but
  discards its result (image_preprocessor.py:33-34), so augmentation never reaches the
  network; ``image_augmenter`` is accepted and, likewise, has no effect.
- ``mixup_batches(X, X_m, y, y_m, prop)``: the mixup step of load_batch (:101-111) for images
  and one-hot labels, returning both mixed batches.

Decoding (cv2.imread) and file I/O stay on the host.  The resize restates cv2.resize's uint8
INTER_LINEAR as OpenCV 4.3 (the reference's pin) defines it: 11-bit fixed-point weights, integer
horizontal pass, FixedPtCast vertical rounding, INTER_AREA for an exact 2x downscale -- integer
work, bit-exact to oracle/pipeline.py.  cv2 is not in this image to pin against (its x86 SIMD
vertical pass can round differently in the last bit), so agreement with cv2 itself is parity
unpinned.  Crop, cast, layout and mixup are exact.
"""
from __future__ import annotations

import numpy as np
import torch

from .._hip import lib, stream_handle


def _u8_device(images) -> torch.Tensor:
    if isinstance(images, torch.Tensor):
        t = images
    else:
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(images, dtype=np.uint8)))
    if t.dtype != torch.uint8 or t.dim() != 4:
        raise ValueError("images must be a uint8 (N, H, W, C) batch, got {} {}".format(t.dtype, tuple(t.shape)))
    return t.to(device="cuda", non_blocking=True).contiguous()


class DeviceImagePreprocessor:
    def __init__(self, image_size, crop_mode=None, precrop_size=None, image_augmenter=None):
        self.image_size = image_size  # as in the reference: [0] rows of the crop, [1] columns
        self.crop_mode = crop_mode
        self.precrop_size = precrop_size if precrop_size is not None else (int(image_size[0] * 1.25),
                                                                           int(image_size[1] * 1.25))
        self.image_augmenter = image_augmenter  # no effect, as in the reference (see module doc)

    def _resize(self, x, size):
        """cv2.resize(im, size): size = (width, height)."""
        N, H, W, C = x.shape
        OW, OH = int(size[0]), int(size[1])
        if (OH, OW) == (H, W):
            return x
        out = torch.empty((N, OH, OW, C), dtype=torch.uint8, device=x.device)
        lib.dk_resize_bilinear_u8(x.data_ptr(), N, H, W, C, OH, OW, out.data_ptr(), stream_handle())
        return out

    def crop_offsets(self, n, shape, rng=np.random):
        """(row, col) per image, drawn as image_preprocessor.py:18-27 draws them."""
        rows, cols = int(self.image_size[0]), int(self.image_size[1])
        if self.crop_mode == "random":
            out = []
            for _ in range(n):
                r = rng.randint(0, int(shape[0] - rows))
                c = rng.randint(0, int(shape[1] - cols))
                out.append((r, c))
            return np.asarray(out, dtype=np.int32)
        if self.crop_mode == "center":
            return np.tile(np.asarray([[int((shape[0] - rows) / 2), int((shape[1] - cols) / 2)]], np.int32), (n, 1))
        return None

    def preprocess_batch(self, images, rng=np.random, offsets=None):
        """uint8 (N, H, W, C) batch -> fp32 (N, C, rows, cols) on the GPU."""
        x = _u8_device(images)
        N, _, _, C = x.shape
        if self.crop_mode in ("random", "center"):
            x = self._resize(x, self.precrop_size)
            rows, cols = int(self.image_size[0]), int(self.image_size[1])
            if offsets is None:
                offsets = self.crop_offsets(N, x.shape[1:3], rng)
            crop = torch.as_tensor(np.asarray(offsets, dtype=np.int32).reshape(N, 2), device=x.device)
        else:
            x = self._resize(x, self.image_size)
            rows, cols = x.shape[1], x.shape[2]
            crop = None
        H, W = x.shape[1], x.shape[2]
        if rows > H or cols > W:
            raise ValueError("crop {}x{} larger than the resized image {}x{}".format(rows, cols, H, W))
        out = torch.empty((N, C, rows, cols), dtype=torch.float32, device=x.device)
        lib.dk_u8_nhwc_to_nchw_f32(x.data_ptr(), N, H, W, C, crop.data_ptr() if crop is not None else 0, rows, cols,
                                   128.0, out.data_ptr(), stream_handle())
        self._keep = (x, crop)  # alive until the stream has run the kernels
        return out


def mixup_batches(X, X_m, y, y_m, prop):
    """image_data_loader.py:101-111: (X_mixed, X_mixed_m, y_mixed, y_mixed_m) with
    X_mixed = prop * X_m + (1 - prop) * X and the mirror; fp32 device tensors in and out."""
    p = np.float32(prop)
    q = np.float32(1 - prop)
    outs = []
    for a, b in ((X, X_m), (y, y_m)):
        a, b = a.contiguous(), b.contiguous()
        if a.shape != b.shape or a.dtype != torch.float32 or b.dtype != torch.float32:
            raise ValueError("mixup needs two fp32 tensors of one shape")
        ab, ba = torch.empty_like(a), torch.empty_like(a)
        lib.dk_mixup_f32(a.data_ptr(), b.data_ptr(), a.numel(), float(p), float(q), ab.data_ptr(), ba.data_ptr(),
                         stream_handle())
        outs.append((ab, ba))
    (xm, xmm), (ym, ymm) = outs
    return xm, xmm, ym, ymm
