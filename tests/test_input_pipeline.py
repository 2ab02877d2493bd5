"""Device-side input pipeline: the oracle restatement of the reference's
preprocessing on CPU (analytic cases), and the HIP kernels bit-exact against it on the GPU.
The resize restates cv2's INTER_LINEAR for uint8 (11-bit fixed point, OpenCV 4.3); cv2 itself
is not installed, so agreement with cv2 is unpinned; the geometry and the exact cases below pin
the restatement."""
import numpy as np
import pytest

from oracle import pipeline as op


def test_resize_identity_and_constant():
    rng = np.random.RandomState(0)
    im = rng.randint(0, 256, size=(7, 9, 3)).astype(np.uint8)
    assert np.array_equal(op.resize_bilinear(im, 9, 7), im)            # same size: the pixels
    c = np.full((5, 6, 3), 77, np.uint8)
    assert np.array_equal(op.resize_bilinear(c, 13, 11), np.full((11, 13, 3), 77, np.uint8))


def test_resize_2x_upsample_geometry():
    # cv2 INTER_LINEAR, 1-D 2x upsample of [0, 100]: source x = (o + 0.5) / 2 - 0.5
    # -> [-0.25 (clamped: 0), 0.25, 0.75, 1.25 (clamped: last)] -> [0, 25, 75, 100]
    im = np.array([[[0], [100]]], np.uint8)
    out = op.resize_bilinear(im, 4, 1)
    assert out[0, :, 0].tolist() == [0, 25, 75, 100]


def test_resize_2x_downsample_averages_pairs():
    # source x = (o + 0.5) * 2 - 0.5 = 2o + 0.5: weights 1024/1024, the mean of each pixel pair,
    # fixed-point rounding half up ((S * 2048 + 2^21) >> 22)
    row = np.array([10, 20, 30, 41, 0, 255], np.uint8)
    out = op.resize_bilinear(row.reshape(1, 6, 1), 3, 1)
    assert out[0, :, 0].tolist() == [15, 36, 128]   # 15, 35.5 -> 36, 127.5 -> 128


def test_resize_exact_2x_is_area():
    # an exact 2x downscale of both axes is INTER_AREA in cv::resize: (a + b + c + d + 2) >> 2
    im = np.array([[1, 2, 200, 201], [3, 5, 202, 255], [0, 0, 9, 9], [0, 1, 9, 10]], np.uint8)[:, :, None]
    out = op.resize_bilinear(im, 2, 2)[:, :, 0]
    assert out.tolist() == [[(1 + 2 + 3 + 5 + 2) >> 2, (200 + 201 + 202 + 255 + 2) >> 2], [0, (9 + 9 + 9 + 10 + 2) >> 2]]


def test_resize_fixed_point_weights():
    # 3 -> 2 pixels: scale 1.5, x = 0.25 and 1.75: weights cvRound(0.75 * 2048) = 1536 / 512 and
    # 512 / 1536; (S * 2048 + 2^21) >> 22
    row = np.array([0, 100, 201], np.uint8).reshape(1, 3, 1)
    out = op.resize_bilinear(row, 2, 1)[0, :, 0]
    s0 = 0 * 1536 + 100 * 512
    s1 = 100 * 512 + 201 * 1536
    assert out.tolist() == [(s0 * 2048 + (1 << 21)) >> 22, (s1 * 2048 + (1 << 21)) >> 22]


def test_preprocess_center_crop_matches_reference_formula():
    rng = np.random.RandomState(1)
    im = rng.randint(0, 256, size=(20, 20, 3)).astype(np.uint8)
    out = op.preprocess(im, (16, 16), "center", precrop_size=(20, 20), offsets=(2, 2))
    ref = im[2:18, 2:18, :].astype(np.float32).transpose(2, 0, 1) - 128.0
    assert out.dtype == np.float32 and np.array_equal(out, ref)


def test_mixup_formula():
    rng = np.random.RandomState(2)
    X, Xm = rng.randn(3, 4).astype(np.float32), rng.randn(3, 4).astype(np.float32)
    a, b = op.mixup(X, Xm, 0.3)
    assert a.dtype == np.float32
    assert np.array_equal(a, np.float32(0.3) * Xm + np.float32(1 - 0.3) * X)
    assert np.array_equal(b, np.float32(0.3) * X + np.float32(1 - 0.3) * Xm)


@pytest.mark.gpu
@pytest.mark.parametrize("crop_mode,size,src", [("random", (48, 48), (97, 83)), ("center", (32, 32), (40, 40)),
                                                 (None, (33, 29), (17, 71)), ("random", (225, 225), (300, 410))])
def test_device_preprocess_bit_exact(crop_mode, size, src):
    import torch
    from dorknet_amd.data_loading.device_pipeline import DeviceImagePreprocessor
    rng = np.random.RandomState(3)
    N = 5
    ims = rng.randint(0, 256, size=(N, src[0], src[1], 3)).astype(np.uint8)
    pp = DeviceImagePreprocessor(size, crop_mode=crop_mode)
    offs = pp.crop_offsets(N, (pp.precrop_size[1], pp.precrop_size[0]), np.random.RandomState(9)) \
        if crop_mode else None
    got = pp.preprocess_batch(torch.as_tensor(ims), offsets=offs).cpu().numpy()
    want = np.stack([op.preprocess(ims[i], size, crop_mode, offsets=None if offs is None else tuple(offs[i]))
                     for i in range(N)])
    assert got.shape == want.shape and np.array_equal(got, want)


@pytest.mark.gpu
def test_device_resize_bit_exact_many_scales():
    import torch
    from dorknet_amd._hip import lib, stream_handle
    rng = np.random.RandomState(4)
    for (H, W, OH, OW) in [(225, 225, 281, 281), (300, 200, 225, 225), (10, 10, 3, 7), (1, 5, 4, 9), (31, 17, 31, 40),
                           (40, 60, 20, 30), (375, 500, 281, 281), (7, 9, 7, 9)]:
        im = rng.randint(0, 256, size=(2, H, W, 3)).astype(np.uint8)
        x = torch.as_tensor(im, device="cuda")
        y = torch.empty((2, OH, OW, 3), dtype=torch.uint8, device="cuda")
        lib.dk_resize_bilinear_u8(x.data_ptr(), 2, H, W, 3, OH, OW, y.data_ptr(), stream_handle())
        got = y.cpu().numpy()
        for n in range(2):
            assert np.array_equal(got[n], op.resize_bilinear(im[n], OW, OH)), (H, W, OH, OW)


@pytest.mark.gpu
def test_device_mixup_bit_exact():
    import torch
    from dorknet_amd.data_loading.device_pipeline import mixup_batches
    rng = np.random.RandomState(5)
    X, Xm = rng.randn(4, 3, 8, 8).astype(np.float32), rng.randn(4, 3, 8, 8).astype(np.float32)
    y, ym = np.eye(10, dtype=np.float32)[[1, 2, 3, 4]], np.eye(10, dtype=np.float32)[[5, 6, 7, 8]]
    p = float(rng.uniform(0.1, 0.4))
    d = lambda a: torch.as_tensor(a, device="cuda")
    outs = [t.cpu().numpy() for t in mixup_batches(d(X), d(Xm), d(y), d(ym), p)]
    want = list(op.mixup(X, Xm, p)) + list(op.mixup(y, ym, p))
    for g, w in zip(outs, want):
        assert np.array_equal(g, w)
