"""GPU baseline JPEG encoder (csrc/jpeg_gpu.hip) vs the host encoder (csrc/jpeg_enc.cpp) and the
decoded pixels: valid JFIF streams (PIL decodes them), one restart marker per MCU row, decoded
images within JPEG-rounding distance of the host encoder's and close to the source."""
import io
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _psnr(a, b):
    mse = float(((a.astype(np.float64) - b.astype(np.float64)) ** 2).mean())
    return math.inf if mse == 0 else 10 * math.log10(255.0 ** 2 / mse)


def _images(B, H, W, seed):
    g = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:H, 0:W]
    out = []
    for b in range(B):
        base = np.stack([(xx * (b + 1)) % 256, (yy * 2) % 256, ((xx + yy) * 3) % 256], -1).astype(np.float64)
        if b % 3 == 1:
            base = g.integers(0, 256, (H, W, 3)).astype(np.float64)  # noise: worst case for the coder
        elif b % 3 == 2:
            base = np.clip(base * 0.5 + g.normal(0, 20, (H, W, 3)), 0, 255)
        out.append(base.astype(np.uint8))
    out[0][:8, :8] = 255  # saturated blocks: 0xFF bytes to stuff
    return np.stack(out)


@pytest.mark.parametrize("B,H,W", [(3, 448, 448), (4, 100, 70), (2, 17, 33)])
def test_gpu_jpeg_decodes_close_to_host_encoder(native_lib, B, H, W):
    from PIL import Image

    from deconv_api_amd.codec import image as ci

    imgs = _images(B, H, W, B + H)
    packed, off = ci.encode_gpu(torch.from_numpy(imgs).cuda(), 95)
    torch.cuda.synchronize()
    off_h = off.cpu()
    n = int(off_h[-1])
    packed_h = packed[:n].cpu()
    for b in range(B):
        jpg = ci.gpu_jpeg_bytes(packed_h, off_h, b, H, W, 95)
        assert jpg[:2] == b"\xff\xd8" and jpg[-2:] == b"\xff\xd9"
        mcuy = (H + 15) // 16
        scan = bytes(packed_h[int(off_h[b]):int(off_h[b + 1])].numpy())
        assert sum(scan.count(bytes([0xFF, 0xD0 + m])) for m in range(8)) == mcuy - 1
        got = np.asarray(Image.open(io.BytesIO(jpg)).convert("RGB"))
        ref = np.asarray(Image.open(io.BytesIO(ci.encode_jpeg(imgs[b], 95))).convert("RGB"))
        assert got.shape == (H, W, 3)
        assert _psnr(got, ref) > 38.0, (b, _psnr(got, ref))
        # as faithful to the source as the host encoder (same tables, same 4:2:0 subsampling)
        assert _psnr(got, imgs[b]) > _psnr(ref, imgs[b]) - 0.5, (b, _psnr(got, imgs[b]), _psnr(ref, imgs[b]))


def test_gpu_jpeg_data_urls(native_lib):
    from deconv_api_amd.codec import image as ci

    imgs = _images(3, 448, 448, 7)
    packed, off = ci.encode_gpu(torch.from_numpy(imgs).cuda())
    off_h = off.cpu()
    urls = ci.gpu_data_urls(packed[: int(off_h[-1])].cpu(), off_h, 448, 448)
    assert len(urls) == 3
    for b, (u, im) in enumerate(zip(urls, imgs)):
        assert u.startswith("data:image/webp;base64,") and "+" not in u and "=" not in u
        dec = ci.parse_result_data_url(u)
        ref = ci.parse_result_data_url(ci.encode_data_url(im, 95))  # the host encoder's response
        assert dec.shape == (448, 448, 3) and _psnr(dec, ref) > 38.0, (b, _psnr(dec, ref))


def test_gpu_jpeg_many_segments_and_width_limit(native_lib):
    """> 1024 segments in one batch (the offsets kernel's chunked scan) and the width limit."""
    from PIL import Image

    from deconv_api_amd.codec import image as ci

    B, H, W = 40, 448, 448
    imgs = _images(B, H, W, 11)
    packed, off = ci.encode_gpu(torch.from_numpy(imgs).cuda(), 95)
    off_h = off.cpu()
    assert int(off_h[0]) == 0 and bool((off_h[1:] > off_h[:-1]).all())
    packed_h = packed[: int(off_h[-1])].cpu()
    for b in (0, 1, 38, 39):
        got = np.asarray(Image.open(io.BytesIO(ci.gpu_jpeg_bytes(packed_h, off_h, b, H, W, 95))).convert("RGB"))
        ref = np.asarray(Image.open(io.BytesIO(ci.encode_jpeg(imgs[b], 95))).convert("RGB"))
        assert _psnr(got, ref) > 38.0, (b, _psnr(got, ref))
    wmax = native_lib.jpeg_gpu_max_width()
    assert ci.gpu_jpeg_fits(wmax) and not ci.gpu_jpeg_fits(wmax + 1)
    with pytest.raises(RuntimeError):
        ci.encode_gpu(torch.zeros(1, 16, wmax + 16, 3, dtype=torch.uint8, device="cuda"))
