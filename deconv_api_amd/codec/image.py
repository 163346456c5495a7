"""Image codec for the HTTP API: data-URL parsing, decode to RGB uint8, JPEG encode, data URL.

Reference behaviour being reproduced (rashanarshad/deconv_api):
  * ``readb64`` (app/main.py:35-39): ``uri.split(',')[1]``, lenient ``base64.b64decode`` (characters
    outside the alphabet are discarded), ``cv2.imdecode(..., IMREAD_COLOR)`` -> 3-channel 8-bit.
    Here PIL decodes (libjpeg-turbo / libpng / libwebp), EXIF orientation is applied like OpenCV's
    IMREAD_COLOR does, alpha is dropped and greyscale is expanded; the array is RGB, which is the
    slot order the reference's BGR decode + channel reversal produced.
  * encode (app/main.py:73-76): ``cv2.imencode('.jpg')`` (quality 95, 4:2:0), base64, then
    ``'data:image/webp;base64,' + urllib.parse.quote(b64)`` — the MIME type says webp but the
    payload is JPEG (quirk Q2) and ``quote`` escapes '+' and '=' (quirk Q3). The mosaic handed to
    the encoder is already channel-reversed on device (quirk Q4), so an RGB encoder writes the same
    colours OpenCV's BGR encoder wrote.
"""
from __future__ import annotations

import base64
import binascii
import io
import os
from urllib.parse import quote

import numpy as np
from PIL import Image, ImageOps, UnidentifiedImageError

DATA_URL_PREFIX = "data:image/webp;base64,"
JPEG_QUALITY = 95


class ImageDecodeError(ValueError):
    pass


def split_data_url(uri: str) -> str:
    parts = uri.split(",", 2)  # == uri.split(",")[1] (reference readb64), without splitting the payload
    if len(parts) < 2:
        raise ImageDecodeError("file must be a data URL ('data:<mime>;base64,<payload>')")
    return parts[1]


def b64decode_lenient(payload: str) -> bytes:
    try:
        return base64.b64decode(payload)  # validate=False: non-alphabet characters are discarded
    except (binascii.Error, ValueError) as e:
        raise ImageDecodeError(f"bad base64 payload: {e}") from e


# service-level cap on decoded pixels (far below PIL's decompression-bomb limit): a request can
# not make the server decode, pin and upload a ~500 MB image (DV_MAX_PIXELS)
MAX_PIXELS = int(os.environ.get("DV_MAX_PIXELS", str(64 << 20)))


def decode_image(data: bytes) -> np.ndarray:
    """bytes -> HxWx3 uint8 RGB (EXIF orientation applied, like cv2.imdecode IMREAD_COLOR)."""
    try:
        im = Image.open(io.BytesIO(data))
        if im.size[0] * im.size[1] > MAX_PIXELS:  # header only: nothing decoded yet
            raise ImageDecodeError(f"image too large: {im.size[0]}x{im.size[1]} > {MAX_PIXELS} pixels")
        ImageOps.exif_transpose(im, in_place=True)  # no copy when there is nothing to rotate
        if im.mode in ("I;16", "I;16B", "I;16L", "I"):
            arr = np.asarray(im, dtype=np.float64)
            arr = np.clip(arr / 257.0, 0, 255).astype(np.uint8)
            im = Image.fromarray(arr)
        if im.mode != "RGB":  # convert() to the same mode would be a full copy
            im = im.convert("RGB")
        arr = np.asarray(im, dtype=np.uint8)
    except Image.DecompressionBombError as e:
        raise ImageDecodeError(f"image too large: {e}") from e
    except (UnidentifiedImageError, OSError, SyntaxError, ValueError) as e:
        if isinstance(e, ImageDecodeError):
            raise
        raise ImageDecodeError(f"undecodable image: {e}") from e
    if arr.ndim != 3 or arr.shape[2] != 3 or arr.shape[0] < 1 or arr.shape[1] < 1:
        raise ImageDecodeError("decoded image has an unexpected shape")
    return np.ascontiguousarray(arr)


def read_data_url(uri: str) -> np.ndarray:
    """The reference's ``readb64``. With the extension built, the payload is split out and
    base64-decoded natively with the GIL released (csrc/jpeg_enc.cpp:data_url_b64decode, CPython's
    non-strict semantics and messages): the Python decode held the GIL ~0.24 ms per 60 KB request,
    serialized across the codec pool's threads."""
    lib = _native()
    if lib is not None and isinstance(uri, str) and uri.isascii():
        if "," not in uri:
            split_data_url(uri)  # raises the data-URL error
        try:
            data = lib.data_url_b64decode(uri)
        except ValueError as e:
            raise ImageDecodeError(f"bad base64 payload: {e}") from e
        return decode_image(data)
    return decode_image(b64decode_lenient(split_data_url(uri)))


def _native():
    """The native encoder (csrc/jpeg_enc.cpp) when the extension is built, else None."""
    global _NATIVE
    if _NATIVE is None:
        try:
            from ..ops import native

            _NATIVE = native.load() if native.available() else False
        except Exception:  # noqa: BLE001 - PIL fallback
            _NATIVE = False
    return _NATIVE or None


_NATIVE = None


def encode_jpeg_pil(rgb: np.ndarray, quality: int = JPEG_QUALITY) -> bytes:
    buf = io.BytesIO()
    Image.fromarray(np.ascontiguousarray(rgb)).save(buf, format="JPEG", quality=quality, subsampling=2)
    return buf.getvalue()


def encode_jpeg(rgb: np.ndarray, quality: int = JPEG_QUALITY) -> bytes:
    """Baseline JPEG (YCbCr 4:2:0, IJG tables) by the native encoder, which releases the GIL and
    scales across threads (PIL's holds it: one core's worth of encodes per process); PIL when
    the extension is not built."""
    lib = _native()
    if lib is None:
        return encode_jpeg_pil(rgb, quality)
    import torch

    return lib.jpeg_encode(torch.from_numpy(np.ascontiguousarray(rgb, dtype=np.uint8)), int(quality))


def encode_data_urls(mosaics: np.ndarray, quality: int = JPEG_QUALITY, threads: int = 8):
    """[B, H, W, 3] uint8 -> B response strings; native: one GIL-free call, images (or restart
    segments of them) spread over ``threads`` native threads."""
    lib = _native()
    if lib is None:
        return [encode_data_url(m, quality) for m in mosaics]
    import torch

    return lib.jpeg_data_urls(torch.from_numpy(np.ascontiguousarray(mosaics, dtype=np.uint8)), int(quality),
                              DATA_URL_PREFIX, int(threads))


def gpu_jpeg_fits(W: int) -> bool:
    """Whether ``encode_gpu`` takes images of width ``W`` (one MCU row per workgroup, in LDS)."""
    from ..ops import native

    return int(W) <= native.lib().jpeg_gpu_max_width()


def encode_gpu(mosaics, quality: int = JPEG_QUALITY):
    """uint8 [B, H, W, 3] DEVICE tensor -> (packed scans, offsets [B + 1]) device tensors: baseline
    JPEG on the GPU (csrc/jpeg_gpu.hip; restart marker per MCU row). Enqueued on the current stream;
    ``gpu_data_urls`` turns the host copies into response strings."""
    from ..ops import native

    return native.lib().jpeg_gpu(mosaics.contiguous(), int(quality))


def gpu_data_urls(packed, off, H: int, W: int, quality: int = JPEG_QUALITY, threads: int = 8):
    """Host copies of ``encode_gpu``'s outputs (only off[-1] bytes of ``packed`` are read) -> B data
    URLs (header + scan + EOI, base64, the reference's quote escaping), GIL released."""
    from ..ops import native

    return native.lib().jpeg_gpu_data_urls(packed, off, int(H), int(W), int(quality), DATA_URL_PREFIX, int(threads))


def gpu_jpeg_bytes(packed, off, b: int, H: int, W: int, quality: int = JPEG_QUALITY) -> bytes:
    """JPEG file of image ``b`` from host copies of ``encode_gpu``'s outputs (tests / tools)."""
    from ..ops import native

    o = off.tolist()
    return native.lib().jpeg_gpu_header(H, W, quality) + bytes(packed[o[b]:o[b + 1]].numpy()) + b"\xff\xd9"


def quote_b64(b64: str) -> str:
    """``urllib.parse.quote`` restricted to base64 text: letters, digits and '/' are kept, so only
    '+' -> '%2B' and '=' -> '%3D' change. Identical output, C-speed (quote() walks the ~100 KB
    string in Python and capped the service at ~200 req/s)."""
    return b64.replace("+", "%2B").replace("=", "%3D")


def to_data_url(jpeg: bytes) -> str:
    return DATA_URL_PREFIX + quote_b64(base64.b64encode(jpeg).decode("ascii"))


def encode_data_url(rgb: np.ndarray, quality: int = JPEG_QUALITY) -> str:
    return to_data_url(encode_jpeg(rgb, quality))


def parse_result_data_url(s: str) -> np.ndarray:
    """Inverse of ``encode_data_url`` (tests / clients)."""
    from urllib.parse import unquote

    assert s.startswith(DATA_URL_PREFIX)
    return decode_image(base64.b64decode(unquote(s[len(DATA_URL_PREFIX):])))


def make_data_url(rgb: np.ndarray, fmt: str = "PNG") -> str:
    """Client helper: an image -> 'data:image/<fmt>;base64,...' as a browser would send it."""
    buf = io.BytesIO()
    Image.fromarray(rgb).save(buf, format=fmt)
    return f"data:image/{fmt.lower()};base64," + base64.b64encode(buf.getvalue()).decode("ascii")
