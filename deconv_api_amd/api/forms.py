"""HTML form body parsing without python-multipart (not installed; FastAPI ``Form(...)`` routes
cannot even be declared without it). Covers what the reference's
``Form(...)`` parameters accepted (app/main.py:46): application/x-www-form-urlencoded and
multipart/form-data (RFC 7578)."""
from __future__ import annotations

from typing import Dict, Optional
from urllib.parse import parse_qsl, unquote_plus


class FormError(ValueError):
    pass


def _param(header_value: str, key: str) -> Optional[str]:
    for part in header_value.split(";")[1:]:
        if "=" in part:
            k, v = part.split("=", 1)
            if k.strip().lower() == key:
                v = v.strip()
                if len(v) >= 2 and v[0] == v[-1] == '"':
                    v = v[1:-1].replace('\\"', '"')
                return v
    return None


def _native_unquote():
    """The extension's GIL-free ``url_unquote_plus`` when built (front ends load it anyway for the
    native base64 decoder), else None."""
    global _NATIVE_UQ
    if _NATIVE_UQ is None:
        _NATIVE_UQ = False
        try:
            from ..ops import native

            if native.available():
                _NATIVE_UQ = getattr(native.lib(), "url_unquote_plus", False)
        except Exception:  # noqa: BLE001 - the urllib path
            pass
    return _NATIVE_UQ or None


_NATIVE_UQ = None


def _unquote_plus(v: str) -> str:
    """``urllib.parse.unquote_plus``; ASCII values (every percent-encoded data URL) go through the
    native decoder: unquote's per-escape Python loop held the GIL ~2-3 ms per ~180 KB request."""
    if "%" not in v:
        return v.replace("+", " ")
    fn = _native_unquote() if v.isascii() else None
    if fn is None:
        return unquote_plus(v)
    return fn(v).decode("utf-8", "replace")


def parse_urlencoded(body: bytes, charset: str = "utf-8") -> Dict[str, str]:
    """'+' decodes to a space and %XX to bytes, as browsers/python-multipart do; the first value
    of a repeated field wins."""
    txt = body.decode(charset, errors="replace")
    out: Dict[str, str] = {}
    if "%" in txt and charset.lower().replace("-", "") == "utf8":
        for pair in txt.split("&"):
            if not pair:
                continue
            k, _, v = pair.partition("=")
            out.setdefault(_unquote_plus(k), _unquote_plus(v))
        return out
    for k, v in parse_qsl(txt, keep_blank_values=True):
        out.setdefault(k, v)
    return out


def parse_multipart(body: bytes, content_type: str) -> Dict[str, str]:
    boundary = _param(content_type, "boundary")
    if not boundary:
        raise FormError("multipart body without boundary")
    delim = b"--" + boundary.encode("latin-1")
    out: Dict[str, str] = {}
    parts = body.split(delim)
    if len(parts) < 2:
        raise FormError("multipart boundary not found in body")
    for part in parts[1:]:
        if part.startswith(b"--"):
            break  # closing delimiter
        if part.startswith(b"\r\n"):
            part = part[2:]
        elif part.startswith(b"\n"):
            part = part[1:]
        sep = part.find(b"\r\n\r\n")
        sl = 4
        if sep < 0:
            sep = part.find(b"\n\n")
            sl = 2
        if sep < 0:
            raise FormError("malformed multipart part (no header/body separator)")
        raw_headers = part[:sep].decode("latin-1")
        data = part[sep + sl:]
        if data.endswith(b"\r\n"):
            data = data[:-2]
        elif data.endswith(b"\n"):
            data = data[:-1]
        name = None
        charset = "utf-8"
        for line in raw_headers.splitlines():
            if ":" not in line:
                continue
            hk, hv = line.split(":", 1)
            hk = hk.strip().lower()
            if hk == "content-disposition":
                name = _param(hv, "name")
            elif hk == "content-type":
                charset = _param(hv, "charset") or charset
        if name is None:
            continue
        try:
            out.setdefault(name, data.decode(charset, errors="replace"))
        except LookupError as e:  # unknown charset name in the part's content-type
            raise FormError(f"unknown charset {charset!r} in multipart field {name!r}") from e
    return out


def parse_form(body: bytes, content_type: Optional[str]) -> Dict[str, str]:
    ct = (content_type or "").lower()
    if ct.startswith("multipart/form-data"):
        return parse_multipart(body, content_type or "")
    if ct.startswith("application/x-www-form-urlencoded") or not ct:
        return parse_urlencoded(body)
    raise FormError(f"unsupported content type {content_type!r}")


def encode_multipart(fields: Dict[str, str], boundary: str = "dvboundary7MA4YWxkTrZu0gW") -> tuple:
    """Client helper (tests, bench): -> (body bytes, content-type)."""
    lines = []
    for k, v in fields.items():
        lines.append(f"--{boundary}\r\nContent-Disposition: form-data; name=\"{k}\"\r\n\r\n{v}\r\n")
    lines.append(f"--{boundary}--\r\n")
    return "".join(lines).encode(), f"multipart/form-data; boundary={boundary}"
