"""The urlencoded fast path (api/forms.py:_unquote_plus) equals urllib's parse_qsl on random bodies,
including percent-encoded data URLs (the reference's form field, app/main.py:46) and arbitrary text."""
import base64
import os
import random
import string
from urllib.parse import parse_qsl, quote, quote_plus

from deconv_api_amd.api.forms import parse_urlencoded


def _want(b: bytes):
    out = {}
    for k, v in parse_qsl(b.decode("utf-8", errors="replace"), keep_blank_values=True):
        out.setdefault(k, v)
    return out


def test_fast_urlencoded_equals_parse_qsl():
    rnd = random.Random(0)
    for _ in range(2000):
        fields = []
        for _ in range(rnd.randint(0, 4)):
            k = "".join(rnd.choice(string.ascii_letters + "_% +&=é") for _ in range(rnd.randint(0, 6)))
            v = rnd.choice(["data:image/png;base64," + base64.b64encode(os.urandom(rnd.randint(0, 300))).decode(),
                            "".join(rnd.choice(string.printable + "é中") for _ in range(rnd.randint(0, 30)))])
            fields.append((k, v))
        enc = [quote_plus, lambda s: quote(s, safe=""), lambda s: s]
        body = "&".join(rnd.choice(enc)(k) + "=" + rnd.choice(enc)(v) for k, v in fields)
        if rnd.random() < 0.1:
            body += "&&x%2b%2F%3d%zz%"
        assert parse_urlencoded(body.encode()) == _want(body.encode()), body


def test_fast_urlencoded_large_data_url():
    u = "data:image/jpeg;base64," + base64.b64encode(os.urandom(120_000)).decode()
    b = f"file={quote_plus(u)}&layer=block5_conv3".encode()
    got = parse_urlencoded(b)
    assert got == {"file": u, "layer": "block5_conv3"} == _want(b)
