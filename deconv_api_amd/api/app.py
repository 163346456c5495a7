"""FastAPI application with the reference's HTTP surface (app/main.py:19-78):

  GET  /health-check -> {"healthy": "true"}                                   (main.py:41-43)
  POST /             form fields ``file`` (image data URL) and ``layer`` -> JSON string
                     ``"data:image/webp;base64,<quoted base64 JPEG>"`` of the 2x2 mosaic
                     of the top-4 deconvnet reconstructions                    (main.py:45-78)
  CORS: every origin, no credentials, all methods/headers                    (main.py:22-32)
  /docs, /redoc, /openapi.json (FastAPI built-ins; the form body is declared by hand because
  ``Form(...)`` needs python-multipart, which is not installed)

Extensions: GET /ready (per-device status), GET /metrics (Prometheus text), GET /layers,
POST /deepdream (when the DeepDream engine is available).

Error handling differs deliberately from the reference (which 500s on all of these):
missing fields -> 422 (FastAPI's own validation shape), undecodable image / malformed data URL /
unknown layer -> 400, queue full -> 503; fewer than 4 positive filters -> black tiles.
"""
from __future__ import annotations

import time
from typing import Optional

from fastapi import FastAPI, Request
from fastapi.middleware.cors import CORSMiddleware
from fastapi.responses import JSONResponse, PlainTextResponse, Response

from ..codec import ImageDecodeError
from ..config import Config
from ..engine.deconvnet import UnknownLayerError
from ..utils import metrics as M
from ..utils.logging import get_logger, new_request_id, setup
from .forms import FormError, parse_form

log = get_logger("deconv_api_amd.api")

_FORM_SCHEMA = {
    "requestBody": {
        "required": True,
        "content": {
            ct: {"schema": {"title": "Body_return_deconv__post", "type": "object", "required": ["file", "layer"],
                            "properties": {"file": {"title": "File", "type": "string"},
                                           "layer": {"title": "Layer", "type": "string"}}}}
            for ct in ("application/x-www-form-urlencoded", "multipart/form-data")
        },
    }
}


def _missing(fields):
    return JSONResponse(status_code=422, content={"detail": [
        {"loc": ["body", f], "msg": "field required", "type": "value_error.missing"} for f in fields]})


def _json_string_response(url) -> Response:
    """The route's JSON string body without ``json.dumps``: the service's data URLs (the prefix, then
    base64 with the reference's '%2B' / '%3D' escapes, from csrc/jpeg_enc.cpp or codec/image.py) hold
    nothing JSON would escape, so the body is the text in quotes. (JSONResponse's encoder walked the
    ~100 KB string at ~0.7 ms per request, the largest GIL cost of a front end; a regex scan for control
    characters cost as much.) Anything else takes JSONResponse."""
    b = url if isinstance(url, (bytes, bytearray)) else url.encode("utf-8")
    if b.startswith(_PREFIX) and b.isascii() and b'"' not in b and b"\\" not in b:
        return Response(content=b'"' + b + b'"', media_type="application/json")
    return JSONResponse(content=url if isinstance(url, str) else bytes(b).decode("utf-8", "replace"))


_PREFIX = b"data:image/webp;base64,"


def create_app(service=None, cfg: Optional[Config] = None, dream_service=None) -> FastAPI:
    cfg = cfg or Config.from_env()
    setup(cfg.log_json)
    app = FastAPI()
    app.add_middleware(CORSMiddleware, allow_origins=list(cfg.cors_origins), allow_credentials=False,
                       allow_methods=["*"], allow_headers=["*"])
    state = {"service": service, "dream": dream_service}

    def get_service():
        if state["service"] is None:
            from ..serve.service import DeconvService

            state["service"] = DeconvService(cfg)
        return state["service"]

    app.state.get_service = get_service

    if cfg.asyncio_debug:  # asyncio debug mode (blocking callbacks, unawaited coroutines)
        @app.on_event("startup")
        async def _loop_debug():
            import asyncio

            loop = asyncio.get_running_loop()
            loop.set_debug(True)
            loop.slow_callback_duration = cfg.slow_callback_ms / 1000.0
            app.state.loop_debug = True

    @app.get("/health-check")
    def healthcheck():
        M.REQUESTS.inc(route="/health-check", status="200")
        return {"healthy": "true"}

    @app.post("/", openapi_extra=_FORM_SCHEMA)
    async def return_deconv(request: Request):
        rid = new_request_id()
        t0 = time.perf_counter()
        status, layer = "200", "-"
        try:
            try:
                form = parse_form(await request.body(), request.headers.get("content-type"))
            except FormError as e:
                status = "400"
                return JSONResponse(status_code=400, content={"detail": str(e)})
            missing = [f for f in ("file", "layer") if f not in form]
            if missing:
                status = "422"
                return _missing(missing)
            layer = form["layer"]
            svc = get_service()
            try:
                url = await svc.deconv(form["file"], layer)
            except UnknownLayerError as e:
                status = "400"
                return JSONResponse(status_code=400, content={"detail": str(e).strip('"')})
            except ImageDecodeError as e:
                status = "400"
                return JSONResponse(status_code=400, content={"detail": str(e)})
            except Exception as e:  # noqa: BLE001
                from ..serve.service import ServiceOverloaded

                code = getattr(e, "status", None)  # serve/frontend.py RemoteError: the GPU owner's answer
                if isinstance(code, int) and code != 500:
                    status = str(code)
                    return JSONResponse(status_code=code, content={"detail": str(e)})

                if isinstance(e, ServiceOverloaded):
                    status = "503"
                    return JSONResponse(status_code=503, content={"detail": str(e)})
                status = "500"
                log.exception("deconv request failed", extra={"fields": {"request_id": rid}})
                return JSONResponse(status_code=500, content={"detail": "internal error"})
            return _json_string_response(url)
        finally:
            M.REQUESTS.inc(route="/", status=status)
            M.LATENCY.observe(time.perf_counter() - t0, route="/", layer=layer)

    @app.get("/ready")
    def ready():
        svc = state["service"]
        if svc is None:
            return JSONResponse(status_code=503, content={"ready": False, "reason": "service not started"})
        st = svc.status()
        ok = st.get("worker_alive", False)
        if state["dream"] is not None and hasattr(state["dream"], "status"):
            st["deepdream"] = state["dream"].status()  # world it runs tiled across, tile size
        return JSONResponse(status_code=200 if ok else 503, content={"ready": ok, **st})

    @app.get("/metrics")
    def metrics():
        svc = state["service"]
        # a front-end process (serve/frontend.py) adds its GPU owner's batch / GPU-stage series
        txt = svc.metrics_text() if hasattr(svc, "metrics_text") else M.REGISTRY.render()
        return PlainTextResponse(txt, media_type="text/plain; version=0.0.4")

    @app.get("/layers")
    def layers():
        return {"layers": get_service().layer_names()}

    @app.post("/deepdream", openapi_extra=_FORM_SCHEMA)
    async def deepdream(request: Request):
        """Extension (not in the reference): DeepDream of the uploaded image. Form fields: file,
        optional model (inception_v3 | resnet50), octaves, steps. Same data-URL conventions."""
        t0 = time.perf_counter()
        status = "200"
        try:
            try:
                form = parse_form(await request.body(), request.headers.get("content-type"))
                if "file" not in form:
                    status = "422"
                    return _missing(["file"])
                model = form.get("model", "inception_v3")
                octaves, steps = int(form.get("octaves", 4)), int(form.get("steps", 20))
            except (FormError, ValueError, LookupError) as e:  # bad body / charset / non-numeric field
                status = "400"
                return JSONResponse(status_code=400, content={"detail": str(e)})
            ds = state["dream"]
            if ds is None:
                from ..serve.dream_service import DreamService

                ds = state["dream"] = DreamService(cfg)
            try:
                url = await ds.dream(form["file"], model, octaves, steps)
            except (ImageDecodeError, ValueError) as e:
                status = "400"
                return JSONResponse(status_code=400, content={"detail": str(e)})
            except Exception as e:  # noqa: BLE001
                code = getattr(e, "status", None)  # RemoteError from the GPU owner (front-end mode)
                if isinstance(code, int) and code != 500:
                    status = str(code)
                    return JSONResponse(status_code=code, content={"detail": str(e)})
                status = "500"
                log.exception("deepdream request failed")
                return JSONResponse(status_code=500, content={"detail": "internal error"})
            return JSONResponse(content=url)
        finally:
            M.REQUESTS.inc(route="/deepdream", status=status)
            M.LATENCY.observe(time.perf_counter() - t0, route="/deepdream", layer="-")

    return app


def main_app() -> FastAPI:
    """uvicorn entry: ``uvicorn deconv_api_amd.api.app:main_app --factory``."""
    return create_app()
