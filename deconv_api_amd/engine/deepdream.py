"""DeepDream octave gradient ascent (BASELINE configs 3 and 5; NOT in the reference — the file
named deepdream.py there holds the deconvnet). Specification from the canonical
Keras ``examples/deep_dream.py``:

  loss  = sum_l coeff_l * sum(act_l[:, 2:-2, 2:-2, :]^2) / numel(act_l)   (per image)
  grad  = d loss / d x, normalized by max(mean|grad|, 1e-7)                (per image)
  x    += step * grad   (step 0.01, 20 iterations per octave, max_loss 10 early stop)
  octaves: successive shapes original / 1.4^i (smallest first); after each octave the detail
  lost by downscaling is re-injected: x += resize(orig, s) - resize(resize(orig, s0), s).

MI355X design:
  * the network runs on the HIP kernels through differentiable units (ops/autograd.py): conv
    fwd with ReLU epilogue, dgrad with the ReLU mask fused into the A prologue, pooling fwd/bwd;
    only the input gradient is computed (weights frozen);
  * one gradient-ascent step (forward, loss, backward, normalization, masked update) is captured
    into a hipGraph per octave shape (torch.cuda.CUDAGraph) and replayed ``iterations`` times —
    no host work or sync inside an octave;
  * ``max_loss`` is evaluated on device: an image stops updating once its loss exceeded it
    (the per-image equivalent of the example's ``break``), so the graph has no host branch.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

from .. import knobs
from ..ops import native
from ..runtime.capture import capture
from ..utils.logging import get_logger
from ..ops.autograd import loss_tap, premasked_grads, sumsq_core

# DV_DREAM_FUSED=0: the step tail (loss, normalization, update) as torch ops instead of the fused
# HIP kernels (A/B); DV_DREAM_GRAPHS: hipGraph cache entries (octave shapes) kept, LRU-evicted
log = get_logger("deconv_api_amd.deepdream")
FUSED_STEP = knobs.ablation("DV_DREAM_FUSED", "1") != "0"
GRAPH_CACHE = int(os.environ.get("DV_DREAM_GRAPHS", "8"))
# DV_DREAM_OCTAVE_GRAPH=0: one graph per step, replayed `iterations` times (A/B). Default: the
# whole octave (every step) is ONE captured graph - each separate replay costs a ~140 us launch
# gap on the GPU (profiles/kstats_c3_r2_fused_step.txt: 166 gaps after dream_update_kernel).
OCTAVE_GRAPH = os.environ.get("DV_DREAM_OCTAVE_GRAPH", "1") != "0"
# DV_DREAM_SPLIT=n: a batch runs as n independent sub-batches, each on its own HIP stream with its
# own graphs, so the latency-bound small-octave launches of one sub-batch overlap the other's
# (images are independent: per-image loss, normalisation and max-loss flag). Measured config 3
# (B=64, 299^2): 1 -> 327, 2 -> 356, 4 -> 232 img/s (4 side streams + the default stream exceed the
# 4 hardware queues per process).
SPLIT = int(knobs.ablation("DV_DREAM_SPLIT", "2"))
# DV_DREAM_TAPS=0: intermediate loss layers get their loss gradient through autograd's sum (A/B);
# default: a loss tap adds it into the gradient from above in the loss-gradient kernel itself
TAPS = knobs.ablation("DV_DREAM_TAPS", "1") != "0"
# tiled multi-rank octaves: capture the per-step all-gathers inside the octave's hipGraph
# (DV_TILE_CAPTURE_COLL=0: per-step graphs + eager collectives); DV_TILE_COLLECTIVE=1 takes the
# collective path even on a 1-rank process group (torchrun rehearsal of the multi-rank octave)
CAPTURE_COLLECTIVE = os.environ.get("DV_TILE_CAPTURE_COLL", "1") != "0"
TILE_COLLECTIVE = os.environ.get("DV_TILE_COLLECTIVE", "0") == "1"
# DV_DREAM_FUSED_LOSS=0: separate forward loss-partial launches (A/B); default: every loss layer's
# partial sums of squares come out of its loss-gradient kernel (one launch per loss layer, not two)
FUSED_LOSS = knobs.ablation("DV_DREAM_FUSED_LOSS", "1") != "0"
LOSS_PARTS = 32
# DV_DREAM_OCTAVE_RESIZE=0: octave transitions as F.interpolate + ATen adds (A/B); default: one
# octave_resize HIP launch per transition writing the next octave's static inputs directly
OCTAVE_RESIZE = knobs.ablation("DV_DREAM_OCTAVE_RESIZE", "1") != "0"
# DV_TILE_CHUNKS: a rank's units per tiled step run as this many chunks when the step all-gathers
# (several ranks): chunk c's pack all-gather is issued (async, captured into the octave graph) right
# behind chunk c's network, tile_update waits for all of them. 1: one all-gather after the whole
# network (round-4 behaviour).
TILE_CHUNKS = max(1, int(os.environ.get("DV_TILE_CHUNKS", "2")))
# DV_TILE_LOCAL_CHUNKS: the same without a collective (one rank).
TILE_LOCAL_CHUNKS = max(1, int(os.environ.get("DV_TILE_LOCAL_CHUNKS", "2")))
# DV_TILE_CHUNK_STREAMS: chunk c runs on stream c % S, forked from and joined back into the step's
# stream around the networks (graph branches when captured). Chunks run back to back on ONE stream
# cost +20 % (every launch's fill / drain exposed twice as often, ~105 launches per chunk-step); on
# two streams they fill each other's gaps: config 5 28.1 -> 31.6 img/s, the 8-rank plan's per-rank
# compute 189 -> 171 ms per batch (profiles/dream_c5_r5_local_chunks.txt).
TILE_CHUNK_STREAMS = max(1, int(os.environ.get("DV_TILE_CHUNK_STREAMS", "2")))

DEFAULT_LAYERS = {"mixed2": 0.2, "mixed3": 0.5, "mixed4": 2.0, "mixed5": 1.5}


@dataclass
class DreamSettings:
    layers: Dict[str, float] = field(default_factory=lambda: dict(DEFAULT_LAYERS))
    step: float = 0.01
    octaves: int = 4
    octave_scale: float = 1.4
    iterations: int = 20
    max_loss: Optional[float] = 10.0
    border: int = 2  # act[:, 2:-2, 2:-2, :]


def resize(x: torch.Tensor, hw: Tuple[int, int]) -> torch.Tensor:
    """NHWC bilinear resize with corner alignment (scipy.ndimage.zoom order=1 in the example)."""
    if tuple(x.shape[1:3]) == tuple(hw):
        return x
    y = F.interpolate(x.permute(0, 3, 1, 2), size=hw, mode="bilinear", align_corners=True)
    return y.permute(0, 2, 3, 1).contiguous()


def inception_preprocess(img_u8: torch.Tensor) -> torch.Tensor:
    return img_u8.float() / 127.5 - 1.0


def inception_deprocess(x: torch.Tensor) -> torch.Tensor:
    return ((x / 2.0 + 0.5) * 255.0).clamp(0, 255).to(torch.uint8)


class DeepDream:
    def __init__(self, net, settings: Optional[DreamSettings] = None, use_graphs: bool = True, dtype=None):
        self.net = net
        self.s = settings or DreamSettings()
        self.device = net.device
        if dtype is None:
            dtype = getattr(net, "dtype", torch.bfloat16) if self.device.type == "cuda" else torch.float32
        self.dtype = dtype
        self.use_graphs = use_graphs and self.device.type == "cuda"
        self.fused = FUSED_STEP and self.device.type == "cuda"
        self._graphs: "OrderedDict[tuple, object]" = OrderedDict()
        self.graph_cache = GRAPH_CACHE
        self.split = SPLIT
        self._slot = 0  # sub-batch index: each concurrent sub-batch owns its graphs/buffers
        self._streams: List[torch.cuda.Stream] = []

    # ------------------------------------------------------------------ one step
    def _net_input(self, x: torch.Tensor) -> torch.Tensor:
        return F.pad(x, (0, 5)).to(self.dtype)

    def loss(self, acts: Dict[str, torch.Tensor]) -> torch.Tensor:
        b = self.s.border
        total = None
        for name, coeff in self.s.layers.items():
            a = acts[name]
            term = coeff * sumsq_core(a, b) / float(a[0].numel())
            total = term if total is None else total + term
        return total

    def loss_and_grad(self, x: torch.Tensor):
        """x: fp32 [B, H, W, 3] (preprocessed). Returns (loss [B], normalized grad [B, H, W, 3])."""
        xin = self._net_input(x).requires_grad_(True)
        with premasked_grads():  # the loss gradient 2*act/numel vanishes where act does
            acts = self.net.forward(xin, list(self.s.layers.keys()))
        loss = self.loss(acts)
        (g,) = torch.autograd.grad(loss.sum(), xin)
        g = g[..., :3].float()
        g = g / g.abs().mean(dim=(1, 2, 3), keepdim=True).clamp_min(1e-7)
        return loss.detach(), g

    def _step(self, x: torch.Tensor, done: torch.Tensor) -> torch.Tensor:
        loss, g = self.loss_and_grad(x)
        if self.s.max_loss is not None:
            done |= loss > self.s.max_loss
        x.add_(g * ((~done).to(g.dtype) * self.s.step).view(-1, 1, 1, 1))
        return loss

    # ------------------------------------------------------------------ fused GPU step
    def _state(self, B: int, hw: Tuple[int, int]):
        """Static buffers of one octave shape: fp32 master image x, the 16-bit network input xin
        (an autograd leaf), loss/|g| partials, per-layer loss scales, done/loss flags."""
        dev = self.device
        names = list(self.s.layers.keys())
        st = type("DreamState", (), {})()
        st.x = torch.zeros(B, *hw, 3, device=dev)
        st.xin = torch.zeros(B, *hw, 8, device=dev, dtype=self.dtype, requires_grad=True)
        st.gpart = torch.zeros(B, 32, device=dev)
        st.lpart = torch.zeros(len(names), B, LOSS_PARTS, device=dev)
        st.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        st.loss = torch.zeros(B, device=dev)
        st.lcoef = None  # filled on the first step (needs the activation shapes)
        st.scales = None
        st.graph = None
        return st

    def _loss_grad(self, st, xin: torch.Tensor) -> torch.Tensor:
        """Fused-path forward + loss partials (into st.lpart) + gradient w.r.t. ``xin``. Every loss
        layer but the deepest is a loss tap (ops.autograd.loss_tap): its loss gradient joins the
        gradient from above inside one kernel, so autograd starts from the deepest layer only."""
        lib = native.lib()
        names = list(self.s.layers.keys())
        b = self.s.border
        if st.scales is None:
            st.scales = {}
        tapped = set()

        def scale(name, a):
            if name not in st.scales:
                st.scales[name] = torch.full((a.shape[0],), self.s.layers[name] / float(a[0].numel()),
                                             dtype=torch.float32, device=self.device)
            return st.scales[name]

        def tap(name, a):
            a = a.contiguous()
            tapped.add(name)
            return loss_tap(a, scale(name, a), b, st.lpart[names.index(name)] if FUSED_LOSS else None)

        with premasked_grads():  # the loss gradient 2*act/numel vanishes where act does
            acts = self.net.forward(xin, names, tap=tap if TAPS else None)
        outs = [acts[n].contiguous() for n in names]
        if st.lcoef is None:
            coef = [self.s.layers[n] / float(a[0].numel()) for n, a in zip(names, outs)]
            st.lcoef = torch.tensor(coef, dtype=torch.float32, device=self.device)
        roots, gacts = [], []
        for i, (n, a) in enumerate(zip(names, outs)):
            if n in tapped:  # its loss partials come from the tap's backward kernel (FUSED_LOSS)
                if not FUSED_LOSS:
                    lib.sumsq_core(a, st.lpart[i], b)
                continue
            ga = torch.empty_like(a)
            if FUSED_LOSS:
                lib.sumsq_core_bwd(a, scale(n, a), ga, b, None, st.lpart[i])
            else:
                lib.sumsq_core(a, st.lpart[i], b)
                lib.sumsq_core_bwd(a, scale(n, a), ga, b)
            roots.append(a)
            gacts.append(ga)
        (g,) = torch.autograd.grad(roots, xin, gacts)
        return g

    def _fused_step(self, st) -> None:
        """forward -> per-layer sumsq partials + loss gradients (HIP) -> autograd backward of the
        network only -> one fused normalize/update kernel that also writes the next xin."""
        lib = native.lib()
        g = self._loss_grad(st, st.xin)
        ml = -1.0 if self.s.max_loss is None else float(self.s.max_loss)
        lib.dream_update(g.contiguous(), st.x, st.xin, st.gpart, st.lpart, st.lcoef, st.done, st.loss,
                         float(self.s.step), ml)

    def _fused_state(self, B: int, hw: Tuple[int, int]):
        steps = self.s.iterations if OCTAVE_GRAPH else 1
        key = (B, tuple(hw), steps, self._slot)
        if key in self._graphs:
            self._graphs.move_to_end(key)
            return self._graphs[key]
        st = self._state(B, hw)
        if self.use_graphs:
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                for _ in range(2):  # warm up allocator / autograd on a side stream before capture
                    self._fused_step(st)
            torch.cuda.current_stream(self.device).wait_stream(s)
            st.graph, _ = capture(lambda: [self._fused_step(st) for _ in range(steps)])
        st.steps = steps
        self._cache_put(key, st)
        return st

    def _cache_put(self, key, val):
        self._graphs[key] = val
        # bounded: request shapes vary (each concurrent sub-batch holds its own graph per shape)
        while len(self._graphs) > max(1, self.graph_cache) * max(1, self.split):
            self._graphs.popitem(last=False)
            torch.cuda.empty_cache()

    # ------------------------------------------------------------------ hipGraph per shape
    def _graph(self, B: int, hw: Tuple[int, int]):
        key = (B, tuple(hw))
        if key in self._graphs:
            self._graphs.move_to_end(key)
            return self._graphs[key]
        x = torch.zeros(B, *hw, 3, device=self.device)
        done = torch.zeros(B, dtype=torch.bool, device=self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(2):  # warm up allocator / autograd on a side stream before capture
                self._step(x, done)
        torch.cuda.current_stream(self.device).wait_stream(s)
        g, loss = capture(lambda: self._step(x, done))
        self._cache_put(key, (g, x, done, loss))
        return self._graphs[key]

    def _ascend(self, st) -> None:
        """The ``iterations`` fused steps on a state whose st.x / st.xin hold the octave's input."""
        st.done.zero_()
        if st.graph is None:
            for _ in range(self.s.iterations):
                self._fused_step(st)
        else:
            for _ in range(self.s.iterations // st.steps):
                st.graph.replay()

    def gradient_ascent(self, x: torch.Tensor) -> torch.Tensor:
        B, H, W, _ = x.shape
        if self.fused:
            st = self._fused_state(B, (H, W))
            with torch.no_grad():
                st.x.copy_(x)
                st.xin.zero_()
                st.xin[..., :3].copy_(x)
            self._ascend(st)
            return st.x.clone()
        if self.use_graphs:
            g, gx, gdone, gloss = self._graph(B, (H, W))
            gx.copy_(x)
            gdone.zero_()
            for _ in range(self.s.iterations):
                g.replay()
            return gx.clone()
        x = x.clone()
        done = torch.zeros(B, dtype=torch.bool, device=x.device)
        for _ in range(self.s.iterations):
            self._step(x, done)
        return x

    # ------------------------------------------------------------------ octaves
    def octave_shapes(self, H: int, W: int) -> List[Tuple[int, int]]:
        shapes = [(H, W)]
        for i in range(1, self.s.octaves):
            shapes.append((int(H / self.s.octave_scale ** i), int(W / self.s.octave_scale ** i)))
        return shapes[::-1]

    def run(self, x: torch.Tensor) -> torch.Tensor:
        """x: preprocessed fp32 [B, H, W, 3] on the engine device -> dreamed fp32 image."""
        n = self.split if (self.fused and x.is_cuda) else 1
        if n <= 1 or x.shape[0] < n:  # (uneven sub-batches allowed: x.chunk)
            return self._run_one(x)
        cur = torch.cuda.current_stream(self.device)
        while len(self._streams) < n:
            self._streams.append(torch.cuda.Stream(self.device))
        outs = []
        try:
            for i, xc in enumerate(x.chunk(n)):
                st = self._streams[i]
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    self._slot = i
                    outs.append(self._run_one(xc))
        finally:
            self._slot = 0
        for st in self._streams[:n]:
            cur.wait_stream(st)
        return torch.cat(outs)

    def _run_one(self, x: torch.Tensor) -> torch.Tensor:
        img = x
        for img in self.octave_steps(x):
            pass
        return img

    def octave_steps(self, x: torch.Tensor):
        """Generator form of one (sub-)batch's dream: yields the image after each octave (its GPU
        work enqueued, not necessarily finished). The multi-rank service drives a dream octave by
        octave through this, polling each octave's completion under its failure deadlines and
        letting other commands run between octaves (parallel/sharded.py)."""
        if self.fused and x.is_cuda and OCTAVE_RESIZE:
            yield from self._octave_steps_fused(x)
            return
        shapes = self.octave_shapes(x.shape[1], x.shape[2])
        original = x
        shrunk = resize(original, shapes[0])
        img = x
        for hw in shapes:
            img = resize(img, hw)
            img = self.gradient_ascent(img)
            upscaled = resize(shrunk, hw)
            same = resize(original, hw)
            img = img + (same - upscaled)
            shrunk = resize(original, hw)
            yield img

    def _octave_steps_fused(self, x: torch.Tensor):
        """``octave_steps`` on the fused GPU path: every octave transition is ONE octave_resize
        launch (csrc/dream.hip) that resizes (dreamed image + lost detail) straight into the next
        octave's static fp32 image and 16-bit network input, instead of F.interpolate x4, two ATen
        adds and the copy/fill/clone around each octave's graph. The lost detail of octave o is
        same_o - up_o with same_o = resize(x, s_o), up_o = resize(same_{o-1}, s_o) (0 for o = 0),
        both enqueued ahead of the octave's replay. Intermediate yields are the octave's dreamed
        image before its detail is re-injected (the detail rides on the next resize); the last
        yield is the finished image, a fresh tensor."""
        lib = native.lib()
        shapes = self.octave_shapes(x.shape[1], x.shape[2])
        x = x.contiguous()
        B = x.shape[0]
        dev = x.device

        def resized(src, hw):
            if tuple(hw) == tuple(src.shape[1:3]):
                return src
            dst = torch.empty(B, *hw, 3, device=dev)
            lib.octave_resize(src, None, None, dst, None)
            return dst

        img = same = up = prev = None
        for o, hw in enumerate(shapes):
            st = self._fused_state(B, hw)
            # the octave's input: x resized (octave 0) or the previous octave's image + its detail
            lib.octave_resize(x if o == 0 else img, same, up, st.x, st.xin)
            cur = resized(x, hw)
            same, up = (None, None) if o == 0 else (cur, resized(prev, hw))
            prev = cur
            self._ascend(st)
            img = st.x
            if o + 1 < len(shapes):
                yield img
        out = torch.empty_like(img)
        lib.octave_resize(img, same, up, out, None)
        yield out

    def dream_u8(self, img_u8: torch.Tensor) -> torch.Tensor:
        """uint8 RGB [B, H, W, 3] -> uint8 dreamed image."""
        x = inception_preprocess(img_u8.to(self.device))
        return inception_deprocess(self.run(x))


RESNET_LAYERS = {"conv3_block4_out": 0.5, "conv4_block3_out": 1.0, "conv4_block6_out": 1.5}


class TiledDeepDream(DeepDream):
    """Large-image DeepDream: every gradient step rolls the image by a random offset (shared seed,
    identical on every rank), cuts it into equal ``<= tile``-sized tiles, computes each tile's input
    gradient independently and stitches them. (tile, image) units are dealt round-robin to the
    ranks (the image-domain analogue of context parallelism); a rank runs ALL of its
    units as ONE batch (tiles are equal-sized: the last row/column of tiles is shifted inwards to
    overlap its neighbour, and each pixel's gradient is taken from exactly one owning tile), so the
    convs see large GEMMs instead of one small launch per tile. The roll, the tile cut and the
    stitch/un-roll are single gathers/scatters with precomputed indices.

    GPU (fused) step, all HIP kernels (csrc/dream.hip):
      tile_gather   rolled tiles of the fp32 image -> 16-bit network input of this rank's units
      network       forward + input-gradient backward of all units as one batch
      tile_pack     owned pixels of each unit's gradient -> a fixed-size pack, + {loss, sum|g|}
      all_gather    of the packs over the ranks (RCCL; each pixel has ONE owner, so gathering the
                    owned tiles moves half the bytes of all-reducing the full gradient, and the
                    unit losses ride along: no separate loss all-reduce)
      tile_update   per-image mean|g| and loss from the pack tails, device-side max_loss flag,
                    x += step * g / mean|g| straight from the packs (identical on every rank)
    The whole octave (``iterations`` steps, shifts in a device table staged through pinned memory)
    is ONE captured hipGraph, the per-step all-gathers included when there are several ranks
    (fallback if the capture is refused: a graph per step, the collective between replays).
    ``virtual_octave`` runs the multi-rank step for W virtual ranks on one device (tests). CPU
    tensors use the torch implementation below (the oracle)."""

    def __init__(self, net, settings: Optional[DreamSettings] = None, tile: int = 512, info=None, seed: int = 0,
                 dtype=None, use_graphs: bool = True):
        super().__init__(net, settings, use_graphs=False, dtype=dtype)
        self.fused = False  # the tiled step assembles the gradient across tiles/ranks (below)
        self.tile = tile
        self.info = info
        self.gen = torch.Generator().manual_seed(seed)
        self._plans: Dict[tuple, tuple] = {}
        # one hipGraph per octave shape for the whole tile forward/backward/stitch
        self.tile_graphs = use_graphs and self.device.type == "cuda"
        self._tgraphs: "OrderedDict[tuple, object]" = OrderedDict()
        self._cgroup = None  # (default group id, process group of the captured all-gathers)
        self.tile_fused = FUSED_STEP and self.device.type == "cuda"
        # coll_wait(work): how an EAGER collective of the tiled step is waited for. None: a blocking
        # call. The multi-rank service sets a poll under its heartbeat / re-form deadlines
        # (ShardedRunner._await), so a peer that dies mid-dream surfaces as PeerLost instead of a
        # collective that never returns. (Collectives captured inside an octave graph are covered by
        # polling the octave's completion event instead.)
        self.coll_wait = None

    @staticmethod
    def _axis_tiles(L: int, tile: int):
        """[(start, own_lo, own_hi)] of equal-size (T) windows covering [0, L); returns (T, list)."""
        n = -(-L // tile)
        T = -(-L // n)
        return T, [(min(i * T, L - T), i * T, min((i + 1) * T, L)) for i in range(n)]

    def _tiles(self, H: int, W: int):
        Th, ys = self._axis_tiles(H, self.tile)
        Tw, xs = self._axis_tiles(W, self.tile)
        return Th, Tw, [(y, x) for y in ys for x in xs]

    def _my_units(self, B: int, ntiles: int, world: int, rank: int):
        """Work units are (tile, image) pairs dealt round-robin to the ranks, so ranks stay busy
        even when an octave has fewer tiles than ranks."""
        return [(u // B, u % B) for u in range(rank, ntiles * B, world)]

    def _plan(self, B: int, H: int, W: int, device):
        """Static gather/scatter indices for one octave shape: (Th, Tw, unit image ids [U],
        tile origins [U, 2], owned (local flat, unit-relative global y, x) index tensors)."""
        key = (B, H, W)
        if key in self._plans:
            return self._plans[key]
        world = self.info.world if self.info is not None else 1
        rank = self.info.rank if self.info is not None else 0
        Th, Tw, tiles = self._tiles(H, W)
        units = self._my_units(B, len(tiles), world, rank)
        img = torch.tensor([b for _, b in units], dtype=torch.long)
        org = torch.tensor([[tiles[t][0][0], tiles[t][1][0]] for t, _ in units], dtype=torch.long).view(-1, 2)
        loc, gy, gx, gb = [], [], [], []
        for u, (t, b) in enumerate(units):
            (y0, oy0, oy1), (x0, ox0, ox1) = tiles[t]
            yy, xx = torch.meshgrid(torch.arange(oy0, oy1), torch.arange(ox0, ox1), indexing="ij")
            loc.append(((u * Th + (yy - y0)) * Tw + (xx - x0)).reshape(-1))
            gy.append(yy.reshape(-1))
            gx.append(xx.reshape(-1))
            gb.append(torch.full((yy.numel(),), b, dtype=torch.long))
        cat = lambda v: (torch.cat(v) if v else torch.zeros(0, dtype=torch.long)).to(device)  # noqa: E731
        plan = (Th, Tw, img.to(device), org.to(device), cat(loc), cat(gb), cat(gy), cat(gx), len(tiles))
        self._plans[key] = plan
        return plan

    def _tile_grad(self, x: torch.Tensor, shift: torch.Tensor, plan, grad: torch.Tensor, loss: torch.Tensor):
        """grad, loss <- this rank's stitched tile gradients / summed tile losses for the image
        rolled by ``shift`` (a device [2] tensor, so a captured graph replays any shift)."""
        B, H, W, _ = x.shape
        Th, Tw, img, org, loc, gb, gyo, gxo, _ = plan
        grad.zero_()
        loss.zero_()
        if not img.numel():
            return
        sy, sx = shift[0], shift[1]
        # rolled[b, y, x] = x[b, (y - sy) % H, (x - sx) % W]; tiles of the rolled image, batched
        iy = (org[:, 0:1] + torch.arange(Th, device=x.device) - sy) % H  # [U, Th]
        ix = (org[:, 1:2] + torch.arange(Tw, device=x.device) - sx) % W  # [U, Tw]
        xt = x[img[:, None, None], iy[:, :, None], ix[:, None, :]]  # [U, Th, Tw, 3]
        xin = self._net_input(xt).requires_grad_(True)
        with premasked_grads():  # the loss gradient 2*act/numel vanishes where act does
            acts = self.net.forward(xin, list(self.s.layers.keys()))
        lt = self.loss(acts)
        (g,) = torch.autograd.grad(lt.sum(), xin)
        # owned pixels of each unit -> un-rolled image positions
        gsrc = g[..., :3].reshape(-1, 3)[loc].float()
        grad.index_put_((gb, (gyo - sy) % H, (gxo - sx) % W), gsrc)
        loss.index_add_(0, img, lt.detach().float())

    def _tile_graph(self, x: torch.Tensor, plan):
        """hipGraph of _tile_grad for one octave shape (static buffers: image, shift, grad, loss)."""
        key = ("torch",) + tuple(x.shape)
        if key in self._tgraphs:
            return self._tgraphs[key]
        bx = x.clone()
        shift = torch.zeros(2, dtype=torch.long, device=x.device)
        grad = torch.zeros_like(x)
        loss = torch.zeros(x.shape[0], device=x.device)
        st = torch.cuda.Stream(x.device)
        st.wait_stream(torch.cuda.current_stream(x.device))
        with torch.cuda.stream(st):
            for _ in range(2):
                self._tile_grad(bx, shift, plan, grad, loss)
        torch.cuda.current_stream(x.device).wait_stream(st)
        g, _ = capture(lambda: self._tile_grad(bx, shift, plan, grad, loss))
        self._tgraphs[key] = (g, bx, shift, grad, loss)
        return self._tgraphs[key]

    # ------------------------------------------------------------------ fused GPU tiled step
    def _gplan(self, B: int, H: int, W: int):
        """int32 [units, 7] plan rows {image, tile origin y, x, owned y0, y1, x0, x1 (tile-local)}
        for every unit of every rank (unit u = tile u // B, image u % B), validated on the host
        (the kernels index with them unchecked)."""
        Th, Tw, tiles = self._tiles(H, W)
        rows = []
        for u in range(len(tiles) * B):
            (y0, oy0, oy1), (x0, ox0, ox1) = tiles[u // B]
            rows.append([u % B, y0, x0, oy0 - y0, oy1 - y0, ox0 - x0, ox1 - x0])
        plan = torch.tensor(rows, dtype=torch.int32)
        assert ((plan[:, 0] >= 0) & (plan[:, 0] < B)).all()
        assert ((plan[:, 1] >= 0) & (plan[:, 1] + Th <= H) & (plan[:, 2] >= 0) & (plan[:, 2] + Tw <= W)).all()
        assert ((plan[:, 3] >= 0) & (plan[:, 3] < plan[:, 4]) & (plan[:, 4] <= Th)).all()
        assert ((plan[:, 5] >= 0) & (plan[:, 5] < plan[:, 6]) & (plan[:, 6] <= Tw)).all()
        return Th, Tw, plan, len(tiles)

    def _chunk_states(self, st, rank: int, mine: int):
        """Per-chunk sub-states of rank ``rank``'s ``mine`` units (chunk c = local units c*ucc ..):
        own 16-bit network input / loss partials / scales, its slot of chunk c's packs."""
        chunks = []
        for c in range(st.C):
            cs = type("TileChunk", (), {})()
            cs.k0 = c * st.ucc
            cs.n = max(0, min(mine, (c + 1) * st.ucc) - cs.k0)
            cs.pack = st.packs[c, rank]
            cs.xin = torch.zeros(max(cs.n, 1), st.Th, st.Tw, 8, dtype=self.dtype, device=self.device, requires_grad=True)
            cs.lpart = torch.zeros(len(self.s.layers), max(cs.n, 1), LOSS_PARTS, device=self.device)
            cs.lcoef, cs.scales = None, None
            chunks.append(cs)
        return chunks

    def _tstate(self, B: int, H: int, W: int):
        key = (B, H, W)
        if key in self._tgraphs:
            self._tgraphs.move_to_end(key)
            return self._tgraphs[key]
        lib = native.lib()
        dev = self.device
        world = self.info.world if self.info is not None else 1
        rank = self.info.rank if self.info is not None else 0
        Th, Tw, plan, ntiles = self._gplan(B, H, W)
        nunits = plan.shape[0]
        ucap = -(-nunits // world)
        mine = len(range(rank, nunits, world))
        st = type("TileState", (), {})()
        st.Th, st.Tw, st.ntiles, st.world, st.rank, st.ucap, st.mine = Th, Tw, ntiles, world, rank, ucap, mine
        probe = type("P", (), {"world": world})()
        # virtual (bench_dream.py --virtual-world): chunked as the real rank's collective step would be
        coll_like = self._collective(probe) or getattr(self, "virtual", False)
        st.C = min(TILE_CHUNKS if coll_like else TILE_LOCAL_CHUNKS, ucap)
        st.ucc = -(-ucap // st.C)  # units per rank and chunk
        st.plan = plan.to(dev)
        st.x = torch.zeros(B, H, W, 3, device=dev)
        st.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        st.loss = torch.zeros(B, device=dev)
        st.shifts = torch.zeros(self.s.iterations, 2, dtype=torch.int32, device=dev)
        pe = lib.tile_pack_elems(st.ucc, Th, Tw)
        st.packs = torch.zeros(st.C, world, pe, dtype=self.dtype, device=dev)  # [chunk][rank][pack]
        st.chunks = self._chunk_states(st, rank, mine)
        st.graph, st.step_graph = None, None
        self._tgraphs[key] = st
        while len(self._tgraphs) > max(1, self.graph_cache):
            self._tgraphs.popitem(last=False)
            torch.cuda.empty_cache()
        return st

    def _tile_compute_chunk(self, st, cs, it: int, rank: int) -> None:
        """gather -> network fwd/bwd -> pack for one chunk of a rank's units, step ``it``."""
        if cs.n == 0:
            return
        lib = native.lib()
        lib.tile_gather(st.x, cs.xin, st.plan, st.shifts[it], rank, st.world, cs.k0)
        g = self._loss_grad(cs, cs.xin)
        lib.tile_pack(g.contiguous(), cs.pack, st.plan, cs.lpart, cs.lcoef, st.ucc, rank, st.world, cs.k0)

    def _tile_compute(self, st, it: int) -> None:
        """every chunk of this rank's units for step ``it`` (shift row it of the device table)."""
        for cs in st.chunks:
            self._tile_compute_chunk(st, cs, it, st.rank)

    def _tile_apply(self, st, it: int) -> None:
        ml = -1.0 if self.s.max_loss is None else float(self.s.max_loss) * st.ntiles
        native.lib().tile_update(st.packs, st.ucc, st.plan, st.shifts[it], st.x, st.done, st.loss, float(self.s.step),
                                 ml, st.world, st.Th, st.Tw)

    def _collective(self, st) -> bool:
        """Whether the octave all-gathers the packs: several ranks, or DV_TILE_COLLECTIVE=1 with a
        real 1-rank process group (the multi-rank code path, rehearsed on one GPU). ``virtual``
        (bench_dream.py --virtual-world): this process times ONE rank's share of a W-rank octave
        (its units, its pack, the update over W packs) without the collective; the result is not
        a dream (the other ranks' packs stay zero)."""
        if getattr(self, "virtual", False):
            return False
        if st.world > 1:
            return True
        return TILE_COLLECTIVE and self.info is not None and self.info.backend != "none"

    def _coll(self, fn, *args) -> None:
        """An eager collective: blocking, or issued async and handed to ``coll_wait``."""
        if self.coll_wait is None:
            fn(*args)
        else:
            self.coll_wait(fn(*args, async_op=True))

    def _gather_chunk(self, st, c: int, group=None):
        """Async all-gather of chunk c's packs (every rank's slot) -> the work object."""
        import torch.distributed as dist

        return dist.all_gather_into_tensor(st.packs[c].view(-1), st.packs[c, st.rank], group=group, async_op=True)

    def _capture_group(self):
        """The process group the CAPTURED all-gathers run on: a second communicator over the same
        ranks, connected eagerly at creation (bound device) and never used by an eager collective.
        Its watchdog therefore never tracks a work, so it can not query an event of the stream an
        octave capture has pulled in (the hipErrorCapturedEvent abort of round 3; the eager
        collectives of the default group - weight broadcast, dream broadcast, deconv scatter /
        gather - live on another stream). Created collectively: every rank reaches the first
        captured octave of a world at the same command. Keyed on the default group, so a group
        re-formed over the survivors gets a new one."""
        import torch.distributed as dist

        key = id(dist.distributed_c10d._get_default_group())
        if self._cgroup is None or self._cgroup[0] != key:
            self._cgroup = (key, dist.new_group(ranks=list(range(dist.get_world_size()))))
        return self._cgroup[1]

    def _finish(self, work) -> None:
        if self.coll_wait is None:
            work.wait()  # stream-ordered: the current stream waits for the collective's stream
        else:
            self.coll_wait(work)

    def _tile_steps(self, st, capturing: bool = False) -> None:
        """The octave's steps. With a collective, chunk c's all-gather is issued right after its pack
        and runs on the collective's stream while chunk c+1's network runs on this one; the update
        waits for every chunk's gather (captured as graph edges when ``capturing``)."""
        coll = self._collective(st)
        group = self._capture_group() if coll and capturing else None
        ns = min(TILE_CHUNK_STREAMS, st.C)
        if ns > 1 and len(getattr(self, "_cstreams", ())) < ns:
            self._cstreams = [torch.cuda.Stream(self.device) for _ in range(ns)]
        for it in range(self.s.iterations):
            works = []
            cur = torch.cuda.current_stream(self.device)
            if ns == 1:
                for c, cs in enumerate(st.chunks):
                    self._tile_compute_chunk(st, cs, it, st.rank)
                    if coll:
                        works.append(self._gather_chunk(st, c, group))
            else:
                # fork: chunk c on stream c % ns. Its all-gather is issued from THIS stream behind an event
                # of the chunk (a collective issued from a forked capture stream is not seen as captured
                # by the process group, whose watchdog then queries a captured event and aborts)
                done = []
                for c, cs in enumerate(st.chunks):
                    sm = self._cstreams[c % ns]
                    sm.wait_stream(cur)
                    with torch.cuda.stream(sm):
                        self._tile_compute_chunk(st, cs, it, st.rank)
                    ev = torch.cuda.Event()
                    ev.record(sm)
                    done.append(ev)
                for c, ev in enumerate(done):
                    cur.wait_event(ev)
                    if coll:
                        works.append(self._gather_chunk(st, c, group))
            for w in works:
                if capturing:
                    w.wait()  # recorded into the octave graph: nothing to poll here
                else:
                    self._finish(w)
            self._tile_apply(st, it)

    def _stage_shifts(self, st) -> None:
        """This octave's random roll table -> the device, without a host sync: through pinned
        buffers of the octave's own state (a pageable H2D copy blocks the host until the stream
        drains; one shared pinned buffer would make octave k+1 wait for octave k's upload, which
        queues behind octave k-1's replay). Two buffers per state, used alternately: reusing one
        waits for this shape's previous upload, which sits behind the whole previous dream batch
        on the stream, so the host could not run more than one batch ahead
        (``host_enqueue_s`` 0.087 s of a 0.30 s config-5 batch)."""
        shifts = torch.randint(-self.tile // 2, self.tile // 2 + 1, (self.s.iterations, 2), generator=self.gen)
        pins = getattr(st, "shift_pins", None)
        if pins is None or pins[0].shape != shifts.shape:
            pins = st.shift_pins = [torch.empty(shifts.shape, dtype=torch.int32, pin_memory=True) for _ in range(2)]
            st.shift_evs = [None, None]
            st.shift_i = 0
        i = st.shift_i
        st.shift_i ^= 1
        if st.shift_evs[i] is not None:
            st.shift_evs[i].synchronize()  # this buffer's previous upload (two dream batches ago)
        pins[i].copy_(shifts)
        st.shifts.copy_(pins[i], non_blocking=True)
        st.shift_evs[i] = torch.cuda.Event()
        st.shift_evs[i].record()

    def _capture(self, fn) -> torch.cuda.CUDAGraph:
        return capture(fn)[0]

    def _gradient_ascent_fused(self, x: torch.Tensor) -> torch.Tensor:
        B, H, W, _ = x.shape
        st = self._tstate(B, H, W)
        st.x.copy_(x)
        self._ascend_tiled(st)
        return st.x.clone()

    def octave_steps(self, x: torch.Tensor):
        """The tiled dream's octaves (see DeepDream.octave_steps). On the fused GPU path every octave
        transition is ONE octave_resize launch straight into the next octave's static fp32 image (the
        tiles gather their 16-bit inputs from it), as the untiled fused path does; the generic path
        (F.interpolate x4 + two adds per transition) is the CPU / DV_DREAM_OCTAVE_RESIZE=0 oracle."""
        if self.tile_fused and x.is_cuda and OCTAVE_RESIZE:
            yield from self._tiled_octave_steps_fused(x)
            return
        yield from DeepDream.octave_steps(self, x)

    def _tiled_octave_steps_fused(self, x: torch.Tensor):
        lib = native.lib()
        shapes = self.octave_shapes(x.shape[1], x.shape[2])
        x = x.contiguous()
        B = x.shape[0]
        dev = x.device

        def resized(src, hw):
            if tuple(hw) == tuple(src.shape[1:3]):
                return src
            dst = torch.empty(B, *hw, 3, device=dev)
            lib.octave_resize(src, None, None, dst, None)
            return dst

        img = same = up = prev = None
        for o, hw in enumerate(shapes):
            st = self._tstate(B, *hw)
            lib.octave_resize(x if o == 0 else img, same, up, st.x, None)
            cur = resized(x, hw)
            same, up = (None, None) if o == 0 else (cur, resized(prev, hw))
            prev = cur
            self._ascend_tiled(st)
            img = st.x
            if o + 1 < len(shapes):
                yield img
        out = torch.empty_like(img)
        lib.octave_resize(img, same, up, out, None)
        yield out

    def _ascend_tiled(self, st) -> None:
        """The octave's ``iterations`` tiled steps on a state whose st.x holds the octave's input."""
        import torch.distributed as dist

        self._stage_shifts(st)
        st.done.zero_()
        coll = self._collective(st)
        if self.tile_graphs and st.graph is None and st.step_graph is None:
            # warm up on a side stream (autograd / allocator), restore the image, capture the octave
            s = torch.cuda.Stream(self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):
                self._tile_compute(st, 0)
            torch.cuda.current_stream(self.device).wait_stream(s)
            if coll and CAPTURE_COLLECTIVE:
                # the captured all-gathers' communicator exists (eagerly connected) before the capture
                # opens, and no eager collective ever runs on it (_capture_group): no warm-up
                # collective, nothing for a watchdog to poll during the capture
                self._capture_group()
                torch.cuda.synchronize(self.device)
            if not coll or CAPTURE_COLLECTIVE:
                # the whole octave, all-gathers included (RCCL collectives are graph-capturable):
                # one replay per octave instead of `iterations` replays + eager collectives
                try:
                    st.graph = self._capture(lambda: self._tile_steps(st, capturing=True))
                except RuntimeError as e:  # capture of the collective refused: per-step graphs
                    if not coll:
                        raise
                    log.warning("octave capture with collectives failed, per-step graphs", extra={"fields": {"err": repr(e)}})
                    st.graph = None
            if st.graph is None and coll:
                st.step_graph = [self._capture(lambda it=it: self._tile_compute(st, it))
                                 for it in range(self.s.iterations)]
        if st.graph is not None:
            st.graph.replay()
        elif st.step_graph is not None:
            for it in range(self.s.iterations):
                st.step_graph[it].replay()
                for c in range(st.C):
                    self._coll(dist.all_gather_into_tensor, st.packs[c].view(-1), st.packs[c, st.rank])
                self._tile_apply(st, it)
        else:
            self._tile_steps(st)

    def virtual_octave(self, x: torch.Tensor, world: int, chunks: int = TILE_CHUNKS) -> torch.Tensor:
        """One octave of the ``world``-rank fused tiled step on THIS device, without collectives: for
        every step each virtual rank gathers its units, runs the network and packs into its own slot
        of the packs buffer (chunked as a real rank would: ``chunks`` slices of its units, packs
        [chunk][rank]), exactly what the all-gathers assemble on every real rank, then ONE
        tile_update with ``world`` packs applies the step. Eager; for tests / tools (the multi-rank
        kernels' rank/world/chunk indexing exercised on a one-GPU box)."""
        lib = native.lib()
        B, H, W, _ = x.shape
        Th, Tw, plan, ntiles = self._gplan(B, H, W)
        nunits = plan.shape[0]
        ucap = -(-nunits // world)
        dev = self.device
        st = type("TileState", (), {})()
        st.Th, st.Tw, st.ntiles, st.world, st.ucap = Th, Tw, ntiles, world, ucap
        st.C = max(1, min(chunks, ucap))
        st.ucc = -(-ucap // st.C)
        st.plan = plan.to(dev)
        st.packs = torch.zeros(st.C, world, lib.tile_pack_elems(st.ucc, Th, Tw), dtype=self.dtype, device=dev)
        st.x = x.clone()
        st.done = torch.zeros(B, dtype=torch.uint8, device=dev)
        st.loss = torch.zeros(B, device=dev)
        st.shifts = torch.zeros(self.s.iterations, 2, dtype=torch.int32, device=dev)
        self._stage_shifts(st)
        ranks = [self._chunk_states(st, r, len(range(r, nunits, world))) for r in range(world)]
        for it in range(self.s.iterations):
            for r, chunks_r in enumerate(ranks):
                for cs in chunks_r:
                    self._tile_compute_chunk(st, cs, it, r)
            self._tile_apply(st, it)
        return st.x

    def gradient_ascent(self, x: torch.Tensor) -> torch.Tensor:
        if self.tile_fused and x.is_cuda:
            return self._gradient_ascent_fused(x)
        return self._gradient_ascent_torch(x)

    def _gradient_ascent_torch(self, x: torch.Tensor) -> torch.Tensor:
        import torch.distributed as dist

        B, H, W, _ = x.shape
        done = torch.zeros(B, dtype=torch.bool, device=x.device)
        world = self.info.world if self.info is not None else 1
        plan = self._plan(B, H, W, x.device)
        ntiles = plan[-1]
        shifts = torch.randint(-self.tile // 2, self.tile // 2 + 1, (self.s.iterations, 2), generator=self.gen)
        if self.tile_graphs:
            graph, bx, shift, grad, loss = self._tile_graph(x, plan)
            bx.copy_(x)
            x = bx
            dshifts = shifts.to(x.device)
        else:
            x = x.clone()
            shift = torch.zeros(2, dtype=torch.long, device=x.device)
            grad = torch.zeros_like(x)
            loss = torch.zeros(B, device=x.device)
        for it in range(self.s.iterations):
            if self.tile_graphs:
                shift.copy_(dshifts[it])
                graph.replay()
            else:
                shift.copy_(shifts[it])
                self._tile_grad(x, shift, plan, grad, loss)
            if world > 1:
                self._coll(dist.all_reduce, grad)
                self._coll(dist.all_reduce, loss)
            g = grad / grad.abs().mean(dim=(1, 2, 3), keepdim=True).clamp_min(1e-7)
            if self.s.max_loss is not None:
                done |= loss > self.s.max_loss * ntiles
            x.add_(g * ((~done).to(g.dtype) * self.s.step).view(-1, 1, 1, 1))
        return x.clone() if self.tile_graphs else x
