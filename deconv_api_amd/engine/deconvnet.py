"""Batched Zeiler-Fergus deconvnet engine on VGG16 (reference: app/deepdream.py:383-476).

What the reference does per request: stack D-layers up to the target (:401-423), run every
``up`` (:425-428), then for every named layer <= target and each of its top-8 filters run a full
``down`` chain to the input (:430-474). The HTTP handler then keeps only the first four
reconstructions of the target layer (app/main.py:67-69).

What this engine does (same outputs, MI355X-shaped):
  * forward in bf16 NHWC through the MFMA implicit-GEMM conv; every 2x2 max-pool that precedes
    the target is fused into its conv's epilogue and leaves only a uint8 switch code per pooled
    element (the backward pass needs switches + weights, never the forward activations);
  * per-image top-k filter selection on device (channel sums -> stable positive top-k);
  * the B images x K filters backward chains are folded into one batch of B*K signals that
    share their image's switch codes (code_div = K); the first step from the one-channel seed
    is a 9-tap stencil, every later conv-down is the same MFMA kernel with the unpool gather
    fused into its A-operand load and ReLU on both sides;
  * the final conv-down writes fp32 reconstructions that the mosaic/deprocess kernel turns into
    the 2x2 uint8 mosaic of app/main.py:67-72.
``visualize_all_layers`` keeps the reference's library API (all layers, top-8, across-batch
filter sums) on top of the same machinery.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from .. import ops
from ..models.vgg16 import VGG16Runtime, LayerSpec
from ..utils import tracing

VALID_MODES = ("all", "max")
# a GPU batch of >= DECONV_SPLIT_MIN images runs as DECONV_STREAMS sub-batches on that many streams forked
# from and joined back into the caller's stream (graph branches when captured; per-image top-k makes the
# parts independent). 1 = off: measured no gain on config 2 (docs/KERNELS.md); kept for tests / tools that
# set the attributes
DECONV_STREAMS = 1
DECONV_SPLIT_MIN = 64
# conv-downs consuming an unpooled map with at most this many input channels expand the unpool themselves
# (64: block1_conv2.down's fused tail); wider consumers get the map from the producer's epilogue
UNPOOL_CONSUMER_MAXC = 64
# DV_POOL_SPLIT=name,...: these convs run WITHOUT the fused pool epilogue (plain conv, which may take the
# persistent KW3P kernel, then the standalone 2x2 max-pool/switch kernel) on the GPU. Default: block3/4's
# last convs (config 2: 7724 vs 7680 img/s mean of 3 interleaved pairs, profiles/final_r6_validation.txt;
# their fused-pool convs ran on the generic DMA kernel); DV_POOL_SPLIT= (empty) fuses every pool
POOL_SPLIT = frozenset(n for n in os.environ.get("DV_POOL_SPLIT", "block3_conv3,block4_conv3").split(",") if n)


class UnknownLayerError(KeyError):
    pass


@dataclass
class ForwardState:
    target: str
    out: torch.Tensor  # target output: [B, H, W, C] or [B, units]
    codes: Dict[str, torch.Tensor] = field(default_factory=dict)  # pool name -> switch codes
    outputs: Dict[str, torch.Tensor] = field(default_factory=dict)  # kept named outputs (all-layers mode)


@dataclass
class DeconvResult:
    recon: torch.Tensor  # fp32 [B, K, 224, 224, 3]
    filters: torch.Tensor  # int32 [B, K] (-1 = no positive filter: zero reconstruction)
    sums: torch.Tensor  # fp32 [B, K] selection scores
    mosaic: Optional[torch.Tensor] = None  # u8 [B, 448, 448, 3] (K == 4)


class DeconvNet:
    def __init__(self, rt: VGG16Runtime):
        self.rt = rt
        self.specs: List[LayerSpec] = rt.specs
        self.names = [s.name for s in self.specs]

    # ------------------------------------------------------------------ helpers
    def _check_layer(self, name: str) -> int:
        if name not in self.names:
            raise UnknownLayerError(f"unknown layer {name!r}; valid: {self.names[1:]}")
        if name == "input_1":
            raise UnknownLayerError("input_1 has no filters to visualize")
        i = self.names.index(name)
        if self.specs[i].kind == "dense" and name not in self.rt.dense:
            raise UnknownLayerError(f"{name!r} needs the classifier head (include_top=True)")
        return i

    def _dense_up(self, x: torch.Tensor, name: str) -> torch.Tensor:
        d = self.rt.dense[name]
        if x.is_cuda and d.up is not None:  # MFMA GEMM with fused bias (+ReLU); HIP row softmax
            B = x.shape[0]
            xin = x.reshape(B, 1, 1, -1).to(self.rt.dtype).contiguous()
            if d.spec.activation == "relu":
                return ops.conv2d(xin, d.up, relu=True, pad=0).reshape(B, -1)
            return ops.softmax_rows(ops.conv2d(xin, d.up, relu=False, pad=0, epilogue="f32").reshape(B, -1)).to(
                self.rt.dtype)
        y = torch.matmul(x.to(d.w.dtype), d.w).float() + d.b
        if d.spec.activation == "relu":
            y = y.clamp_min(0)
        else:
            y = torch.softmax(y, dim=-1)
        return y.to(self.rt.dtype if x.is_cuda else torch.float32)

    # ------------------------------------------------------------------ forward
    def forward(self, x: torch.Tensor, target: str, fuse_pools: bool = True,
                keep_all: bool = False, hook=None) -> ForwardState:
        """x: preprocessed [B, 224, 224, 8] (bf16 on device). Runs ``up`` through ``target``.
        ``hook`` = (layer name, fn): fn() runs on the host right before that layer's forward work is
        enqueued (bench.py issues the previous step's copy-back there, so the PCIe blit overlaps
        MFMA-bound convs instead of the memory-bound first layers)."""
        ti = self._check_layer(target)
        seq = self.specs[1: ti + 1]
        st = ForwardState(target, x)
        i = 0
        while i < len(seq):
            s = seq[i]
            if hook is not None and s.name == hook[0]:
                hook[1]()
            if s.kind == "conv":
                cl = self.rt.convs[s.name]
                nxt = seq[i + 1] if i + 1 < len(seq) else None
                # conv -> conv -> pool at the first layer (VGG16 block1): one fused launch whose
                # intermediate 64-channel map stays in LDS (ops.conv.stem_pool)
                if (i == 0 and fuse_pools and not keep_all and x.is_cuda and i + 2 < len(seq) and
                        nxt.kind == "conv" and seq[i + 2].kind == "pool" and
                        (hook is None or hook[0] != nxt.name)):
                    r = ops.stem_pool(x, cl.fwd, self.rt.convs[nxt.name].fwd)
                    if r is not None:
                        x, code = r
                        st.codes[seq[i + 2].name] = code
                        i += 3
                        continue
                if (fuse_pools and not keep_all and nxt is not None and nxt.kind == "pool" and
                        not (x.is_cuda and s.name in POOL_SPLIT)):
                    x, code = ops.conv2d(x, cl.fwd, relu=True, epilogue="pool")
                    st.codes[nxt.name] = code
                    i += 2
                    continue
                x = ops.conv2d(x, cl.fwd, relu=True)
            elif s.kind == "pool":
                x, code = ops.maxpool2x2(x)
                st.codes[s.name] = code
            elif s.kind == "flatten":
                x = x.reshape(x.shape[0], -1)
            elif s.kind == "dense":
                x = self._dense_up(x, s.name)
            if keep_all:
                st.outputs[s.name] = x
            i += 1
        st.out = x
        return st

    # ------------------------------------------------------------------ selection
    @staticmethod
    def select_filters(out: torch.Tensor, k: int, batch_topk: str = "per_image"):
        """Top-k positive filters (app/deepdream.py:369-380). Returns idx [B, k], val [B, k]."""
        B = out.shape[0]
        sums = ops.channel_sum(out) if out.dim() == 4 else out.float()
        if batch_topk == "global":
            g = sums.sum(dim=0, keepdim=True)
            idx, val = ops.topk_positive(g, k)
            return idx.expand(B, k).contiguous(), val.expand(B, k).contiguous()
        return ops.topk_positive(sums, k)

    # ------------------------------------------------------------------ backward
    def _seed_map(self, out4: torch.Tensor, idx: torch.Tensor, mode: str, batch_topk: str,
                  code: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One-channel seed maps S [B*K, H, W] fp32 from the target output (app/deepdream.py:450-465);
        unpooled to [B*K, 2H, 2W] with ``code`` for pool targets (ops.seed_map: one HIP kernel)."""
        return ops.seed_map(out4, idx, mode, batch_topk, code)

    def backward(self, st: ForwardState, idx: torch.Tensor, mode: str = "all",
                 batch_topk: str = "per_image", layer: Optional[str] = None,
                 stats: Optional[torch.Tensor] = None) -> torch.Tensor:
        """B*K deconv chains from ``layer`` (default: the forward target) to the input.
        Returns fp32 reconstructions [B, K, 224, 224, 3]. ``stats`` (GPU, fp64 [B, 2]) receives each
        image's {sum, sum of squares} over its K reconstructions from the final conv's epilogue."""
        if mode not in VALID_MODES:
            raise ValueError(f"Illegal visualize mode {mode!r}; use 'all' or 'max'")
        layer = layer or st.target
        li = self.names.index(layer)
        spec = self.specs[li]
        B, K = idx.shape
        dev = idx.device
        out = st.outputs.get(layer, st.out) if layer != st.target else st.out
        f = idx.reshape(B * K).to(torch.int32)
        d: Optional[torch.Tensor] = None
        seed_scale: Optional[torch.Tensor] = None  # fp16 dense seeds: per-chain scale of the reconstruction
        pending_code: Optional[torch.Tensor] = None
        j = li  # index of the layer whose down is applied next
        if spec.kind == "conv":
            S = self._seed_map(out, idx, mode, batch_topk)
            d = ops.seed_deconv3x3(S, f, self.rt.convs[layer].seed_wt)
            j = li - 1
        elif spec.kind == "pool":
            # seed at pooled resolution, max-unpooled with this pool's switches (one kernel), then
            # the conv below
            Su = self._seed_map(out, idx, mode, batch_topk, code=st.codes[layer])  # [BK, 2PH, 2PW]
            conv_name = self.specs[li - 1].name
            d = ops.seed_deconv3x3(Su, f, self.rt.convs[conv_name].seed_wt)
            j = li - 2
        else:
            # dense / flatten target: one-hot (unit f) seeds, then linear downs
            units = out.shape[1]
            v = torch.gather(out.float(), 1, idx.long().clamp_min(0))  # [B, K]
            if mode == "max" and batch_topk == "global":
                # the reference's max runs over the batch axis of output[:, f] (:454-457)
                v = v * (v == v.amax(dim=0, keepdim=True))
            v = v * (idx >= 0)
            if dev.type == "cuda" and self.rt.dtype == torch.float16:
                # fp16 (smallest subnormal 6e-8) cannot carry a softmax probability through the dense
                # downs; the deconv chain is positively homogeneous (bias-free convs, ReLU, max-unpool),
                # so it runs from a unit seed and the reconstruction is scaled by |v| at the end
                seed_scale = v.abs().reshape(B * K)
                v = torch.sign(v)
            seed = torch.zeros(B * K, units, device=dev, dtype=torch.float32)
            seed.scatter_(1, idx.reshape(B * K, 1).long().clamp_min(0), v.reshape(B * K, 1))
            d = seed
            j = li
            while self.specs[j].kind == "dense":
                dl = self.rt.dense[self.specs[j].name]
                relu_below = self.specs[j - 1].kind == "dense"  # the lower dense layer's activation.down
                if d.is_cuda and dl.down is not None:
                    M = d.shape[0]
                    d = ops.conv2d(d.reshape(M, 1, 1, -1).to(self.rt.dtype).contiguous(), dl.down, relu=relu_below,
                                   pad=0, epilogue="f32", use_bias=False).reshape(M, -1)
                else:
                    d = torch.matmul(d.to(dl.wt.dtype), dl.wt).float()
                    if relu_below:
                        d = d.clamp_min(0)
                j -= 1
            assert self.specs[j].kind == "flatten"
            fs = self.specs[j]
            d = d.reshape(B * K, fs.out_hw, fs.out_hw, fs.cin).to(self.rt.dtype if dev.type == "cuda" else torch.float32)
            pending_code = st.codes["block5_pool"]
            j -= 2  # skip flatten and block5_pool (its unpool is fused into block5_conv3's down)
        # ---- conv / pool downs to the input ----
        recon = None
        if seed_scale is not None:  # the final conv's epilogue statistics would be of the unit-seed chains
            stats_out, stats = stats, None
        while j >= 1:
            s = self.specs[j]
            if s.kind == "pool":
                pending_code = st.codes[s.name]
                j -= 1
                continue
            assert s.kind == "conv", s
            cl = self.rt.convs[s.name]
            last = j == 1
            kw = dict(relu=True, epilogue="f32" if last else "bf16", use_bias=False)
            if last and stats is not None:
                kw.update(stats=stats, stats_div=K)
            # down = ReLU(convT(ReLU(signal))) (app/deepdream.py:110,260). The input ReLU only acts on
            # an unpooled signal (the unpool consumes it for free): every other input is already a
            # ReLU output (seed stencil, conv-down epilogues), so relu_in would be a no-op pass
            # a conv-down feeding an unpool writes the unpooled map straight from its epilogue (no pooled
            # round trip, no separate unpool pass) unless the consumer is a 64-channel conv, whose
            # halo kernel fuses the unpool into its input staging instead (reads 1/4 of the bytes)
            below = self.specs[j - 1] if j >= 2 else None
            fuse_unpool = (below is not None and below.kind == "pool" and j >= 3 and pending_code is None and
                           cl.dec.cout % 8 == 0 and
                           (not d.is_cuda or self.rt.convs[self.specs[j - 2].name].dec.cin > UNPOOL_CONSUMER_MAXC))
            if pending_code is not None and j == 2 and self.specs[1].kind == "conv" and d.is_cuda:
                # unpool -> block1_conv2.down -> block1_conv1.down as two kernels (the 64-channel map
                # stays on chip: ops.deconv_tail); None if the shape is not the kernel's
                r = ops.deconv_tail(d, pending_code, K, cl.dec, self.rt.convs[self.specs[1].name].dec,
                                    stats=stats, stats_div=K)
                if r is not None:
                    recon = r
                    pending_code = None
                    break
            if pending_code is not None:
                d = ops.conv2d(d, cl.dec, in_mode="unpool", code=pending_code, code_div=K, relu_in=True, **kw)
                pending_code = None
            elif fuse_unpool:
                d = ops.conv2d(d, cl.dec, unpool_out=st.codes[below.name], unpool_div=K, **kw)
                j -= 1  # the pool's unpool is done
            else:
                d = ops.conv2d(d, cl.dec, **kw)
            if last:
                recon = d
            j -= 1
        if recon is None:  # target was block1_conv1: the seed step already produced the image
            recon = d[..., :3].float().contiguous()
            if stats is not None:  # no fp32 conv epilogue on this path: sums over each image's K maps
                r = recon.reshape(B, -1).double()
                stats.copy_(torch.stack([r.sum(1), (r * r).sum(1)], 1))
        if seed_scale is not None:
            recon = recon * seed_scale.view(-1, *([1] * (recon.dim() - 1)))
            if stats_out is not None:
                r = recon.reshape(B, -1).double()
                stats_out.copy_(torch.stack([r.sum(1), (r * r).sum(1)], 1))
        return recon.reshape(B, K, *recon.shape[1:])

    # ------------------------------------------------------------------ one call
    def run(self, x: torch.Tensor, layer: str, k: int = 4, mode: str = "all",
            batch_topk: str = "per_image", mosaic: bool = True, hook=None) -> DeconvResult:
        if mode not in VALID_MODES:
            raise ValueError(f"Illegal visualize mode {mode!r}; use 'all' or 'max'")
        S = DECONV_STREAMS
        if S > 1 and x.is_cuda and batch_topk == "per_image" and x.shape[0] >= max(DECONV_SPLIT_MIN, S):
            return self._run_split(x, layer, k, mode, mosaic, hook, S)
        return self._run1(x, layer, k, mode, batch_topk, mosaic, hook)

    def _run_split(self, x, layer, k, mode, mosaic, hook, S) -> DeconvResult:
        dev = x.device
        if len(getattr(self, "_streams", ())) < S:
            self._streams = [torch.cuda.Stream(dev) for _ in range(S)]
        cur = torch.cuda.current_stream(dev)
        parts = []
        for i, xp in enumerate(x.chunk(S)):
            sm = self._streams[i]
            sm.wait_stream(cur)
            with torch.cuda.stream(sm):
                parts.append(self._run1(xp, layer, k, mode, "per_image", mosaic, hook if i == 0 else None))
        for sm in self._streams[:S]:
            cur.wait_stream(sm)
        for r in parts:  # read on the caller's stream from here on
            for t in (r.recon, r.filters, r.sums, r.mosaic):
                if t is not None:
                    t.record_stream(cur)
        res = DeconvResult(torch.cat([r.recon for r in parts]), torch.cat([r.filters for r in parts]),
                           torch.cat([r.sums for r in parts]))
        if parts[0].mosaic is not None:
            res.mosaic = torch.cat([r.mosaic for r in parts])
        return res

    def _run1(self, x, layer, k, mode, batch_topk, mosaic, hook) -> DeconvResult:
        with tracing.range_("dv.forward"):
            st = self.forward(x, layer, hook=hook)
        with tracing.range_("dv.select"):
            idx, val = self.select_filters(st.out, k, batch_topk)
        stats = None
        if mosaic and k == 4 and x.is_cuda and layer != "block1_conv1":  # deprocess stats from the last conv
            stats = torch.empty(x.shape[0], 2, dtype=torch.float64, device=x.device)
        with tracing.range_("dv.backward"):
            recon = self.backward(st, idx, mode, batch_topk, stats=stats)
        res = DeconvResult(recon, idx, val)
        if mosaic and k == 4:
            B = recon.shape[0]
            with tracing.range_("dv.deprocess"):
                res.mosaic = ops.deprocess_mosaic(recon.reshape(B * 4, *recon.shape[2:]).contiguous(), 4, True,
                                                  stats=stats)
        return res


def visualize_all_layers(engine: DeconvNet, data: torch.Tensor, layer_name: str = "predictions",
                         visualize_mode: str = "all", *, all_layers: bool = True, top: int = 8,
                         batch_topk: str = "global") -> Dict[str, List]:
    """Library-parity API of app/deepdream.py:383-476.

    Returns ``{layer: [recon, ...]}`` with one squeezed reconstruction per selected filter (at most
    ``top``; filters with non-positive sums are dropped as in find_top_filters). With
    ``all_layers=True`` every conv/pool/flatten/dense layer <= ``layer_name`` is visualized, as
    the reference does; ``False`` visualizes only the target. Illegal modes raise ValueError
    (the reference calls sys.exit, :458-460)."""
    if visualize_mode not in VALID_MODES:
        raise ValueError(f"Illegal visualize mode {visualize_mode!r}")
    st = engine.forward(data, layer_name, fuse_pools=not all_layers, keep_all=all_layers)
    ti = engine.names.index(layer_name)
    layers = [s.name for s in engine.specs[1: ti + 1] if s.kind in ("conv", "pool", "flatten", "dense")]
    if not all_layers:
        layers = [layer_name]
    result: Dict[str, List] = {}
    for name in reversed(layers):
        out = st.outputs.get(name, st.out) if all_layers else st.out
        sub = ForwardState(name, out, st.codes, st.outputs)
        idx, val = engine.select_filters(out, top, batch_topk)
        nsel = int((idx[0] >= 0).sum().item()) if batch_topk == "global" else top
        recon = engine.backward(sub, idx, visualize_mode, batch_topk, layer=name)
        lst = []
        for kk in range(nsel):
            r = recon[:, kk]
            lst.append(r.squeeze(0).cpu().numpy() if r.shape[0] == 1 else r.cpu().numpy())
        result[name] = lst
    return result
