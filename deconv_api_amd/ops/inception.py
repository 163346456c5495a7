"""InceptionV3 mixed block as ONE differentiable unit with a hand-written forward and backward.

Branch programs (the Keras topology, models/inception_v3.py) are lists of ops on the block
input: a conv unit name, ``"avg"`` (3x3/1 avg-pool, count_include_pad=False), ``"max"`` (3x3/2
max-pool) or ``("split", a, b)`` (two convs of the same input, concatenated). The block output is
the channel concat of the branches in Keras order.

GPU design (every op a HIP kernel, no torch glue):
  * the concat buffer Y is allocated once; the last op of every branch writes its channel slice
    directly (conv epilogue / pool kernel with an output pixel stride), so there is no torch.cat;
  * the pool branch ``avg -> 1x1 conv`` runs as ``1x1 conv -> avg + bias + ReLU``: both are
    linear and the pool's divisor does not depend on the channel, so they commute; the pool then
    runs over the conv's 32-192 output channels instead of the 192-768 input channels;
  * every 1x1 head conv on the block input that is NOT a branch's only op (b5a, b3a, b7a, b7da,
    the commuted pool conv) is ONE merged GEMM T = x @ [W_b5a | W_b3a | W_pool] with bias + ReLU
    on the leading columns only (``relu_cols``; the pool columns stay pre-activation); the
    branches read their heads as channel slices of T. Backward, the heads' gradients are written
    into the matching slices of one G_T and ONE dgrad GEMM (K = all head channels) accumulates
    them into gx: 2-3 launches fewer per block each way (the small-map blocks are launch-bound);
  * backward reads gY's channel slices in place; every contribution to the block-input gradient
    gx is written by one kernel epilogue into the same buffer (the first writes, the rest use the
    ``accumulate`` epilogue), with the ReLU mask of x (``emask``) fused there: no add kernels, no
    zero fills, no threshold_backward passes. The avg branch's backward pools the small gradient
    first (commuted again), then its 1x1 dgrad accumulates into gx.

The backward follows the premasked-gradient contract of ops/autograd.py: gY is zero where Y is
(DeepDream's sum-of-squares loss and every unit of that module keep it); outside that contract
the block masks gY itself. CPU tensors take the plain torch path (the oracle).
"""
from __future__ import annotations

from typing import Dict, List, Sequence

import torch
import torch.nn.functional as F

from .. import knobs
from . import native
from .autograd import _PREMASKED, ConvUnit, _is_relu_out, _tag, dgrad_strided_into
from .conv import conv2d, conv_group, conv_group_paused

# DV_MERGE_B1=0: the b1 branch as its own GEMM (A/B); default: it joins the merged head GEMM forward
MERGE_B1 = knobs.ablation("DV_MERGE_B1", "1") != "0"


def _pool_out(L: int, k: int, s: int, p: int) -> int:
    return (L + 2 * p - k) // s + 1


class InceptionBlock:
    def __init__(self, name: str, order: Sequence[str], branches: Dict[str, list], units: Dict[str, ConvUnit]):
        self.name = name
        self.order = list(order)
        self.branches = [branches[k] for k in self.order]
        self.units = units
        self.merge = None  # (fwd ConvWeights, bwd ConvWeights, relu_cols, {branch index: (offset, width)})
        self.merge_b1 = None  # (b1 branch index, b1 width, forward ConvWeights of [W_b1 | heads], relu_cols)

    @staticmethod
    def _is_head(u: ConvUnit) -> bool:
        return tuple(u.w.shape[2:]) == (1, 1) and u.stride == 1 and tuple(u.pad) == (0, 0)

    def build(self, device, dtype) -> "InceptionBlock":
        """GPU: pack the merged head GEMM (see module doc) when >= 2 heads qualify."""
        from .conv import ConvWeights, pad_channels_oihw

        self.merge = None
        if torch.device(device).type != "cuda":
            return self
        relu_m, pre_m = [], []
        for bi, ops in enumerate(self.branches):
            if ops[0] == "avg":
                pre_m.append((bi, self.units[ops[1]]))
            elif isinstance(ops[0], str) and ops[0] != "max" and len(ops) > 1 and self._is_head(self.units[ops[0]]):
                relu_m.append((bi, self.units[ops[0]]))
        members = relu_m + pre_m
        if len(members) < 2:
            return self
        cols, off = {}, 0
        ws, bs = [], []
        for k, (bi, u) in enumerate(members):
            cols[bi] = (off, u.cout)
            off += u.cout
            ws.append(u.w)
            bs.append(u.b if k < len(relu_m) else torch.zeros_like(u.b))  # pool bias: after the avg
        w = pad_channels_oihw(torch.cat(ws, 0))                             # [Ntot, Cin8, 1, 1]
        fwd = ConvWeights(w, torch.cat(bs, 0), "fwd").to_device(device, dtype)
        bwd = ConvWeights(pad_channels_oihw(w.transpose(0, 1).contiguous()), None, "fwd").to_device(device, dtype)
        self.merge = (fwd, bwd, sum(u.cout for _, u in relu_m), cols)
        # the b1 branch (a lone 1x1 conv on x, its output a concat slice) joins the FORWARD GEMM as
        # its leading columns, written straight into Y by the two-destination epilogue (out2): one
        # launch fewer per block; its backward stays a separate dgrad (its gradient is a gY slice)
        self.merge_b1 = None
        if MERGE_B1:
            for bi, ops in enumerate(self.branches):
                if len(ops) == 1 and isinstance(ops[0], str) and ops[0] not in ("avg", "max") and \
                        self._is_head(self.units[ops[0]]) and self.units[ops[0]].cout % 8 == 0:
                    u1 = self.units[ops[0]]
                    w1 = pad_channels_oihw(torch.cat([u1.w] + ws, 0))
                    b1 = torch.cat([u1.b] + bs, 0)
                    fwd1 = ConvWeights(w1, b1, "fwd").to_device(device, dtype)
                    self.merge_b1 = (bi, u1.cout, fwd1, u1.cout + self.merge[2])
                    break
        return self

    # ------------------------------------------------------------------ shapes
    def branch_width(self, ops, cin: int) -> int:
        last = ops[-1]
        if last in ("avg", "max"):
            return cin
        if isinstance(last, tuple):
            return self.units[last[1]].cout + self.units[last[2]].cout
        return self.units[last].cout

    def widths(self, cin: int) -> List[int]:
        return [self.branch_width(ops, cin) for ops in self.branches]

    def out_hw(self, H: int, W: int):
        for ops in self.branches:
            for op in ops:
                if op == "max":
                    return _pool_out(H, 3, 2, 0), _pool_out(W, 3, 2, 0)
                if isinstance(op, str) and op != "avg" and self.units[op].stride > 1:
                    u = self.units[op]
                    kh, kw = u.w.shape[2:]
                    return _pool_out(H, kh, u.stride, u.pad[0]), _pool_out(W, kw, u.stride, u.pad[1])
        return H, W

    # ------------------------------------------------------------------ execution
    def __call__(self, x: torch.Tensor) -> torch.Tensor:
        if x.is_cuda:
            return _tag(_InceptionFn.apply(x, self), True)
        return torch.cat([self._branch_ref(x, ops) for ops in self.branches], dim=3)

    def _branch_ref(self, x, ops):
        for op in ops:
            if op == "avg":
                x = F.avg_pool2d(x.permute(0, 3, 1, 2), 3, 1, 1, count_include_pad=False).permute(0, 2, 3, 1)
            elif op == "max":
                x = F.max_pool2d(x.permute(0, 3, 1, 2), 3, 2, 0).permute(0, 2, 3, 1)
            elif isinstance(op, tuple):
                x = torch.cat([self.units[op[1]](x), self.units[op[2]](x)], dim=3)
            else:
                x = self.units[op](x)
        return x


def _conv_fwd(u: ConvUnit, x, out=None, relu=True, bias=True):
    return conv2d(x, u.fwd, stride=u.stride, pad=u.pad, relu=relu, use_bias=bias, out=out)


def _pool_geom(N, H, W, C, k, s, p):
    return [N, H, W, C, _pool_out(H, k, s, p), _pool_out(W, k, s, p), k, s, p]


class _InceptionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, blk: InceptionBlock):
        lib = native.lib()
        x = x.contiguous()
        N, H, W, Cin = x.shape
        OH, OW = blk.out_hw(H, W)
        widths = blk.widths(Cin)
        Y = torch.empty(N, OH, OW, sum(widths), dtype=x.dtype, device=x.device)
        saved = [x, Y]
        T = None
        mcols = {}
        b1_done = None
        if blk.merge is not None:  # every qualifying 1x1 head in one GEMM (pool columns pre-activation)
            mfwd, _, relu_n, mcols = blk.merge
            if blk.merge_b1 is not None:  # + the b1 branch as leading columns, written into its Y slice
                b1i, n1, fwd1, relu1 = blk.merge_b1
                o1 = sum(widths[:b1i])
                T = torch.empty(N, H, W, mfwd.cout, dtype=x.dtype, device=x.device)
                conv2d(x, fwd1, stride=1, pad=(0, 0), relu=True, use_bias=True, relu_cols=relu1,
                       out=Y[..., o1:o1 + n1], out2=T, split_col=n1)
                b1_done = b1i
            else:
                T = conv2d(x, mfwd, stride=1, pad=(0, 0), relu=True, use_bias=True, relu_cols=relu_n)
            saved.append(T)
        # Per branch: (offset, width, kind, info). Pool branches run first; the conv chains then
        # advance in LEVELS: level l runs op l of every chain that still has one (a merged head's
        # op 0 already ran in the head GEMM). The convs of one level read only their own chain's
        # previous output, so each level is one conv_group: its small problems launch together.
        plan = [None] * len(blk.branches)
        chains = {}  # branch index -> [ops, next op index, cur, cur_i, steps, Y slice]
        off = 0
        for bi, (ops, wdt) in enumerate(zip(blk.branches, widths)):
            ysl = Y[..., off:off + wdt]
            if ops[0] == "avg":  # avg -> 1x1 conv  ==  1x1 conv (no bias) -> avg + bias + ReLU
                assert len(ops) == 2 and isinstance(ops[1], str), "avg branch: avg-pool then one 1x1 conv"
                u = blk.units[ops[1]]
                assert u.w.shape[2:] == (1, 1) and u.stride == 1
                if bi in mcols:
                    mo, mw = mcols[bi]
                    t = T[..., mo:mo + mw]
                else:
                    t = _conv_fwd(u, x, relu=False, bias=False)
                lib.pool(t, ysl, None, 1, 0, _pool_geom(N, H, W, u.cout, 3, 1, 1), u.fwd.bias_pad, True)
                plan[bi] = (off, wdt, "avg", [u.name, mcols.get(bi)])
            elif ops == ["max"]:
                idx = torch.empty(N, OH, OW, Cin, dtype=torch.uint8, device=x.device)
                lib.pool(x, ysl, idx, 0, 0, _pool_geom(N, H, W, Cin, 3, 2, 0))
                saved.append(idx)
                plan[bi] = (off, wdt, "max", [len(saved) - 1])
            else:
                steps = []  # (unit name(s), index of its saved input | ("T", cols) for a merged head)
                ch = [ops, 0, x, 0, steps, ysl]
                if bi in mcols:  # the head ran in the merged GEMM: its output is a slice of T
                    mo, mw = mcols[bi]
                    ch[2], ch[3] = T[..., mo:mo + mw], ("T", mo, mw)
                    steps.append(((ops[0],), "merged"))
                    ch[1] = 1
                if bi == b1_done:  # computed by the merged forward GEMM (backward: its own dgrad)
                    steps.append(((ops[0],), 0))
                    ch[1] = len(ops)
                chains[bi] = ch
                plan[bi] = (off, wdt, "convs", steps)
            off += wdt
        while any(ch[1] < len(ch[0]) for ch in chains.values()):
            with conv_group(x.device):
                for ch in chains.values():
                    ops, j, cur, cur_i, steps, ysl = ch
                    if j >= len(ops):
                        continue
                    op = ops[j]
                    last = j == len(ops) - 1
                    if isinstance(op, tuple):
                        assert last, "split must end its branch"
                        ua, ub = blk.units[op[1]], blk.units[op[2]]
                        _conv_fwd(ua, cur, out=ysl[..., : ua.cout])
                        _conv_fwd(ub, cur, out=ysl[..., ua.cout:])
                        steps.append(((op[1], op[2]), cur_i))
                    else:
                        y = _conv_fwd(blk.units[op], cur, out=ysl if last else None)
                        steps.append(((op,), cur_i))
                        if not last:
                            saved.append(y)
                            ch[2], ch[3] = y, len(saved) - 1
                    ch[1] = j + 1
        ctx.blk = blk
        ctx.plan = plan
        ctx.merged = T is not None
        ctx.premasked = _PREMASKED[0]
        ctx.x_relu = _is_relu_out(x)
        ctx.save_for_backward(*saved)
        return Y

    @staticmethod
    def backward(ctx, gY):
        lib = native.lib()
        blk: InceptionBlock = ctx.blk
        saved = ctx.saved_tensors
        x, Y = saved[0], saved[1]
        T = saved[2] if ctx.merged else None
        N, H, W, Cin = x.shape
        gY = gY.contiguous()
        if not ctx.premasked:
            gY = torch.ops.aten.threshold_backward(gY, Y, 0)
        emask_x = x if (ctx.premasked and ctx.x_relu) else None
        gx = torch.empty_like(x)
        GT = torch.empty_like(T) if T is not None else None
        state = {"written": False, "masked": False}

        def inp_of(in_i):
            if isinstance(in_i, tuple):  # merged head output: slice of T
                return T[..., in_i[1]:in_i[1] + in_i[2]]
            return saved[in_i]

        def contribute_conv(cw, g, emask):
            """gradient of a stride-1 conv (packed transposed weights cw) w.r.t. its input,
            written (first contribution) or accumulated into gx, x-mask fused when given"""
            conv2d(g, cw, stride=1, pad=(cw.KH // 2, cw.KW // 2), relu=False, use_bias=False, out=gx,
                   accumulate=state["written"], emask=emask)
            state["written"] = True
            state["masked"] = emask is not None

        def dgrad_into(u, g, inp, out=None, accumulate=False):
            """gradient w.r.t. ``inp`` (a ReLU output) of conv unit u, masked by inp > 0"""
            if u.stride == 1:
                return conv2d(g, u.bwd, stride=1, pad=u.bwd_pad, relu=False, use_bias=False, emask=inp, out=out,
                              accumulate=accumulate)
            if out is None:
                out = torch.empty_like(inp)
            return dgrad_strided_into(u, g, (inp.shape[1], inp.shape[2]), out, accumulate, emask=inp)

        deferred = []  # head-conv contributions on x go last: their epilogue applies the x mask
        chains = []  # per conv branch: [reversed steps, next index, current gradient]
        for off, wdt, kind, info in ctx.plan:
            gsl = gY[..., off:off + wdt]
            if kind == "max":
                idx = saved[info[0]]
                # written before: the kernel adds its window sums to gx in the same pass (no separate
                # pool-into-temporary + ATen add launch)
                lib.pool(gsl, gx, idx, 0, 1, _pool_geom(N, H, W, Cin, 3, 2, 0), accumulate=state["written"])
                state["written"] = True
                state["masked"] = False
                continue
            if kind == "avg":
                u = blk.units[info[0]]
                if info[1] is not None:  # merged: the pooled gradient lands in its G_T columns
                    mo, mw = info[1]
                    lib.pool(gsl, GT[..., mo:mo + mw], None, 1, 1, _pool_geom(N, H, W, u.cout, 3, 1, 1))
                else:
                    gp = torch.empty(N, H, W, u.cout, dtype=gY.dtype, device=gY.device)
                    lib.pool(gsl, gp, None, 1, 1, _pool_geom(N, H, W, u.cout, 3, 1, 1))
                    deferred.append((u.bwd, gp))
                continue
            chains.append([list(reversed(info)), 0, gsl])
        # conv chains walked backwards in levels (step l of every chain; the gradient w.r.t. each
        # ReLU output is premasked): one conv_group per level, like the forward. Inside a group a
        # recorded conv runs only at the group's end, so every step that reads a conv result it
        # launched itself (strided dgrads: sub-pixel GEMMs + copies; a split's accumulating pair)
        # runs with recording paused
        while any(c[1] < len(c[0]) for c in chains):
            with conv_group(x.device):
                for c in chains:
                    if c[1] >= len(c[0]):
                        continue
                    names, in_i = c[0][c[1]]
                    c[1] += 1
                    g = c[2]
                    units = [blk.units[n] for n in names]
                    if in_i == "merged":
                        continue  # the head's own dgrad is part of the merged G_T GEMM below
                    inp = None if in_i == 0 else inp_of(in_i)
                    into = GT[..., in_i[1]:in_i[1] + in_i[2]] if isinstance(in_i, tuple) else None
                    if in_i == 0:  # unmerged head conv(s) on the block input
                        if len(units) == 2:
                            ua, ub = units
                            deferred.append((ua.bwd, g[..., : ua.cout]))
                            deferred.append((ub.bwd, g[..., ua.cout:]))
                        elif units[0].stride == 1:
                            deferred.append((units[0].bwd, g))
                        else:  # strided head on x: straight into gx (written / accumulated)
                            with conv_group_paused():  # may be GEMMs + torch ops reading them
                                dgrad_strided_into(units[0], g, (H, W), gx, accumulate=state["written"])
                            state["written"] = True
                            state["masked"] = False
                        continue
                    if len(units) == 2:  # split: sum of two dgrads, masked by inp > 0
                        ua, ub = units
                        with conv_group_paused():  # the second accumulates into the first: in order
                            gi = dgrad_into(ua, g[..., : ua.cout], inp, out=into)
                            dgrad_into(ub, g[..., ua.cout:], inp, out=gi, accumulate=True)
                        c[2] = gi
                    elif units[0].stride == 1:  # one conv: recorded into the level's group
                        c[2] = dgrad_into(units[0], g, inp, out=into)
                    else:  # strided: sub-pixel GEMMs + torch ops that read them, in order
                        with conv_group_paused():
                            c[2] = dgrad_into(units[0], g, inp, out=into)
        if GT is not None:
            deferred.append((blk.merge[1], GT))
        for cw, g in deferred:
            contribute_conv(cw, g, emask_x)
        if emask_x is not None and not state["masked"]:
            gx = torch.ops.aten.threshold_backward(gx, emask_x, 0)
        return gx, None
