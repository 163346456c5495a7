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

from . import native
from .autograd import _PREMASKED, ConvUnit, _dgrad_strided, _is_relu_out, _tag
from .conv import conv2d


def _pool_out(L: int, k: int, s: int, p: int) -> int:
    return (L + 2 * p - k) // s + 1


class InceptionBlock:
    def __init__(self, name: str, order: Sequence[str], branches: Dict[str, list], units: Dict[str, ConvUnit]):
        self.name = name
        self.order = list(order)
        self.branches = [branches[k] for k in self.order]
        self.units = units

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
        plan = []  # per branch: (offset, width, kind, [saved tensor indices / unit names])
        off = 0
        for ops, wdt in zip(blk.branches, widths):
            ysl = Y[..., off:off + wdt]
            if ops[0] == "avg":  # avg -> 1x1 conv  ==  1x1 conv (no bias) -> avg + bias + ReLU
                assert len(ops) == 2 and isinstance(ops[1], str), "avg branch: avg-pool then one 1x1 conv"
                u = blk.units[ops[1]]
                assert u.w.shape[2:] == (1, 1) and u.stride == 1
                t = _conv_fwd(u, x, relu=False, bias=False)
                lib.pool(t, ysl, None, 1, 0, _pool_geom(N, H, W, u.cout, 3, 1, 1), u.fwd.bias_pad, True)
                plan.append((off, wdt, "avg", [u.name]))
            elif ops == ["max"]:
                idx = torch.empty(N, OH, OW, Cin, dtype=torch.uint8, device=x.device)
                lib.pool(x, ysl, idx, 0, 0, _pool_geom(N, H, W, Cin, 3, 2, 0))
                saved.append(idx)
                plan.append((off, wdt, "max", [len(saved) - 1]))
            else:
                steps = []  # (unit name(s), index of its saved input)
                cur, cur_i = x, 0
                for j, op in enumerate(ops):
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
                            cur, cur_i = y, len(saved) - 1
                plan.append((off, wdt, "convs", steps))
            off += wdt
        ctx.blk = blk
        ctx.plan = plan
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
        N, H, W, Cin = x.shape
        gY = gY.contiguous()
        if not ctx.premasked:
            gY = torch.ops.aten.threshold_backward(gY, Y, 0)
        emask_x = x if (ctx.premasked and ctx.x_relu) else None
        gx = torch.empty_like(x)
        state = {"written": False, "masked": False}

        def contribute_conv(u: ConvUnit, g, emask):
            """gradient of conv unit u (stride 1) w.r.t. its input, written/accumulated into gx"""
            conv2d(g, u.bwd, stride=1, pad=u.bwd_pad, relu=False, use_bias=False, out=gx,
                   accumulate=state["written"], emask=emask)
            state["written"] = True
            state["masked"] = emask is not None

        def contribute_tensor(t):
            if state["written"]:
                gx.add_(t)
            else:
                gx.copy_(t)
            state["written"] = True
            state["masked"] = False

        deferred = []  # stride-1 head-conv contributions go last: their epilogue applies the x mask
        for off, wdt, kind, info in ctx.plan:
            gsl = gY[..., off:off + wdt]
            if kind == "max":
                idx = saved[info[0]]
                if state["written"]:
                    t = torch.empty_like(x)
                    lib.pool(gsl, t, idx, 0, 1, _pool_geom(N, H, W, Cin, 3, 2, 0))
                    contribute_tensor(t)
                else:
                    lib.pool(gsl, gx, idx, 0, 1, _pool_geom(N, H, W, Cin, 3, 2, 0))
                    state["written"] = True
                continue
            if kind == "avg":
                u = blk.units[info[0]]
                gp = torch.empty(N, H, W, u.cout, dtype=gY.dtype, device=gY.device)
                lib.pool(gsl, gp, None, 1, 1, _pool_geom(N, H, W, u.cout, 3, 1, 1))
                deferred.append((u, gp))
                continue
            # conv chain: walk it backwards; gradient w.r.t. each ReLU output is premasked
            g = gsl
            for names, in_i in reversed(info):
                units = [blk.units[n] for n in names]
                inp = saved[in_i]
                if in_i == 0:  # head conv(s) on the block input
                    if len(units) == 2:
                        ua, ub = units
                        deferred.append((ua, g[..., : ua.cout]))
                        deferred.append((ub, g[..., ua.cout:]))
                    elif units[0].stride == 1:
                        deferred.append((units[0], g))
                    else:
                        contribute_tensor(_dgrad_strided(units[0], g, None, (H, W)))
                    continue
                if len(units) == 2:  # split on an intermediate: sum of two dgrads, masked by inp > 0
                    ua, ub = units
                    gi = conv2d(g[..., : ua.cout], ua.bwd, stride=1, pad=ua.bwd_pad, relu=False, use_bias=False,
                                emask=inp)
                    conv2d(g[..., ua.cout:], ub.bwd, stride=1, pad=ub.bwd_pad, relu=False, use_bias=False,
                           emask=inp, out=gi, accumulate=True)
                    g = gi
                    continue
                u = units[0]
                if u.stride == 1:
                    g = conv2d(g, u.bwd, stride=1, pad=u.bwd_pad, relu=False, use_bias=False, emask=inp)
                else:
                    g = torch.ops.aten.threshold_backward(
                        _dgrad_strided(u, g, None, (inp.shape[1], inp.shape[2])), inp, 0)
        for u, g in deferred:
            contribute_conv(u, g, emask_x)
        if emask_x is not None and not state["masked"]:
            gx = torch.ops.aten.threshold_backward(gx, emask_x, 0)
        return gx, None
