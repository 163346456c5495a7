"""Compare one tiled gradient step: torch implementation vs fused kernels (gather/pack)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DreamSettings, TiledDeepDream  # noqa: E402
from deconv_api_amd.models.resnet50 import ResNet50  # noqa: E402

dt = torch.float16 if (len(sys.argv) < 2 or sys.argv[1] == "fp16") else torch.bfloat16
net = ResNet50(0).build("cuda", dt)
s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=1, iterations=1, max_loss=None)
x = (torch.rand(2, 200, 260, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1).cuda()
if len(sys.argv) > 2:
    x = x[:, :int(sys.argv[2]), :int(sys.argv[3])].contiguous()
dd = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=False)
B, H, W, _ = x.shape
plan = dd._plan(B, H, W, x.device)
for sh in [(0, 0), (17, -33)]:
    shift = torch.tensor(sh, dtype=torch.long, device="cuda")
    grad = torch.zeros_like(x)
    loss = torch.zeros(B, device="cuda")
    dd._tile_grad(x, shift, plan, grad, loss)
    st = dd._tstate(B, H, W)
    st.x.copy_(x)
    st.shifts[0] = torch.tensor(sh, dtype=torch.int32)
    dd._tile_compute(st, 0)
    torch.cuda.synchronize()
    pk = st.packs[0, st.rank].float().cpu()
    pl = st.plan.cpu()
    us = ((st.Th * st.Tw * 3 + 7) // 8) * 8
    full = torch.zeros(B, H, W, 3)
    tail = st.packs[0, st.rank][st.ucc * us:].view(torch.float32).cpu()[: 32 * pl.shape[0]].view(-1, 32)[:, :2].reshape(-1) if dt == torch.float16 else None
    for u in range(pl.shape[0]):
        b, oy, ox, y0, y1, x0, x1 = pl[u].tolist()
        blk = pk[u * us: u * us + (y1 - y0) * (x1 - x0) * 3].view(y1 - y0, x1 - x0, 3)
        for ty in range(y0, y1):
            yy = (oy + ty - sh[0]) % H
            xs = [(ox + tx - sh[1]) % W for tx in range(x0, x1)]
            full[b, yy, xs] = blk[ty - y0]
    g = grad.cpu()
    print(sh, "max|old|", g.abs().max().item(), "max|diff|", (full - g).abs().max().item(),
          "rel", ((full - g).norm() / g.norm()).item())
    print(" old loss", loss.tolist(), "unit tails", tail[: 2 * pl.shape[0]].view(-1, 2)[:, 0].tolist() if tail is not None else None)
