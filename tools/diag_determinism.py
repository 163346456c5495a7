"""Run the same DeepDream gradient computation N times and compare results bitwise (kernel races)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.engine.deepdream import RESNET_LAYERS, DreamSettings, TiledDeepDream  # noqa: E402
from deconv_api_amd.models.resnet50 import ResNet50  # noqa: E402

net = ResNet50(0).build("cuda", torch.float16)
s = DreamSettings(layers=dict(RESNET_LAYERS), octaves=1, iterations=1, max_loss=None)
for hw in [(71, 93), (200, 260)]:
    x = (torch.rand(2, *hw, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1).cuda()
    dd = TiledDeepDream(net, s, tile=128, seed=3, use_graphs=False)
    st = dd._tstate(2, *hw)
    st.x.copy_(x)
    ref = None
    bad = 0
    for r in range(20):
        dd._tile_compute(st, 0)
        torch.cuda.synchronize()
        p = st.packs[0, st.rank].clone().view(torch.int16)
        if ref is None:
            ref = p
        elif not torch.equal(p, ref):
            bad += 1
            d = (p.float() - ref.float()).abs()
            print(hw, "run", r, "differs:", int((d > 0).sum()), "elements, max", d.max().item())
    print(hw, "nondeterministic runs:", bad, "/ 19", flush=True)
