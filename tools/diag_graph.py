"""Diagnose graphed-vs-eager mosaic differences (tests/test_engine_gpu.py::test_graphed_engine_equals_eager)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd.engine.deconvnet import DeconvNet  # noqa: E402
from deconv_api_amd.engine.graphs import GraphedDeconv  # noqa: E402
from deconv_api_amd.models.vgg16 import VGG16  # noqa: E402
from tests.test_engine_gpu import _x8  # noqa: E402

m = VGG16.random(0, include_top=False)
eng = DeconvNet(m.build("cuda", torch.bfloat16))
gd = GraphedDeconv(eng)
for seed in (4, 5, 6):
    x = _x8(3, 224, seed).to(torch.bfloat16).cuda()
    e1 = eng.run(x, "block4_pool", k=4)
    e1m, e1f = e1.mosaic.clone(), e1.filters.clone()
    e2 = eng.run(x, "block4_pool", k=4)
    g = gd.run(x, "block4_pool")
    gm, gf = g.mosaic[:3].clone(), g.filters[:3].clone()
    x4 = torch.cat([x, torch.zeros_like(x[:1])])
    e4 = eng.run(x4, "block4_pool", k=4)
    print("seed", seed, "eager-eager", (e1m.int() - e2.mosaic.int()).abs().max().item(),
          "graph-eager", (gm.int() - e1m.int()).abs().amax(dim=(1, 2, 3)).tolist(),
          "eager4-eager3", (e4.mosaic[:3].int() - e1m.int()).abs().amax(dim=(1, 2, 3)).tolist(),
          "graph-eager4", (gm.int() - e4.mosaic[:3].int()).abs().max().item(), flush=True)
    print("  filters eager", e1f.tolist(), "graph", gf.tolist(), "eager4", e4.filters[:3].tolist(), flush=True)
