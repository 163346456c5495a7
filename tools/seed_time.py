#!/usr/bin/env python
"""Time seed_deconv3x3 (block5_conv3.down's first step) at the config-2 shape: 1024 signals x 14^2 x 512."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deconv_api_amd import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
S = torch.relu(torch.randn(1024, 14, 14, device="cuda", generator=g))
f = torch.randint(-1, 512, (1024,), device="cuda", generator=g, dtype=torch.int32)
wt = (torch.randn(512, 3, 3, 512, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
for _ in range(3):
    ops.seed_deconv3x3(S, f, wt)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
e0.record()
for _ in range(50):
    ops.seed_deconv3x3(S, f, wt)
e1.record()
torch.cuda.synchronize()
print(json.dumps({"seed_deconv3x3_us": round(e0.elapsed_time(e1) / 50 * 1000, 1)}))
