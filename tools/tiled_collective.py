"""Rehearse the multi-rank tiled DeepDream octave on a 1-rank RCCL group (torchrun):

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \\
        --master-port 29533 tools/tiled_collective.py

Runs one octave with the collective path forced on (DV_TILE_COLLECTIVE semantics: the per-step
all-gather of the packs over the process group) and captured inside the octave's hipGraph, and the
same octave without collectives; prints one JSON line: backend, whether the collective path ran,
whether the octave was ONE graph (collectives captured) or per-step graphs, and bit equality. Then the
chunked overlapped step (DV_TILE_CHUNKS semantics: each chunk's async all-gather captured beside the
next chunk's network; with DV_TILE_CHUNK_STREAMS=2 (default) the chunks run on two streams and each
all-gather is issued from its chunk's stream): equal to the collective-free octave up to the conv
rounding of smaller batches."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import deconv_api_amd.engine.deepdream as D  # noqa: E402
from deconv_api_amd import ops  # noqa: E402
from deconv_api_amd.models.resnet50 import ResNet50  # noqa: E402
from deconv_api_amd.parallel import dist as pdist  # noqa: E402


def main():
    info = pdist.init()
    ops.native.load()
    net = ResNet50(0).build(info.device, torch.float16)
    s = D.DreamSettings(layers=dict(D.RESNET_LAYERS), octaves=1, iterations=4, max_loss=None)
    x = (torch.rand(2, 256, 320, 3, generator=torch.Generator().manual_seed(3)) * 2 - 1).to(info.device)
    D.TILE_COLLECTIVE = False
    D.TILE_LOCAL_CHUNKS = 1  # the unchunked 1-rank octave is the reference
    ref = D.TiledDeepDream(net, s, tile=128, info=info, seed=5).gradient_ascent(x)
    D.TILE_COLLECTIVE = True
    D.TILE_CHUNKS = 1
    dd = D.TiledDeepDream(net, s, tile=128, info=info, seed=5)
    got = dd.gradient_ascent(x)
    got2 = D.TiledDeepDream(net, s, tile=128, info=info, seed=5).gradient_ascent(x)  # fresh capture, replay
    torch.cuda.synchronize()
    st = next(iter(dd._tgraphs.values()))
    out = {"backend": info.backend, "world": info.world, "collective": dd._collective(st),
           "octave_graph": st.graph is not None, "step_graphs": st.step_graph is not None,
           "equal": bool(torch.equal(got, ref)) and bool(torch.equal(got2, ref))}
    D.TILE_CHUNKS = 2
    dc = D.TiledDeepDream(net, s, tile=128, info=info, seed=5)
    gc = dc.gradient_ascent(x)
    gc2 = dc.gradient_ascent(x)  # replay of the captured chunked octave (fresh rolls)
    torch.cuda.synchronize()
    stc = next(iter(dc._tgraphs.values()))
    a, b = (gc - x).flatten().double(), (ref - x).flatten().double()
    out.update({"chunks": stc.C, "chunk_streams": min(D.TILE_CHUNK_STREAMS, stc.C), "chunked_octave_graph": stc.graph is not None,
                "chunked_cos": float(a @ b / (a.norm() * b.norm() + 1e-30)),
                "chunked_maxdiff": float((gc - ref).abs().max()), "chunked_rerun_finite": bool(torch.isfinite(gc2).all())})
    if info.is_main:
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
