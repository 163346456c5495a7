"""Every ``DV_*`` environment variable the package reads, registered with a one-line justification.

Four kinds (tests/test_knobs.py scans the sources and fails on an unregistered name):

* CONFIG - the serving configuration, ``Config`` fields read by ``Config.from_env`` (config.py);
* RUNTIME - production switches outside ``Config``: kill switches of fused kernels, the multi-rank
  DeepDream tiling, fault injection, tracing, caps. At most 30;
* ABLATION - A/B switches of measured alternatives (the measurement is cited). They are honoured
  only when ``DV_ABLATIONS=1`` (``ablation()`` here, ``dv_ab_env`` in csrc/kernels.h), so a serving
  or benchmark process runs one dispatch per shape whatever its environment holds; tools/*_ab.py and
  the GPU tests that compare variants set it;
* BUILD - compile-time macros and build / loader tooling.
"""
from __future__ import annotations

import os
from typing import Optional

RUNTIME = {
    "DV_NO_KW3_SK": "stream-K off for KW3P convs (the recovery named by the hand-off timeout error, ops/conv.py)",
    "DV_POOL_SPLIT": "layers whose pool runs as a separate vectorized kernel (config 2 option, docs/KERNELS.md)",
    "DV_STEM_FUSE": "kill switch of the fused VGG16 stem (conv -> conv -> pool in one launch)",
    "DV_FUSED_TAIL": "kill switch of the fused deconvnet tail (unpool -> conv -> per-tap products)",
    "DV_CONV_IMPL": "conv kernel policy for tests / bring-up (auto | dma | igemm | halo)",
    "DV_CONV_GROUP": "grouped launch of independent small convs (DeepDream), 0 = per-conv launches",
    "DV_TILE_COLLECTIVE": "run the multi-rank tiled-DeepDream code path on a 1-rank RCCL group (rehearsal)",
    "DV_TILE_CHUNKS": "tile units per rank split into this many chunks whose all-gathers overlap compute",
    "DV_TILE_CHUNK_STREAMS": "streams the chunks of a tiled step fork onto",
    "DV_TILE_LOCAL_CHUNKS": "chunks per rank when the dream is not collective (one GPU)",
    "DV_TILE_CAPTURE_COLL": "capture the tiled octave's all-gathers inside its hipGraph (0: per-step graphs)",
    "DV_DREAM_GRAPHS": "hipGraph replay of DeepDream steps (0: eager, debugging)",
    "DV_DREAM_OCTAVE_GRAPH": "one hipGraph per octave incl. all steps (0: one graph per step)",
    "DV_FAULT": "fault injection for the failover tests (utils/faults.py)",
    "DV_ROCTX": "roctx ranges around engine stages (utils/tracing.py)",
    "DV_MAX_PIXELS": "decoded-pixel cap of a request image (codec/image.py)",
    "DV_FORCE_PG": "create a real process group at world 1 (exercises RCCL collectives on one GPU)",
    "DV_INGEST_DIR": "directory of the front-end <-> GPU-owner Unix sockets (serve/ingest.py)",
    "DV_ABLATIONS": "honour the ABLATION switches below (tools / variant tests only)",
}

ABLATION = {
    # conv_dma_impl.h: KW3P (shared-kw-tap implicit GEMM) variants and tile choices
    "DV_KW3": "KW3 kernel off / forced (tests: small shapes with many borders)",
    "DV_KW3_VAR": "KW3 main-loop variant (profiles/kw3_variants_r3.txt, kw3_staging_ablation_r5.txt)",
    "DV_KW3_TILE": "KW3P tile shape (profiles/kw3_ab_r4.txt)",
    "DV_KW3_SK": "stream-K on every eligible grid, not only short ones (profiles/kw3_skall_ab_r5.txt)",
    "DV_KW3P_EPI": "register-layout 8-B epilogue instead of the LDS-staged 16-B one (profiles/kw3_epi_ab_r5.txt)",
    "DV_KW3P_NO_PRE": "no step-1 DMA ahead of the epilogue (profiles/kw3_pre_ab_r5.txt)",
    "DV_KW3P_UNP_NT": "plain instead of non-temporal unpool stores (profiles/bench_c2_r5_unp_nt_ab.txt)",
    "DV_NO_KW3P_UNPOOL": "unpool-out conv-downs off KW3P (profiles/kw3_store_ablation_r5.txt)",
    "DV_ALLOW_WRONG_ABLATION": "timing-only variants whose outputs are wrong (tools/kw3_ab.py, tools/tail_ab.py)",
    "DV_NO_AUTO_CFG": "size-based DMA tile choice only (docs/KERNELS.md)",
    "DV_SMALL_TILE_KMIN": "K threshold of the 64x64 small-problem tile",
    "DV_NO_SPLITK": "split-K off (tools/small_conv_latency.py)",
    "DV_NO_SMALL_SPLITK": "small-problem split-K off",
    "DV_SMALL_SPLITK_MN": "M x N ceiling of the small-problem split-K",
    # bindings.cpp routing
    "DV_NO_POOL_T": "per-element pool-epilogue stores (profiles/bench_c2_r4_pool_t_ab.txt)",
    "DV_POOL_EPI": "pool epilogue variant (profiles/bench_c2_r5_pool_epi_ab.txt)",
    "DV_NO_VEC_EPI": "scalar conv epilogue",
    "DV_NO_EPI_BATCH": "per-row epilogue batching off (profiles/dream_c3_r2_epi_batch*.log)",
    "DV_NO_C8_STREAM": "first-layer row-streaming kernel off",
    "DV_HS_MIN_W": "smallest map side routed to the halo-stream kernels",
    "DV_HS_EMASK_OFF": "masked dgrads back on the DMA kernel",
    "DV_HS_PAD_OFF": "pad != 1 convs off the halo-stream kernels",
    # conv_halo_stream.hip
    "DV_NO_HS": "halo-stream kernels off",
    "DV_NO_HS16": "16x16-tile halo-stream kernel off",
    "DV_NO_HS_SPLIT": "192/256-channel convs not split into halo-stream halves",
    "DV_HS_RING": "halo-stream ring depth",
    "DV_HS16_EPI": "register-layout epilogue of hs16 (profiles/bench_c2_r5_hs16_epi_ab.txt)",
    # conv_smalln.hip / misc / pool / pw
    "DV_TAIL_V": "fused-tail schedule bits (profiles/bench_c2_r5_tail_v_ab.txt)",
    "DV_STREAM_P": "row-streaming kernel prefetch depth",
    "DV_NO_POOL_UNROLL": "generic k x k pooling loop (profiles/dream_r4_maxpool_bwd_s2_ab.txt)",
    "DV_NO_PW": "persistent 1x1 kernel off (tools/pw_bench.py)",
    "DV_PW_MIN_TILES": "tiles below which 1x1 convs stay on the DMA kernel (profiles/dream_r4_pw_min_tiles.txt)",
    "DV_PW_WG_PER_CU": "persistent 1x1 workgroups per CU",
    # Python engine / DeepDream alternatives
    "DV_NO_STREAM_PROBE": "plain pool streams instead of probed / high-priority ones (runtime/streams.py)",
    "DV_DREAM_OCTAVE_RESIZE": "torch octave resize instead of the HIP kernel (profiles/dream_c3_r4_octave_resize_ab.txt)",
    "DV_DREAM_FUSED": "fused step tail off",
    "DV_DREAM_FUSED_LOSS": "fused loss off",
    "DV_DREAM_TAPS": "tap-split stride-2 dgrads (profiles/dream_c5_r2_taps.log)",
    "DV_DREAM_SPLIT": "concurrent sub-batches per DeepDream batch (profiles/dream_c3_split_sweep_r2.txt)",
    "DV_RELU_BITS": "1-bit ReLU masks off (profiles/dream_c5_r5_relu_bits_ab.txt)",
    "DV_SUBPIXEL": "sub-pixel scatter for stride-2 1x1 dgrads (profiles/kstats_c5_r2_subpixel.txt)",
    "DV_STEM_FUSED": "InceptionV3 stem fusion (profiles/dream_c3_r2_stem*.log)",
    "DV_STEM_DIRECT": "direct stride-2 stem gradient (profiles/dream_c5_r3_stem_ab.txt)",
    "DV_STEM7": "ResNet conv1 tap-paired kernel (profiles/dream_c5_r5_stem7_ab.txt)",
    "DV_COL2IM": "LDS-tiled col2im of the RGB stem gradient",
    "DV_STRIDED_DIRECT_GFLOP": "size threshold of the direct strided dgrad",
    "DV_MERGE_B1": "merged Inception branch-head GEMMs (profiles/dream_c3_r2_merge_b1.txt)",
    "DV_INCEPTION_FUSED": "one-node Inception blocks (profiles/dream_c3_merged.log)",
}

BUILD = {
    "DV_HIP_CHECK": "launch-status check macro (csrc/common.h), not an environment variable",
    "DV_DEBUG": "-DDV_DEBUG=1 build: device bounds checks (python -m deconv_api_amd._build --debug)",
    "DV_BOUNDS": "the bounds-check macro of DV_DEBUG builds (csrc/common.h)",
    "DV_SOURCE_HASH": "sha256 of csrc + flags embedded in _C (_build.py provenance)",
    "DV_OFFLOAD_ARCH": "offload arch of the in-tree build (gfx950)",
    "DV_AUTOBUILD": "ops/native.py: build (or rebuild a stale) _C in-tree on first use",
    "DV_SKIP_PROVENANCE": "ops/native.py: load a _C built from other sources (scratch builds in tools)",
    "DV_S": "kernel-local macro (conv_smalln.hip), not an environment variable",
    "DV_S2": "kernel-local macro (conv_smalln.hip), not an environment variable",
    "DV_P": "kernel-local macro (conv_smalln.hip), not an environment variable",
}


def config_names():
    import dataclasses

    from .config import Config

    return {"DV_" + f.name.upper() for f in dataclasses.fields(Config)}


def ablations_on() -> bool:
    return os.environ.get("DV_ABLATIONS", "") == "1"


def ablation(name: str, default: Optional[str] = None) -> Optional[str]:
    """The value of ABLATION switch ``name`` when ablations are on, else ``default`` (unset)."""
    assert name in ABLATION, f"{name} is not a registered ablation switch (knobs.py)"
    return os.environ.get(name, default) if ablations_on() else default
