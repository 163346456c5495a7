"""Op surface of deconv_api_amd. Device tensors -> gfx950 HIP kernels; CPU tensors -> PyTorch
reference implementations of the same math (used for CPU execution and as test oracles)."""
from .conv import (ConvWeights, conv2d, deconv_tail, deconv_tail_ref, deconv_weights, maxpool_switch_ref, oc_pad,
                   pad_channels_oihw, stem_pool, unpool_ref)
from .misc import (CAFFE_MEAN, channel_sum, softmax_rows, deprocess_mosaic, maxpool2x2, preprocess_ref, resize_mode,
                   resize_preprocess, resize_u8_ref, seed_deconv3x3, seed_map, topk_positive, unpool2x2)
from . import native

__all__ = [
    "ConvWeights", "conv2d", "deconv_tail", "deconv_tail_ref", "deconv_weights", "maxpool_switch_ref", "oc_pad", "pad_channels_oihw", "stem_pool",
    "unpool_ref", "CAFFE_MEAN", "channel_sum", "deprocess_mosaic", "maxpool2x2", "preprocess_ref",
    "resize_mode", "resize_preprocess", "resize_u8_ref", "seed_deconv3x3", "seed_map", "topk_positive", "unpool2x2",
    "softmax_rows",
    "native",
]
