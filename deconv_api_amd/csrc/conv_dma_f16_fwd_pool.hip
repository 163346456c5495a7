// Instantiation unit of the LDS-DMA conv (conv_dma_impl.h): dma_bn<DT_F16, CONV_A_FWD, CONV_E_POOL> (the fp16
// VGG16 deconvnet forward, Config.dtype = fp16: conv + ReLU + 2x2 max-pool / switch epilogue).
#include "conv_dma_impl.h"

namespace dv {

int dma_run_f16_fwd_pool(const ConvArgs& a, hipStream_t s) { return dma_bn<DT_F16, CONV_A_FWD, CONV_E_POOL>(a, s); }

}  // namespace dv
