// Instantiation unit of the LDS-DMA conv (conv_dma_impl.h): dma_bn<DT_BF16, CONV_A_FWD, CONV_E_F32>.
#include "conv_dma_impl.h"

namespace dv {

int dma_run_bf16_fwd_f32(const ConvArgs& a, hipStream_t s) { return dma_bn<DT_BF16, CONV_A_FWD, CONV_E_F32>(a, s); }

}  // namespace dv
