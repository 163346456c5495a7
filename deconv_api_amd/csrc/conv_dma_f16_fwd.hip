// Instantiation unit of the LDS-DMA conv (conv_dma_impl.h): dma_bn<DT_F16, CONV_A_FWD, CONV_E_BF16>.
#include "conv_dma_impl.h"

namespace dv {

int dma_run_f16_fwd(const ConvArgs& a, hipStream_t s) { return dma_bn<DT_F16, CONV_A_FWD, CONV_E_BF16>(a, s); }

}  // namespace dv
