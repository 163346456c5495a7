// Instantiation unit of the LDS-DMA conv (conv_dma_impl.h): dma_bn<DT_F16, CONV_A_FWD, CONV_E_F32> (the fp16
// deconvnet's last conv-down, fp32 reconstruction + per-image deprocess statistics in the epilogue).
#include "conv_dma_impl.h"

namespace dv {

int dma_run_f16_fwd_f32(const ConvArgs& a, hipStream_t s) { return dma_bn<DT_F16, CONV_A_FWD, CONV_E_F32>(a, s); }

}  // namespace dv
