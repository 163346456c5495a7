// LDS-DMA implicit-GEMM conv: dispatch over (dtype, A mode, epilogue), split-K planning and
// reduction, ReLU-masked dgrads and the tuning override. The kernel and its tile configs live in
// conv_dma_impl.h (design notes there); the heavy dma_bn instantiations are in conv_dma_*.hip.
#include "conv_dma_impl.h"

namespace dv {

// Tuning override (tools/tune_dma.py): force tile config `g_cfg` (> 0) and split-K factor
// `g_ks` (> 0) for every DMA conv launch until reset to 0. Host-side globals, set between launches.
int g_cfg = 0, g_ks = 0;
void conv_dma_tune(int cfg, int ks) {
  g_cfg = cfg;
  g_ks = ks;
}

// Split-K factor for a launch that would leave most CUs idle: small M (batch-1 serving, deep
// layers of strong-scaled DeepDream tiles, dense layers) with a long K. 1 = no split.
// The small-problem 64x64 tiles (auto_cfg 8: DeepDream's small octaves, replayed from hipGraphs)
// split a long K into 2 / 4 parts: in a graph the extra reduce launch costs ~2 us while each K
// tile of the serial K loop costs ~0.4 us (tools/small_conv_latency.py: M 1600 x N 160 x K 1440
// 14.8 -> 11.4 us, M 4096 x N 96 x K 2592 23.3 -> 15.2 us; K <= 768 gains nothing).
int conv_dma_splitk(const ConvArgs& a) {
  if (g_ks > 0) return std::min(g_ks, a.Kpad / 64);
  static const bool off = dv_ab_env("DV_NO_SPLITK") != nullptr;
  static const bool small_off = dv_ab_env("DV_NO_SMALL_SPLITK") != nullptr;
  if (off) return 1;
  const int nk = a.Kpad / 64;
  if (g_cfg == 0 && auto_cfg(a) == 8) {
    // only the smallest problems: the reduce pass re-reads ks x M x OCpad fp32 partials, which
    // outweighs the shorter K loop once M x OCpad grows (full-model A/B, docs/KERNELS.md)
    static const long long mn_max =
        dv_ab_env("DV_SMALL_SPLITK_MN") ? std::atoll(dv_ab_env("DV_SMALL_SPLITK_MN")) : 300000LL;
    if (small_off || (long long)a.M * a.OCpad > mn_max) return 1;
    return nk >= 20 ? 4 : (nk >= 16 ? 2 : 1);
  }
  int BM, BN;
  dma_tile_dims(a, a.mask != nullptr, BM, BN);
  const long long nwg = (long long)((a.M + BM - 1) / BM) * (a.OCpad / BN);
  const long long cus = num_cus();
  if (nwg * 2 > cus || nk < 8) return 1;
  long long k = (cus + nwg - 1) / nwg;  // about one workgroup per CU
  k = std::min<long long>(k, nk / 4);   // >= 4 K tiles per split keeps the pipeline primed
  k = std::min<long long>(k, 32);
  return k < 2 ? 1 : (int)k;
}

// The split-K epilogue: out = act(sum_s ws[s] + bias) with the kernel epilogue's full semantics
// (16-bit or fp32 output of row stride out_ld): v = sum + bias, [ReLU] (before an accumulate /
// residual add), += out (accumulate), += res then [ReLU], zeroed where emask <= 0.
template <int DT>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const ConvArgs a, int epi) {
  const long long total = (long long)a.M * a.OC;
  const long long plane = (long long)a.M * a.OCpad;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int row = (int)(t / a.OC), col = (int)(t % a.OC);
    const float* w = a.ws + (long long)row * a.OCpad + col;
    float v = a.bias ? a.bias[col] : 0.f;
    for (int k = 0; k < a.ksplit; ++k) v += w[k * plane];
    if (relu_at(a, col) && !a.res) v = fmaxf(v, 0.f);
    const long long o = (long long)row * a.out_ld + col;
    if (!DV_BOUNDS(o, 1, a.out_elems, "splitk_reduce out")) continue;
    if (epi == CONV_E_F32) {
      float* out = reinterpret_cast<float*>(a.out);
      if (a.accumulate) v += out[o];
      out[o] = v;
      continue;
    }
    uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
    if (a.accumulate) v += to_f<DT>(out[o]);
    if (a.res) {
      v += to_f<DT>(a.res[(long long)row * a.res_ld + col]);
      if (relu_at(a, col)) v = fmaxf(v, 0.f);
    }
    if (a.emask) {
      const uint32_t m = a.emask[(long long)row * a.emask_ld + col];
      if (m == 0u || (m & 0x8000u)) v = 0.f;
    }
    out[o] = from_f<DT>(v);
  }
}

int splitk_reduce_launch(const ConvArgs& a, int epi, hipStream_t s) {
  const long long total = (long long)a.M * a.OC;
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 256LL * 16);
  if (a.dtype == DT_F16)
    hipLaunchKernelGGL(splitk_reduce_kernel<DT_F16>, dim3(grid), dim3(256), 0, s, a, epi);
  else
    hipLaunchKernelGGL(splitk_reduce_kernel<DT_BF16>, dim3(grid), dim3(256), 0, s, a, epi);
  return (int)hipGetLastError();
}

int conv_dma_launch(const ConvArgs& a, int amode, int epi, hipStream_t s) {
  if (a.C % 8 != 0 || a.Kpad % 64 != 0 || a.x_ld % 8 != 0) return -4;
  if (a.mask != nullptr) {
    if (a.mask_ld != a.x_ld || epi != CONV_E_BF16) return -4;
    if (amode == CONV_A_FWD)
      return a.dtype == DT_F16 ? dma_mask_bn<DT_F16, CONV_A_FWD>(a, s) : dma_mask_bn<DT_BF16, CONV_A_FWD>(a, s);
    if (amode == CONV_A_TRANSPOSE)
      return a.dtype == DT_F16 ? dma_mask_bn<DT_F16, CONV_A_TRANSPOSE>(a, s)
                               : dma_mask_bn<DT_BF16, CONV_A_TRANSPOSE>(a, s);
    return -1;
  }
  if (a.dtype == DT_F16) {  // DeepDream fp16 (BASELINE config 5) + the fp16 deconvnet (Config.dtype)
    if (amode == CONV_A_FWD && epi == CONV_E_BF16) return dma_run_f16_fwd(a, s);
    if (amode == CONV_A_FWD && epi == CONV_E_POOL) return dma_run_f16_fwd_pool(a, s);
    if (amode == CONV_A_FWD && epi == CONV_E_F32) return dma_run_f16_fwd_f32(a, s);
    if (amode == CONV_A_TRANSPOSE && epi == CONV_E_BF16) return dma_run_f16_tr(a, s);
    return -1;
  }
  if (amode == CONV_A_FWD) {
    if (epi == CONV_E_BF16) return dma_run_bf16_fwd(a, s);
    if (epi == CONV_E_POOL) return dma_run_bf16_fwd_pool(a, s);
    if (epi == CONV_E_F32) return dma_run_bf16_fwd_f32(a, s);
  } else if (amode == CONV_A_TRANSPOSE) {
    if (epi == CONV_E_BF16) return dma_run_bf16_tr(a, s);
  }
  return -1;
}

}  // namespace dv
