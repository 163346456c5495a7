// Grouped LDS-DMA conv launches (conv_dma_impl.h: conv_dma_group_kernel): several independent
// problems with one tile config in one grid. The small-map InceptionV3 convs of DeepDream's early
// octaves are latency bound (~10 us per dependent launch whatever their size, docs/KERNELS.md), so
// the independent branch convs of a block run as ONE launch (ops/inception.py plans the levels).
#include "conv_dma_impl.h"

namespace dv {

// Tile config of a problem in a grouped launch: the measured small-problem configs of auto_cfg
// (8: 64x64 / 4 waves / 3 stages, 3: 128x128 / 8 waves / 2 stages). 0: not groupable (large
// problems keep their own launch and tile choice; masked A, split-K, tuning overrides).
int conv_dma_group_cfg(const ConvArgs& a, int amode, int epi) {
  if (g_cfg > 0 || a.mask != nullptr || a.ws != nullptr || epi != CONV_E_BF16) return 0;
  if (amode != CONV_A_FWD && amode != CONV_A_TRANSPOSE) return 0;
  if (a.C % 8 != 0 || a.Kpad % 64 != 0 || a.x_ld % 8 != 0) return 0;
  const int c = auto_cfg(a);
  return (c == 8 || c == 3) ? c : 0;
}

namespace {

template <int DT, int AMODE, int WM, int WN, int FM, int FN, int ST>
int group_run(const ConvArgs* ps, int n, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  ConvGroup g{};
  g.n = n;
  long long tot = 0;
  bool aligned = true;
  for (int i = 0; i < n; ++i) {
    g.p[i] = ps[i];
    g.tiles_n[i] = ps[i].OCpad / BN;
    g.start[i] = (int)tot;
    tot += (long long)((ps[i].M + BM - 1) / BM) * g.tiles_n[i];
    aligned = aligned && (ps[i].C % 64) == 0;
  }
  for (int i = n; i <= kGroupMax; ++i) g.start[i] = (int)tot;
  if (tot <= 0 || tot > 0x7fffffffLL) return -2;
  if (aligned)
    hipLaunchKernelGGL((conv_dma_group_kernel<DT, WM, WN, FM, FN, 64, ST, AMODE, CONV_E_BF16, true>), dim3((unsigned)tot),
                       dim3(WM * WN * 64), 0, s, g);
  else
    hipLaunchKernelGGL((conv_dma_group_kernel<DT, WM, WN, FM, FN, 64, ST, AMODE, CONV_E_BF16, false>),
                       dim3((unsigned)tot), dim3(WM * WN * 64), 0, s, g);
  return (int)hipGetLastError();
}

template <int DT, int AMODE>
int group_cfg_run(const ConvArgs* ps, int n, int cfg, hipStream_t s) {
  if (cfg == 8) return group_run<DT, AMODE, 2, 2, 2, 2, 3>(ps, n, s);  // 64x64, 4 waves, 3 stages
  if (cfg == 3) return group_run<DT, AMODE, 4, 2, 2, 4, 2>(ps, n, s);  // 128x128, 8 waves, 2 stages
  return -5;
}

}  // namespace

int conv_dma_group_launch(const ConvArgs* ps, int n, int amode, int epi, hipStream_t s) {
  if (n < 1 || n > kGroupMax || epi != CONV_E_BF16) return -4;
  const int cfg = conv_dma_group_cfg(ps[0], amode, epi);
  if (cfg == 0) return -4;
  for (int i = 1; i < n; ++i)
    if (conv_dma_group_cfg(ps[i], amode, epi) != cfg || ps[i].dtype != ps[0].dtype) return -4;
  const bool f16 = ps[0].dtype == DT_F16;
  if (amode == CONV_A_FWD)
    return f16 ? group_cfg_run<DT_F16, CONV_A_FWD>(ps, n, cfg, s) : group_cfg_run<DT_BF16, CONV_A_FWD>(ps, n, cfg, s);
  return f16 ? group_cfg_run<DT_F16, CONV_A_TRANSPOSE>(ps, n, cfg, s)
             : group_cfg_run<DT_BF16, CONV_A_TRANSPOSE>(ps, n, cfg, s);
}

}  // namespace dv
