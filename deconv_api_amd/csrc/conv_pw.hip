// Persistent pointwise conv for gfx950: 1x1 / stride 1 / pad 0 convs (ResNet bottleneck convs and
// their input gradients, Inception 1x1 heads) at large M, where the LDS-DMA implicit GEMM is
// HBM-latency bound rather than MFMA bound.
//
// Why: with a short K (64..256 = 1..4 K tiles) every workgroup of the one-tile-per-workgroup kernel
// (conv_dma_impl.h) runs a serial chain (prologue -> DMA of its only tiles -> MFMA -> LDS-staged
// epilogue -> stores) with nothing overlapping its memory latency but the one other workgroup on the
// CU. PMC on config 5 (profiles/pmc_c5_r2.txt): the 128x128 tile kernel moved 2.15 TB/s.
//
// Design: a grid of (CUs x 2) workgroups, each walking the tiles first, first + G, first + 2G, ...
// The (tile, K tile) steps of a workgroup form ONE sequence through a 2-stage LDS ring, so the DMA
// of the next step (usually the next tile's A rows and weights) is in flight during this step's
// MFMAs and epilogue. The epilogue is the shared LDS-staged 16-bit one (epilogue_lds: bias, ReLU /
// relu_cols, accumulate, residual, emask; 16-B global accesses), staged in the ring slot of the step
// that just finished (the C tile fits in one operand stage). The A operand is the plain [M, C] matrix
// with row stride x_ld (a 1x1 / stride-1 conv reads pixel m for GEMM row m), so the gather needs no
// tap arithmetic; the buffer range check zero-fills the M tail.
#include "conv_dma_impl.h"

namespace dv {

template <int DT, int WM, int WN, int FM, int FN>
__global__ void __launch_bounds__(WM * WN * 64, 4) conv_pw_kernel(const ConvArgs a, int tiles_n, int tiles_total) {
  constexpr int BK = 64, NW = WM * WN, NT = NW * 64;
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int ROWB = BK * 2, CPR = BK / 8, RPI = 1024 / ROWB;
  constexpr int A_BYTES = BM * ROWB, B_BYTES = BN * ROWB, STAGE = A_BYTES + B_BYTES;
  constexpr int A_I = BM / RPI / NW;
  constexpr int B_GROUPS = BN / RPI, B_FULL = B_GROUPS / NW, B_REM = B_GROUPS % NW;
  static_assert(A_I >= 1 && BM % (RPI * NW) == 0, "BM must cover every wave");
  static_assert(BM * BN * 2 <= STAGE, "the C tile is staged in one operand stage");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int G = gridDim.x;
  const int first = xcd_remap(blockIdx.x, G);  // neighbouring tiles (shared A rows) on one XCD
  const int ntiles = (tiles_total - first + G - 1) / G;  // >= 1: the host sizes G <= tiles_total
  const int nk = a.Kpad / BK;
  const int S = ntiles * nk;

  const __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, (uint64_t)((long long)(a.M - 1) * a.x_ld + a.C) * 2);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (uint64_t)a.OCpad * a.Kpad * 2);
  const int lrow = lane / CPR;
  const int lchunk = (lane % CPR) ^ row_xor<BK>(lrow);

  auto issue = [&](int s, int buf) {
    const int j = s / nk, kt = s - j * nk;
    const int t = first + j * G;
    const int m0 = (t / tiles_n) * BM, n0 = (t - (t / tiles_n) * tiles_n) * BN;
    uint8_t* As = smem + buf * STAGE;
    uint8_t* Bs = As + A_BYTES;
    const int ch = kt * BK + lchunk * 8;
#pragma unroll
    for (int i = 0; i < A_I; ++i) {
      const int gm = m0 + (i * NW + wave) * RPI + lrow;
      const bool ok = gm < a.M && DV_BOUNDS((long long)gm * a.x_ld + ch, 8, a.x_elems, "conv_pw A");
      dma16(xr, As + (i * NW + wave) * 1024, ok ? ((uint32_t)gm * (uint32_t)a.x_ld + (uint32_t)ch) * 2u : kOOB);
    }
#pragma unroll
    for (int i = 0; i < B_FULL + (B_REM ? 1 : 0); ++i) {
      const int grp = i * NW + wave;
      if (grp < B_GROUPS) {
        const int row = grp * RPI + lrow;
        dma16(wr, Bs + grp * 1024, ((uint32_t)(n0 + row) * (uint32_t)a.Kpad + (uint32_t)(kt * BK + lchunk * 8)) * 2u);
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int a_row0 = wm * FM * 16 + (lane & 15);
  const int b_row0 = wn * FN * 16 + (lane & 15);
  const int rx = row_xor<BK>(lane & 15);
  int sw[BK / 32];
#pragma unroll
  for (int q = 0; q < BK / 32; ++q) sw[q] = (((q * 4 + (lane >> 4)) ^ rx) << 4);

  issue(0, 0);
  for (int s = 0; s < S; ++s) {
    const int cur = s & 1;
    // drain: step s's DMA (issued during step s-1) and step s-1's epilogue stores; the raw barrier
    // then also orders every wave's epilogue reads of the slot the next DMA overwrites
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (s + 1 < S) issue(s + 1, cur ^ 1);
    const uint8_t* As = smem + cur * STAGE;
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int q = 0; q < BK / 32; ++q) {
      typedef typename Vec8<DT>::type v8;
      v8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = *reinterpret_cast<const v8*>(Bs + (b_row0 + j * 16) * ROWB + sw[q]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const v8 af = *reinterpret_cast<const v8*>(As + (a_row0 + i * 16) * ROWB + sw[q]);
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af, bfr[j], acc[i][j]);
      }
    }
    const int j = s / nk;
    if (s - j * nk == nk - 1) {  // last K tile of this workgroup's j-th tile: epilogue
      const int t = first + j * G;
      const int m0 = (t / tiles_n) * BM, n0 = (t - (t / tiles_n) * tiles_n) * BN;
      __syncthreads();  // every wave is done reading slot `cur`: it becomes the C staging buffer
      // ucode known null (the launcher rejects it): the epilogue's max-unpool branch folds away
      ConvArgs an = a;
      an.ucode = nullptr;
      epilogue_lds<DT, NT, BM, BN, FM, FN>(an, acc, smem + cur * STAGE, m0, n0, wm, wn, lane, tid, true);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int jj = 0; jj < FN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  }
  wait_vm<0>();
}

// < 0: not a persistent-pointwise problem (the caller falls back to the LDS-DMA kernel)
int conv_pw_launch(const ConvArgs& a, hipStream_t s) {
  static const bool off = dv_ab_env("DV_NO_PW") != nullptr;
  static const long long min_tiles = dv_ab_env("DV_PW_MIN_TILES") ? std::atoll(dv_ab_env("DV_PW_MIN_TILES")) : 0;
  if (off || g_cfg > 0) return -4;
  if (a.KH != 1 || a.KW != 1 || a.stride != 1 || a.pad_h != 0 || a.pad_w != 0 || a.H != a.OH || a.W != a.OW ||
      a.C % 64 != 0 || a.Kpad != a.C || a.K != a.C || a.mask || a.code || a.ucode || a.ws || a.stats ||
      a.relu_in || !a.vec_epi || a.x_ld % 8 != 0 || (long long)a.M * a.x_ld * 2 > 0x7FFFFFF0LL)
    return -4;
  const long long cus = num_cus();
  int BM, BN;
  if (a.OCpad % 128 == 0 && a.OC > 64) {
    BM = 128;
    BN = 128;
  } else if (a.OCpad % 64 == 0 && a.OC > 16) {
    BM = 256;
    BN = 64;
  } else {
    return -4;
  }
  const int tiles_n = a.OCpad / BN;
  const long long tiles_total = (long long)((a.M + BM - 1) / BM) * tiles_n;
  // persistence pays once every CU has a tile: round 4 (kernel without spills) moved the default from 4 to 1 tile
  // per CU (config 5 +0.7 %, config 3 unchanged, profiles/dream_r4_pw_min_tiles.txt)
  if (tiles_total < (min_tiles > 0 ? min_tiles : cus) || tiles_total > 0x7fffffffLL) return -4;
  // DV_PW_WG_PER_CU: persistent workgroups per CU (2 by default: each holds 64 KiB of LDS ring)
  static const long long wpc = dv_ab_env("DV_PW_WG_PER_CU") ? std::max(1LL, std::atoll(dv_ab_env("DV_PW_WG_PER_CU"))) : 2;
  const unsigned G = (unsigned)std::min<long long>(tiles_total, wpc * cus);
  if (BN == 128) {
    if (a.dtype == DT_F16)
      hipLaunchKernelGGL((conv_pw_kernel<DT_F16, 4, 2, 2, 4>), dim3(G), dim3(512), 0, s, a, tiles_n, (int)tiles_total);
    else
      hipLaunchKernelGGL((conv_pw_kernel<DT_BF16, 4, 2, 2, 4>), dim3(G), dim3(512), 0, s, a, tiles_n, (int)tiles_total);
  } else {
    if (a.dtype == DT_F16)
      hipLaunchKernelGGL((conv_pw_kernel<DT_F16, 8, 1, 2, 4>), dim3(G), dim3(512), 0, s, a, tiles_n, (int)tiles_total);
    else
      hipLaunchKernelGGL((conv_pw_kernel<DT_BF16, 8, 1, 2, 4>), dim3(G), dim3(512), 0, s, a, tiles_n, (int)tiles_total);
  }
  return (int)hipGetLastError();
}

}  // namespace dv
