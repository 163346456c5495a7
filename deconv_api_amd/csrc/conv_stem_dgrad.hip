// Fused input gradient of a strided few-channel stem conv (ResNet-50 conv1: 3 -> 64, 7x7 / 2,
// pad 3), the image gradient DeepDream ascends. Replaces GEMM (cols = dy @ W^T, written to HBM)
// + col2im (cols read back): at 1024^2 tiles the cols round trip was 1.3 GB per step and the two
// kernels 11.5 % of config 5 (profiles/kstats_c5_r2_final.txt: col2im_lds 324 us + the 1x1 GEMM
// 161 us per call).
//
// One 256-thread workgroup owns a TH x TW tile of dx. It
//   1. stages the window of dy rows every dx pixel of the tile reads (RN x CN pixels x C channels,
//      out-of-map pixels zero, an optional ReLU mask applied) and the weight matrix B = W^T
//      [J][C] (J = KH*KW*Cr taps x channels, rows padded to a multiple of 16) in LDS, XOR-swizzled
//      16-B chunks (chunk ^ row & 7: conflict-free ds_read_b128 fragment reads);
//   2. P = dy_window @ B^T on MFMA (16x16x32, K = C = 64 in two 32-deep steps: the accumulation
//      order of the 1x1-conv GEMM it replaces), rounded to 16 bits like the cols it replaces, and
//      written TRANSPOSED to LDS (P^T[j][r], row stride padded so the 16 lanes of a fragment row
//      write 16 distinct bank pairs), over the staging area;
//   3. every dx pixel sums its <= ceil(KH/s) x ceil(KW/s) taps from LDS in fp32 (the col2im's tap
//      order: bitwise the same result) and writes its 8-channel padded pixel with one 16-B store.
// The window is recomputed for overlapping tiles (~1.6x the GEMM, which is tiny at K = 64).
#include "common.h"
#include "kernels.h"

namespace dv {

namespace {

constexpr int SD_TH = 16, SD_TW = 32;          // dx tile
constexpr int SD_C = 64;                       // dy channels (conv1 output)
constexpr int SD_MROWS = 256;                  // MFMA rows (window pixels, RN * CN <= 240 used)
constexpr int SD_PROW = 244;                   // P^T row stride in 16-bit elements (488 B: bank spread)

__device__ __forceinline__ int floor_div(int a, int b) { return (a >= 0) ? a / b : -((-a + b - 1) / b); }

template <int DT, int KH, int KW, int S, int KH0, int KW0, int RN, int CN>
__device__ __forceinline__ void col2im_taps(const uint16_t* __restrict__ P, uint16_t* __restrict__ gx,
                                            const StemDgradGeom& g, int n, int ih0, int iw0, int oh_lo, int ow_lo,
                                            int py, int px, int lane) {
  constexpr int NH = (KH - KH0 + S - 1) / S, NW = (KW - KW0 + S - 1) / S;  // taps of this parity class
  constexpr int cw_ = SD_TW / S;                                          // class columns per tile row
#pragma unroll
  for (int q = lane; q < SD_TH * SD_TW / 4; q += 64) {
    const int p = ((q / cw_) * S + py) * SD_TW + (q % cw_) * S + px;
    const int ih = ih0 + p / SD_TW, iw = iw0 + p % SD_TW;
    // window row / column of tap (KH0, KW0); tap (KH0 + S a, KW0 + S b) sits a rows / b columns before it
    const int r0 = (ih + g.pad - KH0) / S - oh_lo, c0 = (iw + g.pad - KW0) / S - ow_lo;
    const uint16_t* base = P + r0 * CN + c0;
    uint16_t v[NH][NW][3];
#pragma unroll
    for (int a = 0; a < NH; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int j = ((KH0 + S * a) * KW + KW0 + S * b) * 3;
        const int off = j * SD_PROW - (a * CN + b);
#pragma unroll
        for (int c = 0; c < 3; ++c) v[a][b][c] = base[off + c * SD_PROW];
      }
    if (ih >= g.H || iw >= g.W) continue;
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
#pragma unroll
    for (int a = 0; a < NH; ++a)
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        a0 += to_f<DT>(v[a][b][0]);
        a1 += to_f<DT>(v[a][b][1]);
        a2 += to_f<DT>(v[a][b][2]);
      }
    uint4 o;
    o.x = pack2<DT>(a0, a1);
    o.y = pack2<DT>(a2, 0.f);
    o.z = 0u;
    o.w = 0u;
    const long long dst = (((long long)n * g.H + ih) * g.W + iw) * 8;
    if (DV_BOUNDS(dst, 8, (long long)g.N * g.H * g.W * 8, "stem_dgrad_fused gx"))
      *reinterpret_cast<uint4*>(gx + dst) = o;
  }
}

template <int DT, int KH, int KW, int S, int JP>
// waves_per_eu(2): two workgroups per CU (the LDS allows two); without it the 40 accumulator tiles
// took 80 VGPRs + 212 AGPRs and ONE workgroup per CU ran its serial phases with nothing to overlap
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
stem_dgrad_fused_kernel(const uint16_t* __restrict__ gy, const uint16_t* __restrict__ mask, const uint16_t* __restrict__ wb,
                        uint16_t* __restrict__ gx, StemDgradGeom g) {
  typedef typename Vec8<DT>::type v8;
  constexpr int RN = (SD_TH + KH - 2) / S + 2, CN = (SD_TW + KW - 2) / S + 2;  // dy rows / cols a tile reads
  static_assert(RN * CN <= 240 && JP % 16 == 0 && JP * SD_PROW * 2 <= 81920, "window / P^T must fit");
  constexpr int A_BYTES = SD_MROWS * SD_C * 2, B_BYTES = JP * SD_C * 2;
  static_assert(A_BYTES + B_BYTES <= JP * SD_PROW * 2, "staging fits under the P^T area");
  __shared__ __attribute__((aligned(16))) uint8_t smem[JP * SD_PROW * 2];
  uint8_t* As = smem;
  uint8_t* Bs = smem + A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.z;
  const int ih0 = blockIdx.y * SD_TH, iw0 = blockIdx.x * SD_TW;
  const int oh_lo = floor_div(ih0 + g.pad - (KH - 1), S), ow_lo = floor_div(iw0 + g.pad - (KW - 1), S);

  // ---- 1. stage the dy window (rows r = wr * CN + wc <-> pixel (oh_lo + wr, ow_lo + wc)) and B ----
  // Every load of the window, mask and B is issued before the first LDS store (fully unrolled, loads
  // at clamped addresses, validity as a predicate): with a load -> store pair per loop iteration the
  // compiler waited for each load before the next was issued, i.e. ~13 serial memory round trips
  // per workgroup (411 us per call at 32 x 512^2, profiles/kstats_c5_r3_before.txt).
  constexpr int A_IT = SD_MROWS * (SD_C / 8) / 256, B_IT = (JP * (SD_C / 8) + 255) / 256;
  uint4 av[A_IT], mv[A_IT], bv[B_IT];
#pragma unroll
  for (int it = 0; it < A_IT; ++it) {
    const int ci = tid + it * 256, r = ci >> 3, ch = ci & 7;
    const int oh = oh_lo + r / CN, ow = ow_lo + r % CN;
    const bool ok = r < RN * CN && (unsigned)oh < (unsigned)g.OH && (unsigned)ow < (unsigned)g.OW;
    const long long o = ok ? (((long long)n * g.OH + oh) * g.OW + ow) * SD_C + ch * 8 : 0;
    av[it] = *reinterpret_cast<const uint4*>(gy + o);
    if (mask != nullptr) mv[it] = *reinterpret_cast<const uint4*>(mask + o);
    if (!ok) av[it] = make_uint4(0u, 0u, 0u, 0u);
  }
#pragma unroll
  for (int it = 0; it < B_IT; ++it) {
    const int ci = min(tid + it * 256, JP * (SD_C / 8) - 1), r = ci >> 3, ch = ci & 7;
    bv[it] = *reinterpret_cast<const uint4*>(wb + (long long)r * g.w_ld + ch * 8);
  }
#pragma unroll
  for (int it = 0; it < A_IT; ++it) {
    const int ci = tid + it * 256, r = ci >> 3, ch = ci & 7;
    uint4 v = av[it];
    if (mask != nullptr) {  // backward through the conv's ReLU: keep dy where y > 0
      v.x = mask_pos_pk(v.x, mv[it].x);
      v.y = mask_pos_pk(v.y, mv[it].y);
      v.z = mask_pos_pk(v.z, mv[it].z);
      v.w = mask_pos_pk(v.w, mv[it].w);
    }
    *reinterpret_cast<uint4*>(As + r * (SD_C * 2) + ((ch ^ (r & 7)) << 4)) = v;
  }
#pragma unroll
  for (int it = 0; it < B_IT; ++it) {
    const int ci = tid + it * 256, r = ci >> 3, ch = ci & 7;
    if (ci < JP * (SD_C / 8)) *reinterpret_cast<uint4*>(Bs + r * (SD_C * 2) + ((ch ^ (r & 7)) << 4)) = bv[it];
  }
  __syncthreads();

  // ---- 2. P = window @ B^T: wave w owns rows [64 w, 64 w + 64) x all JP columns ----
  constexpr int FM = 4, FN = JP / 16;
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int rx = lane & 7;  // (row & 7) of every fragment row this lane reads (16-aligned bases)
#pragma unroll
  for (int s = 0; s < SD_C / 32; ++s) {
    const int sw = ((s * 4 + (lane >> 4)) ^ rx) << 4;
    v8 af[FM];
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[i] = *reinterpret_cast<const v8*>(As + (wave * 64 + i * 16 + (lane & 15)) * (SD_C * 2) + sw);
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const v8 bf = *reinterpret_cast<const v8*>(Bs + (j * 16 + (lane & 15)) * (SD_C * 2) + sw);
#pragma unroll
      for (int i = 0; i < FM; ++i) acc[i][j] = mfma16x16x32<DT>(af[i], bf, acc[i][j]);
    }
  }
  __syncthreads();  // every wave is done reading the staged operands: P^T overwrites them
  uint16_t* P = reinterpret_cast<uint16_t*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int r0 = wave * 64 + i * 16 + (lane >> 4) * 4;
    if (r0 >= 240) continue;  // rows past the window (zero A) are never read
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = j * 16 + (lane & 15);
      uint2 pk;
      pk.x = pack2<DT>(acc[i][j][0], acc[i][j][1]);
      pk.y = pack2<DT>(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(P + col * SD_PROW + r0) = pk;
    }
  }
  __syncthreads();

  // ---- 3. col2im from LDS: each dx pixel gathers its taps (same order as col2im_kernel) ----
  // Pixels are dealt by stride-S parity class: wave w owns the pixels with (ih % S, iw % S) = class w
  // (S * S == 4 waves), so every lane of a wave walks the same tap subset. That subset is a template
  // parameter (col2im_taps<KH0, KW0>): every tap's P^T offset is a compile-time constant from one
  // per-pixel base, so all of a pixel's LDS reads issue back to back instead of one dependent read per
  // tap behind runtime tap predicates (~4 us of serialized LDS latency per workgroup)
  static_assert(S == 2, "parity-class assignment needs S*S == 4 waves");
  const int py = wave / S, px = wave % S;
  const int kh0 = (ih0 + py + g.pad) % S, kw0 = (iw0 + px + g.pad) % S;  // ih0, iw0 even: uniform per wave
  if (kh0 == 0) {
    if (kw0 == 0) col2im_taps<DT, KH, KW, S, 0, 0, RN, CN>(P, gx, g, n, ih0, iw0, oh_lo, ow_lo, py, px, lane);
    else col2im_taps<DT, KH, KW, S, 0, 1, RN, CN>(P, gx, g, n, ih0, iw0, oh_lo, ow_lo, py, px, lane);
  } else {
    if (kw0 == 0) col2im_taps<DT, KH, KW, S, 1, 0, RN, CN>(P, gx, g, n, ih0, iw0, oh_lo, ow_lo, py, px, lane);
    else col2im_taps<DT, KH, KW, S, 1, 1, RN, CN>(P, gx, g, n, ih0, iw0, oh_lo, ow_lo, py, px, lane);
  }
}

}  // namespace

// ResNet-50 conv1 geometry only (7x7 / 2, Cr = 3 -> 64 channels, JP = 160 >= 147 rows of B);
// < 0: not this kernel's shape
int stem_dgrad_fused_launch(const uint16_t* gy, const uint16_t* mask, const uint16_t* wb, uint16_t* gx,
                            const StemDgradGeom& g, int dtype, hipStream_t s) {
  if (g.KH != 7 || g.KW != 7 || g.stride != 2 || g.Cr != 3 || g.C != SD_C || g.w_rows < 160 || g.w_ld % 8 ||
      g.N < 1 || g.N > 65535 || g.pad < 0 || g.pad > 6 || (reinterpret_cast<uintptr_t>(gy) & 15) ||
      (reinterpret_cast<uintptr_t>(wb) & 15) || (reinterpret_cast<uintptr_t>(gx) & 15) ||
      (mask != nullptr && (reinterpret_cast<uintptr_t>(mask) & 15)))
    return -4;
  const dim3 grid((unsigned)((g.W + SD_TW - 1) / SD_TW), (unsigned)((g.H + SD_TH - 1) / SD_TH), (unsigned)g.N);
  if (dtype == DT_F16)
    hipLaunchKernelGGL((stem_dgrad_fused_kernel<DT_F16, 7, 7, 2, 160>), grid, dim3(256), 0, s, gy, mask, wb, gx, g);
  else
    hipLaunchKernelGGL((stem_dgrad_fused_kernel<DT_BF16, 7, 7, 2, 160>), grid, dim3(256), 0, s, gy, mask, wb, gx, g);
  return (int)hipGetLastError();
}

}  // namespace dv
