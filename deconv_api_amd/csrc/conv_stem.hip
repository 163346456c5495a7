// Direct (VALU) kernels for a strided 3x3 conv on a few-channel image: InceptionV3's conv2d_1
// (RGB padded to 8 channels -> 32, 3x3 / stride 2 / 'valid'), forward and input gradient.
//
// Why not the MFMA implicit GEMM: K = 9 taps x 3 real channels = 27 and N = 32 fill a 64x64 MFMA
// tile a quarter, and the input gradient (a transposed conv) went through a 1x1 GEMM into 27
// "column" channels plus an LDS col2im pass: 40 and 17 TF/s, ~0.7 ms per all-octave step at B = 64
// (profiles/dream_layers_c3_r2_hs.txt). Both are bandwidth-sized problems (one 16-B pixel read per
// tap from L2, 64 B written per output pixel); here the fp32 weights [tap][c][co] sit in LDS and
// every read is a same-address float4 broadcast (as wave-uniform scalar loads they were hoisted
// into thousands of spilled SGPRs), and each thread owns one output pixel (forward) or one input
// pixel of one stride-2 parity class (gradient: the class fixes the taps, no divergence).
#include "common.h"
#include "kernels.h"

namespace dv {

// y[n, oy, ox, co] = ReLU?(bias[co] + sum_{kh, kw, c < CR} x[n, oy*S - P + kh, ox*S - P + kw, c] * w[kh][kw][c][co])
template <int DT, int COUT, int CR, int K, int S>
__global__ void __launch_bounds__(256) stem_conv_fwd_kernel(const uint16_t* __restrict__ x, const float* __restrict__ w,
                                                            const float* __restrict__ bias, uint16_t* __restrict__ y,
                                                            int N, int H, int W, int OH, int OW, int pad, int relu,
                                                            long long x_ld, long long y_ld) {
  constexpr int NW4 = K * K * CR * COUT / 4;
  __shared__ float4 wl[NW4];  // all lanes read the same weights: LDS broadcast, no SGPR pressure
  for (int i = threadIdx.x; i < NW4; i += 256) wl[i] = reinterpret_cast<const float4*>(w)[i];
  __syncthreads();
  // one output pixel per thread and no grid-stride loop: with a loop the compiler hoists the
  // (loop-invariant) weight reads out of it into ~860 registers and spills
  const int total = N * OH * OW;
  {
    const int p = blockIdx.x * 256 + threadIdx.x;
    if (p >= total) return;
    const int ox = p % OW, q = p / OW;
    const int oy = q % OH, n = q / OH;
    float acc[COUT];
#pragma unroll
    for (int co = 0; co < COUT; ++co) acc[co] = bias ? bias[co] : 0.f;
    uint2 px[K * K];  // channels 0..3 of every tap's pixel, all loads in flight before the FMAs
#pragma unroll
    for (int kh = 0; kh < K; ++kh)
#pragma unroll
      for (int kw = 0; kw < K; ++kw) {
        const int iy = oy * S - pad + kh, ix = ox * S - pad + kw;
        const bool ok = (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
        px[kh * K + kw] = ok ? *reinterpret_cast<const uint2*>(x + (((long long)n * H + iy) * W + ix) * x_ld)
                             : make_uint2(0u, 0u);
      }
#pragma unroll
    for (int t = 0; t < K * K; ++t) {
      const float xv[4] = {to_f<DT>(px[t].x & 0xFFFFu), to_f<DT>(px[t].x >> 16), to_f<DT>(px[t].y & 0xFFFFu),
                           to_f<DT>(px[t].y >> 16)};
#pragma unroll
      for (int c = 0; c < CR; ++c)
#pragma unroll
        for (int c4 = 0; c4 < COUT / 4; ++c4) {
          const float4 wv = wl[(t * CR + c) * (COUT / 4) + c4];
          acc[4 * c4 + 0] = fmaf(xv[c], wv.x, acc[4 * c4 + 0]);
          acc[4 * c4 + 1] = fmaf(xv[c], wv.y, acc[4 * c4 + 1]);
          acc[4 * c4 + 2] = fmaf(xv[c], wv.z, acc[4 * c4 + 2]);
          acc[4 * c4 + 3] = fmaf(xv[c], wv.w, acc[4 * c4 + 3]);
        }
    }
    uint16_t* yp = y + (long long)p * y_ld;
#pragma unroll
    for (int co = 0; co < COUT; co += 8) {
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = relu ? fmaxf(acc[co + e], 0.f) : acc[co + e];
      *reinterpret_cast<uint4*>(yp + co) =
          uint4{pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7])};
    }
  }
}

// Input gradient of a stride-2 KxK conv from RGB (the 3x3 conv above; ResNet-50's 7x7 conv1) (no bias /
// ReLU: the output gradient gy arrives
// masked): gx[n, y, x, c] = sum over taps (kh, kw) with y = 2 oy - P + kh, x = 2 ox - P + kw of
// gy[n, oy, ox, :] . w[kh][kw][c][:]. Pixels split into the four stride-2 parity classes of
// (y + P, x + P), one class per blockIdx.y: a class's taps are fixed (even: kh 0 and 2, odd: kh 1),
// so every branch is wave-uniform and a thread reads <= 4 output-gradient pixels (64 B each).
// gx gets all 8 (padded) channels, channels >= CR zero.
template <int DT, int COUT, int CR, int K>
__global__ void __launch_bounds__(256) stem_conv_dgrad_s2_kernel(const uint16_t* __restrict__ gy,
                                                                   const float* __restrict__ w,
                                                                   uint16_t* __restrict__ gx, int N, int H, int W,
                                                                   int OH, int OW, int pad, long long gy_ld,
                                                                   long long gx_ld) {
  constexpr int NW4 = K * K * CR * COUT / 4;
  __shared__ float4 wl[NW4];  // LDS broadcast weights [tap][c][co]
  for (int i = threadIdx.x; i < NW4; i += 256) wl[i] = reinterpret_cast<const float4*>(w)[i];
  __syncthreads();
  const int cls = blockIdx.y, py = cls >> 1, px = cls & 1;  // parity of (y + P, x + P)
  const int r0 = pad & 1;
  // class rows y = 2 i + ((py + r0) & 1) - ... : y + P = 2 i' + py  ->  y = 2 i' + py - P
  const int yb = py - pad, xb = px - pad;             // y = 2 i + yb, i >= ceil(-yb / 2)
  const int i0 = yb < 0 ? (-yb + 1) / 2 : 0, j0 = xb < 0 ? (-xb + 1) / 2 : 0;
  const int ni = (H - 1 - yb) >= 0 ? (H - 1 - yb) / 2 + 1 - i0 : 0;
  const int nj = (W - 1 - xb) >= 0 ? (W - 1 - xb) / 2 + 1 - j0 : 0;
  const int total = N * ni * nj;
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= total || ni <= 0 || nj <= 0) return;
  const int jj = p % nj, q = p / nj;
  const int ii = q % ni, n = q / ni;
  const int y = 2 * (ii + i0) + yb, x = 2 * (jj + j0) + xb;
  (void)r0;
  float acc[CR];
#pragma unroll
  for (int c = 0; c < CR; ++c) acc[c] = 0.f;
#pragma unroll
  for (int kh = 0; kh < K; ++kh) {
    if ((kh & 1) != py) continue;  // wave-uniform
    const int oy = (y + pad - kh) >> 1;
#pragma unroll
    for (int kw = 0; kw < K; ++kw) {
      if ((kw & 1) != px) continue;
      const int ox = (x + pad - kw) >> 1;
      if ((unsigned)oy >= (unsigned)OH || (unsigned)ox >= (unsigned)OW) continue;
      const uint16_t* src = gy + (((long long)n * OH + oy) * OW + ox) * gy_ld;
      uint4 g[COUT / 8];
#pragma unroll
      for (int v = 0; v < COUT / 8; ++v) g[v] = *reinterpret_cast<const uint4*>(src + v * 8);
#pragma unroll
      for (int v = 0; v < COUT / 8; ++v) {
        const uint32_t u[4] = {g[v].x, g[v].y, g[v].z, g[v].w};
        float gv[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          gv[2 * e] = to_f<DT>(u[e] & 0xFFFFu);
          gv[2 * e + 1] = to_f<DT>(u[e] >> 16);
        }
#pragma unroll
        for (int c = 0; c < CR; ++c) {
          const float4 w0 = wl[((kh * K + kw) * CR + c) * (COUT / 4) + 2 * v];
          const float4 w1 = wl[((kh * K + kw) * CR + c) * (COUT / 4) + 2 * v + 1];
          float a0 = acc[c];
          a0 = fmaf(gv[0], w0.x, a0);
          a0 = fmaf(gv[1], w0.y, a0);
          a0 = fmaf(gv[2], w0.z, a0);
          a0 = fmaf(gv[3], w0.w, a0);
          a0 = fmaf(gv[4], w1.x, a0);
          a0 = fmaf(gv[5], w1.y, a0);
          a0 = fmaf(gv[6], w1.z, a0);
          acc[c] = fmaf(gv[7], w1.w, a0);
        }
      }
    }
  }
  float v4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < CR && c < 4; ++c) v4[c] = acc[c];
  uint16_t* dst = gx + (((long long)n * H + y) * W + x) * gx_ld;
  *reinterpret_cast<uint4*>(dst) = uint4{pack2<DT>(v4[0], v4[1]), pack2<DT>(v4[2], v4[3]), 0u, 0u};
}

static unsigned stem_grid(long long total) { return (unsigned)((total + 255) / 256); }

// forward: 8-channel (CR = 3 real) input, COUT 32, 3x3, stride 2; < 0 unsupported
int stem_conv_fwd_launch(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W,
                         int OH, int OW, int C, int cr, int cout, int k, int stride, int pad, int relu, long long x_ld,
                         long long y_ld, int dtype, hipStream_t s) {
  if (C != 8 || cr != 3 || cout != 32 || k != 3 || stride != 2 || x_ld % 4 || y_ld % 8 ||
      (long long)N * OH * OW > 0x7FFFFFFFLL)
    return -4;
  const unsigned grid = stem_grid((long long)N * OH * OW);
  if (dtype == DT_F16)
    hipLaunchKernelGGL((stem_conv_fwd_kernel<DT_F16, 32, 3, 3, 2>), dim3(grid), dim3(256), 0, s, x, w, bias, y, N, H, W,
                       OH, OW, pad, relu, x_ld, y_ld);
  else
    hipLaunchKernelGGL((stem_conv_fwd_kernel<DT_BF16, 32, 3, 3, 2>), dim3(grid), dim3(256), 0, s, x, w, bias, y, N, H,
                       W, OH, OW, pad, relu, x_ld, y_ld);
  return (int)hipGetLastError();
}

// input gradient (8-channel gx, channels >= 3 zeroed) of the conv above; < 0 unsupported
int stem_conv_dgrad_launch(const uint16_t* gy, const float* w, uint16_t* gx, int N, int H, int W, int OH, int OW,
                           int C, int cr, int cout, int k, int stride, int pad, long long gy_ld, long long gx_ld,
                           int dtype, hipStream_t s) {
  // (cout, k): InceptionV3 conv2d_1 (32, 3x3) and ResNet-50 conv1 (64, 7x7), both stride 2 from RGB
  const bool inc = cout == 32 && k == 3, res = cout == 64 && k == 7;
  if (C != 8 || cr != 3 || !(inc || res) || stride != 2 || gy_ld % 8 || gx_ld % 8 || pad < 0 || pad >= k ||
      (long long)N * ((H + 2) / 2) * ((W + 2) / 2) > 0x7FFFFFFFLL)
    return -4;
  // grid.y = the 4 parity classes; grid.x sized for the largest class
  const dim3 grid(stem_grid((long long)N * ((H + 2) / 2) * ((W + 2) / 2)), 4);
#define STEM_DG(DT_, CO_, K_)                                                                                  \
  hipLaunchKernelGGL((stem_conv_dgrad_s2_kernel<DT_, CO_, 3, K_>), grid, dim3(256), 0, s, gy, w, gx, N, H, W, OH, \
                     OW, pad, gy_ld, gx_ld)
  if (dtype == DT_F16) {
    if (inc) STEM_DG(DT_F16, 32, 3);
    else STEM_DG(DT_F16, 64, 7);
  } else {
    if (inc) STEM_DG(DT_BF16, 32, 3);
    else STEM_DG(DT_BF16, 64, 7);
  }
#undef STEM_DG
  return (int)hipGetLastError();
}

}  // namespace dv
