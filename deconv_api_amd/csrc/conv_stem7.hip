// Forward of ResNet-50's RGB stem conv (conv1: 3 -> 64, 7x7 / 2, pad 3) on MFMA with a tap-paired K.
//
// The generic implicit GEMM pads every tap to 8 channels (K = 49 x 8 = 392 -> 13 MFMA K steps of 32,
// 5 of every 8 K columns zero): ~0.32 PF/s and ~1 TB/s, 11 us per 512^2 image
// (profiles/pmc_c5_r5_bytes.txt, conv_dma_kernel<1, 8, 1, 4, 4, ...>). Here
//   * a pixel is staged in LDS as 4 channels (8 B: RGB + one zero), and
//   * the K of one 32-deep MFMA step is ONE kernel row kh: lane group q = lane / 16 holds taps
//     (kh, 2q) and (kh, 2q + 1), 4 channels each (kw = 7 is a zero weight column). At stride 2 those
//     two taps read ADJACENT input pixels, so a lane's whole B fragment is one 16-B ds_read_b128
//     (the window origin 2 * ox0 - 3 is odd, so every fragment read is 16-B aligned).
// K = 7 x 32 = 224: 1.9x fewer MFMAs than the 8-channel K.
//
// One 256-thread workgroup owns a 16 x 32 output tile (all 64 channels): it stages the weights
// ([64][224] 16-bit, rows XOR-swizzled in 16-B chunks) and the 37 x 70 pixel input window once, then
// computes the tile as two 8-row halves (wave w: output rows 2w, 2w + 1 of the half; 4 pixel
// fragments x 4 channel fragments). The MFMA is issued transposed (A = weights, B = pixels), so a
// lane ends with 4 consecutive channels of one pixel: bias + ReLU, one 8-B store per fragment.
// 54 KB of LDS: 3 workgroups per CU.
#include "common.h"
#include "kernels.h"

namespace dv {

namespace {

constexpr int S7_TH = 16, S7_TW = 32;                // output tile
constexpr int S7_IR = 2 * S7_TH + 5;                 // input window rows (37)
constexpr int S7_ICU = 2 * S7_TW + 6;                // input window columns read (70: kw = 7 over-reads one)
constexpr int S7_IC = 72;                            // LDS pixels per window row
constexpr int S7_K = 224;                            // 7 kh x (8 kw x 4 c)
constexpr int S7_WROW = 512;                         // weight row bytes in LDS (28 chunks swizzled in 32)
constexpr int S7_LDS = 64 * S7_WROW + S7_IR * S7_IC * 8;

template <int DT>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
stem7_fwd_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w, const float* __restrict__ bias,
                 uint16_t* __restrict__ y, int H, int W, int OH, int OW, int relu) {
  typedef typename Vec8<DT>::type v8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[S7_LDS];
  uint8_t* Ws = smem;
  uint8_t* Xs = smem + 64 * S7_WROW;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int n = blockIdx.z, oy0 = blockIdx.y * S7_TH, ox0 = blockIdx.x * S7_TW;
  const int iy0 = 2 * oy0 - 3, ix0 = 2 * ox0 - 3;

  // ---- stage weights + window: every global load issued before the first LDS store ----
  constexpr int W_IT = 64 * (S7_K / 8) / 256;              // 7 16-B chunks per thread
  constexpr int X_IT = (S7_IR * S7_ICU + 255) / 256;       // 11 pixels per thread
  uint4 wv[W_IT];
  uint2 xv[X_IT];
#pragma unroll
  for (int it = 0; it < W_IT; ++it) {
    const int ci = tid + it * 256;
    wv[it] = *reinterpret_cast<const uint4*>(w + ci * 8);  // row ci / 28, chunk ci % 28: contiguous
  }
#pragma unroll
  for (int it = 0; it < X_IT; ++it) {
    const int ci = tid + it * 256, r = ci / S7_ICU, c = ci % S7_ICU;
    const int iy = iy0 + r, ix = ix0 + c;
    const bool ok = ci < S7_IR * S7_ICU && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    const long long o = ok ? (((long long)n * H + iy) * W + ix) * 8 : 0;
    xv[it] = *reinterpret_cast<const uint2*>(x + o);  // channels 0..3 of the 8-channel pixel
    if (!ok) xv[it] = make_uint2(0u, 0u);
  }
#pragma unroll
  for (int it = 0; it < W_IT; ++it) {
    const int ci = tid + it * 256, r = ci / (S7_K / 8), c = ci % (S7_K / 8);
    *reinterpret_cast<uint4*>(Ws + r * S7_WROW + ((c ^ (r & 7)) << 4)) = wv[it];
  }
#pragma unroll
  for (int it = 0; it < X_IT; ++it) {
    const int ci = tid + it * 256, r = ci / S7_ICU, c = ci % S7_ICU;
    if (ci < S7_IR * S7_ICU) *reinterpret_cast<uint2*>(Xs + (r * S7_IC + c) * 8) = xv[it];
  }
  const int lr = lane & 15, kq = lane >> 4;
  float bs[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs[j][r] = bias != nullptr ? bias[j * 16 + kq * 4 + r] : 0.f;
  __syncthreads();

#pragma unroll 1
  for (int h = 0; h < 2; ++h) {
    const int rl = h * 8 + wave * 2;  // this wave's first local output row
    f32x4 acc[4][4];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kh = 0; kh < 7; ++kh) {
      v8 a[4], b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        a[j] = *reinterpret_cast<const v8*>(Ws + (j * 16 + lr) * S7_WROW + (((kh * 4 + kq) ^ (lr & 7)) << 4));
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const int row = 2 * (rl + (f >> 1)) + kh, col = 2 * ((f & 1) * 16 + lr) + 2 * kq;
        b[f] = *reinterpret_cast<const v8*>(Xs + (row * S7_IC + col) * 8);
      }
#pragma unroll
      for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[f][j] = mfma16x16x32<DT>(a[j], b[f], acc[f][j]);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const int oy = oy0 + rl + (f >> 1), ox = ox0 + (f & 1) * 16 + lr;
      if (oy >= OH || ox >= OW) continue;
      uint16_t* dst = y + (((long long)n * OH + oy) * OW + ox) * 64 + kq * 4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v[r] = acc[f][j][r] + bs[j][r];
          if (relu) v[r] = fmaxf(v[r], 0.f);
        }
        *reinterpret_cast<uint2*>(dst + j * 16) = make_uint2(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]));
      }
    }
  }
}

}  // namespace

// x [N,H,W,8] (channels >= 3 ignored: their weights are zero), w [64][224] (kh, kw 0..7, c 0..3; zero
// where kw = 7 or c = 3), y [N,OH,OW,64], all dense; < 0: not this kernel's geometry
int stem7_fwd_launch(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H, int W, int OH,
                     int OW, int relu, int dtype, hipStream_t s) {
  if (N < 1 || N > 65535 || H < 1 || W < 1 || OH != (H - 1) / 2 + 1 || OW != (W - 1) / 2 + 1 ||
      (reinterpret_cast<uintptr_t>(x) & 15) || (reinterpret_cast<uintptr_t>(w) & 15) ||
      (reinterpret_cast<uintptr_t>(y) & 15))
    return -4;
  const dim3 grid((unsigned)((OW + S7_TW - 1) / S7_TW), (unsigned)((OH + S7_TH - 1) / S7_TH), (unsigned)N);
  if (dtype == DT_F16)
    hipLaunchKernelGGL((stem7_fwd_kernel<DT_F16>), grid, dim3(256), 0, s, x, w, bias, y, H, W, OH, OW, relu);
  else
    hipLaunchKernelGGL((stem7_fwd_kernel<DT_BF16>), grid, dim3(256), 0, s, x, w, bias, y, H, W, OH, OW, relu);
  return (int)hipGetLastError();
}

}  // namespace dv
