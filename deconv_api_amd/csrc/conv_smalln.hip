// Halo-tile 3x3 / stride 1 / pad 1 convolution for narrow outputs (OC tile 16 or 64) at large
// spatial sizes: the deconvnet's block1/block2 conv-downs (64/128 -> 64 channels at 112-224 px,
// with the max-unpool gather fused) and its final step block1_conv1.down (64 -> 3, fp32 out).
//
// Why a separate kernel: with a 64-wide N tile the implicit-GEMM kernel re-fetches every input
// pixel once per tap (9x per 64 output channels) and becomes L2-bandwidth bound. Here a 256-thread
// workgroup owns an 8 x 32 output tile and, per 32-channel input chunk, stages the 10 x 34 halo
// tile (1.33x the tile) and the chunk's weights in LDS once; the 9 taps read shifted windows of
// the same LDS tile as MFMA A fragments (v_mfma_f32_16x16x32_bf16, one 32-deep K step per tap).
// Staging is register-path (all global loads of a chunk issued before any LDS write; the next
// chunk's loads are in flight while the current chunk's MFMAs run), which is what lets the
// unpool switch-select (reference app/deepdream.py:191-209) and ReLU happen on the way in.
// LDS pixel stride 80 B / weight row stride 592 B (odd multiples of 16 B) keep fragment reads of
// 16 consecutive pixels / rows on distinct bank slots.
#include "common.h"
#include "kernels.h"

namespace dv {

namespace {
constexpr int TH = 8, TW = 32;             // output tile (pixels)
constexpr int IH = TH + 2, IW = TW + 2;    // halo tile
constexpr int CK = 32;                     // input channels per chunk (one MFMA K step per tap)
constexpr int PIXB = 80;                   // LDS bytes per halo pixel (64 data + 16 pad)
constexpr int WROWB = 9 * CK * 2 + 16;     // LDS bytes per weight row (576 data + 16 pad)
constexpr int A_LD = IH * IW * 4;          // 16-B chunks to stage for A
}  // namespace

template <int FN, int EPI, bool UNPOOL>
__global__ void __launch_bounds__(256, 2) conv3x3_halo_kernel(const ConvArgs a, int tiles_n) {
  constexpr int BN = FN * 16;
  constexpr int B_LD = BN * 9 * 4;  // 16-B chunks of the weight chunk
  constexpr int A_PER = (A_LD + 255) / 256;
  constexpr int B_PER = (B_LD + 255) / 256;
  constexpr int A_BYTES = IH * IW * PIXB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + BN * WROWB];
  uint8_t* As = smem;
  uint8_t* Bs = smem + A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W, C = a.C;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tn = b % tiles_n;
  b /= tiles_n;
  const int tx = b % tiles_w;
  b /= tiles_w;
  const int ty = b % tiles_h;
  const int n = b / tiles_h;
  const int y0 = ty * TH - 1, x0 = tx * TW - 1;
  const int n0 = tn * BN;
  const int PH = H >> 1, PW = W >> 1;

  uint4 ra[A_PER], rb[B_PER];
  auto load = [&](int cc) {
#pragma unroll
    for (int q = 0; q < A_PER; ++q) {
      const int idx = tid + q * 256;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (idx < A_LD) {
        const int p = idx >> 2, c4 = idx & 3;
        const int iy = y0 + p / IW, ix = x0 + p % IW;
        const int ch = cc * CK + c4 * 8;
        if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
          if constexpr (UNPOOL) {
            const long long pp = ((long long)n * PH + (iy >> 1)) * PW + (ix >> 1);
            v = *reinterpret_cast<const uint4*>(a.x + pp * a.x_ld + ch);
            const long long cp = ((long long)(n / a.code_div) * PH + (iy >> 1)) * PW + (ix >> 1);
            const uint2 cd = *reinterpret_cast<const uint2*>(a.code + cp * C + ch);
            const uint32_t sel4 = (uint32_t)(((iy & 1) << 1) | (ix & 1)) * 0x01010101u;
            const uint32_t e0 = cd.x ^ sel4, e1 = cd.y ^ sel4;
            auto keep2 = [](uint32_t e, int b0) -> uint32_t {
              return ((((e >> (8 * b0)) & 0xFFu) == 0u) ? 0xFFFFu : 0u) |
                     ((((e >> (8 * (b0 + 1))) & 0xFFu) == 0u) ? 0xFFFF0000u : 0u);
            };
            v.x &= keep2(e0, 0);
            v.y &= keep2(e0, 2);
            v.z &= keep2(e1, 0);
            v.w &= keep2(e1, 2);
          } else {
            v = *reinterpret_cast<const uint4*>(a.x + (((long long)n * H + iy) * W + ix) * a.x_ld + ch);
          }
          if (a.relu_in) {
            v.x = relu_bf2(v.x);
            v.y = relu_bf2(v.y);
            v.z = relu_bf2(v.z);
            v.w = relu_bf2(v.w);
          }
        }
      }
      ra[q] = v;
    }
#pragma unroll
    for (int q = 0; q < B_PER; ++q) {
      const int idx = tid + q * 256;
      if (idx < B_LD) {
        const int row = idx / 36, rem = idx % 36;
        const int tap = rem >> 2, c4 = rem & 3;
        rb[q] = *reinterpret_cast<const uint4*>(a.w + (long long)(n0 + row) * a.Kpad + tap * C + cc * CK + c4 * 8);
      }
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int q = 0; q < A_PER; ++q) {
      const int idx = tid + q * 256;
      if (idx < A_LD) *reinterpret_cast<uint4*>(As + (idx >> 2) * PIXB + (idx & 3) * 16) = ra[q];
    }
#pragma unroll
    for (int q = 0; q < B_PER; ++q) {
      const int idx = tid + q * 256;
      if (idx < B_LD) {
        const int row = idx / 36, rem = idx % 36;
        *reinterpret_cast<uint4*>(Bs + row * WROWB + rem * 16) = rb[q];
      }
    }
  };

  f32x4 acc[4][FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nchunks = C / CK;
  load(0);
  store();
  __syncthreads();
  const int kq = lane >> 4, col = lane & 15;
  for (int cc = 0; cc < nchunks; ++cc) {
    const bool more = cc + 1 < nchunks;
    if (more) load(cc + 1);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
      bf16x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + (j * 16 + col) * WROWB + tap * 64 + kq * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 2 * wave + (i >> 1), xo = (i & 1) * 16 + col;
        const int p = (r + kh) * IW + xo + kw;
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + p * PIXB + kq * 16);
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) {
      __syncthreads();
      store();
      __syncthreads();
    }
  }

  // ---- epilogue: fragment i = output row 2*wave + (i>>1), x = (i&1)*16 + (lane>>4)*4 + r ----
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int oc = n0 + j * 16 + col;
    if (oc >= a.OC) continue;
    const float bias = a.bias ? a.bias[oc] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int oy = ty * TH + 2 * wave + (i >> 1);
      if (oy >= H) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ox = tx * TW + (i & 1) * 16 + kq * 4 + r;
        if (ox >= W) continue;
        float v = acc[i][j][r] + bias;
        if (a.relu) v = fmaxf(v, 0.f);
        const long long o = (((long long)n * H + oy) * W + ox) * a.out_ld + oc;
        if constexpr (EPI == CONV_E_F32)
          reinterpret_cast<float*>(a.out)[o] = v;
        else
          reinterpret_cast<uint16_t*>(a.out)[o] = f2bf(v);
      }
    }
  }
}

template <int FN, int EPI, bool UNPOOL>
static int halo_cfg(const ConvArgs& a, hipStream_t s) {
  const int tiles_n = a.OCpad / (FN * 16);
  const long long nwg = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW) * tiles_n;
  if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL((conv3x3_halo_kernel<FN, EPI, UNPOOL>), dim3((unsigned)nwg), dim3(256), 0, s, a, tiles_n);
  return (int)hipGetLastError();
}

int conv3x3_halo_launch(const ConvArgs& a, int unpool, int epi, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C % CK != 0 ||
      a.H != a.OH || a.W != a.OW || a.accumulate || a.mask)
    return -4;
  const bool narrow = a.OC <= 16;
  if (!narrow && a.OCpad % 64 != 0) return -5;
#define DV_HALO(FN, E)                                                          \
  return unpool ? halo_cfg<FN, E, true>(a, s) : halo_cfg<FN, E, false>(a, s)
  if (epi == CONV_E_F32) {
    if (narrow) DV_HALO(1, CONV_E_F32);
    DV_HALO(4, CONV_E_F32);
  }
  if (epi == CONV_E_BF16) {
    if (narrow) DV_HALO(1, CONV_E_BF16);
    DV_HALO(4, CONV_E_BF16);
  }
#undef DV_HALO
  return -1;
}

}  // namespace dv
