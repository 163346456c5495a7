// Halo-tile 3x3 conv for tiny output-channel counts (OC <= 16), e.g. the deconvnet's final step
// block1_conv1.down: 64 -> 3 channels at 224x224 for every (image, filter) pair.
//
// With N = 3 the GEMM view is pure A-operand traffic: the generic implicit-GEMM kernel re-fetches
// every input pixel once per tap (9x). Here a workgroup owns an 8 x 32 output tile, stages the
// 10 x 34 x C input halo tile in LDS once (register path, 16-B loads, zero padding), keeps the
// packed weights [16][9*C] in LDS, and runs v_mfma_f32_16x16x32_bf16 with A fragments read from
// tap-shifted windows of the same LDS tile. Input is read ~1.33x from HBM instead of ~9x from L2.
// LDS pixel rows are XOR-swizzled by 16-B chunk (chunk ^ (pixel & 7)) so a fragment read by 16
// consecutive pixels is bank-conflict free.
#include "common.h"
#include "kernels.h"

namespace dv {

namespace {
constexpr int TH = 8, TW = 32;             // output tile
constexpr int IH = TH + 2, IW = TW + 2;    // input halo tile
constexpr int MAXC = 64;
}  // namespace

template <int C>
__global__ void __launch_bounds__(256, 2) conv3x3_smalln_kernel(const uint16_t* __restrict__ x, const uint16_t* __restrict__ w,
                                                                float* __restrict__ out, int N, int H, int W, int OC,
                                                                int Kpad, int relu_in, int relu, long long out_ld) {
  constexpr int CPP = C / 8;               // 16-B chunks per pixel
  constexpr int PIX_BYTES = C * 2;
  constexpr int A_BYTES = IH * IW * PIX_BYTES;
  constexpr int K = 9 * C;
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + 16 * K * 2];
  uint8_t* As = smem;
  uint8_t* Bs = smem + A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  int b = blockIdx.x;
  const int tx = b % tiles_w;
  b /= tiles_w;
  const int ty = b % tiles_h;
  const int n = b / tiles_h;
  const int y0 = ty * TH - 1, x0 = tx * TW - 1;

  // ---- weights: [16][K] bf16 rows (K contiguous), swizzled per 16-B chunk by row ----
  for (int q = tid; q < 16 * (K / 8); q += 256) {
    const int row = q / (K / 8), ch = q % (K / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(w + (long long)row * Kpad + ch * 8);
    *reinterpret_cast<uint4*>(Bs + row * K * 2 + ((ch ^ (row & 7)) << 4)) = v;
  }
  // ---- input halo tile ----
  const uint16_t* xn = x + (long long)n * H * W * C;
  for (int q = tid; q < IH * IW * CPP; q += 256) {
    const int p = q / CPP, ch = q % CPP;
    const int iy = y0 + p / IW, ix = x0 + p % IW;
    uint4 v = make_uint4(0, 0, 0, 0);
    if ((unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W) {
      v = *reinterpret_cast<const uint4*>(xn + ((long long)iy * W + ix) * C + ch * 8);
      if (relu_in) {
        v.x = relu_bf2(v.x);
        v.y = relu_bf2(v.y);
        v.z = relu_bf2(v.z);
        v.w = relu_bf2(v.w);
      }
    }
    *reinterpret_cast<uint4*>(As + p * PIX_BYTES + ((ch ^ (p & 7)) << 4)) = v;
  }
  __syncthreads();

  // wave owns output rows 2*wave, 2*wave+1 (64 pixels = 4 fragments of 16 along x)
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int col = lane & 15;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int kh = tap / 3, kw = tap % 3;
#pragma unroll
    for (int s = 0; s < C / 32; ++s) {
      // B fragment: k = tap*C + s*32 + 8*(lane>>4) .. +7 of output channel `col`
      const int bch = (tap * C + s * 32) / 8 + (lane >> 4);
      const bf16x8 bf = *reinterpret_cast<const bf16x8*>(Bs + col * K * 2 + ((bch ^ (col & 7)) << 4));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int oy = 2 * wave + (i >> 1), ox = (i & 1) * 16 + col;
        const int p = (oy + kh) * IW + (ox + kw);
        const int ach = s * 4 + (lane >> 4);
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + p * PIX_BYTES + ((ach ^ (p & 7)) << 4));
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, acc[i], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: C[pixel][oc], lane holds pixels (lane>>4)*4 + r of fragment i, channel col ----
  if (col < OC) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pl = (lane >> 4) * 4 + r;
        const int oy = ty * TH + 2 * wave + (i >> 1), ox = tx * TW + (i & 1) * 16 + pl;
        if (oy < H && ox < W) {
          float v = acc[i][r];
          if (relu) v = fmaxf(v, 0.f);
          out[(((long long)n * H + oy) * W + ox) * out_ld + col] = v;
        }
      }
    }
  }
}

int conv3x3_smalln_launch(const uint16_t* x, const uint16_t* w, float* out, int N, int H, int W, int C, int OC,
                          int Kpad, int relu_in, int relu, long long out_ld, hipStream_t s) {
  if (OC > 16 || Kpad < 9 * C) return -1;
  const long long nwg = (long long)N * ((H + TH - 1) / TH) * ((W + TW - 1) / TW);
  if (nwg > 0x7fffffffLL) return -2;
  if (C == 64) {
    hipLaunchKernelGGL(conv3x3_smalln_kernel<64>, dim3((unsigned)nwg), dim3(256), 0, s, x, w, out, N, H, W, OC, Kpad,
                       relu_in, relu, out_ld);
  } else {
    return -3;
  }
  return (int)hipGetLastError();
}

}  // namespace dv
