// Persistent halo-tile 3x3 / stride 1 / pad 1 convolution for 64-channel inputs with narrow
// outputs (OC tile 64 or 16): the deconvnet's block1 conv-downs at 224x224 —
// block1_conv2.down (64 -> 64, max-unpool of the 112x112 signal fused into the staging) and the
// final block1_conv1.down (64 -> 3, fp32 reconstruction out).
//
// Why: with a 64-wide (or 16-wide) N tile, the implicit-GEMM kernel fetches every input pixel
// once per tap (9x) and is L2-bandwidth bound (profiles/layers_r1_*.txt: 430 TF/s and 40 TF/s).
// Here one 512-thread workgroup per CU:
//   * loads the layer's packed weights (<= 64 x 576 bf16 = 72 KiB) into LDS ONCE;
//   * walks 8 x 32 output tiles (grid-stride, persistent); per tile the 10 x 34 x 64-channel
//     halo (48 KiB) is staged once and the 9 taps read shifted windows of it as MFMA A
//     fragments (v_mfma_f32_16x16x32_bf16, 18 K-steps of 32 per tile);
//   * the next tile's halo is loaded into VGPRs (16-B loads; unpool switch-select + ReLU on the
//     way in) while the current tile's MFMAs run, then written to LDS between two barriers.
// Halo pixels use a padded 144-B stride (9 bank slots, coprime with 16: 16 consecutive pixels hit
// 16 distinct slots) so every tap shift is a constant ds_read offset; weight rows (1152 B) are
// XOR-swizzled by 16-B chunk with (row & 7). Both fragment reads are bank-conflict free.
#include "common.h"
#include "kernels.h"

namespace dv {

namespace {
constexpr int TH = 8, TW = 32;             // output tile: 8 waves x (1 row x 32 px)
constexpr int IH = TH + 2, IW = TW + 2;    // halo tile
constexpr int C64 = 64;                    // input channels
constexpr int PIXB = C64 * 2 + 16;         // 144 B per halo pixel: 9 bank slots (coprime with 16)
constexpr int KW9 = 9 * C64;               // K = 576
constexpr int WROWB = KW9 * 2;             // 1152 B per weight row (72 chunks)
constexpr int HALO_CH = IH * IW * 8;       // 16-B chunks per halo (4896)
constexpr int PER_T = (HALO_CH + 511) / 512;  // 6 chunks per thread
constexpr int FM = 2;                      // 16-px fragments per wave (one 32-px row)
}  // namespace

__device__ __forceinline__ int sw_off(int row, int chunk, int rowb) {
  return row * rowb + ((chunk ^ (row & 7)) << 4);
}
__device__ __forceinline__ int p_of(int idx) { return idx >> 3; }

template <int FN, int EPI, bool UNPOOL>
__global__ void __launch_bounds__(512, 1) conv3x3_c64_persist_kernel(const ConvArgs a) {
  constexpr int BN = FN * 16;
  constexpr int A_BYTES = IH * IW * PIXB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + BN * WROWB];
  uint8_t* As = smem;
  uint8_t* Bs = smem + A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  const int ntiles = a.N * tiles_h * tiles_w;
  const int PH = H >> 1, PW = W >> 1;

  // ---- weights -> LDS once: [BN rows][576] with the row-XOR chunk swizzle ----
  for (int q = tid; q < BN * (KW9 / 8); q += 512) {
    const int row = q / (KW9 / 8), ch = q % (KW9 / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(a.w + (long long)row * a.Kpad + ch * 8);
    *reinterpret_cast<uint4*>(Bs + row * WROWB + (((ch & ~7) | ((ch & 7) ^ (row & 7))) << 4)) = v;
  }

  // Raw loads only (no use of the loaded values) so every load of the next tile stays in flight
  // across the current tile's MFMAs; the switch-select and ReLU happen at LDS-store time.
  uint4 ra[PER_T];
  uint2 rc[PER_T];
  int ld_y0 = 0, ld_x0 = 0;
  uint32_t okmask = 0;
  auto load_tile = [&](int t) {
    int b = t;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    ld_y0 = y0;
    ld_x0 = x0;
    const long long nc = (long long)(n / a.code_div);
    okmask = 0;
#pragma unroll
    for (int q = 0; q < PER_T; ++q) {
      // unconditional loads at clamped (always valid) coordinates; validity kept as a bit
      const int idx = min(tid + q * 512, HALO_CH - 1);
      const int p = idx >> 3, c8 = idx & 7;
      const int iy = y0 + p / IW, ix = x0 + p % IW;
      const bool ok = tid + q * 512 < HALO_CH && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      okmask |= (uint32_t)ok << q;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      if constexpr (UNPOOL) {
        const long long pp = ((long long)n * PH + (cy >> 1)) * PW + (cx >> 1);
        ra[q] = *reinterpret_cast<const uint4*>(a.x + pp * a.x_ld + c8 * 8);
        const long long cp = (nc * PH + (cy >> 1)) * PW + (cx >> 1);
        rc[q] = *reinterpret_cast<const uint2*>(a.code + cp * C64 + c8 * 8);
      } else {
        ra[q] = *reinterpret_cast<const uint4*>(a.x + (((long long)n * H + cy) * W + cx) * a.x_ld + c8 * 8);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < PER_T; ++q) {
      const int idx = tid + q * 512;
      if (idx < HALO_CH) {
        uint4 v = ((okmask >> q) & 1u) ? ra[q] : make_uint4(0, 0, 0, 0);
        if constexpr (UNPOOL) {
          const int p = idx >> 3;
          const int iy = ld_y0 + p / IW, ix = ld_x0 + p % IW;
          const uint32_t sel4 = (uint32_t)(((iy & 1) << 1) | (ix & 1)) * 0x01010101u;
          const uint32_t e0 = rc[q].x ^ sel4, e1 = rc[q].y ^ sel4;
          auto keep2 = [](uint32_t e, int b0) -> uint32_t {
            return ((((e >> (8 * b0)) & 0xFFu) == 0u) ? 0xFFFFu : 0u) |
                   ((((e >> (8 * (b0 + 1))) & 0xFFu) == 0u) ? 0xFFFF0000u : 0u);
          };
          v.x &= keep2(e0, 0);
          v.y &= keep2(e0, 2);
          v.z &= keep2(e1, 0);
          v.w &= keep2(e1, 2);
        }
        if (a.relu_in) {
          v.x = relu_bf2(v.x);
          v.y = relu_bf2(v.y);
          v.z = relu_bf2(v.z);
          v.w = relu_bf2(v.w);
        }
        *reinterpret_cast<uint4*>(As + p_of(idx) * PIXB + (idx & 7) * 16) = v;
      }
    }
  };

  const int kq = lane >> 4, col = lane & 15;
  int t = blockIdx.x;
  if (t < ntiles) load_tile(t);
  while (t < ntiles) {
    __syncthreads();  // previous tile's fragment reads done (and, first time, the weights landed)
    store_tile();
    __syncthreads();
    const int tcur = t;
    t += gridDim.x;
    if (t < ntiles) load_tile(t);  // in flight during the MFMAs below

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int kc = s * 4 + kq;  // 16-B chunk within the 64 input channels
        bf16x8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = j * 16 + col;
          const int ch = tap * 8 + kc;
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * WROWB + (((ch & ~7) | ((ch & 7) ^ (row & 7))) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = wave, xo = i * 16 + col;
          const int p = (r + kh) * IW + xo + kw;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + p * PIXB + kc * 16);
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // ---- epilogue: fragment i = output row `wave`, x = i*16 + kq*4 + r ----
    int b = tcur;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    float biasv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) biasv[j] = (a.bias && j * 16 + col < a.OC) ? a.bias[j * 16 + col] : 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int oc = j * 16 + col;
      if (oc >= a.OC) continue;
      const float bias = biasv[j];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int oy = ty * TH + wave;
        if (oy >= H) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ox = tx * TW + i * 16 + kq * 4 + r;
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
}

template <int FN, int EPI, bool UNPOOL>
static int persist_cfg(const ConvArgs& a, hipStream_t s) {
  const long long ntiles = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  if (ntiles <= 0 || ntiles > 0x7fffffffLL) return -2;
  // CU count queried once (keeps the launch path free of runtime queries during graph capture)
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n > 0 ? n : 256;
  }();
  const long long grid = std::min<long long>(ntiles, (long long)cus);
  hipLaunchKernelGGL((conv3x3_c64_persist_kernel<FN, EPI, UNPOOL>), dim3((unsigned)grid), dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

int conv3x3_halo_launch(const ConvArgs& a, int unpool, int epi, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != C64 || a.H != a.OH ||
      a.W != a.OW || a.accumulate || a.mask || a.Kpad < KW9)
    return -4;
  const bool narrow = a.OC <= 16;
  if (!narrow && a.OCpad != 64) return -5;
#define DV_P(FN, E) return unpool ? persist_cfg<FN, E, true>(a, s) : persist_cfg<FN, E, false>(a, s)
  if (epi == CONV_E_F32) {
    if (narrow) DV_P(1, CONV_E_F32);
    DV_P(4, CONV_E_F32);
  }
  if (epi == CONV_E_BF16) {
    if (narrow) DV_P(1, CONV_E_BF16);
    DV_P(4, CONV_E_BF16);
  }
#undef DV_P
  return -1;
}

}  // namespace dv
