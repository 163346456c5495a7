// 2:4 structured-sparse MFMA conv-down for max-unpooled inputs (gfx950 v_smfmac_f32_32x32x32_bf16).
//
// out[n, 2p+a, 2q+b, :] = ReLU( sum over the 3x3 taps of ReLU(unpool(v, code)) * Wdown )
// computed per sub-pixel phase (a, b) straight from the POOLED signal v and its 2-bit switch code:
// the 9 taps of every input channel regroup into 4-row K-groups with <= 2 nonzeros (module docstring
// of deconv_api_amd/ops/sparse_unpool.py, which is also the PyTorch emulation this kernel is tested
// against). Per 16 channels: 5 smfmac K-steps instead of 9 dense 32x32x16 steps. The unpooled map is
// never materialised: the compressed A operand is (relu(v), code) gathered from the 4 pooled pixels
// an output phase touches (centre, row neighbour, column neighbour, corner).
//
// Operand layout (measured on MI355X, tools/smfmac_layout.hip, profiles/smfmac_layout.txt):
//   B: lane l holds column l%32, K rows (l/32)*16 .. +15 (contiguous);
//   A: lane l holds row l%32, 4 groups at K rows {8h..8h+7} u {16+8h..16+8h+7}, h = l/32,
//      2 compressed values per group; sparsity index of compressed slot s in idx bits 2s..2s+1.
//   D: lane l holds column l%32, rows (i/4)*8 + h*4 + i%4 (i < 16) -- as the dense 32x32 MFMA.
//
// Tile: 128 pooled pixels (one phase; flattened over images) x 128 output channels, 4 waves of 64x64;
// packed weights [4 phases][C/16][Ci][160] stream through a double-buffered LDS tile [128][168].
#include "common.h"

namespace dv {

typedef __attribute__((ext_vector_type(16))) __bf16 bf16x16;
typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(4))) uint32_t u32x4;
typedef __attribute__((ext_vector_type(8))) uint32_t u32x8;

namespace {
constexpr int SP_BM = 128, SP_BN = 128, SP_KC = 160, SP_LDB = 168, SP_LDO = 136;
constexpr int SP_PX = 256;
// wave tile: SP_MI x SP_NJ blocks of 32x32; 4 waves as (4 / SP_WN) x SP_WN over the 128 x 128 tile
constexpr int SP_MI = 1, SP_NJ = 4, SP_WN = 1;  // staged pooled pixels per chunk: 128 + PW + 1, PW <= 127

__device__ __forceinline__ uint32_t relu_bf(uint32_t x) { return (x & 0x8000u) ? 0u : x; }

// S1 pair: two channels of the centre pixel -> groups (2t, 2t+1); writes 2 A dwords + 8 idx bits
__device__ __forceinline__ void s1_pair(uint32_t x, uint32_t k, uint32_t& a0, uint32_t& a1, uint32_t& idx) {
  const uint32_t xl = relu_bf(x & 0xffffu), xh = relu_bf(x >> 16);
  const uint32_t kl = k & 3u, kh = (k >> 8) & 3u;
  a0 = (kl < 3 ? xl : 0u) | ((kl == 3 ? xl : 0u) << 16);
  a1 = (kh < 3 ? xh : 0u) | ((kh == 3 ? xh : 0u) << 16);
  idx = (kl < 2 ? kl : 2u) | (3u << 2) | ((kh < 2 ? kh : 2u) << 4) | (3u << 6);
}

// S2 pair: row-neighbour pair xr/kr, column-neighbour pair xc/kc
__device__ __forceinline__ void s2_pair(uint32_t xr, uint32_t kr, uint32_t xc, uint32_t kc, uint32_t r, uint32_t cc,
                                        uint32_t& a0, uint32_t& a1, uint32_t& idx) {
  uint32_t w[2], bits = 0;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint32_t vr = relu_bf((xr >> (16 * t)) & 0xffffu), vc = relu_bf((xc >> (16 * t)) & 0xffffu);
    const uint32_t ka = (kr >> (8 * t)) & 3u, kb = (kc >> (8 * t)) & 3u;
    const uint32_t s0 = (ka >> 1) == r ? vr : 0u, s1 = (kb & 1u) == cc ? vc : 0u;
    w[t] = s0 | (s1 << 16);
    bits |= ((ka & 1u) | ((2u + (kb >> 1)) << 2)) << (4 * t);
  }
  a0 = w[0];
  a1 = w[1];
  idx = bits;
}

// S3 quad: 4 corner channels (2 groups) -> 2 A dwords; index pattern (0, 1) per group is constant
__device__ __forceinline__ void s3_quad(uint2 x, uint32_t k, uint32_t code_hit, uint32_t& a0, uint32_t& a1) {
  uint32_t e[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t xv = relu_bf(((t < 2 ? x.x : x.y) >> (16 * (t & 1))) & 0xffffu);
    e[t] = ((k >> (8 * t)) & 3u) == code_hit ? xv : 0u;
  }
  a0 = e[0] | (e[1] << 16);
  a1 = e[2] | (e[3] << 16);
}

}  // namespace

__global__ void __launch_bounds__(256, 1)
    sparse_unpool_conv_kernel(const uint16_t* __restrict__ v, const uint8_t* __restrict__ code,
                              const uint16_t* __restrict__ wt, uint16_t* __restrict__ out, int NB, int PH, int PW,
                              int C, int Ci, int code_div) {
  __shared__ __attribute__((aligned(16))) uint16_t sB[2][SP_BN * SP_LDB];
  __shared__ __attribute__((aligned(16))) uint32_t sAv[2][SP_PX * 10];
  __shared__ __attribute__((aligned(16))) uint32_t sAk[2][SP_PX * 5];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / SP_WN, wn = wave % SP_WN;
  const int h = lane >> 5, r32 = lane & 31;
  const int ph = blockIdx.z, a = ph >> 1, b = ph & 1;
  const int da = a ? 1 : -1, db = b ? 1 : -1;
  const uint32_t r = 1 - a, cc = 1 - b, corner = 2 * r + cc;
  const long long Mp = (long long)NB * PH * PW;
  const long long m0 = (long long)blockIdx.x * SP_BM;
  const int n0 = blockIdx.y * SP_BN;
  const int nch = C / 16;

  // The 4 pooled pixels an output row touches are flattened-index shifts {0, da*PW, db, da*PW+db} of
  // its own: one contiguous pixel range [m0+lo, m0+128+hi) per tile covers them all. It is staged
  // per 16-channel chunk into LDS with coalesced 16-B loads (values: 10 dwords/pixel, codes: 5).
  const int sh[4] = {0, da * PW, db, da * PW + db};
  const int lo = min(min(sh[0], sh[1]), min(sh[2], sh[3])), hi = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
  const int npx = SP_BM + hi - lo;
  const long long base = m0 + lo;
  int L[SP_MI][4];
  bool ok[SP_MI][4];
#pragma unroll
  for (int i = 0; i < SP_MI; ++i) {
    const long long P = m0 + 32 * SP_MI * wm + 32 * i + r32;
    const bool valid = P < Mp;
    const long long Pc = valid ? P : 0;
    const int n = (int)(Pc / ((long long)PH * PW));
    const int rem = (int)(Pc - (long long)n * PH * PW);
    const int p = rem / PW, q = rem - p * PW;
    const int ys[4] = {p, p + da, p, p + da}, xs[4] = {q, q, q + db, q + db};
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      ok[i][t] = valid && ys[t] >= 0 && ys[t] < PH && xs[t] >= 0 && xs[t] < PW;
      L[i][t] = 32 * SP_MI * wm + 32 * i + r32 + sh[t] - lo;
    }
  }
  u32x4 areg[3];
  auto load_a = [&](int ch) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int e = tid + 256 * u, pix = e / 3, part = e - pix * 3;
      const long long g = base + pix;
      areg[u] = u32x4{0u, 0u, 0u, 0u};
      if (pix < npx && g >= 0 && g < Mp) {
        if (part < 2) {
          areg[u] = *reinterpret_cast<const u32x4*>(v + g * C + ch * 16 + part * 8);
        } else {
          const int n = (int)(g / ((long long)PH * PW));
          const long long cg = g - (long long)(n - n / code_div) * PH * PW;
          areg[u] = *reinterpret_cast<const u32x4*>(code + cg * C + ch * 16);
        }
      }
    }
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 3; ++u) {
      const int e = tid + 256 * u, pix = e / 3, part = e - pix * 3;
      if (pix < npx) {
        if (part < 2) {
          uint32_t* d = &sAv[buf][pix * 10 + part * 4];
          *reinterpret_cast<uint2*>(d) = uint2{areg[u].x, areg[u].y};
          *reinterpret_cast<uint2*>(d + 2) = uint2{areg[u].z, areg[u].w};
        } else {
          uint32_t* d = &sAk[buf][pix * 5];
          d[0] = areg[u].x;
          d[1] = areg[u].y;
          d[2] = areg[u].z;
          d[3] = areg[u].w;
        }
      }
    }
  };

  // B tile staging: 128 rows x 160 bf16 = 20 x 16 B per row, 10 per thread
  const uint16_t* wph = wt + (long long)ph * nch * Ci * SP_KC;
  u32x4 breg[10];
  auto load_b = [&](int ch) {
    const uint16_t* src = wph + ((long long)ch * Ci + n0) * SP_KC;
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int e = tid + 256 * u, row = e / 20, kk = e - row * 20;
      breg[u] = *reinterpret_cast<const u32x4*>(src + row * SP_KC + 8 * kk);
    }
  };
  auto store_b = [&](int buf) {
#pragma unroll
    for (int u = 0; u < 10; ++u) {
      const int e = tid + 256 * u, row = e / 20, kk = e - row * 20;
      *reinterpret_cast<u32x4*>(&sB[buf][row * SP_LDB + 8 * kk]) = breg[u];
    }
  };

  f32x16 acc[SP_MI][SP_NJ];
#pragma unroll
  for (int i = 0; i < SP_MI; ++i)
#pragma unroll
    for (int j = 0; j < SP_NJ; ++j) acc[i][j] = f32x16{};

  load_b(0);
  store_b(0);
  __syncthreads();

  load_a(0);
  store_a(0);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    if (ch + 1 < nch) {
      load_a(ch + 1);
      load_b(ch + 1);
    }
    // this lane's operands from the staged chunk: centre/row/col channel pairs at {2h, 4+2h, 8+2h,
    // 12+2h}, corner quads at {4h, 8+4h}
    uint32_t xv[SP_MI][3][4], kv[SP_MI][3][4], kd[SP_MI][2];
    uint2 xd[SP_MI][2];
    const uint32_t* av_s = sAv[ch & 1];
    const uint32_t* ak_s = sAk[ch & 1];
#pragma unroll
    for (int i = 0; i < SP_MI; ++i) {
#pragma unroll
      for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          xv[i][t][j] = ok[i][t] ? av_s[L[i][t] * 10 + 2 * j + h] : 0u;
          kv[i][t][j] = ok[i][t] ? (ak_s[L[i][t] * 5 + j] >> (16 * h)) & 0xffffu : 0u;
        }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        xd[i][j] = ok[i][3] ? *reinterpret_cast<const uint2*>(&av_s[L[i][3] * 10 + 4 * j + 2 * h]) : uint2{0u, 0u};
        kd[i][j] = ok[i][3] ? ak_s[L[i][3] * 5 + 2 * j + h] : 0u;
      }
    }
    const uint16_t* bb = sB[ch & 1];
#pragma unroll
    for (int step = 0; step < 5; ++step) {
      bf16x16 bf[SP_NJ];
#pragma unroll
      for (int j = 0; j < SP_NJ; ++j) {
        const uint16_t* src = bb + (32 * SP_NJ * wn + 32 * j + r32) * SP_LDB + step * 32 + h * 16;
        u32x8 t;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(src), hi = *reinterpret_cast<const u32x4*>(src + 8);
        t.s0123 = lo;
        t.s4567 = hi;
        bf[j] = __builtin_bit_cast(bf16x16, t);
      }
#pragma unroll
      for (int i = 0; i < SP_MI; ++i) {
        uint32_t aw[4];
        uint32_t idx;
        if (step < 2) {  // S1: groups (2h,2h+1) <- pair j=2*step, groups (4+2h,5+2h) <- pair 2*step+1
          uint32_t i0, i1;
          s1_pair(xv[i][0][2 * step], kv[i][0][2 * step], aw[0], aw[1], i0);
          s1_pair(xv[i][0][2 * step + 1], kv[i][0][2 * step + 1], aw[2], aw[3], i1);
          idx = i0 | (i1 << 8);
        } else if (step < 4) {
          const int s = step - 2;
          uint32_t i0, i1;
          s2_pair(xv[i][1][2 * s], kv[i][1][2 * s], xv[i][2][2 * s], kv[i][2][2 * s], r, cc, aw[0], aw[1], i0);
          s2_pair(xv[i][1][2 * s + 1], kv[i][1][2 * s + 1], xv[i][2][2 * s + 1], kv[i][2][2 * s + 1], r, cc, aw[2],
                  aw[3], i1);
          idx = i0 | (i1 << 8);
        } else {
          s3_quad(xd[i][0], kd[i][0], corner, aw[0], aw[1]);
          s3_quad(xd[i][1], kd[i][1], corner, aw[2], aw[3]);
          idx = 0x4444u;
        }
        const u32x4 av = {aw[0], aw[1], aw[2], aw[3]};
        const bf16x8 af = __builtin_bit_cast(bf16x8, av);
#pragma unroll
        for (int j = 0; j < SP_NJ; ++j)
          acc[i][j] = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(af, bf[j], acc[i][j], (int)idx, 0, 0);
      }
    }
    if (ch + 1 < nch) {
      store_a((ch + 1) & 1);
      store_b((ch + 1) & 1);
    }
    __syncthreads();
  }

  // ---- epilogue: ReLU -> bf16 via LDS -> 16-byte rows of the phase's output pixels ----
  uint16_t* sO = &sB[0][0];  // 128 x 136 bf16 = 34.8 KB, fits in buffer 0 (+1)
#pragma unroll
  for (int i = 0; i < SP_MI; ++i)
#pragma unroll
    for (int j = 0; j < SP_NJ; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = 32 * SP_MI * wm + 32 * i + (e >> 2) * 8 + h * 4 + (e & 3);
        const int col = 32 * SP_NJ * wn + 32 * j + r32;
        sO[row * SP_LDO + col] = f2bf(fmaxf(acc[i][j][e], 0.f));
      }
  __syncthreads();
  const int OH = 2 * PH, OW = 2 * PW;
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const int e = tid + 256 * u, row = e >> 4, cv = e & 15;
    const long long P = m0 + row;
    if (P >= Mp) continue;
    const int n = (int)(P / ((long long)PH * PW));
    const int rem = (int)(P - (long long)n * PH * PW);
    const int p = rem / PW, q = rem - p * PW;
    const long long o = (((long long)n * OH + 2 * p + a) * OW + 2 * q + b) * Ci + n0 + 8 * cv;
    *reinterpret_cast<u32x4*>(out + o) = *reinterpret_cast<const u32x4*>(&sO[row * SP_LDO + 8 * cv]);
  }
}

int sparse_unpool_conv_launch(const uint16_t* v, const uint8_t* code, const uint16_t* wt, uint16_t* out, int NB,
                              int PH, int PW, int C, int Ci, int code_div, hipStream_t s) {
  if (C % 16 || Ci % SP_BN || code_div <= 0 || NB % code_div || PW > SP_PX - SP_BM - 1) return -1;
  const long long Mp = (long long)NB * PH * PW;
  const long long gx = (Mp + SP_BM - 1) / SP_BM;
  if (gx > 0x7fffffffLL) return -1;
  hipLaunchKernelGGL(sparse_unpool_conv_kernel, dim3((unsigned)gx, Ci / SP_BN, 4), dim3(256), 0, s, v, code, wt, out,
                     NB, PH, PW, C, Ci, code_div);
  return (int)hipGetLastError();
}

}  // namespace dv
