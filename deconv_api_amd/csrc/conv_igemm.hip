// MFMA implicit-GEMM convolution for gfx950 (MI355X), NHWC bf16 in, fp32 accumulate.
//
// One kernel family serves every conv-shaped op of the framework:
//   * VGG16 forward conv3x3 + bias + ReLU, optionally with the 2x2 max-pool-with-switch
//     fused into the epilogue (reference: app/deepdream.py:99 conv up, :152-188 pooling);
//   * the deconvnet "down" conv (reference: app/deepdream.py:80-89,110 — a conv with the
//     spatially flipped, in/out-swapped kernel, zero bias and ReLU) with the max-unpooling
//     (reference: app/deepdream.py:191-209) fused into the A-operand gather;
//   * DeepDream input-gradients (dgrad) through ReLU (mask prologue) and strided convs
//     (transposed gather).
//
// GEMM view: M = output pixels, N = output channels, K = KH*KW*C.
// Tile: 256 threads = 4 waves, each wave owns (16*FM) x (16*FN) of C via
// v_mfma_f32_16x16x32_bf16. BK = 64: every LDS row is 128 B = 8 x 16-B chunks, stored with an
// XOR swizzle (chunk ^ (row & 7)) so the 16-lane ds_read_b128 groups of a fragment read are
// bank-conflict free. Register-staged double buffer: tile t+1 is fetched into VGPRs before the
// MFMAs of tile t and written to the other LDS buffer after them (one barrier per K-tile).
//
// POOL epilogue row order: m = (((n*PH+ph)*PW+pw) << 2) | (dy<<1 | dx). The 16x16 MFMA C
// layout gives every lane 4 consecutive rows of one column, i.e. one whole 2x2 window of one
// channel, so pooling + first-max switch selection happen in registers with no shuffles.
#include "common.h"
#include "kernels.h"

namespace dv {

constexpr int kBK = 64;

__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * 128 + ((chunk ^ (row & 7)) << 4);
}

template <int DT, int WM, int WN, int FM, int FN, int AMODE, int EPI, bool MASK_IN>
__global__ void __launch_bounds__(256, 2) conv_igemm_kernel(const ConvArgs a, int tiles_n) {
  constexpr int BM = WM * FM * 16;
  constexpr int BN = WN * FN * 16;
  constexpr int CPR = kBK / 8;             // 16-B chunks per LDS row
  constexpr int RPP = 256 / CPR;           // rows staged per pass of the block
  constexpr int A_CH = BM / RPP;           // A chunks per thread
  constexpr int B_CH = (BN + RPP - 1) / RPP;
  constexpr int A_BYTES = BM * kBK * 2;
  constexpr int B_BYTES = BN * kBK * 2;
  static_assert(BM % RPP == 0, "BM must be a multiple of 32");
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = wgid % tiles_n;
  const int tile_m = wgid / tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const int kc = tid & (CPR - 1);
  const int rbase = tid / CPR;

  const int H = a.H, W = a.W, C = a.C;
  const int PH = H >> 1, PW = W >> 1;  // UNPOOL source dims

  // ---- per-row gather state (rows fixed for the whole K loop) ----
  int r_n[A_CH], r_bh[A_CH], r_bw[A_CH];
  bool r_ok[A_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    const int gm = m0 + rbase + i * RPP;
    r_ok[i] = gm < a.M;
    const int g = r_ok[i] ? gm : 0;
    int n, oh, ow;
    if constexpr (EPI == CONV_E_POOL) {
      const int PWo = a.OW >> 1, PHo = a.OH >> 1;
      const int sub = g & 3;
      int pix = g >> 2;
      const int pw = pix % PWo;
      pix /= PWo;
      const int ph = pix % PHo;
      n = pix / PHo;
      oh = 2 * ph + (sub >> 1);
      ow = 2 * pw + (sub & 1);
    } else {
      ow = g % a.OW;
      const int t = g / a.OW;
      oh = t % a.OH;
      n = t / a.OH;
    }
    r_n[i] = n;
    if constexpr (AMODE == CONV_A_TRANSPOSE) {
      r_bh[i] = oh + a.pad_h;
      r_bw[i] = ow + a.pad_w;
    } else {
      r_bh[i] = oh * a.stride - a.pad_h;
      r_bw[i] = ow * a.stride - a.pad_w;
    }
  }

  // ---- this thread's K-chunk cursor: k = (kh*KW + kw)*C + c ----
  int c_cur, kw_cur, kh_cur;
  {
    const int k = kc * 8;
    const int tap = k / C;
    c_cur = k - tap * C;
    kh_cur = tap / a.KW;
    kw_cur = tap - kh_cur * a.KW;
  }

  uint4 ra[A_CH];
  uint4 rb[B_CH];

  auto load_a = [&](int kh, int kw, int c) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (r_ok[i] && kh < a.KH) {
        int ih, iw;
        bool inb;
        if constexpr (AMODE == CONV_A_TRANSPOSE) {
          const int th = r_bh[i] - kh, tw = r_bw[i] - kw;
          const int s = a.stride;
          inb = th >= 0 && tw >= 0 && (th % s) == 0 && (tw % s) == 0;
          ih = th / s;
          iw = tw / s;
          inb = inb && ih < H && iw < W;
        } else {
          ih = r_bh[i] + kh;
          iw = r_bw[i] + kw;
          inb = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
        }
        if (inb) {
          if constexpr (AMODE == CONV_A_UNPOOL) {
            const int ph = ih >> 1, pw = iw >> 1;
            const long long pix = ((long long)r_n[i] * PH + ph) * PW + pw;
            v = *reinterpret_cast<const uint4*>(a.x + pix * a.x_ld + c);
            const long long cpix = ((long long)(r_n[i] / a.code_div) * PH + ph) * PW + pw;
            const uint2 cd = *reinterpret_cast<const uint2*>(a.code + cpix * C + c);
            v = unpool_pick(v, cd, (uint32_t)(((ih & 1) << 1) | (iw & 1)));
          } else {
            const long long pix = ((long long)r_n[i] * H + ih) * W + iw;
            v = *reinterpret_cast<const uint4*>(a.x + pix * a.x_ld + c);
            if constexpr (MASK_IN) {
              const uint4 m = *reinterpret_cast<const uint4*>(a.mask + pix * a.mask_ld + c);
              v.x = mask_pos_bf2(v.x, m.x);
              v.y = mask_pos_bf2(v.y, m.y);
              v.z = mask_pos_bf2(v.z, m.z);
              v.w = mask_pos_bf2(v.w, m.w);
            }
          }
          if (a.relu_in) {
            v.x = relu_bf2(v.x);
            v.y = relu_bf2(v.y);
            v.z = relu_bf2(v.z);
            v.w = relu_bf2(v.w);
          }
        }
      }
      ra[i] = v;
    }
  };

  auto load_b = [&](int t) {
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int brow = rbase + i * RPP;
      if (brow < BN) {
        const uint16_t* p = a.w + (long long)(n0 + brow) * a.Kpad + t * kBK + kc * 8;
        rb[i] = *reinterpret_cast<const uint4*>(p);
      }
    }
  };

  auto store_tile = [&](int buf) {
    uint8_t* As = smem + buf * (A_BYTES + B_BYTES);
    uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int i = 0; i < A_CH; ++i)
      *reinterpret_cast<uint4*>(As + lds_off(rbase + i * RPP, kc)) = ra[i];
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      const int brow = rbase + i * RPP;
      if (brow < BN) *reinterpret_cast<uint4*>(Bs + lds_off(brow, kc)) = rb[i];
    }
  };

  auto advance = [&]() {
    c_cur += kBK;
    while (c_cur >= C) {
      c_cur -= C;
      if (++kw_cur == a.KW) {
        kw_cur = 0;
        ++kh_cur;
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = a.Kpad / kBK;
  load_a(kh_cur, kw_cur, c_cur);
  load_b(0);
  store_tile(0);
  __syncthreads();

  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    const bool more = (t + 1) < nk;
    if (more) {
      advance();
      load_a(kh_cur, kw_cur, c_cur);
      load_b(t + 1);
    }
    const uint8_t* As = smem + cur * (A_BYTES + B_BYTES);
    const uint8_t* Bs = As + A_BYTES;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      typedef typename Vec8<DT>::type v8;
      v8 af[FM], bfr[FN];
      const int chunk = s * 4 + (lane >> 4);
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const v8*>(As + lds_off(wm * FM * 16 + i * 16 + (lane & 15), chunk));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const v8*>(Bs + lds_off(wn * FN * 16 + j * 16 + (lane & 15), chunk));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = mfma16x16x32<DT>(af[i], bfr[j], acc[i][j]);
    }
    if (more) store_tile(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  const int row_l = (lane >> 4) * 4;
  const int col_l = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = n0 + wn * FN * 16 + j * 16 + col_l;
    if (col >= a.OC) continue;
    const float bias = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rowb = m0 + wm * FM * 16 + i * 16 + row_l;
      if constexpr (EPI == CONV_E_POOL) {
        if (rowb >= a.M) continue;
        float best = -INFINITY;
        int code = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          v = to_f<DT>(from_f<DT>(v));  // pool on the stored (bf16) values: ties resolve like the stored map
          if (v > best) {     // strict: first max in row-major window order wins
            best = v;
            code = r;
          }
        }
        const long long prow = rowb >> 2;
        reinterpret_cast<uint16_t*>(a.out)[prow * a.out_ld + col] = from_f<DT>(best);
        a.out_code[prow * a.OC + col] = (uint8_t)code;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rowb + r;
          if (row >= a.M) continue;
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          const long long o = (long long)row * a.out_ld + col;
          if constexpr (EPI == CONV_E_F32) {
            float* out = reinterpret_cast<float*>(a.out);
            if (a.accumulate) v += out[o];
            out[o] = v;
          } else {
            uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
            if (a.accumulate) v += to_f<DT>(out[o]);
            out[o] = from_f<DT>(v);
          }
        }
      }
    }
  }
}

template <int DT, int WM, int WN, int FM, int FN, int AMODE, int EPI, bool MASK_IN>
static int launch_cfg(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  const int tiles_m = (a.M + BM - 1) / BM;
  const int tiles_n = a.OCpad / BN;
  const long long nwg = (long long)tiles_m * tiles_n;
  if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL((conv_igemm_kernel<DT, WM, WN, FM, FN, AMODE, EPI, MASK_IN>), dim3((unsigned)nwg),
                     dim3(256), 0, s, a, tiles_n);
  return (int)hipGetLastError();
}

template <int DT, int AMODE, int EPI, bool MASK_IN>
static int launch_bn(const ConvArgs& a, hipStream_t s) {
  if (a.OCpad % 128 == 0 && a.OC > 64) return launch_cfg<DT, 2, 2, 4, 4, AMODE, EPI, MASK_IN>(a, s);
  if (a.OCpad % 64 == 0 && a.OC > 16) return launch_cfg<DT, 4, 1, 4, 4, AMODE, EPI, MASK_IN>(a, s);
  if (a.OCpad % 16 == 0) return launch_cfg<DT, 4, 1, 4, 1, AMODE, EPI, MASK_IN>(a, s);
  return -3;
}

int conv_igemm_launch(const ConvArgs& a, int amode, int epi, hipStream_t s) {
  const bool mask = a.mask != nullptr;
  if (a.C % 8 != 0 || a.Kpad % kBK != 0) return -4;
  if (a.dtype == DT_F16) {  // fp16 DeepDream: forward, and dgrad with/without the ReLU mask
    if (epi != CONV_E_BF16) return -1;
    if (amode == CONV_A_FWD)
      return mask ? launch_bn<DT_F16, CONV_A_FWD, CONV_E_BF16, true>(a, s)
                  : launch_bn<DT_F16, CONV_A_FWD, CONV_E_BF16, false>(a, s);
    if (amode == CONV_A_TRANSPOSE)
      return mask ? launch_bn<DT_F16, CONV_A_TRANSPOSE, CONV_E_BF16, true>(a, s)
                  : launch_bn<DT_F16, CONV_A_TRANSPOSE, CONV_E_BF16, false>(a, s);
    return -1;
  }
  if (amode == CONV_A_FWD) {
    if (epi == CONV_E_BF16) return mask ? launch_bn<DT_BF16, CONV_A_FWD, CONV_E_BF16, true>(a, s)
                                        : launch_bn<DT_BF16, CONV_A_FWD, CONV_E_BF16, false>(a, s);
    if (epi == CONV_E_POOL && !mask) return launch_bn<DT_BF16, CONV_A_FWD, CONV_E_POOL, false>(a, s);
    if (epi == CONV_E_F32) return mask ? launch_bn<DT_BF16, CONV_A_FWD, CONV_E_F32, true>(a, s)
                                       : launch_bn<DT_BF16, CONV_A_FWD, CONV_E_F32, false>(a, s);
  } else if (amode == CONV_A_UNPOOL && !mask) {
    if (epi == CONV_E_BF16) return launch_bn<DT_BF16, CONV_A_UNPOOL, CONV_E_BF16, false>(a, s);
    if (epi == CONV_E_F32) return launch_bn<DT_BF16, CONV_A_UNPOOL, CONV_E_F32, false>(a, s);
  } else if (amode == CONV_A_TRANSPOSE) {
    if (epi == CONV_E_BF16) return mask ? launch_bn<DT_BF16, CONV_A_TRANSPOSE, CONV_E_BF16, true>(a, s)
                                        : launch_bn<DT_BF16, CONV_A_TRANSPOSE, CONV_E_BF16, false>(a, s);
  }
  return -1;  // unsupported combination
}

}  // namespace dv
