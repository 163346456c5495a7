// Small gfx950 kernels around the conv core: filter selection, seeded first deconv step,
// mosaic deprocess, fused resize+preprocess, standalone pool/unpool.
#include <cstdlib>
#include "common.h"
#include "kernels.h"

#include <algorithm>

namespace dv {

// ---------------------------------------------------------------------------------------
// channel sums: sums[n][c] = sum_hw x[n][hw][c]   (reference: app/deepdream.py:369-380 sums
// each filter's activation map; here per image, fp32 accumulate of the stored bf16 map).
// One block per image; each thread owns 8 channels (one 16-B chunk) of a pixel group.
// ---------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) channel_sum_kernel(const uint16_t* __restrict__ x,
                                                          float* __restrict__ sums, int HW, int C) {
  __shared__ float red[256 * 8];
  const int n = blockIdx.x;
  const int cpp = C >> 3;                // chunks per pixel
  const int groups = 256 / cpp;          // pixel groups per block (C <= 2048)
  const int tid = threadIdx.x;
  const int chunk = tid % cpp, grp = tid / cpp;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (grp < groups) {
    const uint16_t* base = x + (long long)n * HW * C + chunk * 8;
    for (int p = grp; p < HW; p += groups) {
      const uint4 v = *reinterpret_cast<const uint4*>(base + (long long)p * C);
      acc[0] += to_f<DT>(v.x & 0xFFFF); acc[1] += to_f<DT>(v.x >> 16);
      acc[2] += to_f<DT>(v.y & 0xFFFF); acc[3] += to_f<DT>(v.y >> 16);
      acc[4] += to_f<DT>(v.z & 0xFFFF); acc[5] += to_f<DT>(v.z >> 16);
      acc[6] += to_f<DT>(v.w & 0xFFFF); acc[7] += to_f<DT>(v.w >> 16);
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[tid * 8 + e] = acc[e];
  __syncthreads();
  // deterministic ordered reduction over groups: thread t < C sums channel t
  for (int c = tid; c < C; c += 256) {
    const int ch = c >> 3, e = c & 7;
    float s = 0.f;
    for (int g = 0; g < groups; ++g) s += red[(g * cpp + ch) * 8 + e];
    sums[(long long)n * C + c] = s;
  }
}

int channel_sum_launch(const uint16_t* x, float* sums, int N, int HW, int C, int f16, hipStream_t s) {
  if (C % 8 != 0 || C > 2048 || N <= 0) return -1;
  if (f16) hipLaunchKernelGGL(channel_sum_kernel<DT_F16>, dim3(N), dim3(256), 0, s, x, sums, HW, C);
  else hipLaunchKernelGGL(channel_sum_kernel<DT_BF16>, dim3(N), dim3(256), 0, s, x, sums, HW, C);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Stable top-k of strictly positive values per row (reference: app/deepdream.py:369-380:
// keep sums > 0, sort descending with ties in ascending index order, take `top`).
// One wave per row; k rounds of (value desc, index asc) arg-max over the not-yet-taken set.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(64) topk_pos_kernel(const float* __restrict__ v, int* __restrict__ idx,
                                                      float* __restrict__ val, int C, int k) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* r = v + (long long)row * C;
  float last_v = INFINITY;
  int last_i = -1;
  for (int t = 0; t < k; ++t) {
    float bv = 0.f;  // must be > 0 to count
    int bi = -1;
    for (int c = lane; c < C; c += 64) {
      const float x = r[c];
      const bool after = (x < last_v) || (x == last_v && c > last_i);
      if (after && x > 0.f && (bi < 0 || x > bv || (x == bv && c < bi))) {
        bv = x;
        bi = c;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      const bool take = (oi >= 0) && (bi < 0 || ov > bv || (ov == bv && oi < bi));
      if (take) {
        bv = ov;
        bi = oi;
      }
    }
    if (lane == 0) {
      idx[(long long)row * k + t] = bi;
      val[(long long)row * k + t] = bi >= 0 ? bv : 0.f;
    }
    if (bi < 0) {
      for (int u = t + 1 + lane; u < k; u += 64) {
        idx[(long long)row * k + u] = -1;
        val[(long long)row * k + u] = 0.f;
      }
      break;
    }
    last_v = bv;
    last_i = bi;
  }
}

int topk_pos_launch(const float* v, int* idx, float* val, int N, int C, int k, hipStream_t s) {
  if (N <= 0 || k <= 0) return -1;
  hipLaunchKernelGGL(topk_pos_kernel, dim3(N), dim3(64), 0, s, v, idx, val, C, k);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Seeded first deconv step from a one-channel signal (the selected filter's map):
//   out[b][h][w][ci] = relu( sum_{kh,kw} S[b][h+kh-1][w+kw-1] * wt[f_b][kh][kw][ci] )
// with wt[f][kh][kw][ci] = W[2-kh][2-kw][ci][f] (flipped, in/out swapped Keras kernel,
// reference: app/deepdream.py:80-89). 1/C_out of the work of a dense conv-transpose.
// f_b < 0 (fewer positive filters than requested) produces a zero map.
// ---------------------------------------------------------------------------------------
// f_b is clamped to [-1, F) here (one ALU op; the host no longer runs a clamp launch). Index math is
// 32-bit (the launcher checks B*H*W*Cin/8 < 2^31): the 64-bit div/mod chain per 16-B chunk made this
// memory-bound kernel ALU-bound (141 us for 205 MB at block5, profiles/kseq_c2_r5.txt).
template <int DT>
__global__ void __launch_bounds__(256) seed_deconv3x3_kernel(const float* __restrict__ S,
                                                             const int* __restrict__ f,
                                                             const uint16_t* __restrict__ wt,
                                                             uint16_t* __restrict__ out, int B, int H,
                                                             int W, int Cin, int F) {
  const unsigned cpp = (unsigned)Cin >> 3;
  const unsigned total = (unsigned)B * H * W * cpp;
  for (unsigned g = blockIdx.x * 256u + threadIdx.x; g < total; g += gridDim.x * 256u) {
    const unsigned pix = g / cpp;
    const unsigned chunk = g - pix * cpp;
    const unsigned hw = (unsigned)H * W;
    const unsigned b = pix / hw;
    const unsigned r = pix - b * hw;
    const int h = (int)(r / (unsigned)W);
    const int w = (int)(r - (unsigned)h * W);
    const int fb = min(f[b], F - 1);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (fb >= 0) {
      // all 9 taps' S values and weight chunks are loaded before the first FMA (one memory round trip;
      // a zero-skip branch on each loaded S made every weight load wait for it). A wave is one pixel's
      // 64 chunks: the S loads are wave-uniform, the weight loads 1 KiB coalesced rows.
      const float* Sb = S + (size_t)b * hw;
      const uint16_t* wf = wt + (size_t)fb * 9 * Cin + chunk * 8;
      float sv[9];
      uint4 wv[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int ih = h + t / 3 - 1, iw = w + t % 3 - 1;
        sv[t] = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? Sb[ih * W + iw] : 0.f;
        wv[t] = *reinterpret_cast<const uint4*>(wf + t * Cin);
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        acc[0] += sv[t] * to_f<DT>(wv[t].x & 0xFFFF); acc[1] += sv[t] * to_f<DT>(wv[t].x >> 16);
        acc[2] += sv[t] * to_f<DT>(wv[t].y & 0xFFFF); acc[3] += sv[t] * to_f<DT>(wv[t].y >> 16);
        acc[4] += sv[t] * to_f<DT>(wv[t].z & 0xFFFF); acc[5] += sv[t] * to_f<DT>(wv[t].z >> 16);
        acc[6] += sv[t] * to_f<DT>(wv[t].w & 0xFFFF); acc[7] += sv[t] * to_f<DT>(wv[t].w >> 16);
      }
    }
    uint4 o;
    o.x = pack2<DT>(fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f));
    o.y = pack2<DT>(fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f));
    o.z = pack2<DT>(fmaxf(acc[4], 0.f), fmaxf(acc[5], 0.f));
    o.w = pack2<DT>(fmaxf(acc[6], 0.f), fmaxf(acc[7], 0.f));
    *reinterpret_cast<uint4*>(out + (size_t)g * 8) = o;
  }
}

// One workgroup per signal b for small maps (H*W <= 4096, e.g. block5's 14^2): the map S[b] is staged in
// LDS once, each thread keeps its chunk's 9 weight vectors in registers and walks the pixels (a group of
// Cin/8 lanes per pixel: 1 KiB coalesced stores at Cin = 512), so the per-pixel traffic is one LDS
// broadcast per tap instead of 9 weight rows from L1. Same taps in the same order as the kernel above.
constexpr int kSeedMaxHW = 4096;
template <int DT>
__global__ void __launch_bounds__(256) seed_deconv3x3_smallmap_kernel(const float* __restrict__ S,
                                                                      const int* __restrict__ f,
                                                                      const uint16_t* __restrict__ wt,
                                                                      uint16_t* __restrict__ out, int H, int W,
                                                                      int Cin, int F) {
  __shared__ float Ss[kSeedMaxHW];
  const int b = blockIdx.x, t = threadIdx.x;
  const int hw = H * W, cpp = Cin >> 3, groups = 256 / cpp;
  const int chunk = t % cpp, grp = t / cpp;
  const int fb = min(f[b], F - 1);
  const float* Sb = S + (size_t)b * hw;
  for (int i = t; i < hw; i += 256) Ss[i] = Sb[i];
  uint4 wv[9];
#pragma unroll
  for (int k = 0; k < 9; ++k)
    wv[k] = fb >= 0 ? *reinterpret_cast<const uint4*>(wt + ((size_t)fb * 9 + k) * Cin + chunk * 8) : make_uint4(0, 0, 0, 0);
  __syncthreads();
  if (grp >= groups) return;
  uint16_t* ob = out + (size_t)b * hw * Cin + chunk * 8;
  for (int pix = grp; pix < hw; pix += groups) {
    const int h = pix / W, w = pix - (pix / W) * W;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (fb >= 0) {
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        const int ih = h + k / 3 - 1, iw = w + k % 3 - 1;
        const float sv = ((unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W) ? Ss[ih * W + iw] : 0.f;
        acc[0] += sv * to_f<DT>(wv[k].x & 0xFFFF); acc[1] += sv * to_f<DT>(wv[k].x >> 16);
        acc[2] += sv * to_f<DT>(wv[k].y & 0xFFFF); acc[3] += sv * to_f<DT>(wv[k].y >> 16);
        acc[4] += sv * to_f<DT>(wv[k].z & 0xFFFF); acc[5] += sv * to_f<DT>(wv[k].z >> 16);
        acc[6] += sv * to_f<DT>(wv[k].w & 0xFFFF); acc[7] += sv * to_f<DT>(wv[k].w >> 16);
      }
    }
    uint4 o;
    o.x = pack2<DT>(fmaxf(acc[0], 0.f), fmaxf(acc[1], 0.f));
    o.y = pack2<DT>(fmaxf(acc[2], 0.f), fmaxf(acc[3], 0.f));
    o.z = pack2<DT>(fmaxf(acc[4], 0.f), fmaxf(acc[5], 0.f));
    o.w = pack2<DT>(fmaxf(acc[6], 0.f), fmaxf(acc[7], 0.f));
    *reinterpret_cast<uint4*>(ob + (size_t)pix * Cin) = o;
  }
}

int seed_deconv3x3_launch(const float* S, const int* f, const uint16_t* wt, uint16_t* out, int B, int H,
                          int W, int Cin, int F, int f16, hipStream_t s) {
  if (Cin % 8 != 0 || B <= 0 || F <= 0) return -1;
  const long long total = (long long)B * H * W * (Cin / 8);
  if (total >= (1LL << 31) || (long long)F * 9 * Cin >= (1LL << 31)) return -2;
  if ((long long)H * W <= kSeedMaxHW && Cin / 8 <= 256) {
    if (f16)
      hipLaunchKernelGGL(seed_deconv3x3_smallmap_kernel<DT_F16>, dim3((unsigned)B), dim3(256), 0, s, S, f, wt, out, H, W,
                         Cin, F);
    else
      hipLaunchKernelGGL(seed_deconv3x3_smallmap_kernel<DT_BF16>, dim3((unsigned)B), dim3(256), 0, s, S, f, wt, out, H,
                         W, Cin, F);
    return (int)hipGetLastError();
  }
  const long long blocks = std::min<long long>((total + 255) / 256, 256LL * 16);
  if (f16)
    hipLaunchKernelGGL(seed_deconv3x3_kernel<DT_F16>, dim3((unsigned)blocks), dim3(256), 0, s, S, f, wt, out, B, H, W,
                       Cin, F);
  else
    hipLaunchKernelGGL(seed_deconv3x3_kernel<DT_BF16>, dim3((unsigned)blocks), dim3(256), 0, s, S, f, wt, out, B, H, W,
                       Cin, F);
  return (int)hipGetLastError();
}

// Seed maps of the B*K backward chains (reference app/deepdream.py:450-465): S[b*K+k] is channel
// idx[b,k] of the target activation out4 [B, H, W, C] (16-bit), zero for idx < 0; mode 1 ('max')
// keeps only the positions equal to the map's max (mode 2: the max over the batch, for global
// top-k where all images share the filter); idx >= C reads as -1. With `code` (a max-pool target) the map is
// max-unpooled to [2H, 2W] with that pool's switch codes and clamped at 0 (the seed of the conv
// below the pool). One workgroup per chain: the 'max' reduction stays in the block.
template <int DT>
__global__ void __launch_bounds__(256) seed_map_kernel(const uint16_t* __restrict__ out4, const int* __restrict__ idx,
                                                       const uint8_t* __restrict__ code, float* __restrict__ S, int K,
                                                       int H, int W, int C, int mode) {
  const int bk = blockIdx.x, b = bk / K;
  const int f = idx[bk] < C ? idx[bk] : -1;
  const int HW = H * W;
  const uint16_t* ob = out4 + (long long)b * HW * C;
  __shared__ float red[4];
  float m = -INFINITY;
  if (mode != 0 && f >= 0) {
    // mode 2 ('max' with batch-global top-k: every image shares filter f) reduces over the batch
    const int b0 = mode == 2 ? 0 : b, b1 = mode == 2 ? (int)gridDim.x / K : b + 1;
    for (int bb = b0; bb < b1; ++bb) {
      const uint16_t* o2 = out4 + (long long)bb * HW * C;
      for (int p = threadIdx.x; p < HW; p += 256) m = fmaxf(m, to_f<DT>(o2[(long long)p * C + f]));
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  }
  if (code == nullptr) {
    float* Sb = S + (long long)bk * HW;
    for (int p = threadIdx.x; p < HW; p += 256) {
      float v = f >= 0 ? to_f<DT>(ob[(long long)p * C + f]) : 0.f;
      if (mode != 0 && v != m) v = 0.f;
      Sb[p] = v;
    }
    return;
  }
  const int W2 = 2 * W;
  float* Sb = S + (long long)bk * 4 * HW;
  const uint8_t* cb = code + (long long)b * HW * C;
  for (int q = threadIdx.x; q < 4 * HW; q += 256) {
    const int y = q / W2, x = q - y * W2;
    const long long p = (long long)(y >> 1) * W + (x >> 1);
    float v = 0.f;
    if (f >= 0 && cb[p * C + f] == (uint8_t)(((y & 1) << 1) | (x & 1))) {
      v = to_f<DT>(ob[p * C + f]);
      if (mode != 0 && v != m) v = 0.f;
      v = fmaxf(v, 0.f);
    }
    Sb[q] = v;
  }
}

int seed_map_launch(const uint16_t* out4, const int* idx, const uint8_t* code, float* S, int BK, int K, int H, int W,
                    int C, int mode, int f16, hipStream_t s) {
  if (BK <= 0 || K <= 0 || BK % K) return -1;
  if (f16)
    hipLaunchKernelGGL(seed_map_kernel<DT_F16>, dim3((unsigned)BK), dim3(256), 0, s, out4, idx, code, S, K, H, W, C, mode);
  else
    hipLaunchKernelGGL(seed_map_kernel<DT_BF16>, dim3((unsigned)BK), dim3(256), 0, s, out4, idx, code, S, K, H, W, C, mode);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Mosaic + deprocess (reference: app/main.py:67-72 + app/deepdream.py:483-498):
// the `tiles` reconstructions of one image form a 2x2 mosaic that is normalized as a whole:
//   x = (x - mean) / (std + 1e-7) * 0.1 + 0.5 ; clip[0,1] ; *255 ; clip ; truncate to u8.
// Mean/std are population statistics over the whole mosaic (two passes, fp64 block sums).
// reverse_channels writes channel c at slot 2-c (OpenCV BGR encoder semantics for an RGB
// encoder). One 1024-thread block per image.
// ---------------------------------------------------------------------------------------
__device__ double block_sum_d(double v, double* sh) {
  v = wave_sum_d(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) sh[wid] = v;
  __syncthreads();
  double r = 0.0;
  if (threadIdx.x < 64) {
    r = threadIdx.x < (blockDim.x >> 6) ? sh[threadIdx.x] : 0.0;
    r = wave_sum_d(r);
    if (threadIdx.x == 0) sh[0] = r;
  }
  __syncthreads();
  r = sh[0];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(1024) deprocess_mosaic_kernel(const float* __restrict__ recon,
                                                                uint8_t* __restrict__ out, int H, int W,
                                                                int tiles, int reverse) {
  __shared__ double sh[16];
  const int b = blockIdx.x;
  const long long per_tile = (long long)H * W * 3;
  const long long total = per_tile * tiles;
  const float* src = recon + (long long)b * total;
  const float4* src4 = reinterpret_cast<const float4*>(src);
  const long long n4 = total >> 2;  // total is a multiple of 4 (H*W*3*4)
  double s = 0.0;
  for (long long i = threadIdx.x; i < n4; i += 1024) {
    const float4 v = src4[i];
    s += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
  }
  const double mean_d = block_sum_d(s, sh) / (double)total;
  const float mean = (float)mean_d;
  double q = 0.0;
  for (long long i = threadIdx.x; i < n4; i += 1024) {
    const float4 v = src4[i];
    const double a0 = v.x - mean, a1 = v.y - mean, a2 = v.z - mean, a3 = v.w - mean;
    q += a0 * a0 + a1 * a1 + a2 * a2 + a3 * a3;
  }
  const float stdv = (float)sqrt(block_sum_d(q, sh) / (double)total);
  const float denom = stdv + 1e-7f;
  const int cols = 2;  // 2x2 mosaic, tile t at (t/2, t%2)
  const int OW = W * cols;
  uint8_t* o = out + (long long)b * (long long)H * ((tiles + cols - 1) / cols) * OW * 3;
  for (long long i = threadIdx.x; i < total; i += 1024) {
    const int t = (int)(i / per_tile);
    const long long r = i - t * per_tile;
    const int c = (int)(r % 3);
    const long long p = r / 3;
    const int x = (int)(p % W), y = (int)(p / W);
    float v = src[i];
    v = v - mean;
    v = v / denom;
    v = v * 0.1f;
    v = v + 0.5f;
    v = fminf(fmaxf(v, 0.f), 1.f);
    v = v * 255.f;
    v = fminf(fmaxf(v, 0.f), 255.f);
    const int oy = (t / cols) * H + y, ox = (t % cols) * W + x;
    const int oc = reverse ? 2 - c : c;
    o[((long long)oy * OW + ox) * 3 + oc] = (uint8_t)v;  // truncation, like ndarray.astype
  }
}

int deprocess_mosaic_launch(const float* recon, uint8_t* out, int B, int H, int W, int tiles, int reverse,
                            hipStream_t s) {
  if (B <= 0 || tiles <= 0 || tiles > 4) return -1;
  hipLaunchKernelGGL(deprocess_mosaic_kernel, dim3(B), dim3(1024), 0, s, recon, out, H, W, tiles, reverse);
  return (int)hipGetLastError();
}


// ---------------------------------------------------------------------------------------
// Single-pass deprocess (same arithmetic as deprocess_mosaic_kernel) from per-image statistics
// {sum, sum of squares} in fp64: a grid of 4-pixel quads instead of one block per image with three
// passes. The statistics come from the final conv-down's epilogue (conv3x3_c64_stream_kernel) or
// from recon_stats_kernel. Population variance = E[x^2] - mean^2 in fp64.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) recon_stats_kernel(const float* __restrict__ x, double* __restrict__ stats,
                                                          long long per_group, int blocks_per_group) {
  const int g = blockIdx.x / blocks_per_group, part = blockIdx.x % blocks_per_group;
  const float4* src = reinterpret_cast<const float4*>(x + (long long)g * per_group);
  const long long n4 = per_group >> 2;
  double s1 = 0.0, s2 = 0.0;
  for (long long i = (long long)part * 256 + threadIdx.x; i < n4; i += (long long)blocks_per_group * 256) {
    const float4 v = src[i];
    s1 += (double)v.x + (double)v.y + (double)v.z + (double)v.w;
    s2 += (double)v.x * v.x + (double)v.y * v.y + (double)v.z * v.z + (double)v.w * v.w;
  }
  if (part == 0 && threadIdx.x < (per_group & 3)) {  // tail elements
    const float v = x[(long long)g * per_group + (n4 << 2) + threadIdx.x];
    s1 += v;
    s2 += (double)v * v;
  }
  __shared__ double sh[16];
  s1 = wave_sum_d(s1);
  s2 = wave_sum_d(s2);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sh[wid] = s1;
    sh[8 + wid] = s2;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < 4; ++w) {
      a += sh[w];
      b += sh[8 + w];
    }
    atomicAdd(stats + 2 * g, a);
    atomicAdd(stats + 2 * g + 1, b);
  }
}

int recon_stats_launch(const float* x, double* stats, long long per_group, int groups, hipStream_t s) {
  if (groups <= 0 || per_group <= 0) return -1;
  const int bpg = (int)std::min<long long>(64, (per_group / 4 + 1023) / 1024);
  hipLaunchKernelGGL(recon_stats_kernel, dim3(groups * std::max(bpg, 1)), dim3(256), 0, s, x, stats, per_group,
                     std::max(bpg, 1));
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) deprocess_apply_kernel(const float* __restrict__ recon,
                                                              const double* __restrict__ stats,
                                                              uint8_t* __restrict__ out, int B, int H, int W,
                                                              int tiles, int reverse) {
  const int qpr = W >> 2;  // 4-pixel quads per row
  const long long total = (long long)B * tiles * H * qpr;
  for (long long q = blockIdx.x * 256LL + threadIdx.x; q < total; q += (long long)gridDim.x * 256) {
    const int xq = (int)(q % qpr);
    long long r = q / qpr;
    const int y = (int)(r % H);
    r /= H;
    const int t = (int)(r % tiles);
    const int b = (int)(r / tiles);
    const double cnt = (double)tiles * H * W * 3;
    const double mean_d = stats[2 * b] / cnt;
    const double var = fmax(stats[2 * b + 1] / cnt - mean_d * mean_d, 0.0);
    const float mean = (float)mean_d;
    const float denom = (float)sqrt(var) + 1e-7f;
    const float4* src = reinterpret_cast<const float4*>(recon + ((((long long)b * tiles + t) * H + y) * W + xq * 4) * 3);
    float v[12];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float4 f = src[k];
      v[4 * k] = f.x;
      v[4 * k + 1] = f.y;
      v[4 * k + 2] = f.z;
      v[4 * k + 3] = f.w;
    }
    uint8_t o[12];
#pragma unroll
    for (int e = 0; e < 12; ++e) {
      float x = v[e];
      x = x - mean;
      x = x / denom;
      x = x * 0.1f;
      x = x + 0.5f;
      x = fminf(fmaxf(x, 0.f), 1.f);
      x = x * 255.f;
      x = fminf(fmaxf(x, 0.f), 255.f);
      const int px = e / 3, c = e % 3;
      o[px * 3 + (reverse ? 2 - c : c)] = (uint8_t)x;
    }
    const int cols = 2, OW = W * cols;
    const long long oy = (long long)b * ((tiles + cols - 1) / cols) * H + (t / cols) * H + y;
    const long long ox = (long long)(t % cols) * W + xq * 4;
    uint32_t* dst = reinterpret_cast<uint32_t*>(out + (oy * OW + ox) * 3);
#pragma unroll
    for (int k = 0; k < 3; ++k)
      dst[k] = (uint32_t)o[4 * k] | ((uint32_t)o[4 * k + 1] << 8) | ((uint32_t)o[4 * k + 2] << 16) |
               ((uint32_t)o[4 * k + 3] << 24);
  }
}

int deprocess_apply_launch(const float* recon, const double* stats, uint8_t* out, int B, int H, int W, int tiles,
                           int reverse, hipStream_t s) {
  if (B <= 0 || tiles <= 0 || tiles > 4 || (W & 3)) return -1;
  const long long total = (long long)B * tiles * H * (W / 4);
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 256LL * 32);
  hipLaunchKernelGGL(deprocess_apply_kernel, dim3(grid), dim3(256), 0, s, recon, stats, out, B, H, W, tiles, reverse);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Fused resize + preprocess for one decoded RGB uint8 image (reference: app/main.py:53
// cv2.resize(img,(224,224)) INTER_LINEAR, then :60-61 img_to_array + preprocess_input).
// mode 0: OpenCV INTER_LINEAR fixed point (11-bit coefficients, half-pixel centres, edge
//         clamp; vertical pass as OpenCV's SIMD path: ((S0>>4)*b0>>16 + (S1>>4)*b1>>16 + 2)>>2)
// mode 1: OpenCV's exact-2x fast area path (INTER_LINEAR with integer scale 2 -> INTER_AREA)
// mode 2: same size copy
// Output slot c (c<3) = rgb[c] - mean[c], mean = (103.939, 116.779, 123.68): the RGB image
// is fed in the slot order the reference's BGR->reverse produced.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void lin_coef(int d, double scale, int ssize, int& s0, int& s1, int& a0, int& a1) {
  float fx = (float)((d + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= sx;
  if (sx < 0) {
    fx = 0.f;
    sx = 0;
  }
  if (sx >= ssize - 1) {
    fx = 0.f;
    sx = ssize - 1;
  }
  s0 = sx;
  s1 = sx + 1 < ssize ? sx + 1 : sx;
  a0 = __float2int_rn((1.f - fx) * 2048.f);
  a1 = __float2int_rn(fx * 2048.f);
}

// one output pixel (ox, oy) of the cv2-compatible resize of img [Hs, Ws, 3] u8
__device__ __forceinline__ void resize_px(const uint8_t* __restrict__ img, int Hs, int Ws, int OH, int OW, int ox, int oy,
                                          int mode, int (&px)[3]) {
  if (mode == 2) {
    for (int c = 0; c < 3; ++c) px[c] = img[((long long)oy * Ws + ox) * 3 + c];
  } else if (mode == 1) {
    const int sy = oy * 2, sx = ox * 2;
    for (int c = 0; c < 3; ++c) {
      const int s = img[((long long)sy * Ws + sx) * 3 + c] + img[((long long)sy * Ws + sx + 1) * 3 + c] +
                    img[((long long)(sy + 1) * Ws + sx) * 3 + c] + img[((long long)(sy + 1) * Ws + sx + 1) * 3 + c];
      px[c] = (s + 2) >> 2;
    }
  } else {
    int x0, x1, a0, a1, y0, y1, b0, b1;
    lin_coef(ox, (double)Ws / OW, Ws, x0, x1, a0, a1);
    lin_coef(oy, (double)Hs / OH, Hs, y0, y1, b0, b1);
    for (int c = 0; c < 3; ++c) {
      const int r0 = img[((long long)y0 * Ws + x0) * 3 + c] * a0 + img[((long long)y0 * Ws + x1) * 3 + c] * a1;
      const int r1 = img[((long long)y1 * Ws + x0) * 3 + c] * a0 + img[((long long)y1 * Ws + x1) * 3 + c] * a1;
      const int t0 = ((r0 >> 4) * b0) >> 16;
      const int t1 = ((r1 >> 4) * b1) >> 16;
      int v = (t0 + t1 + 2) >> 2;
      px[c] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
  }
}

// caffe preprocess of one pixel into Cpad 16-bit slots (slot c<3 = rgb[c] - mean[c], quirk Q1);
// DT: the engine's storage dtype (bf16 or fp16, Config.dtype)
template <int DT>
__device__ __forceinline__ void store_pre(uint16_t* __restrict__ o, const int (&px)[3], int Cpad) {
  const float mean[3] = {103.939f, 116.779f, 123.68f};
  if (Cpad == 8) {  // one 16-B store per pixel
    uint4 v;
    v.x = pack2<DT>((float)px[0] - mean[0], (float)px[1] - mean[1]);
    v.y = (uint32_t)from_f<DT>((float)px[2] - mean[2]);
    v.z = 0u;
    v.w = 0u;
    *reinterpret_cast<uint4*>(o) = v;
  } else {
    for (int c = 0; c < Cpad; ++c) o[c] = c < 3 ? from_f<DT>((float)px[c] - mean[c]) : (uint16_t)0;
  }
}

__device__ __forceinline__ void store_pre_dt(uint16_t* __restrict__ o, const int (&px)[3], int Cpad, int f16) {
  if (f16) store_pre<DT_F16>(o, px, Cpad);
  else store_pre<DT_BF16>(o, px, Cpad);
}

__global__ void __launch_bounds__(256) resize_preprocess_kernel(const uint8_t* __restrict__ img_b, int Hs, int Ws,
                                                                uint16_t* __restrict__ out_b, int OH, int OW,
                                                                int Cpad, int mode, int f16) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= OH * OW) return;
  const uint8_t* img = img_b + (long long)blockIdx.y * Hs * Ws * 3;
  uint16_t* out = out_b + (long long)blockIdx.y * OH * OW * Cpad;
  int px[3];
  resize_px(img, Hs, Ws, OH, OW, p % OW, p / OW, mode, px);
  store_pre_dt(out + (long long)p * Cpad, px, Cpad, f16);
}

int resize_preprocess_launch(const uint8_t* img, int B, int Hs, int Ws, uint16_t* out, int OH, int OW, int Cpad,
                             int mode, int f16, hipStream_t s) {
  if (Cpad < 3 || mode < 0 || mode > 2 || B <= 0) return -1;
  hipLaunchKernelGGL(resize_preprocess_kernel, dim3((OH * OW + 255) / 256, B), dim3(256), 0, s, img, Hs, Ws, out,
                     OH, OW, Cpad, mode, f16);
  return (int)hipGetLastError();
}

// Whole request batch in ONE launch: images of any sizes packed back to back in one u8 blob (one
// pinned staging slot, one H2D copy; runtime/staging.py), table[b] = {byte offset, Hs, Ws, mode}.
// fmt 0 / 2: preprocessed bf16 / fp16 [B, OH, OW, Cpad]; fmt 1: resized RGB u8 [B, OH, OW, 3]
// (the 150 KB/image form rank 0 scatters to the other GPUs; preprocess_u8 finishes it there).
__global__ void __launch_bounds__(256) resize_batch_kernel(const uint8_t* __restrict__ blob,
                                                           const long long* __restrict__ table, void* __restrict__ out,
                                                           int OH, int OW, int Cpad, int fmt) {
  const int p = blockIdx.x * 256 + threadIdx.x;
  if (p >= OH * OW) return;
  const long long* t = table + (long long)blockIdx.y * 4;
  int px[3];
  resize_px(blob + t[0], (int)t[1], (int)t[2], OH, OW, p % OW, p / OW, (int)t[3], px);
  const long long pix = (long long)blockIdx.y * OH * OW + p;
  if (fmt == 1) {
    uint8_t* o = reinterpret_cast<uint8_t*>(out) + pix * 3;
    o[0] = (uint8_t)px[0];
    o[1] = (uint8_t)px[1];
    o[2] = (uint8_t)px[2];
  } else {
    store_pre_dt(reinterpret_cast<uint16_t*>(out) + pix * Cpad, px, Cpad, fmt == 2);
  }
}

int resize_batch_launch(const uint8_t* blob, const long long* table, int B, void* out, int OH, int OW, int Cpad,
                        int fmt, hipStream_t s) {
  if (B <= 0 || B > 65535 || fmt < 0 || fmt > 2 || (fmt != 1 && Cpad < 3)) return -1;
  hipLaunchKernelGGL(resize_batch_kernel, dim3((OH * OW + 255) / 256, B), dim3(256), 0, s, blob, table, out, OH, OW,
                     Cpad, fmt);
  return (int)hipGetLastError();
}

// resized RGB u8 [P pixels, 3] -> preprocessed 16-bit [P, Cpad] (the scattered shard on a rank)
__global__ void __launch_bounds__(256) preprocess_u8_kernel(const uint8_t* __restrict__ in, uint16_t* __restrict__ out,
                                                            long long P, int Cpad, int f16) {
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < P; p += (long long)gridDim.x * 256) {
    const int px[3] = {in[p * 3], in[p * 3 + 1], in[p * 3 + 2]};
    store_pre_dt(out + p * Cpad, px, Cpad, f16);
  }
}

int preprocess_u8_launch(const uint8_t* in, uint16_t* out, long long P, int Cpad, int f16, hipStream_t s) {
  if (P <= 0 || Cpad < 3) return -1;
  const unsigned grid = (unsigned)std::min<long long>((P + 255) / 256, 256LL * 32);
  hipLaunchKernelGGL(preprocess_u8_kernel, dim3(grid), dim3(256), 0, s, in, out, P, Cpad, f16);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------
// Standalone 2x2/s2 max pool with first-max switch codes (reference: app/deepdream.py:152-188)
// and max-unpool to full resolution (reference: app/deepdream.py:191-209). The hot paths fuse
// both into the conv kernel; these serve pool-layer targets and tests.
// ---------------------------------------------------------------------------------------
template <int DT>
__global__ void __launch_bounds__(256) maxpool2x2_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out,
                                                         uint8_t* __restrict__ code, int N, int H, int W, int C) {
  const int PH = H >> 1, PW = W >> 1;
  const long long total = (long long)N * PH * PW * C;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total; g += (long long)gridDim.x * 256) {
    const int c = (int)(g % C);
    long long pix = g / C;
    const int pw = (int)(pix % PW);
    const int ph = (int)((pix / PW) % PH);
    const long long n = pix / ((long long)PW * PH);
    float best = -INFINITY;
    int bc = 0;
    for (int r = 0; r < 4; ++r) {
      const int ih = 2 * ph + (r >> 1), iw = 2 * pw + (r & 1);
      const float v = to_f<DT>(x[((n * H + ih) * W + iw) * C + c]);
      if (v > best) {
        best = v;
        bc = r;
      }
    }
    out[g] = from_f<DT>(best);
    code[g] = (uint8_t)bc;
  }
}

// Vectorized form (C % 8 == 0, 16-B aligned rows): one thread per (pooled pixel, 8-channel chunk), four
// 16-B window loads, one 16-B value store and one 8-B code store; 32-bit index math. The same first-max
// rule per channel as the scalar kernel (strict > over the window in (0,0), (0,1), (1,0), (1,1) order).
template <int DT>
__global__ void __launch_bounds__(256) maxpool2x2_vec_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ out,
                                                             uint8_t* __restrict__ code, int N, int H, int W, int C) {
  const unsigned PH = H >> 1, PW = W >> 1, cpp = (unsigned)C >> 3;
  const unsigned total = (unsigned)N * PH * PW * cpp;
  for (unsigned g = blockIdx.x * 256u + threadIdx.x; g < total; g += gridDim.x * 256u) {
    const unsigned pix = g / cpp, ch = g - pix * cpp;
    const unsigned pw = pix % PW, t = pix / PW;
    const unsigned ph = t % PH, n = t / PH;
    const uint16_t* x0 = x + ((size_t)(n * H + 2 * ph) * W + 2 * pw) * C + ch * 8;
    uint4 v[4];
    v[0] = *reinterpret_cast<const uint4*>(x0);
    v[1] = *reinterpret_cast<const uint4*>(x0 + C);
    v[2] = *reinterpret_cast<const uint4*>(x0 + (size_t)W * C);
    v[3] = *reinterpret_cast<const uint4*>(x0 + (size_t)W * C + C);
    uint32_t ob[4], cb[2] = {0u, 0u};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float best = -INFINITY;
      uint32_t bc = 0, bits = 0;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const uint32_t wd = (&v[r].x)[e >> 1];
        const uint32_t h16 = (e & 1) ? (wd >> 16) : (wd & 0xFFFFu);
        const float f = to_f<DT>(h16);
        if (f > best) {
          best = f;
          bc = r;
          bits = h16;
        }
      }
      if (bc == 0 && !(best > -INFINITY)) bits = from_f<DT>(best);  // nothing beat -inf: the scalar kernel's from_f<DT>(-inf)
      if (e & 1) ob[e >> 1] |= bits << 16;
      else ob[e >> 1] = bits;
      cb[e >> 2] |= bc << (8 * (e & 3));
    }
    *reinterpret_cast<uint4*>(out + (size_t)pix * C + ch * 8) = make_uint4(ob[0], ob[1], ob[2], ob[3]);
    *reinterpret_cast<uint2*>(code + (size_t)pix * C + ch * 8) = make_uint2(cb[0], cb[1]);
  }
}

int maxpool2x2_launch(const uint16_t* x, uint16_t* out, uint8_t* code, int N, int H, int W, int C, int f16,
                      hipStream_t s) {
  if ((H | W) & 1) return -1;
  const long long total = (long long)N * (H / 2) * (W / 2) * C;
  if (C % 8 == 0 && total / 8 < (1LL << 31) && (long long)N * H * W * C < (1LL << 32) &&
      !(reinterpret_cast<uintptr_t>(x) & 15) && !(reinterpret_cast<uintptr_t>(out) & 15) &&
      !(reinterpret_cast<uintptr_t>(code) & 7)) {
    const long long blocks = std::min<long long>((total / 8 + 255) / 256, 256LL * 32);
    if (f16)
      hipLaunchKernelGGL(maxpool2x2_vec_kernel<DT_F16>, dim3((unsigned)blocks), dim3(256), 0, s, x, out, code, N, H, W, C);
    else
      hipLaunchKernelGGL(maxpool2x2_vec_kernel<DT_BF16>, dim3((unsigned)blocks), dim3(256), 0, s, x, out, code, N, H, W, C);
    return (int)hipGetLastError();
  }
  const long long blocks = std::min<long long>((total + 255) / 256, 4096);
  if (f16) hipLaunchKernelGGL(maxpool2x2_kernel<DT_F16>, dim3((unsigned)blocks), dim3(256), 0, s, x, out, code, N, H, W, C);
  else hipLaunchKernelGGL(maxpool2x2_kernel<DT_BF16>, dim3((unsigned)blocks), dim3(256), 0, s, x, out, code, N, H, W, C);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(256) unpool2x2_kernel(const uint16_t* __restrict__ p, const uint8_t* __restrict__ code,
                                                        uint16_t* __restrict__ out, int N, int H, int W, int C,
                                                        int code_div, int relu) {
  const int PH = H >> 1, PW = W >> 1;
  const long long total = (long long)N * H * W * C;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total; g += (long long)gridDim.x * 256) {
    const int c = (int)(g % C);
    long long pix = g / C;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const long long n = pix / ((long long)W * H);
    const long long q = ((n * PH + (h >> 1)) * PW + (w >> 1)) * C + c;
    const long long qc = (((n / code_div) * PH + (h >> 1)) * PW + (w >> 1)) * C + c;
    uint16_t v = code[qc] == (((h & 1) << 1) | (w & 1)) ? p[q] : (uint16_t)0;
    if (relu && (v & 0x8000u)) v = 0;
    out[g] = v;
  }
}

// Vectorized unpool: one thread per (pooled pixel, 8-channel chunk): one 16-B pooled load, one
// 8-B code load, four 16-B stores (the 2x2 window); consecutive threads write consecutive chunks.
__global__ void __launch_bounds__(256) unpool2x2_vec_kernel(const uint16_t* __restrict__ p,
                                                            const uint8_t* __restrict__ code,
                                                            uint16_t* __restrict__ out, int N, int H, int W, int C,
                                                            int code_div, int relu) {
  const int PH = H >> 1, PW = W >> 1, cpp = C >> 3;
  const long long total = (long long)N * PH * PW * cpp;
  for (long long g = blockIdx.x * 256LL + threadIdx.x; g < total; g += (long long)gridDim.x * 256) {
    const int chunk = (int)(g % cpp);
    const long long pix = g / cpp;
    const int pw = (int)(pix % PW);
    const long long t = pix / PW;
    const int ph = (int)(t % PH);
    const long long n = t / PH;
    uint4 v = *reinterpret_cast<const uint4*>(p + pix * C + chunk * 8);
    if (relu) {
      v.x = relu_bf2(v.x);
      v.y = relu_bf2(v.y);
      v.z = relu_bf2(v.z);
      v.w = relu_bf2(v.w);
    }
    const long long cpix = ((n / code_div) * PH + ph) * PW + pw;
    const uint2 cd = *reinterpret_cast<const uint2*>(code + cpix * C + chunk * 8);
    const uint4 sp = unpool_spread(cd);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int h = 2 * ph + (s >> 1), w = 2 * pw + (s & 1);
      *reinterpret_cast<uint4*>(out + ((n * H + h) * W + w) * C + chunk * 8) = unpool_pick_s(v, sp, (uint32_t)s);
    }
  }
}

int unpool2x2_launch(const uint16_t* p, const uint8_t* code, uint16_t* out, int N, int H, int W, int C, int code_div,
                     int relu, hipStream_t s) {
  if (((H | W) & 1) || code_div <= 0) return -1;
  if (C % 8 == 0) {
    const long long total = (long long)N * (H / 2) * (W / 2) * (C / 8);
    const long long blocks = std::min<long long>((total + 255) / 256, 256LL * 32);
    hipLaunchKernelGGL(unpool2x2_vec_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, code, out, N, H, W, C,
                       code_div, relu);
    return (int)hipGetLastError();
  }
  const long long total = (long long)N * H * W * C;
  const long long blocks = std::min<long long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(unpool2x2_kernel, dim3((unsigned)blocks), dim3(256), 0, s, p, code, out, N, H, W, C, code_div,
                     relu);
  return (int)hipGetLastError();
}

}  // namespace dv

namespace dv {

// Row softmax for the classifier (predictions, 1000 classes): one 256-thread block per row, fp32,
// max-subtracted; the reference's DActivation softmax (app/deepdream.py:226-235).
__global__ void __launch_bounds__(256) softmax_rows_kernel(const float* __restrict__ x, float* __restrict__ y, int N) {
  __shared__ float red[4];
  const float* xr = x + (long long)blockIdx.x * N;
  float* yr = y + (long long)blockIdx.x * N;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < N; i += 256) m = fmaxf(m, xr[i]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  __syncthreads();
  float s = 0.f;
  for (int i = threadIdx.x; i < N; i += 256) s += __expf(xr[i] - m);
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  const float inv = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  for (int i = threadIdx.x; i < N; i += 256) yr[i] = __expf(xr[i] - m) * inv;
}

int softmax_rows_launch(const float* x, float* y, int M, int N, hipStream_t s) {
  if (M <= 0 || N <= 0) return -1;
  hipLaunchKernelGGL(softmax_rows_kernel, dim3((unsigned)M), dim3(256), 0, s, x, y, N);
  return (int)hipGetLastError();
}

// ---- RCCL all-gather interference model (bench.py --emulate-rccl-world) ----
// A collective's kernel occupies its channels' CUs for as long as the data takes to cross the links, not
// for the HBM time of a local copy (the round-4 D2D-copy emulation ran ~10x shorter than an xGMI transfer
// of the same bytes). `channels` workgroups (one per RCCL channel) copy `bytes` in 16-B vector chunks,
// each workgroup pacing itself against the 100 MHz wall clock so that the whole copy takes bytes /
// bytes_per_us microseconds: the model of an all-gather's receive side (its CUs busy, its bytes written
// to HBM) at a given link bandwidth, running beside the next step's compute on another stream.
__global__ void __launch_bounds__(256) paced_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                         long long n16, long long src16, double ticks_per_16b) {
  const long long per = (n16 + gridDim.x - 1) / gridDim.x;
  const long long lo = (long long)blockIdx.x * per, hi = min(n16, lo + per);
  const unsigned long long t0 = wall_clock64();
  constexpr int CHUNK = 256 * 8;  // 16-B elements per paced chunk (32 KiB)
  for (long long c = lo; c < hi; c += CHUNK) {
    // this chunk may start once the pace allows: (c - lo) elements at ticks_per_16b each
    const unsigned long long due = t0 + (unsigned long long)((double)(c - lo) * ticks_per_16b);
    for (int guard = 0; wall_clock64() < due && guard < (1 << 20); ++guard) __builtin_amdgcn_s_sleep(8);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const long long i = c + k * 256 + threadIdx.x;
      if (i < hi) dst[i] = src[i % src16];
    }
  }
}

int paced_copy_launch(const void* src, long long src_bytes, void* dst, long long bytes, int channels, double gbs,
                      hipStream_t s) {
  if (channels < 1 || channels > 1024 || bytes < 16 || src_bytes < 16 || gbs <= 0 ||
      (reinterpret_cast<uintptr_t>(src) & 15) || (reinterpret_cast<uintptr_t>(dst) & 15))
    return -1;
  const long long n16 = bytes / 16;
  const long long per = (n16 + channels - 1) / channels;
  // each workgroup moves `per` 16-B elements in bytes / gbs: ticks (100 MHz) per element
  const double total_us = (double)bytes / (gbs * 1e3);
  int dev = 0, khz = 100000;  // wall_clock64 rate (100 MHz on gfx9)
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
      khz <= 0)
    khz = 100000;
  const double ticks_per_16b = total_us * (khz / 1000.0) / (double)per;
  hipLaunchKernelGGL(paced_copy_kernel, dim3((unsigned)channels), dim3(256), 0, s, reinterpret_cast<const uint4*>(src),
                     reinterpret_cast<uint4*>(dst), n16, src_bytes / 16, ticks_per_16b);
  return (int)hipGetLastError();
}

}  // namespace dv
