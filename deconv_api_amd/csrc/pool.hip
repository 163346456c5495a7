// k x k pooling forward/backward for the DeepDream networks (InceptionV3 / ResNet-50), NHWC bf16,
// bf16 or fp16 (template DT), one thread per (pixel, 8-channel chunk): 16-B loads/stores throughout.
//   maxpool fwd: first-max (row-major) argmax kept as a uint8 window position per element;
//   maxpool bwd: gather form (no atomics): each input pixel sums the gradients of the (at most
//                ceil(k/s)^2) windows that contain it and chose it;
//   avgpool fwd/bwd: count_include_pad = false (TF/Keras 'same' semantics).
#include "common.h"
#include "kernels.h"

namespace dv {

struct PoolGeom {
  int N, H, W, C, OH, OW, k, s, pad;
  long long x_ld, y_ld;  // elements between consecutive pixels of the full-res (x / gx) and pooled (y / gy)
                         // maps: channel-slice views of concat buffers (InceptionV3 blocks)
  const float* bias;     // avgpool fwd: + bias[c] (the commuted 1x1 conv's bias), or null
  int relu;              // avgpool fwd: ReLU on the output
  int acc;               // backward: gx += (instead of =) the pooled gradient (Inception max branch)
  int generic;           // backward: the data-dependent window loop, not the unrolled 3x3 paths (A/B)
};

template <int DT, int KC, typename IT>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          uint8_t* __restrict__ idx, PoolGeom g) {
  const int cpp = g.C >> 3;
  const int k = KC ? KC : g.k;
  const IT total = (IT)g.N * g.OH * g.OW * cpp;
  for (IT t = (IT)blockIdx.x * 256 + threadIdx.x; t < total; t += (IT)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const IT pix = t / cpp;
    const int ow = (int)(pix % g.OW);
    const IT pq = pix / g.OW;
    const int oh = (int)(pq % g.OH);
    const long long n = (long long)(pq / g.OH);
    float best[8];
    int bi[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      bi[e] = 0;
    }
    // every tap loads from a clamped (in-bounds) pixel and out-of-window taps are skipped in the
    // reduction only, so an unrolled 3x3 window issues all 9 loads before the first use
#pragma unroll
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * g.s - g.pad + kh;
      const bool vh = (unsigned)ih < (unsigned)g.H;
      const int ihc = vh ? ih : (ih < 0 ? 0 : g.H - 1);
#pragma unroll
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * g.s - g.pad + kw;
        const bool vw = (unsigned)iw < (unsigned)g.W;
        const int iwc = vw ? iw : (iw < 0 ? 0 : g.W - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(x + ((n * g.H + ihc) * g.W + iwc) * g.x_ld + ch * 8);
        if (!(vh && vw)) continue;
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
        const int pos = kh * k + kw;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
          if (f > best[e]) {
            best[e] = f;
            bi[e] = pos;
          }
        }
      }
    }
    uint4 o;
    o.x = pack2<DT>(best[0], best[1]);
    o.y = pack2<DT>(best[2], best[3]);
    o.z = pack2<DT>(best[4], best[5]);
    o.w = pack2<DT>(best[6], best[7]);
    *reinterpret_cast<uint4*>(y + (long long)pix * g.y_ld + ch * 8) = o;
    uint2 ix;
    ix.x = (uint32_t)bi[0] | ((uint32_t)bi[1] << 8) | ((uint32_t)bi[2] << 16) | ((uint32_t)bi[3] << 24);
    ix.y = (uint32_t)bi[4] | ((uint32_t)bi[5] << 8) | ((uint32_t)bi[6] << 16) | ((uint32_t)bi[7] << 24);
    *reinterpret_cast<uint2*>(idx + (long long)pix * g.C + ch * 8) = ix;
  }
}

template <int DT, int KC, typename IT>
__global__ void __launch_bounds__(256) maxpool_bwd_kernel(const uint16_t* __restrict__ gy, const uint8_t* __restrict__ idx,
                                                          uint16_t* __restrict__ gx, PoolGeom g) {
  const int cpp = g.C >> 3;
  const int k = KC ? KC : g.k;
  const IT total = (IT)g.N * g.H * g.W * cpp;
  for (IT t = (IT)blockIdx.x * 256 + threadIdx.x; t < total; t += (IT)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const IT pix = t / cpp;
    const int w = (int)(pix % g.W);
    const IT pq = pix / g.W;
    const int h = (int)(pq % g.H);
    const long long n = (long long)(pq / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (KC == 3 && g.s == 2 && !g.generic) {
      // 3x3 / stride 2 (every InceptionV3 / ResNet-50 max pool): at most 2 x 2 windows contain
      // (h, w), oh in {ohh - 1, ohh}; all 8 loads are issued (clamped to a real window) before the
      // first use, and summed in the generic loop's (oh, ow) ascending order: bit-identical results
      const int ohh = (h + g.pad) >> 1, owh = (w + g.pad) >> 1;
      uint4 v[2][2];
      uint2 ix[2][2];
      uint32_t pos[2][2];
      bool ok[2][2];
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int oh = ohh - 1 + a, kh = ((h + g.pad) & 1) + 2 - 2 * a;
        const bool vh = oh >= 0 && oh < g.OH && kh < 3;
        const int ohc = oh < 0 ? 0 : (oh >= g.OH ? g.OH - 1 : oh);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const int ow = owh - 1 + b, kw = ((w + g.pad) & 1) + 2 - 2 * b;
          ok[a][b] = vh && ow >= 0 && ow < g.OW && kw < 3;
          const int owc = ow < 0 ? 0 : (ow >= g.OW ? g.OW - 1 : ow);
          pos[a][b] = (uint32_t)(kh * 3 + kw);
          const long long op = (n * g.OH + ohc) * g.OW + owc;
          v[a][b] = *reinterpret_cast<const uint4*>(gy + op * g.y_ld + ch * 8);
          ix[a][b] = *reinterpret_cast<const uint2*>(idx + op * g.C + ch * 8);
        }
      }
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          if (!ok[a][b]) continue;
          const uint32_t w4[4] = {v[a][b].x, v[a][b].y, v[a][b].z, v[a][b].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const uint32_t ie = ((e < 4 ? ix[a][b].x : ix[a][b].y) >> (8 * (e & 3))) & 0xFFu;
            if (ie == pos[a][b]) acc[e] += to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
          }
        }
    } else {
    // windows containing (h, w): oh*s - pad <= h <= oh*s - pad + k - 1
    const int oh_lo = max(0, (h + g.pad - k + g.s) / g.s), oh_hi = min(g.OH - 1, (h + g.pad) / g.s);
    const int ow_lo = max(0, (w + g.pad - k + g.s) / g.s), ow_hi = min(g.OW - 1, (w + g.pad) / g.s);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = h + g.pad - oh * g.s;
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = w + g.pad - ow * g.s;
        if (kw < 0 || kw >= k) continue;
        const uint32_t pos = (uint32_t)(kh * k + kw);
        const long long op = (n * g.OH + oh) * g.OW + ow;
        const uint4 v = *reinterpret_cast<const uint4*>(gy + op * g.y_ld + ch * 8);
        const uint2 ix = *reinterpret_cast<const uint2*>(idx + op * g.C + ch * 8);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ie = ((e < 4 ? ix.x : ix.y) >> (8 * (e & 3))) & 0xFFu;
          if (ie == pos) acc[e] += to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
        }
      }
    }
    }
    if (g.acc) {  // accumulate into the existing gradient (one pass instead of pool + add)
      const uint4 old = *reinterpret_cast<const uint4*>(gx + (long long)pix * g.x_ld + ch * 8);
      const uint32_t ov[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += to_f<DT>(ov[e] & 0xFFFFu);
        acc[2 * e + 1] += to_f<DT>(ov[e] >> 16);
      }
    }
    uint4 o;
    o.x = pack2<DT>(acc[0], acc[1]);
    o.y = pack2<DT>(acc[2], acc[3]);
    o.z = pack2<DT>(acc[4], acc[5]);
    o.w = pack2<DT>(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(gx + (long long)pix * g.x_ld + ch * 8) = o;
  }
}

__device__ __forceinline__ int win_count(int o, int s, int pad, int k, int L) {
  const int lo = max(0, o * s - pad), hi = min(L - 1, o * s - pad + k - 1);
  return hi - lo + 1;
}

template <int DT, int KC, typename IT>
__global__ void __launch_bounds__(256) avgpool_fwd_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ y,
                                                          PoolGeom g) {
  const int cpp = g.C >> 3;
  const int k = KC ? KC : g.k;
  const IT total = (IT)g.N * g.OH * g.OW * cpp;
  for (IT t = (IT)blockIdx.x * 256 + threadIdx.x; t < total; t += (IT)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const IT pix = t / cpp;
    const int ow = (int)(pix % g.OW);
    const IT pq = pix / g.OW;
    const int oh = (int)(pq % g.OH);
    const long long n = (long long)(pq / g.OH);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int kh = 0; kh < k; ++kh) {
      const int ih = oh * g.s - g.pad + kh;
      const bool vh = (unsigned)ih < (unsigned)g.H;
      const int ihc = vh ? ih : (ih < 0 ? 0 : g.H - 1);
#pragma unroll
      for (int kw = 0; kw < k; ++kw) {
        const int iw = ow * g.s - g.pad + kw;
        const bool vw = (unsigned)iw < (unsigned)g.W;
        const int iwc = vw ? iw : (iw < 0 ? 0 : g.W - 1);
        const uint4 v = *reinterpret_cast<const uint4*>(x + ((n * g.H + ihc) * g.W + iwc) * g.x_ld + ch * 8);
        if (!(vh && vw)) continue;  // clamped load above: all loads of the window issue up front
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
      }
    }
    const float inv = 1.f / (float)(win_count(oh, g.s, g.pad, k, g.H) * win_count(ow, g.s, g.pad, k, g.W));
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      acc[e] = acc[e] * inv + (g.bias ? g.bias[ch * 8 + e] : 0.f);
      if (g.relu) acc[e] = fmaxf(acc[e], 0.f);
    }
    uint4 o;
    o.x = pack2<DT>(acc[0], acc[1]);
    o.y = pack2<DT>(acc[2], acc[3]);
    o.z = pack2<DT>(acc[4], acc[5]);
    o.w = pack2<DT>(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(y + (long long)pix * g.y_ld + ch * 8) = o;
  }
}

template <int DT, int KC, typename IT>
__global__ void __launch_bounds__(256) avgpool_bwd_kernel(const uint16_t* __restrict__ gy, uint16_t* __restrict__ gx,
                                                          PoolGeom g) {
  const int cpp = g.C >> 3;
  const int k = KC ? KC : g.k;
  const IT total = (IT)g.N * g.H * g.W * cpp;
  for (IT t = (IT)blockIdx.x * 256 + threadIdx.x; t < total; t += (IT)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const IT pix = t / cpp;
    const int w = (int)(pix % g.W);
    const IT pq = pix / g.W;
    const int h = (int)(pq % g.H);
    const long long n = (long long)(pq / g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (KC == 3 && g.s == 1 && !g.generic) {
      // 3x3 / stride 1 (the InceptionV3 pool branches): the windows containing (h, w) are
      // oh = h + pad - 2 .. h + pad; all 9 loads issue (clamped) before the first use, summed in the
      // generic loop's ascending (oh, ow) order with the same per-window divisor: bit-identical
      uint4 v[3][3];
      bool ok[3][3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        const int oh = h + g.pad - 2 + a;
        const int ohc = oh < 0 ? 0 : (oh >= g.OH ? g.OH - 1 : oh);
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          const int ow = w + g.pad - 2 + b;
          const int owc = ow < 0 ? 0 : (ow >= g.OW ? g.OW - 1 : ow);
          ok[a][b] = (unsigned)oh < (unsigned)g.OH && (unsigned)ow < (unsigned)g.OW;
          v[a][b] = *reinterpret_cast<const uint4*>(gy + ((n * g.OH + ohc) * g.OW + owc) * g.y_ld + ch * 8);
        }
      }
#pragma unroll
      for (int a = 0; a < 3; ++a)
#pragma unroll
        for (int b = 0; b < 3; ++b) {
          if (!ok[a][b]) continue;
          const int oh = h + g.pad - 2 + a, ow = w + g.pad - 2 + b;
          const float inv = 1.f / (float)(win_count(oh, 1, g.pad, 3, g.H) * win_count(ow, 1, g.pad, 3, g.W));
          const uint32_t w4[4] = {v[a][b].x, v[a][b].y, v[a][b].z, v[a][b].w};
#pragma unroll
          for (int e = 0; e < 8; ++e) acc[e] += inv * to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
        }
    } else {
    const int oh_lo = max(0, (h + g.pad - k + g.s) / g.s), oh_hi = min(g.OH - 1, (h + g.pad) / g.s);
    const int ow_lo = max(0, (w + g.pad - k + g.s) / g.s), ow_hi = min(g.OW - 1, (w + g.pad) / g.s);
    for (int oh = oh_lo; oh <= oh_hi; ++oh) {
      const int kh = h + g.pad - oh * g.s;
      if (kh < 0 || kh >= k) continue;
      for (int ow = ow_lo; ow <= ow_hi; ++ow) {
        const int kw = w + g.pad - ow * g.s;
        if (kw < 0 || kw >= k) continue;
        const float inv = 1.f / (float)(win_count(oh, g.s, g.pad, k, g.H) * win_count(ow, g.s, g.pad, k, g.W));
        const uint4 v = *reinterpret_cast<const uint4*>(gy + ((n * g.OH + oh) * g.OW + ow) * g.y_ld + ch * 8);
        const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[e] += inv * to_f<DT>((w4[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
      }
    }
    }
    if (g.acc) {  // accumulate into the existing gradient (one pass instead of pool + add)
      const uint4 old = *reinterpret_cast<const uint4*>(gx + (long long)pix * g.x_ld + ch * 8);
      const uint32_t ov[4] = {old.x, old.y, old.z, old.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        acc[2 * e] += to_f<DT>(ov[e] & 0xFFFFu);
        acc[2 * e + 1] += to_f<DT>(ov[e] >> 16);
      }
    }
    uint4 o;
    o.x = pack2<DT>(acc[0], acc[1]);
    o.y = pack2<DT>(acc[2], acc[3]);
    o.z = pack2<DT>(acc[4], acc[5]);
    o.w = pack2<DT>(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(gx + (long long)pix * g.x_ld + ch * 8) = o;
  }
}

// Input gradient of a stride-s 1x1 conv (pad 0) from its GEMM result E [N, OH, OW, C]:
// gx[n, h, w] = E[n, h/s, w/s] where h, w are multiples of s, else 0; optionally zeroed where
// emask[n, h, w] <= 0 (the ReLU of the layer that produced the conv's input). Writes all of gx:
// replaces a zero fill, a strided copy per sub-pixel class, an add and a mask pass
// (ops/autograd.py:_BottleneckFn, ResNet-50's stride-2 stage heads).
template <int DT>
__global__ void __launch_bounds__(256) subpixel_scatter_kernel(const uint16_t* __restrict__ E,
                                                               const uint16_t* __restrict__ emask,
                                                               uint16_t* __restrict__ gx, int N, int H, int W, int C,
                                                               int OH, int OW, int s) {
  const int cpp = C >> 3;
  const long long total = (long long)N * H * W * cpp;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const long long pix = t / cpp;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const long long n = pix / ((long long)W * H);
    uint4 o = {0u, 0u, 0u, 0u};
    if (h % s == 0 && w % s == 0 && h / s < OH && w / s < OW) {
      o = *reinterpret_cast<const uint4*>(E + ((n * OH + h / s) * OW + w / s) * C + ch * 8);
      if (emask) {
        const uint4 m = *reinterpret_cast<const uint4*>(emask + pix * C + ch * 8);
        uint32_t ov[4] = {o.x, o.y, o.z, o.w};
        const uint32_t mv[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = to_f<DT>(mv[e] & 0xFFFFu), hi = to_f<DT>(mv[e] >> 16);
          ov[e] = (lo > 0.f ? (ov[e] & 0xFFFFu) : 0u) | (hi > 0.f ? (ov[e] & 0xFFFF0000u) : 0u);
        }
        o = uint4{ov[0], ov[1], ov[2], ov[3]};
      }
    }
    *reinterpret_cast<uint4*>(gx + pix * C + ch * 8) = o;
  }
}

// Sub-pixel merge (strided-conv input gradient assembled from its s x s parity classes, s <= 2): gx[n][h][w]
// = part[(h % s) * s + w % s][n][h / s][w / s] (zero for a missing class), optionally += the old gx, then
// zeroed where emask <= 0 - one pass instead of s^2 strided copies + an add + a threshold pass.
struct SubpixelParts {
  const uint16_t* p[4];
  int hc[4], wc[4], ld[4];
};

template <int DT>
__global__ void __launch_bounds__(256) subpixel_merge_kernel(const SubpixelParts parts, const uint16_t* __restrict__ emask,
                                                             uint16_t* __restrict__ gx, int N, int H, int W, int C, int s,
                                                             int acc) {
  const int cpp = C >> 3;
  const long long total = (long long)N * H * W * cpp;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const long long pix = t / cpp;
    const int w = (int)(pix % W);
    const int h = (int)((pix / W) % H);
    const long long n = pix / ((long long)W * H);
    const int k = (h % s) * s + (w % s);
    uint4 o = {0u, 0u, 0u, 0u};
    const uint16_t* src = parts.p[k];
    if (src != nullptr) {
      const long long q = ((n * parts.hc[k] + h / s) * parts.wc[k] + w / s) * parts.ld[k] + ch * 8;
      o = *reinterpret_cast<const uint4*>(src + q);
    }
    uint32_t ov[4] = {o.x, o.y, o.z, o.w};
    if (acc) {
      const uint4 g = *reinterpret_cast<const uint4*>(gx + pix * C + ch * 8);
      const uint32_t gv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        ov[e] = pack2<DT>(to_f<DT>(ov[e] & 0xFFFFu) + to_f<DT>(gv[e] & 0xFFFFu), to_f<DT>(ov[e] >> 16) + to_f<DT>(gv[e] >> 16));
    }
    if (emask) {
      const uint4 m = *reinterpret_cast<const uint4*>(emask + pix * C + ch * 8);
      const uint32_t mv[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = to_f<DT>(mv[e] & 0xFFFFu), hi = to_f<DT>(mv[e] >> 16);
        ov[e] = (lo > 0.f ? (ov[e] & 0xFFFFu) : 0u) | (hi > 0.f ? (ov[e] & 0xFFFF0000u) : 0u);
      }
    }
    *reinterpret_cast<uint4*>(gx + pix * C + ch * 8) = uint4{ov[0], ov[1], ov[2], ov[3]};
  }
}

static unsigned grid_for(long long total) {
  return (unsigned)std::min<long long>((total + 255) / 256, 256LL * 32);
}

template <int DT, int KC, typename IT>
static int pool_dt_k(int kind, int dir, const uint16_t* in, uint16_t* out, uint8_t* idx, const PoolGeom& g,
                     hipStream_t st) {
  const long long out_total = (long long)g.N * g.OH * g.OW * (g.C / 8), in_total = (long long)g.N * g.H * g.W * (g.C / 8);
  if (kind == 0 && dir == 0)
    hipLaunchKernelGGL((maxpool_fwd_kernel<DT, KC, IT>), dim3(grid_for(out_total)), dim3(256), 0, st, in, out, idx, g);
  else if (kind == 0 && dir == 1)
    hipLaunchKernelGGL((maxpool_bwd_kernel<DT, KC, IT>), dim3(grid_for(in_total)), dim3(256), 0, st, in, idx, out, g);
  else if (kind == 1 && dir == 0)
    hipLaunchKernelGGL((avgpool_fwd_kernel<DT, KC, IT>), dim3(grid_for(out_total)), dim3(256), 0, st, in, out, g);
  else if (kind == 1 && dir == 1)
    hipLaunchKernelGGL((avgpool_bwd_kernel<DT, KC, IT>), dim3(grid_for(in_total)), dim3(256), 0, st, in, out, g);
  else
    return -2;
  return (int)hipGetLastError();
}

// 3x3 windows (every pool of InceptionV3 / ResNet-50) unroll with all loads in flight; 32-bit index
// math whenever the thread count fits (64-bit divisions cost ~100 instructions each per thread)
template <int DT>
static int pool_dt(int kind, int dir, const uint16_t* in, uint16_t* out, uint8_t* idx, const PoolGeom& g,
                   hipStream_t st) {
  const long long big = std::max((long long)g.N * g.OH * g.OW, (long long)g.N * g.H * g.W) * (g.C / 8) + 256LL * 32 * 256;
  const bool i32 = big < 0x7FFFFFFFLL;
  if (g.k == 3 && i32) return pool_dt_k<DT, 3, int>(kind, dir, in, out, idx, g, st);
  if (i32) return pool_dt_k<DT, 0, int>(kind, dir, in, out, idx, g, st);
  return pool_dt_k<DT, 0, long long>(kind, dir, in, out, idx, g, st);
}

int subpixel_scatter_launch(const uint16_t* E, const uint16_t* emask, uint16_t* gx, int N, int H, int W, int C, int OH,
                            int OW, int s, int dtype, hipStream_t st) {
  if (C % 8 != 0 || s < 1) return -1;
  const unsigned grid = grid_for((long long)N * H * W * (C / 8));
  if (dtype == DT_F16)
    hipLaunchKernelGGL(subpixel_scatter_kernel<DT_F16>, dim3(grid), dim3(256), 0, st, E, emask, gx, N, H, W, C, OH, OW, s);
  else
    hipLaunchKernelGGL(subpixel_scatter_kernel<DT_BF16>, dim3(grid), dim3(256), 0, st, E, emask, gx, N, H, W, C, OH, OW, s);
  return (int)hipGetLastError();
}

int subpixel_merge_launch(const uint16_t* const* p, const int* hc, const int* wc, const int* ld, const uint16_t* emask,
                          uint16_t* gx, int N, int H, int W, int C, int s, int acc, int dtype, hipStream_t st) {
  if (C % 8 != 0 || s < 1 || s > 2) return -1;
  SubpixelParts parts{};
  for (int k = 0; k < s * s; ++k) {
    parts.p[k] = p[k];
    parts.hc[k] = hc[k];
    parts.wc[k] = wc[k];
    parts.ld[k] = ld[k];
    if (p[k] != nullptr && (ld[k] % 8 != 0 || ld[k] < C)) return -1;
  }
  const unsigned grid = grid_for((long long)N * H * W * (C / 8));
  if (dtype == DT_F16)
    hipLaunchKernelGGL(subpixel_merge_kernel<DT_F16>, dim3(grid), dim3(256), 0, st, parts, emask, gx, N, H, W, C, s, acc);
  else
    hipLaunchKernelGGL(subpixel_merge_kernel<DT_BF16>, dim3(grid), dim3(256), 0, st, parts, emask, gx, N, H, W, C, s, acc);
  return (int)hipGetLastError();
}

int pool_launch(int kind, int dir, const uint16_t* in, uint16_t* out, uint8_t* idx, int N, int H, int W, int C, int OH,
                int OW, int k, int s, int pad, int dtype, hipStream_t st, long long x_ld, long long y_ld,
                const float* bias, int relu, int acc) {
  if (C % 8 != 0 || k <= 0 || s <= 0 || k > 15) return -1;
  if (x_ld <= 0) x_ld = C;
  if (y_ld <= 0) y_ld = C;
  if (x_ld % 8 || y_ld % 8 || x_ld < C || y_ld < C) return -1;
  if (acc && dir != 1) return -1;
  // DV_NO_POOL_UNROLL=1 (read per call): backward passes on the generic window loop (A/B, bit-identity tests)
  const int generic = dv_ab_env("DV_NO_POOL_UNROLL") != nullptr;
  const PoolGeom g{N, H, W, C, OH, OW, k, s, pad, x_ld, y_ld, bias, relu, acc, generic};
  return dtype == DT_F16 ? pool_dt<DT_F16>(kind, dir, in, out, idx, g, st)
                         : pool_dt<DT_BF16>(kind, dir, in, out, idx, g, st);
}

}  // namespace dv
