// DeepDream loss kernels (engine/deepdream.py): per-image sum of squares over the activation
// "core" (the map without a `b`-pixel border, the Keras example's act[:, 2:-2, 2:-2, :]) and its
// input gradient. NHWC bf16/fp16, 16-B vector loads, fp32 accumulation, deterministic (block
// partials, summed by the caller in a fixed order; no atomics).
#include "common.h"
#include "kernels.h"

namespace dv {

template <int DT>
__global__ void __launch_bounds__(256) sumsq_core_kernel(const uint16_t* __restrict__ x, float* __restrict__ part,
                                                         int H, int W, int C, int b) {
  const int n = blockIdx.y;
  const int Hc = H - 2 * b, Wc = W - 2 * b, cpp = C >> 3;
  const long long total = (long long)Hc * Wc * cpp;
  const uint16_t* xn = x + (long long)n * H * W * C;
  float acc = 0.f;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int ch = (int)(t % cpp);
    const long long pix = t / cpp;
    const int hh = (int)(pix / Wc) + b, ww = (int)(pix % Wc) + b;
    const uint4 v = *reinterpret_cast<const uint4*>(xn + ((long long)hh * W + ww) * C + ch * 8);
    const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float lo = to_f<DT>(w4[e] & 0xFFFFu), hi = to_f<DT>(w4[e] >> 16);
      acc += lo * lo + hi * hi;
    }
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// gx = 2 * scale[n] * x inside the core, 0 on the border
template <int DT>
__global__ void __launch_bounds__(256) sumsq_core_bwd_kernel(const uint16_t* __restrict__ x,
                                                             const float* __restrict__ scale,
                                                             const uint16_t* __restrict__ addend,
                                                             uint16_t* __restrict__ gx, int N, int H, int W, int C,
                                                             int b) {
  const int cpp = C >> 3;
  const long long total = (long long)N * H * W * cpp;
  for (long long t = blockIdx.x * 256LL + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const long long pix = t / cpp;
    const int ww = (int)(pix % W);
    const int hh = (int)((pix / W) % H);
    const int n = (int)(pix / ((long long)W * H));
    const bool core = hh >= b && hh < H - b && ww >= b && ww < W - b;
    // addend (the gradient flowing back from the layers above a loss tap): gx = addend + loss grad
    uint4 o = addend ? *reinterpret_cast<const uint4*>(addend + t * 8) : uint4{0u, 0u, 0u, 0u};
    if (core) {
      const float s2 = 2.f * scale[n];
      const uint4 v = *reinterpret_cast<const uint4*>(x + t * 8);
      const uint32_t vi[4] = {v.x, v.y, v.z, v.w};
      uint32_t oi[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        oi[e] = pack2<DT>(s2 * to_f<DT>(vi[e] & 0xFFFFu) + to_f<DT>(oi[e] & 0xFFFFu),
                          s2 * to_f<DT>(vi[e] >> 16) + to_f<DT>(oi[e] >> 16));
      o = uint4{oi[0], oi[1], oi[2], oi[3]};
    }
    *reinterpret_cast<uint4*>(gx + t * 8) = o;
  }
}

// The same gradient fused with the loss itself: block (p, n) of a (parts, N) grid walks image n's
// elements, writes gx = addend + 2 scale[n] x (core) / addend (border), and its fp32 partial sum of
// x^2 over the core to part[n][p] - the forward sumsq_core launch of every loss layer disappears
// (the loss is consumed only by the update after the backward). Same partial layout as sumsq_core.
template <int DT>
__global__ void __launch_bounds__(256) sumsq_core_fused_kernel(const uint16_t* __restrict__ x,
                                                               const float* __restrict__ scale,
                                                               const uint16_t* __restrict__ addend,
                                                               uint16_t* __restrict__ gx, float* __restrict__ part,
                                                               int H, int W, int C, int b) {
  const int n = blockIdx.y;
  const int cpp = C >> 3;
  const int total = H * W * cpp;
  const long long base = (long long)n * total;
  const float s2 = 2.f * scale[n];
  float acc = 0.f;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const int pix = t / cpp;
    const int ww = pix % W, hh = pix / W;
    const bool core = hh >= b && hh < H - b && ww >= b && ww < W - b;
    uint4 o = addend ? *reinterpret_cast<const uint4*>(addend + (base + t) * 8) : uint4{0u, 0u, 0u, 0u};
    if (core) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + (base + t) * 8);
      const uint32_t vi[4] = {v.x, v.y, v.z, v.w};
      uint32_t oi[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float lo = to_f<DT>(vi[e] & 0xFFFFu), hi = to_f<DT>(vi[e] >> 16);
        acc += lo * lo + hi * hi;
        oi[e] = pack2<DT>(s2 * lo + to_f<DT>(oi[e] & 0xFFFFu), s2 * hi + to_f<DT>(oi[e] >> 16));
      }
      o = uint4{oi[0], oi[1], oi[2], oi[3]};
    }
    *reinterpret_cast<uint4*>(gx + (base + t) * 8) = o;
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// ---- fused DeepDream step tail (engine/deepdream.py:DeepDream._fused_step) ----
// part[n][p] = sum of |g| over channels 0..2 of the network-input gradient g [N, H, W, 8]
template <int DT>
__global__ void __launch_bounds__(256) absmean_part_kernel(const uint16_t* __restrict__ g, float* __restrict__ part,
                                                           int HW) {
  const int n = blockIdx.y;
  const uint16_t* gn = g + (long long)n * HW * 8;
  float acc = 0.f;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    const uint2 v = *reinterpret_cast<const uint2*>(gn + (long long)p * 8);  // channels 0..3
    acc += fabsf(to_f<DT>(v.x & 0xFFFFu)) + fabsf(to_f<DT>(v.x >> 16)) + fabsf(to_f<DT>(v.y & 0xFFFFu));
  }
  __shared__ float red[4];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[(long long)n * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// One gradient-ascent update, per image n (blockIdx.y):
//   loss[n] = sum_l lcoef[l] * sum_p lpart[l][n][p]            (the DeepDream loss)
//   done[n] |= loss[n] > max_loss (max_loss < 0: disabled)      (device-side max_loss early stop)
//   x[n] += step * (!done[n]) * g[n] / max(mean |g[n]|, 1e-7)   (fp32 master image, 3 channels)
//   xin[n] = (x[n], 0, 0, 0, 0, 0) in the 16-bit network-input layout (8 channels)
// Every block recomputes the per-image scalars from the partials (a few hundred floats from L2);
// block 0 publishes done/loss (the others compute the same values, so the write is idempotent).
template <int DT>
__global__ void __launch_bounds__(256) dream_update_kernel(const uint16_t* __restrict__ g, float* __restrict__ x,
                                                           uint16_t* __restrict__ xin, const float* __restrict__ gpart,
                                                           int gparts, const float* __restrict__ lpart,
                                                           const float* __restrict__ lcoef, int L, int lparts, int N,
                                                           uint8_t* __restrict__ done, float* __restrict__ loss,
                                                           float step, float max_loss, int HW) {
  const int n = blockIdx.y;
  __shared__ float sh[3];
  if (threadIdx.x < 64) {
    float gs = 0.f;
    for (int p = threadIdx.x; p < gparts; p += 64) gs += gpart[(long long)n * gparts + p];
    gs = wave_sum(gs);
    float ls = 0.f;
    for (int l = 0; l < L; ++l) {
      float t = 0.f;
      for (int p = threadIdx.x; p < lparts; p += 64) t += lpart[((long long)l * N + n) * lparts + p];
      ls += lcoef[l] * wave_sum(t);
    }
    if (threadIdx.x == 0) {
      const bool dn = done[n] != 0 || (max_loss >= 0.f && ls > max_loss);
      sh[0] = dn ? 0.f : step / fmaxf(gs / (3.f * (float)HW), 1e-7f);
      if (blockIdx.x == 0) {
        done[n] = dn ? 1 : 0;
        loss[n] = ls;
      }
    }
  }
  __syncthreads();
  const float sc = sh[0];
  const uint16_t* gn = g + (long long)n * HW * 8;
  float* xn = x + (long long)n * HW * 3;
  uint16_t* in = xin + (long long)n * HW * 8;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < HW; p += gridDim.x * 256) {
    const uint2 v = *reinterpret_cast<const uint2*>(gn + (long long)p * 8);
    const float x0 = xn[p * 3 + 0] + sc * to_f<DT>(v.x & 0xFFFFu);
    const float x1 = xn[p * 3 + 1] + sc * to_f<DT>(v.x >> 16);
    const float x2 = xn[p * 3 + 2] + sc * to_f<DT>(v.y & 0xFFFFu);
    xn[p * 3 + 0] = x0;
    xn[p * 3 + 1] = x1;
    xn[p * 3 + 2] = x2;
    *reinterpret_cast<uint4*>(in + (long long)p * 8) = uint4{pack2<DT>(x0, x1), pack2<DT>(x2, 0.f), 0u, 0u};
  }
}

// ---- octave transition (engine/deepdream.py:DeepDream.octave_steps) ----
// y[n] = bilinear resize, corner-aligned, of (a[n] + b[n] - c[n]) from [Hs, Ws, 3] to [Hd, Wd, 3] (fp32; b and c
// optional, same shape as a: the dreamed image plus the octave's lost detail), with torch's upsample_bilinear2d index math (src = r * dst, r = (in-1)/(out-1) from the
// host; i0 = floor, i1 = i0 + (i0 < in-1), lambda = src - i0), so it matches F.interpolate(align_corners=True)
// to rounding. yin (optional) receives the same pixels in the 16-bit 8-channel network-input layout (channels
// 3..7 zero), so an octave starts without copy/fill launches. One thread per output pixel.
template <int DT>
__global__ void __launch_bounds__(256) octave_resize_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                            const float* __restrict__ c, float* __restrict__ y, uint16_t* __restrict__ yin, int N,
                                                            int Hs, int Ws, int Hd, int Wd, float rh, float rw) {
  const long long total = (long long)N * Hd * Wd;
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < total; p += (long long)gridDim.x * 256) {
    const int ox = (int)(p % Wd);
    const long long t = p / Wd;
    const int oy = (int)(t % Hd), n = (int)(t / Hd);
    const float sy = rh * (float)oy, sx = rw * (float)ox;
    const int y0 = (int)sy, x0 = (int)sx;
    const int dy = y0 < Hs - 1 ? Ws * 3 : 0, dx = x0 < Ws - 1 ? 3 : 0;
    const float ly = sy - (float)y0, hy = 1.f - ly, lx = sx - (float)x0, hx = 1.f - lx;
    const long long o = (((long long)n * Hs + y0) * Ws + x0) * 3;
    float v[3];
#pragma unroll
    for (int ch = 0; ch < 3; ++ch) {
      const long long i00 = o + ch, i01 = i00 + dx, i10 = i00 + dy, i11 = i10 + dx;
      float v00 = a[i00], v01 = a[i01], v10 = a[i10], v11 = a[i11];
      if (b) {
        v00 += b[i00];
        v01 += b[i01];
        v10 += b[i10];
        v11 += b[i11];
      }
      if (c) {
        v00 -= c[i00];
        v01 -= c[i01];
        v10 -= c[i10];
        v11 -= c[i11];
      }
      v[ch] = hy * (hx * v00 + lx * v01) + ly * (hx * v10 + lx * v11);
      y[p * 3 + ch] = v[ch];
    }
    if (yin) *reinterpret_cast<uint4*>(yin + p * 8) = uint4{pack2<DT>(v[0], v[1]), pack2<DT>(v[2], 0.f), 0u, 0u};
  }
}

// ---- tiled DeepDream step (engine/deepdream.py:TiledDeepDream; BASELINE config 5) ----
// Work units are (tile, image) pairs; unit u has plan row plan[u] = {image, tile origin y, x,
// owned rect y0, y1, x0, x1 (tile-local, half-open)}. The image is rolled by shift = (sy, sx)
// (device int32[2], so one captured graph replays any shift): rolled[Y][X] = x[(Y-sy) mod H][(X-sx) mod W].
constexpr int TPLAN = 7;
// elements per unit in a pack (3 channels x tile, rounded to 16 B so the fp32 tail stays aligned)
__host__ __device__ inline long long tile_ustride(int Th, int Tw) { return ((long long)Th * Tw * 3 + 7) & ~7LL; }
// per-unit fp32 tail: {loss, sum |g| of pixel block 0 .. TP-1} (the pack kernel runs TP blocks per unit)
constexpr int TP = 31, TAILF = TP + 1;

// xin[k] (this rank's (k0 + k)-th unit, global unit u = rank + (k0 + k) * world) <- rolled-image tile,
// 8-channel 16-bit (k0: the first unit of a chunk of this rank's units, TiledDeepDream's overlapped steps)
template <int DT>
__global__ void __launch_bounds__(256) tile_gather_kernel(const float* __restrict__ x, uint16_t* __restrict__ xin,
                                                          const int* __restrict__ plan, const int* __restrict__ shift,
                                                          int rank, int world, int k0, int H, int W, int Th, int Tw) {
  const int k = blockIdx.y;
  const int* pu = plan + (long long)(rank + (k0 + k) * world) * TPLAN;
  const int b = pu[0], oy = pu[1], ox = pu[2];
  const int sy = shift[0], sx = shift[1];
  const float* xb = x + (long long)b * H * W * 3;
  uint16_t* dst = xin + (long long)k * Th * Tw * 8;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < Th * Tw; p += gridDim.x * 256) {
    const int ty = p / Tw, tx = p - ty * Tw;
    int yy = (oy + ty - sy) % H, xx = (ox + tx - sx) % W;
    yy += yy < 0 ? H : 0;
    xx += xx < 0 ? W : 0;
    const float* src = xb + ((long long)yy * W + xx) * 3;
    *reinterpret_cast<uint4*>(dst + (long long)p * 8) = uint4{pack2<DT>(src[0], src[1]), pack2<DT>(src[2], 0.f), 0u, 0u};
  }
}

// pack[k] <- the owned pixels (3 channels, 16-bit, tile-local row-major over the owned rect) of the
// unit's input gradient g[k]; tail (fp32 pairs after units * Th*Tw*3 elements): {loss, sum |g|}
// of the unit, loss = sum_l lcoef[l] * sum_p lpart[l][k][p].
template <int DT>
__global__ void __launch_bounds__(256) tile_pack_kernel(const uint16_t* __restrict__ g, uint16_t* __restrict__ pack,
                                                        const int* __restrict__ plan, const float* __restrict__ lpart,
                                                        const float* __restrict__ lcoef, int L, int lparts, int units,
                                                        int ucap, int rank, int world, int k0, int Th, int Tw) {
  const int k = blockIdx.y;
  const int* pu = plan + (long long)(rank + (k0 + k) * world) * TPLAN;
  const int y0 = pu[3], y1 = pu[4], x0 = pu[5], x1 = pu[6];
  const int ow = x1 - x0, npix = (y1 - y0) * ow;
  const uint16_t* gk = g + (long long)k * Th * Tw * 8;
  uint16_t* dst = pack + (long long)k * tile_ustride(Th, Tw);
  float* tail = reinterpret_cast<float*>(pack + (long long)ucap * tile_ustride(Th, Tw)) + (long long)TAILF * k;
  float asum = 0.f;
  // TP blocks per unit (fixed by the tail layout): PU independent loads per thread in flight per
  // round, else one unit's ~1M owned pixels serialize on load latency (287 us at 1024^2,
  // profiles/kstats_c5_r2_tiled_fused.txt)
  constexpr int PU = 8;
  constexpr int STRIDE = TP * 256;
  for (int base = blockIdx.x * 256 + threadIdx.x; base < npix; base += STRIDE * PU) {
    uint2 v[PU];
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int p = base + u * STRIDE;
      if (p < npix) {
        const int ty = y0 + p / ow, tx = x0 + p % ow;
        v[u] = *reinterpret_cast<const uint2*>(gk + ((long long)ty * Tw + tx) * 8);
      }
    }
#pragma unroll
    for (int u = 0; u < PU; ++u) {
      const int p = base + u * STRIDE;
      if (p < npix) {
        const uint16_t c0 = (uint16_t)(v[u].x & 0xFFFFu), c1 = (uint16_t)(v[u].x >> 16), c2 = (uint16_t)(v[u].y & 0xFFFFu);
        dst[p * 3 + 0] = c0;
        dst[p * 3 + 1] = c1;
        dst[p * 3 + 2] = c2;
        asum += fabsf(to_f<DT>(c0)) + fabsf(to_f<DT>(c1)) + fabsf(to_f<DT>(c2));
      }
    }
  }
  __shared__ float red[4];
  asum = wave_sum(asum);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = asum;
  __syncthreads();
  if (threadIdx.x == 0) tail[1 + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (blockIdx.x == 0 && threadIdx.x < 64) {
    float ls = 0.f;
    for (int l = 0; l < L; ++l) {
      float t = 0.f;
      for (int p = threadIdx.x; p < lparts; p += 64) t += lpart[((long long)l * units + k) * lparts + p];
      ls += lcoef[l] * wave_sum(t);
    }
    if (threadIdx.x == 0) tail[0] = ls;
  }
}

// x += step * (!done) * g / max(mean |g|, 1e-7) straight from the gathered packs of every rank
// (each image pixel is owned by exactly one unit: no races); per-image loss and sum |g| come from
// the unit tails (every block recomputes them; the done/loss writes are idempotent).
// Packs are [chunks][world][pack_elems] of units_per_rank (= per chunk) units each: unit v lives on rank
// v % world as local unit j = v / world, in chunk j / units_per_rank, slot j % units_per_rank (one chunk:
// the un-chunked layout).
__global__ void __launch_bounds__(256) tile_update_kernel(const uint16_t* __restrict__ packs, long long pack_elems,
                                                          int units_per_rank, const int* __restrict__ plan,
                                                          int nunits, const int* __restrict__ shift, float* __restrict__ x,
                                                          uint8_t* __restrict__ done, float* __restrict__ loss,
                                                          float step, float max_loss, int world, int H, int W, int Th,
                                                          int Tw, int dt) {
  const int u = blockIdx.y;
  const int* pu = plan + (long long)u * TPLAN;
  const int b = pu[0];
  __shared__ float sh[1];
  if (threadIdx.x < 64) {
    float ls = 0.f, as = 0.f;
    for (int v = threadIdx.x; v < nunits; v += 64) {
      if (plan[(long long)v * TPLAN] != b) continue;
      const int j = v / world;
      const float* tail = reinterpret_cast<const float*>(packs +
                                                         ((long long)(j / units_per_rank) * world + v % world) * pack_elems +
                                                         (long long)units_per_rank * tile_ustride(Th, Tw)) +
                          (long long)TAILF * (j % units_per_rank);
      ls += tail[0];
      for (int q = 0; q < TP; ++q) as += tail[1 + q];
    }
    ls = wave_sum(ls);
    as = wave_sum(as);
    if (threadIdx.x == 0) {
      const bool dn = done[b] != 0 || (max_loss >= 0.f && ls > max_loss);
      sh[0] = dn ? 0.f : step / fmaxf(as / (3.f * (float)H * (float)W), 1e-7f);
      done[b] = dn ? 1 : 0;
      loss[b] = ls;
    }
  }
  __syncthreads();
  const float sc = sh[0];
  const int oy = pu[1], ox = pu[2], y0 = pu[3], y1 = pu[4], x0 = pu[5], x1 = pu[6];
  const int ow = x1 - x0, npix = (y1 - y0) * ow;
  const int sy = shift[0], sx = shift[1];
  const int ju = u / world;
  const uint16_t* src = packs + ((long long)(ju / units_per_rank) * world + u % world) * pack_elems +
                        (long long)(ju % units_per_rank) * tile_ustride(Th, Tw);
  float* xb = x + (long long)b * H * W * 3;
  for (int p = blockIdx.x * 256 + threadIdx.x; p < npix; p += gridDim.x * 256) {
    const int ty = y0 + p / ow, tx = x0 + p % ow;
    int yy = (oy + ty - sy) % H, xx = (ox + tx - sx) % W;
    yy += yy < 0 ? H : 0;
    xx += xx < 0 ? W : 0;
    float* d = xb + ((long long)yy * W + xx) * 3;
#pragma unroll
    for (int c = 0; c < 3; ++c) d[c] += sc * (dt == DT_F16 ? to_f<DT_F16>(src[p * 3 + c]) : to_f<DT_BF16>(src[p * 3 + c]));
  }
}

long long tile_pack_elems(int ucap, int Th, int Tw) {
  // + 2 halfs per fp32 tail entry; rounded to 8 elements so every pack of a [chunks][world][pack]
  // buffer starts 16-B aligned (an odd unit count left 68-element tails 8-B aligned only)
  return ((long long)ucap * (tile_ustride(Th, Tw) + 2 * TAILF + 4) + 7) & ~7LL;
}

int tile_gather_launch(const float* x, uint16_t* xin, const int* plan, const int* shift, int units, int rank, int world,
                       int k0, int H, int W, int Th, int Tw, int dtype, hipStream_t s) {
  if (units < 1 || units > 65535 || k0 < 0) return -1;
  const dim3 grid((unsigned)std::min((Th * Tw + 255) / 256, 512), (unsigned)units);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(tile_gather_kernel<DT_F16>, grid, dim3(256), 0, s, x, xin, plan, shift, rank, world, k0, H, W, Th, Tw);
  else
    hipLaunchKernelGGL(tile_gather_kernel<DT_BF16>, grid, dim3(256), 0, s, x, xin, plan, shift, rank, world, k0, H, W, Th, Tw);
  return (int)hipGetLastError();
}

int tile_pack_launch(const uint16_t* g, uint16_t* pack, const int* plan, const float* lpart, const float* lcoef, int L,
                     int lparts, int units, int ucap, int rank, int world, int k0, int Th, int Tw, int dtype, hipStream_t s) {
  if (units < 1 || units > ucap || k0 < 0) return -1;
  if (units > 65535) return -1;
  const dim3 grid((unsigned)TP, (unsigned)units);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(tile_pack_kernel<DT_F16>, grid, dim3(256), 0, s, g, pack, plan, lpart, lcoef, L, lparts, units,
                       ucap, rank, world, k0, Th, Tw);
  else
    hipLaunchKernelGGL(tile_pack_kernel<DT_BF16>, grid, dim3(256), 0, s, g, pack, plan, lpart, lcoef, L, lparts, units,
                       ucap, rank, world, k0, Th, Tw);
  return (int)hipGetLastError();
}

int tile_update_launch(const uint16_t* packs, long long pack_elems, int units_per_rank, const int* plan, int nunits,
                       const int* shift, float* x, uint8_t* done, float* loss, float step, float max_loss, int world,
                       int H, int W, int Th, int Tw, int dtype, hipStream_t s) {
  if (nunits < 1 || nunits > 65535) return -1;
  const dim3 grid((unsigned)std::min((Th * Tw + 255) / 256, 512), (unsigned)nunits);
  hipLaunchKernelGGL(tile_update_kernel, grid, dim3(256), 0, s, packs, pack_elems, units_per_rank, plan, nunits, shift, x,
                     done, loss, step, max_loss, world, H, W, Th, Tw, dtype);
  return (int)hipGetLastError();
}

int dream_update_launch(const uint16_t* g, float* x, uint16_t* xin, float* gpart, int gparts, const float* lpart,
                        const float* lcoef, int L, int lparts, uint8_t* done, float* loss, float step, float max_loss,
                        int N, int H, int W, int dtype, hipStream_t s) {
  if (gparts < 1 || N < 1 || N > 65535) return -1;
  const int HW = H * W;
  const dim3 gp((unsigned)gparts, (unsigned)N);
  const unsigned ub = (unsigned)std::min(std::max((HW + 255) / 256, 1), 64);
  if (dtype == DT_F16) {
    hipLaunchKernelGGL(absmean_part_kernel<DT_F16>, gp, dim3(256), 0, s, g, gpart, HW);
    hipLaunchKernelGGL(dream_update_kernel<DT_F16>, dim3(ub, (unsigned)N), dim3(256), 0, s, g, x, xin, gpart, gparts,
                       lpart, lcoef, L, lparts, N, done, loss, step, max_loss, HW);
  } else {
    hipLaunchKernelGGL(absmean_part_kernel<DT_BF16>, gp, dim3(256), 0, s, g, gpart, HW);
    hipLaunchKernelGGL(dream_update_kernel<DT_BF16>, dim3(ub, (unsigned)N), dim3(256), 0, s, g, x, xin, gpart, gparts,
                       lpart, lcoef, L, lparts, N, done, loss, step, max_loss, HW);
  }
  return (int)hipGetLastError();
}

int octave_resize_launch(const float* a, const float* b, const float* c, float* y, uint16_t* yin, int N, int Hs, int Ws, int Hd, int Wd,
                         int dtype, hipStream_t s) {
  if (N < 1 || Hs < 1 || Ws < 1 || Hd < 1 || Wd < 1) return -1;
  const float rh = Hd > 1 ? (float)(Hs - 1) / (float)(Hd - 1) : 0.f;
  const float rw = Wd > 1 ? (float)(Ws - 1) / (float)(Wd - 1) : 0.f;
  const long long total = (long long)N * Hd * Wd;
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 256LL * 16);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(octave_resize_kernel<DT_F16>, dim3(grid), dim3(256), 0, s, a, b, c, y, yin, N, Hs, Ws, Hd, Wd, rh, rw);
  else
    hipLaunchKernelGGL(octave_resize_kernel<DT_BF16>, dim3(grid), dim3(256), 0, s, a, b, c, y, yin, N, Hs, Ws, Hd, Wd, rh, rw);
  return (int)hipGetLastError();
}

int sumsq_core_launch(const uint16_t* x, float* part, int parts, int N, int H, int W, int C, int b, int dtype,
                      hipStream_t s) {
  if (C % 8 != 0 || H <= 2 * b || W <= 2 * b || parts < 1) return -1;
  const dim3 grid((unsigned)parts, (unsigned)N);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(sumsq_core_kernel<DT_F16>, grid, dim3(256), 0, s, x, part, H, W, C, b);
  else
    hipLaunchKernelGGL(sumsq_core_kernel<DT_BF16>, grid, dim3(256), 0, s, x, part, H, W, C, b);
  return (int)hipGetLastError();
}

int sumsq_core_fused_launch(const uint16_t* x, const float* scale, const uint16_t* addend, uint16_t* gx, float* part,
                            int parts, int N, int H, int W, int C, int b, int dtype, hipStream_t s) {
  if (C % 8 != 0 || H <= 2 * b || W <= 2 * b || parts < 1 || (long long)H * W * (C / 8) > 0x7FFFFFFFLL) return -1;
  const dim3 grid((unsigned)parts, (unsigned)N);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(sumsq_core_fused_kernel<DT_F16>, grid, dim3(256), 0, s, x, scale, addend, gx, part, H, W, C, b);
  else
    hipLaunchKernelGGL(sumsq_core_fused_kernel<DT_BF16>, grid, dim3(256), 0, s, x, scale, addend, gx, part, H, W, C, b);
  return (int)hipGetLastError();
}

int sumsq_core_bwd_launch(const uint16_t* x, const float* scale, const uint16_t* addend, uint16_t* gx, int N, int H,
                          int W, int C, int b, int dtype, hipStream_t s) {
  if (C % 8 != 0) return -1;
  const long long total = (long long)N * H * W * (C / 8);
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 256LL * 32);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(sumsq_core_bwd_kernel<DT_F16>, dim3(grid), dim3(256), 0, s, x, scale, addend, gx, N, H, W, C, b);
  else
    hipLaunchKernelGGL(sumsq_core_bwd_kernel<DT_BF16>, dim3(grid), dim3(256), 0, s, x, scale, addend, gx, N, H, W, C, b);
  return (int)hipGetLastError();
}

}  // namespace dv

namespace dv {

// col2im for the input gradient of a strided conv with very few input channels (the RGB stem):
// cols[n][oh][ow][(kh*KW + kw)*Cr + c] = sum_oc dy[n][oh][ow][oc] * w[oc][c][kh][kw] comes from a
// plain GEMM (1x1 conv) that reads dy once; here each dx pixel gathers its <= ceil(KH/s)*ceil(KW/s)
// contributions. One thread per dx pixel, fp32 sums, Cpad (8) channels written with one 16-B store.
template <int DT>
__global__ void __launch_bounds__(256) col2im_kernel(const uint16_t* __restrict__ cols, uint16_t* __restrict__ gx,
                                                     Col2ImGeom g) {
  const long long total = (long long)g.N * g.H * g.W;
  for (long long p = blockIdx.x * 256LL + threadIdx.x; p < total; p += (long long)gridDim.x * 256) {
    const int iw = (int)(p % g.W);
    const int ih = (int)((p / g.W) % g.H);
    const long long n = p / ((long long)g.W * g.H);
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int kh0 = (ih + g.pad_h) % g.stride, kw0 = (iw + g.pad_w) % g.stride;
    for (int kh = kh0; kh < g.KH; kh += g.stride) {
      const int oh = (ih + g.pad_h - kh) / g.stride;
      if (oh < 0 || oh >= g.OH) continue;
      for (int kw = kw0; kw < g.KW; kw += g.stride) {
        const int ow = (iw + g.pad_w - kw) / g.stride;
        if (ow < 0 || ow >= g.OW) continue;
        const uint16_t* src = cols + ((n * g.OH + oh) * g.OW + ow) * g.J_ld + (kh * g.KW + kw) * g.Cr;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c < g.Cr) acc[c] += to_f<DT>(src[c]);
      }
    }
    uint4 o;
    o.x = pack2<DT>(acc[0], acc[1]);
    o.y = pack2<DT>(acc[2], acc[3]);
    o.z = pack2<DT>(acc[4], acc[5]);
    o.w = pack2<DT>(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(gx + p * 8) = o;
  }
}

// LDS-tiled col2im: a workgroup owns a TH x TW tile of dx; the cols rows it needs (a
// contiguous run of ow per oh: rows_n x cols_n x J_ld elements) are staged into LDS with 16-B
// loads, then every dx pixel gathers its taps from LDS. The scattered 6-byte global reads of the
// simple kernel above become coalesced streaming reads.
constexpr int C2I_TH = 8, C2I_TW = 64;

__host__ __device__ inline int c2i_lo(int i0, int pad, int k, int s) {  // first o with o*s - pad + k - 1 >= i0
  const int t = i0 + pad - k + 1;
  return t <= 0 ? 0 : (t + s - 1) / s;
}

template <int DT>
__global__ void __launch_bounds__(256) col2im_lds_kernel(const uint16_t* __restrict__ cols,
                                                         uint16_t* __restrict__ gx, Col2ImGeom g) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int n = blockIdx.z;
  const int ih0 = blockIdx.y * C2I_TH, iw0 = blockIdx.x * C2I_TW;
  const int oh_lo = c2i_lo(ih0, g.pad_h, g.KH, g.stride);
  const int oh_hi = min(g.OH - 1, (min(ih0 + C2I_TH, g.H) - 1 + g.pad_h) / g.stride);
  const int ow_lo = c2i_lo(iw0, g.pad_w, g.KW, g.stride);
  const int ow_hi = min(g.OW - 1, (min(iw0 + C2I_TW, g.W) - 1 + g.pad_w) / g.stride);
  const int rows_n = oh_hi - oh_lo + 1, cols_n = ow_hi - ow_lo + 1;
  uint16_t* tile = reinterpret_cast<uint16_t*>(lds);
  if (rows_n > 0 && cols_n > 0) {
    const int seg = cols_n * g.J_ld / 8;  // 16-B chunks per oh row
    for (int c = threadIdx.x; c < rows_n * seg; c += 256) {
      const int r = c / seg, q = c - r * seg;
      const uint16_t* src = cols + (((long long)n * g.OH + oh_lo + r) * g.OW + ow_lo) * g.J_ld + q * 8;
      *reinterpret_cast<uint4*>(tile + ((long long)r * cols_n * g.J_ld) + q * 8) =
          *reinterpret_cast<const uint4*>(src);
    }
  }
  __syncthreads();
  for (int p = threadIdx.x; p < C2I_TH * C2I_TW; p += 256) {
    const int ih = ih0 + p / C2I_TW, iw = iw0 + p % C2I_TW;
    if (ih >= g.H || iw >= g.W) continue;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int kh0 = (ih + g.pad_h) % g.stride, kw0 = (iw + g.pad_w) % g.stride;
    for (int kh = kh0; kh < g.KH; kh += g.stride) {
      const int oh = (ih + g.pad_h - kh) / g.stride;
      if (ih + g.pad_h - kh < 0 || oh >= g.OH) continue;
      for (int kw = kw0; kw < g.KW; kw += g.stride) {
        const int ow = (iw + g.pad_w - kw) / g.stride;
        if (iw + g.pad_w - kw < 0 || ow >= g.OW) continue;
        const uint16_t* src = tile + ((oh - oh_lo) * cols_n + (ow - ow_lo)) * g.J_ld + (kh * g.KW + kw) * g.Cr;
#pragma unroll
        for (int c = 0; c < 8; ++c)
          if (c < g.Cr) acc[c] += to_f<DT>(src[c]);
      }
    }
    uint4 o;
    o.x = pack2<DT>(acc[0], acc[1]);
    o.y = pack2<DT>(acc[2], acc[3]);
    o.z = pack2<DT>(acc[4], acc[5]);
    o.w = pack2<DT>(acc[6], acc[7]);
    *reinterpret_cast<uint4*>(gx + (((long long)n * g.H + ih) * g.W + iw) * 8) = o;
  }
}

int col2im_launch(const uint16_t* cols, uint16_t* gx, const Col2ImGeom& g, int dtype, hipStream_t s) {
  if (g.Cr < 1 || g.Cr > 8 || g.stride < 1) return -1;
  {
    const int rows_max = (C2I_TH - 1 + g.KH - 1) / g.stride + 1, cols_max = (C2I_TW - 1 + g.KW - 1) / g.stride + 1;
    const size_t lds = (size_t)rows_max * cols_max * g.J_ld * 2;
    if (g.J_ld % 8 == 0 && lds <= 160 * 1024 && g.N <= 65535 && reinterpret_cast<uintptr_t>(cols) % 16 == 0) {
      const dim3 grid((unsigned)((g.W + C2I_TW - 1) / C2I_TW), (unsigned)((g.H + C2I_TH - 1) / C2I_TH), (unsigned)g.N);
      static const bool attr_ok = [] {  // allow > 64 KiB of dynamic LDS (gfx950: 160 KiB per CU)
        return hipFuncSetAttribute((const void*)col2im_lds_kernel<DT_F16>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess &&
               hipFuncSetAttribute((const void*)col2im_lds_kernel<DT_BF16>,
                                   hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) == hipSuccess;
      }();
      if (!attr_ok) return -5;
      if (dtype == DT_F16)
        hipLaunchKernelGGL(col2im_lds_kernel<DT_F16>, grid, dim3(256), lds, s, cols, gx, g);
      else
        hipLaunchKernelGGL(col2im_lds_kernel<DT_BF16>, grid, dim3(256), lds, s, cols, gx, g);
      return (int)hipGetLastError();
    }
  }
  const long long total = (long long)g.N * g.H * g.W;
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 256LL * 64);
  if (dtype == DT_F16)
    hipLaunchKernelGGL(col2im_kernel<DT_F16>, dim3(grid), dim3(256), 0, s, cols, gx, g);
  else
    hipLaunchKernelGGL(col2im_kernel<DT_BF16>, dim3(grid), dim3(256), 0, s, cols, gx, g);
  return (int)hipGetLastError();
}

}  // namespace dv
