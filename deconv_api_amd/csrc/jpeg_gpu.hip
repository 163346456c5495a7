// Baseline JPEG encode of the response mosaics on the GPU (the reference: cv2.imencode('.jpg')
// per request on the CPU, app/main.py:73). Same stream as the host encoder (jpeg_enc.cpp: JFIF,
// 4:2:0, IJG-scaled Annex K quantization, Annex K Huffman tables) with a restart marker after every
// MCU row, so every row is an independent entropy-coded segment. Only the compressed bytes cross
// PCIe (~10x fewer than the RGB mosaic) and the host only base64s them.
//
// Five kernels per batch of B same-size images:
//   jpeg_block   one thread per 8x8 block (4 Y + Cb + Cr per 16x16 MCU): RGB -> YCbCr (edge
//                replication), 2x2 chroma average, level shift, AAN float DCT, quantization (round
//                half away from zero), zig-zag; stores the 64 coefficients, the DC value and the
//                bit count of the block's AC symbols (run/size codes, ZRLs, EOB)
//   jpeg_plan    one workgroup per image: DC differences (predictor reset per segment), each
//                block's bit offset in its segment (block scan), each segment's byte offset in the
//                image's raw scan (segments byte-aligned, padded with 1-bits); zeroes the raw words
//   jpeg_pack    one thread per block: writes its codes at its bit offset (atomicOr on 32-bit
//                words: neighbours share the boundary words); the segment's last block adds the pad
//   jpeg_stuff   one workgroup per image: per segment, 0xFF -> FF 00 byte stuffing (block scan of
//                the output positions) + RSTm marker; the image's scan length
//   jpeg_compact one workgroup per image: scans packed back to back (offsets: exclusive scan of
//                the lengths, computed by the first workgroup per launch from the lengths)
// Bit order: the raw scan is a sequence of big-endian 32-bit words (bit 0 = MSB of byte 0).
#include "common.h"
#include "jpeg_enc.h"
#include "kernels.h"

namespace dv {

namespace {

// zig-zag position k -> index into the DCT output in its transposed (u-major) layout, i.e.
// (zz % 8) * 8 + zz / 8 of the natural-order zig-zag table (jpeg_enc.cpp: Plan::zz_src)
struct ZZ {
  int v[64];
  constexpr ZZ() : v() {
    constexpr int zz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                            12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                            35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                            58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
    for (int k = 0; k < 64; ++k) v[k] = (zz[k] % 8) * 8 + zz[k] / 8;
  }
};
constexpr ZZ kZZ;

__device__ __forceinline__ int nbits_i(int v) {
  v = v < 0 ? -v : v;
  return v ? 32 - __clz((unsigned)v) : 0;
}

// the host encoder's 8-point AAN DCT (jpeg_enc.cpp:aan8_cols) on columns of d
__device__ __forceinline__ void aan8_cols_d(float (&d)[8][8]) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float t0 = d[0][i] + d[7][i], t7 = d[0][i] - d[7][i];
    const float t1 = d[1][i] + d[6][i], t6 = d[1][i] - d[6][i];
    const float t2 = d[2][i] + d[5][i], t5 = d[2][i] - d[5][i];
    const float t3 = d[3][i] + d[4][i], t4 = d[3][i] - d[4][i];
    const float e10 = t0 + t3, e13 = t0 - t3, e11 = t1 + t2, e12 = t1 - t2;
    d[0][i] = e10 + e11;
    d[4][i] = e10 - e11;
    const float z1 = (e12 + e13) * 0.707106781f;
    d[2][i] = e13 + z1;
    d[6][i] = e13 - z1;
    const float o10 = t4 + t5, o11 = t5 + t6, o12 = t6 + t7;
    const float z5 = (o10 - o12) * 0.382683433f;
    const float z2 = 0.541196100f * o10 + z5;
    const float z4 = 1.306562965f * o12 + z5;
    const float z3 = o11 * 0.707106781f;
    const float z11 = t7 + z3, z13 = t7 - z3;
    d[5][i] = z13 + z2;
    d[3][i] = z13 - z2;
    d[1][i] = z11 + z4;
    d[7][i] = z11 - z4;
  }
}

struct Geo {
  int B, H, W, mcux, mcuy;
  long long nblk;        // B * mcux * mcuy * 6
  long long raw_words;   // per-image raw scan capacity (32-bit words)
  long long out_cap;     // per-image stuffed scan capacity (bytes)
};

__device__ __forceinline__ void rgb_at(const uint8_t* img, const Geo& g, int y, int x, float& r, float& gg, float& b) {
  y = min(y, g.H - 1);
  x = min(x, g.W - 1);
  const uint8_t* p = img + ((long long)y * g.W + x) * 3;
  r = p[0];
  gg = p[1];
  b = p[2];
}

__global__ void __launch_bounds__(256) jpeg_block_kernel(const uint8_t* __restrict__ rgb, Geo g,
                                                         const dvjpeg::GpuTables* __restrict__ t,
                                                         int16_t* __restrict__ coef, int* __restrict__ dcv,
                                                         int* __restrict__ acbits) {
  const long long b = blockIdx.x * 256LL + threadIdx.x;
  if (b >= g.nblk) return;
  const int per_img = g.mcux * g.mcuy * 6;
  const int img = (int)(b / per_img);
  const int rem = (int)(b - (long long)img * per_img);
  const int mcu = rem / 6, k = rem - mcu * 6;
  const int my = mcu / g.mcux, mx = mcu - my * g.mcux;
  const uint8_t* im = rgb + (long long)img * g.H * g.W * 3;
  float d[8][8];
  if (k < 4) {
    const int y0 = my * 16 + (k >> 1) * 8, x0 = mx * 16 + (k & 1) * 8;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float R, G, Bc;
        rgb_at(im, g, y0 + r, x0 + c, R, G, Bc);
        d[r][c] = 0.299f * R + 0.587f * G + 0.114f * Bc - 128.f;
      }
  } else {
    const bool cb = k == 4;
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float R, G, Bc;
          rgb_at(im, g, my * 16 + 2 * r + (q >> 1), mx * 16 + 2 * c + (q & 1), R, G, Bc);
          v[q] = cb ? (-0.168736f * R - 0.331264f * G + 0.5f * Bc) : (0.5f * R - 0.418688f * G - 0.081312f * Bc);
        }
        d[r][c] = 0.25f * (v[0] + v[1] + v[2] + v[3]);
      }
  }
  aan8_cols_d(d);
#pragma unroll
  for (int r = 0; r < 8; ++r)
#pragma unroll
    for (int c = r + 1; c < 8; ++c) {
      const float x = d[r][c];
      d[r][c] = d[c][r];
      d[c][r] = x;
    }
  aan8_cols_d(d);
  const float* qs = k < 4 ? t->rl : t->rc;
  // quantize straight into zig-zag order (compile-time indices: the block stays in registers)
  int zz[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const int src = kZZ.v[i];
    const float v = d[src >> 3][src & 7] * qs[src];
    zz[i] = v < 0.f ? -(int)(0.5f - v) : (int)(v + 0.5f);
  }
  // AC symbol bits (host encoder's encode_block, without the DC part)
  const int tc = k < 4 ? 0 : 1;
  int bits = 0, run = 0;
#pragma unroll
  for (int i = 1; i < 64; ++i) {
    const int v = zz[i];
    if (v == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bits += t->ac_len[tc][0xF0];
      run -= 16;
    }
    const int n = nbits_i(v);
    bits += t->ac_len[tc][(run << 4) | n] + n;
    run = 0;
  }
  if (run) bits += t->ac_len[tc][0x00];
  int16_t* cp = coef + b * 64;
#pragma unroll
  for (int i = 0; i < 64; i += 8) {
    uint4 w;
    w.x = (uint16_t)zz[i] | ((uint32_t)(uint16_t)zz[i + 1] << 16);
    w.y = (uint16_t)zz[i + 2] | ((uint32_t)(uint16_t)zz[i + 3] << 16);
    w.z = (uint16_t)zz[i + 4] | ((uint32_t)(uint16_t)zz[i + 5] << 16);
    w.w = (uint16_t)zz[i + 6] | ((uint32_t)(uint16_t)zz[i + 7] << 16);
    *reinterpret_cast<uint4*>(cp + i) = w;
  }
  dcv[b] = zz[0];
  acbits[b] = bits;
}

// component of block j of an MCU row (0: Y, 1: Cb, 2: Cr) and the previous block of that
// component in the row (-1: first of the segment, predictor 0)
__device__ __forceinline__ int prev_same(int j, int& comp) {
  const int k = j % 6;
  comp = k < 4 ? 0 : (k == 4 ? 1 : 2);
  if (comp == 0) return k > 0 ? j - 1 : (j >= 6 ? j - 3 : -1);
  return j >= 6 ? j - 6 : -1;
}

constexpr int PLAN_T = 1024;

// one workgroup per image: dcdiff[b], boff[b] (bit offset of block b in the image's raw scan),
// seg_off[s] (byte offset of segment s), seg_bytes[s]; zeroes the image's used raw words
__global__ void __launch_bounds__(PLAN_T) jpeg_plan_kernel(Geo g, const dvjpeg::GpuTables* __restrict__ t,
                                                           const int* __restrict__ dcv, const int* __restrict__ acbits,
                                                           int* __restrict__ dcdiff, long long* __restrict__ boff,
                                                           long long* __restrict__ seg_off, int* __restrict__ seg_bytes,
                                                           uint32_t* __restrict__ raw) {
  __shared__ long long part[PLAN_T / 64];
  __shared__ long long carry_s;
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nb = g.mcux * 6;  // blocks per segment (one MCU row)
  const long long base = (long long)img * g.mcuy * nb;
  if (tid == 0) carry_s = 0;
  __syncthreads();
  for (int s = 0; s < g.mcuy; ++s) {
    const long long sb = base + (long long)s * nb;
    const long long seg_start = carry_s;  // byte-aligned bit offset of this segment
    long long run = 0;                    // bits of the segment's blocks before this chunk
    for (int j0 = 0; j0 < nb; j0 += PLAN_T) {
      const int j = j0 + tid;
      long long bits = 0;
      if (j < nb) {
        int comp;
        const int pj = prev_same(j, comp);
        const int diff = dcv[sb + j] - (pj >= 0 ? dcv[sb + pj] : 0);
        const int n = nbits_i(diff);
        dcdiff[sb + j] = diff;
        bits = t->dc_len[comp > 0][n] + n + acbits[sb + j];
      }
      // block-wide inclusive scan (wave scan + wave totals)
      long long v = bits;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const long long u = __shfl_up(v, o, 64);
        if (lane >= o) v += u;
      }
      if (lane == 63) part[wave] = v;
      __syncthreads();
      long long before = 0;
      for (int w = 0; w < wave; ++w) before += part[w];
      long long total = 0;
      for (int w = 0; w < PLAN_T / 64; ++w) total += part[w];
      if (j < nb) boff[sb + j] = seg_start * 8 + run + before + v - bits;
      run += total;
      __syncthreads();
    }
    if (tid == 0) {
      const int bytes = (int)((run + 7) >> 3);
      seg_off[(long long)img * g.mcuy + s] = seg_start;
      seg_bytes[(long long)img * g.mcuy + s] = bytes;
      carry_s = seg_start + bytes;
    }
    __syncthreads();
  }
  // zero the used raw words of this image (pack ORs into them)
  const long long words = (carry_s + 3) >> 2;
  uint32_t* r = raw + (long long)img * g.raw_words;
  for (long long w = tid; w < words; w += PLAN_T) r[w] = 0u;
}

struct BitOut {
  uint32_t* raw;
  long long w;
  uint32_t cur;
  int fill;
  __device__ __forceinline__ void put(uint32_t code, int len) {
    while (len > 0) {
      const int take = min(len, 32 - fill);
      const uint32_t bits = (code >> (len - take)) & (take == 32 ? 0xFFFFFFFFu : ((1u << take) - 1u));
      cur |= bits << (32 - fill - take);
      fill += take;
      len -= take;
      if (fill == 32) {
        atomicOr(raw + w, cur);
        ++w;
        cur = 0u;
        fill = 0;
      }
    }
  }
  __device__ __forceinline__ void flush() {
    if (fill > 0) atomicOr(raw + w, cur);
  }
};

__global__ void __launch_bounds__(256) jpeg_pack_kernel(Geo g, const dvjpeg::GpuTables* __restrict__ t,
                                                        const int16_t* __restrict__ coef, const int* __restrict__ dcdiff,
                                                        const long long* __restrict__ boff, uint32_t* __restrict__ raw) {
  const long long b = blockIdx.x * 256LL + threadIdx.x;
  if (b >= g.nblk) return;
  const int nb = g.mcux * 6;
  const long long per_img = (long long)g.mcuy * nb;
  const int img = (int)(b / per_img);
  const long long rem = b - img * per_img;
  const int s = (int)(rem / nb), j = (int)(rem - (long long)s * nb);
  const int k = j % 6, tc = k < 4 ? 0 : 1;
  const long long o = boff[b];
  BitOut bo{raw + (long long)img * g.raw_words, o >> 5, 0u, (int)(o & 31)};
  const int diff = dcdiff[b];
  int n = nbits_i(diff);
  bo.put(t->dc_code[tc][n], t->dc_len[tc][n]);
  if (n) bo.put((uint32_t)(diff < 0 ? diff - 1 : diff), n);
  int zz[64];
#pragma unroll
  for (int i = 0; i < 64; i += 8) {
    const uint4 w = *reinterpret_cast<const uint4*>(coef + b * 64 + i);
    const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      zz[i + 2 * e] = (int)(int16_t)(ws[e] & 0xFFFFu);
      zz[i + 2 * e + 1] = (int)(int16_t)(ws[e] >> 16);
    }
  }
  int run = 0;
#pragma unroll
  for (int i = 1; i < 64; ++i) {
    const int v = zz[i];
    if (v == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bo.put(t->ac_code[tc][0xF0], t->ac_len[tc][0xF0]);
      run -= 16;
    }
    n = nbits_i(v);
    const int sym = (run << 4) | n;
    bo.put(t->ac_code[tc][sym], t->ac_len[tc][sym]);
    bo.put((uint32_t)(v < 0 ? v - 1 : v), n);
    run = 0;
  }
  if (run) bo.put(t->ac_code[tc][0x00], t->ac_len[tc][0x00]);
  if (j == nb - 1) {  // the segment's last block: pad with 1-bits to the next byte boundary
    const long long pos = bo.w * 32 + bo.fill;
    const int pad = (int)((((pos + 7) >> 3) << 3) - pos);
    if (pad) bo.put((1u << pad) - 1u, pad);
  }
  bo.flush();
}

constexpr int STUFF_T = 512;

__device__ __forceinline__ uint8_t raw_byte(const uint32_t* r, long long i) {
  return (uint8_t)(r[i >> 2] >> (24 - 8 * (int)(i & 3)));
}

// one workgroup per image: stuffed scan (+ RST markers) into out[img * out_cap ...], length len[img]
__global__ void __launch_bounds__(STUFF_T) jpeg_stuff_kernel(Geo g, const uint32_t* __restrict__ raw,
                                                             const long long* __restrict__ seg_off,
                                                             const int* __restrict__ seg_bytes,
                                                             uint8_t* __restrict__ out, long long* __restrict__ len) {
  __shared__ int part[STUFF_T / 64];
  const int img = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint32_t* r = raw + (long long)img * g.raw_words;
  uint8_t* o = out + (long long)img * g.out_cap;
  long long pos = 0;  // uniform across the workgroup
  for (int s = 0; s < g.mcuy; ++s) {
    const long long s0 = seg_off[(long long)img * g.mcuy + s];
    const int nbytes = seg_bytes[(long long)img * g.mcuy + s];
    for (int c0 = 0; c0 < nbytes; c0 += STUFF_T) {
      const int i = c0 + tid;
      uint8_t v = 0;
      int n = 0;
      if (i < nbytes) {
        v = raw_byte(r, s0 + i);
        n = v == 0xFF ? 2 : 1;
      }
      int x = n;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int u = __shfl_up(x, d, 64);
        if (lane >= d) x += u;
      }
      if (lane == 63) part[wave] = x;
      __syncthreads();
      int before = 0, total = 0;
      for (int w = 0; w < STUFF_T / 64; ++w) {
        if (w < wave) before += part[w];
        total += part[w];
      }
      const long long at = pos + before + x - n;
      if (i < nbytes && at + n <= g.out_cap) {
        o[at] = v;
        if (n == 2) o[at + 1] = 0;
      }
      pos += total;
      __syncthreads();
    }
    if (s + 1 < g.mcuy) {  // RSTm after every segment but the last
      if (tid == 0 && pos + 2 <= g.out_cap) {
        o[pos] = 0xFF;
        o[pos + 1] = (uint8_t)(0xD0 + (s & 7));
      }
      pos += 2;
    }
  }
  if (tid == 0) len[img] = pos;
}

// scans back to back: off = exclusive scan of len (every workgroup computes it; B is small)
__global__ void __launch_bounds__(256) jpeg_compact_kernel(Geo g, const uint8_t* __restrict__ out,
                                                           const long long* __restrict__ len,
                                                           uint8_t* __restrict__ packed, long long* __restrict__ off) {
  const int img = blockIdx.x;
  long long start = 0;
  for (int b = 0; b < img; ++b) start += len[b];
  if (threadIdx.x == 0) {
    off[img] = start;
    if (img == g.B - 1) off[g.B] = start + len[img];
  }
  const uint8_t* src = out + (long long)img * g.out_cap;
  for (long long i = threadIdx.x; i < len[img]; i += 256) packed[start + i] = src[i];
}

}  // namespace

// Per-image capacities: raw scan words and stuffed scan bytes (worst case: every block at the
// code-length bound of 1660 bits, every byte stuffed)
void jpeg_gpu_caps(int H, int W, long long* raw_words, long long* out_cap) {
  const long long blocks = (long long)((W + 15) / 16) * ((H + 15) / 16) * 6;
  const long long rb = blocks * 1660 / 8 + 8 * ((H + 15) / 16) + 64;
  *raw_words = (rb + 3) / 4;
  *out_cap = 2 * rb + 2 * ((H + 15) / 16) + 64;
}

int jpeg_gpu_launch(const uint8_t* rgb, int B, int H, int W, const void* tables, void* ws, uint8_t* packed,
                    long long* off, hipStream_t s) {
  if (B < 1 || H < 1 || W < 1) return -1;
  Geo g{};
  g.B = B;
  g.H = H;
  g.W = W;
  g.mcux = (W + 15) / 16;
  g.mcuy = (H + 15) / 16;
  g.nblk = (long long)B * g.mcux * g.mcuy * 6;
  jpeg_gpu_caps(H, W, &g.raw_words, &g.out_cap);
  // workspace carve-up (jpeg_gpu_ws_bytes)
  uint8_t* p = reinterpret_cast<uint8_t*>(ws);
  auto take = [&p](size_t bytes) {
    uint8_t* q = p;
    p += (bytes + 255) & ~size_t(255);
    return q;
  };
  int16_t* coef = reinterpret_cast<int16_t*>(take(g.nblk * 128));
  int* dcv = reinterpret_cast<int*>(take(g.nblk * 4));
  int* acb = reinterpret_cast<int*>(take(g.nblk * 4));
  int* dcd = reinterpret_cast<int*>(take(g.nblk * 4));
  long long* boff = reinterpret_cast<long long*>(take(g.nblk * 8));
  long long* seg_off = reinterpret_cast<long long*>(take((size_t)B * g.mcuy * 8));
  int* seg_bytes = reinterpret_cast<int*>(take((size_t)B * g.mcuy * 4));
  uint32_t* raw = reinterpret_cast<uint32_t*>(take((size_t)B * g.raw_words * 4));
  uint8_t* out = take((size_t)B * g.out_cap);
  long long* len = reinterpret_cast<long long*>(take((size_t)B * 8));
  const auto* t = reinterpret_cast<const dvjpeg::GpuTables*>(tables);
  const unsigned nb = (unsigned)((g.nblk + 255) / 256);
  hipLaunchKernelGGL(jpeg_block_kernel, dim3(nb), dim3(256), 0, s, rgb, g, t, coef, dcv, acb);
  hipLaunchKernelGGL(jpeg_plan_kernel, dim3(B), dim3(PLAN_T), 0, s, g, t, dcv, acb, dcd, boff, seg_off, seg_bytes, raw);
  hipLaunchKernelGGL(jpeg_pack_kernel, dim3(nb), dim3(256), 0, s, g, t, coef, dcd, boff, raw);
  hipLaunchKernelGGL(jpeg_stuff_kernel, dim3(B), dim3(STUFF_T), 0, s, g, raw, seg_off, seg_bytes, out, len);
  hipLaunchKernelGGL(jpeg_compact_kernel, dim3(B), dim3(256), 0, s, g, out, len, packed, off);
  return (int)hipGetLastError();
}

long long jpeg_gpu_ws_bytes(int B, int H, int W) {
  long long raw_words, out_cap;
  jpeg_gpu_caps(H, W, &raw_words, &out_cap);
  const long long nblk = (long long)B * ((W + 15) / 16) * ((H + 15) / 16) * 6;
  const long long mcuy = (H + 15) / 16;
  auto r = [](long long b) { return (b + 255) & ~255LL; };
  return r(nblk * 128) + 3 * r(nblk * 4) + r(nblk * 8) + r(B * mcuy * 8) + r(B * mcuy * 4) + r(B * raw_words * 4) +
         r(B * out_cap) + r(B * 8);
}

}  // namespace dv
