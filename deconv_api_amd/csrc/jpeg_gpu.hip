// Baseline JPEG encode of the response mosaics on the GPU (the reference: cv2.imencode('.jpg')
// per request on the CPU, app/main.py:73). Same stream as the host encoder (jpeg_enc.cpp: JFIF,
// 4:2:0, IJG-scaled Annex K quantization, Annex K Huffman tables) with a restart marker after every
// MCU row, so every row is an independent entropy-coded segment (DC predictors reset, byte-aligned)
// and one workgroup can encode it from pixels to stuffed bytes without leaving the CU. Only the
// compressed bytes cross PCIe (~10x fewer than the RGB mosaic) and the host only base64s them.
//
// Three kernels per batch of B same-size images (W <= 896):
//   jpeg_segment  one 256-thread workgroup per (MCU row, image), everything in LDS:
//                 1. RGB -> Y / Cb / Cr float planes (one thread per 2x2 pixel quad: edge
//                    replication, per-pixel chroma averaged over the quad, level shift);
//                 2. one thread per 8x8 block (6 per MCU): AAN float DCT, quantization (round half
//                    away from zero) straight into zig-zag order; coefficients to LDS, the mask of
//                    nonzero AC coefficients in registers (the coders visit only those), DC value
//                    + AC symbol bit count to LDS;
//                 3. DC differences + per-block bit offsets (workgroup scan);
//                 4. Huffman codes OR-ed into an LDS bit buffer (aliasing the planes; the segment's
//                    last block pads with 1-bits to a byte boundary);
//                 5. 0xFF -> FF 00 byte stuffing (workgroup scan over 4-byte words) into the
//                    segment's staging slot in HBM + RSTm, and the stuffed length.
//   jpeg_offsets  one workgroup: exclusive scan of the B * mcuy segment lengths -> destinations,
//                 image offsets
//   jpeg_copy     one workgroup per segment: staging slot -> packed scans (back to back)
// Round 3's first version ran five kernels over HBM intermediates (coefficients, bit offsets, a raw
// bit stream built with global atomics, per-image serial stuffing): 1.15 ms per 256 448^2 mosaics
// (profiles/kstats_c2_r3_jpeg.txt).
// Bit order: the bit buffer is a sequence of big-endian 32-bit words (bit 0 = MSB of byte 0).
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

constexpr int SEG_T = 256;         // threads per segment workgroup
constexpr int SEG_MAX_MCUX = 56;   // W <= 896: <= 336 blocks (2 per thread), ~146 KiB of LDS
constexpr int SEG_BLK_BITS = 1660; // code-length bound of one block (DC 11 + 16 + 63 x (16 + 10))
constexpr int SEG_CROW = 66;       // int16 per coefficient row: 33 words, odd (rows spread over banks)
static_assert(sizeof(dvjpeg::GpuTables) % 4 == 0, "tables are staged as 32-bit words");

// LDS carve-up of jpeg_segment (byte offsets): tables | dcv | acb | diff | boff | part | coef | planes
struct SegLds {
  int tab, dcv, acb, dif, boff, part, coef, planes, total;
  __host__ __device__ SegLds(int mcux) {
    const int nb = 6 * mcux;
    tab = 0;
    dcv = (int)((sizeof(dvjpeg::GpuTables) + 15) & ~15u);
    acb = dcv + nb * 4;
    dif = acb + nb * 4;
    boff = dif + nb * 4;
    part = boff + nb * 4;
    coef = (part + 16 * 4 + 15) & ~15;
    planes = (coef + nb * SEG_CROW * 2 + 15) & ~15;
    // Y: 16 rows x 18 mcux floats, Cb / Cr: 8 rows x 9 mcux floats (one pad float per 8: the
    // 8-column runs a block reads sit 9 banks apart); the bit buffer reuses the area
    total = planes + 1728 * mcux;
  }
};

struct SegGeo {
  int B, H, W, mcux, mcuy;
  long long seg_cap;  // staging bytes per segment
};

__device__ __forceinline__ void rgb_px(const uint8_t* im, int W, int y, int x, float& r, float& g, float& b) {
  const uint8_t* p = im + ((long long)y * W + x) * 3;
  r = p[0];
  g = p[1];
  b = p[2];
}

// block-wide exclusive scan of v (256 threads); total over the workgroup; part = 4 ints of LDS
__device__ __forceinline__ int seg_scan(int v, int* part, int& total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(x, o, 64);
    if (lane >= o) x += u;
  }
  if (lane == 63) part[wave] = x;
  __syncthreads();
  int before = 0;
  total = 0;
#pragma unroll
  for (int w = 0; w < SEG_T / 64; ++w) {
    const int p = part[w];
    before += w < wave ? p : 0;
    total += p;
  }
  __syncthreads();  // part is reused by the next scan
  return before + x - v;
}

// component of block j of an MCU row (0: Y, 1: Cb, 2: Cr) and the previous block of that
// component in the row (-1: first of the segment, predictor 0)
__device__ __forceinline__ int prev_same(int j, int& comp) {
  const int k = j % 6;
  comp = k < 4 ? 0 : (k == 4 ? 1 : 2);
  if (comp == 0) return k > 0 ? j - 1 : (j >= 6 ? j - 3 : -1);
  return j >= 6 ? j - 6 : -1;
}

struct LdsBits {  // MSB-first bit writer into LDS words (neighbouring blocks share boundary words)
  uint32_t* buf;
  int w;
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
        atomicOr(buf + w, cur);
        ++w;
        cur = 0u;
        fill = 0;
      }
    }
  }
  __device__ __forceinline__ void flush() {
    if (fill > 0) atomicOr(buf + w, cur);
  }
};

__global__ void __launch_bounds__(SEG_T) jpeg_segment_kernel(const uint8_t* __restrict__ rgb, SegGeo g,
                                                             const dvjpeg::GpuTables* __restrict__ tg,
                                                             uint8_t* __restrict__ stage, int* __restrict__ seg_len) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const SegLds L(g.mcux);
  const int tid = threadIdx.x;
  const int s = blockIdx.x, img = blockIdx.y;
  const int mcux = g.mcux, nb = 6 * mcux;
  const dvjpeg::GpuTables& t = *reinterpret_cast<const dvjpeg::GpuTables*>(lds + L.tab);
  int* dcv = reinterpret_cast<int*>(lds + L.dcv);
  int* acb = reinterpret_cast<int*>(lds + L.acb);
  int* dif = reinterpret_cast<int*>(lds + L.dif);
  int* boff = reinterpret_cast<int*>(lds + L.boff);
  int* part = reinterpret_cast<int*>(lds + L.part);
  float* Yp = reinterpret_cast<float*>(lds + L.planes);
  const int pitch_y = 18 * mcux, pitch_c = 9 * mcux;
  float* Cbp = Yp + 16 * pitch_y;
  float* Crp = Cbp + 8 * pitch_c;

  for (int i = tid; i < (int)(sizeof(dvjpeg::GpuTables) / 4); i += SEG_T)
    reinterpret_cast<uint32_t*>(lds + L.tab)[i] = reinterpret_cast<const uint32_t*>(tg)[i];

  // ---- 1. planes: one thread per 2x2 quad of the 16-row strip ----
  const uint8_t* im = rgb + (long long)img * g.H * g.W * 3;
  const int qw = 8 * mcux;  // quads per quad row
  for (int q = tid; q < 8 * qw; q += SEG_T) {
    const int qr = q / qw, qc = q - qr * qw;
    const int y0 = min(s * 16 + 2 * qr, g.H - 1), y1 = min(s * 16 + 2 * qr + 1, g.H - 1);
    const int x0 = min(2 * qc, g.W - 1), x1 = min(2 * qc + 1, g.W - 1);
    float R[4], G[4], Bc[4];
    rgb_px(im, g.W, y0, x0, R[0], G[0], Bc[0]);
    rgb_px(im, g.W, y0, x1, R[1], G[1], Bc[1]);
    rgb_px(im, g.W, y1, x0, R[2], G[2], Bc[2]);
    rgb_px(im, g.W, y1, x1, R[3], G[3], Bc[3]);
    const int c0 = 2 * qc, c1 = 2 * qc + 1;
    Yp[(2 * qr) * pitch_y + c0 + (c0 >> 3)] = 0.299f * R[0] + 0.587f * G[0] + 0.114f * Bc[0] - 128.f;
    Yp[(2 * qr) * pitch_y + c1 + (c1 >> 3)] = 0.299f * R[1] + 0.587f * G[1] + 0.114f * Bc[1] - 128.f;
    Yp[(2 * qr + 1) * pitch_y + c0 + (c0 >> 3)] = 0.299f * R[2] + 0.587f * G[2] + 0.114f * Bc[2] - 128.f;
    Yp[(2 * qr + 1) * pitch_y + c1 + (c1 >> 3)] = 0.299f * R[3] + 0.587f * G[3] + 0.114f * Bc[3] - 128.f;
    float cb[4], cr[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      cb[k] = -0.168736f * R[k] - 0.331264f * G[k] + 0.5f * Bc[k];
      cr[k] = 0.5f * R[k] - 0.418688f * G[k] - 0.081312f * Bc[k];
    }
    Cbp[qr * pitch_c + qc + (qc >> 3)] = 0.25f * (cb[0] + cb[1] + cb[2] + cb[3]);
    Crp[qr * pitch_c + qc + (qc >> 3)] = 0.25f * (cr[0] + cr[1] + cr[2] + cr[3]);
  }
  __syncthreads();

  // ---- 2. DCT + quantization: block j = tid + 256 * sl; zig-zag coefficients to LDS, the AC
  // nonzero mask (bit i: coefficient i != 0) in registers ----
  int16_t* coef = reinterpret_cast<int16_t*>(lds + L.coef);
  unsigned long long nzm[2] = {0ull, 0ull};
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int j = tid + SEG_T * sl;
    if (j >= nb) continue;
    const int m = j / 6, k = j - m * 6;
    const float* base;
    int pitch;
    if (k < 4) {
      const int col = m * 16 + (k & 1) * 8;
      base = Yp + (k >> 1) * 8 * pitch_y + col + (col >> 3);
      pitch = pitch_y;
    } else {
      const int col = m * 8;
      base = (k == 4 ? Cbp : Crp) + col + (col >> 3);
      pitch = pitch_c;
    }
    float d[8][8];
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) d[r][c] = base[r * pitch + c];
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
    const float* qs = k < 4 ? t.rl : t.rc;
    uint32_t* crow = reinterpret_cast<uint32_t*>(coef + j * SEG_CROW);
    unsigned long long nz = 0ull;
    int dc = 0;
#pragma unroll
    for (int i = 0; i < 64; i += 2) {
      const int s0 = kZZ.v[i], s1 = kZZ.v[i + 1];
      const float v0 = d[s0 >> 3][s0 & 7] * qs[s0], v1 = d[s1 >> 3][s1 & 7] * qs[s1];
      const int q0 = v0 < 0.f ? -(int)(0.5f - v0) : (int)(v0 + 0.5f);
      const int q1 = v1 < 0.f ? -(int)(0.5f - v1) : (int)(v1 + 0.5f);
      crow[i >> 1] = (uint32_t)(uint16_t)q0 | ((uint32_t)(uint16_t)q1 << 16);
      if (i == 0) dc = q0;
      else nz |= (unsigned long long)(q0 != 0) << i;
      nz |= (unsigned long long)(q1 != 0) << (i + 1);
    }
    nzm[sl] = nz;
    // AC symbol bits (host encoder's encode_block, without the DC part): nonzero coefficients only
    const int tc = k < 4 ? 0 : 1;
    int bits = 0, prev = 0;
    for (unsigned long long mm = nz; mm; mm &= mm - 1) {
      const int i = __builtin_ctzll(mm);
      int run = i - prev - 1;
      prev = i;
      for (; run > 15; run -= 16) bits += t.ac_len[tc][0xF0];
      const int n = nbits_i(coef[j * SEG_CROW + i]);
      bits += t.ac_len[tc][(run << 4) | n] + n;
    }
    if (prev != 63) bits += t.ac_len[tc][0x00];  // EOB unless the last coefficient is nonzero
    dcv[j] = dc;
    acb[j] = bits;
  }
  __syncthreads();

  // ---- 3. DC differences and bit offsets: thread t owns blocks 2t, 2t + 1 ----
  int tot[2] = {0, 0};
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const int j = 2 * tid + e;
    if (j < nb) {
      int comp;
      const int pj = prev_same(j, comp);
      const int diff = dcv[j] - (pj >= 0 ? dcv[pj] : 0);
      const int n = nbits_i(diff);
      dif[j] = diff;
      tot[e] = t.dc_len[comp > 0][n] + n + acb[j];
    }
  }
  int seg_bits;
  const int ex = seg_scan(tot[0] + tot[1], part, seg_bits);
  if (2 * tid < nb) boff[2 * tid] = ex;
  if (2 * tid + 1 < nb) boff[2 * tid + 1] = ex + tot[0];
  // zero the bit buffer (the planes are dead: every DCT read finished before the scan's barriers)
  uint32_t* bitbuf = reinterpret_cast<uint32_t*>(lds + L.planes);
  const int nbytes = (seg_bits + 7) >> 3, nwords = (nbytes + 3) >> 2;
  for (int w = tid; w < nwords; w += SEG_T) bitbuf[w] = 0u;
  __syncthreads();

  // ---- 4. Huffman codes into the bit buffer ----
#pragma unroll
  for (int sl = 0; sl < 2; ++sl) {
    const int j = tid + SEG_T * sl;
    if (j >= nb) continue;
    const int k = j % 6, tc = k < 4 ? 0 : 1;
    const int o = boff[j];
    LdsBits bo{bitbuf, o >> 5, 0u, o & 31};
    const int diff = dif[j];
    int n = nbits_i(diff);
    bo.put(t.dc_code[tc][n], t.dc_len[tc][n]);
    if (n) bo.put((uint32_t)(diff < 0 ? diff - 1 : diff), n);
    int prev = 0;
    for (unsigned long long mm = nzm[sl]; mm; mm &= mm - 1) {
      const int i = __builtin_ctzll(mm);
      int run = i - prev - 1;
      prev = i;
      for (; run > 15; run -= 16) bo.put(t.ac_code[tc][0xF0], t.ac_len[tc][0xF0]);
      const int v = coef[j * SEG_CROW + i];
      n = nbits_i(v);
      const int sym = (run << 4) | n;
      bo.put(t.ac_code[tc][sym], t.ac_len[tc][sym]);
      bo.put((uint32_t)(v < 0 ? v - 1 : v), n);
    }
    if (prev != 63) bo.put(t.ac_code[tc][0x00], t.ac_len[tc][0x00]);
    if (j == nb - 1) {  // the segment's last block: pad with 1-bits to the next byte boundary
      const int pad = nbytes * 8 - seg_bits;
      if (pad) bo.put((1u << pad) - 1u, pad);
    }
    bo.flush();
  }
  __syncthreads();

  // ---- 5. byte stuffing into the segment's staging slot (+ RSTm), 4 bytes per thread ----
  uint8_t* dst = stage + ((long long)img * g.mcuy + s) * g.seg_cap;
  int pos = 0;  // uniform
  for (int w0 = 0; w0 < nwords; w0 += SEG_T) {
    const int w = w0 + tid;
    uint32_t word = 0u;
    int valid = 0, n = 0;
    if (w < nwords) {
      word = bitbuf[w];
      valid = min(4, nbytes - 4 * w);
      n = valid;
      for (int b = 0; b < valid; ++b) n += ((word >> (24 - 8 * b)) & 0xFFu) == 0xFFu;
    }
    int total;
    int at = pos + seg_scan(n, part, total);
    for (int b = 0; b < valid; ++b) {
      const uint8_t v = (uint8_t)(word >> (24 - 8 * b));
      if (at + 2 <= g.seg_cap) {
        dst[at] = v;
        if (v == 0xFF) dst[at + 1] = 0;
      }
      at += v == 0xFF ? 2 : 1;
    }
    pos += total;
  }
  if (s + 1 < g.mcuy) {  // RSTm after every segment but the image's last
    if (tid == 0 && pos + 2 <= g.seg_cap) {
      dst[pos] = 0xFF;
      dst[pos + 1] = (uint8_t)(0xD0 + (s & 7));
    }
    pos += 2;
  }
  if (tid == 0) seg_len[(long long)img * g.mcuy + s] = pos;
}

constexpr int OFF_T = 1024;

// exclusive scan of the B * mcuy segment lengths -> seg_dst; off[b] = image b's first byte, off[B]
__global__ void __launch_bounds__(OFF_T) jpeg_offsets_kernel(int B, int mcuy, const int* __restrict__ seg_len,
                                                             long long* __restrict__ seg_dst,
                                                             long long* __restrict__ off) {
  __shared__ long long part[OFF_T / 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const long long n = (long long)B * mcuy;
  long long carry = 0;
  for (long long i0 = 0; i0 < n; i0 += OFF_T) {
    const long long i = i0 + tid;
    const long long v = i < n ? seg_len[i] : 0;
    long long x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const long long u = __shfl_up(x, o, 64);
      if (lane >= o) x += u;
    }
    if (lane == 63) part[wave] = x;
    __syncthreads();
    long long before = 0, total = 0;
    for (int w = 0; w < OFF_T / 64; ++w) {
      before += w < wave ? part[w] : 0;
      total += part[w];
    }
    if (i < n) {
      const long long d = carry + before + x - v;
      seg_dst[i] = d;
      if (i % mcuy == 0) off[i / mcuy] = d;
    }
    carry += total;
    __syncthreads();
  }
  if (tid == 0) off[B] = carry;
}

// one workgroup per segment: staging slot -> packed[seg_dst]
__global__ void __launch_bounds__(256) jpeg_copy_kernel(const uint8_t* __restrict__ stage, long long seg_cap,
                                                        const int* __restrict__ seg_len,
                                                        const long long* __restrict__ seg_dst,
                                                        uint8_t* __restrict__ packed) {
  const long long i = blockIdx.x;
  const uint32_t* src = reinterpret_cast<const uint32_t*>(stage + i * seg_cap);
  uint8_t* dst = packed + seg_dst[i];
  const int n = seg_len[i];
  for (int w = threadIdx.x; 4 * w < n; w += 256) {
    const uint32_t v = src[w];  // staging bytes in memory order (little-endian word)
    const int m = min(4, n - 4 * w);
    for (int b = 0; b < m; ++b) dst[4 * w + b] = (uint8_t)(v >> (8 * b));
  }
}

long long seg_cap_bytes(int W) {
  const long long nb = 6LL * ((W + 15) / 16);
  return ((2 * ((nb * SEG_BLK_BITS + 7) / 8 + 1) + 2) + 15) & ~15LL;
}

}  // namespace

int jpeg_gpu_max_width() { return 16 * SEG_MAX_MCUX; }

// Per-image capacity of the packed scans (worst case: every block at the code-length bound, every
// byte stuffed, a restart marker per MCU row)
long long jpeg_gpu_out_cap(int H, int W) { return (long long)((H + 15) / 16) * seg_cap_bytes(W); }

long long jpeg_gpu_ws_bytes(int B, int H, int W) {
  const long long segs = (long long)B * ((H + 15) / 16);
  auto r = [](long long b) { return (b + 255) & ~255LL; };
  return r(segs * seg_cap_bytes(W)) + r(segs * 4) + r(segs * 8);
}

int jpeg_gpu_launch(const uint8_t* rgb, int B, int H, int W, const void* tables, void* ws, uint8_t* packed,
                    long long* off, hipStream_t s) {
  if (B < 1 || H < 1 || W < 1 || W > jpeg_gpu_max_width() || B > 65535) return -1;
  SegGeo g{};
  g.B = B;
  g.H = H;
  g.W = W;
  g.mcux = (W + 15) / 16;
  g.mcuy = (H + 15) / 16;
  g.seg_cap = seg_cap_bytes(W);
  const long long segs = (long long)B * g.mcuy;
  uint8_t* p = reinterpret_cast<uint8_t*>(ws);
  auto take = [&p](size_t bytes) {
    uint8_t* q = p;
    p += (bytes + 255) & ~size_t(255);
    return q;
  };
  uint8_t* stage = take(segs * g.seg_cap);
  int* seg_len = reinterpret_cast<int*>(take(segs * 4));
  long long* seg_dst = reinterpret_cast<long long*>(take(segs * 8));
  static const bool attr_ok =  // > 64 KiB of dynamic LDS for the widest rows (gfx950: 160 KiB per CU)
      hipFuncSetAttribute((const void*)jpeg_segment_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          160 * 1024) == hipSuccess;
  if (!attr_ok) return -5;
  const SegLds L(g.mcux);
  const auto* t = reinterpret_cast<const dvjpeg::GpuTables*>(tables);
  hipLaunchKernelGGL(jpeg_segment_kernel, dim3((unsigned)g.mcuy, (unsigned)B), dim3(SEG_T), (size_t)L.total, s, rgb,
                     g, t, stage, seg_len);
  hipLaunchKernelGGL(jpeg_offsets_kernel, dim3(1), dim3(OFF_T), 0, s, B, g.mcuy, seg_len, seg_dst, off);
  hipLaunchKernelGGL(jpeg_copy_kernel, dim3((unsigned)segs), dim3(256), 0, s, stage, g.seg_cap, seg_len, seg_dst,
                     packed);
  return (int)hipGetLastError();
}

}  // namespace dv
