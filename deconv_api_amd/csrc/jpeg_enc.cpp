// Native baseline JPEG encoder + data-URL builder for the serving path (host C++, no GPU).
//
// The reference encodes each response with cv2.imencode('.jpg') (libjpeg, quality 95, 4:2:0) and
// then base64 + urllib.parse.quote (app/main.py:73-76). In Python, PIL's encoder holds the GIL
// (measured: 8 threads encode no faster than 1), which capped the service at ~550 req/s. This
// encoder writes the same kind of stream — baseline sequential DCT, JFIF, IJG quality-scaled
// standard quantization tables, standard (Annex K) Huffman tables, YCbCr 4:2:0 — and runs with
// the GIL released on a native thread pool, so response encoding scales with cores.
//
// Pipeline per image: RGB -> planar YCbCr (JFIF) -> 2x2 box-averaged chroma -> level shift ->
// separable float AAN 8x8 DCT-II (8 columns per vector op) -> quantize (round half away from zero) -> zig-zag -> Huffman with byte
// stuffing. Output bytes are then base64'd with the reference's quote() escaping folded in
// ('+' -> "%2B", '=' -> "%3D"; '/' and alphanumerics are kept).
#include "jpeg_enc.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace dvjpeg {
namespace {

// Annex K.1 example tables (natural order), scaled by the IJG quality rule.
const uint8_t kLumaQ[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                            14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                            18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                            49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const uint8_t kChromaQ[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                              24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                              99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// zig-zag index -> natural index
const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// Annex K.3 standard Huffman tables: code counts per length 1..16, then symbol values.
const uint8_t kDcLumaBits[16] = {0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0};
const uint8_t kDcLumaVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kDcChromaBits[16] = {0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0};
const uint8_t kDcChromaVal[12] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11};
const uint8_t kAcLumaBits[16] = {0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d};
const uint8_t kAcLumaVal[162] = {
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07, 0x22, 0x71,
    0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0, 0x24, 0x33, 0x62, 0x72,
    0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x34, 0x35, 0x36, 0x37,
    0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59,
    0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83,
    0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3,
    0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};
const uint8_t kAcChromaBits[16] = {0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77};
const uint8_t kAcChromaVal[162] = {
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71, 0x13, 0x22,
    0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0, 0x15, 0x62, 0x72, 0xd1,
    0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26, 0x27, 0x28, 0x29, 0x2a, 0x35, 0x36,
    0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58,
    0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a,
    0x82, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a,
    0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba,
    0xc2, 0xc3, 0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8, 0xf9, 0xfa};

struct HuffTable {
  uint16_t code[256];
  uint8_t len[256];
};

// canonical code assignment (Annex C)
HuffTable build_huff(const uint8_t* bits, const uint8_t* vals) {
  HuffTable t{};
  int code = 0, k = 0;
  for (int l = 1; l <= 16; ++l) {
    for (int i = 0; i < bits[l - 1]; ++i, ++k) {
      t.code[vals[k]] = (uint16_t)code++;
      t.len[vals[k]] = (uint8_t)l;
    }
    code <<= 1;
  }
  return t;
}

struct Tables {
  HuffTable dc[2], ac[2];
  Tables() {
    dc[0] = build_huff(kDcLumaBits, kDcLumaVal);
    dc[1] = build_huff(kDcChromaBits, kDcChromaVal);
    ac[0] = build_huff(kAcLumaBits, kAcLumaVal);
    ac[1] = build_huff(kAcChromaBits, kAcChromaVal);
  }
};
const Tables& tables() {
  static const Tables t;
  return t;
}

void scale_quant(const uint8_t* base, int quality, uint8_t* out) {
  quality = std::min(100, std::max(1, quality));
  const int s = quality < 50 ? 5000 / quality : 200 - quality * 2;
  for (int i = 0; i < 64; ++i) out[i] = (uint8_t)std::min(255, std::max(1, (base[i] * s + 50) / 100));
}

// Entropy-coded segment writer: 64-bit accumulator, whole bytes flushed into a preallocated
// buffer; the byte-stuffing check (0xFF -> FF 00) runs per flushed byte only when one is 0xFF.
class BitWriter {
 public:
  explicit BitWriter(uint8_t* buf) : p_(buf) {}
  inline void put(uint32_t code, int len) {
    acc_ = (acc_ << len) | (code & ((1u << len) - 1));
    n_ += len;
    if (n_ >= 32) {
      const uint32_t w = (uint32_t)(acc_ >> (n_ - 32));
      n_ -= 32;
      if (!has_ff(w)) {  // no 0xFF byte: fast path
        p_[0] = (uint8_t)(w >> 24);
        p_[1] = (uint8_t)(w >> 16);
        p_[2] = (uint8_t)(w >> 8);
        p_[3] = (uint8_t)w;
        p_ += 4;
      } else {
        for (int sh = 24; sh >= 0; sh -= 8) {
          const uint8_t b = (uint8_t)(w >> sh);
          *p_++ = b;
          if (b == 0xFF) *p_++ = 0;
        }
      }
    }
  }
  void flush() {  // remaining bits, padded with 1-bits to a byte boundary
    const int pad = (8 - (n_ & 7)) & 7;
    acc_ = (acc_ << pad) | ((1u << pad) - 1);
    n_ += pad;
    while (n_ > 0) {
      const uint8_t b = (uint8_t)(acc_ >> (n_ - 8));
      *p_++ = b;
      if (b == 0xFF) *p_++ = 0;
      n_ -= 8;
    }
  }
  uint8_t* pos() const { return p_; }

 private:
  static inline bool has_ff(uint32_t w) {
    return (w >> 24) == 0xFF || ((w >> 16) & 0xFF) == 0xFF || ((w >> 8) & 0xFF) == 0xFF || (w & 0xFF) == 0xFF;
  }
  uint8_t* p_;
  uint64_t acc_ = 0;
  int n_ = 0;
};

inline int nbits(int v) {
  v = v < 0 ? -v : v;
  return v ? 32 - __builtin_clz((unsigned)v) : 0;
}

// Scaled 8-point DCT-II (Arai-Agui-Nakajima factorization: 5 multiplies, 29 adds per 8 points),
// applied to 8 columns at once: each "element" is a row of 8 floats, so every butterfly is an
// 8-wide vector op the compiler maps to SIMD. Outputs are the true DCT-II coefficients times
// 8 * a(u) * a(v) (a(0) = 1, a(k) = sqrt(2) cos(k pi / 16)); that scale is folded into `qscale`.
inline void aan8_cols(float (&d)[8][8]) {
  float t0[8], t1[8], t2[8], t3[8], t4[8], t5[8], t6[8], t7[8];
  for (int i = 0; i < 8; ++i) {
    t0[i] = d[0][i] + d[7][i];
    t7[i] = d[0][i] - d[7][i];
    t1[i] = d[1][i] + d[6][i];
    t6[i] = d[1][i] - d[6][i];
    t2[i] = d[2][i] + d[5][i];
    t5[i] = d[2][i] - d[5][i];
    t3[i] = d[3][i] + d[4][i];
    t4[i] = d[3][i] - d[4][i];
  }
  for (int i = 0; i < 8; ++i) {
    const float e10 = t0[i] + t3[i], e13 = t0[i] - t3[i], e11 = t1[i] + t2[i], e12 = t1[i] - t2[i];
    d[0][i] = e10 + e11;
    d[4][i] = e10 - e11;
    const float z1 = (e12 + e13) * 0.707106781f;
    d[2][i] = e13 + z1;
    d[6][i] = e13 - z1;
    const float o10 = t4[i] + t5[i], o11 = t5[i] + t6[i], o12 = t6[i] + t7[i];
    const float z5 = (o10 - o12) * 0.382683433f;
    const float z2 = 0.541196100f * o10 + z5;
    const float z4 = 1.306562965f * o12 + z5;
    const float z3 = o11 * 0.707106781f;
    const float z11 = t7[i] + z3, z13 = t7[i] - z3;
    d[5][i] = z13 + z2;
    d[3][i] = z13 - z2;
    d[1][i] = z11 + z4;
    d[7][i] = z11 - z4;
  }
}

inline void transpose8(float (&d)[8][8]) {
  for (int r = 0; r < 8; ++r)
    for (int c = r + 1; c < 8; ++c) std::swap(d[r][c], d[c][r]);
}

// 8x8 block of level-shifted samples (rows = y) -> quantized coefficients in zig-zag order.
// After the vertical pass, a transpose and the horizontal pass, blk[u][v] holds horizontal
// frequency u / vertical frequency v, i.e. the coefficient at natural index v*8 + u; `qscale`
// and `zz_src` are laid out in that transposed order.
void fdct_quant(float (&blk)[8][8], const float* qscale_t, const uint8_t* zz_src, int16_t* zz) {
  aan8_cols(blk);
  transpose8(blk);
  aan8_cols(blk);
  const float* f = &blk[0][0];
  int16_t q[64];
  for (int k = 0; k < 64; ++k) {
    const float v = f[k] * qscale_t[k];
    q[k] = (int16_t)(v < 0.f ? -(int)(0.5f - v) : (int)(v + 0.5f));
  }
  for (int k = 0; k < 64; ++k) zz[k] = q[zz_src[k]];
}

void encode_block(BitWriter& bw, const int16_t* zz, int& pred, const HuffTable& dc, const HuffTable& ac) {
  const int diff = zz[0] - pred;
  pred = zz[0];
  int n = nbits(diff);
  bw.put(dc.code[n], dc.len[n]);
  if (n) bw.put(diff < 0 ? diff - 1 : diff, n);
  int run = 0;
  for (int k = 1; k < 64; ++k) {
    const int v = zz[k];
    if (v == 0) {
      ++run;
      continue;
    }
    while (run > 15) {
      bw.put(ac.code[0xF0], ac.len[0xF0]);  // ZRL
      run -= 16;
    }
    n = nbits(v);
    const int sym = (run << 4) | n;
    bw.put(ac.code[sym], ac.len[sym]);
    bw.put(v < 0 ? v - 1 : v, n);
    run = 0;
  }
  if (run) bw.put(ac.code[0x00], ac.len[0x00]);  // EOB
}

void put16(std::string& o, int v) {
  o.push_back((char)(v >> 8));
  o.push_back((char)(v & 0xFF));
}

void write_dht(std::string& o, int cls_id, const uint8_t* bits, const uint8_t* vals, int nvals) {
  o.append("\xFF\xC4", 2);
  put16(o, 2 + 1 + 16 + nvals);
  o.push_back((char)cls_id);
  o.append(reinterpret_cast<const char*>(bits), 16);
  o.append(reinterpret_cast<const char*>(vals), nvals);
}

}  // namespace

namespace {

// Everything about one (H, W, quality, segments) encode that does not depend on pixel values.
struct Plan {
  int H, W, mcux, mcuy, rows_per_seg, nseg;
  float rl[64], rc[64];  // quantizer reciprocals, transposed (u-major) coefficient layout
  uint8_t zz_src[64];
  std::string header;    // SOI .. SOS
};

Plan make_plan(int H, int W, int quality, int segments) {
  Plan p;
  p.H = H;
  p.W = W;
  p.mcux = (W + 15) / 16;
  p.mcuy = (H + 15) / 16;
  segments = std::max(1, std::min(segments, p.mcuy));
  p.rows_per_seg = (p.mcuy + segments - 1) / segments;
  p.nseg = (p.mcuy + p.rows_per_seg - 1) / p.rows_per_seg;
  uint8_t ql[64], qc[64];
  scale_quant(kLumaQ, quality, ql);
  scale_quant(kChromaQ, quality, qc);
  double a[8];
  a[0] = 1.0;
  for (int k = 1; k < 8; ++k) a[k] = std::sqrt(2.0) * std::cos(k * M_PI / 16.0);
  for (int u = 0; u < 8; ++u)
    for (int v = 0; v < 8; ++v) {
      const int nat = v * 8 + u;
      const double sc = 8.0 * a[u] * a[v];
      p.rl[u * 8 + v] = (float)(1.0 / (ql[nat] * sc));
      p.rc[u * 8 + v] = (float)(1.0 / (qc[nat] * sc));
    }
  for (int k = 0; k < 64; ++k) p.zz_src[k] = (uint8_t)((kZigzag[k] % 8) * 8 + kZigzag[k] / 8);
  std::string& o = p.header;
  o.append("\xFF\xD8", 2);  // SOI
  // APP0 JFIF 1.01, no density units, 1:1
  o.append("\xFF\xE0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00", 18);
  // DQT: two 8-bit tables in zig-zag order
  o.append("\xFF\xDB", 2);
  put16(o, 2 + 2 * 65);
  o.push_back(0);
  for (int k = 0; k < 64; ++k) o.push_back((char)ql[kZigzag[k]]);
  o.push_back(1);
  for (int k = 0; k < 64; ++k) o.push_back((char)qc[kZigzag[k]]);
  // SOF0: 8-bit, 3 components, Y 2x2 (table 0), Cb/Cr 1x1 (table 1)
  o.append("\xFF\xC0", 2);
  put16(o, 17);
  o.push_back(8);
  put16(o, H);
  put16(o, W);
  o.push_back(3);
  o.append("\x01\x22\x00\x02\x11\x01\x03\x11\x01", 9);
  write_dht(o, 0x00, kDcLumaBits, kDcLumaVal, 12);
  write_dht(o, 0x10, kAcLumaBits, kAcLumaVal, 162);
  write_dht(o, 0x01, kDcChromaBits, kDcChromaVal, 12);
  write_dht(o, 0x11, kAcChromaBits, kAcChromaVal, 162);
  if (p.nseg > 1) {  // DRI: a restart marker after every segment of rows_per_seg MCU rows
    o.append("\xFF\xDD", 2);
    put16(o, 4);
    put16(o, p.rows_per_seg * p.mcux);
  }
  // SOS
  o.append("\xFF\xDA", 2);
  put16(o, 12);
  o.append("\x03\x01\x00\x02\x11\x03\x11\x00\x3F\x00", 10);
  return p;
}

// Entropy-coded data of MCU rows [seg*rows_per_seg, ...) (byte-stuffed, padded to a byte):
// colour conversion of just those pixel rows, DCT, quantization and Huffman coding. DC
// predictors start at 0, as they do after a restart marker. Compiled twice (AVX2/FMA and
// baseline x86-64) and dispatched at load time (an ifunc; sanitizer builds, whose runtime is not up
// when ifunc resolvers run, use the baseline version only: -DDVJPEG_NO_CLONES).
#ifndef DVJPEG_NO_CLONES
__attribute__((target_clones("arch=haswell", "default")))
#endif
void encode_segment(const Plan& p, const uint8_t* rgb, int seg, std::string& out) {
  const int H = p.H, W = p.W;
  const int r0 = seg * p.rows_per_seg, r1 = std::min(p.mcuy, r0 + p.rows_per_seg);
  const int PW = p.mcux * 16, SH = (r1 - r0) * 16, CW = PW / 2;
  static thread_local std::vector<float> scratch;
  static thread_local std::vector<uint8_t> ecs;
  const size_t plane = (size_t)PW * SH, cplane = (size_t)CW * (SH / 2);
  if (scratch.size() < 3 * plane + 2 * cplane) scratch.resize(3 * plane + 2 * cplane);
  float* Yp = scratch.data();
  float* Cbp = Yp + plane;
  float* Crp = Cbp + plane;
  float* Cb2 = Crp + plane;
  float* Cr2 = Cb2 + cplane;
  // planar YCbCr of the segment's pixel rows (edge replication past the image)
  for (int py = 0; py < SH; ++py) {
    const uint8_t* row = rgb + (size_t)std::min(r0 * 16 + py, H - 1) * W * 3;
    float* yr = Yp + (size_t)py * PW;
    float* br = Cbp + (size_t)py * PW;
    float* rr = Crp + (size_t)py * PW;
    for (int px = 0; px < W; ++px) {
      const float r = row[px * 3], g = row[px * 3 + 1], b = row[px * 3 + 2];
      yr[px] = 0.299f * r + 0.587f * g + 0.114f * b - 128.f;
      br[px] = -0.168736f * r - 0.331264f * g + 0.5f * b;
      rr[px] = 0.5f * r - 0.418688f * g - 0.081312f * b;
    }
    for (int px = W; px < PW; ++px) {
      yr[px] = yr[W - 1];
      br[px] = br[W - 1];
      rr[px] = rr[W - 1];
    }
  }
  for (int cy = 0; cy < SH / 2; ++cy) {
    const float* b0 = Cbp + (size_t)(2 * cy) * PW;
    const float* q0 = Crp + (size_t)(2 * cy) * PW;
    float* bo = Cb2 + (size_t)cy * CW;
    float* ro = Cr2 + (size_t)cy * CW;
    for (int cx = 0; cx < CW; ++cx) {
      bo[cx] = 0.25f * (b0[2 * cx] + b0[2 * cx + 1] + b0[PW + 2 * cx] + b0[PW + 2 * cx + 1]);
      ro[cx] = 0.25f * (q0[2 * cx] + q0[2 * cx + 1] + q0[PW + 2 * cx] + q0[PW + 2 * cx + 1]);
    }
  }
  // worst case per 8x8 block: 64 codes of <= 16 + 11 bits, doubled by stuffing
  const size_t ecs_max = (size_t)p.mcux * (r1 - r0) * 6 * 64 * 27 * 2 / 8 + 64;
  if (ecs.size() < ecs_max) ecs.resize(ecs_max);
  const auto& T = tables();
  BitWriter bw(ecs.data());
  int pred[3] = {0, 0, 0};
  float blk[8][8];
  int16_t zz[64];
  auto load = [&blk](const float* src, int ld) {
    for (int r = 0; r < 8; ++r)
      for (int c = 0; c < 8; ++c) blk[r][c] = src[(size_t)r * ld + c];
  };
  for (int my = 0; my < r1 - r0; ++my)
    for (int mx = 0; mx < p.mcux; ++mx) {
      for (int k = 0; k < 4; ++k) {
        load(Yp + (size_t)(my * 16 + (k >> 1) * 8) * PW + mx * 16 + (k & 1) * 8, PW);
        fdct_quant(blk, p.rl, p.zz_src, zz);
        encode_block(bw, zz, pred[0], T.dc[0], T.ac[0]);
      }
      load(Cb2 + (size_t)(my * 8) * CW + mx * 8, CW);
      fdct_quant(blk, p.rc, p.zz_src, zz);
      encode_block(bw, zz, pred[1], T.dc[1], T.ac[1]);
      load(Cr2 + (size_t)(my * 8) * CW + mx * 8, CW);
      fdct_quant(blk, p.rc, p.zz_src, zz);
      encode_block(bw, zz, pred[2], T.dc[1], T.ac[1]);
    }
  bw.flush();
  out.assign(reinterpret_cast<const char*>(ecs.data()), bw.pos() - ecs.data());
}

std::string assemble(const Plan& p, const std::vector<std::string>& segs) {
  size_t n = p.header.size() + 2;
  for (auto& sg : segs) n += sg.size() + 2;
  std::string o;
  o.reserve(n);
  o += p.header;
  for (int i = 0; i < (int)segs.size(); ++i) {
    o += segs[i];
    if (i + 1 < (int)segs.size()) {  // RSTm, m = i mod 8
      o.push_back((char)0xFF);
      o.push_back((char)(0xD0 + (i & 7)));
    }
  }
  o.append("\xFF\xD9", 2);  // EOI
  return o;
}

}  // namespace

GpuTables gpu_tables(int quality) {
  const Plan p = make_plan(16, 16, quality, 1);
  GpuTables g{};
  std::memcpy(g.rl, p.rl, sizeof g.rl);
  std::memcpy(g.rc, p.rc, sizeof g.rc);
  std::memcpy(g.zz_src, p.zz_src, sizeof g.zz_src);
  const auto& T = tables();
  for (int c = 0; c < 2; ++c) {
    for (int i = 0; i < 12; ++i) {
      g.dc_code[c][i] = T.dc[c].code[i];
      g.dc_len[c][i] = T.dc[c].len[i];
    }
    for (int i = 0; i < 256; ++i) {
      g.ac_code[c][i] = T.ac[c].code[i];
      g.ac_len[c][i] = T.ac[c].len[i];
    }
  }
  return g;
}

std::string jpeg_header(int H, int W, int quality, int restart_rows) {
  const int mcuy = (H + 15) / 16;
  return make_plan(H, W, quality, restart_rows > 0 ? (mcuy + restart_rows - 1) / restart_rows : 1).header;
}

std::vector<std::string> data_urls_from_scans(const std::string& header, const uint8_t* scans, const int64_t* off,
                                              int B, const std::string& prefix, int threads) {
  std::vector<std::string> out(B);
  std::atomic<int> next{0};
  auto work = [&]() {
    std::string jpg;
    for (int b = next++; b < B; b = next++) {
      jpg.assign(header);
      jpg.append(reinterpret_cast<const char*>(scans + off[b]), (size_t)(off[b + 1] - off[b]));
      jpg.append("\xFF\xD9", 2);  // EOI
      out[b] = data_url(jpg, prefix);
    }
  };
  const int nt = std::max(1, std::min(threads, B));
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(work);
  work();
  for (auto& th : pool) th.join();
  return out;
}

std::string encode_jpeg(const uint8_t* rgb, int H, int W, int quality, int segments) {
  const Plan p = make_plan(H, W, quality, segments);
  std::vector<std::string> segs(p.nseg);
  for (int sg = 0; sg < p.nseg; ++sg) encode_segment(p, rgb, sg, segs[sg]);
  return assemble(p, segs);
}

std::string data_url(const std::string& jpeg, const std::string& prefix) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
  std::string o;
  o.reserve(prefix.size() + jpeg.size() * 4 / 3 + 64);
  o += prefix;
  auto emit = [&o](char c) {
    if (c == '+')
      o.append("%2B", 3);
    else
      o.push_back(c);
  };
  const auto* s = reinterpret_cast<const uint8_t*>(jpeg.data());
  const size_t n = jpeg.size();
  size_t i = 0;
  for (; i + 3 <= n; i += 3) {
    const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8 | s[i + 2];
    emit(A[v >> 18]);
    emit(A[(v >> 12) & 63]);
    emit(A[(v >> 6) & 63]);
    emit(A[v & 63]);
  }
  if (n - i == 1) {
    const uint32_t v = (uint32_t)s[i] << 16;
    emit(A[v >> 18]);
    emit(A[(v >> 12) & 63]);
    o.append("%3D%3D", 6);
  } else if (n - i == 2) {
    const uint32_t v = (uint32_t)s[i] << 16 | (uint32_t)s[i + 1] << 8;
    emit(A[v >> 18]);
    emit(A[(v >> 12) & 63]);
    emit(A[(v >> 6) & 63]);
    o.append("%3D", 3);
  }
  return o;
}

std::vector<std::string> encode_data_urls(const uint8_t* rgb, int B, int H, int W, int quality,
                                          const std::string& prefix, int threads) {
  std::vector<std::string> out(B);
  if (B == 0) return out;
  threads = std::max(1, threads);
  // few images: split each into restart-marker segments so all threads share every image
  const int segments = std::max(1, std::min((threads + B - 1) / B, (H + 15) / 16));
  const Plan p = make_plan(H, W, quality, segments);
  const size_t stride = (size_t)H * W * 3;
  std::vector<std::vector<std::string>> segs(B, std::vector<std::string>(p.nseg));
  const int tasks = B * p.nseg;
  auto run = [threads](int n, const auto& fn) {  // fn(i) for i < n on up to `threads` threads
    std::atomic<int> next{0};
    auto work = [&]() {
      for (int i = next++; i < n; i = next++) fn(i);
    };
    const int nt = std::min(threads, n);
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; ++t) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  };
  // phase 1: every (image, segment); phase 2 (after all segments exist): stitch + base64
  run(tasks, [&](int t) { encode_segment(p, rgb + (t / p.nseg) * stride, t % p.nseg, segs[t / p.nseg][t % p.nseg]); });
  run(B, [&](int b) { out[b] = data_url(assemble(p, segs[b]), prefix); });
  return out;
}

// Request side: the payload of a data URL (text between the first and second comma, the
// reference's uri.split(',')[1]) base64-decoded the way CPython's non-strict a2b_base64 does it
// (base64.b64decode(s), validate=False): characters outside the alphabet are skipped, a '=' that
// completes a quad (at least two data characters before it) ends the input, and a quad left open
// at the end is an error. Returns false with CPython's message on error.
bool data_url_b64decode(const char* uri, size_t n, std::string& out, std::string& err) {
  static const struct Table {
    int8_t v[256];
    Table() {
      for (int i = 0; i < 256; ++i) v[i] = -1;
      const char* a = "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/";
      for (int i = 0; i < 64; ++i) v[(uint8_t)a[i]] = (int8_t)i;
    }
  } T;
  const char* c1 = static_cast<const char*>(std::memchr(uri, ',', n));
  if (c1 == nullptr) {
    err = "not a data URL";
    return false;
  }
  const char* p = c1 + 1;
  const char* end = uri + n;
  if (const char* c2 = static_cast<const char*>(std::memchr(p, ',', (size_t)(end - p)))) end = c2;
  out.resize((size_t)(end - p) / 4 * 3 + 3);
  uint8_t* o = reinterpret_cast<uint8_t*>(&out[0]);
  int quad = 0, pads = 0;
  long long ndata = 0;
  uint32_t left = 0;
  bool stop = false;
  while (p < end && !stop) {
    // fast path: whole quads of alphabet characters (the common, clean payload)
    while (quad == 0 && end - p >= 4) {
      const int a = T.v[(uint8_t)p[0]], b = T.v[(uint8_t)p[1]], c = T.v[(uint8_t)p[2]], d = T.v[(uint8_t)p[3]];
      if ((a | b | c | d) < 0) break;
      const uint32_t w = ((uint32_t)a << 18) | ((uint32_t)b << 12) | ((uint32_t)c << 6) | (uint32_t)d;
      o[0] = (uint8_t)(w >> 16);
      o[1] = (uint8_t)(w >> 8);
      o[2] = (uint8_t)w;
      o += 3;
      p += 4;
      ndata += 4;
      pads = 0;
    }
    if (p >= end) break;
    const uint8_t ch = (uint8_t)*p++;
    if (ch == '=') {
      if (quad >= 2 && quad + ++pads >= 4) stop = true;  // a completed pad sequence ends the input
      continue;
    }
    const int v = T.v[ch];
    if (v < 0) continue;
    pads = 0;
    ++ndata;
    switch (quad) {
      case 0: left = (uint32_t)v; quad = 1; break;
      case 1: *o++ = (uint8_t)((left << 2) | (uint32_t)(v >> 4)); left = (uint32_t)v & 0xF; quad = 2; break;
      case 2: *o++ = (uint8_t)((left << 4) | (uint32_t)(v >> 2)); left = (uint32_t)v & 0x3; quad = 3; break;
      default: *o++ = (uint8_t)((left << 6) | (uint32_t)v); quad = 0; break;
    }
  }
  out.resize((size_t)(o - reinterpret_cast<uint8_t*>(&out[0])));
  if (stop) return true;
  if (quad == 1) {
    err = "Invalid base64-encoded string: number of data characters (" + std::to_string(ndata) +
          ") cannot be 1 more than a multiple of 4";
    return false;
  }
  if (quad != 0) {
    err = "Incorrect padding";
    return false;
  }
  return true;
}

}  // namespace dvjpeg
