// Halo-stream 3x3 conv for gfx950 (MI355X): 3x3 / stride 1 / pad 1, C % 32 == 0, 64 or 128 output
// channels, 16-bit in/out, fp32 accumulation. Targets the 112x112 layers of VGG16 whose implicit-GEMM
// launches are bound by the A-operand LDS-DMA stream (block2 forward and conv-downs at B*K = 1024):
// the implicit GEMM re-fetches every input pixel once per tap (9x) from L2, this kernel once.
//
// Work decomposition: one 512-thread workgroup per 16 x 32 output tile (512 pixels) x all output
// channels. K runs as (32-channel chunk c, tap t): the (16+2) x (32+2) input halo of chunk c is staged
// ONCE into LDS and serves all 9 taps (each tap reads a shifted window of it); the weights of one
// (chunk, tap) step (OC x 32 channels) stream through a 3-slot LDS ring. Both are staged by LDS-DMA
// (`buffer_load_dwordx4 ... lds`), with conv zero padding / the image border from the buffer range
// check (an out-of-range offset reads 0).
//
// MFMA `v_mfma_f32_32x32x16_*` transposed: A = weights (32 output channels x 16 K), B = pixels (16 K x
// 32 pixels of one tile row), so C holds 4 consecutive output channels of one pixel per register
// quad and the epilogue packs them into one 8-B store per lane (lanes h = 0/1 cover 16 contiguous B).
//
// LDS layouts: a halo pixel and a weight row both hold 32 channels (64 B) in an 80-B slot (5 bank
// slots of 16 B): the 32 rows a fragment read touches start at 5j mod 16 = a permutation of the 16 slots
// for every ds_read_b128 lane group ({0-3,12-15,20-27} etc.) and any base -> conflict-free for every
// tap shift. The DMA destination stays lane-linear (1 KiB per wave instruction); the per-lane SOURCE
// maps slot s -> (pixel s/5, chunk s%5), chunk 4 is the pad (reads out of range -> 0).
//
// Pipeline per step k = 9c + t (one barrier per step): wait until this wave's DMA of B(k) landed
// (counted vmcnt: every wave issues the same number of DMAs per step, dummy out-of-range ones pad the
// count), barrier, issue [halo(c+1) if t == 0] + B(k+RING-1) (4-5 steps of weight prefetch: one step is
// only ~0.25-0.5 us of MFMA work, less than an L2 round trip), then 2 x (FN + 2) fragment reads and
// 4 FN MFMAs.
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <cstring>

namespace dv {

namespace {

constexpr int HS_TH = 16, HS_TW = 32;                 // output tile
constexpr int HS_HH = HS_TH + 2, HS_HW = HS_TW + 2;   // 18 x 34 halo
constexpr int HS_PS = 80;                              // bytes per halo pixel / weight row slot
constexpr int HS_HSLOTS = HS_HH * HS_HW * 5;           // 3060 16-B slots
constexpr int HS_HI = (HS_HSLOTS + 511) / 512;         // halo DMA instructions per wave (6)
constexpr int HS_HBUF = HS_HI * 8 * 1024;              // 49152 B per halo buffer (incl. overrun of the last)
constexpr uint32_t HS_OOB = 0x80000000u;

typedef int hs_i32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA of 16 B per lane as inline asm (as conv_smalln.hip's dma16_asm): with the intrinsic the
// compiler's waitcnt pass drains the prefetch (vmcnt(0)) before ds_reads that reuse the offset VGPR;
// here the only waits are the kernel's counted ones. M0 = LDS base of the 64 x 16 B destination.
__device__ __forceinline__ void hs_dma16(const hs_i32x4& rsrc, const uint8_t* lds_dst, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst)), "v"(voff), "s"(rsrc)
               : "memory");
}

__device__ __forceinline__ void hs_dma4(const hs_i32x4& rsrc, const uint8_t* lds_dst, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds_dst)), "v"(voff), "s"(rsrc)
               : "memory");
}

__device__ __forceinline__ hs_i32x4 hs_rsrc(const void* base, long long bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  hs_i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
  r.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(b >> 32) & 0xFFFFu));
  r.z = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)bytes));
  r.w = 0x00020000;
  return r;
}

template <int N>
__device__ __forceinline__ void hs_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

typedef __attribute__((ext_vector_type(16))) float f32x16;

template <int DT>
__device__ __forceinline__ f32x16 hs_mfma(const typename Vec8<DT>::type& a, const typename Vec8<DT>::type& b,
                                          const f32x16& c) {
  if constexpr (DT == DT_BF16) return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  else return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

}  // namespace

// OCT: output channels per workgroup (= OCpad, 64 or 128); POOL: fused 2x2 max-pool + switch epilogue.
// Any symmetric pad (0: 'valid', 1: 'same', 2: the full-pad input gradient of a 'valid' conv): the
// halo of output tile (ty0, tx0) starts at input (ty0 - pad, tx0 - pad); output OH x OW.
// NB1 (one 32-channel chunk, C == 32): ONE halo buffer (72 KiB of LDS -> 2 workgroups per CU; with a
// single chunk there is no next-chunk prefetch to double-buffer).
// emask (non-pool): the output is zeroed where emask <= 0 (an input gradient masked by its ReLU).
// LEPI (plain / emask epilogue; host: OC, out_ld, emask_ld % 8 == 0, 16-B aligned rows): the C tile goes
// through LDS one tile row per pass (32 px x OCT channels per wave, in the operand buffers freed after the K
// loop) and every lane stores whole 16-B chunks, OCT / 8 lanes per pixel: each store instruction writes
// complete pixel rows instead of 32 pixels x 16 B (as hs16's LEPI and KW3P's LDS epilogue).
template <int DT, int OCT, bool POOL, int RING, bool NB1 = false, bool LEPI = false>
__global__ void __launch_bounds__(512, NB1 && OCT == 64 ? 4 : 1) conv3x3_hs_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
  static_assert(!LEPI || !POOL, "LDS epilogue: plain / emask outputs");
  constexpr int FN = OCT / 32;  // 32-channel A blocks per wave
  // weights of one step: OCT rows x 80 B. OCT = 128: 10 KiB = one 1-KiB dwordx4 DMA + one 256-B dword
  // DMA per wave (exact); OCT = 64: 5 KiB in one dwordx4 DMA per wave, 3 of them out-of-range dummies
  constexpr int BI = OCT == 128 ? 2 : 1;          // weight DMA instructions per wave and step
  constexpr int BSLOT = OCT == 128 ? 10240 : 8192;
  constexpr int LA = RING - 1;                    // B(k + RING - 1) is issued at step k
  constexpr int STEPS_PER_CHUNK = 9;
  typedef typename Vec8<DT>::type v8;
  constexpr int NHB = NB1 ? 1 : 2;  // halo buffers
  __shared__ __attribute__((aligned(16))) uint8_t smem[NHB * HS_HBUF + RING * BSLOT];
  uint8_t* halo = smem;
  uint8_t* ring = smem + NHB * HS_HBUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 5, px = lane & 31;
  const int H = a.H, W = a.W, C = a.C;
  const int per_img = tiles_x * tiles_y;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / per_img;
  const int tr = bid - n * per_img;
  const int ty0 = (tr / tiles_x) * HS_TH, tx0 = (tr % tiles_x) * HS_TW;

  const long long img = (long long)H * W * a.x_ld;
  const hs_i32x4 xr = hs_rsrc(a.x + (long long)n * img, img * 2);
  const hs_i32x4 wr = hs_rsrc(a.w, (long long)a.OCpad * a.Kpad * 2);

  // per-lane DMA source offsets (chunk 0 / tap 0); slot s of instruction m -> (row s/5, 16-B chunk s%5)
  uint32_t hoff[HS_HI];
#pragma unroll
  for (int u = 0; u < HS_HI; ++u) {
    const int s = (u * 8 + wave) * 64 + lane;
    const int p = s / 5, q = s - 5 * (s / 5);
    const int hy = p / HS_HW, hx = p - HS_HW * (p / HS_HW);
    const int y = ty0 - a.pad_h + hy, x = tx0 - a.pad_w + hx;
    const bool ok = q < 4 && p < HS_HH * HS_HW && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    hoff[u] = ok ? (uint32_t)((((long long)y * W + x) * a.x_ld + q * 8) * 2) : HS_OOB;
  }
  uint32_t woff[BI];
  {
    const int s = wave * 64 + lane;  // dwordx4 part: 16-B slot s of the ring slot
    const int r = s / 5, q = s - 5 * (s / 5);
    woff[0] = (q < 4 && r < OCT) ? (uint32_t)(((long long)r * a.Kpad + q * 8) * 2) : HS_OOB;
    if constexpr (BI == 2) {  // dword part: bytes 8192 + 256 wave + 4 lane
      const int s2 = 512 + wave * 16 + (lane >> 2), d = lane & 3;
      const int r2 = s2 / 5, q2 = s2 - 5 * (s2 / 5);
      woff[BI - 1] = q2 < 4 ? (uint32_t)(((long long)r2 * a.Kpad + q2 * 8) * 2 + d * 4) : HS_OOB;
    }
  }
  const int nch = C / 32;
  const int nsteps = nch * STEPS_PER_CHUNK;
  auto issue_halo = [&](int c, int buf) {  // c >= nch: dummy (out-of-range) loads keep the count uniform
    const uint32_t add = c < nch ? (uint32_t)(c * 64) : HS_OOB;  // chunk c: channels 32c.. (64 B)
#pragma unroll
    for (int u = 0; u < HS_HI; ++u)
      hs_dma16(xr, halo + buf * HS_HBUF + (u * 8 + wave) * 1024,
               hoff[u] == HS_OOB || add == HS_OOB ? HS_OOB : hoff[u] + add);
  };
  auto issue_w = [&](int k) {  // weights of step k = 9c + t: K columns t*C + 32c .. +32
    const int c = k / STEPS_PER_CHUNK, t = k - STEPS_PER_CHUNK * (k / STEPS_PER_CHUNK);
    const uint32_t add = k < nsteps ? (uint32_t)((t * C + c * 32) * 2) : HS_OOB;
    uint8_t* dst = ring + (k % RING) * BSLOT;
    hs_dma16(wr, dst + wave * 1024, woff[0] == HS_OOB || add == HS_OOB ? HS_OOB : woff[0] + add);
    if constexpr (BI == 2)
      hs_dma4(wr, dst + 8192 + wave * 256, woff[1] == HS_OOB || add == HS_OOB ? HS_OOB : woff[1] + add);
  };

  f32x16 acc[2][FN];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // fragment read bases: weights row 32j + px, pixel (tile row 2*wave + i, column px), chunk 2s + h
  const int wrow = px * HS_PS + h * 16;
  const int prow = ((2 * wave) * HS_HW + px) * HS_PS + h * 16;

  issue_halo(0, 0);
#pragma unroll
  for (int p = 0; p < LA; ++p) issue_w(p);
  for (int c = 0; c < nch; ++c) {
    const uint8_t* hb = halo + (NB1 ? 0 : (c & 1)) * HS_HBUF + prow;
#pragma unroll
    for (int t = 0; t < STEPS_PER_CHUNK; ++t) {
      const int k = c * STEPS_PER_CHUNK + t;
      // younger than B(k): the B's of steps k-LA+1 .. k-1 (or of the prologue), plus halo(c+1) when
      // step 9c lies in that window (1 <= t <= LA-1; NB1 issues no next-chunk halo)
      if (!NB1 && t >= 1 && t <= LA - 1) hs_wait<(LA - 1) * BI + HS_HI>();
      else hs_wait<(LA - 1) * BI>();
      __builtin_amdgcn_s_barrier();
      if (!NB1 && t == 0) issue_halo(c + 1, (c + 1) & 1);
      issue_w(k + LA);
      const uint8_t* wb = ring + (k % RING) * BSLOT + wrow;
      const int kh = t / 3, kw = t % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        v8 wf[FN], pf[2];
#pragma unroll
        for (int j = 0; j < FN; ++j) wf[j] = *reinterpret_cast<const v8*>(wb + j * 32 * HS_PS + s * 32);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          pf[i] = *reinterpret_cast<const v8*>(hb + ((i + kh) * HS_HW + kw) * HS_PS + s * 32);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = hs_mfma<DT>(wf[j], pf[i], acc[i][j]);
      }
    }
  }
  hs_wait<0>();  // the dummy DMAs of the last steps land before the workgroup retires

  // epilogue: lane = pixel (tile row 2*wave + i, column px); register r of block j = output channel
  // 32j + 8(r >> 2) + 4h + (r & 3): 4 consecutive channels -> one 8-B store
  const int ox = tx0 + px;
  if constexpr (LEPI) {
    constexpr int ROWB = OCT * 2, CPR = OCT / 8, PPI = 64 / CPR, NT = 32 / PPI;
    static_assert(8 * 32 * ROWB <= (int)sizeof(smem), "LDS epilogue slices");
    float4 bv[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        bv[j][g] = a.bias ? *reinterpret_cast<const float4*>(a.bias + 32 * j + 8 * g + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
    const float lo = a.relu ? 0.f : -INFINITY;
    uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
    uint8_t* wreg = smem + wave * 32 * ROWB;
    const int pc = lane % CPR;
    __syncthreads();  // every wave's last fragment reads of the halo / weight buffers are done
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const float v0 = fmaxf(acc[i][j][4 * g + 0] + bv[j][g].x, lo), v1 = fmaxf(acc[i][j][4 * g + 1] + bv[j][g].y, lo);
          const float v2 = fmaxf(acc[i][j][4 * g + 2] + bv[j][g].z, lo), v3 = fmaxf(acc[i][j][4 * g + 3] + bv[j][g].w, lo);
          const int ch = 4 * j + g;  // 16-B chunk; lanes h = 0 / 1 hold its two halves
          *reinterpret_cast<uint2*>(wreg + px * ROWB + ((ch ^ (px & (CPR - 1))) << 4) + h * 8) =
              make_uint2(pack2<DT>(v0, v1), pack2<DT>(v2, v3));
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: this wave's writes before its reads
      const int oy = ty0 + 2 * wave + i;
      uint4 em[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {  // every output-mask load of the row before its first store
        const int lp = t * PPI + lane / CPR, lc = pc ^ (lp & (CPR - 1)), x = tx0 + lp;
        const long long pix = ((long long)n * a.OH + oy) * a.OW + x;
        em[t] = make_uint4(0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u);  // any > 0
        if (a.ebits && oy < a.OH && x < a.OW && lc * 8 < a.OC)  // 1-bit mask: one byte per chunk
          em[t].x = a.ebits[pix * a.ebits_ld + lc];
        else if (a.emask && oy < a.OH && x < a.OW && lc * 8 < a.OC &&
                 DV_BOUNDS(pix * a.emask_ld + lc * 8, 8, a.emask_elems, "halo-stream emask"))
          em[t] = *reinterpret_cast<const uint4*>(a.emask + pix * a.emask_ld + lc * 8);
      }
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int lp = t * PPI + lane / CPR, lc = pc ^ (lp & (CPR - 1)), x = tx0 + lp;
        uint4 v = *reinterpret_cast<const uint4*>(wreg + lp * ROWB + pc * 16);
        if (a.ebits) {
          v = mask_bits8(v, em[t].x);
        } else if (a.emask) {
          v.x = mask_pos_pk(v.x, em[t].x);
          v.y = mask_pos_pk(v.y, em[t].y);
          v.z = mask_pos_pk(v.z, em[t].z);
          v.w = mask_pos_pk(v.w, em[t].w);
        }
        const long long pix = ((long long)n * a.OH + oy) * a.OW + x;
        if (oy < a.OH && x < a.OW && lc * 8 < a.OC && DV_BOUNDS(pix * a.out_ld + lc * 8, 8, a.out_elems, "halo-stream out")) {
          *reinterpret_cast<uint4*>(out + pix * a.out_ld + lc * 8) = v;
          if (a.obits) a.obits[pix * a.obits_ld + lc] = (uint8_t)pos_bits8(v);
        }
      }
    }
    return;
  }
  if (ox >= a.OW) return;
  // the lane's bias values (the same for both pixel rows), all loads in flight together
  float4 bv[FN][4];
#pragma unroll
  for (int j = 0; j < FN; ++j)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      bv[j][g] = a.bias ? *reinterpret_cast<const float4*>(a.bias + 32 * j + 8 * g + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float lo = a.relu ? 0.f : -INFINITY;
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
  if constexpr (POOL) {
    // fused 2x2/s2 max-pool + first-max (row-major) switch code: the lane holds both window rows
    // (i = 0, 1) of its column; the odd column comes from lane ^ 1 (DPP quad_perm [1,0,3,2]).
    // Values are compared at storage precision (like the CPU reference and the DMA kernel's epilogue).
    const int PH = H >> 1, PW = W >> 1;
    const long long prow = ((long long)n * PH + (ty0 >> 1) + wave) * PW + (ox >> 1);
    const bool st = (px & 1) == 0 && ty0 + 2 * wave < H;
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int oc = 32 * j + 8 * g + 4 * h;
        const float b4[4] = {bv[j][g].x, bv[j][g].y, bv[j][g].z, bv[j][g].w};
        float best[4];
        uint32_t codes = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float w4[4];  // window order (dy, dx) = (0,0), (0,1), (1,0), (1,1)
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const float v = to_f<DT>(from_f<DT>(fmaxf(acc[i][j][4 * g + r] + b4[r], lo)));
            const float pv = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
            w4[2 * i] = v;
            w4[2 * i + 1] = pv;
          }
          float m = w4[0];
          uint32_t c = 0;
#pragma unroll
          for (int q = 1; q < 4; ++q)
            if (w4[q] > m) {
              m = w4[q];
              c = q;
            }
          best[r] = m;
          codes |= c << (8 * r);
        }
        if (st && oc + 4 <= a.OC && DV_BOUNDS(prow * a.out_ld + oc, 4, a.out_elems, "halo-stream pool out")) {
          *reinterpret_cast<uint2*>(out + prow * a.out_ld + oc) =
              make_uint2(pack2<DT>(best[0], best[1]), pack2<DT>(best[2], best[3]));
          *reinterpret_cast<uint32_t*>(a.out_code + prow * a.OC + oc) = codes;
        } else if (st && oc < a.OC) {
          for (int r = 0; r < a.OC - oc; ++r) {
            if (DV_BOUNDS(prow * a.out_ld + oc + r, 1, a.out_elems, "halo-stream pool out"))
              out[prow * a.out_ld + oc + r] = from_f<DT>(best[r]);
            a.out_code[prow * a.OC + oc + r] = (uint8_t)(codes >> (8 * r));
          }
        }
      }
    return;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int oy = ty0 + 2 * wave + i;
    if (oy >= a.OH) continue;
    const long long pix = ((long long)n * a.OH + oy) * a.OW + ox;
    uint16_t* orow = out + pix * a.out_ld;
    // output mask of this pixel row: every 8-B quad loaded before the row's first store
    uint2 em[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int oc = 32 * j + 8 * g + 4 * h;
        em[j][g] = make_uint2(0x3C003C00u, 0x3C003C00u);  // any > 0
        if (a.emask && oc + 4 <= a.OC &&
            DV_BOUNDS(pix * a.emask_ld + oc, 4, a.emask_elems, "halo-stream emask"))
          em[j][g] = *reinterpret_cast<const uint2*>(a.emask + pix * a.emask_ld + oc);
      }
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int oc = 32 * j + 8 * g + 4 * h;
        const float v0 = fmaxf(acc[i][j][4 * g + 0] + bv[j][g].x, lo);
        const float v1 = fmaxf(acc[i][j][4 * g + 1] + bv[j][g].y, lo);
        const float v2 = fmaxf(acc[i][j][4 * g + 2] + bv[j][g].z, lo);
        const float v3 = fmaxf(acc[i][j][4 * g + 3] + bv[j][g].w, lo);
        if (oc + 4 <= a.OC) {
          if (DV_BOUNDS(pix * a.out_ld + oc, 4, a.out_elems, "halo-stream out"))
            *reinterpret_cast<uint2*>(orow + oc) = make_uint2(mask_pos_pk(pack2<DT>(v0, v1), em[j][g].x),
                                                              mask_pos_pk(pack2<DT>(v2, v3), em[j][g].y));
        } else if (oc < a.OC) {  // OC % 4 tail (never for VGG16)
          const float v[4] = {v0, v1, v2, v3};
          for (int r = 0; r < a.OC - oc; ++r) {
            float f = v[r];
            if (a.emask) {
              const uint32_t m = a.emask[pix * a.emask_ld + oc + r];
              if (m == 0u || (m & 0x8000u)) f = 0.f;
            }
            orow[oc + r] = from_f<DT>(f);
          }
        }
      }
  }
}

// ---------------------------------------------------------------------------------------------
// hs16: the same halo-stream scheme on 16 x 16 output tiles for maps whose sides are multiples of 16
// (VGG16 112x112: the 16 x 32 tiles above waste 12.5 % there), with `v_mfma_f32_16x16x32_*`:
// A = weights (16 output channels x 32 K = one whole (chunk, tap) step), B = pixels (32 K x 16 pixels
// of one tile row); C: lane = pixel, its 4 registers = 4 consecutive output channels (8-B store).
// 4 waves (256 threads), wave w owns tile rows 4w..4w+3; 72 KiB of LDS -> 2 workgroups per CU, so
// one workgroup's barrier stalls hide behind the other's MFMAs.
// LDS: halo pixels and weight rows are 64 B (4 chunks) with the chunk XOR-swizzled by bit 2 of the
// row/pixel index (q ^ 2*((p >> 2) & 1)): for every ds_read_b128 lane group the 16 (pixel, chunk)
// pairs of a 16-row fragment hit 16 distinct bank slots for ANY base pixel (brute-force checked over
// strides 4..13 and swizzles on p mod 2..16: the smallest conflict-free layout), i.e. every tap shift.
// Exact DMA counts: halo 18 x 18 x 64 B = 20.25 KiB -> 6 x 1 KiB per wave (overrun into the buffer's
// tail), weights OC x 64 B = 8 / 4 KiB -> 2 / 1 per wave.
namespace {
constexpr int H16_T = 16, H16_HW = 18;
constexpr int H16_HI = 6;                     // halo DMA instructions per wave (24 x 64 slots >= 18*18*4)
constexpr int H16_HBUF = H16_HI * 4 * 1024;   // 24 KiB per halo buffer
__device__ __forceinline__ int h16_swz(int p) { return ((p >> 2) & 1) << 1; }
}  // namespace

// UNPOOL: the input is a max-pooled map (H/2 x W/2, a.x) + switch codes (a.code, per image n/code_div)
// and the conv reads its max-unpooled, ReLU'd version (the deconvnet's unpool -> conv-down). Per chunk
// the 10 x 10 pooled pixels and their codes under the tile are LDS-DMA'd into a staging buffer
// (3 instructions per wave) and expanded by all threads into the 18 x 18 full-resolution halo layout
// at the end of the previous chunk's last step: a quarter of the input bytes of a materialized unpool.
constexpr int HU_PI = 2, HU_CI = 1;           // pooled-value / code DMA instructions per wave and chunk
constexpr int HU_PBUF = HU_PI * 4 * 1024, HU_CBUF = HU_CI * 4 * 1024;

// TPS (taps per K step): 1, or 3 for 64-channel outputs (!UNPOOL): a step is one kernel row (three
// taps, 48 MFMAs per wave between barriers instead of 16), the weight slot holds the row's three
// taps, and a 2-slot ring with the next step's weights issued right after the barrier (prefetch
// distance one 48-MFMA step) keeps 72 KiB of LDS -> 2 workgroups per CU.
// LEPI (plain / emask epilogue, host: OC, out_ld, emask_ld % 8 == 0, 16-B aligned rows): the C tile goes
// through LDS (the operand buffers, free after the K loop: 16 or 8 KiB per wave) and every lane stores
// whole 16-B chunks, OCT / 8 lanes per pixel row: each store instruction writes 4 (OCT 128) or 8 pixels'
// complete 256 / 128-B rows instead of 16 pixels x 32 B (the register layout's 8-B stores). The same
// change on the persistent KW3P kernel took 9-13 % off its launches (profiles/kw3_epi_ab_r5.txt).
// STEM (VGG16 block1_conv1 -> block1_conv2 -> pool, conv3x3_stem_pool_launch): a.x is the 8-channel RGB
// image; both 32-channel halo buffers are COMPUTED in the prologue as the first conv (a.w2 / a.bias2) of
// the tile's 18 x 18 halo from a 20 x 20 RGB window, instead of DMA'd from its 64-channel output map. The
// first conv runs exactly as conv3x3_c8_stream_kernel does it (same MFMA operands and K order, bias,
// ReLU, bf16 rounding), so the result is bit-identical to the two-launch path while the 2 x 128 B/px of
// that map's HBM write + read disappear.
template <int DT, int OCT, bool POOL, bool UNPOOL, int TPS = 1, bool LEPI = false, bool STEM = false>
__global__ void __launch_bounds__(256, 2) conv3x3_hs16_kernel(const ConvArgs a, int tiles_x, int tiles_y) {
  static_assert(!LEPI || !POOL, "LDS epilogue: plain / emask outputs");
  static_assert(!STEM || (TPS == 3 && POOL && !UNPOOL && DT == DT_BF16), "fused stem: 64 -> 64 + pool, bf16");
  static_assert(TPS == 1 || (TPS == 3 && OCT == 64 && !UNPOOL), "3-tap steps: 64 output channels, no unpool");
  constexpr int FN = OCT / 16;                // output-channel blocks
  constexpr int BI = OCT / 64 * TPS;          // weight DMA instructions per wave and step (TPS*OCT*64 B / 4 KiB)
  constexpr int BSLOT = OCT * 64 * TPS;
  constexpr int RING = TPS == 1 ? 3 : 2;
  constexpr int STEPS_PER_CHUNK = 9 / TPS;
  constexpr int HI = UNPOOL ? HU_PI + HU_CI : H16_HI;  // input DMA instructions per wave and chunk
  typedef typename Vec8<DT>::type v8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * H16_HBUF + RING * BSLOT + (UNPOOL ? HU_PBUF + HU_CBUF : 0)];
  uint8_t* halo = smem;
  uint8_t* ring = smem + 2 * H16_HBUF;
  uint8_t* pstage = ring + RING * BSLOT;      // UNPOOL: pooled values [100 px][64 B], codes [100 px][32 B]
  uint8_t* cstage = pstage + HU_PBUF;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, px = lane & 15;
  const int H = a.H, W = a.W, C = a.C;
  const int per_img = tiles_x * tiles_y;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / per_img;
  const int tr = bid - n * per_img;
  const int ty0 = (tr / tiles_x) * H16_T, tx0 = (tr % tiles_x) * H16_T;

  const int PH = H >> 1, PW = W >> 1;
  const long long img = UNPOOL ? (long long)PH * PW * a.x_ld : (long long)H * W * a.x_ld;
  const hs_i32x4 xr = hs_rsrc(a.x + (long long)n * img, img * 2);
  const hs_i32x4 wr = hs_rsrc(a.w, (long long)a.OCpad * a.Kpad * 2);
  const long long cimg = (long long)PH * PW * C;  // UNPOOL: code bytes per image
  const hs_i32x4 cr = hs_rsrc(UNPOOL ? a.code + (long long)(n / a.code_div) * cimg : a.code, cimg);

  uint32_t hoff[HI];
  if constexpr (UNPOOL) {
    // pooled staging: slot s -> pooled pixel sp = s / 4 of the 10 x 10 block (rows ty0/2 - 1 ..), chunk s % 4;
    // codes: slot s -> pooled pixel s / 2, 16-B half s % 2 (32 channel codes = 32 B per pixel)
    const int py0 = (ty0 >> 1) - 1, px0 = (tx0 >> 1) - 1;
#pragma unroll
    for (int u = 0; u < HU_PI; ++u) {
      const int s = (u * 4 + wave) * 64 + lane;
      const int sp = s >> 2, ch = s & 3;
      const int y = py0 + sp / 10, x = px0 + sp % 10;
      const bool ok = sp < 100 && (unsigned)y < (unsigned)PH && (unsigned)x < (unsigned)PW;
      hoff[u] = ok ? (uint32_t)((((long long)y * PW + x) * a.x_ld + ch * 8) * 2) : HS_OOB;
    }
    {
      const int s = wave * 64 + lane;
      const int sp = s >> 1, hf = s & 1;
      const int y = py0 + sp / 10, x = px0 + sp % 10;
      const bool ok = sp < 100 && (unsigned)y < (unsigned)PH && (unsigned)x < (unsigned)PW;
      hoff[HU_PI] = ok ? (uint32_t)(((long long)y * PW + x) * C + hf * 16) : HS_OOB;
    }
  } else {
#pragma unroll
    for (int u = 0; u < H16_HI; ++u) {
      const int s = (u * 4 + wave) * 64 + lane;
      const int p = s >> 2, ch = (s & 3) ^ h16_swz(s >> 2);
      const int hy = p / H16_HW, hx = p - H16_HW * (p / H16_HW);
      const int y = ty0 - a.pad_h + hy, x = tx0 - a.pad_w + hx;
      const bool ok = p < H16_HW * H16_HW && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
      hoff[u] = ok ? (uint32_t)((((long long)y * W + x) * a.x_ld + ch * 8) * 2) : HS_OOB;
    }
  }
  // weight DMA u of a step: tap (kw) u / (OCT / 64) of the step's row, rows ((u % (OCT/64)) * 4 + wave) * 16 ..
  uint32_t woff[BI];
#pragma unroll
  for (int u = 0; u < BI; ++u) {
    const int s = ((u % (OCT / 64)) * 4 + wave) * 64 + lane;
    const int r = s >> 2, ch = (s & 3) ^ h16_swz(s >> 2);
    woff[u] = (uint32_t)(((long long)r * a.Kpad + (u / (OCT / 64)) * C + ch * 8) * 2);
  }
  const int nch = C / 32;
  const int nsteps = nch * STEPS_PER_CHUNK;
  auto issue_halo = [&](int c, int buf) {
    const uint32_t add = c < nch ? (uint32_t)(c * 64) : HS_OOB;
    if constexpr (UNPOOL) {
#pragma unroll
      for (int u = 0; u < HU_PI; ++u)
        hs_dma16(xr, pstage + (u * 4 + wave) * 1024, hoff[u] == HS_OOB || add == HS_OOB ? HS_OOB : hoff[u] + add);
      const uint32_t cadd = c < nch ? (uint32_t)(c * 32) : HS_OOB;
      hs_dma16(cr, cstage + wave * 1024, hoff[HU_PI] == HS_OOB || cadd == HS_OOB ? HS_OOB : hoff[HU_PI] + cadd);
    } else {
#pragma unroll
      for (int u = 0; u < H16_HI; ++u)
        hs_dma16(xr, halo + buf * H16_HBUF + (u * 4 + wave) * 1024,
                 hoff[u] == HS_OOB || add == HS_OOB ? HS_OOB : hoff[u] + add);
    }
  };
  // UNPOOL: staged pooled chunk -> full-resolution halo buffer `buf` (ReLU, switch select, zero
  // outside the image); 18 x 18 pixels x 4 chunks of 16 B over 256 threads
  auto expand = [&](int buf) {
    uint8_t* hd = halo + buf * H16_HBUF;
    for (int it = tid; it < H16_HW * H16_HW * 4; it += 256) {
      const int p = it >> 2, ch = it & 3;
      const int hy = p / H16_HW, hx = p - H16_HW * (p / H16_HW);
      const int y = ty0 - 1 + hy, x = tx0 - 1 + hx;
      uint4 v = make_uint4(0u, 0u, 0u, 0u);
      if ((unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W) {
        const int sp = ((y >> 1) - ((ty0 >> 1) - 1)) * 10 + ((x >> 1) - ((tx0 >> 1) - 1));
        const uint4 pv = *reinterpret_cast<const uint4*>(pstage + sp * 64 + ch * 16);
        const uint2 cd = *reinterpret_cast<const uint2*>(cstage + sp * 32 + ch * 8);
        const uint32_t pos = (uint32_t)(((y & 1) << 1) | (x & 1));
        // ReLU (sign-bit test: valid for fp16 bit patterns too), then the switch select
        v = unpool_pick(make_uint4(relu_bf2(pv.x), relu_bf2(pv.y), relu_bf2(pv.z), relu_bf2(pv.w)), cd, pos);
      }
      *reinterpret_cast<uint4*>(hd + p * 64 + ((ch ^ h16_swz(p)) << 4)) = v;
    }
  };
  auto issue_w = [&](int k) {  // step k = (chunk c, tap t) or, TPS = 3, (chunk c, kernel row t)
    const int c = k / STEPS_PER_CHUNK, t = k - STEPS_PER_CHUNK * (k / STEPS_PER_CHUNK);
    const uint32_t add = k < nsteps ? (uint32_t)((t * TPS * C + c * 32) * 2) : HS_OOB;
    uint8_t* dst = ring + (k % RING) * BSLOT;
#pragma unroll
    for (int u = 0; u < BI; ++u)
      hs_dma16(wr, dst + (u * 4 + wave) * 1024, add == HS_OOB ? HS_OOB : woff[u] + add);
  };

  f32x4 acc[4][FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // weight row 16j + px: the swizzle term depends on bit 2 of the row, the same for every j
  const int wrd = px * 64 + ((q ^ h16_swz(px)) << 4);
  // pixel reads: halo pixel (4 wave + i + kh) * 18 + px + kw; its swizzle term varies with kw only
  // through (px + kw) (the row term 18 * r shifts bit 2 too, so it is folded per (i + kh) at compile
  // time via the row's base pixel index)
  if constexpr (!STEM) issue_halo(0, 0);
  if constexpr (STEM) {
    // step 0's weights (slot 0) go out first: their DMA latency overlaps the prologue instead of following it
    issue_w(0);
    // RGB window rows ty0 - 2 .., cols tx0 - 2 ..
    uint8_t* rgb = ring + BSLOT;
    const uint16_t* xs = a.x + (long long)n * H * W * 8;
    // every global read of the prologue is issued before the first use (one memory round trip, not
    // one per dependent load): the RGB window, then the first conv's weights (A = weights, K-step s =
    // taps 4s .. 4s+3 x 8 channels; taps >= 9 are zero columns) and bias (lane (q, px) -> output
    // channel 16 j + px / 16 j + 4 q + r)
    uint4 rv[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int e = tid + 256 * u;
      const int ry = e / 20, rx = e - 20 * (e / 20);
      const int y = ty0 - 2 + ry, x = tx0 - 2 + rx;
      rv[u] = make_uint4(0u, 0u, 0u, 0u);
      if (e < 400 && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W &&
          DV_BOUNDS(((long long)n * H * W + (long long)y * W + x) * 8, 8, a.x_elems, "stem rgb"))
        rv[u] = *reinterpret_cast<const uint4*>(xs + ((long long)y * W + x) * 8);
    }
    v8 wa[3][4];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        wa[s][j] = *reinterpret_cast<const v8*>(a.w2 + (long long)(j * 16 + px) * a.kpad2 + s * 32 + q * 8);
    float b1[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) b1[j][r] = a.bias2 ? a.bias2[j * 16 + q * 4 + r] : 0.f;
    // -> weight ring slot 1 (20 x 20 px x 16 B, zero outside the image), which the first weight DMA into it
    // (issue_w(1), after step 0's barrier) overwrites
#pragma unroll
    for (int u = 0; u < 2; ++u)
      if (tid + 256 * u < 400) *reinterpret_cast<uint4*>(rgb + (tid + 256 * u) * 16) = rv[u];
    __syncthreads();
    // halo pixel p = 16 f + px (18 x 18, row-major): 21 fragments round-robin over the 4 waves
    for (int f = wave; f < 21; f += 4) {
      const int p = f * 16 + px;
      const int hy = p / H16_HW, hx = p - H16_HW * (p / H16_HW);
      f32x4 c1[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) c1[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int t = 4 * s + q;
        const int kh = t / 3, kw = t - 3 * (t / 3);
        uint4 bv = make_uint4(0u, 0u, 0u, 0u);
        if (t < 9 && p < H16_HW * H16_HW) bv = *reinterpret_cast<const uint4*>(rgb + ((hy + kh) * 20 + hx + kw) * 16);
#pragma unroll
        for (int j = 0; j < 4; ++j) c1[j] = mfma16x16x32<DT>(wa[s][j], __builtin_bit_cast(v8, bv), c1[j]);
      }
      if (p < H16_HW * H16_HW) {
        const int y = ty0 - 1 + hy, x = tx0 - 1 + hx;  // the second conv's zero padding outside the image
        const bool in = (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = in ? fmaxf(c1[j][r] + b1[j][r], 0.f) : 0.f;
          // channel 16 j + 4 q + r: halo buffer j / 2, 16-B chunk (j & 1) * 2 + q / 2, byte 8 (q & 1)
          const int ch = (j & 1) * 2 + (q >> 1);
          *reinterpret_cast<uint2*>(halo + (j >> 1) * H16_HBUF + p * 64 + ((ch ^ h16_swz(p)) << 4) + (q & 1) * 8) =
              make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ordered before every reader by step 0's barrier
  }
  if constexpr (UNPOOL) {
    hs_wait<0>();
    __builtin_amdgcn_s_barrier();  // every wave's share of the staging DMA has landed
    expand(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ordered before readers by step 0's barrier
  }
  if constexpr (TPS == 3) {
    // step k = (chunk c, kernel row kh): weights W(k) -> slot k % 2, issued at step k - 1 right after
    // its barrier, BEFORE that step's halo(c + 1) DMAs (kh == 0), so the wait for W(k) leaves the
    // younger halo in flight at kh == 1 and drains it at kh == 2 (two steps to land)
    if constexpr (!STEM) issue_w(0);
    for (int c = 0; c < nch; ++c) {
      const uint8_t* hb = halo + (c & 1) * H16_HBUF;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const int k = c * 3 + kh;
        if (kh == 1 && !STEM) hs_wait<HI>();
        else hs_wait<0>();
        __builtin_amdgcn_s_barrier();
        issue_w(k + 1);
        if (kh == 0 && !STEM) issue_halo(c + 1, (c + 1) & 1);
        const uint8_t* wb = ring + (k % RING) * BSLOT + wrd;
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          v8 wf[FN], pf[4];
#pragma unroll
          for (int j = 0; j < FN; ++j) wf[j] = *reinterpret_cast<const v8*>(wb + kw * OCT * 64 + j * 16 * 64);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int p = (4 * wave + i + kh) * H16_HW + px + kw;
            pf[i] = *reinterpret_cast<const v8*>(hb + p * 64 + ((q ^ h16_swz(p)) << 4));
          }
          __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(wf[j], pf[i], acc[i][j]);
          __builtin_amdgcn_s_setprio(0);
        }
      }
    }
  } else {
  issue_w(0);
  issue_w(1);
  for (int c = 0; c < nch; ++c) {
    const uint8_t* hb = halo + (c & 1) * H16_HBUF;
#pragma unroll
    for (int t = 0; t < STEPS_PER_CHUNK; ++t) {
      const int k = c * STEPS_PER_CHUNK + t;
      if (t == 1) hs_wait<BI + HI>();
      else hs_wait<BI>();
      __builtin_amdgcn_s_barrier();
      if (t == 0) issue_halo(c + 1, (c + 1) & 1);
      issue_w(k + 2);
      const uint8_t* wb = ring + (k % RING) * BSLOT + wrd;
      const int kh = t / 3, kw = t % 3;
      v8 wf[FN], pf[4];
#pragma unroll
      for (int j = 0; j < FN; ++j) wf[j] = *reinterpret_cast<const v8*>(wb + j * 16 * 64);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int p = (4 * wave + i + kh) * H16_HW + px + kw;
        pf[i] = *reinterpret_cast<const v8*>(hb + p * 64 + ((q ^ h16_swz(p)) << 4));
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(wf[j], pf[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      if constexpr (UNPOOL) {
        // last step of chunk c: expand chunk c+1 (staged at step 9c; younger than it: the 9 weight
        // DMAs of steps 9c..9c+8) into the other halo buffer, last read during chunk c-1
        if (t == STEPS_PER_CHUNK - 1 && c + 1 < nch) {
          hs_wait<STEPS_PER_CHUNK * BI>();
          __builtin_amdgcn_s_barrier();  // every wave's share of the staging DMA has landed
          expand((c + 1) & 1);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
      }
    }
  }
  }  // TPS == 1
  hs_wait<0>();

  // epilogue: lane = pixel (tile row 4 wave + i, column px); register r of block j = channel 16j + 4q + r
  const int ox = tx0 + px;
  float4 bv[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j)
    bv[j] = a.bias ? *reinterpret_cast<const float4*>(a.bias + 16 * j + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float lo = a.relu ? 0.f : -INFINITY;
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
  if constexpr (POOL) {  // windows (rows 4w+i, 4w+i+1) x (px, px^1): i = 0, 2; the odd column via DPP
    const int PH = H >> 1, PW = W >> 1;
#pragma unroll
    for (int i = 0; i < 4; i += 2) {
      const long long prow = ((long long)n * PH + ((ty0 >> 1) + 2 * wave + (i >> 1))) * PW + (ox >> 1);
      const bool st = (px & 1) == 0;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int oc = 16 * j + 4 * q;
        const float b4[4] = {bv[j].x, bv[j].y, bv[j].z, bv[j].w};
        float best[4];
        uint32_t codes = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float w4[4];
#pragma unroll
          for (int d = 0; d < 2; ++d) {
            const float v = to_f<DT>(from_f<DT>(fmaxf(acc[i + d][j][r] + b4[r], lo)));
            w4[2 * d] = v;
            w4[2 * d + 1] = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
          }
          float m = w4[0];
          uint32_t cc = 0;
#pragma unroll
          for (int e = 1; e < 4; ++e)
            if (w4[e] > m) {
              m = w4[e];
              cc = e;
            }
          best[r] = m;
          codes |= cc << (8 * r);
        }
        if (st && oc < a.OC && DV_BOUNDS(prow * a.out_ld + oc, 4, a.out_elems, "hs16 pool out")) {
          *reinterpret_cast<uint2*>(out + prow * a.out_ld + oc) =
              make_uint2(pack2<DT>(best[0], best[1]), pack2<DT>(best[2], best[3]));
          *reinterpret_cast<uint32_t*>(a.out_code + prow * a.OC + oc) = codes;
        }
      }
    }
    return;
  }
  if constexpr (LEPI) {
    // every wave's last fragment reads of the operand buffers are done before any wave overwrites them
    __syncthreads();
    constexpr int ROWB = OCT * 2, CPR = OCT / 8;  // bytes / 16-B chunks per pixel row
    uint8_t* wreg = smem + wave * 64 * ROWB;      // this wave's 4 x 16 pixels
    static_assert(4 * 64 * ROWB <= (int)sizeof(smem), "LDS epilogue slices");
    // C -> LDS: lane (px, q) writes channels 16 j + 4 q .. + 3 of pixel (i, px) as one 8-B write; the 16-B
    // chunk index is XOR-swizzled by the pixel (chunk ^ (px mod CPR)) so the 16 lanes of a ds_write_b64
    // group (16 pixels, one chunk) hit distinct bank slots
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const float v0 = fmaxf(acc[i][j][0] + bv[j].x, lo), v1 = fmaxf(acc[i][j][1] + bv[j].y, lo);
        const float v2 = fmaxf(acc[i][j][2] + bv[j].z, lo), v3 = fmaxf(acc[i][j][3] + bv[j].w, lo);
        const int ch = 2 * j + (q >> 1);
        *reinterpret_cast<uint2*>(wreg + (i * 16 + px) * ROWB + ((ch ^ (px & (CPR - 1))) << 4) + (q & 1) * 8) =
            make_uint2(pack2<DT>(v0, v1), pack2<DT>(v2, v3));
      }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: this wave's writes before its reads
    // LDS -> global: lane reads the chunk physically at (lane mod CPR) of local pixel lp (logical chunk
    // = that ^ the pixel's swizzle), so the 16 lanes of every ds_read_b128 group read 16 distinct slots
    constexpr int PPI = 64 / CPR, NT = 64 / PPI;  // pixels per instruction, instructions per lane
    const int pc = lane % CPR;
    uint4 em[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {  // every output-mask load before the first store
      const int lp = t * PPI + lane / CPR;
      const int lc = pc ^ (lp & (CPR - 1));
      const long long pix = ((long long)n * a.OH + ty0 + 4 * wave + (lp >> 4)) * a.OW + tx0 + (lp & 15);
      em[t] = make_uint4(0x3C003C00u, 0x3C003C00u, 0x3C003C00u, 0x3C003C00u);  // any > 0
      if (a.ebits && lc * 8 < a.OC)  // 1-bit mask: one byte per chunk
        em[t].x = a.ebits[pix * a.ebits_ld + lc];
      else if (a.emask && lc * 8 < a.OC && DV_BOUNDS(pix * a.emask_ld + lc * 8, 8, a.emask_elems, "hs16 emask"))
        em[t] = *reinterpret_cast<const uint4*>(a.emask + pix * a.emask_ld + lc * 8);
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int lp = t * PPI + lane / CPR;
      const int lc = pc ^ (lp & (CPR - 1));
      const long long pix = ((long long)n * a.OH + ty0 + 4 * wave + (lp >> 4)) * a.OW + tx0 + (lp & 15);
      uint4 v = *reinterpret_cast<const uint4*>(wreg + lp * ROWB + pc * 16);
      if (a.ebits) {
        v = mask_bits8(v, em[t].x);
      } else if (a.emask) {
        v.x = mask_pos_pk(v.x, em[t].x);
        v.y = mask_pos_pk(v.y, em[t].y);
        v.z = mask_pos_pk(v.z, em[t].z);
        v.w = mask_pos_pk(v.w, em[t].w);
      }
      if (lc * 8 < a.OC && DV_BOUNDS(pix * a.out_ld + lc * 8, 8, a.out_elems, "hs16 out")) {
        *reinterpret_cast<uint4*>(out + pix * a.out_ld + lc * 8) = v;
        if (a.obits) a.obits[pix * a.obits_ld + lc] = (uint8_t)pos_bits8(v);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oy = ty0 + 4 * wave + i;
    const long long pix = ((long long)n * a.OH + oy) * a.OW + ox;
    uint16_t* orow = out + pix * a.out_ld;
    // output mask (emask: an input gradient zeroed where its ReLU input was <= 0), row loaded up front
    uint2 em[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int oc = 16 * j + 4 * q;
      em[j] = make_uint2(0x3C003C00u, 0x3C003C00u);  // any > 0
      if (a.emask && oc < a.OC && DV_BOUNDS(pix * a.emask_ld + oc, 4, a.emask_elems, "hs16 emask"))
        em[j] = *reinterpret_cast<const uint2*>(a.emask + pix * a.emask_ld + oc);
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int oc = 16 * j + 4 * q;
      if (oc >= a.OC) continue;
      const float v0 = fmaxf(acc[i][j][0] + bv[j].x, lo), v1 = fmaxf(acc[i][j][1] + bv[j].y, lo);
      const float v2 = fmaxf(acc[i][j][2] + bv[j].z, lo), v3 = fmaxf(acc[i][j][3] + bv[j].w, lo);
      if (DV_BOUNDS(pix * a.out_ld + oc, 4, a.out_elems, "hs16 out"))
        *reinterpret_cast<uint2*>(orow + oc) =
            make_uint2(mask_pos_pk(pack2<DT>(v0, v1), em[j].x), mask_pos_pk(pack2<DT>(v2, v3), em[j].y));
    }
  }
}

// weight ring depth (slots; B(k + ring - 1) is prefetched at step k). DV_HS_RING = 3 / 4 / 5 (A/B)
static int hs_ring() {
  static int v = [] {
    const char* e = dv_ab_env("DV_HS_RING");
    const int r = e ? std::atoi(e) : 3;
    return r == 4 || r == 5 ? r : 3;
  }();
  return v;
}

#define HS_LAUNCH(DT_, OCT_, POOL_)                                                                    \
  do {                                                                                                 \
    if (ring == 5)                                                                                     \
      hipLaunchKernelGGL((conv3x3_hs_kernel<DT_, OCT_, POOL_, 5>), grid, block, 0, s, a, tx, ty);      \
    else if (ring == 4)                                                                                \
      hipLaunchKernelGGL((conv3x3_hs_kernel<DT_, OCT_, POOL_, 4>), grid, block, 0, s, a, tx, ty);      \
    else                                                                                               \
      hipLaunchKernelGGL((conv3x3_hs_kernel<DT_, OCT_, POOL_, 3>), grid, block, 0, s, a, tx, ty);      \
  } while (0)

int conv3x3_hs_launch(const ConvArgs& a, int epi, hipStream_t s, bool* lepi_used) {
  if (lepi_used) *lepi_used = false;  // set when the LDS-staged epilogue (the only one with 1-bit masks) runs
  if (dv_ab_env("DV_NO_HS") != nullptr) return -4;
  // 192 / 256 padded output channels (InceptionV3 conv2d_5: 96 -> 192): two launches over the
  // channel halves [0, 128) and [128, OCpad), each re-reading the (small) input halo
  if ((a.OCpad == 192 || a.OCpad == 256) && a.OC > 128 && epi == CONV_E_BF16 && dv_ab_env("DV_NO_HS_SPLIT") == nullptr) {
    ConvArgs a1 = a, a2 = a;
    a1.OC = 128;
    a1.OCpad = 128;
    a2.OC = a.OC - 128;
    a2.OCpad = a.OCpad - 128;
    a2.w = a.w + (long long)128 * a.Kpad;
    a2.bias = a.bias ? a.bias + 128 : nullptr;
    a2.out = reinterpret_cast<uint16_t*>(a.out) + 128;
    a2.out_elems = a.out_elems - 128;
    if (a.emask) {
      a2.emask = a.emask + 128;
      a2.emask_elems = a.emask_elems - 128;
    }
    a1.obits = a2.obits = nullptr;  // no 1-bit masks on the channel-split form
    a1.ebits = a2.ebits = nullptr;
    if (a2.OC % 4 != 0) return -4;
    // both halves must be supported before either launches
    const int r1 = conv3x3_hs_launch(a1, epi, s);
    if (r1 < 0) return r1;
    return conv3x3_hs_launch(a2, epi, s);
  }
  // 3x3 / stride 1, symmetric pad 0..2 (output = input + 2 pad - 2)
  const bool geom = a.KH == 3 && a.KW == 3 && a.stride == 1 && a.pad_h == a.pad_w && a.pad_h >= 0 && a.pad_h <= 2 &&
                    a.OH == a.H + 2 * a.pad_h - 2 && a.OW == a.W + 2 * a.pad_w - 2 && a.OH > 0 && a.OW > 0;
  if (!geom || a.C % 32 != 0 || a.x_ld % 8 != 0 || (a.OCpad != 64 && a.OCpad != 128) || a.relu_in || a.accumulate ||
      a.mask || a.code || a.res || a.ws || a.stats || a.ucode || a.relu_cols > 0 || a.out_ld % 4 != 0 ||
      (reinterpret_cast<uintptr_t>(a.out) & 7) || (reinterpret_cast<uintptr_t>(a.x) & 15) ||
      (reinterpret_cast<uintptr_t>(a.bias) & 15) ||
      (a.emask && (a.emask_ld % 4 != 0 || (reinterpret_cast<uintptr_t>(a.emask) & 7))) ||
      (long long)a.Kpad < 9LL * a.C || (long long)a.H * a.W * a.x_ld * 2 > 0x7FFFFFF0LL)
    return -4;
  const bool pool = epi == CONV_E_POOL;
  if (!pool && epi != CONV_E_BF16) return -4;
  if (pool && (a.pad_h != 1 || a.emask || a.H % 2 || a.W % 2 || a.out_code == nullptr || a.OC % 4 ||
               a.dtype != DT_BF16 || (reinterpret_cast<uintptr_t>(a.out_code) & 3)))
    return -4;
  // exact 16 x 16 tiling of the output (OC % 4 == 0: whole 8-B channel quads) -> hs16
  if (a.OH % 16 == 0 && a.OW % 16 == 0 && a.OC % 4 == 0 && dv_ab_env("DV_NO_HS16") == nullptr) {
    const int t16x = a.OW / 16, t16y = a.OH / 16;
    const long long n16 = (long long)a.N * t16x * t16y;
    if (n16 <= 0 || n16 > 0x7fffffffLL) return -2;
    const dim3 g16((unsigned)n16), b16(256);
#define HS16(DT_, OCT_, POOL_, LEPI_)                                                                            \
  hipLaunchKernelGGL((conv3x3_hs16_kernel<DT_, OCT_, POOL_, false, OCT_ == 64 ? 3 : 1, LEPI_>), g16, b16, 0, s, a, t16x, \
                     t16y)
    // the LDS-staged 16-B store epilogue (DV_HS16_EPI=reg: the register layout's 8-B stores, A/B; read per launch)
    const char* he = dv_ab_env("DV_HS16_EPI");
    const bool lepi = !pool && !(he && std::strcmp(he, "reg") == 0) && a.OC % 8 == 0 && a.out_ld % 8 == 0 &&
                      !(reinterpret_cast<uintptr_t>(a.out) & 15) &&
                      (!a.emask || (a.emask_ld % 8 == 0 && !(reinterpret_cast<uintptr_t>(a.emask) & 15)));
    if (lepi_used) *lepi_used = lepi;
    if (pool) {
      if (a.OCpad == 128) HS16(DT_BF16, 128, true, false);
      else HS16(DT_BF16, 64, true, false);
    } else if (a.dtype == DT_F16) {
      if (a.OCpad == 128) {
        if (lepi) HS16(DT_F16, 128, false, true);
        else HS16(DT_F16, 128, false, false);
      } else {
        if (lepi) HS16(DT_F16, 64, false, true);
        else HS16(DT_F16, 64, false, false);
      }
    } else {
      if (a.OCpad == 128) {
        if (lepi) HS16(DT_BF16, 128, false, true);
        else HS16(DT_BF16, 128, false, false);
      } else {
        if (lepi) HS16(DT_BF16, 64, false, true);
        else HS16(DT_BF16, 64, false, false);
      }
    }
#undef HS16
    return (int)hipGetLastError();
  }
  const int tx = (a.OW + HS_TW - 1) / HS_TW, ty = (a.OH + HS_TH - 1) / HS_TH;
  const long long nwg = (long long)a.N * tx * ty;
  if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
  const dim3 grid((unsigned)nwg), block(512);
  const int ring = hs_ring();
  // the LDS-staged 16-B store epilogue (DV_HS16_EPI=reg: the register layout's 8-B stores, A/B; per launch)
  const char* he = dv_ab_env("DV_HS16_EPI");
  const bool lepi = !pool && ring == 3 && !(he && std::strcmp(he, "reg") == 0) && a.OC % 8 == 0 && a.out_ld % 8 == 0 &&
                    !(reinterpret_cast<uintptr_t>(a.out) & 15) &&
                    (!a.emask || (a.emask_ld % 8 == 0 && !(reinterpret_cast<uintptr_t>(a.emask) & 15)));
  if (lepi_used) *lepi_used = lepi;
#define HS_LEPI(DT_, OCT_, NB1_) \
  hipLaunchKernelGGL((conv3x3_hs_kernel<DT_, OCT_, false, 3, NB1_, true>), grid, block, 0, s, a, tx, ty)
  if (pool) {
    if (a.OCpad == 128) HS_LAUNCH(DT_BF16, 128, true);
    else HS_LAUNCH(DT_BF16, 64, true);
  } else if (a.C == 32 && a.OCpad == 64) {  // one channel chunk: single halo buffer, 2 workgroups per CU
    if (a.dtype == DT_F16) {
      if (lepi) HS_LEPI(DT_F16, 64, true);
      else hipLaunchKernelGGL((conv3x3_hs_kernel<DT_F16, 64, false, 3, true>), grid, block, 0, s, a, tx, ty);
    } else {
      if (lepi) HS_LEPI(DT_BF16, 64, true);
      else hipLaunchKernelGGL((conv3x3_hs_kernel<DT_BF16, 64, false, 3, true>), grid, block, 0, s, a, tx, ty);
    }
  } else if (lepi) {
    if (a.dtype == DT_F16) {
      if (a.OCpad == 128) HS_LEPI(DT_F16, 128, false);
      else HS_LEPI(DT_F16, 64, false);
    } else {
      if (a.OCpad == 128) HS_LEPI(DT_BF16, 128, false);
      else HS_LEPI(DT_BF16, 64, false);
    }
  } else if (a.dtype == DT_F16) {
    if (a.OCpad == 128) HS_LAUNCH(DT_F16, 128, false);
    else HS_LAUNCH(DT_F16, 64, false);
  } else {
    if (a.OCpad == 128) HS_LAUNCH(DT_BF16, 128, false);
    else HS_LAUNCH(DT_BF16, 64, false);
  }
#undef HS_LEPI
  return (int)hipGetLastError();
}

// fused VGG16 stem (block1_conv1 -> block1_conv2 -> 2x2 max-pool + switch): the hs16 pool kernel with the
// halo computed from the RGB image (STEM above). a: the SECOND conv's geometry (C = OC = 64, pad 1)
// with a.x = the 8-channel image (x_ld 8), a.w2 / a.bias2 / a.kpad2 the first conv's packed weights.
// Forward-only and bf16; DV_STEM_FUSE=0 (Python side) keeps the two-launch path.
int conv3x3_stem_pool_launch(const ConvArgs& a, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != 64 || a.OC != 64 ||
      a.OCpad != 64 || a.x_ld != 8 || a.H != a.OH || a.W != a.OW || a.H % 16 || a.W % 16 || a.H <= 0 || a.W <= 0 ||
      a.N <= 0 || a.dtype != DT_BF16 || a.w2 == nullptr || a.kpad2 < 96 || a.Kpad < 9 * 64 || a.out_code == nullptr ||
      a.out_ld != 64 || a.relu != 1 || a.relu_in || a.accumulate || a.mask || a.code || a.res || a.emask || a.ws ||
      a.ucode || (reinterpret_cast<uintptr_t>(a.x) & 15) || (reinterpret_cast<uintptr_t>(a.out) & 7) ||
      (reinterpret_cast<uintptr_t>(a.out_code) & 3) || (reinterpret_cast<uintptr_t>(a.w2) & 15) ||
      (long long)a.H * a.W * 8 * 2 > 0x7FFFFFF0LL)
    return -4;
  const int tx = a.W / 16, ty = a.H / 16;
  const long long nwg = (long long)a.N * tx * ty;
  if (nwg > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL((conv3x3_hs16_kernel<DT_BF16, 64, true, false, 3, false, true>), dim3((unsigned)nwg), dim3(256), 0,
                     s, a, tx, ty);
  return (int)hipGetLastError();
}

}  // namespace dv
