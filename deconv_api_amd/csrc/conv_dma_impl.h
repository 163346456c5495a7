// LDS-DMA implicit-GEMM convolution for gfx950 (MI355X): the high-throughput path for plain
// (non-unpool) conv forward and transposed-conv dgrad.
//
// Differences from conv_igemm.hip (the register-staged kernel that also handles the
// unpool-gather and ReLU-mask prologues):
//   * operands are staged global -> LDS by `buffer_load_dwordx4 ... lds` (LDS-DMA): no VGPR
//     round trip and no ds_write issue cost. Conv zero padding, the M tail and the K tail come
//     for free from the buffer descriptor's range check (an out-of-range offset returns 0);
//   * 8 waves per workgroup, each owning a (16*FM) x (16*FN) C tile (up to 128 x 64, i.e.
//     256 x 256 per workgroup), so each ds_read_b128 fragment feeds FN (or FM) MFMAs;
//   * the LDS image is lane-linear per DMA instruction (1 KiB = 1024/(2*BK) rows); the XOR
//     swizzle is applied to the per-lane SOURCE chunk and to the fragment read address, never
//     to the DMA destination (cdna_hip_programming.md rule 21). BK=64 rows (128 B): chunk ^
//     (row & 7). BK=32 rows (64 B): chunk ^ ((4 - ((row >> 2) & 3)) & 3), which puts the 16
//     rows x 4 chunks of every ds_read_b128 lane group of a 16x16x32 fragment read on distinct
//     16-B bank slots (derivation in docs/KERNELS.md);
//   * STAGES-deep LDS ring, one barrier per K tile: the DMA for tile t+STAGES-1 is issued right
//     after the barrier of tile t and a counted `s_waitcnt vmcnt(N)` leaves the younger tiles in
//     flight across the barrier (raw s_barrier, never __syncthreads, so nothing drains them).
// LDS-DMA implicit-GEMM conv: kernel templates, tile configs and per-problem tile choice.
// Shared by the instantiation units conv_dma_<dtype>_<mode>.hip (one dma_bn<DT, AMODE, EPI>
// each, compiled in parallel) and conv_dma.hip (dispatch, split-K, masked dgrads, tuning state).
#pragma once
#include "common.h"
#include "kernels.h"

#include <cstdlib>
#include <cstring>
#include <type_traits>

namespace dv {

namespace {

constexpr uint32_t kOOB = 0x80000000u;  // any offset >= num_records reads as zero

typedef __attribute__((address_space(3))) void lds_void;

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rsrc, uint8_t* lds_dst, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void*)lds_dst, 16, voff, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint32_t nrec = bytes > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nrec, 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// vmcnt wait leaving `pend` (<= P) younger K tiles of LO (HI: this wave issues one more B row
// group) DMAs each in flight; deep rings (STAGES > 4) keep more tiles in flight for the
// latency-bound small GEMMs
template <int P, int LO, int HI>
__device__ __forceinline__ void wait_pend(int pend, bool hi) {
  if constexpr (P <= 0) {
    wait_vm<0>();
  } else {
    if (pend >= P) {
      if (hi) wait_vm<P * HI>(); else wait_vm<P * LO>();
    } else {
      wait_pend<P - 1, LO, HI>(pend, hi);
    }
  }
}

// swizzle term of LDS row `row` for a BK-wide tile
template <int BK>
__device__ __forceinline__ int row_xor(int row) {
  if constexpr (BK == 64)
    return row & 7;
  else
    return (4 - ((row >> 2) & 3)) & 3;
}

}  // namespace

template <int DT, int FM, int FN, int EPI, bool accum>
__device__ __forceinline__ void epilogue(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int mw, int nw, int lane);
template <int DT, int FM, int FN>
__device__ __forceinline__ void epilogue_res(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int mw, int nw,
                                             int lane);
template <int DT, int NT, int BM, int BN, int FM, int FN>
__device__ __forceinline__ void epilogue_lds(const ConvArgs& a, const f32x4 (&acc)[FM][FN], uint8_t* smem, int m0,
                                             int n0, int wm, int wn, int lane, int tid, bool writer = true);
template <int DT, int NT, int BM, int BN, int FM, int FN>
__device__ __forceinline__ void epilogue_pool_lds(const ConvArgs& a, const f32x4 (&acc)[FM][FN], uint8_t* smem, int m0,
                                                  int n0, int wm, int wn, int lane, int tid);

// DT: 16-bit storage/MFMA dtype of x, w and a 16-bit output (DT_BF16 / DT_F16, common.h)
// MASK: backward through a ReLU: A elements are kept only where mask (same layout and pixel
// stride as x) is > 0. The mask tile is DMA'd into LDS next to the A tile with the same offsets
// and applied to each A fragment in registers right before its MFMAs.
// The workgroup body: output tile ``wgid`` (row-major over tiles_n column tiles) of problem ``a``,
// K slice ky of nky. Shared by the one-problem kernel below and the grouped kernel
// (conv_dma_group_kernel), whose workgroups each look their problem up in a table.
template <int DT, int WM, int WN, int FM, int FN, int BK, int STAGES, int AMODE, int EPI, bool CALIGNED,
          bool MASK = false, bool FRAGPIPE = false>
__device__ __forceinline__ void conv_dma_body(const ConvArgs& a, int tiles_n, int wgid, int ky, int nky) {
  constexpr int NW = WM * WN;
  constexpr int BM = WM * FM * 16;
  constexpr int BN = WN * FN * 16;
  constexpr int ROWB = BK * 2;              // LDS bytes per row
  constexpr int CPR = BK / 8;               // 16-B chunks per row
  constexpr int RPI = 1024 / ROWB;          // rows per DMA instruction
  constexpr int A_BYTES = BM * ROWB;
  constexpr int B_BYTES = BN * ROWB;
  constexpr int M_BYTES = MASK ? A_BYTES : 0;
  constexpr int STAGE = A_BYTES + M_BYTES + B_BYTES;
  constexpr int A_I = BM / RPI / NW;        // A DMA instructions per wave per K tile
  constexpr int B_GROUPS = BN / RPI;        // RPI-row groups of the B tile
  constexpr int B_FULL = B_GROUPS / NW, B_REM = B_GROUPS % NW;
  static_assert(A_I >= 1 && BM % (RPI * NW) == 0, "BM must cover every wave");
  static_assert(STAGES >= 2 && STAGES <= 8, "stages");
  __shared__ __attribute__((aligned(16))) uint8_t smem[STAGES * STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int tile_n = wgid % tiles_n;
  const int tile_m = wgid / tiles_n;
  const int m0 = a.m_base + tile_m * BM, n0 = tile_n * BN;
  const int H = a.H, W = a.W, C = a.C;

  // ---- tile base image: every A source offset is relative to it (32-bit voffsets) ----
  int n_base;
  {
    const int g = m0 < a.M ? m0 : a.M - 1;
    int pix = g;
    if constexpr (EPI == CONV_E_POOL) pix = g >> 2;
    const int per_img = (EPI == CONV_E_POOL) ? (a.OH >> 1) * (a.OW >> 1) : a.OH * a.OW;
    n_base = pix / per_img;
  }
  const long long img_elems = (long long)H * W * a.x_ld;
  const uint16_t* xb = a.x + (long long)n_base * img_elems;
  const long long x_total = (long long)a.N * img_elems;
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(xb, (uint64_t)(x_total - (long long)n_base * img_elems) * 2);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (uint64_t)a.OCpad * a.Kpad * 2);
  __amdgpu_buffer_rsrc_t mr = xr;
  if constexpr (MASK)
    mr = make_rsrc(a.mask + (long long)n_base * img_elems, (uint64_t)(x_total - (long long)n_base * img_elems) * 2);

  // lane -> (row within its DMA row group, logical 16-B chunk at LDS position lane % CPR)
  const int lrow = lane / CPR;
  const int lchunk = (lane % CPR) ^ row_xor<BK>(lrow);  // group bases are multiples of 16 rows

  // ---- per-row A gather state (rows fixed for the whole K loop) ----
  int r_off[A_I], r_h[A_I], r_w[A_I];
#pragma unroll
  for (int j = 0; j < A_I; ++j) {
    const int row = (j * NW + wave) * RPI + lrow;
    const int gm = m0 + row;
    int n, oh, ow;
    const int g = gm < a.M ? gm : 0;
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
    if constexpr (AMODE == CONV_A_TRANSPOSE) {
      r_h[j] = oh + a.pad_h;
      r_w[j] = ow + a.pad_w;
    } else {
      r_h[j] = oh * a.stride - a.pad_h;
      r_w[j] = ow * a.stride - a.pad_w;
    }
    r_off[j] = (n - n_base) * H * W;  // pixel index of the image's first pixel, relative to base
    if (gm >= a.M) r_h[j] = -(1 << 28);  // never in bounds
  }
  // Fast path (forward convs with <= 32 taps): per row, a tap-validity bitmask and the element
  // offset of tap (0,0); per K tile the gather is then mask-test + add (the uniform tap delta).
  // measured: neutral on K>=2304 layers, and its per-row prologue costs 20-40% on K=576 layers
  // (profiles/layers_r1_fastmask.txt), so it is compiled out
  constexpr bool FAST = false;
  const bool fast = FAST && a.KH * a.KW <= 32;
  uint32_t r_mask[A_I];
  int r_base[A_I];
#pragma unroll
  for (int j = 0; j < A_I; ++j) {
    uint32_t m = 0;
    if (fast) {
      for (int kh = 0; kh < a.KH; ++kh) {
        const bool okh = (unsigned)(r_h[j] + kh) < (unsigned)H;
        for (int kw = 0; kw < a.KW; ++kw)
          if (okh && (unsigned)(r_w[j] + kw) < (unsigned)W) m |= 1u << (kh * a.KW + kw);
      }
    }
    r_mask[j] = m;
    r_base[j] = m ? (int)(((long long)r_off[j] + (long long)r_h[j] * W + r_w[j]) * a.x_ld) : 0;
  }

  // K decomposition (tap = (kh, kw), channel) of the NEXT tile to issue, advanced incrementally:
  // issue() runs for kt = k_first, k_first + 1, ... in order, so one division pair up front replaces
  // the two integer divisions per K tile (~40 scalar/vector instructions of a ~150-instruction K step
  // that bounds the latency of the small, few-workgroup GEMMs). CALIGNED: wave-uniform tile base;
  // otherwise per lane (its 8-channel chunk may sit in a later tap than the tile's first element).
  int nk_tap, nk_kh, nk_kw, nk_ch, nk_k;
  auto k_init = [&](int kt) {
    nk_k = kt * BK + (CALIGNED ? 0 : lchunk * 8);
    nk_tap = nk_k / C;
    nk_kh = nk_tap / a.KW;
    nk_kw = nk_tap - nk_kh * a.KW;
    nk_ch = nk_k - nk_tap * C;
  };
  auto issue = [&](int kt, int buf) {
    uint8_t* As = smem + buf * STAGE;
    uint8_t* Bs = As + A_BYTES + M_BYTES;
    const int tap = nk_tap, kh = nk_kh, kw = nk_kw;
    const int ch = nk_ch + (CALIGNED ? lchunk * 8 : 0);
    const bool kval = CALIGNED ? tap < a.KH * a.KW : nk_k < a.K;
    nk_k += BK;
    nk_ch += BK;
    while (nk_ch >= C) {  // CALIGNED: exactly one wrap per C / BK tiles; else <= BK / C + 1 wraps
      nk_ch -= C;
      ++nk_tap;
      if (++nk_kw == a.KW) {
        nk_kw = 0;
        ++nk_kh;
      }
    }
    if (FAST && fast) {
      const int delta = (kh * W + kw) * (int)a.x_ld + ch;
      const uint32_t tbit = kval ? (1u << tap) : 0u;
#pragma unroll
      for (int j = 0; j < A_I; ++j) {
        const uint32_t voff = (r_mask[j] & tbit) ? (uint32_t)(r_base[j] + delta) * 2u : kOOB;
        dma16(xr, As + (j * NW + wave) * 1024, voff);
      }
    } else {
#pragma unroll
    for (int j = 0; j < A_I; ++j) {
      int ih, iw;
      bool ok;
      if constexpr (AMODE == CONV_A_TRANSPOSE) {
        const int th = r_h[j] - kh, tw = r_w[j] - kw;
        const int s = a.stride;
        ih = th / s;
        iw = tw / s;
        ok = th >= 0 && tw >= 0 && ih * s == th && iw * s == tw && ih < H && iw < W;
      } else {
        ih = r_h[j] + kh;
        iw = r_w[j] + kw;
        ok = (unsigned)ih < (unsigned)H && (unsigned)iw < (unsigned)W;
      }
      ok = ok && kval;
      ok = ok && DV_BOUNDS((long long)n_base * img_elems + ((long long)(r_off[j] + ih * W + iw)) * a.x_ld + ch, 8,
                           a.x_elems, "conv_dma A gather");
      // 32-bit offset math: the DMA offset is 32-bit anyway, and the 64-bit multiply it was truncated from cost
      // ~4 more VALU per DMA in a K step that is issue-bound on the small GEMMs
      const uint32_t voff =
          ok ? ((uint32_t)(r_off[j] + ih * W + iw) * (uint32_t)a.x_ld + (uint32_t)ch) * 2u : kOOB;
      dma16(xr, As + (j * NW + wave) * 1024, voff);
      if constexpr (MASK) dma16(mr, As + A_BYTES + (j * NW + wave) * 1024, voff);
    }
    }
#pragma unroll
    for (int j = 0; j < B_FULL + (B_REM ? 1 : 0); ++j) {
      const int grp = j * NW + wave;
      if (grp < B_GROUPS) {
        const int row = grp * RPI + lrow;
        const uint32_t voff = ((uint32_t)(n0 + row) * (uint32_t)a.Kpad + (uint32_t)(kt * BK + lchunk * 8)) * 2u;
        if (DV_BOUNDS((long long)voff / 2, 8, (long long)a.OCpad * a.Kpad, "conv_dma B weights"))
          dma16(wr, Bs + grp * 1024, voff);
      }
    }
  };

  // wait until this wave's DMAs of the current tile landed, leaving `pend` younger tiles in flight
  auto wait_tiles = [&](int pend) {
    constexpr int PT_LO = A_I * (MASK ? 2 : 1) + B_FULL, PT_HI = PT_LO + 1;
    static_assert((STAGES - 2) * PT_HI <= 63, "vmcnt holds at most 63 outstanding DMAs");
    wait_pend<STAGES - 2, PT_LO, PT_HI>(pend, B_REM && wave < B_REM);
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets: row = 16-aligned base + (lane & 15)
  const int a_row0 = wm * FM * 16 + (lane & 15);
  const int b_row0 = wn * FN * 16 + (lane & 15);
  const int rx = row_xor<BK>(lane & 15);
  int sw[BK / 32];
#pragma unroll
  for (int s = 0; s < BK / 32; ++s) sw[s] = (((s * 4 + (lane >> 4)) ^ rx) << 4);

  // split-K (nky > 1): this workgroup reduces K tiles [k0, k0 + nk) into a partial sum
  const int nk_all = a.Kpad / BK;
  const int k0 = (int)(((long long)nk_all * ky) / nky);
  const int nk = (int)(((long long)nk_all * (ky + 1)) / nky) - k0;
  k_init(k0);
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nk) issue(k0 + p, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt % STAGES;
    const int pend = min(STAGES - 2, nk - 1 - kt);
    wait_tiles(pend);
    __builtin_amdgcn_s_barrier();
    if (kt + STAGES - 1 < nk) issue(k0 + kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
    const uint8_t* As = smem + cur * STAGE;
    const uint8_t* Bs = As + A_BYTES + M_BYTES;
    if constexpr (FRAGPIPE && !MASK) {
      // all fragments of a 32-K sub-step are read up front, and the next sub-step's reads are
      // issued before this sub-step's MFMAs (register double buffer), so LDS latency hides
      // behind FM*FN MFMAs instead of being exposed per A fragment
      typedef typename Vec8<DT>::type v8;
      v8 af[2][FM], bf[2][FN];
      auto ld = [&](int s, int b) {
#pragma unroll
        for (int j = 0; j < FN; ++j) bf[b][j] = *reinterpret_cast<const v8*>(Bs + (b_row0 + j * 16) * ROWB + sw[s]);
#pragma unroll
        for (int i = 0; i < FM; ++i) af[b][i] = *reinterpret_cast<const v8*>(As + (a_row0 + i * 16) * ROWB + sw[s]);
      };
      ld(0, 0);
#pragma unroll
      for (int s = 0; s < BK / 32; ++s) {
        if (s + 1 < BK / 32) ld(s + 1, (s + 1) & 1);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af[s & 1][i], bf[s & 1][j], acc[i][j]);
        __builtin_amdgcn_s_setprio(0);
      }
      continue;
    }
#pragma unroll
    for (int s = 0; s < BK / 32; ++s) {
      typedef typename Vec8<DT>::type v8;
      v8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const v8*>(Bs + (b_row0 + j * 16) * ROWB + sw[s]);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        v8 af = *reinterpret_cast<const v8*>(As + (a_row0 + i * 16) * ROWB + sw[s]);
        if constexpr (MASK) {
          uint4 av = __builtin_bit_cast(uint4, af);
          const uint4 mv = *reinterpret_cast<const uint4*>(As + A_BYTES + (a_row0 + i * 16) * ROWB + sw[s]);
          av.x = mask_pos_pk(av.x, mv.x);
          av.y = mask_pos_pk(av.y, mv.y);
          av.z = mask_pos_pk(av.z, mv.z);
          av.w = mask_pos_pk(av.w, mv.w);
          af = __builtin_bit_cast(v8, av);
        }
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af, bfr[j], acc[i][j]);
      }
    }
  }

  // ---- epilogue ----
  if (a.ws != nullptr) {  // split-K partial: raw fp32 sums to ws[split][row][OCpad]
    float* ws = a.ws + (long long)ky * a.M * a.OCpad;
    const int row_l = (lane >> 4) * 4, col_l = lane & 15;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int col = n0 + wn * FN * 16 + j * 16 + col_l;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = m0 + wm * FM * 16 + i * 16 + row_l + r;
          if (row < a.M) ws[(long long)row * a.OCpad + col] = acc[i][j][r];
        }
    }
    return;
  }
  if constexpr (EPI == CONV_E_BF16) {
    if (a.vec_epi) {
      static_assert(BM * BN * 2 <= STAGES * STAGE, "C tile must fit in the operand stages");
      __syncthreads();  // every wave is done reading the operand stages
      epilogue_lds<DT, NW * 64, BM, BN, FM, FN>(a, acc, smem, m0, n0, wm, wn, lane, tid);
      return;
    }
  }
  if constexpr (EPI == CONV_E_POOL && FM % 4 == 0 && BN % 16 == 0 && (BM / 4) * BN * 3 <= STAGES * STAGE) {
    if (a.pool_t == 2) {
      __syncthreads();  // every wave is done reading the operand stages
      epilogue_pool_lds<DT, NW * 64, BM, BN, FM, FN>(a, acc, smem, m0, n0, wm, wn, lane, tid);
      return;
    }
  }
  if constexpr (EPI == CONV_E_BF16) {
    if (a.res || a.emask) {
      epilogue_res<DT, FM, FN>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
      return;
    }
  }
  if (a.accumulate)
    epilogue<DT, FM, FN, EPI, true>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
  else
    epilogue<DT, FM, FN, EPI, false>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
}

template <int DT, int WM, int WN, int FM, int FN, int BK, int STAGES, int AMODE, int EPI, bool CALIGNED,
          bool MASK = false, bool FRAGPIPE = false>
__global__ void __launch_bounds__(WM * WN * 64) conv_dma_kernel(const ConvArgs a, int tiles_n) {
  conv_dma_body<DT, WM, WN, FM, FN, BK, STAGES, AMODE, EPI, CALIGNED, MASK, FRAGPIPE>(
      a, tiles_n, xcd_remap(blockIdx.x, gridDim.x), blockIdx.y, gridDim.y);
}

// Grouped launch: up to kGroupMax INDEPENDENT problems of one tile config in one grid (the parallel
// branch convs / dgrads of an InceptionV3 block, ops/inception.py). Workgroup b (XCD-remapped over
// the whole grid) runs tile b - start[p] of the problem p with start[p] <= b < start[p + 1]: one
// launch instead of n dependent ones, and the small problems' tiles run side by side.
template <int DT, int WM, int WN, int FM, int FN, int BK, int STAGES, int AMODE, int EPI, bool CALIGNED>
__global__ void __launch_bounds__(WM * WN * 64) conv_dma_group_kernel(const ConvGroup g) {
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  int p = 0;
#pragma unroll
  for (int i = 1; i < kGroupMax; ++i) p += (i < g.n && wgid >= g.start[i]) ? 1 : 0;
  conv_dma_body<DT, WM, WN, FM, FN, BK, STAGES, AMODE, EPI, CALIGNED>(g.p[p], g.tiles_n[p], wgid - g.start[p], 0, 1);
}

// residual epilogue (ResNet block tail): out = [ReLU](acc + bias + res), then optionally zeroed
// where emask <= 0 (backward: the input gradient of a block whose input is a ReLU output, with the
// shortcut gradient as `res`). Each column group's residual/emask values are all loaded before its
// first store, so the loads overlap each other instead of each waiting behind the previous store.
template <int DT, int FM, int FN>
__device__ __forceinline__ void epilogue_res(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int mw, int nw,
                                             int lane) {
  const int row_l = (lane >> 4) * 4;
  const int col_l = lane & 15;
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = nw + j * 16 + col_l;
    if (col >= a.OC) continue;
    const float bias = a.bias ? a.bias[col] : 0.f;
    uint16_t rv[FM][4], ev[FM][4];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = min(mw + i * 16 + row_l + r, a.M - 1);
        rv[i][r] = a.res ? a.res[(long long)row * a.res_ld + col] : (uint16_t)0u;
        ev[i][r] = a.emask ? a.emask[(long long)row * a.emask_ld + col] : (uint16_t)0x3C00u;  // any > 0
      }
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mw + i * 16 + row_l + r;
        if (row >= a.M) continue;
        float v = acc[i][j][r] + bias;
        if (relu_at(a, col) && !a.res) v = fmaxf(v, 0.f);  // same order as epilogue_lds
        v += to_f<DT>(rv[i][r]);
        if (a.accumulate) v += to_f<DT>(out[(long long)row * a.out_ld + col]);
        if (relu_at(a, col) && a.res) v = fmaxf(v, 0.f);
        const uint32_t e = ev[i][r];
        if (e == 0u || (e & 0x8000u)) v = 0.f;
        if (DV_BOUNDS((long long)row * a.out_ld + col, 1, a.out_elems, "conv_dma epilogue_res out"))
          out[(long long)row * a.out_ld + col] = from_f<DT>(v);
      }
  }
}

// Pooled-max epilogue with 8-B stores: a lane's 4 accumulators are one 2x2 window of one channel (pool-major M
// order), so the max / first-max code per (fragment, channel) comes out one value per lane; a 4 x 4 transpose
// over each lane quad (two DPP swaps, as KW3P's epilogue) then gives every lane 4 consecutive channels of one
// pooled pixel: one 8-B value store + one 4-B code store per 4 fragments instead of 4 two-byte + 4 one-byte
// stores, each with its own 64-bit address. Needs FM % 4 == 0 and 4-aligned channel counts / strides (host).
template <int DT, int FM, int FN>
__device__ __forceinline__ void epilogue_pool_t(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int mw, int nw,
                                                int lane) {
  const int q = lane >> 4, cl = lane & 15, ce = cl & 1, cu = (cl >> 1) & 1, csub = cl & ~3, tsel = ce * 2 + cu;
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col0 = nw + j * 16;
    const float bias = (a.bias && col0 + cl < a.OC) ? a.bias[col0 + cl] : 0.f;
#pragma unroll
    for (int ig = 0; ig < FM / 4; ++ig) {
      float best[4];
      uint32_t code[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = ig * 4 + t;
        float b = -INFINITY;
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          v = to_f<DT>(from_f<DT>(v));
          if (v > b) {
            b = v;
            c = (uint32_t)r;
          }
        }
        best[t] = b;
        code[t] = c;
      }
      // rows = the 4 fragments, columns = channels: lane (quad position tsel) ends with fragment ig*4 + tsel,
      // channels csub .. csub + 3
      auto tr = [&](uint32_t p0, uint32_t p1, uint32_t& w0, uint32_t& w1) {
        const uint32_t keep = ce ? p1 : p0;
        const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(ce ? p0 : p1), 0xB1, 0xF, 0xF, false);
        const uint32_t lo = ce ? recv : keep, hi = ce ? keep : recv;
        const uint32_t d0 = (lo & 0xFFFFu) | (hi << 16), d1 = (lo >> 16) | (hi & 0xFFFF0000u);
        const uint32_t recv2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(cu ? d0 : d1), 0x4E, 0xF, 0xF, false);
        w0 = cu ? recv2 : d0;
        w1 = cu ? d1 : recv2;
      };
      uint32_t w0, w1, k0, k1;
      tr(pack2<DT>(best[0], best[1]), pack2<DT>(best[2], best[3]), w0, w1);
      tr(code[0] | (code[1] << 16), code[2] | (code[3] << 16), k0, k1);
      const int rowb = mw + (ig * 4 + tsel) * 16 + q * 4;  // first M row of this lane's window
      const int col = col0 + csub;
      if (rowb >= a.M || col >= a.OC) continue;
      const long long prow = rowb >> 2;
      if (DV_BOUNDS(prow * a.out_ld + col, 4, a.out_elems, "conv_dma pool epilogue out")) {
        *reinterpret_cast<uint2*>(out + prow * a.out_ld + col) = make_uint2(w0, w1);
        *reinterpret_cast<uint32_t*>(a.out_code + prow * a.OC + col) =
            (k0 & 0xFFu) | ((k0 >> 8) & 0xFF00u) | ((k1 & 0xFFu) << 16) | ((k1 >> 16) << 24);
      }
    }
  }
}

// Pooled-max epilogue staged through LDS (ConvArgs::pool_t == 2): the transposed (max, code) quads of
// epilogue_pool_t go to the freed operand stages as [BM/4 pooled rows][BN] values and codes, then every lane
// stores whole 16-B chunks of one pooled row (values: BN / 8 lanes per row, codes BN / 16): each store
// instruction writes complete row segments instead of 16 rows x 32 B (values) / 16 B (codes). The same change
// took 9-13 % off the persistent KW3P launches (profiles/kw3_epi_ab_r5.txt). Bit-identical to epilogue_pool_t.
// Swizzles (16-B chunk index XOR a function of the pooled row) make the quad-transposed ds_write_b64 /
// ds_write_b32 groups and the row-wise ds_read_b128 groups conflict-free.
template <int DT, int NT, int BM, int BN, int FM, int FN>
__device__ __forceinline__ void epilogue_pool_lds(const ConvArgs& a, const f32x4 (&acc)[FM][FN], uint8_t* smem, int m0,
                                                  int n0, int wm, int wn, int lane, int tid) {
  static_assert(FM % 4 == 0 && BN % 16 == 0, "pool LDS epilogue shape");
  constexpr int VROW = BN * 2, CROW = BN;  // bytes per pooled row: values / codes
  uint8_t* vs = smem;
  uint8_t* cs = smem + (BM / 4) * VROW;
  const int q = lane >> 4, cl = lane & 15, ce = cl & 1, cu = (cl >> 1) & 1, csub = cl & ~3, tsel = ce * 2 + cu;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col0 = n0 + wn * FN * 16 + j * 16;
    const float bias = (a.bias && col0 + cl < a.OC) ? a.bias[col0 + cl] : 0.f;
#pragma unroll
    for (int ig = 0; ig < FM / 4; ++ig) {
      float best[4];
      uint32_t code[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int i = ig * 4 + t;
        float b = -INFINITY;
        uint32_t c = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          v = to_f<DT>(from_f<DT>(v));
          if (v > b) {
            b = v;
            c = (uint32_t)r;
          }
        }
        best[t] = b;
        code[t] = c;
      }
      auto tr = [&](uint32_t p0, uint32_t p1, uint32_t& w0, uint32_t& w1) {
        const uint32_t keep = ce ? p1 : p0;
        const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(ce ? p0 : p1), 0xB1, 0xF, 0xF, false);
        const uint32_t lo = ce ? recv : keep, hi = ce ? keep : recv;
        const uint32_t d0 = (lo & 0xFFFFu) | (hi << 16), d1 = (lo >> 16) | (hi & 0xFFFF0000u);
        const uint32_t recv2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(cu ? d0 : d1), 0x4E, 0xF, 0xF, false);
        w0 = cu ? recv2 : d0;
        w1 = cu ? d1 : recv2;
      };
      uint32_t w0, w1, k0, k1;
      tr(pack2<DT>(best[0], best[1]), pack2<DT>(best[2], best[3]), w0, w1);
      tr(code[0] | (code[1] << 16), code[2] | (code[3] << 16), k0, k1);
      const int prl = (wm * FM * 16 + (ig * 4 + tsel) * 16 + q * 4) >> 2;  // pooled row in the tile
      const int cc = wn * FN * 16 + j * 16 + csub;                       // channel in the tile
      const int vch = (cc >> 3) ^ (((prl >> 2) & 3) << 1);
      *reinterpret_cast<uint2*>(vs + prl * VROW + (vch << 4) + (cc & 4) * 2) = make_uint2(w0, w1);
      const int cch = (cc >> 4) ^ (((prl >> 2) & 3) | ((prl & 1) << 2));
      *reinterpret_cast<uint32_t*>(cs + prl * CROW + (cch << 4) + (cc & 12)) =
          (k0 & 0xFFu) | ((k0 >> 8) & 0xFF00u) | ((k1 & 0xFFu) << 16) | ((k1 >> 16) << 24);
    }
  }
  __syncthreads();
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
  const int prow0 = m0 >> 2, prows = a.M >> 2;
  constexpr int VCPR = VROW / 16, CCPR = CROW / 16;  // 16-B chunks per pooled row
#pragma unroll
  for (int c = tid; c < (BM / 4) * VCPR; c += NT) {
    const int r = c / VCPR, pc = c % VCPR;
    const int lc = pc ^ (((r >> 2) & 3) << 1);
    const int col = n0 + lc * 8;
    if (prow0 + r >= prows || col >= a.OC) continue;
    const long long o = (long long)(prow0 + r) * a.out_ld + col;
    if (DV_BOUNDS(o, 8, a.out_elems, "conv_dma pool lds out"))
      *reinterpret_cast<uint4*>(out + o) = *reinterpret_cast<const uint4*>(vs + r * VROW + pc * 16);
  }
#pragma unroll
  for (int c = tid; c < (BM / 4) * CCPR; c += NT) {
    const int r = c / CCPR, pc = c % CCPR;
    const int lc = pc ^ (((r >> 2) & 3) | ((r & 1) << 2));
    const int col = n0 + lc * 16;
    if (prow0 + r >= prows || col >= a.OC) continue;
    *reinterpret_cast<uint4*>(a.out_code + (long long)(prow0 + r) * a.OC + col) =
        *reinterpret_cast<const uint4*>(cs + r * CROW + pc * 16);
  }
}

template <int DT, int FM, int FN, int EPI, bool accum>
__device__ __forceinline__ void epilogue(const ConvArgs& a, const f32x4 (&acc)[FM][FN], int mw, int nw, int lane) {
  if constexpr (EPI == CONV_E_POOL && FM % 4 == 0) {
    if (a.pool_t) {
      epilogue_pool_t<DT, FM, FN>(a, acc, mw, nw, lane);
      return;
    }
  }
  const int row_l = (lane >> 4) * 4;
  const int col_l = lane & 15;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int col = nw + j * 16 + col_l;
    if (col >= a.OC) continue;
    const float bias = a.bias ? a.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int rowb = mw + i * 16 + row_l;
      if (rowb >= a.M) continue;
      if constexpr (EPI == CONV_E_POOL) {
        float best = -INFINITY;
        int code = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          v = to_f<DT>(from_f<DT>(v));
          if (v > best) {
            best = v;
            code = r;
          }
        }
        const long long prow = rowb >> 2;
        if (!DV_BOUNDS(prow * a.out_ld + col, 1, a.out_elems, "conv_dma pool epilogue out")) continue;
        reinterpret_cast<uint16_t*>(a.out)[prow * a.out_ld + col] = from_f<DT>(best);
        a.out_code[prow * a.OC + col] = (uint8_t)code;
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = rowb + r;
          if (row >= a.M) continue;
          float v = acc[i][j][r] + bias;
          if (relu_at(a, col)) v = fmaxf(v, 0.f);
          const long long o = (long long)row * a.out_ld + col;
          if (!DV_BOUNDS(o, 1, a.out_elems, "conv_dma epilogue out")) continue;
          if constexpr (EPI == CONV_E_F32) {
            float* out = reinterpret_cast<float*>(a.out);
            if (accum) v += out[o];
            out[o] = v;
          } else {
            uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
            if (accum) v += to_f<DT>(out[o]);
            out[o] = from_f<DT>(v);
          }
        }
      }
    }
  }
}

// one 16-bit output chunk's v (+ accumulate operand ad) (+ residual rs) [ReLU after a residual]
template <int DT>
__device__ __forceinline__ uint4 epi_combine(const ConvArgs& a, uint4 v, uint4 ad, uint4 rs) {
  const uint32_t vv[4] = {v.x, v.y, v.z, v.w}, aa[4] = {ad.x, ad.y, ad.z, ad.w}, rr[4] = {rs.x, rs.y, rs.z, rs.w};
  uint32_t ov[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    float lo = to_f<DT>(vv[e] & 0xFFFFu) + to_f<DT>(aa[e] & 0xFFFFu) + to_f<DT>(rr[e] & 0xFFFFu);
    float hi = to_f<DT>(vv[e] >> 16) + to_f<DT>(aa[e] >> 16) + to_f<DT>(rr[e] >> 16);
    if (a.relu && a.res) {
      lo = fmaxf(lo, 0.f);
      hi = fmaxf(hi, 0.f);
    }
    ov[e] = pack2<DT>(lo, hi);
  }
  return uint4{ov[0], ov[1], ov[2], ov[3]};
}

// a row's last partial chunk (OC % 8): element-wise, no 16-B access past OC
template <int DT>
__device__ __forceinline__ void epi_tail(const ConvArgs& a, uint4 v, int grow, int gcol, long long o) {
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
  if (!DV_BOUNDS(o, a.OC - gcol, a.out_elems, "conv_dma epilogue tail out")) return;
  const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
  for (int e = 0; e < a.OC - gcol; ++e) {
    float f = to_f<DT>((vv[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
    if (a.accumulate) f += to_f<DT>(out[o + e]);
    if (a.res) {
      f += to_f<DT>(a.res[(long long)grow * a.res_ld + gcol + e]);
      if (relu_at(a, gcol + e)) f = fmaxf(f, 0.f);
    }
    if (a.emask) {
      const uint32_t m = a.emask[(long long)grow * a.emask_ld + gcol + e];
      if (m == 0u || (m & 0x8000u)) f = 0.f;
    }
    out[o + e] = from_f<DT>(f);
  }
}

// LDS-staged 16-bit epilogue. The MFMA C layout gives each lane 4 rows x 1 column per 16x16
// block, i.e. 2-byte scattered stores; instead the tile is written to LDS (the freed operand
// stages, 16-B chunks XOR-swizzled by row) and read back as 8-channel chunks: every global
// store, residual load, emask load and accumulate load is one 16-B access. Semantics as
// epilogue/epilogue_res: v = acc + bias, [ReLU] (before a += out), + res, [ReLU] (after a res
// add), zeroed where emask <= 0. Stores of a row's last partial chunk (OC % 8) go per element.
template <int DT, int NT, int BM, int BN, int FM, int FN>
__device__ __forceinline__ void epilogue_lds(const ConvArgs& a, const f32x4 (&acc)[FM][FN], uint8_t* smem, int m0,
                                             int n0, int wm, int wn, int lane, int tid, bool writer) {
  constexpr int CPR = BN / 8;                       // 16-B chunks per C-tile row
  constexpr int SWZ = (CPR < 8 ? CPR : 8) - 1;
  const int col_l = lane & 15;
  const bool pre_relu = a.relu && a.res == nullptr;
  // C tile -> LDS: each 16 x 16 block's 4 rows x 1 column per lane are transposed within the lane quad
  // (two DPP swaps, as the KW3P epilogue) to 1 row x 4 consecutive columns, written as ONE ds_write_b64
  // (the per-element form was 4 converts, 4 address computations and 4 ds_write_b16 per block)
  const int ce = col_l & 1, cu = (col_l >> 1) & 1;
  const int rsub = (lane >> 4) * 4 + ce * 2 + cu, csub = col_l & ~3;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    if (!writer) break;
    const int gcol = n0 + wn * FN * 16 + j * 16 + col_l;
    const float bias = (a.bias && gcol < a.OCpad) ? a.bias[gcol] : 0.f;
    const bool rl = pre_relu && relu_at(a, gcol);
    const int col = wn * FN * 16 + j * 16 + csub;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      float f0 = acc[i][j][0] + bias, f1 = acc[i][j][1] + bias, f2 = acc[i][j][2] + bias, f3 = acc[i][j][3] + bias;
      if (rl) {
        f0 = fmaxf(f0, 0.f);
        f1 = fmaxf(f1, 0.f);
        f2 = fmaxf(f2, 0.f);
        f3 = fmaxf(f3, 0.f);
      }
      const uint32_t p0 = pack2<DT>(f0, f1), p1 = pack2<DT>(f2, f3);
      const uint32_t keep = ce ? p1 : p0;
      const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(ce ? p0 : p1), 0xB1, 0xF, 0xF, false);
      const uint32_t lo = ce ? recv : keep, hi = ce ? keep : recv;
      const uint32_t d0 = (lo & 0xFFFFu) | (hi << 16), d1 = (lo >> 16) | (hi & 0xFFFF0000u);
      const uint32_t recv2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(cu ? d0 : d1), 0x4E, 0xF, 0xF, false);
      const int row = wm * FM * 16 + i * 16 + rsub;
      *reinterpret_cast<uint2*>(smem + row * (BN * 2) + ((((col >> 3) ^ (row & SWZ))) << 4) + (col & 7) * 2) =
          make_uint2(cu ? recv2 : d0, cu ? d1 : recv2);
    }
  }
  __syncthreads();
  uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
  const bool post = a.accumulate || a.res != nullptr;
  // Batched operand loads: with residual / accumulate / output-mask operands, each thread first
  // issues the loads of ALL its (<= 8) chunks, then combines and stores, so the chunks' HBM round
  // trips overlap instead of serializing once per loop iteration. Fully unrolled with constant
  // indices (the operand arrays stay in VGPRs; the C tile is already in LDS, acc is dead here).
  // The short-K GEMMs with such epilogues (ResNet block convs and dgrads, K = 64..576) are
  // epilogue-latency bound. DV_NO_EPI_BATCH=1 (host) falls back to the per-chunk loop (A/B).
  constexpr int ITER = (BM * CPR + NT - 1) / NT;
  if constexpr (ITER <= 8) {
    if (a.epi_batch && a.ucode == nullptr && (post || a.emask != nullptr || a.ebits != nullptr || a.obits != nullptr)) {
      uint4 rv[ITER], av[ITER], mv[ITER];
      uint32_t eb[ITER];
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        rv[it] = av[it] = mv[it] = uint4{0u, 0u, 0u, 0u};
        eb[it] = 0u;
        const int c = tid + it * NT;
        const int row = c / CPR, cc = c % CPR;
        const int grow = m0 + row, gcol = n0 + cc * 8;
        if (c >= BM * CPR || grow >= a.M || gcol + 8 > a.OC) continue;
        const long long o = (long long)grow * a.out_ld + gcol;
        if (a.accumulate && DV_BOUNDS(o, 8, a.out_elems, "conv_dma epilogue_lds acc load"))
          av[it] = *reinterpret_cast<const uint4*>(out + o);
        if (a.res && DV_BOUNDS((long long)grow * a.res_ld + gcol, 8, a.res_elems, "conv_dma epilogue_lds res load"))
          rv[it] = *reinterpret_cast<const uint4*>(a.res + (long long)grow * a.res_ld + gcol);
        if (a.ebits)
          eb[it] = a.ebits[(long long)grow * a.ebits_ld + (gcol >> 3)];
        else if (a.emask &&
                 DV_BOUNDS((long long)grow * a.emask_ld + gcol, 8, a.emask_elems, "conv_dma epilogue_lds emask load"))
          mv[it] = *reinterpret_cast<const uint4*>(a.emask + (long long)grow * a.emask_ld + gcol);
      }
#pragma unroll
      for (int it = 0; it < ITER; ++it) {
        const int c = tid + it * NT;
        const int row = c / CPR, cc = c % CPR;
        const int grow = m0 + row, gcol = n0 + cc * 8;
        if (c >= BM * CPR || grow >= a.M || gcol >= a.OC) continue;
        uint4 v = *reinterpret_cast<const uint4*>(smem + row * (BN * 2) + ((cc ^ (row & SWZ)) << 4));
        const long long o = (long long)grow * a.out_ld + gcol;
        if (gcol + 8 > a.OC) {
          epi_tail<DT>(a, v, grow, gcol, o);
          continue;
        }
        if (!DV_BOUNDS(o, 8, a.out_elems, "conv_dma epilogue_lds out")) continue;
        if (post) v = epi_combine<DT>(a, v, av[it], rv[it]);
        if (a.ebits) {
          v = mask_bits8(v, eb[it]);
        } else if (a.emask) {
          v.x = mask_pos_pk(v.x, mv[it].x);
          v.y = mask_pos_pk(v.y, mv[it].y);
          v.z = mask_pos_pk(v.z, mv[it].z);
          v.w = mask_pos_pk(v.w, mv[it].w);
        }
        *reinterpret_cast<uint4*>(out + o) = v;
        if (a.obits) a.obits[(long long)grow * a.obits_ld + (gcol >> 3)] = (uint8_t)pos_bits8(v);
      }
      return;
    }
  }
  for (int c = tid; c < BM * CPR; c += NT) {
    const int row = c / CPR, cc = c % CPR;
    const int grow = m0 + row, gcol = n0 + cc * 8;
    if (grow >= a.M || gcol >= a.OC) continue;
    uint4 v = *reinterpret_cast<const uint4*>(smem + row * (BN * 2) + ((cc ^ (row & SWZ)) << 4));
    if (a.out2 != nullptr && gcol >= a.split_col) {  // two-destination merged GEMM (plain epilogue)
      const long long o2 = (long long)grow * a.out2_ld + (gcol - a.split_col);
      if (DV_BOUNDS(o2, 8, a.out2_elems, "conv_dma epilogue_lds out2"))
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out2) + o2) = v;
      continue;
    }
    const long long o = (long long)grow * a.out_ld + gcol;
    if (!a.ucode && !DV_BOUNDS(o, gcol + 8 > a.OC ? a.OC - gcol : 8, a.out_elems, "conv_dma epilogue_lds out")) continue;
    if (a.res && !DV_BOUNDS((long long)grow * a.res_ld + gcol, gcol + 8 > a.OC ? a.OC - gcol : 8, a.res_elems,
                            "conv_dma epilogue_lds res"))
      continue;
    if (a.emask && !DV_BOUNDS((long long)grow * a.emask_ld + gcol, gcol + 8 > a.OC ? a.OC - gcol : 8, a.emask_elems,
                              "conv_dma epilogue_lds emask"))
      continue;
    if (gcol + 8 > a.OC) {  // a row's last partial chunk: element-wise (no 16-B access past OC)
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      for (int e = 0; e < a.OC - gcol; ++e) {
        float f = to_f<DT>((vv[e >> 1] >> (16 * (e & 1))) & 0xFFFFu);
        if (a.accumulate) f += to_f<DT>(out[o + e]);
        if (a.res) {
          f += to_f<DT>(a.res[(long long)grow * a.res_ld + gcol + e]);
          if (relu_at(a, gcol + e)) f = fmaxf(f, 0.f);
        }
        if (a.emask) {
          const uint32_t m = a.emask[(long long)grow * a.emask_ld + gcol + e];
          if (m == 0u || (m & 0x8000u)) f = 0.f;
        }
        out[o + e] = from_f<DT>(f);
      }
      continue;
    }
    if (post) {
      uint4 ad = {0u, 0u, 0u, 0u}, rs = {0u, 0u, 0u, 0u};
      if (a.accumulate) ad = *reinterpret_cast<const uint4*>(out + o);
      if (a.res) rs = *reinterpret_cast<const uint4*>(a.res + (long long)grow * a.res_ld + gcol);
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w}, aa[4] = {ad.x, ad.y, ad.z, ad.w}, rr[4] = {rs.x, rs.y, rs.z, rs.w};
      uint32_t ov[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = to_f<DT>(vv[e] & 0xFFFFu) + to_f<DT>(aa[e] & 0xFFFFu) + to_f<DT>(rr[e] & 0xFFFFu);
        float hi = to_f<DT>(vv[e] >> 16) + to_f<DT>(aa[e] >> 16) + to_f<DT>(rr[e] >> 16);
        if (a.relu && a.res) {
          lo = fmaxf(lo, 0.f);
          hi = fmaxf(hi, 0.f);
        }
        ov[e] = pack2<DT>(lo, hi);
      }
      v = uint4{ov[0], ov[1], ov[2], ov[3]};
    }
    if (a.ebits) {
      v = mask_bits8(v, a.ebits[(long long)grow * a.ebits_ld + (gcol >> 3)]);
    } else if (a.emask) {
      const uint4 em = *reinterpret_cast<const uint4*>(a.emask + (long long)grow * a.emask_ld + gcol);
      v.x = mask_pos_pk(v.x, em.x);
      v.y = mask_pos_pk(v.y, em.y);
      v.z = mask_pos_pk(v.z, em.z);
      v.w = mask_pos_pk(v.w, em.w);
    }
    if (a.obits) a.obits[(long long)grow * a.obits_ld + (gcol >> 3)] = (uint8_t)pos_bits8(v);
    if (a.ucode) {  // max-unpool: the value goes to the window position its switch code names, 0 elsewhere
      const int hw = a.OH * a.OW;
      const int n = grow / hw, rem = grow - n * hw;
      const int oh = rem / a.OW, ow = rem - oh * a.OW;
      const uint2 cd = *reinterpret_cast<const uint2*>(a.ucode + ((long long)(n / a.ucode_div) * hw + rem) * a.OC + gcol);
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      const long long ob = (((long long)n * 2 * a.OH + 2 * oh) * 2 * a.OW + 2 * ow) * a.out_ld + gcol;
#pragma unroll
      for (int pos = 0; pos < 4; ++pos) {
        uint32_t ov[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint32_t cw = e < 2 ? cd.x : cd.y;
          const uint32_t c0 = (cw >> (16 * (e & 1))) & 0xFFu, c1 = (cw >> (16 * (e & 1) + 8)) & 0xFFu;
          ov[e] = (c0 == (uint32_t)pos ? vv[e] & 0xFFFFu : 0u) | (c1 == (uint32_t)pos ? vv[e] & 0xFFFF0000u : 0u);
        }
        const long long po = ob + ((long long)(pos >> 1) * 2 * a.OW + (pos & 1)) * a.out_ld;
        if (DV_BOUNDS(po, 8, a.out_elems, "conv_dma unpool-out store"))
          *reinterpret_cast<uint4*>(out + po) = uint4{ov[0], ov[1], ov[2], ov[3]};
      }
      continue;
    }
    *reinterpret_cast<uint4*>(out + o) = v;
  }
}

// ---------------------------------------------------------------------------------------------
// KW3: 3x3 / stride 1 / pad 1 forward conv, 256 x 256 tile, where the three kw taps of a kernel row
// share ONE staged A tile. A K step is (kernel row kh, 32-channel chunk): the A tile holds the
// kernel-row-kh input pixels of the tile's output rows, B the three kw sub-tiles of the weights
// (A ~17-19 KB + B 3 x 256 x 64 B per step: 1.47x fewer staged bytes per FLOP than the plain
// implicit GEMM, which stages A once per tap).
//
// Zero-padded slot layout: the A tile is staged in *padded* pixel coordinates, W + 8 slots per
// image row ([0 x 4, pixel 0 .. pixel W-1, 0 x 4]), so output row r's kw tap is simply
// slot(r) + kw - 1 and the conv's left/right zero padding are real zero slots (the DMA's
// out-of-range offset writes zeros). Eight pad slots make consecutive output rows across an image
// row boundary 9 slots apart, i.e. the same slot index mod 8 as adjacent rows, so a 16-row fragment
// read that spans a boundary is as conflict-free as one that does not (with 2 pad slots, as first
// built this round, KW3 ran at SQ_LDS_BANK_CONFLICT / IDX_ACTIVE 0.19). A 256-row tile touching b
// image-row boundaries stages 258 + 8b slots (<= 512: W >= 9, host check; 160 KiB of LDS). The
// round-1..2 layout staged 258 unpadded rows and zeroed the border rows of the A fragments in
// registers: 64 v_cndmask per wave per K step, each sub-step's MFMAs waiting on ALL its fragment
// reads first. Now every A fragment address is a per-lane constant (FM x 3 VGPRs, one v_add each
// per step for the stage offset; LDS: B0 | B1 | A0 | A1).
// K step order: kh innermost (step = 3 cc + kh). The A tiles of kh = 0, 1, 2 for one channel chunk
// are the same pixels shifted by one image row, so two of every three steps find their A rows in
// L2 (the round-1..3 order, cc innermost, read a new 64-B chunk of every pixel each step): config-2
// KW3 launches 0-4 % faster (tools/kw3_ab.py, profiles/kw3_ab_r4.txt; an ablation without the DMA
// showed the A stream costing 4-13 % of a launch on the HBM-streamed 56^2 / 28^2 maps).
// LDS rows are 64 B with the 16-B chunk XOR-swizzled by bit 2 of the slot (q ^ 2((slot >> 2) & 1)):
// conflict-free ds_read_b128 fragment reads for 16 slots of consecutive indices mod 8 at any base.
namespace {
__device__ __forceinline__ int kw3_swz(int row) { return ((row >> 2) & 1) << 1; }
// staged A slots per workgroup: 8 waves x 16 x A_I >= BM + 2 + 8 x (row boundaries), host-checked
constexpr int kw3_a_i(int bm) { return bm == 256 ? 4 : 5; }
constexpr int kKw3Pad = 8;  // zero slots between image rows: a row jump is +9 slots = +1 (mod 8)
constexpr int kKw3DefaultVar = 2;
}  // namespace

// BM_ x BN_: 256 x 256 (8 waves of 128 x 64) or 512 x 128 (8 waves of 128 x 64: the same per-wave
// MFMA:LDS-read ratio and FLOPs per K step as 256 x 256, for 128-channel outputs; the round-1..2
// 256 x 128 tile ran 8 waves of 64 x 64 at MFMA util 0.35, profiles/pmc_c2_r3.txt).
// (Measured and removed, round 3: issuing the next step's DMAs in three parts between the kw
// sub-steps' fragment reads and MFMAs instead of all right after the barrier: config 2 fell from
// 6.85-7.03k to 5.80-5.83k img/s, profiles/bench_c2_r3_ab.txt. Equal within noise and removed:
// static priority for waves 4-7 instead of the per-sub-step flips, a 320-row M tile, and the DMAs
// issued behind the first sub-step's fragment reads, profiles/kw3_variants_r3.txt.)
// VAR (kw3_var(), DV_KW3_VAR): 0 = this kernel; 2 (default) = the persistent KW3P kernel below for
// plain epilogues (this kernel otherwise); 8 / 9: ablations for tools/kw3_ab.py only (no epilogue
// stores / no K loop): NOT correct outputs.
template <int DT, int EPI, int BN_ = 256, int BM_ = 256, int VAR = 0>
__global__ void __launch_bounds__(512) conv_dma_kw3_kernel(const ConvArgs a, int tiles_n) {
  constexpr int BN = BN_, BM = BM_, NW = 8;
  constexpr int WN = BN / 64, FN = 4, WM = NW / WN, FM = BM / (16 * WM);
  constexpr int A_I = kw3_a_i(BM);         // A DMA instructions (16 slots each) per wave
  constexpr int B_I = 3 * BN / 16 / NW;    // B: 3 kw sub-tiles x BN rows (6 / 3 per wave)
  constexpr int A_BYTES = A_I * NW * 1024, B_BYTES = 3 * BN * 64;
  static_assert(BM * BN * 2 <= 2 * (A_BYTES + B_BYTES), "C tile must fit in the operand stages");
  typedef typename Vec8<DT>::type v8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int tile_n = wgid % tiles_n, tile_m = wgid / tiles_n;
  const int m0 = a.m_base + tile_m * BM, n0 = tile_n * BN;
  const int H = a.H, W = a.W, C = a.C, HW = a.H * a.W, Wp = a.W + kKw3Pad;

  const int n_base = (m0 < a.M ? m0 : a.M - 1) / HW;
  const long long img_elems = (long long)HW * a.x_ld;
  const long long x_total = (long long)a.N * img_elems;
  const __amdgpu_buffer_rsrc_t xr =
      make_rsrc(a.x + (long long)n_base * img_elems, (uint64_t)(x_total - (long long)n_base * img_elems) * 2);
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (uint64_t)a.OCpad * a.Kpad * 2);

  // padded coordinate of output row m (global image row R = m / W, W + 8 slots per row: 4 zero
  // slots on each side, so consecutive output rows across a row boundary sit 9 slots apart, the
  // same slot index mod 8 as adjacent ones: the bit-2 swizzle stays conflict-free for them)
  auto padded = [&](int m) {
    const int R = m / W;
    return R * Wp + kKw3Pad / 2 + (m - R * W);
  };
  const int P0 = padded(m0) - 1;                    // slot 0: the left neighbour of row m0
  const int nslots = padded(m0 + BM - 1) - P0 + 2;  // through the right neighbour of row m0 + 255

  // DMA lanes: 16 slots x 4 chunks per instruction; slot group bases are multiples of 16
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ kw3_swz(lrow);
  int r_pix[A_I], r_oh[A_I];
#pragma unroll
  for (int u = 0; u < A_I; ++u) {
    const int t = (u * NW + wave) * 16 + lrow;
    const int P = P0 + t;
    const int R = P / Wp, c = P - R * Wp;
    const int px = c - kKw3Pad / 2;
    const int m = R * W + px;
    const bool valid = t < nslots && px >= 0 && px < W && m < a.M;  // else a zero slot
    const int n = R / H, oh = R - n * H;
    r_pix[u] = valid ? (n - n_base) * HW + oh * W + px : 0;
    r_oh[u] = valid ? oh : -(1 << 28);
  }
  const int nch = C / 32;
  const int nsteps = 3 * nch;
  auto issue = [&](int step, int buf) {
    const int kh = step % 3, cc = step / 3;  // kh innermost (see the KW3 header)
    uint8_t* As = smem + 2 * B_BYTES + buf * A_BYTES;
    uint8_t* Bs = smem + buf * B_BYTES;
#pragma unroll
    for (int u = 0; u < A_I; ++u) {
      if ((u * NW + wave) * 16 >= nslots) continue;  // slots past the tile's last are never read
      const bool ok = (unsigned)(r_oh[u] + kh - 1) < (unsigned)H;
      const uint32_t voff =
          ok ? ((uint32_t)(r_pix[u] + (kh - 1) * W) * (uint32_t)a.x_ld + (uint32_t)(cc * 32 + lchunk * 8)) * 2u : kOOB;
      dma16(xr, As + (u * NW + wave) * 1024, voff);
    }
#pragma unroll
    for (int u = 0; u < B_I; ++u) {
      const int v = u * NW + wave;  // kw sub-tile v >> 4, rows (v & 15) * 16 + lrow
      const int kw = v / (BN / 16), brow = (v % (BN / 16)) * 16 + lrow;
      const uint32_t voff =
          ((uint32_t)(n0 + brow) * (uint32_t)a.Kpad + (uint32_t)((kh * 3 + kw) * C + cc * 32 + lchunk * 8)) * 2u;
      dma16(wr, Bs + v * 1024, voff);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q = lane >> 4;
  const int arow0 = wm * FM * 16 + (lane & 15);
  const int brow0 = wn * FN * 16 + (lane & 15);
  const int bswz = ((q ^ kw3_swz(brow0)) << 4);  // brow0 + 16 j: same bit 2
  // per-lane LDS byte addresses: A fragments (stage 0; stage 1 = + A_BYTES) and the B base of each
  // stage; opaque so each stays ONE VGPR (the compiler otherwise re-splits them into base + swizzle
  // pairs: 2 VALU per fragment read and 241 VGPRs)
  int aaddr[FM][3];
#pragma unroll
  for (int i = 0; i < FM; ++i) {
    const int s1 = padded(m0 + arow0 + i * 16) - P0;  // the kw = 1 slot of this lane's row
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      const int sl = s1 + kw - 1;
      aaddr[i][kw] = 2 * B_BYTES + sl * 64 + ((q ^ kw3_swz(sl)) << 4);
      asm volatile("" : "+v"(aaddr[i][kw]));
    }
  }
  int baddr[2];
  baddr[0] = brow0 * 64 + bswz;
  baddr[1] = baddr[0] + B_BYTES;
  asm volatile("" : "+v"(baddr[0]), "+v"(baddr[1]));

  issue(0, 0);
  const int nk = VAR == 9 ? 0 : nsteps;
  for (int k = 0; k < nk; ++k) {
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    const int aoff = (k & 1) * A_BYTES;
    const uint8_t* Bs = smem + baddr[k & 1];
    if (k + 1 < nsteps) issue(k + 1, (k + 1) & 1);
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      v8 bf[FN], af[FM];
#pragma unroll
      for (int j = 0; j < FN; ++j) bf[j] = *reinterpret_cast<const v8*>(Bs + kw * (BN * 64) + j * 1024);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const v8*>(smem + aoff + aaddr[i][kw]);
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af[i], bf[j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  wait_vm<0>();
  if constexpr (VAR == 8) {  // ablation: keep the accumulators live, store nothing
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) asm volatile("" ::"v"(acc[i][j]));
    return;
  }

  if constexpr (EPI == CONV_E_BF16) {
    if (a.vec_epi) {
      __syncthreads();
      epilogue_lds<DT, NW * 64, BM, BN, FM, FN>(a, acc, smem, m0, n0, wm, wn, lane, tid);
      return;
    }
    if (a.res || a.emask) {
      epilogue_res<DT, FM, FN>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
      return;
    }
  }
  if (a.accumulate)
    epilogue<DT, FM, FN, EPI, true>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
  else
    epilogue<DT, FM, FN, EPI, false>(a, acc, m0 + wm * FM * 16, n0 + wn * FN * 16, lane);
}

// ---------------------------------------------------------------------------------------------
// KW3P: persistent KW3 for plain 16-bit epilogues (no residual / emask / accumulate / unpool / split
// output). tools/kw3_ab.py priced the non-persistent kernel's tile boundaries on the config-2 shapes:
// without epilogue stores a launch runs 9-14 % faster (VAR 8) and prologue + epilogue alone are
// 12-17 % of it (VAR 9). Every workgroup of a round reaches its epilogue at the same moment, so the
// whole chip writes its C tiles (32 MB for 256 256 x 256 tiles) in one burst while no MFMA runs,
// and the next round starts with every CU waiting for its first DMA. Here one workgroup per CU walks
// tiles v = blockIdx.x, + gridDim.x, ... (XCD-remapped as before) and
//   * the LAST K step of tile t issues step 0 of tile t + 1 (its gather state computed there), so
//     the next tile's first operands land while this tile's last MFMAs and epilogue run;
//   * the epilogue never touches LDS: each 16 x 16 accumulator block is transposed in registers by
//     two DPP lane swaps (quad_perm [1,0,3,2], then [2,3,0,1]) so a lane holds 4 consecutive
//     channels of one pixel, and goes out as one 8-B buffer store (rows past M: out-of-range
//     offset, discarded);
//   * those stores drain while tile t + 1's first K step computes (the wait at the end of that step
//     is the first one that covers them).
// Main loop: a fragment pipeline (the next kw sub-step's B fragments read into a second register
// set, each A fragment register refilled with the next sub-step's fragment right after its 4
// MFMAs; the order pinned by sched_group_barrier), so only a K step's first sub-step waits for LDS
// reads. Numerics equal the LDS-staged epilogue (same fp32 ops, same rounding). Buffer parity
// follows a global step counter (odd step counts per tile).
// Measured (tools/kw3_ab.py, profiles/kw3_ab_r4.txt): 2-4 % faster per launch than KW3 on every
// config-2 shape. Measured and removed: the fragment pipeline alone in the non-persistent kernel
// (-2 % .. +2 %, noise) and the next step's DMA pieces issued one per MFMA group instead of all
// after the first reads (-3 % .. +3 % vs this kernel, shape-dependent).
//
// UNP = true: the max-unpool-out epilogue (the deconvnet's block{3,4,5}_conv1.down, which write the
// 2x-upsampled map with each value at its switch position and zeros elsewhere). Round 4 tried the
// register-transposed form (each lane's 4 channels stored to the 4 window positions as 8-B stores):
// bit-identical but config 2 -3 %, because 8-B stores to every other pixel touch 32-B pieces of many
// lines. Here each wave stages its 128 x 64 C tile through a private 4 KiB slice of the LDS stage the
// last K step just released (32 rows per pass, 4 passes), reads it back as 16-B chunks (8 lanes per
// row: every unpooled store instruction writes 8 whole 128-B lines) and stores value-or-zero to the
// 4 window positions. The switch codes of all 16 of a lane's rows are loaded before the first pass.
// One workgroup barrier per tile (after the last pass's LDS reads) keeps the next tile's first DMA
// into that stage behind every wave's reads; the stores drain behind the next tile's first K step.
// LDS layout per wave slice: row r (128 B) holds its 8 chunks at chunk ^ 2 (r & 3): the quad-
// transposed ds_write_b64 of 4 rows x 4 column groups hits 16 distinct 8-B slots per lane group, and
// each lane reads the chunk physically at (lane & 7) of row lane >> 3 (conflict-free ds_read_b128).
// SV (store variant, timing experiments through DV_KW3_VAR): 0 = default, 1 = no epilogue stores (ablation:
// wrong outputs), 2 = non-temporal (nt) epilogue stores.
//
// SK = true: stream-K. The plain persistent walk (tile v, v + G, ...) ends every workgroup's tiles at the
// same moment, so the whole chip writes its C tiles in one burst and the next tile's first K step waits
// for it (tools/kw3_ab.py, VAR 10 = no epilogue stores: 5-9 % faster on the plain config-2 shapes, 10-15 %
// on the unpool-out ones, profiles/kw3_store_ablation_r5.txt), and a grid of R.f rounds pays a whole
// round (or a 128 x 128 tail launch, kw3_split) for its fraction f. Here the G = gridDim workgroups of
// each output-column group (tile_n; the tiles_n groups interleave so the two workgroups sharing a row
// range sit side by side on one XCD and share its A rows in L2) split the group's tiles_m x nsteps
// K steps into G / tiles_n equal contiguous ranges: every workgroup does the same work, and its tile
// boundaries sit at a different K-step phase than its neighbours', so the C-tile stores of the chip
// are spread over the whole launch. A range of >= nsteps steps (host-checked) starts with at most one
// partial tile (its tail K steps) and ends with at most one (its head steps): the tail piece is computed
// first and published as fp32 partial accumulators (write-through sc1 stores, counted drain, barrier,
// one agent-scope flag store: the MI355X hand-off recipe); the workgroup holding the head finishes it
// last, polls the flag (bounded), reads the partial with sc1 loads and applies the epilogue to the sum.
// Split tiles round differently from one-pass accumulation (fp32, tests compare to the reference).
// EM (epilogue mode): 0 = register-transposed 8-B stores; 1 = max-unpool-out through the per-wave LDS slices
// (UNP below); 2 = the same LDS slices for the plain output: 16-B stores, every store instruction writes
// 8 whole 128-B line segments instead of 16 rows x 32 B (the default; DV_KW3P_EPI=reg for mode 0, A/B).
// Mode 0's scattered 8-B stores cost 9-13 % of a config-2 KW3P launch (a no-store ablation ran 11-15 %
// faster); mode 2 recovers most of it (profiles/kw3_epi_ab_r5.txt).
template <int DT, int BN_ = 256, int BM_ = 256, int EM = 0, int SV = 0, bool SK = false>
__global__ void __launch_bounds__(512) conv_dma_kw3p_kernel(const ConvArgs a, int tiles_n, int ntiles, int use_pre) {
  constexpr bool UNP = EM == 1, LDSEPI = EM != 0;
  constexpr int BN = BN_, BM = BM_, NW = 8;
  constexpr int WN = BN / 64, FN = 4, WM = NW / WN, FM = BM / (16 * WM);
  constexpr int A_I = kw3_a_i(BM);
  constexpr int B_I = 3 * BN / 16 / NW;
  constexpr int A_BYTES = A_I * NW * 1024, B_BYTES = 3 * BN * 64;
  typedef typename Vec8<DT>::type v8;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * (A_BYTES + B_BYTES)];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int H = a.H, W = a.W, C = a.C, HW = a.H * a.W, Wp = a.W + kKw3Pad;
  const long long img_elems = (long long)HW * a.x_ld;
  const long long x_total = (long long)a.N * img_elems;
  const __amdgpu_buffer_rsrc_t wr = make_rsrc(a.w, (uint64_t)a.OCpad * a.Kpad * 2);
  const __amdgpu_buffer_rsrc_t orr = make_rsrc(a.out, (uint64_t)a.out_elems * 2);
  const int lrow = lane >> 2;
  const int lchunk = (lane & 3) ^ kw3_swz(lrow);
  const int q = lane >> 4;
  const int arow0 = wm * FM * 16 + (lane & 15);
  const int brow0 = wn * FN * 16 + (lane & 15);
  int baddr0 = brow0 * 64 + ((q ^ kw3_swz(brow0)) << 4);  // stage 1: + B_BYTES
  asm volatile("" : "+v"(baddr0));
  const int nch = C / 32;
  const int nsteps = 3 * nch;

  auto padded = [&](int m) {
    const int R = m / W;
    return R * Wp + kKw3Pad / 2 + (m - R * W);
  };

  // ---- gather state of the tile whose DMAs are being issued ----
  int m0 = 0, n0 = 0, P0 = 0, nslots = 0;
  // per A slot: (pixel index relative to the tile's first image) << 12 | output row oh, or ~0 for a
  // zero slot (host: H < 4096 and 2 HW + BM < 2^19); one VGPR per slot instead of two
  uint32_t r_po[A_I];
  __amdgpu_buffer_rsrc_t xr = make_rsrc(a.x, 16);
  auto setup = [&](int tile_m, int tile_n) {
    m0 = a.m_base + tile_m * BM;
    n0 = tile_n * BN;
    const int n_base = (m0 < a.M ? m0 : a.M - 1) / HW;
    xr = make_rsrc(a.x + (long long)n_base * img_elems, (uint64_t)(x_total - (long long)n_base * img_elems) * 2);
    P0 = padded(m0) - 1;
    nslots = padded(m0 + BM - 1) - P0 + 2;
#pragma unroll
    for (int u = 0; u < A_I; ++u) {
      const int t = (u * NW + wave) * 16 + lrow;
      const int P = P0 + t;
      const int R = P / Wp, c = P - R * Wp;
      const int px = c - kKw3Pad / 2;
      const int m = R * W + px;
      const bool valid = t < nslots && px >= 0 && px < W && m < a.M;
      const int n = R / H, oh = R - n * H;
      r_po[u] = valid ? ((uint32_t)((n - n_base) * HW + oh * W + px) << 12) | (uint32_t)oh : ~0u;
    }
  };
  // SV 3 / 4 (timing ablations, WRONG outputs): after the first step, no DMA at all / no weight (B) DMA:
  // how much of a launch waits on operand staging (tools/kw3_ab.py VAR 20 / 21)
  bool abl_first = true;
  auto issue = [&](int step, int buf) {
    const int kh = step % 3, cc = step / 3;  // kh innermost (see the KW3 header)
    uint8_t* As = smem + 2 * B_BYTES + buf * A_BYTES;
    uint8_t* Bs = smem + buf * B_BYTES;
    const bool abl_skip = (SV == 3 || SV == 4) && !abl_first;
    abl_first = false;
    if (SV == 3 && abl_skip) return;
#pragma unroll
    for (int u = 0; u < A_I; ++u) {
      if ((u * NW + wave) * 16 >= nslots) continue;
      const int oh = (int)(r_po[u] & 0xFFFu), pix = (int)(r_po[u] >> 12);
      const bool ok = r_po[u] != ~0u && (unsigned)(oh + kh - 1) < (unsigned)H;
      const uint32_t voff =
          ok ? ((uint32_t)(pix + (kh - 1) * W) * (uint32_t)a.x_ld + (uint32_t)(cc * 32 + lchunk * 8)) * 2u : kOOB;
      dma16(xr, As + (u * NW + wave) * 1024, voff);
    }
    if (SV == 4 && abl_skip) return;
#pragma unroll
    for (int u = 0; u < B_I; ++u) {
      const int vv = u * NW + wave;
      const int kw = vv / (BN / 16), brow = (vv % (BN / 16)) * 16 + lrow;
      const uint32_t voff =
          ((uint32_t)(n0 + brow) * (uint32_t)a.Kpad + (uint32_t)((kh * 3 + kw) * C + cc * 32 + lchunk * 8)) * 2u;
      dma16(wr, Bs + vv * 1024, voff);
    }
  };

  // segment walk: [k0, k1) K steps of tile (tm, tn); plain persistent: whole tiles v, v + G, ...;
  // stream-K: this workgroup's contiguous range [u, ue) of its column group's tiles_m x nsteps steps
  const int tiles_m = ntiles / tiles_n;
  int tm = 0, tn = 0, k0 = 0, k1 = nsteps, v = blockIdx.x;
  int ue = 0;    // stream-K: end of this workgroup's step range (host: tiles_m * nsteps < 2^31)
  int slot = 0;  // stream-K: this workgroup's partial slot (its XCD-remapped index)
  if constexpr (SK) {
    slot = xcd_remap(blockIdx.x, gridDim.x);
    tn = slot % tiles_n;
    const long long gq = gridDim.x / tiles_n, qi = slot / tiles_n, U = (long long)tiles_m * nsteps;
    const int u = (int)(qi * U / gq);
    ue = (int)((qi + 1) * U / gq);
    tm = u / nsteps;
    k0 = u - tm * nsteps;
    k1 = min(nsteps, ue - tm * nsteps);
  } else {
    if (v >= ntiles) return;
    const int wgid = xcd_remap(v, ntiles);
    tn = wgid % tiles_n;
    tm = wgid / tiles_n;
  }
  setup(tm, tn);
  issue(k0, 0);
  wait_vm<0>();
  __builtin_amdgcn_s_barrier();
  int g = 0;  // global K step counter: LDS stage parity
  // PRE (plain epilogue): the previous tile's epilogue issued this segment's step-1 DMA BEFORE its C-tile
  // stores, so this segment's first K step issues nothing and waits with vmcnt(kPreStores) (the stores
  // are the youngest vector-memory ops: in-order counting lets them stay in flight). The stores then
  // have two K steps, not one, to be acknowledged before a wait covers them (tools/kw3_ab.py: KW3P
  // without stores ran 5-9 % faster; stream-K spreading of the bursts did not recover it)
  constexpr int kPreStores = FM * FN;  // buffer stores per wave of the plain epilogue (rows past M: kOOB)
  static_assert(kPreStores <= 63, "vmcnt immediate");
  bool pre = false;
  for (;;) {
    const int cm0 = m0, cn0 = n0;
    // per-lane A fragment addresses of this tile (stage 0; opaque: one VGPR each, as in KW3)
    int aaddr[FM][3];
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int s1 = padded(cm0 + arow0 + i * 16) - P0;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int sl = s1 + kw - 1;
        aaddr[i][kw] = 2 * B_BYTES + sl * 64 + ((q ^ kw3_swz(sl)) << 4);
        asm volatile("" : "+v"(aaddr[i][kw]));
      }
    }
    auto aad = [&](int i, int kw) { return aaddr[i][kw]; };
    // the next segment (its first step is issued by this segment's last K step)
    int ntm = tm, ntn = tn, nk1 = nsteps, vnext = v;
    bool more;
    if constexpr (SK) {
      const int un = (tm + 1) * nsteps;  // next segment starts at its tile's step 0
      more = un < ue;
      ntm = tm + 1;
      nk1 = min(nsteps, ue - un);
    } else {
      vnext = v + (int)gridDim.x;
      more = vnext < ntiles;
      if (more) {
        const int wgid = xcd_remap(vnext, ntiles);
        ntn = wgid % tiles_n;
        ntm = wgid / tiles_n;
      }
    }
    const int ck0 = k0, ck1 = k1;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // one K step on stage `cur` (its DMAs landed and every wave passed the barrier); `nxt` issues
    // the following step's DMAs behind the first fragment reads; ends with the wait + barrier that
    // make the next step's stage readable
    auto kstep = [&](int cur, auto nxt, bool counted) {
      const int aoff = cur * A_BYTES;
      const uint8_t* Bs = smem + baddr0 + cur * B_BYTES;
      v8 bA[FN], bB[FN], af[FM];
#pragma unroll
      for (int j = 0; j < FN; ++j) bA[j] = *reinterpret_cast<const v8*>(Bs + j * 1024);
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = *reinterpret_cast<const v8*>(smem + aoff + aad(i, 0));
      nxt();
#pragma unroll
      for (int j = 0; j < FN; ++j) bB[j] = *reinterpret_cast<const v8*>(Bs + BN * 64 + j * 1024);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af[i], bA[j], acc[i][j]);
        af[i] = *reinterpret_cast<const v8*>(smem + aoff + aad(i, 1));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) bA[j] = *reinterpret_cast<const v8*>(Bs + 2 * BN * 64 + j * 1024);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af[i], bB[j], acc[i][j]);
        af[i] = *reinterpret_cast<const v8*>(smem + aoff + aad(i, 2));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma16x16x32<DT>(af[i], bA[j], acc[i][j]);
      __builtin_amdgcn_sched_group_barrier(0x100, FN, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, FN, 0);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, FN, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, FM * FN, 0);
      // my next-stage DMAs landed AND every fragment read of this stage returned (the barrier may
      // be scheduled among the last MFMAs: with reads still in flight, another wave's next DMA
      // into this stage could overwrite what they have not fetched yet)
      if (counted)
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" ::"n"(kPreStores) : "memory");
      else
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    };
#pragma unroll 1
    for (int k = ck0; k + 1 < ck1; ++k, ++g) {
      const bool first_pre = pre && k == ck0;
      kstep(
          g & 1,
          [&] {
            if (!first_pre) issue(k + 1, (g & 1) ^ 1);
          },
          first_pre);
    }
    // the last step issues the next tile's first step (gather state computed before its fragments
    // are live): those operands land behind this step's MFMAs, its trailing wait covers them, and
    // the epilogue's stores below are younger than them
    if (more) setup(ntm, ntn);
    // this tile's bias, loaded before the last K step (whose vmcnt(0) covers it): a load issued after
    // the PRE DMA below would make the epilogue wait for that DMA
    const int cl = lane & 15;
    float bias[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) bias[j] = a.bias ? a.bias[cn0 + wn * FN * 16 + j * 16 + cl] : 0.f;
    kstep(
        g & 1,
        [&] {
          if (more) issue(0, (g & 1) ^ 1);
        },
        false);
    ++g;
    // advance the walk (the epilogue below uses cm0 / cn0 / ck0 / ck1 only)
    tm = ntm;
    tn = ntn;
    v = vnext;
    k0 = 0;
    k1 = nk1;
    // step 1 of the next segment into the stage the last K step just released (every wave passed its
    // barrier), ahead of the epilogue's stores (see PRE above); the UNP epilogue stages through that stage
    pre = !LDSEPI && SV != 1 && use_pre && more && nk1 > 1;
    if (pre) issue(1, (g & 1) ^ 1);
    if constexpr (SK) {
      typedef __attribute__((ext_vector_type(4))) float f32x4v;
      const __amdgpu_buffer_rsrc_t skr = make_rsrc(a.skw, (uint64_t)gridDim.x * kSkSlotFloats * 4);
      // this wave's slice of a slot: [wave][i][j][lane] f32x4 (1 KiB per (i, j): coalesced)
      auto sk_off = [&](int s_, int i, int j) {
        return (uint32_t)(((((long long)s_ * NW + wave) * FM + i) * FN + j) * 64 + lane) * 16u;
      };
      if (ck0 > 0) {  // tail piece (this range's first segment): publish the partial accumulators
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4v, acc[i][j]), skr, (int)sk_off(slot, i, j), 0,
                                                   16 /* sc1: write-through */);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its partial stores
        __syncthreads();
        if (tid == 0)
          __hip_atomic_store(a.skflag + slot, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!more) break;
        continue;
      }
      if (ck1 < nsteps) {  // head piece (this range's last segment): add the tail's partial, then the epilogue
        const int src = (slot + tiles_n) % (int)gridDim.x;  // the next workgroup of this column group
        if (tid == 0) {
          // bounded poll (~1 s): a lost hand-off must not hang the GPU. A timeout (the producer never
          // became resident, e.g. every other CU held by kernels of other streams that spin on peers)
          // leaves this tile wrong, so it is COUNTED in host-coherent memory and the host raises
          // (bindings.cpp sk_errors(), checked after each serving batch / bench / test)
          bool ok = false;
          for (int it = 0; it < (1 << 22); ++it) {
            if (__hip_atomic_load(a.skflag + src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 1u) {
              ok = true;
              break;
            }
            __builtin_amdgcn_s_sleep(8);
          }
          if (!ok && a.skerr != nullptr) __hip_atomic_fetch_add(a.skerr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // no load moves above the poll
        __syncthreads();
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          f32x4v pv[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j)
            pv[j] = __builtin_bit_cast(f32x4v, __builtin_amdgcn_raw_buffer_load_b128(skr, (int)sk_off(src, i, j), 0,
                                                                                  16 /* sc1 */));
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            acc[i][j][0] += pv[j][0];
            acc[i][j][1] += pv[j][1];
            acc[i][j][2] += pv[j][2];
            acc[i][j][3] += pv[j][3];
          }
        }
      }
    }
    // ---- epilogue: register transpose -> 8-B stores (no LDS, no barrier) ----
    // lane roles (see the header; derived here, not kept live across the K loop): this lane stores
    // row rsub of each 16-row block, 4 columns from csub
    const int ce = cl & 1, cu = (cl >> 1) & 1;
    const int rsub = (lane >> 4) * 4 + ce * 2 + cu, csub = cl & ~3;
    const bool pre_relu = a.relu != 0;
    if constexpr (LDSEPI) {
      static_assert(FN == 4 && FM % 2 == 0 && A_BYTES >= NW * 4096, "KW3P LDS epilogue: 128 x 64 wave tiles, 4 KiB slices");
      uint8_t* wreg = smem + 2 * B_BYTES + ((g & 1) ^ 1) * A_BYTES + wave * 4096;
      const int rl = lane >> 3, pc = lane & 7, lch = pc ^ ((rl & 3) << 1);
      const int gcol = cn0 + wn * FN * 16 + lch * 8;
      const int mb = cm0 + wm * FM * 16 + rl;  // this lane's rows: mb + 8 k, k = 0 .. 2 FM - 1
      const int nb = UNP ? mb / HW : 0, remb = mb - nb * HW, ohb = UNP ? remb / W : 0, owb = remb - ohb * W;
      const int ndb = UNP ? nb / a.ucode_div : 0, nrb = nb - ndb * (UNP ? a.ucode_div : 1);
      // step (n, oh, ow) and (n / ucode_div, n % ucode_div) by 8 rows (host: W >= 8)
      auto step8 = [&](int& n, int& nd, int& nr, int& oh, int& ow) {
        ow += 8;
        if (ow >= W) {
          ow -= W;
          if (++oh == H) {
            oh = 0;
            ++n;
            if (++nr == a.ucode_div) {
              nr = 0;
              ++nd;
            }
          }
        }
      };
      uint2 cd[2 * FM];
      if constexpr (UNP) {
        int n = nb, nd = ndb, nr = nrb, oh = ohb, ow = owb;
#pragma unroll
        for (int k = 0; k < 2 * FM; ++k) {
          cd[k] = make_uint2(0u, 0u);
          if (mb + 8 * k < a.M)
            cd[k] = *reinterpret_cast<const uint2*>(a.ucode + ((long long)nd * HW + oh * W + ow) * a.OC + gcol);
          step8(n, nd, nr, oh, ow);
        }
      }
      uint16_t* out = reinterpret_cast<uint16_t*>(a.out);
      int n = nb, nd = ndb, nr = nrb, oh = ohb, ow = owb;
#pragma unroll
      for (int p = 0; p < FM / 2; ++p) {
        asm volatile("" ::: "memory");
#pragma unroll
        for (int ii = 0; ii < 2; ++ii) {
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int i = 2 * p + ii;
            const bool rl_ = pre_relu && relu_at(a, cn0 + wn * FN * 16 + j * 16 + cl);
            float f0 = acc[i][j][0] + bias[j], f1 = acc[i][j][1] + bias[j], f2 = acc[i][j][2] + bias[j],
                  f3 = acc[i][j][3] + bias[j];
            if (rl_) {
              f0 = fmaxf(f0, 0.f);
              f1 = fmaxf(f1, 0.f);
              f2 = fmaxf(f2, 0.f);
              f3 = fmaxf(f3, 0.f);
            }
            const uint32_t p0 = pack2<DT>(f0, f1), p1 = pack2<DT>(f2, f3);
            const uint32_t keep = ce ? p1 : p0;
            const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(ce ? p0 : p1), 0xB1, 0xF, 0xF, false);
            const uint32_t lo = ce ? recv : keep, hi = ce ? keep : recv;
            const uint32_t d0 = (lo & 0xFFFFu) | (hi << 16), d1 = (lo >> 16) | (hi & 0xFFFF0000u);
            const uint32_t recv2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(cu ? d0 : d1), 0x4E, 0xF, 0xF, false);
            const int lr = ii * 16 + rsub, lc = j * 16 + csub;
            *reinterpret_cast<uint2*>(wreg + lr * 128 + (((lc >> 3) ^ ((lr & 3) << 1)) << 4) + (lc & 4) * 2) =
                make_uint2(cu ? recv2 : d0, cu ? d1 : recv2);
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // wave-local: this wave's writes before its reads
        uint4 cv[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) cv[t] = *reinterpret_cast<const uint4*>(wreg + (t * 8 + rl) * 128 + pc * 16);
        if (p == FM / 2 - 1) {  // every wave's reads of the stage done before the next tile's DMA into it
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        if constexpr (!UNP) {  // plain: one 16-B store per chunk (rows past M: out-of-range offset, dropped)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            const int m = mb + 8 * (4 * p + t);
            const uint32_t off = m < a.M ? ((uint32_t)m * (uint32_t)a.out_ld + (uint32_t)gcol) * 2u : kOOB;
            typedef __attribute__((ext_vector_type(4))) unsigned int u32x4e;
            __builtin_amdgcn_raw_buffer_store_b128(u32x4e{cv[t].x, cv[t].y, cv[t].z, cv[t].w}, orr, (int)off, 0, 0);
          }
          continue;
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int k = 4 * p + t;
          if (mb + 8 * k < a.M) {
            const uint4 sp = unpool_spread(cd[k]);
            const long long ob = (((long long)n * 2 * H + 2 * oh) * 2 * W + 2 * ow) * a.out_ld + gcol;
#pragma unroll
            for (int pos = 0; pos < 4; ++pos) {
              const long long po = ob + (long long)((pos >> 1) * 2 * W + (pos & 1)) * a.out_ld;
              if constexpr (SV == 1) {
                const uint4 pv = unpool_pick_s(cv[t], sp, (uint32_t)pos);
                asm volatile("" ::"v"(pv.x), "v"(pv.y), "v"(pv.z), "v"(pv.w), "v"((uint32_t)po));
              } else if constexpr (SV == 2) {
                typedef __attribute__((ext_vector_type(4))) unsigned int u32x4_nt;
                const uint4 pv = unpool_pick_s(cv[t], sp, (uint32_t)pos);
                __builtin_nontemporal_store(u32x4_nt{pv.x, pv.y, pv.z, pv.w}, reinterpret_cast<u32x4_nt*>(out + po));
              } else if (DV_BOUNDS(po, 8, a.out_elems, "kw3p unpool-out store")) {
                *reinterpret_cast<uint4*>(out + po) = unpool_pick_s(cv[t], sp, (uint32_t)pos);
              }
            }
          }
          step8(n, nd, nr, oh, ow);
        }
      }
      if (!more) break;
      continue;
    }
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int gcol = cn0 + wn * FN * 16 + j * 16 + cl;
      const bool rl = pre_relu && relu_at(a, gcol);
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        float f0 = acc[i][j][0] + bias[j], f1 = acc[i][j][1] + bias[j], f2 = acc[i][j][2] + bias[j],
              f3 = acc[i][j][3] + bias[j];
        if (rl) {
          f0 = fmaxf(f0, 0.f);
          f1 = fmaxf(f1, 0.f);
          f2 = fmaxf(f2, 0.f);
          f3 = fmaxf(f3, 0.f);
        }
        const uint32_t p0 = pack2<DT>(f0, f1), p1 = pack2<DT>(f2, f3);  // rows (r0, r1) / (r2, r3)
        // swap with lane ^ 1: even lanes end with rows r0, r1 of columns (c, c + 1), odd lanes with r2, r3
        const uint32_t keep = ce ? p1 : p0;
        const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)(ce ? p0 : p1), 0xB1, 0xF, 0xF, false);
        const uint32_t lo = ce ? recv : keep, hi = ce ? keep : recv;
        const uint32_t d0 = (lo & 0xFFFFu) | (hi << 16), d1 = (lo >> 16) | (hi & 0xFFFF0000u);
        // swap with lane ^ 2: one row x 4 consecutive columns per lane
        const uint32_t recv2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)(cu ? d0 : d1), 0x4E, 0xF, 0xF, false);
        const uint32_t w0 = cu ? recv2 : d0, w1 = cu ? d1 : recv2;
        const int row = cm0 + wm * FM * 16 + i * 16 + rsub;
        const int col = cn0 + wn * FN * 16 + j * 16 + csub;
        const uint32_t off = row < a.M ? ((uint32_t)row * (uint32_t)a.out_ld + (uint32_t)col) * 2u : kOOB;
        typedef __attribute__((ext_vector_type(2))) unsigned int u32x2;
        if constexpr (SV == 1)
          asm volatile("" ::"v"(w0), "v"(w1), "v"(off));
        else
          __builtin_amdgcn_raw_buffer_store_b64(u32x2{w0, w1}, orr, (int)off, 0, SV == 2 ? 2 : 0);
      }
    }
    if (!more) break;
  }
}

static int num_cus() {
  static int n = [] {
    int dev = 0, cu = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cu = 256;
    return cu > 0 ? cu : 256;
  }();
  return n;
}

// DV_KW3: 0 disables the shared-kw-tap kernel (A/B), 2 forces it for every eligible launch regardless
// of the grid size (tests: small shapes with many image borders per tile). Read per launch.
static int kw3_mode() {
  const char* e = dv_ab_env("DV_KW3");
  return e ? std::atoi(e) : 1;
}
// DV_KW3_VAR: the KW3 main-loop variant (conv_dma_kw3_kernel VAR; 8 / 9 and 10 (KW3P without stores) are
// timing ablations that produce wrong outputs; 11 = KW3P with nt stores, tools/kw3_ab.py only: they also need DV_ALLOW_WRONG_ABLATION=1, so a stray
// DV_KW3_VAR in a serving process cannot corrupt convs; without it they fall back to the default).
// Read per launch.
static int kw3_var() {
  const char* e = dv_ab_env("DV_KW3_VAR");
  const int v = e ? std::atoi(e) : kKw3DefaultVar;
  if (v == 8 || v == 9 || v == 10 || v == 20 || v == 21) {
    static bool warned = false;
    if (dv_ab_env("DV_ALLOW_WRONG_ABLATION") == nullptr) {
      if (!warned) fprintf(stderr, "deconv_api_amd: DV_KW3_VAR=%d ignored (needs DV_ALLOW_WRONG_ABLATION=1)\n", v);
      warned = true;
      return kKw3DefaultVar;
    }
    if (!warned) fprintf(stderr, "deconv_api_amd: DV_KW3_VAR=%d: timing ablation, outputs are WRONG\n", v);
    warned = true;
  }
  return v;
}

// DV_KW3P_NO_PRE=1: KW3P without the step-1 DMA issued ahead of the epilogue stores (A/B; read per launch)
static int kw3p_pre() { return dv_ab_env("DV_KW3P_NO_PRE") == nullptr ? 1 : 0; }

// KW3P stream-K applies (conv_dma_kw3p_kernel SK): a workspace was passed (bindings.cpp), not switched off
// (DV_NO_KW3_SK=1, read per launch), one workgroup per CU with the column groups dividing the grid, more
// tiles than workgroups, and every workgroup's range at least one tile long (at most one split tile at
// each end of a range). The caller checked the KW3P epilogue conditions.
static bool kw3_sk_ok(const ConvArgs& a, int BM, int BN) {
  if (a.skw == nullptr || a.skflag == nullptr || a.m_base != 0 || std::getenv("DV_NO_KW3_SK") != nullptr) return false;
  if (a.res != nullptr || a.emask != nullptr || a.accumulate || a.out2 != nullptr || a.OC != a.OCpad || a.OC % 8 ||
      a.out_ld % 8 || a.H >= 4096 || 2LL * a.H * a.W + BM >= (1LL << 19) || a.dtype != DT_BF16 && a.dtype != DT_F16)
    return false;  // (the KW3P epilogue conditions of kw3_try)
  if (a.ucode != nullptr ? (a.W < 8 || a.ucode_div < 1) : a.out_elems * 2 >= 0x7FFFFFF0LL) return false;
  const int G = num_cus(), tiles_n = a.OCpad / BN;
  const long long tiles_m = (a.M + BM - 1) / BM;
  // (only short grids: stream-K removes a partial last round, 1.53 rounds on the block5 forward convs,
  // 0.26 -> 0.22 ms; on many-round grids its split-tile traffic and lost A sharing cost 1-3 %,
  // profiles/kw3_sk_ab_r5.txt)
  // (DV_KW3_SK=all: every eligible grid, A/B; read per launch)
  const char* ska = dv_ab_env("DV_KW3_SK");
  const long long max_tiles = ska && std::strcmp(ska, "all") == 0 ? (1LL << 40) : 4LL * G;
  return G <= kSkMaxWg && G <= a.skslots && (long long)BM * BN <= kSkSlotFloats && tiles_n >= 1 && G % tiles_n == 0 &&
         tiles_m * tiles_n > G && tiles_m * tiles_n < max_tiles && tiles_m >= G / tiles_n &&
         tiles_m * (3LL * a.C / 32) < (1LL << 31);
}

// tiles_m_limit > 0: launch only the first tiles_m_limit row tiles (kw3_split's full rounds)
template <int DT, int AMODE, int EPI, int BN = 256, int BM = 256>
static int kw3_try(const ConvArgs& a, hipStream_t s, int tiles_m_limit = 0) {
  if constexpr (AMODE != CONV_A_FWD || EPI == CONV_E_POOL) {
    return -4;
  } else {
    if (kw3_mode() == 0 || a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.H != a.OH ||
        a.W != a.OW || a.W < 1 || a.C % 32 || a.mask || a.ws || a.OCpad % BN || (long long)a.Kpad < 9LL * a.C)
      return -4;
    // zero-padded slots of a BM-row tile: BM + 2 + 8 x (image-row boundaries, <= (BM - 1) / W + 1)
    if (BM + 2 + kKw3Pad * ((BM - 1) / a.W + 1) > kw3_a_i(BM) * 8 * 16) return -4;  // W >= 9 (256), >= 35 (512)
    if (a.m_base != 0) return -4;
    int tiles_m = (a.M + BM - 1) / BM;
    if (tiles_m_limit > 0 && tiles_m_limit < tiles_m) tiles_m = tiles_m_limit;
    const int tiles_n = a.OCpad / BN;
    const long long nwg = (long long)tiles_m * tiles_n;
    if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
    // (a B-fragment double buffer across the kw sub-steps measured equal and was removed,
    // profiles/layers_r1_kw3_{nofp,on}.txt)
    const int var = kw3_var();
    const dim3 grid((unsigned)nwg);
    if constexpr (EPI == CONV_E_BF16) {
      // VAR 10 / 11 (bf16 only): KW3P without epilogue stores (timing ablation) / with nt stores
      const bool pvar = var == 2 || (DT == DT_BF16 && (var == 10 || var == 11 || var == 20 || var == 21));
      auto launch_p = [&](auto em) -> int {
        constexpr int U = decltype(em)::value;
        const unsigned g = (unsigned)(nwg < (long long)num_cus() ? nwg : (long long)num_cus());
        if constexpr (DT == DT_BF16) {
          if (var == 10) {
            hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 1>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg, kw3p_pre());
            return (int)hipGetLastError();
          }
          if (var == 11) {
            hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 2>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg, kw3p_pre());
            return (int)hipGetLastError();
          }
          if (var == 20 || var == 21) {
            if (var == 20)
              hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 3>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg, 0);
            else
              hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 4>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg, 0);
            return (int)hipGetLastError();
          }
        }
        // the unpool-out epilogue's stores are non-temporal (the 4x-upsampled map, 3/4 zeros, streams past the
        // caches): config 2 +0.3 % (3 / 3 pairs, profiles/bench_c2_r5_unp_nt_ab.txt). DV_KW3P_UNP_NT=0: plain
        // stores (A/B; read per launch)
        if constexpr (U == 1) {
          const char* unt = dv_ab_env("DV_KW3P_UNP_NT");
          if (!(unt && std::strcmp(unt, "0") == 0) && !(tiles_m_limit == 0 && kw3_sk_ok(a, BM, BN))) {
            hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 2>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg,
                               kw3p_pre());
            return (int)hipGetLastError();
          }
        }
        if (tiles_m_limit == 0 && kw3_sk_ok(a, BM, BN)) {  // stream-K over the whole grid (no tail launch)
          const int G = num_cus();
          if (hipMemsetAsync(a.skflag, 0, (size_t)G * sizeof(unsigned), s) != hipSuccess) return (int)hipGetLastError();
          hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U, 0, true>), dim3(G), dim3(512), 0, s, a, tiles_n,
                             (int)nwg, kw3p_pre());
          return (int)hipGetLastError();
        }
        hipLaunchKernelGGL((conv_dma_kw3p_kernel<DT, BN, BM, U>), dim3(g), dim3(512), 0, s, a, tiles_n, (int)nwg, kw3p_pre());
        return (int)hipGetLastError();
      };
      // persistent KW3P: plain 16-bit epilogue only (its register-transpose stores write exactly
      // the C tile), output addressable by a 31-bit buffer offset, one workgroup per CU
      if (pvar && a.res == nullptr && a.emask == nullptr && !a.accumulate && a.ucode == nullptr &&
          a.out2 == nullptr && a.OC == a.OCpad && a.OC % 4 == 0 && a.out_ld % 4 == 0 &&
          a.out_elems * 2 < 0x7FFFFFF0LL && a.H < 4096 && 2LL * a.H * a.W + BM < (1LL << 19))
        // the LDS-sliced 16-B store epilogue unless DV_KW3P_EPI=reg (A/B) or the rows are not 16-B aligned:
        // config-2 KW3P launches 9-13 % faster than with the register-transposed 8-B stores
        // (profiles/kw3_epi_ab_r5.txt), config 2 +6.6 % (7418 / 7457 vs 6966 / 6985 img/s, same box)
        return (dv_ab_env("DV_KW3P_EPI") == nullptr || std::strcmp(dv_ab_env("DV_KW3P_EPI"), "reg") != 0) &&
                       a.OC % 8 == 0 && a.out_ld % 8 == 0
                   ? launch_p(std::integral_constant<int, 2>{})
                   : launch_p(std::integral_constant<int, 0>{});
      // persistent KW3P with the LDS-sliced max-unpool-out epilogue (DV_NO_KW3P_UNPOOL=1: the
      // non-persistent KW3 kernel's workgroup-staged one, A/B; read per launch)
      if (pvar && a.ucode != nullptr && a.res == nullptr && a.emask == nullptr && !a.accumulate &&
          a.out2 == nullptr && a.OC == a.OCpad && a.OC % 8 == 0 && a.out_ld % 8 == 0 && a.W >= 8 && a.ucode_div >= 1 &&
          a.H < 4096 && 2LL * a.H * a.W + BM < (1LL << 19) && dv_ab_env("DV_NO_KW3P_UNPOOL") == nullptr)
        return launch_p(std::integral_constant<int, 1>{});
    }
    if constexpr (DT == DT_BF16 && EPI == CONV_E_BF16) {
      if (var == 8 || var == 9) {
        if (var == 8)
          hipLaunchKernelGGL((conv_dma_kw3_kernel<DT, EPI, BN, BM, 8>), grid, dim3(512), 0, s, a, tiles_n);
        else
          hipLaunchKernelGGL((conv_dma_kw3_kernel<DT, EPI, BN, BM, 9>), grid, dim3(512), 0, s, a, tiles_n);
        return (int)hipGetLastError();
      }
    }
    hipLaunchKernelGGL((conv_dma_kw3_kernel<DT, EPI, BN, BM, 0>), grid, dim3(512), 0, s, a, tiles_n);
    return (int)hipGetLastError();
  }
}

template <int DT, int WM, int WN, int FM, int FN, int BK, int ST, int AMODE, int EPI, bool MASK = false,
          bool FP = false>
static int dma_cfg(const ConvArgs& a, hipStream_t s) {
  constexpr int BM = WM * FM * 16, BN = WN * FN * 16;
  constexpr int NT = WM * WN * 64;
  const int tiles_m = (a.M - a.m_base + BM - 1) / BM;
  const int tiles_n = a.OCpad / BN;
  const long long nwg = (long long)tiles_m * tiles_n;
  if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
  const bool aligned = (a.C % BK) == 0;
  const dim3 grid((unsigned)nwg, (unsigned)(a.ws ? a.ksplit : 1));
  if (aligned)
    hipLaunchKernelGGL((conv_dma_kernel<DT, WM, WN, FM, FN, BK, ST, AMODE, EPI, true, MASK, FP>), grid,
                       dim3(NT), 0, s, a, tiles_n);
  else
    hipLaunchKernelGGL((conv_dma_kernel<DT, WM, WN, FM, FN, BK, ST, AMODE, EPI, false, MASK, FP>), grid,
                       dim3(NT), 0, s, a, tiles_n);
  return (int)hipGetLastError();
}

// KW3 256 x 256 runs one workgroup per CU (144 KiB of LDS), so a grid of R.f rounds pays a whole
// round for its fraction f (block5 at B*K = 1024: 1568 tiles = 6.125 rounds; at B = 256: 392 =
// 1.53). Split: the full rounds as KW3, the last partial round's rows as a tail launch of 128 x 128
// DMA tiles (4x the workgroups, 2 per CU) starting at row m_base. Same stream, in order.
template <int DT, int AMODE, int EPI>
static int kw3_split(const ConvArgs& a, hipStream_t s, long long cus) {
  if (kw3_sk_ok(a, 256, 256) && kw3_var() == 2) {  // stream-K: no partial round, no tail launch
    const int rc = kw3_try<DT, AMODE, EPI>(a, s);
    if (rc != -4) return rc;
  }
  const int tiles_m = (a.M + 255) / 256, tiles_n = a.OCpad / 256;
  const long long nwg = (long long)tiles_m * tiles_n;
  const long long full = nwg / cus, rem = nwg % cus;
  const long long main_m = full * cus / tiles_n;  // row tiles of the full rounds
  if (full < 1 || rem == 0 || (full * cus) % tiles_n != 0 || main_m >= tiles_m)
    return kw3_try<DT, AMODE, EPI>(a, s);
  const int rc = kw3_try<DT, AMODE, EPI>(a, s, (int)main_m);
  if (rc != 0) return rc;  // -4 (unsupported) before anything launched, or a launch error
  ConvArgs t = a;
  t.m_base = (int)(main_m * 256);
  return dma_cfg<DT, 4, 2, 2, 4, 64, 2, AMODE, EPI>(t, s);  // 128 x 128 tail
}

// Measured and removed (rounds 1-3, profiles/layers_r1_dmav{0,5,6}.txt, layers_r1_ks2_{off,on}.txt,
// layers_r1_pipeline.txt): BK32 x 4-stage rings on 256x256 / 512x64, all-2-stage rings, 4-wave
// 256x128 / 128x256 workgroups (0.53-0.72 vs 0.99-1.28 PF/s: 1.5x the staged bytes per FLOP), and
// the in-workgroup K split (two wave groups per C tile, partial sums through LDS: the 256x128 /
// 512x64 tiles are bound by the A-operand DMA stream, not by LDS fragment reads).

// Tuning override (tools/tune_dma.py): force tile config `g_cfg` (> 0) and split-K factor
// `g_ks` (> 0) for every DMA conv launch until reset to 0. Host-side globals, set between launches.
extern int g_cfg, g_ks;  // tuning override, defined in conv_dma.hip

// every tile config the DMA kernel is instantiated with; -5 = config does not fit this problem
template <int DT, int AMODE, int EPI>
static int dma_forced(const ConvArgs& a, hipStream_t s, int cfg) {
  auto okn = [&](int bn) { return a.OCpad % bn == 0; };
  switch (cfg) {
    case 1: return okn(256) ? dma_cfg<DT, 2, 4, 8, 4, 64, 2, AMODE, EPI, false, true>(a, s) : -5;  // 256x256
    case 2: return okn(256) ? dma_cfg<DT, 2, 4, 4, 4, 64, 3, AMODE, EPI>(a, s) : -5;               // 128x256
    case 3: return okn(128) ? dma_cfg<DT, 4, 2, 2, 4, 64, 2, AMODE, EPI>(a, s) : -5;               // 128x128
    case 4: return okn(128) ? dma_cfg<DT, 4, 2, 4, 4, 64, 3, AMODE, EPI>(a, s) : -5;               // 256x128
    case 5: return okn(64) ? dma_cfg<DT, 8, 1, 2, 4, 64, 2, AMODE, EPI>(a, s) : -5;                // 256x64
    case 6: return okn(64) ? dma_cfg<DT, 8, 1, 4, 4, 64, 2, AMODE, EPI>(a, s) : -5;                // 512x64
    case 7: return okn(64) ? dma_cfg<DT, 4, 1, 2, 4, 64, 3, AMODE, EPI>(a, s) : -5;                // 128x64, 4 waves
    case 8: return okn(64) ? dma_cfg<DT, 2, 2, 2, 2, 64, 3, AMODE, EPI>(a, s) : -5;                // 64x64, 4 waves
    case 9: return okn(128) ? dma_cfg<DT, 2, 2, 4, 4, 64, 2, AMODE, EPI>(a, s) : -5;               // 128x128, 4 waves
    case 10: return okn(128) ? dma_cfg<DT, 2, 2, 2, 4, 64, 3, AMODE, EPI>(a, s) : -5;              // 64x128, 4 waves
    case 11: return okn(64) ? dma_cfg<DT, 4, 1, 4, 4, 64, 2, AMODE, EPI>(a, s) : -5;               // 256x64, 4 waves
    // deep rings for latency-bound small GEMMs (more K tiles in flight per workgroup)
    case 12: return okn(64) ? dma_cfg<DT, 2, 2, 2, 2, 64, 6, AMODE, EPI>(a, s) : -5;               // 64x64 w4 ST6
    case 13: return okn(64) ? dma_cfg<DT, 2, 2, 2, 2, 64, 8, AMODE, EPI>(a, s) : -5;               // 64x64 w4 ST8
    case 14: return okn(64) ? dma_cfg<DT, 4, 1, 2, 4, 64, 6, AMODE, EPI>(a, s) : -5;               // 128x64 w4 ST6
    case 15: return okn(128) ? dma_cfg<DT, 2, 2, 2, 4, 64, 6, AMODE, EPI>(a, s) : -5;              // 64x128 w4 ST6
    // 8 waves on a 64x64 tile: half the LDS-DMA issues per wave and K tile (the small tiles' K loop
    // is DMA-issue bound: 4 x ~100 cycles per wave per K tile at 4 waves)
    case 16: return okn(64) ? dma_cfg<DT, 4, 2, 1, 2, 64, 3, AMODE, EPI>(a, s) : -5;               // 64x64 w8
    case 17: return okn(64) ? dma_cfg<DT, 4, 2, 1, 2, 64, 4, AMODE, EPI>(a, s) : -5;               // 64x64 w8 ST4
    default: return -5;
  }
}

// Measured override of the size-based choice below for small and narrow-K problems (the DeepDream
// nets' 1x1 / 1x7 / 5x5 convs and dgrads; tools/tune_dma.py sweep of every launch of configs 3 and 5,
// profiles/tune_dma_c{3,5}.txt): conv time 9.80 -> 8.52 ms (InceptionV3, 4 octaves) and 6.45 -> 6.07
// ms (ResNet-50 512^2 x 32). Small problems are bound by per-K-step latency, not MFMA rate: a 64x64
// 4-wave tile with a 3-stage ring and no split-K; mid-size / short-K ones by the epilogue and DMA
// issue of one big tile per CU: 128x128. The big-K VGG16 layers keep the large tiles.
static int auto_cfg(const ConvArgs& a) {
  static const bool off = dv_ab_env("DV_NO_AUTO_CFG") != nullptr;  // A/B: the size-based choice only
  if (a.mask != nullptr || off) return 0;
  const long long mn = (long long)a.M * a.OCpad;
  // (short K too: M 1600 x N 64 x K 64 4.2 vs 6.0 us for the size-based 256 x 64 tile in a graph,
  // tools/small_conv_latency.py; DV_SMALL_TILE_KMIN=256 restores the round-1 rule)
  static const int kmin = dv_ab_env("DV_SMALL_TILE_KMIN") ? std::atoi(dv_ab_env("DV_SMALL_TILE_KMIN")) : 0;
  // (an 8-wave 64x64 tile with a 4-deep ring, config 17, was -8 % per launch in isolation but
  // neutral end to end, 417 vs 418 img/s: it stays a tuner-only config)
  if (a.OCpad % 64 == 0 && a.OC > 16 && mn <= 3000000LL && a.Kpad >= kmin) return 8;
  if (a.OCpad % 128 == 0 && a.OC > 64 && a.Kpad < 4096 && (a.Kpad < 1024 || mn < 50000000LL)) return 3;
  return 0;
}

// Tile choice: the largest tile (best MFMA:LDS ratio) unless it leaves CUs idle. A problem with
// fewer big tiles than the chip has CUs (deep layers at small batch, strong-scaled tiles) drops to
// the next smaller tile, which doubles the workgroup count and fits 2 workgroups per CU in LDS.
template <int DT, int AMODE, int EPI>
static int dma_bn(const ConvArgs& a, hipStream_t s) {
  if (g_cfg > 0) return dma_forced<DT, AMODE, EPI>(a, s, g_cfg);
  if (const int c = auto_cfg(a)) return dma_forced<DT, AMODE, EPI>(a, s, c);
  // (the 3-stage BK=64 ring wins slightly on 256x128; 2 stages elsewhere)
  const long long cus = num_cus();
  auto nwg = [&](int BM, int BN) { return (long long)((a.M + BM - 1) / BM) * (a.OCpad / BN); };
  if (a.OCpad % 256 == 0 && a.OC > 128) {
    {  // DV_KW3_TILE=512x128 (per launch): the 512 x 128 KW3P tile for these shapes too (A/B)
      const char* kt = dv_ab_env("DV_KW3_TILE");
      if (kt && std::strcmp(kt, "512x128") == 0) {
        const int rc = kw3_try<DT, AMODE, EPI, 128, 512>(a, s);
        if (rc != -4) return rc;
      }
    }
    if (kw3_mode() == 2) {
      const int rc = kw3_try<DT, AMODE, EPI>(a, s);
      if (rc != -4) return rc;
    }
    if (nwg(256, 256) < cus && nwg(128, 256) >= cus)
      return dma_cfg<DT, 2, 4, 4, 4, 64, 3, AMODE, EPI>(a, s);  // 128 x 256, 3-stage
    if (nwg(256, 256) < cus) return dma_cfg<DT, 4, 2, 2, 4, 64, 2, AMODE, EPI>(a, s);  // 128 x 128
    {  // 3x3 s1 p1 forward: the three kw taps share one staged A tile
      const int rc = kw3_split<DT, AMODE, EPI>(a, s, cus);
      if (rc != -4) return rc;
    }
    // 256 x 256 with register double-buffered fragments: +3% on the big VGG layers (profiles/)
    return dma_cfg<DT, 2, 4, 8, 4, 64, 2, AMODE, EPI, false, true>(a, s);
  }
  if (a.OCpad % 128 == 0 && a.OC > 64) {
    if (kw3_mode() == 2 || nwg(512, 128) >= cus) {  // 3x3 s1 p1 forward: shared-kw-tap 512 x 128 tile
      const int rc = kw3_try<DT, AMODE, EPI, 128, 512>(a, s);
      if (rc != -4) return rc;
    }
    if (nwg(256, 128) < cus) return dma_cfg<DT, 4, 2, 2, 4, 64, 2, AMODE, EPI>(a, s);  // 128 x 128
    return dma_cfg<DT, 4, 2, 4, 4, 64, 3, AMODE, EPI>(a, s);  // 256 x 128
  }
  if (a.OCpad % 64 == 0 && a.OC > 16) {
    if (nwg(512, 64) < cus) return dma_cfg<DT, 8, 1, 2, 4, 64, 2, AMODE, EPI>(a, s);  // 256 x 64
    return dma_cfg<DT, 8, 1, 4, 4, 64, 2, AMODE, EPI>(a, s);  // 512 x 64
  }
  if (a.OCpad % 16 == 0) {
    if (nwg(512, 16) < cus) return dma_cfg<DT, 8, 1, 2, 1, 64, 2, AMODE, EPI>(a, s);  // 256 x 16
    return dma_cfg<DT, 8, 1, 4, 1, 64, 2, AMODE, EPI>(a, s);  // 512 x 16
  }
  return -3;
}

// ReLU-masked dgrad: the mask tile doubles A's LDS footprint, so smaller tiles than dma_bn
// (<= 128 KiB of LDS per workgroup at 2 stages)
template <int DT, int AMODE>
static int dma_mask_bn(const ConvArgs& a, hipStream_t s) {
  if (a.OCpad % 256 == 0 && a.OC > 128) return dma_cfg<DT, 2, 4, 4, 4, 64, 2, AMODE, CONV_E_BF16, true>(a, s);  // 128x256
  if (a.OCpad % 128 == 0 && a.OC > 64) return dma_cfg<DT, 4, 2, 2, 4, 64, 2, AMODE, CONV_E_BF16, true>(a, s);   // 128x128
  if (a.OCpad % 64 == 0 && a.OC > 16) return dma_cfg<DT, 8, 1, 2, 4, 64, 2, AMODE, CONV_E_BF16, true>(a, s);    // 256x64
  if (a.OCpad % 16 == 0) return dma_cfg<DT, 8, 1, 2, 1, 64, 2, AMODE, CONV_E_BF16, true>(a, s);                // 256x16
  return -3;
}

// Tile dims the default selection above picks, for split-K planning.
static void dma_tile_dims(const ConvArgs& a, bool mask, int& BM, int& BN) {
  const long long cus = num_cus();
  auto nwg = [&](int bm, int bn) { return (long long)((a.M + bm - 1) / bm) * (a.OCpad / bn); };
  BM = 256;
  BN = 16;
  if (!mask) {
    const int c = auto_cfg(a);
    if (c == 8 || c == 17) { BM = 64; BN = 64; return; }
    if (c == 3) { BM = 128; BN = 128; return; }
  }
  if (mask) {
    if (a.OCpad % 256 == 0 && a.OC > 128) { BM = 128; BN = 256; }
    else if (a.OCpad % 128 == 0 && a.OC > 64) { BM = 128; BN = 128; }
    else if (a.OCpad % 64 == 0 && a.OC > 16) { BM = 256; BN = 64; }
    return;
  }
  if (a.OCpad % 256 == 0 && a.OC > 128) {
    if (nwg(256, 256) >= cus) { BM = 256; BN = 256; }
    else if (nwg(128, 256) >= cus) { BM = 128; BN = 256; }
    else { BM = 128; BN = 128; }
  } else if (a.OCpad % 128 == 0 && a.OC > 64) {
    BM = nwg(256, 128) < cus ? 128 : 256;
    BN = 128;
  } else if (a.OCpad % 64 == 0 && a.OC > 16) {
    BM = nwg(512, 64) < cus ? 256 : 512;
    BN = 64;
  } else {
    BM = nwg(512, 16) < cus ? 256 : 512;
  }
}

// one dma_bn<DT, AMODE, EPI> per instantiation unit (conv_dma_*.hip)
int dma_run_bf16_fwd(const ConvArgs& a, hipStream_t s);
int dma_run_bf16_fwd_pool(const ConvArgs& a, hipStream_t s);
int dma_run_bf16_fwd_f32(const ConvArgs& a, hipStream_t s);
int dma_run_bf16_tr(const ConvArgs& a, hipStream_t s);
int dma_run_f16_fwd(const ConvArgs& a, hipStream_t s);
int dma_run_f16_fwd_pool(const ConvArgs& a, hipStream_t s);
int dma_run_f16_fwd_f32(const ConvArgs& a, hipStream_t s);
int dma_run_f16_tr(const ConvArgs& a, hipStream_t s);

}  // namespace dv
