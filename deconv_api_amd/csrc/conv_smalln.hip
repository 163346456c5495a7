// Persistent halo-tile 3x3 / stride 1 / pad 1 convolution for 64-channel inputs with narrow
// outputs (OC tile 64 or 16): the deconvnet's block1 conv-downs at 224x224 —
// block1_conv2.down (64 -> 64, max-unpool of the 112x112 signal fused into the staging) and the
// final block1_conv1.down (64 -> 3, fp32 reconstruction out).
//
// Why: with a 64-wide (or 16-wide) N tile, the implicit-GEMM kernel fetches every input pixel
// once per tap (9x) and is L2-bandwidth bound (profiles/layers_r1_*.txt: 430 TF/s and 40 TF/s).
// Here one 512-thread workgroup per CU:
//   * loads the layer's packed weights (<= 64 x 576 bf16 = 72 KiB) into LDS ONCE;
//   * walks 8 x 32 output tiles (grid-stride, persistent); per tile the 10 x 34 x 64-channel
//     halo (48 KiB) is staged once and the 9 taps read shifted windows of it as MFMA A
//     fragments (v_mfma_f32_16x16x32_bf16, 18 K-steps of 32 per tile);
//   * the next tile's halo is loaded into VGPRs (16-B loads; unpool switch-select + ReLU on the
//     way in) while the current tile's MFMAs run, then written to LDS between two barriers.
// Halo pixels use a padded 144-B stride (9 bank slots, coprime with 16: 16 consecutive pixels hit
// 16 distinct slots) so every tap shift is a constant ds_read offset; weight rows (1152 B) are
// XOR-swizzled by 16-B chunk with (row & 7). Both fragment reads are bank-conflict free.
#include "common.h"
#include "kernels.h"

#include <cstdlib>

namespace dv {

namespace {
constexpr int TH = 8, TW = 32;             // output tile: 8 waves x (1 row x 32 px)
constexpr int IH = TH + 2, IW = TW + 2;    // halo tile
constexpr int C64 = 64;                    // input channels
// 160 B per halo pixel (10 bank slots): conflict-free ds_read_b128 fragment reads of 16 consecutive
// pixels at any base, chunk q or q + 4 (tools/lds_bank_check.py). The round-1..2 144-B pitch (9
// slots) was 2-way on every lane group: SQ_LDS_BANK_CONFLICT / IDX_ACTIVE 0.40 on the v2 unpool
// kernel (profiles/pmc_c2_r3.txt).
constexpr int PIXB = C64 * 2 + 32;
constexpr int KW9 = 9 * C64;               // K = 576
constexpr int WROWB = KW9 * 2;             // 1152 B per weight row (72 chunks)
constexpr int HALO_CH = IH * IW * 8;       // 16-B chunks per halo (4896)
constexpr int PER_T = (HALO_CH + 511) / 512;  // 6 chunks per thread
constexpr int FM = 2;                      // 16-px fragments per wave (one 32-px row)
}  // namespace

__device__ __forceinline__ int sw_off(int row, int chunk, int rowb) {
  return row * rowb + ((chunk ^ (row & 7)) << 4);
}
__device__ __forceinline__ int p_of(int idx) { return idx >> 3; }

template <int FN, int EPI, bool UNPOOL>
__global__ void __launch_bounds__(512, 1) conv3x3_c64_persist_kernel(const ConvArgs a) {
  constexpr int BN = FN * 16;
  constexpr int A_BYTES = IH * IW * PIXB;
  __shared__ __attribute__((aligned(16))) uint8_t smem[A_BYTES + BN * WROWB];
  uint8_t* As = smem;
  uint8_t* Bs = smem + A_BYTES;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  const int ntiles = a.N * tiles_h * tiles_w;
  const int PH = H >> 1, PW = W >> 1;

  // ---- weights -> LDS once: [BN rows][576] with the row-XOR chunk swizzle ----
  for (int q = tid; q < BN * (KW9 / 8); q += 512) {
    const int row = q / (KW9 / 8), ch = q % (KW9 / 8);
    const uint4 v = *reinterpret_cast<const uint4*>(a.w + (long long)row * a.Kpad + ch * 8);
    *reinterpret_cast<uint4*>(Bs + row * WROWB + (((ch & ~7) | ((ch & 7) ^ (row & 7))) << 4)) = v;
  }

  // Raw loads only (no use of the loaded values) so every load of the next tile stays in flight
  // across the current tile's MFMAs; the switch-select and ReLU happen at LDS-store time.
  uint4 ra[PER_T];
  uint2 rc[PER_T];
  int ld_y0 = 0, ld_x0 = 0;
  uint32_t okmask = 0;
  auto load_tile = [&](int t) {
    int b = t;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    ld_y0 = y0;
    ld_x0 = x0;
    const long long nc = (long long)(n / a.code_div);
    okmask = 0;
#pragma unroll
    for (int q = 0; q < PER_T; ++q) {
      // unconditional loads at clamped (always valid) coordinates; validity kept as a bit
      const int idx = min(tid + q * 512, HALO_CH - 1);
      const int p = idx >> 3, c8 = idx & 7;
      const int iy = y0 + p / IW, ix = x0 + p % IW;
      const bool ok = tid + q * 512 < HALO_CH && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
      okmask |= (uint32_t)ok << q;
      const int cy = min(max(iy, 0), H - 1), cx = min(max(ix, 0), W - 1);
      if constexpr (UNPOOL) {
        const long long pp = ((long long)n * PH + (cy >> 1)) * PW + (cx >> 1);
        ra[q] = *reinterpret_cast<const uint4*>(a.x + pp * a.x_ld + c8 * 8);
        const long long cp = (nc * PH + (cy >> 1)) * PW + (cx >> 1);
        rc[q] = *reinterpret_cast<const uint2*>(a.code + cp * C64 + c8 * 8);
      } else {
        ra[q] = *reinterpret_cast<const uint4*>(a.x + (((long long)n * H + cy) * W + cx) * a.x_ld + c8 * 8);
      }
    }
  };
  auto store_tile = [&]() {
#pragma unroll
    for (int q = 0; q < PER_T; ++q) {
      const int idx = tid + q * 512;
      if (idx < HALO_CH) {
        uint4 v = ((okmask >> q) & 1u) ? ra[q] : make_uint4(0, 0, 0, 0);
        if constexpr (UNPOOL) {
          const int p = idx >> 3;
          const int iy = ld_y0 + p / IW, ix = ld_x0 + p % IW;
          v = unpool_pick(v, rc[q], (uint32_t)(((iy & 1) << 1) | (ix & 1)));
        }
        if (a.relu_in) {
          v.x = relu_bf2(v.x);
          v.y = relu_bf2(v.y);
          v.z = relu_bf2(v.z);
          v.w = relu_bf2(v.w);
        }
        *reinterpret_cast<uint4*>(As + p_of(idx) * PIXB + (idx & 7) * 16) = v;
      }
    }
  };

  const int kq = lane >> 4, col = lane & 15;
  int t = blockIdx.x;
  if (t < ntiles) load_tile(t);
  while (t < ntiles) {
    __syncthreads();  // previous tile's fragment reads done (and, first time, the weights landed)
    store_tile();
    __syncthreads();
    const int tcur = t;
    t += gridDim.x;
    if (t < ntiles) load_tile(t);  // in flight during the MFMAs below

    f32x4 acc[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      const int kh = tap / 3, kw = tap % 3;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int kc = s * 4 + kq;  // 16-B chunk within the 64 input channels
        bf16x8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int row = j * 16 + col;
          const int ch = tap * 8 + kc;
          bfr[j] = *reinterpret_cast<const bf16x8*>(Bs + row * WROWB + (((ch & ~7) | ((ch & 7) ^ (row & 7))) << 4));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int r = wave, xo = i * 16 + col;
          const int p = (r + kh) * IW + xo + kw;
          const bf16x8 af = *reinterpret_cast<const bf16x8*>(As + p * PIXB + kc * 16);
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // ---- epilogue: fragment i = output row `wave`, x = i*16 + kq*4 + r ----
    int b = tcur;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    float biasv[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) biasv[j] = (a.bias && j * 16 + col < a.OC) ? a.bias[j * 16 + col] : 0.f;
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int oc = j * 16 + col;
      if (oc >= a.OC) continue;
      const float bias = biasv[j];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int oy = ty * TH + wave;
        if (oy >= H) continue;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ox = tx * TW + i * 16 + kq * 4 + r;
          if (ox >= W) continue;
          float v = acc[i][j][r] + bias;
          if (a.relu) v = fmaxf(v, 0.f);
          const long long o = (((long long)n * H + oy) * W + ox) * a.out_ld + oc;
          if (!DV_BOUNDS(o, 1, a.out_elems, "halo conv out")) continue;
          if constexpr (EPI == CONV_E_F32)
            reinterpret_cast<float*>(a.out)[o] = v;
          else
            reinterpret_cast<uint16_t*>(a.out)[o] = f2bf(v);
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// v2: unpool + 3x3 conv 64 -> 64 (block1_conv2.down), weights resident in VGPRs.
//
// v1 above keeps the weights in LDS and every wave re-reads all 64 output channels' fragments per
// tile (8x redundant LDS traffic), and stages each halo between two barriers with the MFMA pipes
// idle (PMC: ~19% MFMA-busy, half of all wave cycles parked on s_waitcnt / s_barrier;
// profiles/pmc_flagship_sq_pass1.txt). Here:
//   * wave w owns output rows {2(w/2), 2(w/2)+1} x 32 px x channels [32 (w%2), +32): FM=4 x FN=2
//     fragments; its 32 channels' weights (18 K-steps x 2 fragments = 144 VGPRs) are loaded once;
//   * the halo is double-buffered in LDS (2 x 48 KiB, 144-B padded pixels): tile t+1 is expanded
//     into the other buffer right after tile t's MFMAs, so one barrier separates the tiles;
//   * the halo is fed from POOLED pixels: each 16-B pooled chunk (+ its 8 switch codes) is loaded
//     once and written to the <= 4 unpooled positions it covers (v1 loaded it 4x);
//   * the output tile is staged in LDS (16-B chunks XOR-swizzled by pixel) and written with 16-B
//     stores, 128 contiguous bytes per pixel.
namespace {
constexpr int V2_PH = TH / 2 + 2, V2_PW = TW / 2 + 2;   // pooled halo (6 x 18)
constexpr int V2_TASKS = V2_PH * V2_PW * 8;              // 16-B pooled chunks per tile (864)
constexpr int V2_PER_T = (V2_TASKS + 511) / 512;         // 2
constexpr int V2_A = IH * IW * PIXB;                     // 54400
constexpr int V2_C = TH * TW * 128;                      // 32768: bf16 output tile staging
}  // namespace

//
// ZOUT (block1_conv2.down feeding the final 64 -> 3 block1_conv1.down): instead of the 64-channel map
// (128 B/px written here, read back by the next conv), the epilogue multiplies the ReLU'd bf16 tile
// by that conv's weights arranged as W2 [32][64] (row tap*3 + c; rows 27..31 zero) on MFMA and writes
// Z = D W2^T [N, H, W, 32] bf16 (64 B/px); zsum3x3_kernel finishes the conv as a 9-tap shift-add.
// Wave w owns tile row w for this GEMM (32 px x 32 Z channels, K = 64: 8 MFMAs); the B operand is the
// staged output tile read straight from Cst.
//
// V (bit mask): 1 = transposed MFMA (D^T = W A^T: a lane holds 4 consecutive channels of one pixel), so
// the output tile is staged with one ds_write_b64 per fragment instead of four ds_write_b16; 2 = the
// next tile's halo expansion is issued inside this tile's MFMA loop (the other halo buffer was last
// read by the previous tile's MFMAs, which every wave finished before this tile's first barrier)
// instead of between the two barriers with the MFMA pipes idle.
template <bool ZOUT, int V = 0>
__global__ void __launch_bounds__(512, 1) conv3x3_unpool_c64_v2_kernel(const ConvArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * V2_A + V2_C + (ZOUT ? 32 * 128 : 0)];
  uint8_t* Cst = smem + 2 * V2_A;
  uint8_t* W2s = Cst + V2_C;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int kq = lane >> 4, col = lane & 15;
  const int H = a.H, W = a.W, PH = H >> 1, PW = W >> 1;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  const int ntiles = a.N * tiles_h * tiles_w;

  // ---- this wave's weights -> registers: k-step s = tap*2 + half, fragment j (16 channels) ----
  bf16x8 bw[18][2];
#pragma unroll
  for (int s = 0; s < 18; ++s)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int oc = wc * 32 + j * 16 + col;
      const int k = (s >> 1) * C64 + (s & 1) * 32 + kq * 8;
      bw[s][j] = *reinterpret_cast<const bf16x8*>(a.w + (long long)oc * a.Kpad + k);
    }
  constexpr bool TR = (V & 1) != 0, ILV = (V & 2) != 0;
  // timing ablations (WRONG outputs, DV_TAIL_V with DV_ALLOW_WRONG_ABLATION=1, tools/tail_ab.py): 4 = no Z
  // GEMM / Z stores, 8 = no halo expansion (the MFMAs read a stale halo)
  constexpr bool NO_Z = (V & 4) != 0, NO_EXP = (V & 8) != 0;
  float biasv[2][TR ? 4 : 1];
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < (TR ? 4 : 1); ++r) {
      const int oc = wc * 32 + j * 16 + (TR ? kq * 4 + r : col);
      biasv[j][r] = (a.bias && oc < a.OC) ? a.bias[oc] : 0.f;
    }
  // ZOUT: W2 [32][64] bf16 staged once in LDS (4 KiB, 16-B chunks XOR-swizzled by row; in VGPRs it
  // would spill next to the 144 weight registers); A fragment = row 16 jz + col, K chunk 32 ks + 8 kq
  if constexpr (ZOUT) {
    const int r = tid >> 3, c8 = tid & 7;
    if (tid < 256)
      *reinterpret_cast<uint4*>(W2s + r * 128 + ((c8 ^ (r & 7)) << 4)) = *reinterpret_cast<const uint4*>(a.w2 + r * C64 + c8 * 8);
  }

  uint4 ra[V2_PER_T];
  uint2 rc[V2_PER_T];
  int ld_py0 = 0, ld_px0 = 0;
  // per-tile index math is recomputed from an opaque copy of the thread id: hoisted out of the
  // persistent loop, these loop-invariant values would be held (and spilled) across the MFMAs,
  // whose 144 weight registers leave no room for them
  auto opaque_tid = [tid]() {
    int v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "v"(tid));
    return v;
  };
  auto load_tile = [&](int t) {  // raw pooled chunks + codes of tile t (zeros outside the map)
    const int tid = opaque_tid();
    int b = t;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = b / tiles_h;
    ld_py0 = ((ty * TH - 1) >> 1);  // floor: -1 for ty == 0
    ld_px0 = ((tx * TW - 1) >> 1);
    const long long nc = (long long)(n / a.code_div);
#pragma unroll
    for (int q = 0; q < V2_PER_T; ++q) {
      const int idx = min(tid + q * 512, V2_TASKS - 1);
      const int pp = idx >> 3, c8 = idx & 7;
      const int py = ld_py0 + pp / V2_PW, px = ld_px0 + pp % V2_PW;
      const int cy = min(max(py, 0), PH - 1), cx = min(max(px, 0), PW - 1);
      ra[q] = *reinterpret_cast<const uint4*>(a.x + (((long long)n * PH + cy) * PW + cx) * a.x_ld + c8 * 8);
      rc[q] = *reinterpret_cast<const uint2*>(a.code + ((nc * PH + cy) * PW + cx) * C64 + c8 * 8);
    }
  };
  auto store_tile = [&](uint8_t* As, int t) {  // expand pooled chunks into the unpooled halo
    const int tid = opaque_tid();
    int b = t;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;  // halo origin (unpooled)
#pragma unroll
    for (int q = 0; q < V2_PER_T; ++q) {
      const int idx = tid + q * 512;
      if (idx >= V2_TASKS) continue;
      const int pp = idx >> 3, c8 = idx & 7;
      const int py = ld_py0 + pp / V2_PW, px = ld_px0 + pp % V2_PW;
      const bool in = (unsigned)py < (unsigned)PH && (unsigned)px < (unsigned)PW;
      uint4 v = in ? ra[q] : make_uint4(0, 0, 0, 0);
      if (a.relu_in) {
        v.x = relu_bf2(v.x);
        v.y = relu_bf2(v.y);
        v.z = relu_bf2(v.z);
        v.w = relu_bf2(v.w);
      }
      const uint4 sp = unpool_spread(rc[q]);
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int hy = 2 * py + (d >> 1) - y0, hx = 2 * px + (d & 1) - x0;
        if ((unsigned)hy >= (unsigned)IH || (unsigned)hx >= (unsigned)IW) continue;
        const uint4 o = unpool_pick_s(v, sp, (uint32_t)d);
        *reinterpret_cast<uint4*>(As + (hy * IW + hx) * PIXB + c8 * 16) = o;
      }
    }
  };

  int t = blockIdx.x;
  if (t < ntiles) {
    load_tile(t);
    store_tile(smem, t);
  }
  __syncthreads();
  int cur = 0;
  while (t < ntiles) {
    const int tcur = t;
    t += gridDim.x;
    if (t < ntiles) load_tile(t);  // in flight during the MFMAs
    const uint8_t* As = smem + cur * V2_A;
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // A fragment address = per-fragment base (lane-dependent) + a compile-time tap/half offset
    const uint8_t* Ab[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) Ab[i] = As + ((2 * wr + (i >> 1)) * IW + (i & 1) * 16 + col) * PIXB + kq * 16;
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int tap = s >> 1, kh = tap / 3, kw = tap % 3;
      const int off = (kh * IW + kw) * PIXB + (s & 1) * 64;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(Ab[i] + off);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = TR ? __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[s][j], af, acc[i][j], 0, 0, 0)
                         : __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bw[s][j], acc[i][j], 0, 0, 0);
      }
      if constexpr (ILV) {
        if (!NO_EXP && s == 12 && t < ntiles) store_tile(smem + (cur ^ 1) * V2_A, t);  // behind the remaining MFMAs
      }
    }
    __syncthreads();  // every wave is done with the previous tile's Cst reads and this halo
    // ---- output tile -> Cst (bias, ReLU); C row = pixel, C col = channel ----
    if constexpr (TR) {  // lane (col, kq): pixel col of fragment i, channels j*16 + kq*4 .. + 3
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ch = wc * 32 + j * 16 + kq * 4;
          const int pix = (2 * wr + (i >> 1)) * TW + (i & 1) * 16 + col;
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[i][j][r] + biasv[j][r];
            if (a.relu) v[r] = fmaxf(v[r], 0.f);
          }
          *reinterpret_cast<uint2*>(Cst + pix * 128 + ((((ch >> 3) ^ (pix & 7))) << 4) + (ch & 7) * 2) =
              make_uint2(pack_bf2(v[0], v[1]), pack_bf2(v[2], v[3]));
        }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int ch = wc * 32 + j * 16 + col;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int pix = (2 * wr + (i >> 1)) * TW + (i & 1) * 16 + kq * 4 + r;
            float v = acc[i][j][r] + biasv[j][0];
            if (a.relu) v = fmaxf(v, 0.f);
            *reinterpret_cast<uint16_t*>(Cst + pix * 128 + ((((ch >> 3) ^ (pix & 7))) << 4) + (ch & 7) * 2) = f2bf(v);
          }
        }
    }
    if constexpr (!ILV) {
      if (t < ntiles) store_tile(smem + (cur ^ 1) * V2_A, t);
    }
    __syncthreads();
    if constexpr (NO_Z) {  // ablation: no Z GEMM and no output stores at all
    } else if constexpr (ZOUT) {  // ---- Z = D W2^T for tile row `wave`, 8-B stores (4 Z channels of one px) ----
      int b = tcur;
      const int tx = b % tiles_w;
      b /= tiles_w;
      const int ty = b % tiles_h;
      const int n = b / tiles_h;
      const int oy = ty * TH + wave;
      f32x4 z[2][2];
#pragma unroll
      for (int jz = 0; jz < 2; ++jz)
#pragma unroll
        for (int pf = 0; pf < 2; ++pf) z[jz][pf] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int pf = 0; pf < 2; ++pf) {
        const int pix = wave * TW + pf * 16 + col;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          const bf16x8 bd = *reinterpret_cast<const bf16x8*>(Cst + pix * 128 + (((ks * 4 + kq) ^ (pix & 7)) << 4));
#pragma unroll
          for (int jz = 0; jz < 2; ++jz) {
            const bf16x8 wa = *reinterpret_cast<const bf16x8*>(W2s + (jz * 16 + col) * 128 + (((ks * 4 + kq) ^ (col & 7)) << 4));
            z[jz][pf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa, bd, z[jz][pf], 0, 0, 0);
          }
        }
      }
      // Z[px][zc]: lane (col, kq) holds Z channels jz*16 + kq*4 + r of pixel col. One v_permlane16_swap per
      // dword (rows kq <-> kq ^ 1, as the c8 stream kernel) leaves lane kq with block kq & 1, channels
      // (kq >> 1) * 8 .. + 7: ONE 16-B store per pixel block, each store instruction writing 16 pixels'
      // complete 64-B Z rows (1 KiB contiguous) instead of two instructions of 16 x 32-B halves
#pragma unroll
      for (int pf = 0; pf < 2; ++pf) {
        uint32_t pk[2][2];
#pragma unroll
        for (int jz = 0; jz < 2; ++jz) {
          pk[jz][0] = pack_bf2(z[jz][pf][0], z[jz][pf][1]);
          pk[jz][1] = pack_bf2(z[jz][pf][2], z[jz][pf][3]);
        }
#pragma unroll
        for (int d = 0; d < 2; ++d) {  // odd rows of pk[0] <-> even rows of pk[1]
          const auto sw = __builtin_amdgcn_permlane16_swap(pk[0][d], pk[1][d], false, false);
          pk[0][d] = sw[0];
          pk[1][d] = sw[1];
        }
        const int ox = tx * TW + pf * 16 + col;
        if (oy >= H || ox >= W) continue;
        const int zc = (kq & 1) * 16 + (kq >> 1) * 8;
        const long long zo = (((long long)n * H + oy) * W + ox) * a.out_ld + zc;
        if (DV_BOUNDS(zo, 8, a.out_elems, "unpool_z out"))
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out) + zo) =
              make_uint4(pk[0][0], pk[0][1], pk[1][0], pk[1][1]);
      }
    } else {  // ---- Cst -> global, 16 B per store ----
      const int tid = opaque_tid();
      int b = tcur;
      const int tx = b % tiles_w;
      b /= tiles_w;
      const int ty = b % tiles_h;
      const int n = b / tiles_h;
#pragma unroll
      for (int q = 0; q < (TH * TW * 8) / 512; ++q) {
        const int c = tid + q * 512, pix = c >> 3, cc = c & 7;
        const int oy = ty * TH + pix / TW, ox = tx * TW + pix % TW;
        if (oy >= H || ox >= W || cc * 8 >= a.OC) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(Cst + pix * 128 + ((cc ^ (pix & 7)) << 4));
        *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out) + (((long long)n * H + oy) * W + ox) * a.out_ld +
                                  cc * 8) = v;
      }
    }
    cur ^= 1;
  }
}

// ---------------------------------------------------------------------------------------------
// Row-streaming 3x3 conv, 64 -> OC <= 16 channels (the final block1_conv1.down: 64 -> 3, fp32).
//
// This layer is an HBM stream: 6.6 GB of bf16 input per 1024 signals against 0.18 TFLOP of useful
// math. The persistent halo kernel above re-stages a 10x34 halo per 8x32 tile between two
// barriers (1.33x input, MFMAs idle while staging) and reached 2.1 TB/s. Here one workgroup
// (4 waves) owns a 32-px column strip of one image and walks it top to bottom:
//   * input rows (34 px x 128 B) go straight to LDS by buffer_load...lds into a ring of
//     R = 4 (P + 2) row slots; conv padding and the strip/image edges are out-of-range offsets
//     that read as 0. Every input row is fetched once per strip (1.06x instead of 1.33x);
//   * P groups of 4 rows stay in flight behind the 2 groups being consumed (counted vmcnt, one
//     raw s_barrier per group: loads are never drained by a barrier);
//   * wave w computes output row 4i + w: 2 fragments of 16 px x one 16-wide N fragment, the 18
//     K-step weight fragments live in VGPRs (72 registers), A fragments are read at a per-lane
//     pixel address with the chunk XOR (pixel & 7) applied on the source side of the DMA;
//   * fp32 output of a full strip row (32 px x 3 ch = 384 contiguous bytes) is staged in LDS and
//     written with 16-B stores.
namespace {
constexpr int ST_W = 32;                  // output px per strip
constexpr int ST_IN = ST_W + 2;           // input px per strip row
constexpr int ST_SLOT = ST_IN * 128;      // 34 px: 4 x 1 KiB dwordx4 DMA + one 256-B dword DMA (2 px)
}  // namespace

typedef int i32x4 __attribute__((ext_vector_type(4)));
// LDS-DMA of 16 B per lane as inline asm. With the intrinsic, the compiler's waitcnt pass treats the
// instruction's offset VGPR as pending until the load returns and put an s_waitcnt vmcnt(0) in
// front of the first ds_read whose destination reused that register, draining every prefetched
// row each iteration; here the only waits are the counted vmcnt's of the kernel. M0 (LDS base of
// the 64 x 16 B destination) is set right before the load; nothing else in these kernels uses M0.
__device__ __forceinline__ void dma16_asm(const i32x4& rsrc, uint32_t lds_addr, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc)
               : "memory");
}

__device__ __forceinline__ void dma4_asm(const i32x4& rsrc, uint32_t lds_addr, uint32_t voff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dword %1, %2, 0 offen lds"
               :
               : "s"(__builtin_amdgcn_readfirstlane(lds_addr)), "v"(voff), "s"(rsrc)
               : "memory");
}

// ReLU of 2 packed 16-bit floats as one v_pk_max_i16: negative values (sign bit set) are negative
// int16, so max(v, 0) zeroes them (and -0) and keeps every non-negative value bit-exactly
__device__ __forceinline__ uint32_t relu_pk16(uint32_t v) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  const s16x2 r = __builtin_elementwise_max(__builtin_bit_cast(s16x2, v), (s16x2){0, 0});
  return __builtin_bit_cast(uint32_t, r);
}

template <int P, int EPI, bool RELU_IN>
__global__ void __launch_bounds__(256, 1) conv3x3_c64_stream_kernel(const ConvArgs a) {
  constexpr int R = 4 * (P + 2);
  __shared__ __attribute__((aligned(16))) uint8_t smem[R * ST_SLOT + 4 * ST_W * 3 * 4];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, col = lane & 15;
  const int H = a.H, W = a.W;
  const int strips_w = (W + ST_W - 1) / ST_W;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / strips_w;
  const int x0 = (bid - n * strips_w) * ST_W;  // first output px of the strip

  const long long img = (long long)H * W * a.x_ld;
  const long long rem = (long long)a.N * img - (long long)n * img;
  const uint64_t bytes = (uint64_t)(rem * 2);
  // buffer descriptor as 4 SGPRs {base lo, base hi (stride 0), num_records, flags}
  i32x4 xr;
  {
    const uint64_t base = reinterpret_cast<uint64_t>(a.x + (long long)n * img);
    xr.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    xr.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFFu));
    xr.z = __builtin_amdgcn_readfirstlane((int)(bytes > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)bytes));
    xr.w = 0x00020000;
  }

  // weights: k-step s = tap*2 + half; B fragment lane (col = out channel, kq = 8-element K chunk)
  bf16x8 bw[18];
#pragma unroll
  for (int s = 0; s < 18; ++s) {
    const int k = (s >> 1) * C64 + (s & 1) * 32 + kq * 8;
    bw[s] = *reinterpret_cast<const bf16x8*>(a.w + (long long)col * a.Kpad + k);
  }
  float bias = (a.bias && col < a.OC) ? a.bias[col] : 0.f;
  // consume the weight loads here, so the compiler's wait for them sits before the prologue DMAs
  // (it cannot see the asm DMAs; a vmcnt(0) after them would drain the whole prefetch)
#pragma unroll
  for (int s = 0; s < 18; ++s) asm volatile("" : "+v"(bw[s]));
  asm volatile("" : "+v"(bias));

  // DMA lane geometry: instruction j covers strip pixels 8j..8j+7, lane -> (pixel, chunk slot)
  const int lp = lane >> 3, lc = lane & 7;
  auto issue_row = [&](int r) {  // input row r (may be -1 or >= H: zeros) -> its ring slot
    uint8_t* dst = smem + ((r + 1) % R) * ST_SLOT;
    const bool rok = (unsigned)r < (unsigned)H;
#pragma unroll
    for (int j = 0; j < 4; ++j) {  // pixels 0..31: lane -> (pixel 8j + lane/8, 16-B chunk slot lane%8)
      const int pix = j * 8 + lp;
      const int x = x0 - 1 + pix;
      const bool ok = rok && (unsigned)x < (unsigned)W;
      const uint32_t voff = ok ? (uint32_t)((((long long)r * W + x) * a.x_ld + ((lc ^ (pix & 7)) * 8)) * 2) : 0x80000000u;
      dma16_asm(xr, (uint32_t)(uintptr_t)(dst + j * 1024), voff);
    }
    {  // pixels 32, 33: 4 B per lane, lane -> (pixel 32 + lane/32, dword lane%32 of the swizzled pixel)
      const int pix = ST_W + (lane >> 5), wd = lane & 31;
      const int x = x0 - 1 + pix;
      const bool ok = rok && (unsigned)x < (unsigned)W;
      const uint32_t voff =
          ok ? (uint32_t)((((long long)r * W + x) * a.x_ld + (((wd >> 2) ^ (pix & 7)) * 8)) * 2 + (wd & 3) * 4) : 0x80000000u;
      dma4_asm(xr, (uint32_t)(uintptr_t)(dst + 4 * 1024), voff);
    }
  };
  // group g = input rows 4g-1 .. 4g+2, row 4g-1+w loaded by wave w
#pragma unroll
  for (int g = 0; g <= P; ++g) issue_row(4 * g - 1 + wave);

  // per-lane A-fragment chunk offsets: pixel p = fi*16 + col + kw, chunk kc = half*4 + kq
  int xo[3][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int h = 0; h < 2; ++h) xo[kw][h] = (col + kw) * 128 + (((h * 4 + kq) ^ ((col + kw) & 7)) << 4);
  float* stage = reinterpret_cast<float*>(smem + R * ST_SLOT) + wave * ST_W * 3;
  const bool vec_out = EPI == CONV_E_F32 && a.OC == 3 && a.out_ld == 3 && x0 + ST_W <= W && (W & 3) == 0 &&
                       (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;

  double st1 = 0.0, st2 = 0.0;  // this lane's share of sum(out), sum(out^2) (a.stats)
  const int iters = (H + 3) / 4;
  for (int i = 0; i < iters; ++i) {
    if constexpr (P >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(5 * (P - 1)) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_row(4 * (i + P + 1) - 1 + wave);  // past the map: zero rows (keeps the vmcnt count uniform)
    const int y = 4 * i + wave;
    if (y < H) {
      f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
      // all 36 A fragments of the row are read before the first MFMA (LDS latency overlaps the
      // reads instead of serializing read -> MFMA pairs: one wave per SIMD has nothing to hide it)
      uint4 af[36];
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const uint8_t* rowp = smem + ((y + kh) % R) * ST_SLOT;  // input row y-1+kh
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int fi = 0; fi < 2; ++fi)
              af[((kh * 3 + kw) * 2 + h) * 2 + fi] = *reinterpret_cast<const uint4*>(rowp + fi * 16 * 128 + xo[kw][h]);
      }
#pragma unroll
      for (int s = 0; s < 18; ++s)
#pragma unroll
        for (int fi = 0; fi < 2; ++fi) {
          uint4 v = af[s * 2 + fi];
          if constexpr (RELU_IN) {
            v.x = relu_pk16(v.x);
            v.y = relu_pk16(v.y);
            v.z = relu_pk16(v.z);
            v.w = relu_pk16(v.w);
          }
          acc[fi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, v), bw[s], acc[fi], 0, 0, 0);
        }
      // C fragment: lane holds px fi*16 + kq*4 + r of output channel col
      const long long obase = ((long long)n * H + y) * W + x0;
      if (vec_out) {
        if (col < 3) {
#pragma unroll
          for (int fi = 0; fi < 2; ++fi)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float v = acc[fi][r] + bias;
              if (a.relu) v = fmaxf(v, 0.f);
              st1 += v;
              st2 += (double)v * v;
              stage[(fi * 16 + kq * 4 + r) * 3 + col] = v;
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (lane < ST_W * 3 / 4)
          *reinterpret_cast<float4*>(reinterpret_cast<float*>(a.out) + obase * 3 + lane * 4) =
              *reinterpret_cast<const float4*>(stage + lane * 4);
        __builtin_amdgcn_wave_barrier();
      } else if (col < a.OC) {
#pragma unroll
        for (int fi = 0; fi < 2; ++fi)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int ox = x0 + fi * 16 + kq * 4 + r;
            if (ox >= W) continue;
            float v = acc[fi][r] + bias;
            if (a.relu) v = fmaxf(v, 0.f);
            st1 += v;
            st2 += (double)v * v;
            const long long o = (obase + (ox - x0)) * a.out_ld + col;
            if (!DV_BOUNDS(o, 1, a.out_elems, "stream conv out")) continue;
            if constexpr (EPI == CONV_E_F32)
              reinterpret_cast<float*>(a.out)[o] = v;
            else
              reinterpret_cast<uint16_t*>(a.out)[o] = f2bf(v);
          }
      }
    }
  }
  if (a.stats) {  // per-image statistics for the single-pass deprocess (one atomic pair per wave)
    st1 = wave_sum_d(st1);
    st2 = wave_sum_d(st2);
    if (lane == 0) {
      double* d = a.stats + 2 * (n / a.stats_div);
      atomicAdd(d, st1);
      atomicAdd(d + 1, st2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA may land after the workgroup retires
}


// ---------------------------------------------------------------------------------------------
// v3: forward 3x3 conv 64 -> 64 + bias + ReLU + fused 2x2 max-pool with switch codes
// (block1_conv2 forward: 224x224x64 -> pooled 112x112x64 + uint8 codes).
//
// The implicit-GEMM kernel runs this layer at ~0.5 PF/s (512x64 tiles re-fetch every input pixel
// per tap). Here (one 512-thread workgroup per CU, persistent over 8x32 output tiles):
//   * wave w owns output rows {2(w/2), 2(w/2)+1} x 32 px x channels [32 (w%2), +32); its weights
//     (18 K-steps x 2 fragments) stay in VGPRs, as in v2;
//   * the 10 x 34 x 64 halo of the NEXT tile is LDS-DMA'd row by row (4 x 1 KiB + 256 B per row,
//     chunk XOR (pixel & 7) applied on the source side) into the other half of a double buffer
//     while this tile's MFMAs run: no register staging, no VALU on the input;
//   * each lane's accumulators already hold whole 2x2 pool windows (rows i>>1, columns r, r+1), so
//     max + first-max switch code are computed in registers; pooled bf16 values and codes are
//     staged in LDS and written with 16-B stores (the full-resolution activation is never stored).
namespace {
constexpr int V3_BUF = IH * ST_SLOT;                 // 10 rows x 4352 B
constexpr int V3_PV = (TH / 2) * (TW / 2) * 128;     // pooled bf16 staging (64 px x 64 ch)
constexpr int V3_PC = (TH / 2) * (TW / 2) * 64;      // pooled code staging
}  // namespace

__global__ void __launch_bounds__(256, 1) conv3x3_c64_pool_v3_kernel(const ConvArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * V3_BUF + V3_PV + V3_PC];
  __shared__ float bias_s[64];
  uint8_t* Pv = smem + 2 * V3_BUF;
  uint8_t* Pc = Pv + V3_PV;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave;  // output rows 2 wr, 2 wr + 1; all 64 channels
  const int kq = lane >> 4, col = lane & 15;
  const int H = a.H, W = a.W, PH = H >> 1, PW = W >> 1;
  const int tiles_w = (W + TW - 1) / TW, tiles_h = (H + TH - 1) / TH;
  const int ntiles = a.N * tiles_h * tiles_w;

  bf16x8 bw[18][4];
#pragma unroll
  for (int s = 0; s < 18; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int oc = j * 16 + col;
      const int k = (s >> 1) * C64 + (s & 1) * 32 + kq * 8;
      bw[s][j] = *reinterpret_cast<const bf16x8*>(a.w + (long long)oc * a.Kpad + k);
    }
  if (tid < 64) bias_s[tid] = a.bias ? a.bias[tid] : 0.f;  // read back in the epilogue (frees VGPRs)
#pragma unroll
  for (int s = 0; s < 18; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(bw[s][j]));  // weight loads done before any DMA

  // lane-dependent DMA address terms are recomputed from an opaque lane id in every call: hoisted
  // out of the persistent loop they would be held across the MFMAs (weights fill the VGPRs)
  auto issue_tile = [&](int t, uint8_t* buf) {  // 10 halo rows of tile t -> buf (50 DMA pieces)
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    const int lp = ln >> 3, lc = ln & 7;
    int b = t;
    const int tx = b % tiles_w;
    b /= tiles_w;
    const int ty = b % tiles_h;
    const int n = __builtin_amdgcn_readfirstlane(b / tiles_h);
    const int y0 = ty * TH - 1, x0 = tx * TW - 1;
    const long long img = (long long)H * W * a.x_ld;
    const uint64_t base = reinterpret_cast<uint64_t>(a.x + (long long)n * img);
    i32x4 xr;
    xr.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    xr.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFFu));
    xr.z = __builtin_amdgcn_readfirstlane((int)(img * 2 > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)(img * 2)));
    xr.w = 0x00020000;
    for (int q = wave; q < IH * 5; q += 4) {  // wave-uniform piece list
      const int hr = q / 5, piece = q - hr * 5;
      const int y = y0 + hr;
      const bool rok = (unsigned)y < (unsigned)H;
      uint8_t* dst = buf + hr * ST_SLOT + piece * 1024;
      if (piece < 4) {
        const int pix = piece * 8 + lp;
        const int x = x0 + pix;
        const bool ok = rok && (unsigned)x < (unsigned)W;
        const uint32_t voff = ok ? (uint32_t)((((long long)y * W + x) * a.x_ld + ((lc ^ (pix & 7)) * 8)) * 2) : 0x80000000u;
        dma16_asm(xr, (uint32_t)(uintptr_t)dst, voff);
      } else {
        const int pix = TW + (ln >> 5), wd = ln & 31;
        const int x = x0 + pix;
        const bool ok = rok && (unsigned)x < (unsigned)W;
        const uint32_t voff = ok ? (uint32_t)((((long long)y * W + x) * a.x_ld + (((wd >> 2) ^ (pix & 7)) * 8)) * 2 +
                                              (wd & 3) * 4)
                                 : 0x80000000u;
        dma4_asm(xr, (uint32_t)(uintptr_t)dst, voff);
      }
    }
  };


  int t = blockIdx.x;
  if (t < ntiles) issue_tile(t, smem);
  int cur = 0;
  while (t < ntiles) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int tcur = t;
    t += gridDim.x;
    if (t < ntiles) issue_tile(t, smem + (cur ^ 1) * V3_BUF);
    const uint8_t* buf = smem + cur * V3_BUF;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 18; ++s) {
      const int tap = s >> 1, kh = tap / 3, kw = tap % 3, h = s & 1;
      const int p = col + kw;  // A-fragment pixel within the halo row (+ 16 for i & 1)
      const int xo = p * 128 + (((h * 4 + kq) ^ (p & 7)) << 4);
      uint4 af[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const uint4*>(buf + (2 * wr + (i >> 1) + kh) * ST_SLOT + (i & 1) * 2048 + xo);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]), bw[s][j], acc[i][j], 0,
                                                              0, 0);
    }
    // ---- 2x2 max-pool in registers: window (rows i>>1 = 0/1) x (columns r = 2q, 2q+1) ----
#pragma unroll
    for (int hx = 0; hx < 2; ++hx)      // 16-px half of the row (fragment i & 1)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int ch = j * 16 + col;
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          float best = -INFINITY;
          int code = 0;
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            float v = acc[hx + 2 * (d >> 1)][j][2 * q + (d & 1)] + bias_s[ch];
            if (a.relu) v = fmaxf(v, 0.f);
            v = bf2f(f2bf(v));
            if (v > best) {
              best = v;
              code = d;
            }
          }
          const int pix = wr * 16 + hx * 8 + kq * 2 + q;  // pooled pixel within the 4 x 16 tile
          *reinterpret_cast<uint16_t*>(Pv + pix * 128 + ((((ch >> 3) ^ (pix & 7))) << 4) + (ch & 7) * 2) = f2bf(best);
          Pc[pix * 64 + ch] = (uint8_t)code;
        }
      }
    __syncthreads();
    {
      int b = tcur;
      const int tx = b % tiles_w;
      b /= tiles_w;
      const int ty = b % tiles_h;
      const int n = b / tiles_h;
#pragma unroll
      for (int q = 0; q < 2; ++q) {  // 64 px x 8 chunks = two 16-B chunks per thread
        const int c = tid + q * 256, pix = c >> 3, cc = c & 7;
        const int py = ty * (TH / 2) + (pix >> 4), px = tx * (TW / 2) + (pix & 15);
        if (py < PH && px < PW) {
          const long long prow = ((long long)n * PH + py) * PW + px;
          *reinterpret_cast<uint4*>(reinterpret_cast<uint16_t*>(a.out) + prow * a.out_ld + cc * 8) =
              *reinterpret_cast<const uint4*>(Pv + pix * 128 + ((cc ^ (pix & 7)) << 4));
          if (cc < 4)
            *reinterpret_cast<uint4*>(a.out_code + prow * 64 + cc * 16) =
                *reinterpret_cast<const uint4*>(Pc + pix * 64 + cc * 16);
        }
      }
    }
    cur ^= 1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}


// ---------------------------------------------------------------------------------------------
// Row-streaming first layer: 3x3 conv of an 8-channel (RGB padded) image -> OC <= 64 channels,
// bias + ReLU, bf16 out (VGG16 block1_conv1 forward). K = 9 taps x 8 channels = 72 (3 MFMA K-steps
// of 32, taps 9..11 have zero weights). The layer is output-write bound (64 bf16 channels per pixel
// from 3 real input channels): the input strip rows (34 px x 16 B) stream through a small LDS ring
// (one 1 KiB LDS-DMA per row), and the MFMA is issued TRANSPOSED (A = weights, B = pixels) so each
// lane's accumulator holds 4 consecutive channels of one pixel: the epilogue packs them into one
// 8-B store per lane and MFMA tile, 16 pixels x 32 contiguous bytes per store instruction.
namespace {
constexpr int S8_W = 32;        // output px per strip
constexpr int S8_SLOT = 1024;   // 64 px x 16 B per row slot (34 used)
}  // namespace

// FULL (H % 4 == 0, W % 32 == 0, OC == 64): every wave issues exactly 1 DMA + 8 stores per iteration,
// so the wait counts the younger stores instead of draining them (vmcnt counts loads, stores and
// LDS-DMA in issue order); otherwise the wait conservatively drains the previous stores too.
// Iteration i needs row group i+1. Younger than it: the prologue's groups i+2..P and iterations
// 0..i-1 (1 DMA + 8 stores each) while i < P, i.e. P-1+8i; in the steady state (i >= P) the stores of
// iteration i-P and iterations i-P+1..i-1, i.e. 9P-1. The first P iterations need their own
// (smaller) immediates: waiting with the steady-state count there does not wait at all.
template <int P, int I = 0>
__device__ __forceinline__ void c8_full_wait(int i) {
  if constexpr (I >= P) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(9 * P - 1) : "memory");
  } else {
    if (i == I)
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P - 1 + 8 * I) : "memory");
    else
      c8_full_wait<P, I + 1>(i);
  }
}

template <int P, bool FULL>
__global__ void __launch_bounds__(256) conv3x3_c8_stream_kernel(const ConvArgs a) {
  constexpr int R = 4 * (P + 2);
  __shared__ __attribute__((aligned(16))) uint8_t smem[R * S8_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kq = lane >> 4, col = lane & 15;
  const int H = a.H, W = a.W;
  const int strips_w = (W + S8_W - 1) / S8_W;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / strips_w;
  const int x0 = (bid - n * strips_w) * S8_W;

  const long long img = (long long)H * W * a.x_ld;
  i32x4 xr;
  {
    const uint64_t base = reinterpret_cast<uint64_t>(a.x + (long long)n * img);
    xr.x = __builtin_amdgcn_readfirstlane((int)(uint32_t)base);
    xr.y = __builtin_amdgcn_readfirstlane((int)((uint32_t)(base >> 32) & 0xFFFFu));
    xr.z = __builtin_amdgcn_readfirstlane((int)(img * 2 > 0x7FFFFFF0LL ? 0x7FFFFFF0u : (uint32_t)(img * 2)));
    xr.w = 0x00020000;
  }
  // A = weights: fragment (K-step s, 16-channel block j): lane -> channel j*16 + col, K chunk kq
  bf16x8 wa[3][4];
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      wa[s][j] = *reinterpret_cast<const bf16x8*>(a.w + (long long)(j * 16 + col) * a.Kpad + s * 32 + kq * 8);
  float bias[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int oc = j * 16 + kq * 4 + r;
      bias[j][r] = (a.bias && oc < a.OC) ? a.bias[oc] : 0.f;
    }
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(wa[s][j]));
#pragma unroll
  for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(bias[j][0]), "+v"(bias[j][1]), "+v"(bias[j][2]), "+v"(bias[j][3]));

  auto issue_row = [&](int r) {  // input row r -> slot; lane = strip pixel (x0 - 1 + lane), 16 B
    const int x = x0 - 1 + lane;
    const bool ok = lane < S8_W + 2 && (unsigned)x < (unsigned)W && (unsigned)r < (unsigned)H;
    const uint32_t voff = ok ? (uint32_t)((((long long)r * W + x) * a.x_ld) * 2) : 0x80000000u;
    dma16_asm(xr, (uint32_t)(uintptr_t)(smem + ((r + 1) % R) * S8_SLOT), voff);
  };
#pragma unroll
  for (int g = 0; g <= P; ++g) issue_row(4 * g - 1 + wave);

  // B operand of K-step s: tap t = 4 s + kq (zero for t >= 9) at strip pixel fi*16 + col + kw
  const int iters = (H + 3) / 4;
  for (int i = 0; i < iters; ++i) {
    if constexpr (FULL) c8_full_wait<P>(i);
    else if constexpr (P >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P - 1) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    issue_row(4 * (i + P + 1) - 1 + wave);
    const int y = 4 * i + wave;
    if (FULL || y < H) {
      f32x4 acc[2][4];
#pragma unroll
      for (int fi = 0; fi < 2; ++fi)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[fi][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int t = 4 * s + kq;
        const int kh = t / 3, kw = t - 3 * (t / 3);
        const bool tv = t < 9;
#pragma unroll
        for (int fi = 0; fi < 2; ++fi) {
          uint4 bv = make_uint4(0, 0, 0, 0);
          if (tv) bv = *reinterpret_cast<const uint4*>(smem + ((y + kh) % R) * S8_SLOT + (fi * 16 + col + kw) * 16);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            acc[fi][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wa[s][j], __builtin_bit_cast(bf16x8, bv), acc[fi][j],
                                                                 0, 0, 0);
        }
      }
      // C[channel][px]: lane (px = fi*16 + col, kq) holds channels j*16 + kq*4 + r, r = 0..3. A
      // v_permlane16_swap per dword of each block pair (j, j+1) gathers 8 consecutive channels per
      // lane (row kq: block j + (kq & 1), channels (kq >> 1) * 8 + 0..7): one 16-B store per pair
      // instead of two 8-B ones (the layer is store-issue bound: dwordx2 stores issue at half the
      // bytes per instruction, MI355X_MICROARCH T21). All lanes swap; only the stores are guarded.
#pragma unroll
      for (int fi = 0; fi < 2; ++fi) {
        const int ox = x0 + fi * 16 + col;
        uint32_t pk[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            v[r] = acc[fi][j][r] + bias[j][r];
            if (a.relu) v[r] = fmaxf(v[r], 0.f);
          }
          pk[j][0] = pack_bf2(v[0], v[1]);
          pk[j][1] = pack_bf2(v[2], v[3]);
        }
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2)
#pragma unroll
          for (int d = 0; d < 2; ++d) {  // odd rows of pk[jp] <-> even rows of pk[jp + 1]
            const auto sw = __builtin_amdgcn_permlane16_swap(pk[jp][d], pk[jp + 1][d], false, false);
            pk[jp][d] = sw[0];
            pk[jp + 1][d] = sw[1];
          }
        if (!FULL && ox >= W) continue;
        uint16_t* orow = reinterpret_cast<uint16_t*>(a.out) + (((long long)n * H + y) * W + ox) * a.out_ld;
#pragma unroll
        for (int jp = 0; jp < 4; jp += 2) {
          const int oc = (jp + (kq & 1)) * 16 + (kq >> 1) * 8;
          if (!FULL && oc >= a.OC) continue;
          *reinterpret_cast<uint4*>(orow + oc) = make_uint4(pk[jp][0], pk[jp][1], pk[jp + 1][0], pk[jp + 1][1]);
        }
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int conv3x3_c8_stream_launch(const ConvArgs& a, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != 8 || a.x_ld != 8 || a.relu_in ||
      a.OC > 64 || a.OCpad != 64 || a.OC % 8 != 0 || a.H != a.OH || a.W != a.OW || a.accumulate || a.mask ||
      a.Kpad < 96 || a.out_ld % 8 != 0 || a.dtype != DT_BF16 || a.res || a.emask ||
      (reinterpret_cast<uintptr_t>(a.out) & 15))
    return -4;
  const long long nwg = (long long)a.N * ((a.W + S8_W - 1) / S8_W);
  if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
  if (a.H % 4 == 0 && a.W % S8_W == 0 && a.OC == 64)
    hipLaunchKernelGGL((conv3x3_c8_stream_kernel<4, true>), dim3((unsigned)nwg), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((conv3x3_c8_stream_kernel<4, false>), dim3((unsigned)nwg), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

static int stream_variant() {
  static int v = [] {
    const char* e = dv_ab_env("DV_STREAM_P");  // measured: P=1 (3 WG/CU) 1.57 ms, P=2 1.60, P=3 1.94
    return e ? std::atoi(e) : 1;
  }();
  return v;
}

template <int FN, int EPI, bool UNPOOL>
static int persist_cfg(const ConvArgs& a, hipStream_t s) {
  const long long ntiles = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  if (ntiles <= 0 || ntiles > 0x7fffffffLL) return -2;
  // CU count queried once (keeps the launch path free of runtime queries during graph capture)
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const long long grid = std::min<long long>(ntiles, (long long)cus);
  hipLaunchKernelGGL((conv3x3_c64_persist_kernel<FN, EPI, UNPOOL>), dim3((unsigned)grid), dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

int conv3x3_pool_v3_launch(const ConvArgs& a, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != C64 || a.OC != 64 ||
      a.OCpad != 64 || a.H != a.OH || a.W != a.OW || (a.H & 1) || (a.W & 1) || a.accumulate || a.mask ||
      a.Kpad < KW9 || a.x_ld % 8 || a.out_ld % 8 || a.dtype != DT_BF16 || a.res || a.emask ||
      (reinterpret_cast<uintptr_t>(a.out) & 15) || (reinterpret_cast<uintptr_t>(a.out_code) & 15))
    return -4;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const long long ntiles = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  if (ntiles <= 0 || ntiles > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL(conv3x3_c64_pool_v3_kernel, dim3((unsigned)std::min<long long>(ntiles, cus)), dim3(256), 0, s, a);
  return (int)hipGetLastError();
}

int conv3x3_halo_launch(const ConvArgs& a, int unpool, int epi, hipStream_t s, bool* stats_done) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != C64 || a.H != a.OH ||
      a.W != a.OW || a.accumulate || a.mask || a.Kpad < KW9)
    return -4;
  const bool narrow = a.OC <= 16;
  if (!narrow && a.OCpad != 64) return -5;
  // v2: unpool + 64 -> 64 with a 16-B aligned bf16 output of 64-channel rows (block1_conv2.down)
  if (unpool && !narrow && epi == CONV_E_BF16 && a.OC == 64 && a.out_ld % 8 == 0 && a.x_ld % 8 == 0 &&
      (a.H % 2) == 0 && (a.W % 2) == 0) {
    static const int cus = [] {
      int dev = 0, n = 256;
      if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n = 256;
      return n > 0 ? n : 256;
    }();
    const long long ntiles = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
    if (ntiles <= 0 || ntiles > 0x7fffffffLL) return -2;
    hipLaunchKernelGGL(conv3x3_unpool_c64_v2_kernel<false>, dim3((unsigned)std::min<long long>(ntiles, cus)), dim3(512), 0, s,
                       a);
    return (int)hipGetLastError();
  }
  if (!unpool && narrow) {  // row-streaming strips
    const long long nwg = (long long)a.N * ((a.W + ST_W - 1) / ST_W);
    if (nwg <= 0 || nwg > 0x7fffffffLL) return -2;
    const int P = stream_variant();
    if (stats_done) *stats_done = a.stats != nullptr;
#define DV_S2(PP, E)                                                                                               \
  do {                                                                                                             \
    if (a.relu_in)                                                                                                 \
      hipLaunchKernelGGL((conv3x3_c64_stream_kernel<PP, E, true>), dim3((unsigned)nwg), dim3(256), 0, s, a);       \
    else                                                                                                           \
      hipLaunchKernelGGL((conv3x3_c64_stream_kernel<PP, E, false>), dim3((unsigned)nwg), dim3(256), 0, s, a);      \
  } while (0)
#define DV_S(PP)                                                 \
  do {                                                           \
    if (epi == CONV_E_F32) DV_S2(PP, CONV_E_F32);                \
    else DV_S2(PP, CONV_E_BF16);                                 \
    return (int)hipGetLastError();                               \
  } while (0)
    if (P == 1) DV_S(1);
    if (P == 3) DV_S(3);
    if (P == 4) DV_S(4);
    DV_S(2);
#undef DV_S
#undef DV_S2
  }
#define DV_P(FN, E) return unpool ? persist_cfg<FN, E, true>(a, s) : persist_cfg<FN, E, false>(a, s)
  if (epi == CONV_E_F32) {
    if (narrow) DV_P(1, CONV_E_F32);
    DV_P(4, CONV_E_F32);
  }
  if (epi == CONV_E_BF16) {
    if (narrow) DV_P(1, CONV_E_BF16);
    DV_P(4, CONV_E_BF16);
  }
#undef DV_P
  return -1;
}

int conv3x3_unpool_z_launch(const ConvArgs& a, hipStream_t s) {
  if (a.KH != 3 || a.KW != 3 || a.stride != 1 || a.pad_h != 1 || a.pad_w != 1 || a.C != C64 || a.OC != 64 ||
      a.OCpad != 64 || a.H != a.OH || a.W != a.OW || (a.H & 1) || (a.W & 1) || a.Kpad < KW9 || a.x_ld % 8 ||
      a.out_ld != 32 || a.w2 == nullptr || a.code == nullptr || a.code_div < 1 || a.N % a.code_div ||
      a.dtype != DT_BF16 || a.accumulate || a.mask || a.res || a.emask || a.ucode || a.stats || a.bias ||
      (reinterpret_cast<uintptr_t>(a.out) & 15) || (reinterpret_cast<uintptr_t>(a.w2) & 15) ||
      (reinterpret_cast<uintptr_t>(a.x) & 15) || (reinterpret_cast<uintptr_t>(a.code) & 7))
    return -4;
  static const int cus = [] {
    int dev = 0, n = 256;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      n = 256;
    return n > 0 ? n : 256;
  }();
  const long long ntiles = (long long)a.N * ((a.H + TH - 1) / TH) * ((a.W + TW - 1) / TW);
  if (ntiles <= 0 || ntiles > 0x7fffffffLL) return -2;
  // DV_TAIL_V: variant bits (see the kernel); 3 by default, 0 = the round-4 schedule (A/B)
  const char* tve = dv_ab_env("DV_TAIL_V");  // per launch: tests switch it in one process
  int tv = tve ? std::atoi(tve) : 3;
  if ((tv & ~3) && dv_ab_env("DV_ALLOW_WRONG_ABLATION") == nullptr) tv &= 3;  // ablation bits: tools only
  const dim3 g((unsigned)std::min<long long>(ntiles, cus));
  if (tv == 0) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 0>), g, dim3(512), 0, s, a);
  else if (tv == 1) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 1>), g, dim3(512), 0, s, a);
  else if (tv == 2) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 2>), g, dim3(512), 0, s, a);
  else if (tv == 3) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 3>), g, dim3(512), 0, s, a);
  else if (tv == 3 + 4) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 3 + 4>), g, dim3(512), 0, s, a);
  else if (tv == 3 + 8) hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 3 + 8>), g, dim3(512), 0, s, a);
  else hipLaunchKernelGGL((conv3x3_unpool_c64_v2_kernel<true, 3 + 4 + 8>), g, dim3(512), 0, s, a);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// 9-tap shift-add finishing a Z map (see ZOUT above): out[y, x, c] = ReLU(sum_{kh,kw}
// Z[y+kh-1, x+kw-1, (kh*3+kw)*3 + c]) in fp32, zero padding. One 256-thread workgroup per 16 x 32 output
// tile: the 18 x 34-px halo of Z (27 used channels of 32, 16-B loads, all in flight before the LDS
// writes) is staged at a 34-halfword pixel pitch (17 dwords: odd, so the 32 lanes of a row reading
// consecutive pixels hit distinct banks), each thread sums 2 pixels x 3 channels x 9 taps from LDS.
// Per-image {sum, sum^2} of the output (the single-pass deprocess) are reduced per workgroup and
// added with one fp64 atomic pair.
namespace {
constexpr int ZS_TH = 16, ZS_TW = 32, ZS_IH = ZS_TH + 2, ZS_IW = ZS_TW + 2;
constexpr int ZS_PITCH = 34;                               // halfwords per staged pixel
constexpr int ZS_TASKS = ZS_IH * ZS_IW * 4;                // 16-B chunks (channels 0..31)
constexpr int ZS_PER_T = (ZS_TASKS + 255) / 256;           // 10
}  // namespace

__global__ void __launch_bounds__(256) zsum3x3_kernel(const uint16_t* __restrict__ z, float* __restrict__ out, int H,
                                                      int W, int tiles_x, int tiles_y, double* __restrict__ stats,
                                                      int stats_div, long long z_elems, long long out_elems) {
  __shared__ uint32_t zs[ZS_IH * ZS_IW * ZS_PITCH / 2];
  __shared__ double red[2][4];
  const int tid = threadIdx.x;
  const int per_img = tiles_x * tiles_y;
  const int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int n = bid / per_img;
  const int tr = bid - n * per_img;
  const int y0 = (tr / tiles_x) * ZS_TH, x0 = (tr % tiles_x) * ZS_TW;
  uint4 v[ZS_PER_T];
#pragma unroll
  for (int q = 0; q < ZS_PER_T; ++q) {
    const int idx = tid + q * 256;
    const int p = idx >> 2, ch = idx & 3;
    const int y = y0 - 1 + p / ZS_IW, x = x0 - 1 + p % ZS_IW;
    v[q] = make_uint4(0u, 0u, 0u, 0u);
    const long long off = (((long long)n * H + y) * W + x) * 32 + ch * 8;
    if (idx < ZS_TASKS && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W &&
        DV_BOUNDS(off, 8, z_elems, "zsum in"))
      v[q] = *reinterpret_cast<const uint4*>(z + off);
  }
#pragma unroll
  for (int q = 0; q < ZS_PER_T; ++q) {
    const int idx = tid + q * 256;
    if (idx >= ZS_TASKS) continue;
    const int p = idx >> 2, ch = idx & 3;
    uint32_t* d = zs + p * (ZS_PITCH / 2) + ch * 4;
    d[0] = v[q].x;
    d[1] = v[q].y;
    d[2] = v[q].z;
    d[3] = v[q].w;
  }
  __syncthreads();
  const uint16_t* zh = reinterpret_cast<const uint16_t*>(zs);
  const int lx = tid & 31, ly = tid >> 5;
  double s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int ry = ly + 8 * h;
    float o[3] = {0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < 3; ++kh)
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const uint16_t* zp = zh + ((ry + kh) * ZS_IW + lx + kw) * ZS_PITCH + (kh * 3 + kw) * 3;
#pragma unroll
        for (int c = 0; c < 3; ++c) o[c] += bf2f(zp[c]);
      }
    const int y = y0 + ry, x = x0 + lx;
    if (y < H && x < W) {
      const long long pix = ((long long)n * H + y) * W + x;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float r = fmaxf(o[c], 0.f);
        s1 += r;
        s2 += (double)r * r;
        if (DV_BOUNDS(pix * 3 + c, 1, out_elems, "zsum out")) out[pix * 3 + c] = r;
      }
    }
  }
  if (stats) {
    s1 = wave_sum_d(s1);
    s2 = wave_sum_d(s2);
    const int wave = tid >> 6, lane = tid & 63;
    if (lane == 0) {
      red[0][wave] = s1;
      red[1][wave] = s2;
    }
    __syncthreads();
    if (tid == 0) {
      double* d = stats + 2 * (n / stats_div);
      atomicAdd(d, red[0][0] + red[0][1] + red[0][2] + red[0][3]);
      atomicAdd(d + 1, red[1][0] + red[1][1] + red[1][2] + red[1][3]);
    }
  }
}

int zsum3x3_launch(const uint16_t* z, float* out, int N, int H, int W, double* stats, int stats_div, hipStream_t s) {
  if (N <= 0 || H <= 0 || W <= 0 || (stats && (stats_div < 1 || N % stats_div)) ||
      (reinterpret_cast<uintptr_t>(z) & 15))
    return -4;
  const int tx = (W + ZS_TW - 1) / ZS_TW, ty = (H + ZS_TH - 1) / ZS_TH;
  const long long nwg = (long long)N * tx * ty;
  if (nwg > 0x7fffffffLL) return -2;
  const long long pix = (long long)N * H * W;
  hipLaunchKernelGGL(zsum3x3_kernel, dim3((unsigned)nwg), dim3(256), 0, s, z, out, H, W, tx, ty, stats, stats_div,
                     pix * 32, pix * 3);
  return (int)hipGetLastError();
}

}  // namespace dv
