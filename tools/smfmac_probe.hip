// Probe for gfx950 2:4 structured-sparse MFMA (v_smfmac_f32_32x32x32_bf16): pins down the operand
// lane layout + sparsity-index encoding against a host fp32 reference, and measures its issue rate
// next to the dense v_mfma_f32_32x32x16_bf16 it would replace.
//
// Why: in the deconvnet backward, every conv-down that consumes a max-unpooled map (block1_conv2,
// block2_conv2, block3_conv3, block4_conv3 .down; 14 of the flagship's 38 conv-ms) reads an input
// where each channel has <= 1 nonzero per 2x2 pooling window. Re-grouping the 3x3 taps of one output
// sub-pixel phase by pooling window gives K-groups of 4 with <= 2 nonzeros (docs/KERNELS.md,
// "2:4 sparse MFMA for unpool-fed conv-downs"), i.e. exactly the SMFMAC contract, with the
// compressed A operand equal to the pooled value + its switch code. This probe is step 1.
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/smfmac_probe.hip -o build/smfmac_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) __bf16 bf16x16;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

// one wave: D = smfmac(Acomp, B, idx)
__global__ void __launch_bounds__(64) sparse_once(const uint16_t* a, const uint16_t* b, const uint32_t* idx,
                                                  float* d, int abid) {
  const int l = threadIdx.x;
  bf16x8 av;
  bf16x16 bv;
  for (int j = 0; j < 8; ++j) av[j] = __builtin_bit_cast(__bf16, a[l * 8 + j]);
  for (int j = 0; j < 16; ++j) bv[j] = __builtin_bit_cast(__bf16, b[l * 16 + j]);
  f32x16 c = {};
  if (abid == 0)
    c = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(av, bv, c, (int)idx[l], 0, 0);
  else
    c = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(av, bv, c, (int)idx[l], 0, 1);
  for (int i = 0; i < 16; ++i) d[l * 16 + i] = c[i];
}

template <bool SPARSE>
__global__ void __launch_bounds__(256) rate(float* out, int iters, uint32_t seed) {
  bf16x8 a8;
  bf16x16 b16;
  for (int j = 0; j < 8; ++j) a8[j] = (__bf16)(float)((threadIdx.x + j + seed) & 7);
  for (int j = 0; j < 16; ++j) b16[j] = (__bf16)(float)((threadIdx.x * 3 + j) & 7);
  const int idx = 0x4e4e4e4e;  // (2,3),(0,1) pairs: i0 < i1 in every group
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  for (int it = 0; it < iters; ++it) {
    if constexpr (SPARSE) {
      c0 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a8, b16, c0, idx, 0, 0);
      c1 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a8, b16, c1, idx, 0, 0);
      c2 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a8, b16, c2, idx, 0, 0);
      c3 = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(a8, b16, c3, idx, 0, 0);
    } else {
      bf16x8 b8 = __builtin_shufflevector(b16, b16, 0, 1, 2, 3, 4, 5, 6, 7);
      c0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a8, b8, c3, 0, 0, 0);
    }
  }
  float s = 0.f;
  for (int i = 0; i < 16; ++i) s += c0[i] + c1[i] + c2[i] + c3[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

// logical K index held by lane l in slot j (0..15) under layout hypothesis h
static int kmap(int h, int l, int j) {
  if (h == 0) return (l / 32) * 16 + j;                    // contiguous 16 per lane half
  return (j / 8) * 16 + (l / 32) * 8 + (j % 8);            // two 8-wide halves interleaved
}

int main() {
  srand(1234);
  const int M = 32, N = 32, K = 32;
  // logical sparse A: every aligned 4-group along K has exactly two nonzeros at i0 < i1
  std::vector<float> A(M * K, 0.f), B(K * N);
  std::vector<int> nzpos(M * K / 4 * 2);
  for (int m = 0; m < M; ++m)
    for (int g = 0; g < K / 4; ++g) {
      int i0 = rand() % 4, i1;
      do i1 = rand() % 4; while (i1 == i0);
      if (i0 > i1) std::swap(i0, i1);
      A[m * K + g * 4 + i0] = bf2f(f2bf((rand() % 17 - 8) / 4.f));
      A[m * K + g * 4 + i1] = bf2f(f2bf((rand() % 17 - 8) / 4.f));
      nzpos[(m * K / 4 + g) * 2] = i0;
      nzpos[(m * K / 4 + g) * 2 + 1] = i1;
    }
  for (auto& x : B) x = bf2f(f2bf((rand() % 17 - 8) / 8.f));
  std::vector<float> Dref(M * N, 0.f);
  for (int m = 0; m < M; ++m)
    for (int n = 0; n < N; ++n) {
      float s = 0;
      for (int k = 0; k < K; ++k) s += A[m * K + k] * B[k * N + n];
      Dref[m * N + n] = s;
    }
  uint16_t *da, *db;
  uint32_t* di;
  float* dd;
  CK(hipMalloc(&da, 64 * 8 * 2));
  CK(hipMalloc(&db, 64 * 16 * 2));
  CK(hipMalloc(&di, 64 * 4));
  CK(hipMalloc(&dd, 64 * 16 * 4));
  int found = 0;
  // Measured with tools/smfmac_layout.hip: B lane l holds K (l/32)*16 + j (contiguous); the A lane's
  // 4 groups sit at K {8h..8h+7} U {16+8h..16+8h+7}, h = l/32 (the interleaved map).
  for (int h = 0; h < 2; ++h)
    for (int abid = 0; abid < 2; ++abid) {
      std::vector<uint16_t> ha(64 * 8), hb(64 * 16);
      std::vector<uint32_t> hi(64, 0);
      for (int l = 0; l < 64; ++l) {
        const int m = l % 32, n = l % 32;
        for (int j = 0; j < 16; ++j) hb[l * 16 + j] = f2bf(B[kmap(0, l, j) * N + n]);
        // the lane's 16 logical K (4 groups) -> 8 compressed values + 8 two-bit indices
        for (int g = 0; g < 4; ++g) {
          const int k0 = kmap(h, l, g * 4);  // first K of the group (groups stay 4-aligned in both maps)
          const int gg = k0 / 4;
          for (int t = 0; t < 2; ++t) {
            const int p = nzpos[(m * K / 4 + gg) * 2 + t];
            ha[l * 8 + g * 2 + t] = f2bf(A[m * K + k0 + p]);
            hi[l] |= (uint32_t)p << ((g * 2 + t) * 2 + abid * 16);
          }
        }
      }
      CK(hipMemcpy(da, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(db, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
      CK(hipMemcpy(di, hi.data(), hi.size() * 4, hipMemcpyHostToDevice));
      hipLaunchKernelGGL(sparse_once, dim3(1), dim3(64), 0, 0, da, db, di, dd, abid);
      CK(hipGetLastError());
      std::vector<float> hd(64 * 16);
      CK(hipMemcpy(hd.data(), dd, hd.size() * 4, hipMemcpyDeviceToHost));
      double err = 0, ref = 0;
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 16; ++i) {
          const int n = l % 32, m = (i / 4) * 8 + (l / 32) * 4 + i % 4;
          err = fmax(err, fabs(hd[l * 16 + i] - Dref[m * N + n]));
          ref = fmax(ref, fabs(Dref[m * N + n]));
        }
      printf("A layout h%d (B contiguous) abid%d: max|err| %.3g (max|ref| %.3g) %s\n", h, abid, err, ref,
             err < 1e-3 * ref ? "MATCH" : "mismatch");
      found += err < 1e-3 * ref;
    }
  // issue rate: 256 CUs x 8 waves, 4 independent accumulator chains per wave
  float* dout;
  const int blocks = 256 * 2, iters = 4096;
  CK(hipMalloc(&dout, blocks * 256 * 4));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int s = 0; s < 2; ++s) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipEventRecord(e0));
      if (s) hipLaunchKernelGGL(rate<true>, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
      else hipLaunchKernelGGL(rate<false>, dim3(blocks), dim3(256), 0, 0, dout, iters, 1u);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double instr = (double)blocks * 4 * iters * 4;  // waves * chains * iters
      const double kdim = s ? 32 : 16;
      if (rep)
        printf("%s: %.3f ms, %.1f instr/us, %.0f logical TFLOP/s (%.0f TFLOP/s of nonzero MACs)\n",
               s ? "smfmac_f32_32x32x32_bf16" : "mfma_f32_32x32x16_bf16  ", ms, instr / ms / 1e3,
               instr * 2 * 32 * 32 * kdim / ms / 1e9, instr * 2 * 32 * 32 * 16 / ms / 1e9);
    }
  }
  printf("layout hypotheses matched: %d\n", found);
  return 0;
}
