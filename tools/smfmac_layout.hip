// Layout discovery for v_smfmac_f32_32x32x32_bf16 (see tools/smfmac_probe.hip): one-hot compressed A
// (lane la, slot sa, sparsity index p), B tagged with its lane (run 0) or slot (run 1); prints which
// output row lights up and which B element (lane, slot) it selected.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(16))) __bf16 bf16x16;
typedef __attribute__((ext_vector_type(16))) float f32x16;
__global__ void once(const float* a, const float* b, const int* idx, float* d) {
  const int l = threadIdx.x;
  bf16x8 av;
  bf16x16 bv;
  for (int j = 0; j < 8; ++j) av[j] = (__bf16)a[l * 8 + j];
  for (int j = 0; j < 16; ++j) bv[j] = (__bf16)b[l * 16 + j];
  f32x16 c = {};
  c = __builtin_amdgcn_smfmac_f32_32x32x32_bf16(av, bv, c, idx[l], 0, 0);
  for (int i = 0; i < 16; ++i) d[l * 16 + i] = c[i];
}
int main() {
  float *da, *db, *dd;
  int* di;
  hipMalloc(&da, 64 * 8 * 4); hipMalloc(&db, 64 * 16 * 4); hipMalloc(&dd, 64 * 16 * 4); hipMalloc(&di, 64 * 4);
  const int lanes[3] = {0, 5, 37};
  for (int li = 0; li < 3; ++li)
    for (int sa = 0; sa < 8; ++sa)
      for (int p = 0; p < 4; ++p) {
        int res[2][4];  // per run: row, col-lane, value
        int nnz[2];
        for (int run = 0; run < 2; ++run) {
          std::vector<float> a(64 * 8, 0.f), b(64 * 16), d(64 * 16);
          std::vector<int> idx(64, 0);
          a[lanes[li] * 8 + sa] = 1.f;
          idx[lanes[li]] = (int)(p * 0x55555555u);  // same index in every 2-bit field
          for (int l = 0; l < 64; ++l)
            for (int j = 0; j < 16; ++j) b[l * 16 + j] = run == 0 ? (float)(l + 1) : (float)(j + 1);
          hipMemcpy(da, a.data(), a.size() * 4, hipMemcpyHostToDevice);
          hipMemcpy(db, b.data(), b.size() * 4, hipMemcpyHostToDevice);
          hipMemcpy(di, idx.data(), idx.size() * 4, hipMemcpyHostToDevice);
          hipLaunchKernelGGL(once, dim3(1), dim3(64), 0, 0, da, db, di, dd);
          hipMemcpy(d.data(), dd, d.size() * 4, hipMemcpyDeviceToHost);
          nnz[run] = 0;
          res[run][0] = res[run][1] = res[run][2] = -1;
          for (int l = 0; l < 64; ++l)
            for (int i = 0; i < 16; ++i)
              if (d[l * 16 + i] != 0.f) {
                if (nnz[run] == 0 || (l % 32) == 0) {
                  res[run][0] = l; res[run][1] = i; res[run][2] = (int)d[l * 16 + i];
                }
                ++nnz[run];
              }
        }
        // with C layout lane=col+32*g, reg i: row=(i/4)*8+g*4+i%4
        const int l = res[0][0], i = res[0][1];
        const int row = l < 0 ? -1 : (i / 4) * 8 + (l / 32) * 4 + i % 4;
        printf("A lane %2d slot %d p %d -> nnz %d/%d row %2d | B lane %2d (col0 lane) slot %2d\n", lanes[li], sa, p,
               nnz[0], nnz[1], row, res[0][2] - 1, res[1][2] - 1);
      }
  return 0;
}
