// Host-visible launcher declarations for the gfx950 kernels.
// Included by the HIP translation units and by bindings.cpp (host-only).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

#include <cstdlib>

// Runtime A/B switch of a measured alternative (deconv_api_amd/knobs.py ABLATION): the variable is read
// only when DV_ABLATIONS=1, so a serving / benchmark process takes one dispatch per shape whatever its
// environment holds; tools/*_ab.py and the variant tests set DV_ABLATIONS=1. (Host code only.)
static inline const char* dv_ab_env(const char* name) {
  const char* on = std::getenv("DV_ABLATIONS");
  return (on != nullptr && on[0] == '1' && on[1] == 0) ? std::getenv(name) : nullptr;
}

namespace dv {

// A-operand (implicit-GEMM gather) modes of the conv kernel.
enum ConvAMode : int {
  CONV_A_FWD = 0,        // x[n][oh*s-p+kh][ow*s-p+kw][c]
  CONV_A_UNPOOL = 1,     // max-unpool gather: x is pooled (H/2 x W/2), switch codes select
  CONV_A_TRANSPOSE = 2,  // transposed conv (dgrad of a strided conv): ih=(oh+p-kh)/s when divisible
};
// Epilogues.
enum ConvEpi : int {
  CONV_E_BF16 = 0,  // (+bias)(ReLU)(+=out) -> bf16
  CONV_E_POOL = 1,  // (+bias)(ReLU) -> fused 2x2/s2 max-pool, bf16 pooled + uint8 switch code
  CONV_E_F32 = 2,   // (+bias)(ReLU)(+=out) -> fp32
};

// 16-bit storage dtypes (ConvArgs::dtype, pool_launch)
enum { DT_BF16 = 0, DT_F16 = 1 };

struct ConvArgs {
  const uint16_t* x;      // NHWC bf16 input (pooled map in UNPOOL mode, dy in TRANSPOSE mode)
  long long x_ld;         // elements between consecutive pixels of x (>= C; concat slices)
  const uint16_t* mask;   // optional: zero A elements where mask <= 0 (backward through ReLU)
  long long mask_ld;
  const uint8_t* code;    // UNPOOL: switch codes [N/code_div][H/2][W/2][C]
  int code_div;
  const uint16_t* w;      // packed weights [OCpad][Kpad] bf16, K index = (kh*KW+kw)*C + c
  const float* bias;      // [OCpad] fp32 or nullptr
  void* out;              // bf16 or fp32 output, row stride out_ld elements
  long long out_ld;
  uint8_t* out_code;      // POOL: switch codes [M/4][OC]
  int N, H, W, C;         // conv input geometry (UNPOOL: the unpooled H, W)
  int OH, OW, OC, OCpad;
  int KH, KW, stride, pad_h, pad_w;
  int K, Kpad;
  int M;                  // GEMM rows = N*OH*OW
  int m_base;             // LDS-DMA / KW3 launches: first GEMM row of tile 0 (a tail launch after a
                          //   full-round one, conv_dma_impl.h:kw3_split); 0 otherwise
  int relu, relu_in, accumulate;
  int dtype;              // 16-bit storage dtype of x/w/mask/16-bit out: 0 bf16, 1 fp16
  const uint16_t* res;    // optional residual (LDS-DMA FWD, 16-bit out): out = [ReLU](acc + bias + res)
  long long res_ld;
  const uint16_t* emask;  // optional (16-bit out): out = 0 where emask <= 0 (same layout as out)
  long long emask_ld;
  int vec_epi;            // host-checked: 16-bit out/res/emask rows 16-B aligned -> LDS-staged epilogue
  int epi_batch;          // LDS-staged epilogue: load every chunk's res/acc/emask operands up front
  float* ws;              // split-K: fp32 partials [ksplit][M][OCpad] (LDS-DMA kernel), else nullptr
  int ksplit;
  double* stats;          // optional (row-streaming kernel): stats[n / stats_div] += {sum out, sum out^2}
  int stats_div;
  const uint8_t* ucode;   // optional (LDS-DMA, vector epilogue): max-unpool the output with these switch
  int ucode_div;          //   codes [N/ucode_div][OH][OW][OC]; out is then [N][2 OH][2 OW] rows of out_ld
  // storage extents in elements from each base pointer (bindings.cpp: storage bytes past the data
  // pointer); read only by the DV_DEBUG bounds checks (common.h DV_BOUNDS)
  long long x_elems, out_elems, res_elems, emask_elems;
  int relu_cols;          // > 0: ReLU only on output columns < relu_cols (merged GEMMs whose trailing
                          //   columns are pre-activation values, ops/inception.py); 0: every column
  void* out2;             // optional (LDS-staged 16-bit epilogue, plain): columns >= split_col go to
  long long out2_ld;      //   out2[row * out2_ld + col - split_col] instead of out (a merged GEMM whose
  int split_col;          //   leading columns are one consumer's output and the rest another's)
  long long out2_elems;
  const uint16_t* w2;     // optional second-GEMM weights of a fused epilogue (conv3x3_unpool_z_launch: the
                          //   next conv-down's taps as a [32][64] matrix, row tap*3+c = W[c][tap][:])
  int pool_t;             // host-checked (POOL epilogue): OC, out_ld % 4 == 0, out 8-B / out_code 4-B aligned ->
                          //   the transposed pooled-max epilogue (conv_dma_impl.h:epilogue_pool_t)
  float* skw;             // optional: KW3P stream-K workspace, kSkSlotFloats fp32 per workgroup (partial tiles)
  unsigned* skflag;       //   + one ready flag per workgroup; zeroed by the launcher before each launch
  int skslots;            //   workspace slots (workgroups) allocated: the launch needs G <= skslots
  unsigned* skerr;        //   host-coherent counter of hand-offs that timed out (bindings.cpp sk_errors())
  // 1-bit ReLU masks (LDS-staged epilogue only; host: OC % 8 == 0): bit c % 8 of byte c / 8 of row m.
  // obits: written with the output, bit = (stored 16-bit value > 0); ebits: replaces emask (read 1/16
  // of its bytes). The launcher sets them only on kernels whose epilogue is epilogue_lds (conv_pw).
  uint8_t* obits;
  long long obits_ld;     // bytes per row
  const uint8_t* ebits;
  long long ebits_ld;
  // fused stem (conv3x3_stem_pool_launch): the first conv's packed weights are w2 ([64][kpad2], K index
  // tap * 8 + c of the 8-channel RGB input) and its fp32 bias bias2
  const float* bias2;
  int kpad2;
};
// KW3P stream-K: fp32 partial-tile slot per workgroup (BM x BN = 65536 for both KW3P tile shapes)
constexpr long long kSkSlotFloats = 256LL * 256LL;
constexpr int kSkMaxWg = 1024;

// grouped LDS-DMA launch of up to kGroupMax independent problems (conv_dma.hip:conv_dma_group_launch)
constexpr int kGroupMax = 4;
struct ConvGroup {
  ConvArgs p[kGroupMax];
  int start[kGroupMax + 1];  // first workgroup of each problem (prefix sums of the tile counts)
  int tiles_n[kGroupMax];
  int n;
};

int conv_igemm_launch(const ConvArgs& a, int amode, int epi, hipStream_t stream);
// LDS-DMA variant (FWD / TRANSPOSE, no mask): 8-wave 128x64-per-wave tiles
int conv_dma_launch(const ConvArgs& a, int amode, int epi, hipStream_t stream);
// split-K planning (1 = none) and the reduction epilogue (bias, ReLU, 16-bit / fp32 out)
int conv_dma_splitk(const ConvArgs& a);
// tuning override: force DMA tile config cfg (> 0, conv_dma.hip:dma_forced) and split-K ks (> 0); 0 = auto
void conv_dma_tune(int cfg, int ks);
int splitk_reduce_launch(const ConvArgs& a, int epi, hipStream_t stream);
// tile config a grouped launch of ``a`` would use (conv_dma.hip), 0 = not groupable; and the launch
// of 1..kGroupMax problems that share it (same dtype, A mode, epilogue and config; no split-K)
int conv_dma_group_cfg(const ConvArgs& a, int amode, int epi);
int conv_dma_group_launch(const ConvArgs* ps, int n, int amode, int epi, hipStream_t stream);
// direct VALU kernels for InceptionV3's conv2d_1 (8-ch padded RGB -> 32, 3x3 / stride 2): forward and
// input gradient (conv_stem.hip); < 0: unsupported geometry
int stem_conv_fwd_launch(const uint16_t* x, const float* w, const float* bias, uint16_t* y, int N, int H, int W,
                         int OH, int OW, int C, int cr, int cout, int k, int stride, int pad, int relu, long long x_ld,
                         long long y_ld, int dtype, hipStream_t s);
int stem_conv_dgrad_launch(const uint16_t* gy, const float* w, uint16_t* gx, int N, int H, int W, int OH, int OW,
                           int C, int cr, int cout, int k, int stride, int pad, long long gy_ld, long long gx_ld,
                           int dtype, hipStream_t s);
// persistent pointwise (1x1 / s1 / p0) conv at large M, 16-bit LDS-staged epilogue (conv_pw.hip);
// < 0: unsupported shape / mode (use conv_dma_launch)
int conv_pw_launch(const ConvArgs& a, hipStream_t stream);

// ---- misc kernels (misc.hip) ----
// per-(image, channel) sums of a NHWC bf16 / fp16 (f16 = 1) tensor: sums[n][c] = sum_{hw} x[n][hw][c]
int channel_sum_launch(const uint16_t* x, float* sums, int N, int HW, int C, int f16, hipStream_t s);
// per-row stable top-k of positive values: idx[n][k] (-1 when fewer than k positives)
int topk_pos_launch(const float* v, int* idx, float* val, int N, int C, int k, hipStream_t s);
// one-channel seeded deconv: out[b][h][w][ci] = relu(sum_taps S[b][h+kh-1][w+kw-1] * wt[f_b][kh][kw][ci])
int seed_deconv3x3_launch(const float* S, const int* f, const uint16_t* wt, uint16_t* out,
                          int B, int H, int W, int Cin, int F, int f16, hipStream_t s);
// fp32 recon [B*4][224][224][3] -> u8 mosaic [B][448][448][3] (channel-reversed), Keras deprocess
int deprocess_mosaic_launch(const float* recon, uint8_t* out, int B, int H, int W, int tiles,
                            int reverse_channels, hipStream_t s);
// per-group {sum, sum of squares} (fp64, atomically ADDED to stats[g][2]) of fp32 data [groups][per_group]
int recon_stats_launch(const float* x, double* stats, long long per_group, int groups, hipStream_t s);
// deprocess with precomputed per-image stats (single pass, 4 px per thread); W % 4 == 0
int deprocess_apply_launch(const float* recon, const double* stats, uint8_t* out, int B, int H, int W, int tiles,
                           int reverse_channels, hipStream_t s);
// uint8 [B][Hs][Ws][3] RGB -> bf16 / fp16 (f16 = 1) NHWC [B][OH][OW][Cpad]: cv2 INTER_LINEAR resize +
// caffe mean subtract
int resize_preprocess_launch(const uint8_t* img, int B, int Hs, int Ws, uint16_t* out, int OH, int OW,
                             int Cpad, int mode, int f16, hipStream_t s);
// fmt: 0 bf16 preprocessed, 1 u8 resized RGB, 2 fp16 preprocessed
int resize_batch_launch(const uint8_t* blob, const long long* table, int B, void* out, int OH, int OW, int Cpad,
                        int fmt, hipStream_t s);
int preprocess_u8_launch(const uint8_t* in, uint16_t* out, long long P, int Cpad, int f16, hipStream_t s);
// standalone 2x2/s2 max pool with switch codes, and its inverse (unpool scatter to full res)
int maxpool2x2_launch(const uint16_t* x, uint16_t* out, uint8_t* code, int N, int H, int W, int C,
                      int f16, hipStream_t s);
// seed maps of the deconvnet's B*K chains (all / max mode, optional max-unpool for pool targets)
int seed_map_launch(const uint16_t* out4, const int* idx, const uint8_t* code, float* S, int BK, int K, int H, int W,
                    int C, int mode, int f16, hipStream_t s);
int unpool2x2_launch(const uint16_t* p, const uint8_t* code, uint16_t* out, int N, int H, int W,
                     int C, int code_div, int relu, hipStream_t s);

}  // namespace dv

namespace dv {
// k x k pooling (pool.hip). kind 0 max (idx = uint8 window position), 1 avg (count_include_pad=0);
// dir 0 forward (in = x [N,H,W,C], out = y [N,OH,OW,C]), 1 backward (in = gy, out = gx)
// strided-conv input gradient from its s x s (s <= 2) parity-class parts [N, hc, wc, ld] (nullptr: zero class),
// optional accumulate into gx and emask (zero where emask <= 0)
int subpixel_merge_launch(const uint16_t* const* p, const int* hc, const int* wc, const int* ld, const uint16_t* emask,
                          uint16_t* gx, int N, int H, int W, int C, int s, int acc, int dtype, hipStream_t st);
int subpixel_scatter_launch(const uint16_t* E, const uint16_t* emask, uint16_t* gx, int N, int H, int W, int C, int OH,
                            int OW, int s, int dtype, hipStream_t st);
int pool_launch(int kind, int dir, const uint16_t* in, uint16_t* out, uint8_t* idx, int N, int H, int W, int C,
                int OH, int OW, int k, int s, int pad, int dtype, hipStream_t st, long long x_ld = 0,
                long long y_ld = 0, const float* bias = nullptr, int relu = 0, int acc = 0);
// DeepDream loss: per-(image, block) partial sums of x^2 over the map minus a b-pixel border
// (part [N][parts]), and its gradient gx = 2*scale[n]*x in the core, 0 on the border
// fused DeepDream update: per-image mean |g| partials, loss from the sumsq partials, device-side
// max_loss flag, x += step * g / mean|g| (fp32) and the next 16-bit network input (8 channels)
int dream_update_launch(const uint16_t* g, float* x, uint16_t* xin, float* gpart, int gparts, const float* lpart,
                        const float* lcoef, int L, int lparts, uint8_t* done, float* loss, float step, float max_loss,
                        int N, int H, int W, int dtype, hipStream_t s);
// DeepDream octave transition: y = corner-aligned bilinear resize of (a + b - c) (fp32 NHWC, 3 channels; b, c may
// be null), optionally also written as the 16-bit 8-channel network input yin
int octave_resize_launch(const float* a, const float* b, const float* c, float* y, uint16_t* yin, int N, int Hs, int Ws, int Hd, int Wd,
                         int dtype, hipStream_t s);
// tiled DeepDream step: rolled tile gather -> owned-pixel pack (+ unit loss / sum|g| tail) ->
// [all-gather of packs over ranks] -> update of the fp32 image straight from the packs
int tile_gather_launch(const float* x, uint16_t* xin, const int* plan, const int* shift, int units, int rank, int world,
                       int k0, int H, int W, int Th, int Tw, int dtype, hipStream_t s);
int tile_pack_launch(const uint16_t* g, uint16_t* pack, const int* plan, const float* lpart, const float* lcoef, int L,
                     int lparts, int units, int ucap, int rank, int world, int k0, int Th, int Tw, int dtype, hipStream_t s);
long long tile_pack_elems(int ucap, int Th, int Tw);  // 16-bit elements of one rank's pack
// packs: [chunks][world][pack_elems], units_per_rank = units per rank and chunk (dream.hip:tile_update_kernel)
int tile_update_launch(const uint16_t* packs, long long pack_elems, int units_per_rank, const int* plan, int nunits,
                       const int* shift, float* x, uint8_t* done, float* loss, float step, float max_loss, int world,
                       int H, int W, int Th, int Tw, int dtype, hipStream_t s);
int sumsq_core_launch(const uint16_t* x, float* part, int parts, int N, int H, int W, int C, int b, int dtype,
                      hipStream_t s);
int sumsq_core_bwd_launch(const uint16_t* x, const float* scale, const uint16_t* addend, uint16_t* gx, int N, int H, int W, int C, int b,
                          int dtype, hipStream_t s);
// sumsq_core_bwd + the forward partials (part [N][parts], as sumsq_core) in one pass
int sumsq_core_fused_launch(const uint16_t* x, const float* scale, const uint16_t* addend, uint16_t* gx, float* part,
                            int parts, int N, int H, int W, int C, int b, int dtype, hipStream_t s);
// col2im of a strided conv's input gradient for <= 8 input channels (output padded to 8 channels)
struct Col2ImGeom {
  int N, H, W, OH, OW, KH, KW, stride, pad_h, pad_w, Cr, J_ld;
};
int col2im_launch(const uint16_t* cols, uint16_t* gx, const Col2ImGeom& g, int dtype, hipStream_t s);
// fused GEMM + col2im input gradient of ResNet-50's conv1 (conv_stem_dgrad.hip): dy [N,OH,OW,C],
// optional ReLU mask like dy, wb = the cols GEMM's B^T [w_rows][w_ld] (row (kh*KW+kw)*Cr+c),
// gx [N,H,W,8]; < 0: geometry not covered
struct StemDgradGeom {
  int N, H, W, OH, OW, C, KH, KW, stride, pad, Cr, w_rows, w_ld;
};
// ResNet-50 conv1 forward (7x7 / 2, pad 3, RGB -> 64) on the tap-paired MFMA kernel (conv_stem7.hip);
// < 0: not its geometry
int stem7_fwd_launch(const uint16_t* x, const uint16_t* w, const float* bias, uint16_t* y, int N, int H, int W, int OH,
                     int OW, int relu, int dtype, hipStream_t s);
int stem_dgrad_fused_launch(const uint16_t* gy, const uint16_t* mask, const uint16_t* wb, uint16_t* gx,
                            const StemDgradGeom& g, int dtype, hipStream_t s);
// GPU baseline JPEG encode of B same-size RGB images (jpeg_gpu.hip): entropy-coded scans (restart
// marker after every MCU row, no header/EOI) packed back to back into `packed` at off[0..B];
// `tables` = a device copy of dvjpeg::GpuTables, `ws` = jpeg_gpu_ws_bytes(B, H, W) of workspace,
// `packed` >= B * jpeg_gpu_out_cap(H, W) bytes; W <= jpeg_gpu_max_width()
long long jpeg_gpu_ws_bytes(int B, int H, int W);
long long jpeg_gpu_out_cap(int H, int W);
int jpeg_gpu_max_width();
int jpeg_gpu_launch(const uint8_t* rgb, int B, int H, int W, const void* tables, void* ws, uint8_t* packed,
                    long long* off, hipStream_t s);
// row softmax (fp32 [M][N])
int softmax_rows_launch(const float* x, float* y, int M, int N, hipStream_t s);
// bench.py --emulate-rccl-world: `channels` workgroups copy `bytes` (src repeated) paced to `gbs` GB/s (misc.hip)
int paced_copy_launch(const void* src, long long src_bytes, void* dst, long long bytes, int channels, double gbs,
                      hipStream_t s);
// halo-tile 3x3/s1/p1 conv for OC tiles of 16/64 at large spatial sizes (optional fused unpool)
int conv3x3_halo_launch(const ConvArgs& a, int unpool, int epi, hipStream_t s, bool* stats_done = nullptr);
// 3x3 conv 64 -> 64 + bias + ReLU + fused 2x2 max-pool/switch (bf16); < 0 if the shape is unsupported
int conv3x3_pool_v3_launch(const ConvArgs& a, hipStream_t s);
// unpool + 3x3 conv 64 -> 64 (ReLU) whose epilogue multiplies the tile by a.w2 ([32][64]): writes the
// per-tap partial products Z [N, H, W, 32] (bf16, out_ld 32) of the following 64 -> 3 conv-down
int conv3x3_unpool_z_launch(const ConvArgs& a, hipStream_t s);
// out[n, y, x, c] = ReLU(sum_taps Z[n, y+kh-1, x+kw-1, (kh*3+kw)*3 + c]) fp32 [N, H, W, 3] + optional
// per-image {sum, sum^2} (fp64, image n / stats_div): the 3x3 shift-add that finishes a Z map
int zsum3x3_launch(const uint16_t* z, float* out, int N, int H, int W, double* stats, int stats_div, hipStream_t s);
// first layer: 3x3 conv of an 8-channel image -> <= 64 channels, bias + ReLU, bf16 (< 0: unsupported)
int conv3x3_c8_stream_launch(const ConvArgs& a, hipStream_t s);
// fused VGG16 stem: 3x3 conv 8 (RGB) -> 64 + ReLU (weights a.w2 / a.bias2), 3x3 conv 64 -> 64 + ReLU
// (a.w / a.bias) and the 2x2 max-pool with switches, one hs16 launch; the 64-channel map between the two
// convs lives only in LDS (conv_halo_stream.hip; < 0: unsupported)
int conv3x3_stem_pool_launch(const ConvArgs& a, hipStream_t s);
// halo-stream 3x3 s1 p1 conv, C % 32 == 0 -> OCpad 64 / 128, 16-bit out or fused 2x2 max-pool +
// switch (epi CONV_E_BF16 / CONV_E_POOL; < 0: unsupported)
int conv3x3_hs_launch(const ConvArgs& a, int epi, hipStream_t s, bool* lepi_used = nullptr);
}  // namespace dv
