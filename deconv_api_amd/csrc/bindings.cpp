// torch bindings for the gfx950 kernels. Host-only translation unit: validates shapes and
// storage extents (an out-of-bounds kernel access can take down the whole GPU node), then
// calls the raw launchers on the current HIP stream (so torch.cuda graphs capture them).
#include <torch/extension.h>
#include <ATen/hip/impl/HIPGuardImplMasqueradingAsCUDA.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>

#include "jpeg_enc.h"
#include "kernels.h"

#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <optional>

namespace {

using at::Tensor;

// torch-ROCm exposes HIP devices as device type "cuda": use the masquerading guard/stream
hipStream_t cur_stream() { return c10::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

void check_cuda(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
}

// bytes from t.data_ptr() to the end of its storage
int64_t avail_bytes(const Tensor& t) {
  const int64_t total = (int64_t)t.storage().nbytes();
  return total - t.storage_offset() * (int64_t)t.element_size();
}

void need(const Tensor& t, int64_t bytes, const char* name) {
  TORCH_CHECK(bytes <= avail_bytes(t), name, ": kernel would read/write ", bytes, " bytes but only ",
              avail_bytes(t), " are available");
}

static bool is16(const Tensor& t) { return t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf; }
static int f16(const Tensor& t) { return t.scalar_type() == at::kHalf ? 1 : 0; }

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " launch failed with code ", rc);
}

// Grouped launches (conv_group_begin / conv_group_end): between the two calls every conv that would
// run on the LDS-DMA kernel with a groupable small-problem tile config (dv::conv_dma_group_cfg) is
// recorded instead of launched; the end call launches the recorded problems as grouped kernels of up
// to kGroupMax problems per (A mode, epilogue, config, dtype), in recording order. The caller
// guarantees the recorded convs are independent (no one reads what another writes) and keeps their
// tensors alive until the end call (ops/conv.py:conv_group). One group per thread at a time.
struct PendingConv {
  dv::ConvArgs a;
  int amode, epi, cfg;
};
thread_local bool g_group_active = false;
thread_local bool g_group_paused = false;  // recording suspended: convs launch at once, in order
thread_local std::vector<PendingConv> g_group;

void conv_group_begin() {
  TORCH_CHECK(!g_group_active, "conv_group_begin: a group is already open on this thread");
  g_group_active = true;
  g_group.clear();
}

// returns the number of grouped kernel launches issued
int64_t conv_group_end() {
  TORCH_CHECK(g_group_active, "conv_group_end: no open group");
  g_group_active = false;
  g_group_paused = false;
  std::vector<PendingConv> pend;
  pend.swap(g_group);
  std::vector<bool> done(pend.size(), false);
  int64_t launches = 0;
  for (size_t i = 0; i < pend.size(); ++i) {
    if (done[i]) continue;
    dv::ConvArgs ps[dv::kGroupMax];
    int n = 0;
    for (size_t j = i; j < pend.size() && n < dv::kGroupMax; ++j) {
      if (done[j] || pend[j].amode != pend[i].amode || pend[j].epi != pend[i].epi || pend[j].cfg != pend[i].cfg ||
          pend[j].a.dtype != pend[i].a.dtype)
        continue;
      ps[n++] = pend[j].a;
      done[j] = true;
    }
    if (n == 1) {  // nothing to run beside it: the one-problem path, with its split-K planning
      dv::ConvArgs a = ps[0];
      const int ks = dv::conv_dma_splitk(a);
      Tensor ws;
      if (ks > 1) {
        int dev = 0;
        check_rc((int)hipGetDevice(&dev), "hipGetDevice");
        ws = at::empty({(int64_t)ks * a.M * a.OCpad}, at::TensorOptions().dtype(at::kFloat).device(at::kCUDA, dev));
        a.ws = ws.data_ptr<float>();
        a.ksplit = ks;
      }
      check_rc(dv::conv_dma_launch(a, pend[i].amode, pend[i].epi, cur_stream()), "conv_dma");
      if (ks > 1) check_rc(dv::splitk_reduce_launch(a, pend[i].epi, cur_stream()), "splitk_reduce");
    } else {
      check_rc(dv::conv_dma_group_launch(ps, n, pend[i].amode, pend[i].epi, cur_stream()), "conv_dma_group");
    }
    ++launches;
  }
  return launches;
}

// KW3P stream-K hand-off timeouts (conv_dma_impl.h): one process-wide counter in host-coherent pinned
// memory, written by the kernel with a system-scope atomic, read by the host without any copy or sync
static unsigned* sk_error_host() {
  static unsigned* p = [] {
    void* h = nullptr;
    check_rc((int)hipHostMalloc(&h, 64, hipHostMallocCoherent | hipHostMallocMapped), "hipHostMalloc(sk errors)");
    std::memset(h, 0, 64);
    return reinterpret_cast<unsigned*>(h);
  }();
  return p;
}
static unsigned* sk_error_counter() {
  unsigned* h = sk_error_host();
  void* d = nullptr;
  check_rc((int)hipHostGetDevicePointer(&d, h, 0), "hipHostGetDevicePointer(sk errors)");
  return reinterpret_cast<unsigned*>(d);
}
int64_t sk_errors(bool reset) {
  volatile unsigned* h = sk_error_host();
  const unsigned v = *h;
  if (reset) *h = 0u;
  return (int64_t)v;
}

// compute units of the current device (cached per device)
int64_t device_cus() {
  static std::mutex mu;
  static std::map<int, int64_t> cache;
  int dev = 0;
  check_rc((int)hipGetDevice(&dev), "hipGetDevice");
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find(dev);
  if (it != cache.end()) return it->second;
  int cu = 0;
  check_rc((int)hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev), "hipDeviceGetAttribute");
  return cache[dev] = cu > 0 ? cu : 256;
}

// geom: N,H,W,C, OH,OW,OC,OCpad, KH,KW,stride,pad_h,pad_w, K,Kpad, M, relu,relu_in,accumulate,
//       code_div, x_ld, mask_ld, out_ld
// Returns bit flags: 1 = obits written, 2 = ebits used (both only on the persistent 1x1 kernel; otherwise
// the caller's emask applies and obits stays unwritten).
int64_t conv(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor out, c10::optional<Tensor> out_code,
             c10::optional<Tensor> code, c10::optional<Tensor> mask, std::vector<int64_t> g, int64_t amode,
             int64_t epi, int64_t impl, c10::optional<Tensor> res, c10::optional<Tensor> emask,
             c10::optional<Tensor> stats, int64_t stats_div, c10::optional<Tensor> ucode, int64_t ucode_div,
             int64_t relu_cols, c10::optional<Tensor> out2, int64_t split_col, c10::optional<Tensor> obits,
             c10::optional<Tensor> ebits) {
  TORCH_CHECK(g.size() == 23, "conv: geometry vector must have 23 entries");
  check_cuda(x, "x");
  check_cuda(w, "w");
  check_cuda(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  dv::ConvArgs a{};
  a.N = (int)g[0]; a.H = (int)g[1]; a.W = (int)g[2]; a.C = (int)g[3];
  a.OH = (int)g[4]; a.OW = (int)g[5]; a.OC = (int)g[6]; a.OCpad = (int)g[7];
  a.KH = (int)g[8]; a.KW = (int)g[9]; a.stride = (int)g[10]; a.pad_h = (int)g[11]; a.pad_w = (int)g[12];
  a.K = (int)g[13]; a.Kpad = (int)g[14]; a.M = (int)g[15];
  a.relu = (int)g[16]; a.relu_in = (int)g[17]; a.accumulate = (int)g[18];
  a.code_div = (int)g[19]; a.x_ld = g[20]; a.mask_ld = g[21]; a.out_ld = g[22];
  a.relu_cols = (int)relu_cols;
  TORCH_CHECK(relu_cols == 0 || (impl == 2 && relu_cols > 0 && relu_cols <= a.OC && epi != dv::CONV_E_POOL),
              "conv: relu_cols needs the LDS-DMA kernel (impl 2) and 0 < relu_cols <= OC");

  const auto dt = x.scalar_type();
  TORCH_CHECK((dt == at::kBFloat16 || dt == at::kHalf) && w.scalar_type() == dt, "conv: x, w must both be bf16 or fp16");
  a.dtype = dt == at::kHalf ? dv::DT_F16 : dv::DT_BF16;
  // fp16 (DeepDream, Config.dtype = fp16): the bf16-only kernels (weight-resident halo, pool v3, c8 stream,
  // stem, tail) decline it and the launch lands on the dtype-generic DMA / halo-stream / pw kernels; an
  // unpool input is materialized by the (16-bit move) unpool2x2 first. A combination no kernel has raises.
  TORCH_CHECK(w.is_contiguous() && w.numel() == (int64_t)a.OCpad * a.Kpad, "conv: w must be [OCpad, Kpad]");
  TORCH_CHECK(a.K == a.KH * a.KW * a.C && a.Kpad >= a.K && a.Kpad % 64 == 0, "conv: bad K/Kpad");
  TORCH_CHECK(a.C % 8 == 0 && a.x_ld % 8 == 0 && a.x_ld >= a.C, "conv: C and x_ld must be multiples of 8");
  TORCH_CHECK(a.M == a.N * a.OH * a.OW && a.M > 0, "conv: M must be N*OH*OW");
  TORCH_CHECK(a.OC <= a.OCpad && a.stride >= 1 && a.code_div >= 1, "conv: bad OC/stride/code_div");
  TORCH_CHECK(reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(w.data_ptr()) % 16 == 0,
              "conv: x and w must be 16-byte aligned");
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  a.x_elems = avail_bytes(x) / 2;
  a.out_elems = avail_bytes(out) / (int64_t)out.element_size();

  // input extent
  int64_t in_pix = (int64_t)a.N * a.H * a.W;
  if (amode == dv::CONV_A_UNPOOL) {
    TORCH_CHECK(a.H % 2 == 0 && a.W % 2 == 0, "conv unpool: H, W must be even");
    in_pix = (int64_t)a.N * (a.H / 2) * (a.W / 2);
    TORCH_CHECK(code.has_value(), "conv unpool: code required");
    check_cuda(*code, "code");
    TORCH_CHECK(code->scalar_type() == at::kByte, "code must be uint8");
    TORCH_CHECK(a.N % a.code_div == 0, "conv unpool: N % code_div");
    need(*code, (int64_t)(a.N / a.code_div) * (a.H / 2) * (a.W / 2) * a.C, "code");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(code->data_ptr()) % 8 == 0, "code must be 8-byte aligned");
    a.code = reinterpret_cast<const uint8_t*>(code->data_ptr());
  }
  need(x, ((in_pix - 1) * a.x_ld + a.C) * 2, "x");
  if (mask.has_value()) {
    check_cuda(*mask, "mask");
    TORCH_CHECK(mask->scalar_type() == dt && a.mask_ld % 8 == 0, "mask must have x's dtype, ld%8");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(mask->data_ptr()) % 16 == 0, "mask must be 16-byte aligned");
    need(*mask, ((in_pix - 1) * a.mask_ld + a.C) * 2, "mask");
    a.mask = reinterpret_cast<const uint16_t*>(mask->data_ptr());
  }
  if (bias.has_value()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= a.OCpad, "bias must be fp32 [OCpad]");
    a.bias = bias->data_ptr<float>();
  }
  // output extent
  int64_t out_rows = ucode.has_value() ? 4 * (int64_t)a.M : a.M;
  if (epi == dv::CONV_E_POOL) {
    TORCH_CHECK(a.OH % 2 == 0 && a.OW % 2 == 0, "conv pool: OH, OW must be even");
    out_rows = a.M / 4;
    TORCH_CHECK(out_code.has_value(), "conv pool: out_code required");
    check_cuda(*out_code, "out_code");
    TORCH_CHECK(out_code->scalar_type() == at::kByte, "out_code must be uint8");
    need(*out_code, out_rows * a.OC, "out_code");
    a.out_code = reinterpret_cast<uint8_t*>(out_code->data_ptr());
    TORCH_CHECK(out.scalar_type() == dt, "pool out must have x's dtype");
    const bool no_pool_t = dv_ab_env("DV_NO_POOL_T") != nullptr;  // A/B: the per-element pool stores (per call)
    a.pool_t = !no_pool_t && a.OC % 4 == 0 && a.out_ld % 4 == 0 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 8 == 0 &&
               reinterpret_cast<uintptr_t>(a.out_code) % 4 == 0;
    // 2 (opt-in, DV_POOL_EPI=lds, per call): the LDS-staged pooled epilogue (whole 16-B value / code chunks
    // per lane). Measured equal to slightly slower than the transposed 8-B stores on config 2 (the pooled
    // output is a quarter of the conv's: 7478 / 7506 / 7547 vs 7504 / 7531 / 7549 img/s, same box,
    // alternating; profiles/bench_c2_r5_pool_epi_ab.txt)
    const char* pe = dv_ab_env("DV_POOL_EPI");
    if (a.pool_t && pe && std::strcmp(pe, "lds") == 0 && a.OC % 16 == 0 && a.out_ld % 8 == 0 &&
        reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(a.out_code) % 16 == 0)
      a.pool_t = 2;
  } else if (epi == dv::CONV_E_F32) {
    TORCH_CHECK(out.scalar_type() == at::kFloat, "f32 epilogue needs fp32 out");
  } else {
    TORCH_CHECK(out.scalar_type() == dt, "16-bit epilogue needs out of x's dtype");
  }
  // with out2 only the leading split_col channels land in out
  const int64_t out_cols = out2.has_value() ? std::min<int64_t>(split_col, a.OC) : a.OC;
  need(out, ((out_rows - 1) * a.out_ld + out_cols) * (int64_t)out.element_size(), "out");
  a.out = out.data_ptr();
  if (res.has_value()) {  // fused residual: LDS-DMA forward conv with a 16-bit output only
    check_cuda(*res, "res");
    TORCH_CHECK(res->scalar_type() == dt && res->dim() == 4 && res->stride(3) == 1, "res: x's dtype, NHWC");
    TORCH_CHECK(amode == dv::CONV_A_FWD && epi == dv::CONV_E_BF16 && !a.accumulate && impl != 1 && impl != 3 &&
                    (!mask.has_value() || a.mask_ld == a.x_ld),
                "res: forward conv with a 16-bit epilogue on the LDS-DMA kernel only");
    a.res_ld = res->stride(2);
    TORCH_CHECK(res->stride(1) == a.OW * a.res_ld && res->stride(0) == (int64_t)a.OH * a.OW * a.res_ld,
                "res: pixels must be dense");
    need(*res, ((int64_t)(a.M - 1) * a.res_ld + a.OC) * 2, "res");
    a.res = reinterpret_cast<const uint16_t*>(res->data_ptr());
    a.res_elems = avail_bytes(*res) / 2;
    if (emask.has_value()) {
      check_cuda(*emask, "emask");
      TORCH_CHECK(emask->scalar_type() == dt && emask->dim() == 4 && emask->stride(3) == 1, "emask: x's dtype, NHWC");
      a.emask_ld = emask->stride(2);
      TORCH_CHECK(emask->stride(1) == a.OW * a.emask_ld && emask->stride(0) == (int64_t)a.OH * a.OW * a.emask_ld,
                  "emask: pixels must be dense");
      need(*emask, ((int64_t)(a.M - 1) * a.emask_ld + a.OC) * 2, "emask");
      a.emask = reinterpret_cast<const uint16_t*>(emask->data_ptr());
      a.emask_elems = avail_bytes(*emask) / 2;
    }
  }
  if (emask.has_value() && a.emask == nullptr) {  // output mask without a residual
    check_cuda(*emask, "emask");
    TORCH_CHECK(emask->scalar_type() == dt && emask->dim() == 4 && emask->stride(3) == 1, "emask: x's dtype, NHWC");
    TORCH_CHECK(epi == dv::CONV_E_BF16 && impl != 1 && impl != 3, "emask: 16-bit epilogue on the LDS-DMA kernel only");
    a.emask_ld = emask->stride(2);
    TORCH_CHECK(emask->stride(1) == a.OW * a.emask_ld && emask->stride(0) == (int64_t)a.OH * a.OW * a.emask_ld,
                "emask: pixels must be dense");
    need(*emask, ((int64_t)(a.M - 1) * a.emask_ld + a.OC) * 2, "emask");
    a.emask = reinterpret_cast<const uint16_t*>(emask->data_ptr());
    a.emask_elems = avail_bytes(*emask) / 2;
  }
  if (out2.has_value()) {  // columns >= split_col to a second tensor (plain LDS-staged epilogue only)
    check_cuda(*out2, "out2");
    TORCH_CHECK(out2->scalar_type() == dt && out2->dim() == 4 && out2->stride(3) == 1 && epi == dv::CONV_E_BF16 &&
                    amode == dv::CONV_A_FWD && !a.accumulate && !res.has_value() && !emask.has_value() &&
                    !ucode.has_value() && !stats.has_value() && impl == 2 && split_col > 0 && split_col % 8 == 0 &&
                    split_col < a.OC && a.OC % 8 == 0,
                "conv out2: plain 16-bit forward on the LDS-DMA kernel, split_col % 8 == 0 < OC, OC % 8 == 0");
    a.out2_ld = out2->stride(2);
    TORCH_CHECK(out2->size(3) >= a.OC - split_col && out2->stride(1) == a.OW * a.out2_ld &&
                    out2->stride(0) == (int64_t)a.OH * a.OW * a.out2_ld && a.out2_ld % 8 == 0 &&
                    reinterpret_cast<uintptr_t>(out2->data_ptr()) % 16 == 0,
                "out2: dense pixels, 16-B aligned rows");
    need(*out2, ((int64_t)(a.M - 1) * a.out2_ld + (a.OC - split_col)) * 2, "out2");
    a.out2 = out2->data_ptr();
    a.out2_elems = avail_bytes(*out2) / 2;
    a.split_col = (int)split_col;
  }
  {  // LDS-staged vector epilogue: 16-bit rows (out / res / emask) 16-B aligned
    auto al = [](const void* p, int64_t ld) { return reinterpret_cast<uintptr_t>(p) % 16 == 0 && ld % 8 == 0; };
    a.vec_epi = epi == dv::CONV_E_BF16 && al(a.out, a.out_ld) && (!a.res || al(a.res, a.res_ld)) &&
                (!a.emask || al(a.emask, a.emask_ld)) && (dv_ab_env("DV_NO_VEC_EPI") == nullptr || a.out2);
    TORCH_CHECK(!a.out2 || a.vec_epi, "conv out2: 16-B aligned out rows (LDS-staged epilogue)");
    static const bool no_batch = dv_ab_env("DV_NO_EPI_BATCH") != nullptr;
    a.epi_batch = !no_batch;
  }
  if (ucode.has_value()) {  // max-unpooled output (the consumer of this conv reads the full-res map)
    check_cuda(*ucode, "ucode");
    TORCH_CHECK(ucode->scalar_type() == at::kByte && ucode_div >= 1 && a.N % ucode_div == 0,
                "ucode: uint8 switch codes, N % ucode_div == 0");
    TORCH_CHECK(epi == dv::CONV_E_BF16 && a.vec_epi && !a.res && !a.emask && !a.accumulate && a.OC % 8 == 0 &&
                    impl != 1 && impl != 3 && !stats.has_value(),
                "ucode: 16-bit LDS-staged epilogue of the LDS-DMA kernel (16-B aligned rows, OC % 8 == 0)");
    need(*ucode, (int64_t)(a.N / ucode_div) * a.OH * a.OW * a.OC, "ucode");
    TORCH_CHECK(reinterpret_cast<uintptr_t>(ucode->data_ptr()) % 8 == 0, "ucode must be 8-byte aligned");
    a.ucode = reinterpret_cast<const uint8_t*>(ucode->data_ptr());
    a.ucode_div = (int)ucode_div;
  }
  bool stats_done = false;
  if (stats.has_value()) {  // per-(image) {sum, sum^2} of the fp32 output for the single-pass deprocess
    check_cuda(*stats, "stats");
    TORCH_CHECK(epi == dv::CONV_E_F32 && stats->scalar_type() == at::kDouble && stats->is_contiguous() &&
                    stats_div >= 1 && a.N % stats_div == 0 && stats->numel() == 2 * (a.N / stats_div) &&
                    a.out_ld == a.OC,
                "conv stats: fp64 [N/stats_div, 2], fp32 dense output");
    check_rc((int)hipMemsetAsync(stats->data_ptr(), 0, stats->numel() * 8, cur_stream()), "stats memset");
    a.stats = stats->data_ptr<double>();
    a.stats_div = (int)stats_div;
  }
  // statistics the chosen kernel did not produce: one extra pass over the fp32 output
  auto finish_stats = [&]() {
    if (stats.has_value() && !stats_done)
      check_rc(dv::recon_stats_launch(reinterpret_cast<const float*>(a.out), a.stats,
                                      (long long)a.stats_div * a.OH * a.OW * a.OC, a.N / a.stats_div, cur_stream()),
               "recon_stats");
  };
  // 1-bit ReLU masks ([M, OC / 8] bytes, csrc/kernels.h): set on a COPY of the args handed to a kernel whose
  // epilogue honours them (the persistent 1x1 kernel, the halo-stream LDS-staged epilogues); returns the
  // flags to report if that kernel runs with them (every other path ignores obits / ebits: emask applies)
  auto with_bits = [&](dv::ConvArgs& ap) -> int64_t {
    int64_t f = 0;
    auto ok = [&](const Tensor& b) {
      check_cuda(b, "bits");
      return b.scalar_type() == at::kByte && b.is_contiguous() && a.OC % 8 == 0 && a.ucode == nullptr &&
             a.out2 == nullptr && a.out_ld == a.OC && b.numel() >= (int64_t)a.M * (a.OC / 8);
    };
    if (obits.has_value() && ok(*obits)) {
      ap.obits = obits->data_ptr<uint8_t>();
      ap.obits_ld = a.OC / 8;
      f |= 1;
    }
    if (ebits.has_value() && a.emask != nullptr && ok(*ebits)) {
      ap.ebits = ebits->data_ptr<uint8_t>();
      ap.ebits_ld = a.OC / 8;
      f |= 2;
    }
    return f;
  };
  // Kernel choice. impl: 0 auto, 1 register-staged (conv_igemm), 2 LDS-DMA (conv_dma), 3 halo-tile.
  //  * halo-tile (3x3 s1 p1, OC tile <= 64, >= 56x56 maps): input staged once per tile, unpool fused
  //  * LDS-DMA: FWD / TRANSPOSE (optionally ReLU-masked); an unpool input is first materialized
  //  * register-staged: everything else (mask with its own pixel stride, fused unpool gather)
  const bool halo_ok = (amode == dv::CONV_A_FWD || amode == dv::CONV_A_UNPOOL) && a.KH == 3 && a.KW == 3 &&
                       a.stride == 1 && a.pad_h == 1 && a.pad_w == 1 && a.C == 64 && a.H == a.OH &&
                       a.W == a.OW && !a.accumulate && !mask.has_value() && a.dtype == dv::DT_BF16 &&
                       (epi == dv::CONV_E_BF16 || epi == dv::CONV_E_F32) && (a.OC <= 16 || a.OCpad == 64) &&
                       a.res == nullptr && a.emask == nullptr && a.ucode == nullptr;
  // persistent weight-resident halo kernel: 64-channel inputs at large maps (block1 of VGG16)
  // the 16 x 16-tile halo-stream kernel (conv_halo_stream.hip) beats the weight-resident halo kernel
  // on plain 16-bit-output convs whose sides are multiples of 16 (measured on the pool variant:
  // VGG16 block1_conv2 fwd 1.28 -> 1.04 ms, profiles/layers_r1_ab{0,1}.txt)
  const bool hs16_ok = a.H % 16 == 0 && a.W % 16 == 0 && a.C % 32 == 0 && a.OC % 4 == 0 && !a.relu_in &&
                       (a.OCpad == 64 || a.OCpad == 128) && dv_ab_env("DV_NO_HS") == nullptr;
  const bool halo_auto = halo_ok && a.H * a.W >= 112 * 112 && a.res == nullptr && a.emask == nullptr &&
                         !(hs16_ok && amode == dv::CONV_A_FWD && epi == dv::CONV_E_BF16);
  // conv 64 -> 64 + fused 2x2 max-pool at large maps (VGG16 block1_conv2 forward): weight-resident
  // halo kernel with LDS-DMA staging and the pool in registers
  if (epi == dv::CONV_E_POOL && amode == dv::CONV_A_FWD && (impl == 0 || impl == 3) && a.H * a.W >= 112 * 112 &&
      !mask.has_value() && (impl == 3 || !hs16_ok)) {
    const int rc = dv::conv3x3_pool_v3_launch(a, cur_stream());
    if (rc >= 0) {
      check_rc(rc, "conv_pool_v3");
      finish_stats();
      return 0;
    }
  }
  // first layer (8-channel padded RGB image -> 64 channels): row-streaming, output-write bound
  if (epi == dv::CONV_E_BF16 && amode == dv::CONV_A_FWD && (impl == 0 || impl == 3) && a.C == 8 && !a.ucode &&
      !a.res && !a.emask && a.relu_cols <= 0 && a.H * a.W >= 56 * 56 && !mask.has_value() &&
      dv_ab_env("DV_NO_C8_STREAM") == nullptr) {
    const int rc = dv::conv3x3_c8_stream_launch(a, cur_stream());
    if (rc >= 0) {
      check_rc(rc, "conv_c8_stream");
      finish_stats();
      return 0;
    }
  }
  if (impl == 3 || (impl == 0 && halo_auto)) {
    TORCH_CHECK(halo_ok, "conv: halo-tile kernel does not support this shape/mode");
    check_rc(dv::conv3x3_halo_launch(a, amode == dv::CONV_A_UNPOOL ? 1 : 0, (int)epi, cur_stream(), &stats_done),
             "conv_halo");
    finish_stats();
    return 0;
  }
  // ReLU-masked A (dgrad): the DMA kernel stages the mask with x's offsets, so it needs mask_ld == x_ld
  const bool mask_dma = mask.has_value() && a.mask_ld == a.x_ld && epi == dv::CONV_E_BF16 &&
                        (amode == dv::CONV_A_FWD || amode == dv::CONV_A_TRANSPOSE);
  const bool dma_mode = ((amode == dv::CONV_A_FWD || amode == dv::CONV_A_UNPOOL ||
                          (amode == dv::CONV_A_TRANSPOSE && epi == dv::CONV_E_BF16)) && !mask.has_value()) ||
                        mask_dma;
  TORCH_CHECK(impl != 2 || dma_mode, "conv: LDS-DMA kernel does not support this mode");
  TORCH_CHECK(dma_mode || (a.res == nullptr && a.emask == nullptr && a.ucode == nullptr),
              "conv: res / emask / ucode need the LDS-DMA kernel");
  if (dma_mode && impl != 1) {
    Tensor unpooled;
    if (amode == dv::CONV_A_UNPOOL) {  // materialize the unpooled map, then a plain DMA conv
      TORCH_CHECK(a.x_ld == a.C, "conv unpool (split): pooled input must be channel-dense");
      unpooled = at::empty({a.N, a.H, a.W, a.C}, x.options());
      check_rc(dv::unpool2x2_launch(a.x, a.code, reinterpret_cast<uint16_t*>(unpooled.data_ptr()), a.N, a.H, a.W,
                                    a.C, a.code_div, a.relu_in, cur_stream()),
               "unpool2x2");
      a.x = reinterpret_cast<const uint16_t*>(unpooled.data_ptr());
      a.x_elems = unpooled.numel();
      a.x_ld = a.C;
      a.relu_in = 0;
      a.code = nullptr;
      amode = dv::CONV_A_FWD;
    }
    Tensor relu_x, dense_mask;
    if (a.relu_in) {  // the DMA kernel stages A verbatim: ReLU a dense copy first (the deconvnet passes
                      // relu_in = false for inputs that already are ReLU outputs and never takes this pass)
      const std::vector<int64_t> sz{a.N, a.H, a.W, a.C};
      const std::vector<int64_t> st{(int64_t)a.H * a.W * a.x_ld, (int64_t)a.W * a.x_ld, (int64_t)a.x_ld, 1};
      relu_x = at::relu(x.as_strided(sz, st));
      a.x = reinterpret_cast<const uint16_t*>(relu_x.data_ptr());
      a.x_elems = relu_x.numel();
      if (mask.has_value()) {  // the mask is staged with x's offsets: same dense layout
        dense_mask = mask->as_strided(sz, st).contiguous();
        a.mask = reinterpret_cast<const uint16_t*>(dense_mask.data_ptr());
        a.mask_ld = a.C;
      }
      a.x_ld = a.C;
      a.relu_in = 0;
    }
    // A/B switches: DV_HS_EMASK_OFF (masked dgrads back on the DMA kernel), DV_HS_PAD_OFF (pad != 1)
    static const bool hs_emask_off = dv_ab_env("DV_HS_EMASK_OFF") != nullptr;
    static const bool hs_pad_off = dv_ab_env("DV_HS_PAD_OFF") != nullptr;
    // smallest map side routed to the halo-stream kernels (DV_HS_MIN_W, default 64)
    static const int64_t hs_min_w = dv_ab_env("DV_HS_MIN_W") ? std::atoll(dv_ab_env("DV_HS_MIN_W")) : 64;
    // 3x3 s1 convs (pad 0..2) with 64/128 padded output channels at large maps: halo-stream kernel
    // (every input pixel fetched once per 32-channel chunk instead of once per tap); also the ReLU-
    // masked (emask) input gradients of such convs (InceptionV3 stem / ResNet 3x3 dgrads)
    if (impl == 0 && amode == dv::CONV_A_FWD && (epi == dv::CONV_E_BF16 || epi == dv::CONV_E_POOL) &&
        !mask.has_value() && !a.res && !a.ucode && !a.accumulate && a.relu_cols <= 0 &&
        (int64_t)a.H * a.W >= hs_min_w * hs_min_w && a.W >= hs_min_w && (!a.emask || !hs_emask_off) &&
        (a.pad_h == 1 || !hs_pad_off)) {
      dv::ConvArgs ap = a;
      const int64_t want = with_bits(ap);
      bool lepi = false;
      const int rc = dv::conv3x3_hs_launch(ap, (int)epi, cur_stream(), &lepi);
      if (rc >= 0) {
        check_rc(rc, "conv_halo_stream");
        finish_stats();
        return lepi ? want : 0;
      }
    }
    // the DMA kernel addresses A with 32-bit offsets relative to the tile's first image
    const int64_t imgs_per_tile = 512 / std::max(1, a.OH * a.OW) + 2;
    TORCH_CHECK((int64_t)a.H * a.W * a.x_ld * 2 * imgs_per_tile < 0x7FFFFFF0LL, "conv dma: image too large");
    if (g_group_active && !g_group_paused && (impl == 0 || impl == 2) && !mask.has_value() && !unpooled.defined() &&
        !relu_x.defined() && !a.ucode && !a.out2 && !stats.has_value()) {
      const int cfg = dv::conv_dma_group_cfg(a, (int)amode, (int)epi);
      if (cfg != 0) {  // recorded (no split-K: the group runs its problems side by side); launched by conv_group_end
        g_group.push_back(PendingConv{a, (int)amode, (int)epi, cfg});
        return 0;
      }
    }
    // split-K when the tile grid would leave most CUs idle (plain epilogues only)
    // (the reduce kernel applies bias / ReLU / accumulate / residual / emask; not the unpool scatter)
    const bool plain_epi = (epi == dv::CONV_E_BF16 || epi == dv::CONV_E_F32) && !a.ucode && !a.out2;
    const int ks = plain_epi ? dv::conv_dma_splitk(a) : 1;
    Tensor ws;
    if (ks > 1) {
      ws = at::empty({(int64_t)ks * a.M * a.OCpad}, x.options().dtype(at::kFloat));
      a.ws = ws.data_ptr<float>();
      a.ksplit = ks;
    }
    if (ks == 1 && (impl == 0 || impl == 2) && amode == dv::CONV_A_FWD && epi == dv::CONV_E_BF16 && !mask.has_value()) {
      dv::ConvArgs ap = a;
      const int64_t flags = with_bits(ap);
      const int rc = dv::conv_pw_launch(ap, cur_stream());  // large-M 1x1 convs: persistent pipeline
      if (rc >= 0) {
        check_rc(rc, "conv_pw");
        finish_stats();
        return flags;
      }
    }
    // KW3P stream-K workspace (conv_dma_impl.h:kw3_sk_ok decides whether it is used): one fp32 partial-tile
    // slot + one flag per CU, from the stream-ordered caching allocator (graph-capture safe; concurrent
    // streams never share one)
    Tensor skws;
    const int64_t cus = device_cus();
    if (ks == 1 && amode == dv::CONV_A_FWD && epi == dv::CONV_E_BF16 && !mask.has_value() && a.KH == 3 && a.KW == 3 &&
        a.stride == 1 && a.pad_h == 1 && a.pad_w == 1 && a.C % 32 == 0 && a.OCpad % 128 == 0 && !a.res && !a.emask &&
        !a.accumulate && (int64_t)a.M * a.OCpad > cus * dv::kSkSlotFloats && cus <= dv::kSkMaxWg &&
        std::getenv("DV_NO_KW3_SK") == nullptr) {
      skws = at::empty({cus * dv::kSkSlotFloats + cus}, x.options().dtype(at::kFloat));
      a.skw = skws.data_ptr<float>();
      a.skflag = reinterpret_cast<unsigned*>(a.skw + cus * dv::kSkSlotFloats);
      a.skslots = (int)cus;
      a.skerr = sk_error_counter();
    }
    check_rc(dv::conv_dma_launch(a, (int)amode, (int)epi, cur_stream()), "conv_dma");
    if (ks > 1) check_rc(dv::splitk_reduce_launch(a, (int)epi, cur_stream()), "splitk_reduce");
  } else {
    check_rc(dv::conv_igemm_launch(a, (int)amode, (int)epi, cur_stream()), "conv_igemm");
  }
  finish_stats();
  return 0;
}

// kind 0 max / 1 avg; dir 0 fwd (in=x, out=y) / 1 bwd (in=gy, out=gx); geom = N,H,W,C,OH,OW,k,s,pad.
// x/gx and y/gy may be channel-slice views (dense pixels, channel stride 1, pixel stride % 8 == 0):
// the InceptionV3 blocks pool straight out of / into their concat buffers. avgpool fwd may add a
// per-channel fp32 bias and apply ReLU (the block's pool branch with its 1x1 conv commuted first).
static int64_t pix_ld(const Tensor& t, int64_t H, int64_t W, int64_t C, const char* name) {
  TORCH_CHECK(t.dim() == 4 && t.stride(3) == 1, name, ": NHWC with channel stride 1");
  const int64_t ld = t.stride(2);
  TORCH_CHECK(ld >= C && ld % 8 == 0 && t.stride(1) == W * ld && t.stride(0) == H * W * ld &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              name, ": dense pixels with a pixel stride % 8 == 0, 16-B aligned");
  return ld;
}

void pool(Tensor in, Tensor out, c10::optional<Tensor> idx, int64_t kind, int64_t dir, std::vector<int64_t> g,
          c10::optional<Tensor> bias, bool relu, bool accumulate) {
  check_cuda(in, "in");
  check_cuda(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(in.device());
  TORCH_CHECK(g.size() == 9, "pool: geometry");
  TORCH_CHECK(!accumulate || dir == 1, "pool accumulate: backward only");
  const int64_t N = g[0], H = g[1], W = g[2], C = g[3], OH = g[4], OW = g[5], k = g[6], s = g[7], pad = g[8];
  TORCH_CHECK(C % 8 == 0 && k >= 1 && s >= 1 && pad >= 0 && pad < k, "pool: C%8, k, s, pad");
  TORCH_CHECK(OH == (H + 2 * pad - k) / s + 1 && OW == (W + 2 * pad - k) / s + 1, "pool: output size");
  const auto dt = in.scalar_type();
  TORCH_CHECK((dt == at::kBFloat16 || dt == at::kHalf) && out.scalar_type() == dt, "pool: bf16 or fp16, one dtype");
  const Tensor& full = dir == 0 ? in : out;
  const Tensor& pooled = dir == 0 ? out : in;
  TORCH_CHECK(full.size(0) == N && full.size(1) == H && full.size(2) == W && full.size(3) == C, "pool: x shape");
  TORCH_CHECK(pooled.size(0) == N && pooled.size(1) == OH && pooled.size(2) == OW && pooled.size(3) == C,
              "pool: y shape");
  const int64_t x_ld = pix_ld(full, H, W, C, "pool x"), y_ld = pix_ld(pooled, OH, OW, C, "pool y");
  need(full, ((N * H * W - 1) * x_ld + C) * 2, "pool x");
  need(pooled, ((N * OH * OW - 1) * y_ld + C) * 2, "pool y");
  uint8_t* ip = nullptr;
  if (kind == 0) {
    TORCH_CHECK(idx.has_value() && idx->scalar_type() == at::kByte && idx->is_contiguous() &&
                    idx->numel() == N * OH * OW * C,
                "maxpool: idx [N,OH,OW,C] u8");
    ip = idx->data_ptr<uint8_t>();
  }
  const float* bp = nullptr;
  if (bias.has_value()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(kind == 1 && dir == 0 && bias->scalar_type() == at::kFloat && bias->is_contiguous() &&
                    bias->numel() >= C,
                "pool bias: avgpool forward, fp32 [>= C]");
    bp = bias->data_ptr<float>();
  }
  TORCH_CHECK(!relu || (kind == 1 && dir == 0), "pool relu: avgpool forward only");
  check_rc(dv::pool_launch((int)kind, (int)dir, reinterpret_cast<const uint16_t*>(in.data_ptr()),
                           reinterpret_cast<uint16_t*>(out.data_ptr()), ip, (int)N, (int)H, (int)W, (int)C, (int)OH,
                           (int)OW, (int)k, (int)s, (int)pad, dt == at::kHalf ? dv::DT_F16 : dv::DT_BF16, cur_stream(),
                           x_ld, y_ld, bp, relu ? 1 : 0, accumulate ? 1 : 0),
           "pool");
}

static int dt_of(const Tensor& t);

// gx [N, H, W, C] <- E [N, OH, OW, C] at every s-th pixel, 0 elsewhere, [masked by emask > 0]
void subpixel_scatter(Tensor E, c10::optional<Tensor> emask, Tensor gx, int64_t s) {
  check_cuda(E, "E");
  check_cuda(gx, "gx");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(E.device());
  TORCH_CHECK(E.dim() == 4 && gx.dim() == 4 && E.is_contiguous() && gx.is_contiguous() && E.size(0) == gx.size(0) &&
                  E.size(3) == gx.size(3) && E.size(3) % 8 == 0 && E.scalar_type() == gx.scalar_type() && s >= 1,
              "subpixel_scatter: E [N,OH,OW,C], gx [N,H,W,C] contiguous, one dtype, C % 8");
  TORCH_CHECK(E.size(1) == (gx.size(1) + s - 1) / s && E.size(2) == (gx.size(2) + s - 1) / s,
              "subpixel_scatter: OH = ceil(H / s), OW = ceil(W / s)");
  const uint16_t* mp = nullptr;
  if (emask.has_value()) {
    check_cuda(*emask, "emask");
    TORCH_CHECK(emask->sizes() == gx.sizes() && emask->is_contiguous() && emask->scalar_type() == gx.scalar_type(),
                "subpixel_scatter: emask like gx");
    mp = reinterpret_cast<const uint16_t*>(emask->data_ptr());
  }
  check_rc(dv::subpixel_scatter_launch(reinterpret_cast<const uint16_t*>(E.data_ptr()), mp,
                                       reinterpret_cast<uint16_t*>(gx.data_ptr()), (int)gx.size(0), (int)gx.size(1),
                                       (int)gx.size(2), (int)gx.size(3), (int)E.size(1), (int)E.size(2), (int)s,
                                       dt_of(gx), cur_stream()),
           "subpixel_scatter");
}

// gx [N,H,W,C] (=|+=) the strided-conv input gradient assembled from parts[(h%s)*s + w%s] ([N, ceil-class
// H, W, ld >= C] 16-bit, or None for an empty class), zeroed where emask <= 0 (ops/autograd.py _subpixel_dgrad)
void subpixel_merge(std::vector<c10::optional<Tensor>> parts, c10::optional<Tensor> emask, Tensor gx, int64_t s,
                    bool accumulate) {
  check_cuda(gx, "gx");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gx.device());
  TORCH_CHECK(gx.dim() == 4 && gx.is_contiguous() && gx.size(3) % 8 == 0 && (s == 1 || s == 2) &&
                  (int64_t)parts.size() == s * s,
              "subpixel_merge: gx [N,H,W,C] contiguous, C % 8, s in {1, 2}, s^2 parts");
  const int64_t N = gx.size(0), H = gx.size(1), W = gx.size(2), C = gx.size(3);
  const uint16_t* p[4] = {nullptr, nullptr, nullptr, nullptr};
  int hc[4] = {0, 0, 0, 0}, wc[4] = {0, 0, 0, 0}, ld[4] = {0, 0, 0, 0};
  for (int k = 0; k < (int)parts.size(); ++k) {
    if (!parts[k].has_value()) continue;
    const Tensor& t = *parts[k];
    check_cuda(t, "part");
    const int rh = k / (int)s, rw = k % (int)s;
    const int64_t want_h = (H - rh + s - 1) / s, want_w = (W - rw + s - 1) / s;
    TORCH_CHECK(t.dim() == 4 && t.scalar_type() == gx.scalar_type() && t.size(0) == N && t.size(1) == want_h &&
                    t.size(2) == want_w && t.stride(3) == 1 && t.stride(2) >= C && t.stride(2) % 8 == 0 &&
                    t.stride(1) == t.size(2) * t.stride(2) && t.stride(0) == t.size(1) * t.stride(1) &&
                    reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
                "subpixel_merge: part k = [N, ceil((H - rh) / s), ceil((W - rw) / s), >= C] dense pixels, 16-B aligned");
    p[k] = reinterpret_cast<const uint16_t*>(t.data_ptr());
    hc[k] = (int)t.size(1);
    wc[k] = (int)t.size(2);
    ld[k] = (int)t.stride(2);
  }
  const uint16_t* mp = nullptr;
  if (emask.has_value()) {
    check_cuda(*emask, "emask");
    TORCH_CHECK(emask->sizes() == gx.sizes() && emask->is_contiguous() && emask->scalar_type() == gx.scalar_type(),
                "subpixel_merge: emask like gx");
    mp = reinterpret_cast<const uint16_t*>(emask->data_ptr());
  }
  check_rc(dv::subpixel_merge_launch(p, hc, wc, ld, mp, reinterpret_cast<uint16_t*>(gx.data_ptr()), (int)N, (int)H,
                                     (int)W, (int)C, (int)s, accumulate ? 1 : 0, dt_of(gx), cur_stream()),
           "subpixel_merge");
}

static int dt_of(const Tensor& t) {
  TORCH_CHECK(t.scalar_type() == at::kBFloat16 || t.scalar_type() == at::kHalf, "expected a bf16 or fp16 tensor");
  return t.scalar_type() == at::kHalf ? dv::DT_F16 : dv::DT_BF16;
}

// strided few-channel stem conv (InceptionV3 conv2d_1) on the direct VALU kernels; w: fp32
// [KH][KW][cr][cout]. g = {N, H, W, OH, OW, C, cr, cout, k, stride, pad, relu}. dir 0: x [N,H,W,C] ->
// out [N,OH,OW,cout] (+bias, ReLU); dir 1: x = gy [N,OH,OW,cout] -> out = gx [N,H,W,C]. Returns false
// when the geometry is not covered (the caller takes the GEMM path).
bool stem_conv(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor out, std::vector<int64_t> g, int64_t dir) {
  check_cuda(x, "x");
  check_cuda(out, "out");
  check_cuda(w, "w");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(g.size() == 12, "stem_conv: geometry");
  const int N = (int)g[0], H = (int)g[1], W = (int)g[2], OH = (int)g[3], OW = (int)g[4], C = (int)g[5];
  const int cr = (int)g[6], cout = (int)g[7], k = (int)g[8], st = (int)g[9], pad = (int)g[10], relu = (int)g[11];
  TORCH_CHECK(w.scalar_type() == at::kFloat && w.is_contiguous() && w.numel() == (int64_t)k * k * cr * cout,
              "stem_conv: w fp32 [k][k][cr][cout]");
  TORCH_CHECK(x.scalar_type() == out.scalar_type() && x.dim() == 4 && out.dim() == 4 && x.stride(3) == 1 &&
                  out.stride(3) == 1 && reinterpret_cast<uintptr_t>(x.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "stem_conv: 16-bit NHWC, 16-B aligned");
  const Tensor& full = dir == 0 ? x : out;
  const Tensor& red = dir == 0 ? out : x;
  TORCH_CHECK(full.size(0) == N && full.size(1) == H && full.size(2) == W && full.size(3) >= C &&
                  red.size(0) == N && red.size(1) == OH && red.size(2) == OW && red.size(3) >= cout,
              "stem_conv: shapes");
  TORCH_CHECK(full.stride(1) == W * full.stride(2) && full.stride(0) == (int64_t)H * W * full.stride(2) &&
                  red.stride(1) == OW * red.stride(2) && red.stride(0) == (int64_t)OH * OW * red.stride(2),
              "stem_conv: dense pixels");
  int rc;
  if (dir == 0) {
    const float* bp = nullptr;
    if (bias.has_value()) {
      check_cuda(*bias, "bias");
      TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->numel() >= cout, "stem_conv: bias fp32");
      bp = bias->data_ptr<float>();
    }
    rc = dv::stem_conv_fwd_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), w.data_ptr<float>(), bp,
                                  reinterpret_cast<uint16_t*>(out.data_ptr()), N, H, W, OH, OW, C, cr, cout, k, st, pad,
                                  relu, x.stride(2), out.stride(2), dt_of(x), cur_stream());
  } else {
    rc = dv::stem_conv_dgrad_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), w.data_ptr<float>(),
                                    reinterpret_cast<uint16_t*>(out.data_ptr()), N, H, W, OH, OW, C, cr, cout, k, st,
                                    pad, x.stride(2), out.stride(2), dt_of(x), cur_stream());
  }
  if (rc == -4) return false;
  check_rc(rc, "stem_conv");
  return true;
}

// DeepDream loss core: part [N, P] fp32 partial sums of x^2 over x[:, b:H-b, b:W-b, :]
void sumsq_core(Tensor x, Tensor part, int64_t b) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(3) % 8 == 0, "sumsq: x contiguous NHWC, C % 8");
  TORCH_CHECK(part.dim() == 2 && part.scalar_type() == at::kFloat && part.is_contiguous() &&
                  part.size(0) == x.size(0),
              "sumsq: part [N, P] fp32");
  check_rc(dv::sumsq_core_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), part.data_ptr<float>(),
                                 (int)part.size(1), (int)x.size(0), (int)x.size(1), (int)x.size(2), (int)x.size(3),
                                 (int)b, dt_of(x), cur_stream()),
           "sumsq_core");
}

// gx = 2 * scale[n] * x on the border-b core (0 elsewhere), plus `addend` (same layout) when given
void sumsq_core_bwd(Tensor x, Tensor scale, Tensor gx, int64_t b, c10::optional<Tensor> addend,
                    c10::optional<Tensor> part) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && x.is_contiguous() && x.size(3) % 8 == 0, "sumsq_bwd: x contiguous NHWC, C % 8");
  TORCH_CHECK(gx.sizes() == x.sizes() && gx.scalar_type() == x.scalar_type() && gx.is_contiguous(), "sumsq_bwd: gx");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_contiguous() && scale.numel() == x.size(0),
              "sumsq_bwd: scale [N] fp32");
  const uint16_t* ap = nullptr;
  if (addend.has_value()) {
    check_cuda(*addend, "addend");
    TORCH_CHECK(addend->sizes() == x.sizes() && addend->scalar_type() == x.scalar_type() && addend->is_contiguous(),
                "sumsq_bwd: addend like x");
    ap = reinterpret_cast<const uint16_t*>(addend->data_ptr());
  }
  if (part.has_value()) {  // + the loss partials of x (the forward sumsq_core, fused)
    check_cuda(*part, "part");
    TORCH_CHECK(part->dim() == 2 && part->scalar_type() == at::kFloat && part->is_contiguous() &&
                    part->size(0) == x.size(0),
                "sumsq_bwd: part [N, P] fp32");
    check_rc(dv::sumsq_core_fused_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), scale.data_ptr<float>(), ap,
                                         reinterpret_cast<uint16_t*>(gx.data_ptr()), part->data_ptr<float>(),
                                         (int)part->size(1), (int)x.size(0), (int)x.size(1), (int)x.size(2),
                                         (int)x.size(3), (int)b, dt_of(x), cur_stream()),
             "sumsq_core_fused");
    return;
  }
  check_rc(dv::sumsq_core_bwd_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), scale.data_ptr<float>(), ap,
                                     reinterpret_cast<uint16_t*>(gx.data_ptr()), (int)x.size(0), (int)x.size(1),
                                     (int)x.size(2), (int)x.size(3), (int)b, dt_of(x), cur_stream()),
           "sumsq_core_bwd");
}

// Fused DeepDream update (engine/deepdream.py): g [N,H,W,8] 16-bit input gradient, x [N,H,W,3] fp32
// master image (updated in place), xin [N,H,W,8] next network input, gpart [N, P] scratch, lpart
// [L, N, LP] sumsq partials of the L loss layers, lcoef [L] fp32 coefficient / numel, done u8 [N],
// loss fp32 [N]; max_loss < 0 disables the early stop.
void dream_update(Tensor g, Tensor x, Tensor xin, Tensor gpart, Tensor lpart, Tensor lcoef, Tensor done, Tensor loss,
                  double step, double max_loss) {
  check_cuda(g, "g");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  TORCH_CHECK(g.dim() == 4 && g.size(3) == 8 && g.is_contiguous(), "dream_update: g [N,H,W,8] contiguous");
  const int64_t N = g.size(0), H = g.size(1), W = g.size(2);
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(0) == N && x.size(1) == H &&
                  x.size(2) == W && x.size(3) == 3,
              "dream_update: x fp32 [N,H,W,3] contiguous");
  TORCH_CHECK(xin.sizes() == g.sizes() && xin.scalar_type() == g.scalar_type() && xin.is_contiguous(),
              "dream_update: xin like g");
  TORCH_CHECK(gpart.scalar_type() == at::kFloat && gpart.is_contiguous() && gpart.dim() == 2 && gpart.size(0) == N,
              "dream_update: gpart fp32 [N, P]");
  TORCH_CHECK(lpart.scalar_type() == at::kFloat && lpart.is_contiguous() && lpart.dim() == 3 && lpart.size(1) == N,
              "dream_update: lpart fp32 [L, N, LP]");
  TORCH_CHECK(lcoef.scalar_type() == at::kFloat && lcoef.is_contiguous() && lcoef.numel() == lpart.size(0),
              "dream_update: lcoef fp32 [L]");
  TORCH_CHECK(done.scalar_type() == at::kByte && done.is_contiguous() && done.numel() == N, "dream_update: done u8 [N]");
  TORCH_CHECK(loss.scalar_type() == at::kFloat && loss.is_contiguous() && loss.numel() == N, "dream_update: loss [N]");
  for (const Tensor* t : {&x, &xin, &gpart, &lpart, &lcoef, &done, &loss}) check_cuda(*t, "dream_update operand");
  check_rc(dv::dream_update_launch(reinterpret_cast<const uint16_t*>(g.data_ptr()), x.data_ptr<float>(),
                                   reinterpret_cast<uint16_t*>(xin.data_ptr()), gpart.data_ptr<float>(),
                                   (int)gpart.size(1), lpart.data_ptr<float>(), lcoef.data_ptr<float>(),
                                   (int)lpart.size(0), (int)lpart.size(2), done.data_ptr<uint8_t>(),
                                   loss.data_ptr<float>(), (float)step, (float)max_loss, (int)N, (int)H, (int)W,
                                   dt_of(g), cur_stream()),
           "dream_update");
}

// DeepDream octave transition (engine/deepdream.py:DeepDream.octave_steps): y [N,Hd,Wd,3] fp32 = corner-aligned
// bilinear resize of (a + b - c) (a, b, c [N,Hs,Ws,3] fp32; b, c optional); yin (optional) [N,Hd,Wd,8] 16-bit
// network input.
void octave_resize(Tensor a, c10::optional<Tensor> b, c10::optional<Tensor> c, Tensor y, c10::optional<Tensor> yin) {
  check_cuda(a, "a");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(a.device());
  auto f3 = [](const Tensor& t) {
    return t.scalar_type() == at::kFloat && t.is_contiguous() && t.dim() == 4 && t.size(3) == 3;
  };
  TORCH_CHECK(f3(a) && f3(y) && y.size(0) == a.size(0), "octave_resize: a, y fp32 [N,H,W,3] contiguous");
  check_cuda(y, "y");
  const float* bp = nullptr;
  if (b && b->defined()) {
    TORCH_CHECK(b->sizes() == a.sizes() && f3(*b), "octave_resize: b like a");
    check_cuda(*b, "b");
    bp = b->data_ptr<float>();
  }
  const float* cp = nullptr;
  if (c && c->defined()) {
    TORCH_CHECK(c->sizes() == a.sizes() && f3(*c), "octave_resize: c like a");
    check_cuda(*c, "c");
    cp = c->data_ptr<float>();
  }
  uint16_t* ip = nullptr;
  int dt = dv::DT_BF16;
  if (yin && yin->defined()) {
    TORCH_CHECK(yin->dim() == 4 && yin->size(0) == y.size(0) && yin->size(1) == y.size(1) && yin->size(2) == y.size(2) &&
                    yin->size(3) == 8 && yin->is_contiguous(),
                "octave_resize: yin 16-bit [N,Hd,Wd,8] contiguous");
    check_cuda(*yin, "yin");
    dt = dt_of(*yin);
    ip = reinterpret_cast<uint16_t*>(yin->data_ptr());
  }
  check_rc(dv::octave_resize_launch(a.data_ptr<float>(), bp, cp, y.data_ptr<float>(), ip, (int)a.size(0), (int)a.size(1),
                                    (int)a.size(2), (int)y.size(1), (int)y.size(2), dt, cur_stream()),
           "octave_resize");
}

// Tiled DeepDream step (engine/deepdream.py:TiledDeepDream). plan: int32 [units_total, 7] rows
// {image, tile origin y, x, owned y0, y1, x0, x1 (tile-local)}, validated on the host when built;
// shift: int32 [2] device (sy, sx). This rank's units are u = rank + k * world, k < xin.size(0).
static void check_plan(const Tensor& plan, const Tensor& shift) {
  check_cuda(plan, "plan");
  check_cuda(shift, "shift");
  TORCH_CHECK(plan.scalar_type() == at::kInt && plan.is_contiguous() && plan.dim() == 2 && plan.size(1) == 7,
              "tile plan: int32 [U, 7]");
  TORCH_CHECK(shift.scalar_type() == at::kInt && shift.numel() >= 2 && shift.stride(-1) == 1, "tile shift: int32 [2]");
}

// k0: the chunk's first unit among this rank's units (TiledDeepDream's overlapped all-gather)
void tile_gather(Tensor x, Tensor xin, Tensor plan, Tensor shift, int64_t rank, int64_t world, int64_t k0) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  check_plan(plan, shift);
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3, "tile_gather: x");
  TORCH_CHECK(xin.dim() == 4 && xin.size(3) == 8 && xin.is_contiguous(), "tile_gather: xin [U, Th, Tw, 8]");
  const int64_t U = xin.size(0);
  TORCH_CHECK(world >= 1 && rank >= 0 && rank < world && k0 >= 0 && rank + (k0 + U - 1) * world < plan.size(0),
              "tile_gather: units");
  check_rc(dv::tile_gather_launch(x.data_ptr<float>(), reinterpret_cast<uint16_t*>(xin.data_ptr()), plan.data_ptr<int>(),
                                  shift.data_ptr<int>(), (int)U, (int)rank, (int)world, (int)k0, (int)x.size(1),
                                  (int)x.size(2), (int)xin.size(1), (int)xin.size(2), dt_of(xin), cur_stream()),
           "tile_gather");
}

void tile_pack(Tensor g, Tensor pack, Tensor plan, Tensor lpart, Tensor lcoef, int64_t ucap, int64_t rank, int64_t world,
               int64_t k0) {
  check_cuda(g, "g");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(g.device());
  check_cuda(plan, "plan");
  TORCH_CHECK(plan.scalar_type() == at::kInt && plan.is_contiguous() && plan.dim() == 2 && plan.size(1) == 7, "plan");
  TORCH_CHECK(g.dim() == 4 && g.size(3) == 8 && g.is_contiguous(), "tile_pack: g [U, Th, Tw, 8]");
  const int64_t U = g.size(0), Th = g.size(1), Tw = g.size(2);
  TORCH_CHECK(U <= ucap && k0 >= 0 && world >= 1 && rank >= 0 && rank < world && rank + (k0 + U - 1) * world < plan.size(0),
              "tile_pack: units");
  TORCH_CHECK(pack.scalar_type() == g.scalar_type() && pack.is_contiguous() &&
                  pack.numel() >= dv::tile_pack_elems((int)ucap, (int)Th, (int)Tw) &&
                  reinterpret_cast<uintptr_t>(pack.data_ptr()) % 16 == 0,
              "tile_pack: pack too small / misaligned");
  TORCH_CHECK(lpart.scalar_type() == at::kFloat && lpart.is_contiguous() && lpart.dim() == 3 && lpart.size(1) == U,
              "tile_pack: lpart [L, U, LP]");
  TORCH_CHECK(lcoef.scalar_type() == at::kFloat && lcoef.numel() == lpart.size(0), "tile_pack: lcoef [L]");
  check_rc(dv::tile_pack_launch(reinterpret_cast<const uint16_t*>(g.data_ptr()), reinterpret_cast<uint16_t*>(pack.data_ptr()),
                                plan.data_ptr<int>(), lpart.data_ptr<float>(), lcoef.data_ptr<float>(), (int)lpart.size(0),
                                (int)lpart.size(2), (int)U, (int)ucap, (int)rank, (int)world, (int)k0, (int)Th, (int)Tw,
                                dt_of(g), cur_stream()),
           "tile_pack");
}

// packs: [chunks][world][tile_pack_elems(ucap)] (chunks inferred), ucap = units per rank and chunk
void tile_update(Tensor packs, int64_t ucap, Tensor plan, Tensor shift, Tensor x, Tensor done, Tensor loss, double step,
                 double max_loss, int64_t world, int64_t Th, int64_t Tw) {
  check_cuda(packs, "packs");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(packs.device());
  check_plan(plan, shift);
  const long long pe = dv::tile_pack_elems((int)ucap, (int)Th, (int)Tw);
  TORCH_CHECK(packs.is_contiguous() && world >= 1 && packs.numel() % (world * pe) == 0,
              "tile_update: packs [chunks, world, pack_elems]");
  const int64_t chunks = packs.numel() / (world * pe);
  TORCH_CHECK(chunks >= 1 && plan.size(0) <= chunks * world * ucap, "tile_update: plan larger than the packs");
  TORCH_CHECK(x.scalar_type() == at::kFloat && x.is_contiguous() && x.dim() == 4 && x.size(3) == 3, "tile_update: x");
  TORCH_CHECK(done.scalar_type() == at::kByte && done.numel() == x.size(0) && loss.scalar_type() == at::kFloat &&
                  loss.numel() == x.size(0),
              "tile_update: done u8 [B], loss fp32 [B]");
  check_rc(dv::tile_update_launch(reinterpret_cast<const uint16_t*>(packs.data_ptr()), pe, (int)ucap, plan.data_ptr<int>(),
                                  (int)plan.size(0), shift.data_ptr<int>(), x.data_ptr<float>(), done.data_ptr<uint8_t>(),
                                  loss.data_ptr<float>(), (float)step, (float)max_loss, (int)world, (int)x.size(1),
                                  (int)x.size(2), (int)Th, (int)Tw, dt_of(packs), cur_stream()),
           "tile_update");
}

int64_t tile_pack_elems(int64_t ucap, int64_t Th, int64_t Tw) { return dv::tile_pack_elems((int)ucap, (int)Th, (int)Tw); }

// geom: KH, KW, stride, pad_h, pad_w, Cr; cols [N, OH, OW, J_ld] (J = KH*KW*Cr), gx [N, H, W, 8]
// g = KH, KW, stride, pad, Cr; false: not the fused kernel's geometry (caller falls back)
// ResNet-50 conv1 forward on the tap-paired MFMA kernel (conv_stem7.hip): x [N,H,W,8], w [64][224]
// (kh, kw 0..7, c 0..3; zero where kw = 7 or c = 3), bias fp32 >= 64, out [N,OH,OW,64], all dense.
// Returns false when the geometry is not covered (the caller takes the implicit GEMM).
bool stem7_fwd(Tensor x, Tensor w, c10::optional<Tensor> bias, Tensor out, int64_t relu) {
  check_cuda(x, "x");
  check_cuda(w, "w");
  check_cuda(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && out.dim() == 4 && x.size(3) == 8 && out.size(3) == 64 && x.is_contiguous() &&
                  out.is_contiguous() && w.is_contiguous() && w.numel() == 64 * 224 &&
                  x.scalar_type() == out.scalar_type() && w.scalar_type() == x.scalar_type() &&
                  out.size(0) == x.size(0),
              "stem7_fwd: x [N,H,W,8], w [64][224], out [N,OH,OW,64], dense, one 16-bit dtype");
  const float* bp = nullptr;
  if (bias.has_value()) {
    check_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == at::kFloat && bias->is_contiguous() && bias->numel() >= 64,
                "stem7_fwd: bias fp32");
    bp = bias->data_ptr<float>();
  }
  const int rc = dv::stem7_fwd_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                      reinterpret_cast<const uint16_t*>(w.data_ptr()), bp,
                                      reinterpret_cast<uint16_t*>(out.data_ptr()), (int)x.size(0), (int)x.size(1),
                                      (int)x.size(2), (int)out.size(1), (int)out.size(2), (int)relu, dt_of(x),
                                      cur_stream());
  if (rc == -4) return false;
  check_rc(rc, "stem7_fwd");
  return true;
}

bool stem_dgrad_fused(Tensor gy, c10::optional<Tensor> mask, Tensor w, Tensor gx, std::vector<int64_t> g) {
  check_cuda(gy, "gy");
  check_cuda(w, "w");
  check_cuda(gx, "gx");
  TORCH_CHECK(g.size() == 5, "stem_dgrad_fused: geometry");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(gy.device());
  TORCH_CHECK(gy.dim() == 4 && gx.dim() == 4 && w.dim() == 2 && gy.is_contiguous() && gx.is_contiguous() &&
                  w.is_contiguous() && gy.scalar_type() == gx.scalar_type() && w.scalar_type() == gy.scalar_type() &&
                  gx.size(3) == 8 && gx.size(0) == gy.size(0),
              "stem_dgrad_fused: gy [N,OH,OW,C], gx [N,H,W,8], w [rows, C] contiguous, one 16-bit dtype");
  dv::StemDgradGeom G{(int)gy.size(0), (int)gx.size(1), (int)gx.size(2), (int)gy.size(1), (int)gy.size(2),
                      (int)gy.size(3), (int)g[0], (int)g[1], (int)g[2], (int)g[3], (int)g[4], (int)w.size(0),
                      (int)w.size(1)};
  TORCH_CHECK(w.size(1) >= G.C, "stem_dgrad_fused: w rows must hold C weights");
  const uint16_t* m = nullptr;
  if (mask.has_value()) {
    check_cuda(*mask, "mask");
    TORCH_CHECK(mask->sizes() == gy.sizes() && mask->is_contiguous() && mask->scalar_type() == gy.scalar_type(),
                "stem_dgrad_fused: mask like gy");
    m = reinterpret_cast<const uint16_t*>(mask->data_ptr());
  }
  const int rc = dv::stem_dgrad_fused_launch(reinterpret_cast<const uint16_t*>(gy.data_ptr()), m,
                                             reinterpret_cast<const uint16_t*>(w.data_ptr()),
                                             reinterpret_cast<uint16_t*>(gx.data_ptr()), G, dt_of(gy), cur_stream());
  if (rc == -4) return false;
  check_rc(rc, "stem_dgrad_fused");
  return true;
}

void col2im(Tensor cols, Tensor gx, std::vector<int64_t> g) {
  check_cuda(cols, "cols");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(cols.device());
  TORCH_CHECK(g.size() == 6, "col2im: geometry");
  TORCH_CHECK(cols.dim() == 4 && cols.is_contiguous() && gx.dim() == 4 && gx.is_contiguous() && gx.size(3) == 8 &&
                  gx.scalar_type() == cols.scalar_type() && gx.size(0) == cols.size(0),
              "col2im: cols [N,OH,OW,J_ld], gx [N,H,W,8] contiguous, same dtype");
  dv::Col2ImGeom G{(int)gx.size(0), (int)gx.size(1), (int)gx.size(2), (int)cols.size(1), (int)cols.size(2),
                   (int)g[0], (int)g[1], (int)g[2], (int)g[3], (int)g[4], (int)g[5], (int)cols.size(3)};
  TORCH_CHECK(G.Cr >= 1 && G.Cr <= 8 && (int64_t)G.KH * G.KW * G.Cr <= G.J_ld && G.stride >= 1, "col2im: K/Cr/J_ld");
  check_rc(dv::col2im_launch(reinterpret_cast<const uint16_t*>(cols.data_ptr()),
                             reinterpret_cast<uint16_t*>(gx.data_ptr()), G, dt_of(cols), cur_stream()),
           "col2im");
}

// Response encoding (host): uint8 RGB [B, H, W, 3] (CPU) -> B data URLs, JPEG + base64 + the
// reference's quote() escaping, on `threads` native threads with the GIL released.
py::list jpeg_data_urls(Tensor img, int64_t quality, std::string prefix, int64_t threads) {
  TORCH_CHECK(!img.is_cuda() && img.scalar_type() == at::kByte && img.dim() == 4 && img.size(3) == 3 &&
                  img.is_contiguous(),
              "jpeg_data_urls: uint8 CPU [B, H, W, 3] contiguous");
  std::vector<std::string> out;
  {
    py::gil_scoped_release nogil;
    out = dvjpeg::encode_data_urls(img.data_ptr<uint8_t>(), (int)img.size(0), (int)img.size(1), (int)img.size(2),
                                   (int)quality, prefix, (int)threads);
  }
  py::list res;
  for (auto& s : out) res.append(py::str(s));
  return res;
}

// GPU JPEG (jpeg_gpu.hip): img uint8 [B, H, W, 3] on the device -> {packed entropy-coded scans
// (device uint8, capacity B * worst case), offsets int64 [B + 1] (device)}; the stream of image b is
// jpeg_gpu_header(H, W, q) + packed[off[b]:off[b+1]] + EOI
std::vector<Tensor> jpeg_gpu(Tensor img, int64_t quality) {
  check_cuda(img, "img");
  TORCH_CHECK(img.scalar_type() == at::kByte && img.dim() == 4 && img.size(3) == 3 && img.is_contiguous(),
              "jpeg_gpu: uint8 [B, H, W, 3] contiguous");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(img.device());
  const int B = (int)img.size(0), H = (int)img.size(1), W = (int)img.size(2);
  TORCH_CHECK(B >= 1 && B <= 65535 && H >= 1 && W >= 1 && H <= 65500 && W <= dv::jpeg_gpu_max_width(),
              "jpeg_gpu: image size (W <= ", dv::jpeg_gpu_max_width(), ")");
  static std::mutex mu;
  static std::map<std::pair<int, int>, Tensor> tables;  // (device, quality) -> device GpuTables
  Tensor tab;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto key = std::make_pair((int)img.get_device(), (int)quality);
    auto it = tables.find(key);
    if (it == tables.end()) {
      const dvjpeg::GpuTables t = dvjpeg::gpu_tables((int)quality);
      Tensor h = at::empty({(int64_t)sizeof(t)}, at::TensorOptions().dtype(at::kByte));
      std::memcpy(h.data_ptr(), &t, sizeof(t));
      it = tables.emplace(key, h.to(img.device())).first;
    }
    tab = it->second;
  }
  const long long out_cap = dv::jpeg_gpu_out_cap(H, W);
  auto opt = img.options();
  Tensor ws = at::empty({dv::jpeg_gpu_ws_bytes(B, H, W)}, opt);
  Tensor packed = at::empty({(int64_t)B * out_cap}, opt);
  Tensor off = at::empty({B + 1}, opt.dtype(at::kLong));
  check_rc(dv::jpeg_gpu_launch(img.data_ptr<uint8_t>(), B, H, W, tab.data_ptr(), ws.data_ptr(),
                               packed.data_ptr<uint8_t>(), reinterpret_cast<long long*>(off.data_ptr<int64_t>()),
                               cur_stream()),
           "jpeg_gpu");
  return {packed, off};
}

// data URL (ASCII str) -> decoded payload bytes, GIL released while decoding; raises ValueError
// with CPython's base64 message (the caller maps it to a 400), TypeError for a non-ASCII str
py::bytes data_url_b64decode(py::str uri) {
  PyObject* o = uri.ptr();
  if (!PyUnicode_IS_ASCII(o)) throw py::type_error("string argument should contain only ASCII characters");
  Py_ssize_t n = 0;
  const char* p = PyUnicode_AsUTF8AndSize(o, &n);  // the str's own ASCII buffer: no copy
  if (p == nullptr) throw py::error_already_set();
  std::string out, err;
  bool ok;
  {
    std::optional<py::gil_scoped_release> nogil;  // (large payloads only: see url_unquote_plus)
    if (n >= (1 << 15)) nogil.emplace();
    ok = dvjpeg::data_url_b64decode(p, (size_t)n, out, err);
  }
  if (!ok) throw py::value_error(err);
  return py::bytes(out);
}

// urllib.parse.unquote_plus of an ASCII str up to the final UTF-8 decode (the caller's): '+' -> ' ', %XX ->
// byte XX, anything else (a '%' without two hex digits too) verbatim. GIL released: a percent-encoded
// ~180 KB data URL has thousands of escapes, which urllib walks in a Python loop (api/forms.py).
py::bytes url_unquote_plus(py::str s) {
  PyObject* o = s.ptr();
  if (!PyUnicode_IS_ASCII(o)) throw py::type_error("url_unquote_plus: ASCII text only");
  Py_ssize_t n = 0;
  const char* p = PyUnicode_AsUTF8AndSize(o, &n);
  if (p == nullptr) throw py::error_already_set();
  std::string out;
  {
    // the GIL goes only for large inputs: a short release hands it to a waiting thread and getting it
    // back costs up to the switch interval (0.2 ms per call measured on tiny bodies)
    std::optional<py::gil_scoped_release> nogil;
    if (n >= (1 << 15)) nogil.emplace();
    out.resize((size_t)n);
    auto hex = [](char c) -> int {
      return c >= '0' && c <= '9' ? c - '0' : (c >= 'a' && c <= 'f' ? c - 'a' + 10 : (c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1));
    };
    size_t j = 0;
    for (Py_ssize_t i = 0; i < n; ++i) {
      const char c = p[i];
      if (c == '+') {
        out[j++] = ' ';
      } else if (c == '%' && i + 2 < n && hex(p[i + 1]) >= 0 && hex(p[i + 2]) >= 0) {
        out[j++] = (char)(hex(p[i + 1]) * 16 + hex(p[i + 2]));
        i += 2;
      } else {
        out[j++] = c;
      }
    }
    out.resize(j);
  }
  return py::bytes(out);
}

py::bytes jpeg_gpu_header(int64_t H, int64_t W, int64_t quality) {
  return py::bytes(dvjpeg::jpeg_header((int)H, (int)W, (int)quality, 1));
}

// host: GPU scans (CPU tensors) -> data URLs (header + scan + EOI, base64, quote escaping), GIL released
py::list jpeg_gpu_data_urls(Tensor packed, Tensor off, int64_t H, int64_t W, int64_t quality, std::string prefix,
                            int64_t threads) {
  TORCH_CHECK(!packed.is_cuda() && !off.is_cuda() && packed.scalar_type() == at::kByte &&
                  off.scalar_type() == at::kLong && off.dim() == 1 && off.size(0) >= 1 && packed.is_contiguous() &&
                  off.is_contiguous(),
              "jpeg_gpu_data_urls: CPU uint8 scans + int64 offsets");
  const int B = (int)off.size(0) - 1;
  const int64_t* o = off.data_ptr<int64_t>();
  TORCH_CHECK(o[0] == 0 && o[B] <= packed.numel(), "jpeg_gpu_data_urls: offsets outside the scans");
  for (int b = 0; b < B; ++b) TORCH_CHECK(o[b + 1] >= o[b], "jpeg_gpu_data_urls: offsets not increasing");
  const std::string header = dvjpeg::jpeg_header((int)H, (int)W, (int)quality, 1);
  std::vector<std::string> out;
  {
    py::gil_scoped_release nogil;
    out = dvjpeg::data_urls_from_scans(header, packed.data_ptr<uint8_t>(), o, B, prefix, (int)threads);
  }
  py::list l;
  for (auto& u : out) l.append(py::str(u));
  return l;
}

py::bytes jpeg_encode(Tensor img, int64_t quality) {
  TORCH_CHECK(!img.is_cuda() && img.scalar_type() == at::kByte && img.dim() == 3 && img.size(2) == 3 &&
                  img.is_contiguous(),
              "jpeg_encode: uint8 CPU [H, W, 3] contiguous");
  std::string s;
  {
    py::gil_scoped_release nogil;
    s = dvjpeg::encode_jpeg(img.data_ptr<uint8_t>(), (int)img.size(0), (int)img.size(1), (int)quality);
  }
  return py::bytes(s);
}

// bench.py --emulate-rccl-world: a paced copy occupying `channels` CUs for bytes / gbs (an all-gather's
// receive side at a given link bandwidth; misc.hip:paced_copy_kernel)
void paced_copy(Tensor src, Tensor dst, int64_t channels, double gbs) {
  check_cuda(src, "src");
  check_cuda(dst, "dst");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(dst.device());
  TORCH_CHECK(src.is_contiguous() && dst.is_contiguous(), "paced_copy: contiguous tensors");
  const int64_t sb = src.numel() * src.element_size(), db = dst.numel() * dst.element_size();
  check_rc(dv::paced_copy_launch(src.data_ptr(), sb, dst.data_ptr(), db, (int)channels, gbs, cur_stream()), "paced_copy");
}

void softmax_rows(Tensor x, Tensor y) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 2 && x.scalar_type() == at::kFloat && x.is_contiguous() && y.sizes() == x.sizes() &&
                  y.scalar_type() == at::kFloat && y.is_contiguous(),
              "softmax_rows: fp32 [M, N] contiguous");
  check_rc(dv::softmax_rows_launch(x.data_ptr<float>(), y.data_ptr<float>(), (int)x.size(0), (int)x.size(1),
                                   cur_stream()),
           "softmax_rows");
}

void channel_sum(Tensor x, Tensor sums, int64_t N, int64_t HW, int64_t C) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(is16(x) && x.is_contiguous(), "channel_sum: x bf16 / fp16 contiguous");
  TORCH_CHECK(sums.scalar_type() == at::kFloat && sums.is_contiguous(), "channel_sum: sums fp32");
  need(x, N * HW * C * 2, "x");
  need(sums, N * C * 4, "sums");
  check_rc(dv::channel_sum_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()), sums.data_ptr<float>(), (int)N,
                                  (int)HW, (int)C, f16(x), cur_stream()),
           "channel_sum");
}

void topk_pos(Tensor v, Tensor idx, Tensor val, int64_t k) {
  check_cuda(v, "v");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(v.device());
  TORCH_CHECK(v.dim() == 2 && v.scalar_type() == at::kFloat && v.is_contiguous(), "topk: v [N, C] fp32");
  const int64_t N = v.size(0), C = v.size(1);
  TORCH_CHECK(idx.scalar_type() == at::kInt && idx.is_contiguous() && idx.numel() == N * k, "topk: idx [N, k] int32");
  TORCH_CHECK(val.scalar_type() == at::kFloat && val.is_contiguous() && val.numel() == N * k, "topk: val [N, k] fp32");
  check_rc(dv::topk_pos_launch(v.data_ptr<float>(), idx.data_ptr<int>(), val.data_ptr<float>(), (int)N, (int)C, (int)k,
                               cur_stream()),
           "topk_pos");
}

// out4 [B, H, W, C] bf16 target activation, idx [B, K] int32 (< C), code u8 [B, H, W, C] or none,
// S fp32 [B*K, H, W] (or [B*K, 2H, 2W] with code); mode 0 all, 1 max per image, 2 max over the batch
void seed_map(Tensor out4, Tensor idx, c10::optional<Tensor> code, Tensor S, int64_t mode) {
  check_cuda(out4, "out4");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(out4.device());
  TORCH_CHECK(out4.dim() == 4 && out4.is_contiguous() && is16(out4), "seed_map: out4 bf16 / fp16 NHWC");
  TORCH_CHECK(idx.dim() == 2 && idx.scalar_type() == at::kInt && idx.is_contiguous() && idx.size(0) == out4.size(0),
              "seed_map: idx int32 [B, K]");
  const int64_t B = out4.size(0), H = out4.size(1), W = out4.size(2), C = out4.size(3), K = idx.size(1);
  const int64_t up = code.has_value() ? 2 : 1;
  TORCH_CHECK(S.scalar_type() == at::kFloat && S.is_contiguous() && S.numel() == B * K * H * W * up * up,
              "seed_map: S fp32 [B*K, H, W] (x4 with code)");
  TORCH_CHECK(mode >= 0 && mode <= 2, "seed_map: mode");
  const uint8_t* cp = nullptr;
  if (code.has_value()) {
    check_cuda(*code, "code");
    TORCH_CHECK(code->sizes() == out4.sizes() && code->scalar_type() == at::kByte && code->is_contiguous(),
                "seed_map: code u8 like out4");
    cp = code->data_ptr<uint8_t>();
  }
  check_rc(dv::seed_map_launch(reinterpret_cast<const uint16_t*>(out4.data_ptr()), idx.data_ptr<int>(), cp,
                               S.data_ptr<float>(), (int)(B * K), (int)K, (int)H, (int)W, (int)C, (int)mode,
                               f16(out4), cur_stream()),
           "seed_map");
}

void seed_deconv3x3(Tensor S, Tensor f, Tensor wt, Tensor out) {
  check_cuda(S, "S");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(S.device());
  TORCH_CHECK(S.dim() == 3 && S.scalar_type() == at::kFloat && S.is_contiguous(), "seed: S [B,H,W] fp32");
  const int64_t B = S.size(0), H = S.size(1), W = S.size(2);
  TORCH_CHECK(f.scalar_type() == at::kInt && f.numel() == B && f.is_contiguous(), "seed: f [B] int32");
  TORCH_CHECK(wt.dim() == 4 && wt.size(1) == 3 && wt.size(2) == 3 && is16(wt) && wt.is_contiguous(),
              "seed: wt [F,3,3,Cin] bf16 / fp16");
  const int64_t Cin = wt.size(3);
  TORCH_CHECK(out.scalar_type() == wt.scalar_type() && out.is_contiguous() && out.numel() == B * H * W * Cin,
              "seed: out [B,H,W,Cin] of wt's dtype");
  // f values >= F are clamped to F - 1 in the kernel; < 0 gives a zero map
  check_rc(dv::seed_deconv3x3_launch(S.data_ptr<float>(), f.data_ptr<int>(),
                                     reinterpret_cast<const uint16_t*>(wt.data_ptr()),
                                     reinterpret_cast<uint16_t*>(out.data_ptr()), (int)B, (int)H, (int)W, (int)Cin,
                                     (int)wt.size(0), f16(wt), cur_stream()),
           "seed_deconv3x3");
}

void deprocess_mosaic(Tensor recon, Tensor out, int64_t tiles, bool reverse, c10::optional<Tensor> stats) {
  check_cuda(recon, "recon");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(recon.device());
  TORCH_CHECK(recon.dim() == 4 && recon.size(3) == 3 && recon.scalar_type() == at::kFloat && recon.is_contiguous(),
              "deprocess: recon [B*tiles, H, W, 3] fp32");
  const int64_t BT = recon.size(0), H = recon.size(1), W = recon.size(2);
  TORCH_CHECK(tiles >= 1 && tiles <= 4 && BT % tiles == 0, "deprocess: tiles");
  const int64_t B = BT / tiles;
  const int64_t rows = (tiles + 1) / 2;
  TORCH_CHECK(out.scalar_type() == at::kByte && out.is_contiguous() && out.numel() == B * rows * H * 2 * W * 3,
              "deprocess: out [B, rows*H, 2*W, 3] u8");
  if (W % 4 != 0) {  // one block per image, two-pass statistics
    check_rc(dv::deprocess_mosaic_launch(recon.data_ptr<float>(), out.data_ptr<uint8_t>(), (int)B, (int)H, (int)W,
                                         (int)tiles, reverse ? 1 : 0, cur_stream()),
             "deprocess_mosaic");
    return;
  }
  Tensor st;
  if (stats.has_value()) {  // {sum, sum^2} per image, from the final conv's epilogue
    TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->is_contiguous() && stats->numel() == 2 * B &&
                    stats->device() == recon.device(),
                "deprocess: stats fp64 [B, 2]");
    st = *stats;
  } else {
    st = at::zeros({B, 2}, recon.options().dtype(at::kDouble));
    check_rc(dv::recon_stats_launch(recon.data_ptr<float>(), st.data_ptr<double>(), tiles * H * W * 3, (int)B,
                                    cur_stream()),
             "recon_stats");
  }
  check_rc(dv::deprocess_apply_launch(recon.data_ptr<float>(), st.data_ptr<double>(), out.data_ptr<uint8_t>(), (int)B,
                                      (int)H, (int)W, (int)tiles, reverse ? 1 : 0, cur_stream()),
           "deprocess_apply");
}

// blob: u8 [bytes] (device), table: int64 [B, 4] {offset, Hs, Ws, mode} (device; validated on the
// host by the caller against the blob size: runtime/staging.py), out: bf16 [B, OH, OW, Cpad] or
// u8 [B, OH, OW, 3]
void resize_batch(Tensor blob, Tensor table, Tensor out, int64_t max_end) {
  check_cuda(blob, "blob");
  check_cuda(table, "table");
  check_cuda(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(blob.device());
  TORCH_CHECK(blob.scalar_type() == at::kByte && blob.is_contiguous() && blob.dim() == 1, "resize_batch: blob u8 [bytes]");
  TORCH_CHECK(max_end <= blob.numel(), "resize_batch: table addresses past the blob");
  TORCH_CHECK(table.scalar_type() == at::kLong && table.is_contiguous() && table.dim() == 2 && table.size(1) == 4,
              "resize_batch: table int64 [B, 4]");
  TORCH_CHECK(out.dim() == 4 && out.is_contiguous() && out.size(0) == table.size(0), "resize_batch: out [B, OH, OW, C]");
  const bool u8 = out.scalar_type() == at::kByte;
  const bool f16 = out.scalar_type() == at::kHalf;
  TORCH_CHECK(u8 ? out.size(3) == 3 : ((out.scalar_type() == at::kBFloat16 || f16) && out.size(3) >= 3 &&
                                       reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0),
              "resize_batch: out u8 [..., 3] or bf16 / fp16 [..., Cpad]");
  check_rc(dv::resize_batch_launch(blob.data_ptr<uint8_t>(), reinterpret_cast<const long long*>(table.data_ptr<int64_t>()), (int)table.size(0), out.data_ptr(),
                                   (int)out.size(1), (int)out.size(2), (int)out.size(3), u8 ? 1 : (f16 ? 2 : 0), cur_stream()),
           "resize_batch");
}

void preprocess_u8(Tensor in, Tensor out) {
  check_cuda(in, "in");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(in.device());
  TORCH_CHECK(in.scalar_type() == at::kByte && in.is_contiguous() && in.dim() == 4 && in.size(3) == 3,
              "preprocess_u8: in u8 [B, H, W, 3]");
  const bool f16 = out.scalar_type() == at::kHalf;
  TORCH_CHECK((out.scalar_type() == at::kBFloat16 || f16) && out.is_contiguous() && out.dim() == 4 &&
                  out.size(0) == in.size(0) && out.size(1) == in.size(1) && out.size(2) == in.size(2) &&
                  out.size(3) >= 3 && reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0,
              "preprocess_u8: out bf16 / fp16 [B, H, W, Cpad]");
  check_rc(dv::preprocess_u8_launch(in.data_ptr<uint8_t>(), reinterpret_cast<uint16_t*>(out.data_ptr()),
                                    in.numel() / 3, (int)out.size(3), f16 ? 1 : 0, cur_stream()),
           "preprocess_u8");
}

void resize_preprocess(Tensor img, Tensor out, int64_t mode) {
  check_cuda(img, "img");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(img.device());
  TORCH_CHECK(img.dim() == 4 && img.size(3) == 3 && img.scalar_type() == at::kByte && img.is_contiguous(),
              "resize_preprocess: img [B, H, W, 3] u8");
  const bool f16 = out.scalar_type() == at::kHalf;
  TORCH_CHECK(out.dim() == 4 && (out.scalar_type() == at::kBFloat16 || f16) && out.is_contiguous() &&
                  out.size(0) == img.size(0),
              "resize_preprocess: out [B, OH, OW, Cpad] bf16 / fp16");
  const int64_t B = img.size(0), Hs = img.size(1), Ws = img.size(2), OH = out.size(1), OW = out.size(2),
                Cp = out.size(3);
  if (mode == 1) TORCH_CHECK(Hs == 2 * OH && Ws == 2 * OW, "area mode needs exact 2x");
  if (mode == 2) TORCH_CHECK(Hs == OH && Ws == OW, "copy mode needs equal size");
  TORCH_CHECK(Cp >= 3 && (Cp != 8 || reinterpret_cast<uintptr_t>(out.data_ptr()) % 16 == 0), "resize_preprocess: Cpad");
  check_rc(dv::resize_preprocess_launch(img.data_ptr<uint8_t>(), (int)B, (int)Hs, (int)Ws,
                                        reinterpret_cast<uint16_t*>(out.data_ptr()), (int)OH, (int)OW, (int)Cp,
                                        (int)mode, f16 ? 1 : 0, cur_stream()),
           "resize_preprocess");
}

// block1_conv2.down + block1_conv1.down tail: unpool (pooled x + codes) -> 3x3 conv 64 -> 64 -> ReLU ->
// Z = D W2^T (bf16 [N, H, W, 32]); false if the kernel does not take the shape (caller falls back)
bool conv_unpool_z(Tensor x, Tensor code, int64_t code_div, Tensor w, Tensor w2, Tensor z) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.size(3) == 64,
              "conv_unpool_z: x pooled bf16 [N, H/2, W/2, 64]");
  TORCH_CHECK(z.dim() == 4 && z.scalar_type() == at::kBFloat16 && z.is_contiguous() && z.size(0) == x.size(0) &&
                  z.size(1) == 2 * x.size(1) && z.size(2) == 2 * x.size(2) && z.size(3) == 32,
              "conv_unpool_z: z bf16 [N, H, W, 32]");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.is_contiguous() && code_div >= 1 && x.size(0) % code_div == 0 &&
                  code.numel() == x.numel() / code_div,
              "conv_unpool_z: code u8 [N/code_div, H/2, W/2, 64]");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 && w.is_contiguous() && w.dim() == 2 && w.size(0) == 64 &&
                  w.size(1) >= 576 && w.size(1) % 64 == 0,
              "conv_unpool_z: w bf16 [64, Kpad >= 576]");
  TORCH_CHECK(w2.scalar_type() == at::kBFloat16 && w2.is_contiguous() && w2.numel() == 32 * 64, "conv_unpool_z: w2 bf16 [32, 64]");
  check_cuda(code, "code");
  check_cuda(w, "w");
  check_cuda(w2, "w2");
  check_cuda(z, "z");
  dv::ConvArgs a{};
  a.N = (int)z.size(0); a.H = a.OH = (int)z.size(1); a.W = a.OW = (int)z.size(2); a.C = 64;
  a.OC = a.OCpad = 64; a.KH = a.KW = 3; a.stride = 1; a.pad_h = a.pad_w = 1;
  a.K = 576; a.Kpad = (int)w.size(1); a.M = a.N * a.H * a.W;
  a.relu = 1; a.relu_in = 1; a.code_div = (int)code_div; a.x_ld = 64; a.out_ld = 32;
  a.dtype = dv::DT_BF16;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.w = reinterpret_cast<const uint16_t*>(w.data_ptr());
  a.w2 = reinterpret_cast<const uint16_t*>(w2.data_ptr());
  a.code = code.data_ptr<uint8_t>();
  a.out = z.data_ptr();
  a.x_elems = avail_bytes(x) / 2;
  a.out_elems = avail_bytes(z) / 2;
  const int rc = dv::conv3x3_unpool_z_launch(a, cur_stream());
  if (rc == -4) return false;
  check_rc(rc, "conv_unpool_z");
  return true;
}

// fused VGG16 stem: x bf16 [N, H, W, 8] (preprocessed RGB, channels 3..7 zero) -> conv1 (w1 [64][>= 96],
// b1) + ReLU -> conv2 (w2 [64][>= 576], b2) + ReLU -> 2x2 max-pool: out bf16 [N, H/2, W/2, 64] + switch
// codes u8 (the layout conv(..., CONV_E_POOL) writes). false: shape unsupported (caller runs 2 launches)
bool conv_stem_pool(Tensor x, Tensor w1, c10::optional<Tensor> b1, Tensor w2, c10::optional<Tensor> b2, Tensor out,
                    Tensor out_code) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && x.scalar_type() == at::kBFloat16 && x.is_contiguous() && x.size(3) == 8,
              "conv_stem_pool: x bf16 [N, H, W, 8]");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2);
  TORCH_CHECK(H % 2 == 0 && W % 2 == 0, "conv_stem_pool: even H, W");
  TORCH_CHECK(out.dim() == 4 && out.scalar_type() == at::kBFloat16 && out.is_contiguous() && out.size(0) == N &&
                  out.size(1) == H / 2 && out.size(2) == W / 2 && out.size(3) == 64,
              "conv_stem_pool: out bf16 [N, H/2, W/2, 64]");
  TORCH_CHECK(out_code.scalar_type() == at::kByte && out_code.is_contiguous() && out_code.numel() == out.numel(),
              "conv_stem_pool: out_code u8 [N, H/2, W/2, 64]");
  TORCH_CHECK(w1.scalar_type() == at::kBFloat16 && w1.is_contiguous() && w1.dim() == 2 && w1.size(0) == 64 &&
                  w1.size(1) >= 96,
              "conv_stem_pool: w1 bf16 [64, Kpad >= 96]");
  TORCH_CHECK(w2.scalar_type() == at::kBFloat16 && w2.is_contiguous() && w2.dim() == 2 && w2.size(0) == 64 &&
                  w2.size(1) >= 576,
              "conv_stem_pool: w2 bf16 [64, Kpad >= 576]");
  for (const auto* b : {&b1, &b2})
    if (b->has_value())
      TORCH_CHECK((*b)->scalar_type() == at::kFloat && (*b)->is_contiguous() && (*b)->numel() >= 64 && (*b)->is_cuda(),
                  "conv_stem_pool: bias fp32 [>= 64] on the device");
  check_cuda(w1, "w1");
  check_cuda(w2, "w2");
  check_cuda(out, "out");
  check_cuda(out_code, "out_code");
  dv::ConvArgs a{};
  a.N = (int)N; a.H = a.OH = (int)H; a.W = a.OW = (int)W; a.C = 64;
  a.OC = a.OCpad = 64; a.KH = a.KW = 3; a.stride = 1; a.pad_h = a.pad_w = 1;
  a.K = 576; a.Kpad = (int)w2.size(1); a.M = (int)(N * H * W);
  a.relu = 1; a.code_div = 1; a.x_ld = 8; a.out_ld = 64;
  a.dtype = dv::DT_BF16;
  a.x = reinterpret_cast<const uint16_t*>(x.data_ptr());
  a.w = reinterpret_cast<const uint16_t*>(w2.data_ptr());
  a.bias = b2.has_value() ? b2->data_ptr<float>() : nullptr;
  a.w2 = reinterpret_cast<const uint16_t*>(w1.data_ptr());
  a.bias2 = b1.has_value() ? b1->data_ptr<float>() : nullptr;
  a.kpad2 = (int)w1.size(1);
  a.out = out.data_ptr();
  a.out_code = out_code.data_ptr<uint8_t>();
  a.x_elems = avail_bytes(x) / 2;
  a.out_elems = avail_bytes(out) / 2;
  const int rc = dv::conv3x3_stem_pool_launch(a, cur_stream());
  if (rc == -4) return false;
  check_rc(rc, "conv_stem_pool");
  return true;
}

// out fp32 [N, H, W, 3] = ReLU(9-tap shift-add of z [N, H, W, 32]); optional per-image stats
void zsum3x3(Tensor z, Tensor out, c10::optional<Tensor> stats, int64_t stats_div) {
  check_cuda(z, "z");
  check_cuda(out, "out");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(z.device());
  TORCH_CHECK(z.dim() == 4 && z.scalar_type() == at::kBFloat16 && z.is_contiguous() && z.size(3) == 32,
              "zsum3x3: z bf16 [N, H, W, 32]");
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() == z.numel() / 32 * 3,
              "zsum3x3: out fp32 [N, H, W, 3]");
  const int N = (int)z.size(0);
  double* st = nullptr;
  if (stats.has_value()) {
    check_cuda(*stats, "stats");
    TORCH_CHECK(stats->scalar_type() == at::kDouble && stats->is_contiguous() && stats_div >= 1 && N % stats_div == 0 &&
                    stats->numel() == 2 * (N / stats_div),
                "zsum3x3: stats fp64 [N/stats_div, 2]");
    check_rc((int)hipMemsetAsync(stats->data_ptr(), 0, stats->numel() * 8, cur_stream()), "stats memset");
    st = stats->data_ptr<double>();
  }
  check_rc(dv::zsum3x3_launch(reinterpret_cast<const uint16_t*>(z.data_ptr()), out.data_ptr<float>(), N,
                              (int)z.size(1), (int)z.size(2), st, (int)stats_div, cur_stream()),
           "zsum3x3");
}

void maxpool2x2(Tensor x, Tensor out, Tensor code) {
  check_cuda(x, "x");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(x.device());
  TORCH_CHECK(x.dim() == 4 && is16(x) && x.is_contiguous(), "maxpool: x NHWC bf16 / fp16");
  const int64_t N = x.size(0), H = x.size(1), W = x.size(2), C = x.size(3);
  TORCH_CHECK(out.scalar_type() == x.scalar_type() && out.is_contiguous() && out.numel() == N * (H / 2) * (W / 2) * C,
              "maxpool: out");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.is_contiguous() && code.numel() == out.numel(), "maxpool: code");
  check_rc(dv::maxpool2x2_launch(reinterpret_cast<const uint16_t*>(x.data_ptr()),
                                 reinterpret_cast<uint16_t*>(out.data_ptr()), code.data_ptr<uint8_t>(), (int)N, (int)H,
                                 (int)W, (int)C, f16(x), cur_stream()),
           "maxpool2x2");
}

void unpool2x2(Tensor p, Tensor code, Tensor out, int64_t code_div, bool relu) {
  check_cuda(p, "p");
  c10::hip::HIPGuardMasqueradingAsCUDA guard(p.device());
  // 16-bit moves + a sign-bit ReLU: the same kernel for bf16 and fp16
  TORCH_CHECK(out.dim() == 4 && is16(out) && out.is_contiguous(), "unpool: out NHWC bf16 / fp16");
  const int64_t N = out.size(0), H = out.size(1), W = out.size(2), C = out.size(3);
  TORCH_CHECK(p.scalar_type() == out.scalar_type() && p.is_contiguous() && p.numel() == N * (H / 2) * (W / 2) * C,
              "unpool: p");
  TORCH_CHECK(code_div >= 1 && N % code_div == 0, "unpool: code_div");
  TORCH_CHECK(code.scalar_type() == at::kByte && code.is_contiguous() && code.numel() == p.numel() / code_div,
              "unpool: code");
  check_rc(dv::unpool2x2_launch(reinterpret_cast<const uint16_t*>(p.data_ptr()), code.data_ptr<uint8_t>(),
                                reinterpret_cast<uint16_t*>(out.data_ptr()), (int)N, (int)H, (int)W, (int)C,
                                (int)code_div, relu ? 1 : 0, cur_stream()),
           "unpool2x2");
}


}  // namespace

// build provenance (_build.py): sha256 of the csrc tree + compile flags, found in the file by
// ops/native.py before it loads this module
#ifndef DV_SOURCE_HASH
#define DV_SOURCE_HASH "unknown"
#endif
static const char kSourceHash[] = "DV_SOURCE_HASH:" DV_SOURCE_HASH;

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("source_hash", [] { return std::string(kSourceHash + 15); }, "sha256 of the sources this binary was built from");
  m.def("subpixel_merge", &subpixel_merge, "strided-conv input gradient from its parity-class parts (+accumulate, emask)");
  m.def("sk_errors", &sk_errors, py::arg("reset") = false,
        "KW3P stream-K hand-offs that timed out since the last reset (their tiles are wrong)");
  m.doc() = "deconv_api_amd gfx950 (MI355X) HIP kernels";
  m.def("conv", &conv, "MFMA implicit-GEMM conv (fwd / unpool-gather / transposed; bf16/pool/f32 epilogues)",
        py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("out"), py::arg("out_code"), py::arg("code"),
        py::arg("mask"), py::arg("geom"), py::arg("amode"), py::arg("epi"), py::arg("impl"),
        py::arg("res") = py::none(), py::arg("emask") = py::none(), py::arg("stats") = py::none(),
        py::arg("stats_div") = 1, py::arg("ucode") = py::none(), py::arg("ucode_div") = 1,
        py::arg("relu_cols") = 0, py::arg("out2") = py::none(), py::arg("split_col") = 0,
        py::arg("obits") = py::none(), py::arg("ebits") = py::none());
  m.def("conv_group_begin", &conv_group_begin, "start recording groupable small-problem convs (this thread)");
  m.def("conv_group_pause", [](bool p) { g_group_paused = p; }, "suspend / resume recording (dependent convs)");
  m.def("conv_group_end", &conv_group_end, "launch the recorded convs as grouped kernels; returns the launch count");
  m.def("dma_tune", [](int64_t cfg, int64_t ks) { dv::conv_dma_tune((int)cfg, (int)ks); },
        "force the LDS-DMA conv tile config / split-K factor (0 = automatic); tuning only");
  m.def("pool", &pool, "k x k max/avg pooling forward/backward", py::arg("in"), py::arg("out"), py::arg("idx"),
        py::arg("kind"), py::arg("dir"), py::arg("geom"), py::arg("bias") = py::none(), py::arg("relu") = false,
        py::arg("accumulate") = false);
  m.def("subpixel_scatter", &subpixel_scatter, "input gradient of a stride-s 1x1 conv from its GEMM result");
  m.def("sumsq_core", &sumsq_core, "DeepDream loss: per-image partial sums of squares over the core");
  m.def("stem_conv", &stem_conv, "strided few-channel stem conv (direct VALU kernels), fwd (dir 0) / dgrad (dir 1)");
  m.def("sumsq_core_bwd", &sumsq_core_bwd, "DeepDream loss gradient (+ optional addend)", py::arg("x"),
        py::arg("scale"), py::arg("gx"), py::arg("b"), py::arg("addend") = py::none(), py::arg("part") = py::none());
  m.def("tile_gather", &tile_gather, "tiled DeepDream: rolled tile gather into the 16-bit network input", py::arg("x"),
        py::arg("xin"), py::arg("plan"), py::arg("shift"), py::arg("rank"), py::arg("world"), py::arg("k0") = 0);
  m.def("tile_pack", &tile_pack, "tiled DeepDream: owned-pixel gradient pack + unit loss / sum|g| tail", py::arg("g"),
        py::arg("pack"), py::arg("plan"), py::arg("lpart"), py::arg("lcoef"), py::arg("ucap"), py::arg("rank"),
        py::arg("world"), py::arg("k0") = 0);
  m.def("tile_update", &tile_update, "tiled DeepDream: normalize + update the image from every rank's packs");
  m.def("tile_pack_elems", &tile_pack_elems);
  m.def("dream_update", &dream_update, "fused DeepDream normalize + update + next network input");
  m.def("octave_resize", &octave_resize, "DeepDream octave transition: corner-aligned bilinear resize of (a + b - c)",
        py::arg("a"), py::arg("b"), py::arg("c"), py::arg("y"), py::arg("yin") = py::none());
  m.def("stem7_fwd", &stem7_fwd, "ResNet-50 conv1 forward (7x7 / 2, RGB -> 64) on the tap-paired MFMA kernel");
  m.def("stem_dgrad_fused", &stem_dgrad_fused, "fused GEMM + col2im input gradient of a 7x7/2 RGB stem conv");
  m.def("col2im", &col2im, "col2im of a strided few-channel conv's input gradient");
  m.def("jpeg_data_urls", &jpeg_data_urls, "native JPEG + base64/quote data URLs (GIL released)");
  m.def("softmax_rows", &softmax_rows, "row softmax (classifier head)");
  m.def("paced_copy", &paced_copy, "bench: CU-occupying copy paced to a link bandwidth (all-gather interference model)");
  m.def("jpeg_gpu", &jpeg_gpu, "GPU baseline JPEG scans of uint8 [B,H,W,3] (restart per MCU row)");
  m.def("data_url_b64decode", &data_url_b64decode, "data URL payload -> bytes (lenient base64, GIL released)");
  m.def("url_unquote_plus", &url_unquote_plus, "unquote_plus of an ASCII str -> bytes (GIL released)");
  m.def("jpeg_gpu_header", &jpeg_gpu_header, "SOI..SOS of the GPU encoder's streams");
  m.def("jpeg_gpu_max_width", &dv::jpeg_gpu_max_width, "widest image the GPU encoder takes");
  m.def("jpeg_gpu_data_urls", &jpeg_gpu_data_urls, "GPU scans -> data URLs (host base64, GIL released)");
  m.def("jpeg_encode", &jpeg_encode, "native baseline JPEG encode (GIL released)");
  m.def("channel_sum", &channel_sum);
  m.def("topk_pos", &topk_pos);
  m.def("seed_deconv3x3", &seed_deconv3x3);
  m.def("seed_map", &seed_map, "deconvnet seed maps (all / max, optional max-unpool for pool targets)");
  m.def("deprocess_mosaic", &deprocess_mosaic, py::arg("recon"), py::arg("out"), py::arg("tiles"), py::arg("reverse"),
        py::arg("stats") = py::none());
  m.def("resize_preprocess", &resize_preprocess);
  m.def("resize_batch", &resize_batch, "variable-size batch resize (+preprocess) from one staged blob");
  m.def("preprocess_u8", &preprocess_u8, "resized RGB u8 -> caffe-preprocessed bf16 network input");
  m.def("maxpool2x2", &maxpool2x2);
  m.def("unpool2x2", &unpool2x2);
  m.def("conv_stem_pool", &conv_stem_pool, "fused VGG16 stem: conv 8->64 -> conv 64->64 -> 2x2 max-pool + switches");
  m.def("conv_unpool_z", &conv_unpool_z, "unpool -> conv3x3 64->64 -> ReLU -> per-tap products of the next 64->3 conv");
  m.def("zsum3x3", &zsum3x3, "9-tap shift-add of a per-tap product map (+ ReLU, per-image stats)");
  m.attr("ARCH") = "gfx950";
}
