// Python bindings for the determined_amd HIP kernels (one in-tree .so: _hip_ops).
// Host-only translation unit: all device code lives in the *.hip files, which include
// only hip_runtime.h so they compile in seconds; this file carries the torch headers.
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include <hip/hip_runtime.h>

#include <cstring>
#include <map>
#include <mutex>
#include <vector>

namespace damd {
[[noreturn]] void launch_failed(hipError_t err, const char* func, const char* file, int line);  // common.h
constexpr int kMaxGroups = 8;
struct MTChunk {
  void* p;
  const void* g;
  float* s0;
  float* s1;
  void* p_lp;
  int32_t n;
  int32_t group;
};
struct GroupHyper {
  float lr[kMaxGroups];
  float wd[kMaxGroups];
  float beta1[kMaxGroups];
  float beta2[kMaxGroups];
  float eps[kMaxGroups];
  int32_t flag[kMaxGroups];
};
}  // namespace damd

using damd::GroupHyper;
using damd::MTChunk;

// launchers (optim.hip)
void damd_adam_launch(const void*, int, const GroupHyper&, const float*, const int32_t*, const float*, int,
                      int, int, int, hipStream_t);
void damd_sgd_launch(const void*, int, const GroupHyper&, const float*, const int32_t*, const float*, int,
                     int, int, int, int, hipStream_t);
void damd_l2norm_partial_launch(const void*, int, float*, int, hipStream_t);
void damd_finalize_launch(const float*, int, float, const float*, float, float*, int32_t*, float*, int,
                          hipStream_t);
void damd_step_incr_launch(float*, const int32_t*, hipStream_t);
void damd_scale_launch(const void*, int, const float*, int, hipStream_t);
// launchers (norm.hip)
void damd_norm_fwd_launch(const void*, const void*, const void*, void*, float*, float*, int64_t, int, float,
                          int, int, int, hipStream_t);
int damd_norm_bwd_blocks(int64_t);
int damd_norm_bwd_launch(const void*, const void*, const float*, const float*, const void*, void*, float*,
                         float*, int64_t, int, int, int, int, hipStream_t);
void damd_norm_wgrad_finalize_launch(const float*, const float*, int, int, void*, void*, int, hipStream_t);
int damd_resid_norm_supported(int);
void damd_resid_norm_fwd_launch(const void*, const void*, const void*, const void*, void*, void*, uint8_t*, float*,
                                float*, int64_t, int, float, float, uint32_t, const int64_t*, int, int, hipStream_t);
int damd_resid_norm_bwd_launch(const void*, const void*, const void*, const float*, const float*, const void*,
                               const uint8_t*, float, void*, void*, float*, float*, int64_t, int, int, int,
                               hipStream_t);
void damd_col_reduce_launch(const float*, float*, int, int, hipStream_t);
// launchers (conv_igemm.hip)
extern "C" int damd_conv_num_cfgs();
extern "C" int damd_conv_default_cfg(int, int64_t);
extern "C" int damd_conv_supported(int, int, int, int, int, int, int, int);
extern "C" int damd_conv_groups(int64_t, int, int, int, int);
extern "C" int damd_wgrad_num_cfgs();
extern "C" int damd_conv1x1_bwd_fused_supported(int, int);
extern "C" int damd_conv1x1_bwd_fused_blocks(int64_t);
extern "C" int damd_conv1x1_bwd_fused_launch(const void*, const void*, const float*, const void*, const void*,
                                             const void*, const float*, int64_t, void*, float*, float*, void*, int,
                                             int, int, hipStream_t);
extern "C" int damd_wgrad3x3_supported(int, int, int, int, int);
extern "C" int damd_wgrad3x3_num_cfgs();
extern "C" int damd_wgrad3x3_splits(int64_t, int, int, int, int, int, int);
extern "C" int damd_wgrad3x3_launch(const void*, const void*, float*, void*, int, int, int, int, int, int, int, int,
                                    hipStream_t);
extern "C" int damd_wgrad_supported(int, int, int);
extern "C" int damd_wgrad_splits(int64_t, int, int, int, int, int, int);
extern "C" int damd_wgrad_launch(const void*, const void*, float*, void*, int, int, int, int, int, int, int, int, int,
                                 int, int, int, hipStream_t);
extern "C" int damd_conv_fwd_launch(const void*, const void*, void*, float*, int, int, int, int, int, int, int, int,
                                    int, int, int, hipStream_t, int, const void*, const void*, const uint8_t*,
                                    const float*, const float*, const float*, int, const void*, const float*,
                                    const float*, const float*, void*, uint8_t*, float*, int*, int, int ophase = 0);
extern "C" int damd_conv_pro_supported(int, int, int, int, int, int, int);
extern "C" void damd_occupy_launch(int, double, int*, hipStream_t);
extern "C" int damd_conv_pro_supported_w(int, int, int, int, int, int, int, int);
extern "C" int64_t damd_conv_sk_ws_floats(int, int, int);
extern "C" int damd_conv_sk_flag_words();
extern "C" int damd_conv_cfg_is_sk(int);
// launchers (conv3x3v2.hip): zero-padded-halo 3x3 kernels, exposed as conv configs
// damd_conv_num_cfgs() .. + damd_v2_num_cfgs() - 1 (same launch contract as damd_conv_fwd_launch)
extern "C" int damd_v2_num_cfgs();
extern "C" int damd_v2_supported(int, int, int, int, int, int, int, int, int);
extern "C" int damd_v2_groups(int, int, int, int);
extern "C" int damd_v2_launch(const void*, const void*, void*, float*, int, int, int, int, int, int, int, int, int,
                              int, int, hipStream_t, int, const void*, const void*, const uint8_t*, const float*,
                              const float*, const float*, int, const void*, const float*, const float*, const float*,
                              void*, uint8_t*, float*, int*, int, int);
namespace {
int conv_num_cfgs_all() { return damd_conv_num_cfgs() + damd_v2_num_cfgs(); }
bool is_v2(int cfg) { return cfg >= damd_conv_num_cfgs(); }
int cfg_supported(int C, int K, int R, int S, int stride, int pad, int H, int W, int cfg) {
  if (cfg < 0 || cfg >= conv_num_cfgs_all()) return 0;
  return is_v2(cfg) ? damd_v2_supported(C, K, R, S, stride, pad, H, W, cfg - damd_conv_num_cfgs())
                    : damd_conv_supported(C, K, R, S, stride, pad, W, cfg);
}
int cfg_pro_supported(int C, int K, int R, int S, int stride, int pad, int H, int W, int cfg) {
  if (cfg < 0 || cfg >= conv_num_cfgs_all()) return 0;
  return is_v2(cfg) ? damd_v2_supported(C, K, R, S, stride, pad, H, W, cfg - damd_conv_num_cfgs())
                    : damd_conv_pro_supported_w(C, K, R, S, stride, pad, W, cfg);
}
int cfg_groups(int64_t M, int K, int W, int cfg, int groups_override, int64_t N, int64_t H) {
  return is_v2(cfg) ? damd_v2_groups(static_cast<int>(N), static_cast<int>(H), K, cfg - damd_conv_num_cfgs())
                    : damd_conv_groups(M, K, W, cfg, groups_override);
}
int cfg_launch(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K, int R, int S,
               int stride, int pad, int cfg, int groups, hipStream_t st, int epi, const void* d2, const void* yb,
               const uint8_t* mask, const float* mean, const float* scale, const float* shift, int pro,
               const void* p_res, const float* p_scale, const float* p_shift, const float* p_rscale, void* p_aout,
               uint8_t* p_mout, float* sk_ws, int* sk_flags, int d2hw, int ophase = 0) {
  if (is_v2(cfg))
    return damd_v2_launch(x, w, y, part, N, H, W, C, K, R, S, stride, pad, cfg - damd_conv_num_cfgs(), groups, st,
                          epi, d2, yb, mask, mean, scale, shift, pro, p_res, p_scale, p_shift, p_rscale, p_aout, p_mout,
                          sk_ws, sk_flags, d2hw, ophase);
  return damd_conv_fwd_launch(x, w, y, part, N, H, W, C, K, R, S, stride, pad, cfg, groups, st, epi, d2, yb, mask,
                              mean, scale, shift, pro, p_res, p_scale, p_shift, p_rscale, p_aout, p_mout, sk_ws,
                              sk_flags, d2hw, ophase);
}
}  // namespace
// launchers (bn.hip)
int damd_bn_num_blocks(int64_t, int);
void damd_bn_fwd_launch(const void*, const void*, void*, int64_t, int, const void*, const void*, float*, float*,
                        float, float, float*, float*, float*, float*, float*, int, int, int, hipStream_t, uint8_t*, const float*, int);
void damd_bn_bwd_from_part_launch(const void*, const void*, int64_t, int, const float*, const float*, const float*,
                                  const float*, int, float*, void*, void*, void*, int, int, hipStream_t);
void damd_bn_bwd_finalize_launch(const float*, int, int, int64_t, const float*, const float*, const float*, float*, void*,
                                 void*, int, hipStream_t);
void damd_bn_bwd_apply_coef_launch(const void*, const void*, int64_t, int, const float*, void*, int, hipStream_t);
void damd_bn_finalize_launch(const float*, int, int, int64_t, const void*, const void*, float*, float*, float, float,
                             float*, float*, float*, float*, int, hipStream_t);
void damd_bn_apply_only_launch(const void*, const void*, void*, int64_t, int, const float*, const float*, int, int,
                               hipStream_t);
void damd_bn_bwd_launch(const void*, const void*, const void*, int64_t, int, const float*, const float*,
                        const float*, const float*, float*, float*, void*, void*, void*, void*, int, int, int,
                        hipStream_t, const uint8_t*, const void*);
void damd_bn_pool_fwd_launch(const void*, void*, uint8_t*, int64_t, int, int, int, int, int, const void*, const void*,
                             float*, float*, float, float, float*, float*, float*, float*, float*, int, int, hipStream_t,
                             const float*, int, void*);
void damd_bn_pool_bwd_launch(const void*, const uint8_t*, const void*, int64_t, int, int, int, int, int, const float*,
                             const float*, const float*, const float*, float*, float*, void*, void*, void*, int, int,
                             hipStream_t, const void*, const void*);
void damd_hw_broadcast_launch(const void*, void*, int64_t, int64_t, int, float, int, hipStream_t);
void damd_stem_pool_bn_fwd_launch(const float*, int, int64_t, const void*, void*, int64_t, int, const void*,
                                  const void*, float*, float*, float, float, float*, float*, float*, float*, int,
                                  hipStream_t);
void damd_stem_pool_bn_bwd_launch(const void*, const void*, const void*, const float*, const float*, const float*,
                                  const float*, float*, float*, void*, void*, void*, int64_t, int64_t, int, int,
                                  hipStream_t);
// launchers (conv_stem.hip)
extern "C" int damd_stem_pool_supported(int64_t, int64_t);
extern "C" int damd_stem_pool_blocks(int64_t, int64_t, int64_t);
extern "C" void damd_stem_pool_fwd_launch(const void*, const void*, const void*, int, void*, uint8_t*, float*, int64_t,
                                          int, int, hipStream_t);
extern "C" void damd_stem_pool_bwd_launch(const void*, const void*, const void*, const uint8_t*, const float*, float*,
                                          void*, int, int64_t, int, int, hipStream_t);
extern "C" int damd_stem_supported(int64_t, int64_t);
extern "C" int damd_stem_fwd_blocks(int64_t, int);
extern "C" void damd_stem_fwd_launch(const void*, const void*, void*, float*, int64_t, int, int, hipStream_t);
extern "C" int damd_stem_wgrad_blocks(int64_t, int);
extern "C" void damd_stem_wgrad_launch(const void*, const void*, float*, void*, int, int64_t, int, int, hipStream_t);
// launchers (attention.hip)
extern "C" void damd_attn_fwd_launch(const void*, const void*, const void*, void*, float*, const int64_t*, int, int,
                                     int, int, float, int, const uint8_t*, int64_t, uint32_t, const int64_t*, float,
                                     hipStream_t);
extern "C" void damd_attn_bwd_launch(const void*, const void*, const void*, const void*, const void*, const float*,
                                     float*, float*, void*, void*, void*, const int64_t*, int, int, int, int, float,
                                     int, const uint8_t*, int64_t, uint32_t, const int64_t*, float, hipStream_t);
// launchers (fused.hip)
extern "C" void damd_lm_ce_fwd_launch(const void*, const int64_t*, int64_t, int, int, int, int64_t, float*, float*,
                                      hipStream_t);
extern "C" void damd_lm_ce_bwd_launch(const void*, const int64_t*, const float*, const float*, int64_t, int, int,
                                      int, int64_t, void*, hipStream_t);
extern "C" int damd_bias_grad_splits(int64_t, int);
extern "C" void damd_bias_grad_launch(const void*, int64_t, int, int, float*, void*, int, hipStream_t);
extern "C" void damd_gelu_fwd_launch(const void*, void*, int64_t, hipStream_t);
extern "C" void damd_gelu_bwd_bias_launch(const void*, const void*, void*, int64_t, int, int, float*, hipStream_t);
extern "C" void damd_debug_launch(float*, int, int, hipStream_t);

// common.h: every DAMD_LAUNCH / DAMD_CHECK failure in the device TUs ends here and becomes a
// c10::Error (Python RuntimeError) naming the launcher and source line.
[[noreturn]] void damd::launch_failed(hipError_t err, const char* func, const char* file, int line) {
  const char* base = std::strrchr(file, '/');
  TORCH_CHECK(false, "determined_amd kernel launch failed in ", func, " (", base ? base + 1 : file, ":", line,
              "): ", hipGetErrorName(err), ": ", hipGetErrorString(err));
  __builtin_unreachable();
}

namespace {

hipStream_t cur_stream() { return at::hip::getCurrentHIPStream().stream(); }

int dtype_code(const at::Tensor& t) {
  if (t.scalar_type() == at::kFloat) return 0;
  if (t.scalar_type() == at::kBFloat16) return 1;
  TORCH_CHECK(false, "determined_amd kernels support float32 and bfloat16 only, got ", t.scalar_type());
}

void check_cuda(const at::Tensor& t, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), what, " must be contiguous");
}

// Elementwise multi-tensor kernels only need dense storage (any memory format, e.g.
// channels-last conv weights) with identical strides across param / grad / state.
void check_dense_like(const at::Tensor& t, const at::Tensor& ref, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  TORCH_CHECK(t.is_non_overlapping_and_dense(), what, " must be dense (non-overlapping)");
  TORCH_CHECK(t.strides() == ref.strides(), what, " strides must match the parameter's");
}

const float* opt_fptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kFloat && t->is_cuda(), "expected a float32 GPU tensor");
  return t->data_ptr<float>();
}
int32_t* opt_iptr(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kInt && t->is_cuda(), "expected an int32 GPU tensor");
  return t->data_ptr<int32_t>();
}

// Builds the persistent chunk table for a list of same-dtype parameters.
// Returns a uint8 GPU tensor holding MTChunk[n_chunks]; n = numel / sizeof(MTChunk).
at::Tensor build_chunk_table(const std::vector<at::Tensor>& params, const std::vector<at::Tensor>& grads,
                             const std::vector<at::Tensor>& s0, const std::vector<at::Tensor>& s1,
                             const std::vector<at::Tensor>& lp, const std::vector<int64_t>& groups,
                             int64_t chunk_size) {
  const size_t n = params.size();
  TORCH_CHECK(grads.size() == n && groups.size() == n, "params/grads/groups length mismatch");
  TORCH_CHECK(s0.empty() || s0.size() == n, "state0 length mismatch");
  TORCH_CHECK(s1.empty() || s1.size() == n, "state1 length mismatch");
  TORCH_CHECK(lp.empty() || lp.size() == n, "low-precision copy length mismatch");
  TORCH_CHECK(chunk_size > 0 && chunk_size % 4 == 0, "chunk_size must be a positive multiple of 4");
  std::vector<MTChunk> table;
  at::Device dev = at::kCPU;
  for (size_t i = 0; i < n; ++i) {
    const auto& p = params[i];
    check_dense_like(p, p, "param");
    dev = p.device();
    const int64_t numel = p.numel();
    TORCH_CHECK(grads[i].numel() == numel, "grad numel mismatch at index ", i);
    check_dense_like(grads[i], p, "grad");
    if (!s0.empty()) check_dense_like(s0[i], p, "state0");
    if (!s1.empty()) check_dense_like(s1[i], p, "state1");
    if (!lp.empty()) check_dense_like(lp[i], p, "low-precision param");
    TORCH_CHECK(groups[i] >= 0 && groups[i] < damd::kMaxGroups, "group index out of range");
    const int64_t pe = p.element_size(), ge = grads[i].element_size();
    for (int64_t off = 0; off < numel; off += chunk_size) {
      MTChunk c;
      c.p = static_cast<char*>(p.data_ptr()) + off * pe;
      c.g = static_cast<const char*>(grads[i].data_ptr()) + off * ge;
      c.s0 = s0.empty() ? nullptr : s0[i].data_ptr<float>() + off;
      c.s1 = s1.empty() ? nullptr : s1[i].data_ptr<float>() + off;
      c.p_lp = lp.empty() ? nullptr : static_cast<char*>(lp[i].data_ptr()) + off * lp[i].element_size();
      c.n = static_cast<int32_t>(std::min<int64_t>(chunk_size, numel - off));
      c.group = static_cast<int32_t>(groups[i]);
      table.push_back(c);
    }
  }
  auto cpu = at::empty({static_cast<int64_t>(table.size() * sizeof(MTChunk))}, at::kByte);
  if (!table.empty()) std::memcpy(cpu.data_ptr(), table.data(), table.size() * sizeof(MTChunk));
  if (dev.is_cpu()) return cpu;
  return cpu.to(dev);
}

int64_t chunk_entry_bytes() { return sizeof(MTChunk); }

GroupHyper make_hyper(const std::vector<double>& lr, const std::vector<double>& wd,
                      const std::vector<double>& b1, const std::vector<double>& b2,
                      const std::vector<double>& eps, const std::vector<int64_t>& flag) {
  GroupHyper h{};
  TORCH_CHECK(lr.size() <= damd::kMaxGroups, "at most 8 param groups per fused launch");
  for (size_t i = 0; i < lr.size(); ++i) {
    h.lr[i] = static_cast<float>(lr[i]);
    h.wd[i] = static_cast<float>(wd.at(i));
    h.beta1[i] = static_cast<float>(b1.at(i));
    h.beta2[i] = static_cast<float>(b2.at(i));
    h.eps[i] = static_cast<float>(eps.at(i));
    h.flag[i] = static_cast<int32_t>(flag.at(i));
  }
  return h;
}

int n_chunks_of(const at::Tensor& table) {
  TORCH_CHECK(table.is_cuda() && table.scalar_type() == at::kByte, "chunk table must be a GPU uint8 tensor");
  return static_cast<int>(table.numel() / sizeof(MTChunk));
}

void adam_step(const at::Tensor& table, std::vector<double> lr, std::vector<double> wd, std::vector<double> b1,
               std::vector<double> b2, std::vector<double> eps, std::vector<int64_t> decoupled,
               const c10::optional<at::Tensor>& scale, const c10::optional<at::Tensor>& found_inf,
               const at::Tensor& step, bool maximize, int64_t p_dtype, int64_t g_dtype, bool has_lp) {
  TORCH_CHECK(step.scalar_type() == at::kFloat && step.is_cuda(), "step must be a float32 GPU scalar");
  const GroupHyper h = make_hyper(lr, wd, b1, b2, eps, decoupled);
  damd_adam_launch(table.data_ptr(), n_chunks_of(table), h, opt_fptr(scale), opt_iptr(found_inf),
                   step.data_ptr<float>(), maximize, p_dtype, g_dtype, has_lp, cur_stream());
}

void sgd_step(const at::Tensor& table, std::vector<double> lr, std::vector<double> wd, std::vector<double> mom,
              std::vector<double> damp, std::vector<int64_t> nesterov, const c10::optional<at::Tensor>& scale,
              const c10::optional<at::Tensor>& found_inf, const at::Tensor& step, bool maximize, int64_t p_dtype,
              int64_t g_dtype, bool has_lp, bool momentum) {
  TORCH_CHECK(step.scalar_type() == at::kFloat && step.is_cuda(), "step must be a float32 GPU scalar");
  std::vector<double> eps(lr.size(), 0.0);
  const GroupHyper h = make_hyper(lr, wd, mom, damp, eps, nesterov);
  damd_sgd_launch(table.data_ptr(), n_chunks_of(table), h, opt_fptr(scale), opt_iptr(found_inf),
                  step.data_ptr<float>(), maximize, p_dtype, g_dtype, has_lp, momentum, cur_stream());
}

void l2norm_partial(const at::Tensor& table, at::Tensor partial, int64_t g_dtype) {
  const int n = n_chunks_of(table);
  TORCH_CHECK(partial.scalar_type() == at::kFloat && partial.numel() >= n, "partial buffer too small");
  damd_l2norm_partial_launch(table.data_ptr(), n, partial.data_ptr<float>(), g_dtype, cur_stream());
}

void finalize(const at::Tensor& partial, int64_t n_partial, double inv_loss_scale,
              const c10::optional<at::Tensor>& inv_scale, double max_norm, at::Tensor out,
              const c10::optional<at::Tensor>& found_inf, const c10::optional<at::Tensor>& step, bool check_inf) {
  TORCH_CHECK(out.scalar_type() == at::kFloat && out.numel() >= 2, "out must hold 2 floats");
  float* step_ptr = nullptr;
  if (step.has_value() && step->defined()) step_ptr = step->data_ptr<float>();
  damd_finalize_launch(partial.data_ptr<float>(), static_cast<int>(n_partial), static_cast<float>(inv_loss_scale),
                       opt_fptr(inv_scale), static_cast<float>(max_norm), out.data_ptr<float>(),
                       opt_iptr(found_inf), step_ptr, check_inf, cur_stream());
}

void step_incr(at::Tensor step, const c10::optional<at::Tensor>& found_inf) {
  damd_step_incr_launch(step.data_ptr<float>(), opt_iptr(found_inf), cur_stream());
}

void scale_grads(const at::Tensor& table, const at::Tensor& scale, int64_t g_dtype) {
  damd_scale_launch(table.data_ptr(), n_chunks_of(table), scale.data_ptr<float>(), g_dtype, cur_stream());
}

// ----------------------------------------------------------------------------- norms
std::vector<at::Tensor> norm_fwd(const at::Tensor& x, const at::Tensor& gamma, const c10::optional<at::Tensor>& beta,
                                 double eps, bool rms) {
  check_cuda(x, "x");
  check_cuda(gamma, "gamma");
  const int64_t H = gamma.numel();
  TORCH_CHECK(x.size(-1) == H, "last dim of x must equal normalized size");
  const int64_t rows = x.numel() / H;
  auto y = at::empty_like(x);
  auto opts = x.options().dtype(at::kFloat);
  auto rstd = at::empty({rows}, opts);
  at::Tensor mean = rms ? at::empty({0}, opts) : at::empty({rows}, opts);
  const void* bp = nullptr;
  if (!rms && beta.has_value() && beta->defined()) {
    check_cuda(*beta, "beta");
    TORCH_CHECK(beta->scalar_type() == gamma.scalar_type(), "beta dtype must match gamma");
    bp = beta->data_ptr();
  }
  if (rows > 0)
    damd_norm_fwd_launch(x.data_ptr(), gamma.data_ptr(), bp, y.data_ptr(), rms ? nullptr : mean.data_ptr<float>(),
                         rstd.data_ptr<float>(), rows, static_cast<int>(H), static_cast<float>(eps), rms,
                         dtype_code(x), dtype_code(gamma), cur_stream());
  return {y, mean, rstd};
}

std::vector<at::Tensor> norm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& mean,
                                 const at::Tensor& rstd, const at::Tensor& gamma, bool rms) {
  check_cuda(dy, "dy");
  check_cuda(x, "x");
  const int64_t H = gamma.numel();
  const int64_t rows = x.numel() / H;
  auto dx = at::empty_like(x);
  auto fopts = x.options().dtype(at::kFloat);
  // weight gradients come out in the weight dtype, finalized inside the backward kernel
  // (register-resident path) or by one finalize pass over per-wave partials (generic path)
  auto dgamma = at::empty({H}, gamma.options());
  auto dbeta = rms ? at::empty({0}, gamma.options()) : at::empty({H}, gamma.options());
  if (rows > 0) {
    const int cap = damd_norm_bwd_blocks(rows) * 4;
    auto part_g = at::empty({cap, H}, fopts);
    auto part_b = rms ? at::empty({0}, fopts) : at::empty({cap, H}, fopts);
    const int W = damd_norm_bwd_launch(dy.data_ptr(), x.data_ptr(), rms ? nullptr : mean.data_ptr<float>(),
                                       rstd.data_ptr<float>(), gamma.data_ptr(), dx.data_ptr(),
                                       part_g.data_ptr<float>(), rms ? nullptr : part_b.data_ptr<float>(), rows,
                                       static_cast<int>(H), rms, dtype_code(x), dtype_code(gamma), cur_stream());
    damd_norm_wgrad_finalize_launch(part_g.data_ptr<float>(), rms ? nullptr : part_b.data_ptr<float>(), W,
                                    static_cast<int>(H), dgamma.data_ptr(), rms ? nullptr : dbeta.data_ptr(),
                                    dtype_code(gamma), cur_stream());
  } else {
    dgamma.zero_();
    dbeta.zero_();
  }
  return {dx, dgamma, dbeta};
}

// ----------------------------------------------------------------------------- BatchNorm(+add)+ReLU, NHWC
bool nhwc_dense(const at::Tensor& t) {
  if (t.dim() == 4) return t.is_contiguous(at::MemoryFormat::ChannelsLast);
  return t.is_contiguous();
}

void check_bn_tensor(const at::Tensor& t, const at::Tensor& ref, const char* what) {
  TORCH_CHECK(t.is_cuda(), what, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == ref.scalar_type(), what, " dtype must match x");
  TORCH_CHECK(t.sizes() == ref.sizes(), what, " shape must match x");
  TORCH_CHECK(nhwc_dense(t), what, " must be channels-last dense");
  TORCH_CHECK((reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0, what, " must be 16-byte aligned");
}

int64_t bn_channels(const at::Tensor& x) { return x.dim() == 4 ? x.size(1) : x.size(-1); }

bool bn_supported(const at::Tensor& x) {
  const int64_t C = bn_channels(x);
  const int64_t tpr = C / 8;
  return x.is_cuda() && (C % 8) == 0 && tpr > 0 && (tpr & (tpr - 1)) == 0 && nhwc_dense(x) &&
         (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
         (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat);
}

std::vector<at::Tensor> bn_act_fwd(const at::Tensor& x, const at::Tensor& weight, const at::Tensor& bias,
                                   const c10::optional<at::Tensor>& running_mean,
                                   const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                                   const c10::optional<at::Tensor>& residual, bool relu, bool want_mask,
                                   const c10::optional<at::Tensor>& stats_part) {
  TORCH_CHECK(bn_supported(x), "bn_act_fwd: unsupported input layout/shape");
  const int64_t C = bn_channels(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(weight.numel() == C && bias.numel() == C && weight.scalar_type() == bias.scalar_type(),
              "weight/bias must have C elements and one dtype");
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_bn_tensor(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    TORCH_CHECK(running_mean->scalar_type() == at::kFloat && running_var->scalar_type() == at::kFloat,
                "running stats must be float32");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  auto fopts = x.options().dtype(at::kFloat);
  // stats_part: (sum, sum sq) partials [nb, 2, C] the producer of x already computed (conv_fwd)
  const float* pre = nullptr;
  int pre_nb = 0;
  if (stats_part.has_value() && stats_part->defined()) {
    TORCH_CHECK(stats_part->scalar_type() == at::kFloat && stats_part->dim() == 3 && stats_part->size(1) == 2 &&
                stats_part->size(2) == C && stats_part->is_contiguous() && stats_part->device() == x.device(),
                "bn_act_fwd: stats_part must be a float32 [nb, 2, C] tensor");
    pre = stats_part->data_ptr<float>();
    pre_nb = static_cast<int>(stats_part->size(0));
  }
  const int nb = pre ? 1 : damd_bn_num_blocks(M, static_cast<int>(C));
  auto part = at::empty({nb, 2, C}, fopts);
  auto stats = at::empty({4, C}, fopts);  // mean, invstd, scale, shift
  auto y = at::empty_like(x);
  // ReLU bit mask (1 byte per 8 channels) for the residual+ReLU case: the backward reads it
  // instead of the residual tensor
  const bool mk = want_mask && relu && rp != nullptr;
  at::Tensor mask = mk ? at::empty({M * C / 8}, x.options().dtype(at::kByte)) : at::empty({0}, x.options().dtype(at::kByte));
  damd_bn_fwd_launch(x.data_ptr(), rp, y.data_ptr(), M, static_cast<int>(C), weight.data_ptr(), bias.data_ptr(), rm, rv,
                     static_cast<float>(momentum), static_cast<float>(eps), part.data_ptr<float>(),
                     stats[0].data_ptr<float>(), stats[1].data_ptr<float>(), stats[2].data_ptr<float>(),
                     stats[3].data_ptr<float>(), relu, dtype_code(x), dtype_code(weight), cur_stream(),
                     mk ? mask.data_ptr<uint8_t>() : nullptr, pre, pre_nb);
  return {y, stats, mask};
}

at::Tensor bn_apply(const at::Tensor& x, const at::Tensor& scale, const at::Tensor& shift,
                    const c10::optional<at::Tensor>& residual, bool relu) {
  TORCH_CHECK(bn_supported(x), "bn_apply: unsupported input layout/shape");
  const int64_t C = bn_channels(x);
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_bn_tensor(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  auto y = at::empty_like(x);
  auto sc = scale.to(at::kFloat).contiguous();
  auto sh = shift.to(at::kFloat).contiguous();
  damd_bn_apply_only_launch(x.data_ptr(), rp, y.data_ptr(), x.numel() / C, static_cast<int>(C), sc.data_ptr<float>(),
                            sh.data_ptr<float>(), relu, dtype_code(x), cur_stream());
  return y;
}

std::vector<at::Tensor> bn_act_bwd(const at::Tensor& dy, const at::Tensor& x,
                                   const c10::optional<at::Tensor>& residual, const at::Tensor& stats,
                                   const at::Tensor& weight, bool relu, bool need_dres,
                                   const c10::optional<at::Tensor>& mask, const c10::optional<at::Tensor>& dy2) {
  check_bn_tensor(dy, x, "dy");
  const int64_t C = bn_channels(x);
  const int64_t M = x.numel() / C;
  const void* rp = nullptr;
  if (residual.has_value() && residual->defined()) {
    check_bn_tensor(*residual, x, "residual");
    rp = residual->data_ptr();
  }
  const uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined() && mask->numel() > 0) {
    TORCH_CHECK(relu && mask->scalar_type() == at::kByte && mask->is_contiguous() && mask->numel() == M * C / 8 &&
                mask->device() == x.device(), "bn_act_bwd: mask must be a uint8 [M*C/8] tensor (ReLU path)");
    mp = mask->data_ptr<uint8_t>();
  }
  // dy2: gradient of the output's second consumer (ops/bn.py split_grad), summed in-kernel
  const void* d2 = nullptr;
  if (dy2.has_value() && dy2->defined()) {
    TORCH_CHECK(mp != nullptr, "bn_act_bwd: a second gradient needs the masked ReLU path");
    check_bn_tensor(*dy2, x, "dy2");
    d2 = dy2->data_ptr();
  }
  auto fopts = x.options().dtype(at::kFloat);
  const int nb = damd_bn_num_blocks(M, static_cast<int>(C));
  auto part = at::empty({nb, 2, C}, fopts);
  auto coef = at::empty({3, C}, fopts);
  auto dgamma = at::empty({C}, weight.options());
  auto dbeta = at::empty({C}, weight.options());
  auto dx = at::empty_like(x);
  // dres == dy' (masked dy).  Without ReLU it is dy itself: no kernel write needed.
  const bool write_dres = need_dres && relu;
  at::Tensor dres = write_dres ? at::empty_like(x) : (need_dres ? dy : at::Tensor());
  damd_bn_bwd_launch(dy.data_ptr(), x.data_ptr(), rp, M, static_cast<int>(C), stats[0].data_ptr<float>(),
                     stats[1].data_ptr<float>(), stats[2].data_ptr<float>(), stats[3].data_ptr<float>(),
                     part.data_ptr<float>(), coef.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(),
                     dx.data_ptr(), write_dres ? dres.data_ptr() : nullptr, relu, dtype_code(x), dtype_code(weight),
                     cur_stream(), mp, d2);
  return {dx, dgamma, dbeta, dres};
}

// BN backward (no ReLU, no residual) without its apply pass: reduce + finalize of dz over x ->
// (coef [3, C] with dx = A*dz + B*x + Cc, dgamma, dbeta); the apply runs in the consumer's operand
// staging (conv_fwd_pro2, ops/conv.py _LazyBNGrad).
std::vector<at::Tensor> bn_bwd_coef(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& stats,
                                    const at::Tensor& weight) {
  check_bn_tensor(dz, x, "dz");
  const int64_t C = bn_channels(x);
  const int64_t M = x.numel() / C;
  auto fopts = x.options().dtype(at::kFloat);
  const int nb = damd_bn_num_blocks(M, static_cast<int>(C));
  auto part = at::empty({nb, 2, C}, fopts);
  auto coef = at::empty({3, C}, fopts);
  auto dgamma = at::empty({C}, weight.options());
  auto dbeta = at::empty({C}, weight.options());
  damd_bn_bwd_launch(dz.data_ptr(), x.data_ptr(), nullptr, M, static_cast<int>(C), stats[0].data_ptr<float>(),
                     stats[1].data_ptr<float>(), stats[2].data_ptr<float>(), stats[3].data_ptr<float>(),
                     part.data_ptr<float>(), coef.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(), nullptr,
                     nullptr, 0, dtype_code(x), dtype_code(weight), cur_stream(), nullptr, nullptr);
  return {coef, dgamma, dbeta};
}

// BN backward finalize only: (coef [3, C] = A, B, Cc with dx = A*dz + B*x + Cc, dgamma, dbeta)
std::vector<at::Tensor> bn_bwd_finalize_part(const at::Tensor& x, const at::Tensor& stats, const at::Tensor& weight,
                                             const at::Tensor& part) {
  TORCH_CHECK(bn_supported(x), "bn_bwd_finalize_part: unsupported x");
  const int64_t C = bn_channels(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.dim() == 3 && part.size(1) == 2 && part.size(2) == C &&
              part.is_contiguous(), "bn_bwd_finalize_part: part must be float32 [nb, 2, C]");
  auto coef = at::empty({3, C}, x.options().dtype(at::kFloat));
  auto dgamma = at::empty({C}, weight.options());
  auto dbeta = at::empty({C}, weight.options());
  damd_bn_bwd_finalize_launch(part.data_ptr<float>(), static_cast<int>(part.size(0)), static_cast<int>(C), M,
                              stats[0].data_ptr<float>(), stats[1].data_ptr<float>(), stats[2].data_ptr<float>(),
                              coef.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(), dtype_code(weight),
                              cur_stream());
  return {coef, dgamma, dbeta};
}

// dx = coef[0] * dz + coef[1] * x + coef[2] (the BN backward apply pass, no mask)
at::Tensor bn_bwd_apply_coef(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& coef) {
  check_bn_tensor(dz, x, "dz");
  TORCH_CHECK(bn_supported(x), "bn_bwd_apply_coef: unsupported x");
  const int64_t C = bn_channels(x);
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.numel() == 3 * C && coef.is_contiguous(), "bn_bwd_apply_coef: coef");
  auto dx = at::empty_like(x);
  damd_bn_bwd_apply_coef_launch(dz.data_ptr(), x.data_ptr(), x.numel() / C, static_cast<int>(C), coef.data_ptr<float>(),
                                dx.data_ptr(), dtype_code(x), cur_stream());
  return dx;
}

// BN forward statistics (mean, invstd, scale, shift) [4, C] from producer partials [nb, 2, C]
// of a tensor with M rows; updates the running statistics.
at::Tensor bn_finalize_part(const at::Tensor& part, int64_t M, const at::Tensor& weight, const at::Tensor& bias,
                            const c10::optional<at::Tensor>& running_mean, const c10::optional<at::Tensor>& running_var,
                            double momentum, double eps) {
  TORCH_CHECK(part.is_cuda() && part.scalar_type() == at::kFloat && part.dim() == 3 && part.size(1) == 2 &&
              part.is_contiguous(), "bn_finalize_part: part must be float32 [nb, 2, C]");
  const int64_t C = part.size(2);
  TORCH_CHECK(weight.numel() == C && bias.numel() == C && weight.scalar_type() == bias.scalar_type(),
              "bn_finalize_part: weight/bias must have C elements");
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    TORCH_CHECK(running_mean->scalar_type() == at::kFloat && running_var->scalar_type() == at::kFloat,
                "running stats must be float32");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  auto stats = at::empty({4, C}, part.options());
  damd_bn_finalize_launch(part.data_ptr<float>(), static_cast<int>(part.size(0)), static_cast<int>(C), M,
                          weight.data_ptr(), bias.data_ptr(), rm, rv, static_cast<float>(momentum),
                          static_cast<float>(eps), stats[0].data_ptr<float>(), stats[1].data_ptr<float>(),
                          stats[2].data_ptr<float>(), stats[3].data_ptr<float>(), dtype_code(weight), cur_stream());
  return stats;
}

// BN backward from producer-computed reduce partials (conv_dgrad_bn): dz already carries the
// ReLU mask; returns (dx, dgamma, dbeta).
std::vector<at::Tensor> bn_bwd_from_part(const at::Tensor& dz, const at::Tensor& x, const at::Tensor& stats,
                                         const at::Tensor& weight, const at::Tensor& part) {
  check_bn_tensor(dz, x, "dz");
  TORCH_CHECK(bn_supported(x), "bn_bwd_from_part: unsupported x");
  const int64_t C = bn_channels(x);
  const int64_t M = x.numel() / C;
  TORCH_CHECK(part.scalar_type() == at::kFloat && part.dim() == 3 && part.size(1) == 2 && part.size(2) == C &&
              part.is_contiguous(), "bn_bwd_from_part: part must be float32 [nb, 2, C]");
  auto coef = at::empty({3, C}, x.options().dtype(at::kFloat));
  auto dgamma = at::empty({C}, weight.options());
  auto dbeta = at::empty({C}, weight.options());
  auto dx = at::empty_like(x);
  damd_bn_bwd_from_part_launch(dz.data_ptr(), x.data_ptr(), M, static_cast<int>(C), stats[0].data_ptr<float>(),
                               stats[1].data_ptr<float>(), stats[2].data_ptr<float>(), part.data_ptr<float>(),
                               static_cast<int>(part.size(0)), coef.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(),
                               dx.data_ptr(), dtype_code(x), dtype_code(weight), cur_stream());
  return {dx, dgamma, dbeta};
}

// ---------------------------------------------------------------- residual add + dropout + LayerNorm
// optional device-side dropout seed: a 1-element int64 tensor on x's device, read by the kernel at run time
const int64_t* seed_ptr(const c10::optional<at::Tensor>& t, const at::Tensor& x) {
  if (!t.has_value() || !t->defined()) return nullptr;
  TORCH_CHECK(t->scalar_type() == at::kLong && t->numel() >= 1 && t->device() == x.device(),
              "seed_t: int64 tensor on the input's device");
  return t->data_ptr<int64_t>();
}

bool resid_norm_supported(const at::Tensor& x) {
  return x.is_cuda() && x.is_contiguous() && (x.scalar_type() == at::kBFloat16 || x.scalar_type() == at::kFloat) &&
         damd_resid_norm_supported(static_cast<int>(x.size(-1)));
}

// s = x + dropout(branch, p); y = LayerNorm(s).  Returns (s, y, mean, rstd, keep bits).
std::vector<at::Tensor> resid_norm_fwd(const at::Tensor& x, const at::Tensor& branch, const at::Tensor& gamma,
                                       const c10::optional<at::Tensor>& beta, double eps, double p, int64_t seed,
                                       const c10::optional<at::Tensor>& seed_t) {
  TORCH_CHECK(resid_norm_supported(x), "resid_norm_fwd: unsupported input");
  TORCH_CHECK(branch.sizes() == x.sizes() && branch.scalar_type() == x.scalar_type() && branch.is_contiguous(),
              "resid_norm_fwd: branch must match x");
  const int64_t H = x.size(-1), rows = x.numel() / H;
  TORCH_CHECK(gamma.numel() == H, "gamma must have H elements");
  auto fopts = x.options().dtype(at::kFloat);
  auto sum = at::empty_like(x);
  auto y = at::empty_like(x);
  auto mean = at::empty({rows}, fopts);
  auto rstd = at::empty({rows}, fopts);
  auto mask = at::empty({x.numel() / 8}, x.options().dtype(at::kByte));
  const void* bp = beta.has_value() && beta->defined() ? beta->data_ptr() : nullptr;
  damd_resid_norm_fwd_launch(x.data_ptr(), branch.data_ptr(), gamma.data_ptr(), bp, sum.data_ptr(), y.data_ptr(),
                             mask.data_ptr<uint8_t>(), mean.data_ptr<float>(), rstd.data_ptr<float>(), rows,
                             static_cast<int>(H), static_cast<float>(eps), static_cast<float>(p),
                             static_cast<uint32_t>(seed), seed_ptr(seed_t, x), dtype_code(x), dtype_code(gamma),
                             cur_stream());
  return {sum, y, mean, rstd, mask};
}

// Returns (d residual input, d branch, dgamma, dbeta).
std::vector<at::Tensor> resid_norm_bwd(const at::Tensor& dy, const c10::optional<at::Tensor>& dres,
                                       const at::Tensor& s, const at::Tensor& mean, const at::Tensor& rstd,
                                       const at::Tensor& gamma, const at::Tensor& mask, double p, bool has_beta) {
  TORCH_CHECK(dy.sizes() == s.sizes() && dy.is_contiguous() && dy.scalar_type() == s.scalar_type(), "bad dy");
  const void* rp = nullptr;
  if (dres.has_value() && dres->defined()) {
    TORCH_CHECK(dres->sizes() == s.sizes() && dres->is_contiguous() && dres->scalar_type() == s.scalar_type(), "bad dres");
    rp = dres->data_ptr();
  }
  const int64_t H = s.size(-1), rows = s.numel() / H;
  TORCH_CHECK(mask.numel() == s.numel() / 8 && mask.scalar_type() == at::kByte, "bad keep-bit tensor");
  auto fopts = s.options().dtype(at::kFloat);
  auto dx = at::empty_like(s);
  auto dbranch = at::empty_like(s);
  const int cap = damd_norm_bwd_blocks(rows);
  auto part_g = at::empty({cap, H}, fopts);
  auto part_b = at::empty({cap, H}, fopts);  // the LayerNorm backward always writes both partial sets
  const int W = damd_resid_norm_bwd_launch(dy.data_ptr(), rp, s.data_ptr(), mean.data_ptr<float>(),
                                           rstd.data_ptr<float>(), gamma.data_ptr(), mask.data_ptr<uint8_t>(),
                                           static_cast<float>(p), dx.data_ptr(), dbranch.data_ptr(),
                                           part_g.data_ptr<float>(), part_b.data_ptr<float>(), rows,
                                           static_cast<int>(H), dtype_code(s), dtype_code(gamma), cur_stream());
  auto dgamma = at::empty({H}, gamma.options());
  auto dbeta = has_beta ? at::empty({H}, gamma.options()) : at::empty({0}, gamma.options());
  damd_norm_wgrad_finalize_launch(part_g.data_ptr<float>(), has_beta ? part_b.data_ptr<float>() : nullptr, W,
                                  static_cast<int>(H), dgamma.data_ptr(), has_beta ? dbeta.data_ptr() : nullptr,
                                  dtype_code(gamma), cur_stream());
  return {dx, dbranch, dgamma, dbeta};
}

// ---------------------------------------------------------------- ResNet stem: BN + ReLU + MaxPool(3, 2, 1)
// x: [N, C, H, W] channels-last (NHWC storage); returns (y [N, C, OH, OW] channels-last, argmax
// uint8 [N*OH*OW*C], stats [4, C]).
std::vector<at::Tensor> bn_pool_fwd(const at::Tensor& x, const at::Tensor& weight, const at::Tensor& bias,
                                    const c10::optional<at::Tensor>& running_mean,
                                    const c10::optional<at::Tensor>& running_var, double momentum, double eps,
                                    const c10::optional<at::Tensor>& stats_part) {
  TORCH_CHECK(x.dim() == 4 && bn_supported(x), "bn_pool_fwd: need a 4-d channels-last tensor with C % 8 == 0");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  TORCH_CHECK(weight.numel() == C && bias.numel() == C, "weight/bias must have C elements");
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    TORCH_CHECK(running_mean->scalar_type() == at::kFloat && running_var->scalar_type() == at::kFloat,
                "running stats must be float32");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  auto fopts = x.options().dtype(at::kFloat);
  const int nb = damd_bn_num_blocks(N * H * W, static_cast<int>(C));
  auto part = at::empty({nb, 2, C}, fopts);
  auto stats = at::empty({4, C}, fopts);
  auto y = at::empty({N, C, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto idx = at::empty({N * OH * OW * C}, x.options().dtype(at::kByte));
  // input value at each window's argmax: lets the backward reduce run in the pooled domain
  auto xarg = at::empty_like(y);
  // stats_part: (sum, sum sq) partials [nb, 2, C] already produced with x (stem_conv_fwd)
  const float* pre = nullptr;
  int pre_nb = 0;
  if (stats_part.has_value() && stats_part->defined()) {
    TORCH_CHECK(stats_part->scalar_type() == at::kFloat && stats_part->dim() == 3 && stats_part->size(1) == 2 &&
                stats_part->size(2) == C && stats_part->is_contiguous() && stats_part->device() == x.device(),
                "bn_pool_fwd: stats_part must be a float32 [nb, 2, C] tensor");
    pre = stats_part->data_ptr<float>();
    pre_nb = static_cast<int>(stats_part->size(0));
  }
  TORCH_CHECK(N * OH * OW * C < (int64_t{1} << 31), "bn_pool_fwd: pooled tensor too large (32-bit indexing)");
  damd_bn_pool_fwd_launch(x.data_ptr(), y.data_ptr(), idx.data_ptr<uint8_t>(), N, static_cast<int>(H), static_cast<int>(W),
                          static_cast<int>(C), static_cast<int>(OH), static_cast<int>(OW), weight.data_ptr(),
                          bias.data_ptr(), rm, rv, static_cast<float>(momentum), static_cast<float>(eps),
                          part.data_ptr<float>(), stats[0].data_ptr<float>(), stats[1].data_ptr<float>(),
                          stats[2].data_ptr<float>(), stats[3].data_ptr<float>(), dtype_code(x), dtype_code(weight),
                          cur_stream(), pre, pre_nb, xarg.data_ptr());
  return {y, idx, stats, xarg};
}

std::vector<at::Tensor> bn_pool_bwd(const at::Tensor& dp, const at::Tensor& idx, const at::Tensor& x,
                                    const at::Tensor& stats, const at::Tensor& weight,
                                    const c10::optional<at::Tensor>& dp2, const c10::optional<at::Tensor>& xarg) {
  TORCH_CHECK(x.dim() == 4 && bn_supported(x), "bn_pool_bwd: bad x");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t OH = (H + 2 - 3) / 2 + 1, OW = (W + 2 - 3) / 2 + 1;
  TORCH_CHECK(dp.dim() == 4 && dp.size(0) == N && dp.size(1) == C && dp.size(2) == OH && dp.size(3) == OW &&
              nhwc_dense(dp) && dp.scalar_type() == x.scalar_type(), "bn_pool_bwd: dp must be [N, C, OH, OW] channels-last");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == N * OH * OW * C && idx.is_contiguous(),
              "bn_pool_bwd: bad argmax tensor");
  auto fopts = x.options().dtype(at::kFloat);
  const int nb = damd_bn_num_blocks(N * H * W, static_cast<int>(C));
  auto part = at::empty({nb, 2, C}, fopts);
  auto coef = at::empty({3, C}, fopts);
  auto dgamma = at::empty({C}, weight.options());
  auto dbeta = at::empty({C}, weight.options());
  auto dx = at::empty_like(x);
  const void* d2 = nullptr;
  if (dp2.has_value() && dp2->defined()) {
    TORCH_CHECK(dp2->sizes() == dp.sizes() && dp2->strides() == dp.strides() &&
                dp2->scalar_type() == dp.scalar_type() && dp2->device() == dp.device(),
                "bn_pool_bwd: dp2 must match dp");
    d2 = dp2->data_ptr();
  }
  const void* xa = nullptr;
  if (xarg.has_value() && xarg->defined()) {
    TORCH_CHECK(xarg->sizes() == dp.sizes() && xarg->strides() == dp.strides() &&
                xarg->scalar_type() == x.scalar_type() && xarg->device() == dp.device(),
                "bn_pool_bwd: xarg must match dp");
    xa = xarg->data_ptr();
  }
  TORCH_CHECK(N * OH * OW * C < (int64_t{1} << 31), "bn_pool_bwd: pooled tensor too large (32-bit indexing)");
  damd_bn_pool_bwd_launch(dp.data_ptr(), idx.data_ptr<uint8_t>(), x.data_ptr(), N, static_cast<int>(H),
                          static_cast<int>(W), static_cast<int>(C), static_cast<int>(OH), static_cast<int>(OW),
                          stats[0].data_ptr<float>(), stats[1].data_ptr<float>(), stats[2].data_ptr<float>(),
                          stats[3].data_ptr<float>(), part.data_ptr<float>(), coef.data_ptr<float>(), dgamma.data_ptr(),
                          dbeta.data_ptr(), dx.data_ptr(), dtype_code(x), dtype_code(weight), cur_stream(), d2, xa);
  return {dx, dgamma, dbeta};
}

// backward of a global average pool over a channels-last [N, C, H, W] input: g [N, C] -> dx
at::Tensor global_avgpool_bwd(const at::Tensor& g, int64_t H, int64_t W) {
  TORCH_CHECK(g.is_cuda() && g.dim() == 2 && g.is_contiguous() && g.size(1) % 8 == 0 &&
              (reinterpret_cast<uintptr_t>(g.data_ptr()) & 15) == 0, "global_avgpool_bwd: g must be a contiguous [N, C%8==0] GPU tensor");
  TORCH_CHECK(H > 0 && W > 0, "global_avgpool_bwd: bad spatial size");
  const int64_t N = g.size(0), C = g.size(1);
  auto dx = at::empty({N, C, H, W}, g.options().memory_format(at::MemoryFormat::ChannelsLast));
  damd_hw_broadcast_launch(g.data_ptr(), dx.data_ptr(), N, H * W, static_cast<int>(C), 1.f / static_cast<float>(H * W),
                           dtype_code(g), cur_stream());
  return dx;
}

// ---------------------------------------------------------------- ResNet stem convolution
// x: [N, 3, H, W] bf16 channels-last (NHWC); w: [64, 3, 7, 7]; stride 2, padding 3.
bool stem_conv_supported(const at::Tensor& x, const at::Tensor& w) {
  return x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 && x.size(1) == 3 &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
         w.dim() == 4 && w.size(0) == 64 && w.size(1) == 3 && w.size(2) == 7 && w.size(3) == 7 &&
         damd_stem_supported(x.size(2), x.size(3));
}

// [64][7][32] bf16 weight image: k' = 4*kw + ci with zero pad at kw = 7 / ci = 3 (28 KB)
at::Tensor stem_weight_image(const at::Tensor& w) {
  return at::constant_pad_nd(w.to(at::kBFloat16).permute({0, 2, 3, 1}), {0, 1, 0, 1}).reshape({64, 7, 32}).contiguous();
}

// returns (y, stats partials [nb, 2, 64] or an empty tensor) -- see conv_stem.hip
std::vector<at::Tensor> stem_conv_fwd(const at::Tensor& x, const at::Tensor& w, bool want_stats) {
  TORCH_CHECK(stem_conv_supported(x, w), "stem_conv_fwd: unsupported input");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  auto wl = stem_weight_image(w);
  auto y = at::empty({N, 64, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  at::Tensor part = want_stats ? at::empty({damd_stem_fwd_blocks(N, static_cast<int>(H)), 2, 64},
                                          x.options().dtype(at::kFloat))
                               : at::empty({0}, x.options().dtype(at::kFloat));
  damd_stem_fwd_launch(x.data_ptr(), wl.data_ptr(), y.data_ptr(), want_stats ? part.data_ptr<float>() : nullptr, N,
                       static_cast<int>(H), static_cast<int>(W), cur_stream());
  return {y, part};
}

// dW for the stem convolution, in w's dtype and memory format.
at::Tensor stem_conv_wgrad(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& w) {
  TORCH_CHECK(stem_conv_supported(x, w), "stem_conv_wgrad: unsupported input");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  TORCH_CHECK(dy.dim() == 4 && dy.size(0) == N && dy.size(1) == 64 && dy.size(2) == (H - 1) / 2 + 1 &&
              dy.size(3) == (W - 1) / 2 + 1 && dy.scalar_type() == at::kBFloat16 &&
              dy.is_contiguous(at::MemoryFormat::ChannelsLast) && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0,
              "stem_conv_wgrad: dy must be a [N, 64, OH, OW] bf16 channels-last tensor");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat, "stem_conv_wgrad: weight dtype");
  const int nb = damd_stem_wgrad_blocks(N, static_cast<int>(H));
  auto part = at::empty({nb, 64, 7 * 32}, x.options().dtype(at::kFloat));
  auto dw = at::empty({64, 3, 7, 7}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  damd_stem_wgrad_launch(x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), dtype_code(w), N,
                         static_cast<int>(H), static_cast<int>(W), cur_stream());
  return w.is_contiguous(at::MemoryFormat::ChannelsLast) ? dw : dw.contiguous();
}

// ---------------------------------------------------------------- fused stem: conv + BN + ReLU + max-pool
// conv7x7/s2 -> BatchNorm (training statistics) -> ReLU -> maxpool3x3/s2/p1 without the conv's
// full-size output (conv_stem.hip stem_pool_*).  gamma/beta: the BN affine parameters (bf16/fp32).
bool stem_pool_supported(const at::Tensor& x, const at::Tensor& w) {
  return stem_conv_supported(x, w) && damd_stem_pool_supported(x.size(2), x.size(3));
}

// returns (y [N, 64, PH, PW] channels-last, window positions uint8, stats [4, 64] (mean, invstd,
// scale, shift), xarg: the raw conv value each window selected)
std::vector<at::Tensor> stem_pool_fwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& gamma,
                                      const at::Tensor& beta, const c10::optional<at::Tensor>& running_mean,
                                      const c10::optional<at::Tensor>& running_var, double momentum, double eps) {
  TORCH_CHECK(stem_pool_supported(x, w), "stem_pool_fwd: unsupported input");
  TORCH_CHECK(gamma.numel() == 64 && beta.numel() == 64 && gamma.is_contiguous() && beta.is_contiguous() &&
              gamma.scalar_type() == beta.scalar_type() &&
              (gamma.scalar_type() == at::kBFloat16 || gamma.scalar_type() == at::kFloat),
              "stem_pool_fwd: BN weight/bias must be 64-element bf16/fp32 tensors");
  float* rm = nullptr;
  float* rv = nullptr;
  if (running_mean.has_value() && running_mean->defined()) {
    TORCH_CHECK(running_mean->scalar_type() == at::kFloat && running_var->scalar_type() == at::kFloat,
                "running stats must be float32");
    rm = running_mean->data_ptr<float>();
    rv = running_var->data_ptr<float>();
  }
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, PH = OH / 2, PW = OW / 2;
  auto wl = stem_weight_image(w);
  const int nb = damd_stem_pool_blocks(N, H, W);
  auto fopts = x.options().dtype(at::kFloat);
  auto part = at::empty({nb, 2, 64}, fopts);
  auto stats = at::empty({4, 64}, fopts);
  auto xarg = at::empty({N, 64, PH, PW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto y = at::empty_like(xarg);
  auto idx = at::empty({N * PH * PW * 64}, x.options().dtype(at::kByte));
  TORCH_CHECK(N * PH * PW * 64 < (int64_t{1} << 31), "stem_pool_fwd: pooled tensor too large (32-bit indexing)");
  damd_stem_pool_fwd_launch(x.data_ptr(), wl.data_ptr(), gamma.data_ptr(), dtype_code(gamma), xarg.data_ptr(),
                            idx.data_ptr<uint8_t>(), part.data_ptr<float>(), N, static_cast<int>(H), static_cast<int>(W),
                            cur_stream());
  damd_stem_pool_bn_fwd_launch(part.data_ptr<float>(), nb, N * OH * OW, xarg.data_ptr(), y.data_ptr(), N * PH * PW, 64,
                               gamma.data_ptr(), beta.data_ptr(), rm, rv, static_cast<float>(momentum),
                               static_cast<float>(eps), stats[0].data_ptr<float>(), stats[1].data_ptr<float>(),
                               stats[2].data_ptr<float>(), stats[3].data_ptr<float>(), dtype_code(gamma), cur_stream());
  return {y, idx, stats, xarg};
}

// returns (dW in w's dtype / memory format, dgamma, dbeta); dp [+ dp2]: the pooled output's gradient(s)
std::vector<at::Tensor> stem_pool_bwd(const at::Tensor& x, const at::Tensor& w, const at::Tensor& dp,
                                      const c10::optional<at::Tensor>& dp2, const at::Tensor& idx,
                                      const at::Tensor& xarg, const at::Tensor& stats, const at::Tensor& gamma) {
  TORCH_CHECK(stem_pool_supported(x, w), "stem_pool_bwd: unsupported input");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat, "stem_pool_bwd: weight dtype");
  const int64_t N = x.size(0), H = x.size(2), W = x.size(3);
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, PH = OH / 2, PW = OW / 2;
  TORCH_CHECK(dp.dim() == 4 && dp.size(0) == N && dp.size(1) == 64 && dp.size(2) == PH && dp.size(3) == PW &&
              dp.scalar_type() == at::kBFloat16 && dp.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              (reinterpret_cast<uintptr_t>(dp.data_ptr()) & 15) == 0,
              "stem_pool_bwd: dp must be a [N, 64, PH, PW] bf16 channels-last tensor");
  TORCH_CHECK(xarg.sizes() == dp.sizes() && xarg.strides() == dp.strides() && xarg.scalar_type() == at::kBFloat16,
              "stem_pool_bwd: xarg must match dp");
  TORCH_CHECK(idx.scalar_type() == at::kByte && idx.numel() == N * PH * PW * 64 && idx.is_contiguous(),
              "stem_pool_bwd: bad window-position tensor");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.size(0) == 4 && stats.size(1) == 64 && stats.is_contiguous(),
              "stem_pool_bwd: bad stats");
  const void* d2 = nullptr;
  if (dp2.has_value() && dp2->defined()) {
    TORCH_CHECK(dp2->sizes() == dp.sizes() && dp2->strides() == dp.strides() && dp2->scalar_type() == dp.scalar_type() &&
                dp2->device() == dp.device(), "stem_pool_bwd: dp2 must match dp");
    d2 = dp2->data_ptr();
  }
  auto fopts = x.options().dtype(at::kFloat);
  const int64_t Q = N * PH * PW;
  auto part_r = at::empty({damd_bn_num_blocks(Q, 64), 2, 64}, fopts);
  auto coef = at::empty({3, 64}, fopts);
  auto dgamma = at::empty({64}, gamma.options());
  auto dbeta = at::empty({64}, gamma.options());
  auto dz = at::empty_like(dp);
  damd_stem_pool_bn_bwd_launch(dp.data_ptr(), d2, xarg.data_ptr(), stats[0].data_ptr<float>(), stats[1].data_ptr<float>(),
                               stats[2].data_ptr<float>(), stats[3].data_ptr<float>(), part_r.data_ptr<float>(),
                               coef.data_ptr<float>(), dgamma.data_ptr(), dbeta.data_ptr(), dz.data_ptr(), Q, N * OH * OW,
                               64, dtype_code(gamma), cur_stream());
  auto wl = stem_weight_image(w);
  const int nbw = damd_stem_pool_blocks(N, H, W);
  auto part_w = at::empty({nbw, 64, 7 * 32}, fopts);
  auto dw = at::empty({64, 3, 7, 7}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  damd_stem_pool_bwd_launch(x.data_ptr(), wl.data_ptr(), dz.data_ptr(), idx.data_ptr<uint8_t>(), coef.data_ptr<float>(),
                            part_w.data_ptr<float>(), dw.data_ptr(), dtype_code(w), N, static_cast<int>(H),
                            static_cast<int>(W), cur_stream());
  return {w.is_contiguous(at::MemoryFormat::ChannelsLast) ? dw : dw.contiguous(), dgamma, dbeta};
}

// ---------------------------------------------------------------- implicit-GEMM convolution
// Stream-K configs (conv_igemm.hip make_plan) hand partial tiles between blocks: a per-call fp32
// slab workspace from the caching allocator (stream-ordered reuse) and a buffer of flag words per
// (device, stream) that the kernels leave zeroed (+ a poll time-out counter at its end).  Launches
// on one stream are ordered, so one buffer per stream is never shared between live launches;
// stream-K convs issued from two streams at once get separate buffers.
struct SkWorkspace {
  at::Tensor ws;
  float* wsp = nullptr;
  int* flags = nullptr;
};

std::mutex& sk_mutex() {
  static std::mutex mu;
  return mu;
}

std::map<std::pair<int, hipStream_t>, at::Tensor>& sk_flag_buffers() {
  static std::map<std::pair<int, hipStream_t>, at::Tensor> bufs;
  return bufs;
}

at::Tensor sk_flag_buffer(const at::Device& dev, hipStream_t stream) {
  std::lock_guard<std::mutex> lk(sk_mutex());
  at::Tensor& t = sk_flag_buffers()[{static_cast<int>(dev.index()), stream}];
  if (!t.defined()) t = at::zeros({damd_conv_sk_flag_words()}, at::TensorOptions().device(dev).dtype(at::kInt));
  return t;
}

SkWorkspace sk_workspace(const at::Tensor& like, int64_t K, int64_t W, int64_t cfg) {
  SkWorkspace s;
  const int64_t n = damd_conv_sk_ws_floats(static_cast<int>(K), static_cast<int>(W), static_cast<int>(cfg));
  if (n == 0) return s;
  s.ws = at::empty({n}, like.options().dtype(at::kFloat).memory_format(at::MemoryFormat::Contiguous));
  s.wsp = s.ws.data_ptr<float>();
  s.flags = sk_flag_buffer(like.device(), cur_stream()).data_ptr<int>();
  return s;
}

// Poll time-outs recorded by stream-K launches on this device, over every stream (0 unless a
// hand-off never arrived; such a tile was written as NaN).  Synchronises the device.  With
// reset=true the flag words and counters are zeroed afterwards (a timed-out consumer leaves its
// producer's flag set), so the buffers are clean for later launches.
int64_t conv_sk_timeouts(const at::Tensor& like, bool reset) {
  std::vector<at::Tensor> bufs;
  {
    std::lock_guard<std::mutex> lk(sk_mutex());
    for (auto& kv : sk_flag_buffers())
      if (kv.first.first == like.device().index()) bufs.push_back(kv.second);
  }
  if (bufs.empty()) return 0;
  TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "conv_sk_timeouts: device synchronize failed");
  int64_t n = 0;
  for (auto& t : bufs) n += t.narrow(0, damd_conv_sk_flag_words() - 16, 1).item<int>();
  if (reset && n > 0) {
    for (auto& t : bufs) t.zero_();
    TORCH_CHECK(hipDeviceSynchronize() == hipSuccess, "conv_sk_timeouts: device synchronize failed");
  }
  return n;
}

// x: [N, C, H, W] bf16 channels-last; w: [K, C, R, S] bf16 (made channels-last = [K][R][S][C]);
// returns (y [N, K, OH, OW] channels-last, stats partials [groups, 2, K] or an empty tensor).
bool conv_supported(const at::Tensor& x, const at::Tensor& w, int64_t cfg, int64_t stride, int64_t pad) {
  if (cfg < 0) cfg = damd_conv_default_cfg(static_cast<int>(w.size(0)), 0);
  return x.is_cuda() && x.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
         x.numel() * 2 < 0xF0000000LL &&  // 32-bit buffer offsets in the kernels (conv_igemm.hip)
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
         w.dim() == 4 && w.scalar_type() == at::kBFloat16 && w.size(1) == x.size(1) &&
         cfg_supported(static_cast<int>(x.size(1)), static_cast<int>(w.size(0)), static_cast<int>(w.size(2)),
                       static_cast<int>(w.size(3)), static_cast<int>(stride), static_cast<int>(pad),
                       static_cast<int>(x.size(2)), static_cast<int>(x.size(3)), static_cast<int>(cfg));
}

// One phase (a, b) of the input gradient of a stride-2, pad-1 3x3 conv (even input size 2*OH x 2*OW):
// dX[n, 2i+a, 2j+b] = sum over the phase's taps of dY[n, i+dh, j+dw] . W[k, c, r, s] -- a stride-1,
// pad-0 conv of dY with the (1|2)x(1|2) sub-kernel wsub ([C][Rp][Sp][K] channels-last, taps ordered by
// dh, dw = 0, +1), written straight into its pixels of dX (conv_igemm.hip Geo::ost).
void conv_dgrad_phase(const at::Tensor& dy, const at::Tensor& wsub, at::Tensor& dx, int64_t a, int64_t b, int64_t cfg) {
  TORCH_CHECK(!damd_conv_cfg_is_sk(static_cast<int>(cfg)) && conv_supported(dy, wsub, cfg, 1, 0),
              "conv_dgrad_phase: unsupported input / weight / config");
  TORCH_CHECK(dx.is_cuda() && dx.scalar_type() == at::kBFloat16 && dx.is_contiguous(at::MemoryFormat::ChannelsLast) &&
              dx.size(0) == dy.size(0) && dx.size(1) == wsub.size(0) && dx.size(2) == 2 * dy.size(2) &&
              dx.size(3) == 2 * dy.size(3) && wsub.size(2) <= 2 && wsub.size(3) <= 2 && (a | b) >= 0 && a < 2 && b < 2,
              "conv_dgrad_phase: bad geometry");
  const int64_t N = dy.size(0), K = dy.size(1), H = dy.size(2), W = dy.size(3), C = wsub.size(0);
  TORCH_CHECK(N * 4 * H * W < (int64_t{1} << 31) - 4096, "conv_dgrad_phase: tensor too large");
  auto wl = wsub.contiguous(at::MemoryFormat::ChannelsLast);
  const int G = cfg_groups(N * H * W, static_cast<int>(C), static_cast<int>(W), static_cast<int>(cfg), 0, N, H);
  const int rc = cfg_launch(dy.data_ptr(), wl.data_ptr(), dx.data_ptr(), nullptr, static_cast<int>(N),
                                      static_cast<int>(H), static_cast<int>(W), static_cast<int>(K), static_cast<int>(C),
                                      static_cast<int>(wsub.size(2)), static_cast<int>(wsub.size(3)), 1, 0,
                                      static_cast<int>(cfg), G, cur_stream(), 0, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
                                      nullptr, 0, 4 | static_cast<int>(a << 1) | static_cast<int>(b));
  TORCH_CHECK(rc == 0, "conv_dgrad_phase: launch rejected");
}

std::vector<at::Tensor> conv_fwd(const at::Tensor& x, const at::Tensor& w, int64_t stride, int64_t pad,
                                 bool want_stats, int64_t cfg, int64_t groups) {
  if (cfg < 0) cfg = damd_conv_default_cfg(static_cast<int>(w.size(0)), 0);
  TORCH_CHECK(conv_supported(x, w, cfg, stride, pad), "conv_fwd: unsupported input / weight / config");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(stride >= 1 && pad >= 0 && H + 2 * pad >= R && W + 2 * pad >= S, "conv_fwd: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  const int64_t M = N * OH * OW;
  TORCH_CHECK(M < (int64_t{1} << 31) - 4096 && x.numel() < (int64_t{1} << 40), "conv_fwd: tensor too large");
  auto wl = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto y = at::empty({N, K, OH, OW}, x.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int G = cfg_groups(M, static_cast<int>(K), static_cast<int>(W), static_cast<int>(cfg),
                           static_cast<int>(groups), N, H);
  at::Tensor part = want_stats ? at::empty({G, 2, K}, x.options().dtype(at::kFloat)) : at::empty({0}, x.options().dtype(at::kFloat));
  const SkWorkspace sk = sk_workspace(x, K, W, cfg);
  const int rc = cfg_launch(x.data_ptr(), wl.data_ptr(), y.data_ptr(), want_stats ? part.data_ptr<float>() : nullptr,
                                      static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                      static_cast<int>(K), static_cast<int>(R), static_cast<int>(S), static_cast<int>(stride),
                                      static_cast<int>(pad), static_cast<int>(cfg), G, cur_stream(), want_stats ? 1 : 0,
                                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 0, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, sk.wsp, sk.flags, 0);
  TORCH_CHECK(rc == 0, "conv_fwd: launch rejected");
  return {y, part};
}

// z = conv1x1(a, w) with a = relu(y * stats[2] + stats[3] [+ res]) computed inside the conv's
// operand staging (ProArgs); returns (z, z's BN statistic partials [groups, 2, K], a, a's ReLU bit
// mask or an empty tensor).  stats: [4, C] of y's BatchNorm (mean, invstd, scale, shift).
// res_stats: [4, C] stats of a BatchNorm (no ReLU) whose output is the residual: `res` is then
// that BN's INPUT and a = relu(y * scale + shift + res * res_scale + res_shift) (the residual BN's
// forward apply folded into this staging too).
std::vector<at::Tensor> conv_bnact_fwd(const at::Tensor& y, const at::Tensor& w, const c10::optional<at::Tensor>& res,
                                       const at::Tensor& stats, bool want_mask, int64_t cfg,
                                       const c10::optional<at::Tensor>& res_stats) {
  const int64_t R = w.size(2), S = w.size(3), pad = (R - 1) / 2;  // 1x1, or 3x3 / pad 1 (halo kernel)
  TORCH_CHECK(R == S && (R == 1 || R == 3) && conv_supported(y, w, cfg, 1, pad), "conv_bnact_fwd: unsupported input");
  const int64_t N = y.size(0), C = y.size(1), H = y.size(2), W = y.size(3), K = w.size(0);
  TORCH_CHECK(cfg_pro_supported(static_cast<int>(C), static_cast<int>(K), static_cast<int>(R),
                                static_cast<int>(S), 1, static_cast<int>(pad), static_cast<int>(H), static_cast<int>(W),
                                static_cast<int>(cfg)),
              "conv_bnact_fwd: config has no prologue variant");
  TORCH_CHECK(R == 1 || !(res.has_value() && res->defined()), "conv_bnact_fwd: no residual operand for 3x3 convs");
  TORCH_CHECK(R == 1 || !want_mask, "conv_bnact_fwd: no ReLU mask output for 3x3 convs");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.dim() == 2 && stats.size(0) == 4 && stats.size(1) == C &&
              stats.is_contiguous(), "conv_bnact_fwd: stats must be float32 [4, C]");
  const void* rp = nullptr;
  if (res.has_value() && res->defined()) {
    TORCH_CHECK(res->sizes() == y.sizes() && res->strides() == y.strides() && res->scalar_type() == y.scalar_type(),
                "conv_bnact_fwd: res must match y");
    rp = res->data_ptr();
  }
  const float* shift = stats[3].data_ptr<float>();
  const float* rscale = nullptr;
  at::Tensor shift_comb;
  if (res_stats.has_value() && res_stats->defined()) {
    TORCH_CHECK(rp != nullptr && res_stats->scalar_type() == at::kFloat && res_stats->dim() == 2 &&
                res_stats->size(0) == 4 && res_stats->size(1) == C && res_stats->is_contiguous(),
                "conv_bnact_fwd: res_stats must be float32 [4, C] with a residual");
    shift_comb = stats[3] + (*res_stats)[3];
    shift = shift_comb.data_ptr<float>();
    rscale = (*res_stats)[2].data_ptr<float>();
  }
  const int64_t M = N * H * W;
  TORCH_CHECK(M < (int64_t{1} << 31) - 4096, "conv_bnact_fwd: tensor too large");
  auto wl = w.contiguous(at::MemoryFormat::ChannelsLast);
  auto z = at::empty({N, K, H, W}, y.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto a = at::empty_like(y);
  auto mask = want_mask ? at::empty({M * C / 8}, y.options().dtype(at::kByte)) : at::empty({0}, y.options().dtype(at::kByte));
  const int G = cfg_groups(M, static_cast<int>(K), static_cast<int>(W), static_cast<int>(cfg), 0, N, H);
  auto part = at::empty({G, 2, K}, y.options().dtype(at::kFloat));
  const SkWorkspace sk = sk_workspace(y, K, W, cfg);
  const int rc = cfg_launch(y.data_ptr(), wl.data_ptr(), z.data_ptr(), part.data_ptr<float>(),
                                      static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                      static_cast<int>(K), static_cast<int>(R), static_cast<int>(S), 1,
                                      static_cast<int>(pad), static_cast<int>(cfg), G, cur_stream(), 1,
                                      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 1, rp,
                                      stats[2].data_ptr<float>(), shift, rscale, a.data_ptr(),
                                      want_mask ? mask.data_ptr<uint8_t>() : nullptr, sk.wsp, sk.flags, 0);
  TORCH_CHECK(rc == 0, "conv_bnact_fwd: launch rejected");
  return {z, part, a, mask};
}

bool conv_pro_supported(const at::Tensor& y, const at::Tensor& w, int64_t cfg) {
  const int64_t R = w.dim() == 4 ? w.size(2) : 0, pad = (R - 1) / 2;
  return (R == 1 || R == 3) && w.size(3) == R && conv_supported(y, w, cfg, 1, pad) &&
         cfg_pro_supported(static_cast<int>(y.size(1)), static_cast<int>(w.size(0)), static_cast<int>(R),
                           static_cast<int>(R), 1, static_cast<int>(pad), static_cast<int>(y.size(2)),
                           static_cast<int>(y.size(3)), static_cast<int>(cfg));
}

// Stride-1 input gradient dX = conv(dY, wt, pad) (wt = flipped, transposed weights) of a conv
// whose input was a = relu(bn(yb) [+ residual]), with the BN backward's reduce fused into the
// epilogue: returns (dz, part [groups, 2, C]) where dz = (dX [+ d2]) * [a > 0] (the gradient at
// the BN's output; also the residual's gradient) and part = (sum dz, sum dz * (yb - mean)) for
// the BN backward finalize.  mask: the forward's ReLU bit mask, or absent to recompute the ReLU
// from yb * scale + shift (no residual).  stats: [4, C] (mean, invstd, scale, shift).
std::vector<at::Tensor> conv_dgrad_bn(const at::Tensor& dy, const at::Tensor& wt, int64_t pad, int64_t cfg,
                                      const c10::optional<at::Tensor>& d2, const at::Tensor& yb,
                                      const c10::optional<at::Tensor>& mask, const at::Tensor& stats,
                                      const c10::optional<at::Tensor>& pro_y, const c10::optional<at::Tensor>& pro_coef) {
  if (cfg < 0) cfg = damd_conv_default_cfg(static_cast<int>(wt.size(0)), 0);
  TORCH_CHECK(conv_supported(dy, wt, cfg, 1, pad), "conv_dgrad_bn: unsupported input / weight / config");
  const int64_t N = dy.size(0), C = dy.size(1), H = dy.size(2), W = dy.size(3);
  const int64_t K = wt.size(0), R = wt.size(2), S = wt.size(3);
  TORCH_CHECK(R == S && 2 * pad == R - 1, "conv_dgrad_bn: stride-1 same-size convolutions only");
  TORCH_CHECK(yb.scalar_type() == at::kBFloat16 && yb.dim() == 4 && yb.size(0) == N && yb.size(1) == K &&
              yb.size(2) == H && yb.size(3) == W && yb.is_contiguous(at::MemoryFormat::ChannelsLast),
              "conv_dgrad_bn: yb must be the [N, K, H, W] channels-last bf16 BN input");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.dim() == 2 && stats.size(0) == 4 && stats.size(1) == K &&
              stats.is_contiguous(), "conv_dgrad_bn: stats must be float32 [4, K]");
  const void* d2p = nullptr;
  int d2hw = 0;
  if (d2.has_value() && d2->defined()) {
    // d2 on yb's grid, or the compact [N, K, ceil(H/2), ceil(W/2)] input gradient of a 1x1 stride-2
    // shortcut conv (nonzero only at the even (h, w) of yb's grid; ops/conv.py _StridedGrad)
    const bool compact = d2->dim() == 4 && d2->size(0) == N && d2->size(1) == K && d2->size(2) == (H + 1) / 2 &&
                         d2->size(3) == (W + 1) / 2 && d2->is_contiguous(at::MemoryFormat::ChannelsLast) &&
                         (H > 1 || W > 1);
    TORCH_CHECK(((d2->sizes() == yb.sizes() && d2->strides() == yb.strides()) || compact) &&
                d2->scalar_type() == at::kBFloat16, "conv_dgrad_bn: d2 must match yb (or be its stride-2 compact grid)");
    d2p = d2->data_ptr();
    if (d2->sizes() != yb.sizes()) d2hw = static_cast<int>(((H + 1) / 2) << 16 | ((W + 1) / 2));
  }
  const uint8_t* mp = nullptr;
  if (mask.has_value() && mask->defined() && mask->numel() > 0) {
    TORCH_CHECK(mask->scalar_type() == at::kByte && mask->numel() == yb.numel() / 8 && mask->is_contiguous(),
                "conv_dgrad_bn: mask must be uint8 [numel / 8]");
    mp = mask->data_ptr<uint8_t>();
  }
  const int64_t M = N * H * W;
  TORCH_CHECK(M < (int64_t{1} << 31) - 4096, "conv_dgrad_bn: tensor too large");
  auto wl = wt.contiguous(at::MemoryFormat::ChannelsLast);
  auto dz = at::empty_like(yb);
  const int G = cfg_groups(M, static_cast<int>(K), static_cast<int>(W), static_cast<int>(cfg), 0, N, H);
  auto part = at::empty({G, 2, K}, dy.options().dtype(at::kFloat));
  // Deferred BN-backward apply (ops/conv.py _LazyBNGrad): with pro_y given, `dy` holds the
  // following BatchNorm's output gradient dz and the conv's real output gradient is
  // pro_coef[0] * dz + pro_coef[1] * pro_y + pro_coef[2] (per channel), formed in the operand
  // staging and returned materialised as a third output for the weight gradient.
  int pro = 0;
  const void* p_res = nullptr;
  const float *p_a = nullptr, *p_b = nullptr, *p_c = nullptr;
  void* p_out = nullptr;
  at::Tensor dyo;
  if (pro_y.has_value() && pro_y->defined()) {
    TORCH_CHECK(pro_coef.has_value() && pro_coef->defined() && pro_coef->scalar_type() == at::kFloat &&
                pro_coef->dim() == 2 && pro_coef->size(0) == 3 && pro_coef->size(1) == C && pro_coef->is_contiguous(),
                "conv_dgrad_bn: pro_coef must be float32 [3, C]");
    TORCH_CHECK(pro_y->sizes() == dy.sizes() && pro_y->strides() == dy.strides() &&
                pro_y->scalar_type() == at::kBFloat16, "conv_dgrad_bn: pro_y must match dy");
    TORCH_CHECK(cfg_pro_supported(static_cast<int>(C), static_cast<int>(K), static_cast<int>(R),
                                  static_cast<int>(S), 1, static_cast<int>(pad), static_cast<int>(H), static_cast<int>(W),
                                  static_cast<int>(cfg)),
                "conv_dgrad_bn: config has no prologue variant");
    pro = 2;
    p_res = pro_y->data_ptr();
    p_a = (*pro_coef)[0].data_ptr<float>();
    p_b = (*pro_coef)[1].data_ptr<float>();
    p_c = (*pro_coef)[2].data_ptr<float>();
    dyo = at::empty_like(dy);
    p_out = dyo.data_ptr();
  }
  const SkWorkspace sk = sk_workspace(dy, K, W, cfg);
  const int rc = cfg_launch(dy.data_ptr(), wl.data_ptr(), dz.data_ptr(), part.data_ptr<float>(),
                                      static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                      static_cast<int>(K), static_cast<int>(R), static_cast<int>(S), 1,
                                      static_cast<int>(pad), static_cast<int>(cfg), G, cur_stream(), mp ? 2 : 3, d2p,
                                      yb.data_ptr(), mp, stats[0].data_ptr<float>(), stats[2].data_ptr<float>(),
                                      stats[3].data_ptr<float>(), pro, p_res, p_a, p_c, p_b, p_out, nullptr, sk.wsp,
                                      sk.flags, d2hw);
  TORCH_CHECK(rc == 0, "conv_dgrad_bn: launch rejected");
  if (pro) return {dz, part, dyo};
  return {dz, part};
}

// Stride-1 1x1 input gradient whose operand is a deferred BN backward: dX = conv1x1(dy, wt) with
// dy = coef[0] * dz + coef[1] * y + coef[2] formed in the operand staging (PRO 2) and returned
// materialised for the weight gradient: (dX, dy).  No epilogue.
std::vector<at::Tensor> conv_fwd_pro2(const at::Tensor& dz, const at::Tensor& wt, const at::Tensor& y,
                                      const at::Tensor& coef, int64_t cfg) {
  TORCH_CHECK(wt.dim() == 4 && wt.size(2) == 1 && wt.size(3) == 1 && conv_supported(dz, wt, cfg, 1, 0),
              "conv_fwd_pro2: unsupported input / weight / config");
  const int64_t N = dz.size(0), C = dz.size(1), H = dz.size(2), W = dz.size(3), K = wt.size(0);
  TORCH_CHECK(cfg_pro_supported(static_cast<int>(C), static_cast<int>(K), 1, 1, 1, 0, static_cast<int>(H),
                                static_cast<int>(W), static_cast<int>(cfg)), "conv_fwd_pro2: config has no prologue variant");
  TORCH_CHECK(y.sizes() == dz.sizes() && y.strides() == dz.strides() && y.scalar_type() == at::kBFloat16,
              "conv_fwd_pro2: y must match dz");
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.dim() == 2 && coef.size(0) == 3 && coef.size(1) == C &&
              coef.is_contiguous(), "conv_fwd_pro2: coef must be float32 [3, C]");
  const int64_t M = N * H * W;
  TORCH_CHECK(M < (int64_t{1} << 31) - 4096, "conv_fwd_pro2: tensor too large");
  auto wl = wt.contiguous(at::MemoryFormat::ChannelsLast);
  auto out = at::empty({N, K, H, W}, dz.options().memory_format(at::MemoryFormat::ChannelsLast));
  auto dyo = at::empty_like(dz);
  const int G = cfg_groups(M, static_cast<int>(K), static_cast<int>(W), static_cast<int>(cfg), 0, N, H);
  const SkWorkspace sk = sk_workspace(dz, K, W, cfg);
  const int rc = cfg_launch(dz.data_ptr(), wl.data_ptr(), out.data_ptr(), nullptr, static_cast<int>(N),
                                      static_cast<int>(H), static_cast<int>(W), static_cast<int>(C), static_cast<int>(K),
                                      1, 1, 1, 0, static_cast<int>(cfg), G, cur_stream(), 0, nullptr, nullptr, nullptr,
                                      nullptr, nullptr, nullptr, 2, y.data_ptr(), coef[0].data_ptr<float>(),
                                      coef[2].data_ptr<float>(), coef[1].data_ptr<float>(), dyo.data_ptr(), nullptr,
                                      sk.wsp, sk.flags, 0);
  TORCH_CHECK(rc == 0, "conv_fwd_pro2: launch rejected");
  return {out, dyo};
}

// dW of the convolution y = conv(x, w) (stride, pad) from dY, in w's dtype, as a channels-last
// [K, C, R, S] tensor (physically [K][R][S][C]).
bool wgrad_supported(const at::Tensor& x, const at::Tensor& dy, int64_t K, int64_t cfg) {
  return x.is_cuda() && x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
         dy.dim() == 4 && x.is_contiguous(at::MemoryFormat::ChannelsLast) &&
         dy.is_contiguous(at::MemoryFormat::ChannelsLast) && (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 &&
         (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0 && dy.size(1) == K &&
         damd_wgrad_supported(static_cast<int>(x.size(1)), static_cast<int>(K), static_cast<int>(cfg));
}

at::Tensor conv_wgrad(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& w, int64_t stride, int64_t pad,
                      int64_t cfg, int64_t splits) {
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3);
  const int64_t K = w.size(0), R = w.size(2), S = w.size(3);
  TORCH_CHECK(wgrad_supported(x, dy, K, cfg) && w.size(1) == C, "conv_wgrad: unsupported input / config");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat, "conv_wgrad: weight dtype");
  const int64_t OH = (H + 2 * pad - R) / stride + 1, OW = (W + 2 * pad - S) / stride + 1;
  TORCH_CHECK(dy.size(0) == N && dy.size(2) == OH && dy.size(3) == OW, "conv_wgrad: dy shape");
  const int64_t M = N * OH * OW;
  const int sp = damd_wgrad_splits(M, static_cast<int>(C), static_cast<int>(K), static_cast<int>(R), static_cast<int>(S),
                                   static_cast<int>(cfg), static_cast<int>(splits));
  auto part = at::empty({sp, K * R * S * C}, x.options().dtype(at::kFloat));
  auto dw = at::empty({K, C, R, S}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = damd_wgrad_launch(x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), dtype_code(w),
                                   static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                   static_cast<int>(K), static_cast<int>(R), static_cast<int>(S), static_cast<int>(stride),
                                   static_cast<int>(pad), static_cast<int>(cfg), sp, cur_stream());
  TORCH_CHECK(rc == 0, "conv_wgrad: launch rejected");
  return dw;
}

// dW of a 3x3 / stride-1 / pad-1 convolution by the halo kernel (cfg 0: 128 output channels per
// block, 1: 64; 2 ..: conv3x3v2.hip's whole-row-tile kernel), in w's dtype, channels-last [K, C, 3, 3].
bool wgrad3x3_supported(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& w, int64_t cfg) {
  return x.is_cuda() && x.scalar_type() == at::kBFloat16 && dy.scalar_type() == at::kBFloat16 && x.dim() == 4 &&
         dy.dim() == 4 && w.dim() == 4 && w.size(2) == 3 && w.size(3) == 3 && w.size(1) == x.size(1) &&
         dy.size(1) == w.size(0) && dy.size(0) == x.size(0) && dy.size(2) == x.size(2) && dy.size(3) == x.size(3) &&
         x.is_contiguous(at::MemoryFormat::ChannelsLast) && dy.is_contiguous(at::MemoryFormat::ChannelsLast) &&
         (reinterpret_cast<uintptr_t>(x.data_ptr()) & 15) == 0 && (reinterpret_cast<uintptr_t>(dy.data_ptr()) & 15) == 0 &&
         damd_wgrad3x3_supported(static_cast<int>(x.size(1)), static_cast<int>(w.size(0)), static_cast<int>(x.size(2)),
                                 static_cast<int>(x.size(3)),
                                 static_cast<int>(cfg));
}

at::Tensor conv3x3_wgrad(const at::Tensor& x, const at::Tensor& dy, const at::Tensor& w, int64_t cfg, int64_t splits) {
  TORCH_CHECK(wgrad3x3_supported(x, dy, w, cfg), "conv3x3_wgrad: unsupported input / config");
  TORCH_CHECK(w.scalar_type() == at::kBFloat16 || w.scalar_type() == at::kFloat, "conv3x3_wgrad: weight dtype");
  const int64_t N = x.size(0), C = x.size(1), H = x.size(2), W = x.size(3), K = w.size(0);
  const int sp = damd_wgrad3x3_splits(N, static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                      static_cast<int>(K), static_cast<int>(cfg), static_cast<int>(splits));
  auto part = at::empty({sp, K * 9 * C}, x.options().dtype(at::kFloat));
  auto dw = at::empty({K, C, 3, 3}, w.options().memory_format(at::MemoryFormat::ChannelsLast));
  const int rc = damd_wgrad3x3_launch(x.data_ptr(), dy.data_ptr(), part.data_ptr<float>(), dw.data_ptr(), dtype_code(w),
                                      static_cast<int>(N), static_cast<int>(H), static_cast<int>(W), static_cast<int>(C),
                                      static_cast<int>(K), static_cast<int>(cfg), sp, cur_stream());
  TORCH_CHECK(rc == 0, "conv3x3_wgrad: launch rejected");
  return dw;
}

// Fused backward of z = conv1x1(a) (K = 256 <- C = 64), z's gradient a deferred BN backward
// (dy = coef[0] * dzn + coef[1] * yn + coef[2]) and a = relu(bn(yb)) without a residual: returns
// (dz = dX * relu'(bn(yb)), its BN-backward partials [G, 2, C], dW in w's dtype / layout).
bool conv1x1_bwd_fused_supported(const at::Tensor& w) {
  return w.dim() == 4 && w.size(2) == 1 && w.size(3) == 1 &&
         damd_conv1x1_bwd_fused_supported(static_cast<int>(w.size(0)), static_cast<int>(w.size(1)));
}

std::vector<at::Tensor> conv1x1_bwd_fused(const at::Tensor& dzn, const at::Tensor& yn, const at::Tensor& coef,
                                          const at::Tensor& w, const at::Tensor& a, const at::Tensor& yb,
                                          const at::Tensor& stats) {
  TORCH_CHECK(conv1x1_bwd_fused_supported(w), "conv1x1_bwd_fused: unsupported weight shape");
  const int64_t K = w.size(0), C = w.size(1);
  auto cl = at::MemoryFormat::ChannelsLast;
  for (const at::Tensor* t : {&dzn, &yn, &a, &yb})
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kBFloat16 && t->dim() == 4 && t->is_contiguous(cl) &&
                (reinterpret_cast<uintptr_t>(t->data_ptr()) & 15) == 0, "conv1x1_bwd_fused: bf16 channels-last inputs");
  TORCH_CHECK(dzn.size(1) == K && yn.sizes() == dzn.sizes() && a.size(1) == C && yb.sizes() == a.sizes() &&
              a.size(0) == dzn.size(0) && a.size(2) == dzn.size(2) && a.size(3) == dzn.size(3), "conv1x1_bwd_fused: shapes");
  TORCH_CHECK(coef.scalar_type() == at::kFloat && coef.dim() == 2 && coef.size(0) == 3 && coef.size(1) == K &&
              coef.is_contiguous(), "conv1x1_bwd_fused: coef must be float32 [3, K]");
  TORCH_CHECK(stats.scalar_type() == at::kFloat && stats.dim() == 2 && stats.size(0) == 4 && stats.size(1) == C,
              "conv1x1_bwd_fused: stats must be float32 [4, C]");
  const int64_t M = a.size(0) * a.size(2) * a.size(3);
  auto wt = w.reshape({K, C}).t().contiguous().to(at::kBFloat16);
  auto bnp = at::stack({stats[0], stats[2], stats[3]}).contiguous();
  const int G = damd_conv1x1_bwd_fused_blocks(M);
  auto dzo = at::empty_like(yb);
  auto part = at::empty({G, 2, C}, a.options().dtype(at::kFloat));
  auto wpart = at::empty({G, K * C}, a.options().dtype(at::kFloat));
  auto dw = at::empty({K, C, 1, 1}, w.options().memory_format(cl));
  const int rc = damd_conv1x1_bwd_fused_launch(dzn.data_ptr(), yn.data_ptr(), coef.data_ptr<float>(), wt.data_ptr(),
                                               a.data_ptr(), yb.data_ptr(), bnp.data_ptr<float>(), M, dzo.data_ptr(),
                                               part.data_ptr<float>(), wpart.data_ptr<float>(), dw.data_ptr(),
                                               dtype_code(w), static_cast<int>(K), static_cast<int>(C), cur_stream());
  TORCH_CHECK(rc == 0, "conv1x1_bwd_fused: launch rejected");
  return {dzo, part, dw};
}

// ---------------------------------------------------------------- flash attention
// q, k, v, o, ... are [B, H, T, D] views (any batch/head/token strides, contiguous D,
// 16-byte aligned rows); D in {64, 128}; bf16.
bool attn_supported(const at::Tensor& t) {
  if (!t.is_cuda() || t.scalar_type() != at::kBFloat16 || t.dim() != 4) return false;
  const int64_t D = t.size(3);
  if (D != 64 && D != 128) return false;
  if (t.stride(3) != 1) return false;
  for (int i = 0; i < 3; ++i)
    if (t.stride(i) % 8 != 0) return false;
  return (reinterpret_cast<uintptr_t>(t.data_ptr()) & 15) == 0;
}

void check_attn(const at::Tensor& t, const at::Tensor& ref, const char* what) {
  TORCH_CHECK(attn_supported(t), what, ": unsupported layout (need bf16 [B,H,T,D], D in {64,128}, contiguous D, "
              "16-byte aligned strides)");
  TORCH_CHECK(t.sizes() == ref.sizes(), what, " shape mismatch");
}

void push_strides(std::vector<int64_t>& s, const at::Tensor& t) {
  s.push_back(t.stride(0));
  s.push_back(t.stride(1));
  s.push_back(t.stride(2));
}

// Optional key-padding mask: uint8 [B, Tpad] (contiguous rows, Tpad a multiple of 64 and >= T;
// zero = padded key).  Dropout: probability drop_p in [0, 1) with a 32-bit seed.
const uint8_t* check_kmask(const c10::optional<at::Tensor>& km, const at::Tensor& q, int64_t* stride) {
  *stride = 0;
  if (!km.has_value() || !km->defined()) return nullptr;
  const at::Tensor& m = *km;
  TORCH_CHECK(m.is_cuda() && m.scalar_type() == at::kByte && m.dim() == 2 && m.stride(1) == 1,
              "key mask: uint8 [B, Tpad] with contiguous rows");
  TORCH_CHECK(m.size(0) == q.size(0) && m.size(1) >= q.size(2) && m.size(1) % 64 == 0 && m.stride(0) % 64 == 0,
              "key mask: [B, Tpad] with Tpad >= T a multiple of 64");
  TORCH_CHECK(m.device() == q.device(), "key mask on another device");
  *stride = m.stride(0);
  return m.data_ptr<uint8_t>();
}

std::vector<at::Tensor> attn_fwd(const at::Tensor& q, const at::Tensor& k, const at::Tensor& v, bool causal,
                                 double scale, const c10::optional<at::Tensor>& kmask, double drop_p, int64_t seed,
                                 const c10::optional<at::Tensor>& seed_t) {
  check_attn(q, q, "q");
  check_attn(k, q, "k");
  check_attn(v, q, "v");
  TORCH_CHECK(drop_p >= 0.0 && drop_p < 1.0, "dropout probability must be in [0, 1)");
  int64_t kms = 0;
  const uint8_t* km = check_kmask(kmask, q, &kms);
  const int64_t B = q.size(0), H = q.size(1), T = q.size(2), D = q.size(3);
  // output in [B, T, H, D] memory (so "merge heads" is a free view), returned as [B, H, T, D]
  auto o = at::empty({B, T, H, D}, q.options()).permute({0, 2, 1, 3});
  auto lse = at::empty({B, H, T}, q.options().dtype(at::kFloat));
  std::vector<int64_t> s;
  push_strides(s, q);
  push_strides(s, k);
  push_strides(s, v);
  push_strides(s, o);
  if (B * H * T > 0)
    damd_attn_fwd_launch(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr<float>(), s.data(),
                         static_cast<int>(B), static_cast<int>(H), static_cast<int>(T), static_cast<int>(D),
                         static_cast<float>(scale), causal ? 1 : 0, km, kms, static_cast<uint32_t>(seed),
                         seed_ptr(seed_t, q), static_cast<float>(drop_p), cur_stream());
  return {o, lse};
}

void attn_bwd(const at::Tensor& dout, const at::Tensor& q, const at::Tensor& k, const at::Tensor& v,
              const at::Tensor& o, const at::Tensor& lse, at::Tensor& dq, at::Tensor& dk, at::Tensor& dv, bool causal,
              double scale, const c10::optional<at::Tensor>& kmask, double drop_p, int64_t seed,
              const c10::optional<at::Tensor>& seed_t) {
  check_attn(q, q, "q");
  check_attn(k, q, "k");
  check_attn(v, q, "v");
  check_attn(o, q, "o");
  check_attn(dout, q, "dout");
  check_attn(dq, q, "dq");
  check_attn(dk, q, "dk");
  check_attn(dv, q, "dv");
  const int64_t B = q.size(0), H = q.size(1), T = q.size(2), D = q.size(3);
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == B * H * T, "lse [B,H,T] f32");
  auto delta = at::empty({B, H, T}, lse.options());
  int64_t kms = 0;
  const uint8_t* km = check_kmask(kmask, q, &kms);

  std::vector<int64_t> s;
  const at::Tensor* order[] = {&q, &k, &v, &o, &dout, &dk, &dv, &dq};
  for (const at::Tensor* t : order) push_strides(s, *t);
  if (B * H * T > 0)
    damd_attn_bwd_launch(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dout.data_ptr(),
                         lse.data_ptr<float>(), delta.data_ptr<float>(), nullptr, dq.data_ptr(),
                         dk.data_ptr(), dv.data_ptr(), s.data(), static_cast<int>(B), static_cast<int>(H),
                         static_cast<int>(T), static_cast<int>(D), static_cast<float>(scale), causal ? 1 : 0,
                         km, kms, static_cast<uint32_t>(seed), seed_ptr(seed_t, q), static_cast<float>(drop_p),
                         cur_stream());
}

// ---------------------------------------------------------------- fused LM loss / bias grad
void check_lm(const at::Tensor& logits, const at::Tensor& labels) {
  TORCH_CHECK(logits.is_cuda() && logits.scalar_type() == at::kBFloat16 && logits.is_contiguous(),
              "logits must be a contiguous bf16 GPU tensor [B, T, Vp]");
  TORCH_CHECK(logits.dim() == 3 && logits.size(2) % 8 == 0, "logits must be [B, T, Vp] with Vp % 8 == 0");
  TORCH_CHECK(labels.is_cuda() && labels.scalar_type() == at::kLong && labels.is_contiguous() && labels.dim() == 2 &&
                  labels.size(0) == logits.size(0) && labels.size(1) == logits.size(1),
              "labels must be contiguous int64 [B, T]");
}

std::vector<at::Tensor> lm_ce_fwd(const at::Tensor& logits, const at::Tensor& labels, int64_t V,
                                  int64_t ignore_index) {
  check_lm(logits, labels);
  const int64_t B = logits.size(0), T = logits.size(1), Vp = logits.size(2);
  TORCH_CHECK(V > 0 && V <= Vp, "valid vocabulary must be in (0, Vp]");
  auto opts = logits.options().dtype(at::kFloat);
  auto loss = at::empty({B, T}, opts);
  auto lse = at::empty({B, T}, opts);
  damd_lm_ce_fwd_launch(logits.data_ptr(), labels.data_ptr<int64_t>(), B * T, static_cast<int>(T),
                        static_cast<int>(V), static_cast<int>(Vp), ignore_index, loss.data_ptr<float>(),
                        lse.data_ptr<float>(), cur_stream());
  return {loss, lse};
}

void lm_ce_bwd(const at::Tensor& logits, const at::Tensor& labels, const at::Tensor& lse, const at::Tensor& scale,
               int64_t V, int64_t ignore_index, at::Tensor& dlogits) {
  check_lm(logits, labels);
  TORCH_CHECK(dlogits.sizes() == logits.sizes() && dlogits.is_contiguous() &&
                  dlogits.scalar_type() == at::kBFloat16, "dlogits must match logits");
  TORCH_CHECK(lse.scalar_type() == at::kFloat && lse.is_contiguous() && lse.numel() == labels.numel(), "lse");
  TORCH_CHECK(scale.scalar_type() == at::kFloat && scale.is_cuda() && scale.numel() == 1, "scale: f32 scalar");
  const int64_t B = logits.size(0), T = logits.size(1), Vp = logits.size(2);
  damd_lm_ce_bwd_launch(logits.data_ptr(), labels.data_ptr<int64_t>(), lse.data_ptr<float>(), scale.data_ptr<float>(),
                        B * T, static_cast<int>(T), static_cast<int>(V), static_cast<int>(Vp), ignore_index,
                        dlogits.data_ptr(), cur_stream());
}

at::Tensor bias_grad(const at::Tensor& g, at::ScalarType out_dtype) {
  TORCH_CHECK(g.is_cuda() && g.scalar_type() == at::kBFloat16 && g.is_contiguous(), "g: contiguous bf16 GPU tensor");
  const int64_t N = g.size(-1), M = g.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(N % 8 == 0, "bias_grad needs N % 8 == 0");
  TORCH_CHECK(out_dtype == at::kFloat || out_dtype == at::kBFloat16, "out dtype f32/bf16");
  auto out = at::empty({N}, g.options().dtype(out_dtype));
  const int splits = damd_bias_grad_splits(M, static_cast<int>(N));
  auto part = at::empty({splits, N}, g.options().dtype(at::kFloat));
  damd_bias_grad_launch(g.data_ptr(), M, static_cast<int>(N), splits, part.data_ptr<float>(), nullptr, 0,
                        cur_stream());  // partial rows only
  damd_norm_wgrad_finalize_launch(part.data_ptr<float>(), nullptr, splits, static_cast<int>(N), out.data_ptr(),
                                  nullptr, out_dtype == at::kFloat ? 0 : 1, cur_stream());
  return out;
}

// gelu (tanh approximation) of a contiguous bf16 tensor (numel % 8 == 0)
at::Tensor gelu_fwd(const at::Tensor& h) {
  TORCH_CHECK(h.is_cuda() && h.scalar_type() == at::kBFloat16 && h.is_contiguous() && h.numel() % 8 == 0 &&
              (reinterpret_cast<uintptr_t>(h.data_ptr()) & 15) == 0, "gelu_fwd: contiguous bf16 GPU tensor, numel % 8 == 0");
  auto g = at::empty_like(h);
  damd_gelu_fwd_launch(h.data_ptr(), g.data_ptr(), h.numel(), cur_stream());
  return g;
}

// (dh, dbias) for g = gelu(h), h = x W^T + b: dh = gelu'(h) * dg and dbias = column sums of dh
std::vector<at::Tensor> gelu_bwd_bias(const at::Tensor& dg, const at::Tensor& h, at::ScalarType bias_dtype) {
  TORCH_CHECK(dg.is_cuda() && dg.scalar_type() == at::kBFloat16 && dg.is_contiguous() && h.is_contiguous() &&
              h.scalar_type() == at::kBFloat16 && dg.sizes() == h.sizes(), "gelu_bwd_bias: matching contiguous bf16 tensors");
  const int64_t N = h.size(-1), M = h.numel() / std::max<int64_t>(N, 1);
  TORCH_CHECK(N % 8 == 0, "gelu_bwd_bias needs N % 8 == 0");
  TORCH_CHECK(bias_dtype == at::kFloat || bias_dtype == at::kBFloat16, "bias dtype f32/bf16");
  auto dh = at::empty_like(h);
  auto db = at::empty({N}, h.options().dtype(bias_dtype));
  const int splits = damd_bias_grad_splits(M, static_cast<int>(N));
  auto part = at::empty({splits, N}, h.options().dtype(at::kFloat));
  damd_gelu_bwd_bias_launch(dg.data_ptr(), h.data_ptr(), dh.data_ptr(), M, static_cast<int>(N), splits,
                            part.data_ptr<float>(), cur_stream());
  damd_norm_wgrad_finalize_launch(part.data_ptr<float>(), nullptr, splits, static_cast<int>(N), db.data_ptr(),
                                  nullptr, bias_dtype == at::kFloat ? 0 : 1, cur_stream());
  return {dh, db};
}

}  // namespace

at::Tensor debug_launch(int64_t n, int64_t mode) {
  TORCH_CHECK(mode >= 0 && mode <= 2, "debug_launch: mode must be 0, 1 or 2");
  at::Tensor out = at::zeros({n}, at::TensorOptions().device(at::kCUDA).dtype(at::kFloat));
  damd_debug_launch(out.data_ptr<float>(), static_cast<int>(n), static_cast<int>(mode), cur_stream());
  return out;
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.def("occupy", [](int64_t nblk, double usec) {  // CU-occupancy probe on the current stream
    static at::Tensor sink;
    if (!sink.defined()) sink = at::empty({256}, at::TensorOptions().dtype(at::kInt).device(at::kCUDA));
    damd_occupy_launch(static_cast<int>(nblk), usec, sink.data_ptr<int>(), cur_stream());
  });
  m.def("lm_ce_fwd", &lm_ce_fwd);
  m.def("lm_ce_bwd", &lm_ce_bwd);
  m.def("bias_grad", &bias_grad);
  m.def("gelu_fwd", &gelu_fwd);
  m.def("debug_launch", &debug_launch, "launch-check probe: mode 0 valid, 1 LDS over the limit, 2 oversized block");
  m.def("gelu_bwd_bias", &gelu_bwd_bias);
  m.def("attn_supported", &attn_supported);
  m.def("attn_fwd", &attn_fwd, py::arg("q"), py::arg("k"), py::arg("v"), py::arg("causal"), py::arg("scale"),
        py::arg("kmask") = py::none(), py::arg("drop_p") = 0.0, py::arg("seed") = 0, py::arg("seed_t") = py::none());
  m.def("attn_bwd", &attn_bwd, py::arg("dout"), py::arg("q"), py::arg("k"), py::arg("v"), py::arg("o"),
        py::arg("lse"), py::arg("dq"), py::arg("dk"), py::arg("dv"), py::arg("causal"), py::arg("scale"),
        py::arg("kmask") = py::none(), py::arg("drop_p") = 0.0, py::arg("seed") = 0, py::arg("seed_t") = py::none());
  m.def("bn_supported", &bn_supported);
  m.def("bn_act_fwd", &bn_act_fwd);
  m.def("bn_act_bwd", &bn_act_bwd);
  m.def("bn_bwd_from_part", &bn_bwd_from_part);
  m.def("bn_finalize_part", &bn_finalize_part);
  m.def("bn_bwd_finalize_part", &bn_bwd_finalize_part);
  m.def("bn_bwd_coef", &bn_bwd_coef);
  m.def("conv_fwd_pro2", &conv_fwd_pro2);
  m.def("bn_bwd_apply_coef", &bn_bwd_apply_coef);
  m.def("bn_apply", &bn_apply);
  m.def("bn_pool_fwd", &bn_pool_fwd);
  m.def("resid_norm_supported", &resid_norm_supported);
  m.def("resid_norm_fwd", &resid_norm_fwd, py::arg("x"), py::arg("branch"), py::arg("gamma"), py::arg("beta"),
        py::arg("eps"), py::arg("p"), py::arg("seed"), py::arg("seed_t") = py::none());
  m.def("resid_norm_bwd", &resid_norm_bwd);
  m.def("bn_pool_bwd", &bn_pool_bwd);
  m.def("global_avgpool_bwd", &global_avgpool_bwd);
  m.def("conv_supported", &conv_supported);
  m.def("conv_fwd", &conv_fwd);
  m.def("conv_dgrad_bn", &conv_dgrad_bn);
  m.def("conv_bnact_fwd", &conv_bnact_fwd);
  m.def("conv_pro_supported", &conv_pro_supported);
  m.def("conv_num_cfgs", &conv_num_cfgs_all);
  m.def("conv_v2_num_cfgs", &damd_v2_num_cfgs);  // the last conv_v2_num_cfgs() conv cfgs are conv3x3v2.hip's
  m.def("wgrad3x3_supported", &wgrad3x3_supported);
  m.def("conv1x1_bwd_fused_supported", &conv1x1_bwd_fused_supported);
  m.def("conv1x1_bwd_fused", &conv1x1_bwd_fused);
  m.def("conv3x3_wgrad", &conv3x3_wgrad);
  m.def("wgrad3x3_num_cfgs", &damd_wgrad3x3_num_cfgs);
  m.def("conv_sk_timeouts", &conv_sk_timeouts, py::arg("like"), py::arg("reset") = false);
  m.def("conv_dgrad_phase", &conv_dgrad_phase);
  m.def("conv_sk_cfg", [](int64_t cfg) { return damd_conv_cfg_is_sk(static_cast<int>(cfg)) != 0; });
  m.def("wgrad_num_cfgs", &damd_wgrad_num_cfgs);
  m.def("wgrad_supported", &wgrad_supported);
  m.def("conv_wgrad", &conv_wgrad);
  m.def("conv_default_cfg", [](int64_t K) { return damd_conv_default_cfg(static_cast<int>(K), 0); });
  m.def("stem_conv_supported", &stem_conv_supported);
  m.def("stem_conv_fwd", &stem_conv_fwd);
  m.def("stem_conv_wgrad", &stem_conv_wgrad);
  m.def("stem_pool_supported", &stem_pool_supported);
  m.def("stem_pool_fwd", &stem_pool_fwd);
  m.def("stem_pool_bwd", &stem_pool_bwd);
  m.doc() = "determined_amd CDNA4 HIP kernels";
  m.def("build_chunk_table", &build_chunk_table);
  m.def("chunk_entry_bytes", &chunk_entry_bytes);
  m.def("adam_step", &adam_step);
  m.def("sgd_step", &sgd_step);
  m.def("l2norm_partial", &l2norm_partial);
  m.def("finalize", &finalize);
  m.def("step_incr", &step_incr);
  m.def("scale_grads", &scale_grads);
  m.def("norm_fwd", &norm_fwd);
  m.def("norm_bwd", &norm_bwd);
}
