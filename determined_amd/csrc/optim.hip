// Multi-tensor optimizer kernels for CDNA4 (gfx950).
//
// One launch updates every parameter of an optimizer: the host builds a persistent
// chunk table (device memory, rebuilt only when tensor storage moves) so a step is
// three launches total, with no host synchronisation:
//   1. l2norm_partial   : sum(g^2) per chunk (+ non-finite detection)      [optional]
//   2. finalize         : global norm, clip coefficient, AMP inv-scale,
//                         found_inf, device-side step counter update
//   3. adamw / sgd      : reads the device scale + found_inf, updates p/m/v and
//                         the optional bf16 shadow copy of the parameter.
// This replaces the reference's per-parameter torch optimizer loop plus the
// separate clip_grad_norm_ / GradScaler.unscale_ passes
// (reference: harness/determined/pytorch/_pytorch_context.py:814 step_optimizer).
//
// Work decomposition: one 256-thread block (4 waves) per chunk of <= kChunk
// elements; 16-byte vector accesses when every pointer of a chunk is aligned.

#include "common.h"
#include <math.h>

namespace damd {

constexpr int kChunk = 16384;
constexpr int kMaxGroups = 8;
constexpr int kOptThreads = 256;

struct MTChunk {
  void* p;         // parameter (fp32 master or param storage)
  const void* g;   // gradient
  float* s0;       // exp_avg | momentum buffer
  float* s1;       // exp_avg_sq
  void* p_lp;      // optional bf16 shadow copy of p (nullptr if none)
  int32_t n;       // elements in this chunk
  int32_t group;   // param-group index (< kMaxGroups)
};

struct GroupHyper {
  float lr[kMaxGroups];
  float wd[kMaxGroups];
  float beta1[kMaxGroups];   // adam beta1 | sgd momentum
  float beta2[kMaxGroups];   // adam beta2 | sgd dampening
  float eps[kMaxGroups];
  int32_t flag[kMaxGroups];  // adam: 1=decoupled (AdamW); sgd: 1=nesterov
};

// ----------------------------------------------------------------------------- AdamW
template <typename PT, typename GT, bool LP>
__global__ void __launch_bounds__(kOptThreads)
adam_kernel(const MTChunk* __restrict__ chunks, GroupHyper hp, const float* __restrict__ scale_ptr,
            const int32_t* __restrict__ found_inf, const float* __restrict__ step_ptr, int maximize) {
  if (found_inf != nullptr && *found_inf) return;
  const MTChunk c = chunks[blockIdx.x];
  const int grp = c.group;
  const float lr = hp.lr[grp], wd = hp.wd[grp], b1 = hp.beta1[grp], b2 = hp.beta2[grp],
              eps = hp.eps[grp];
  const bool decoupled = hp.flag[grp] != 0;
  const float step = *step_ptr;
  const float bc1 = 1.f - powf(b1, step);
  const float bc2_sqrt = sqrtf(1.f - powf(b2, step));
  const float step_size = lr / bc1;
  const float gs = scale_ptr ? *scale_ptr : 1.f;
  const float sgn = maximize ? -1.f : 1.f;
  const float decay = 1.f - lr * wd;

  PT* __restrict__ p = static_cast<PT*>(c.p);
  const GT* __restrict__ g = static_cast<const GT*>(c.g);
  float* __restrict__ m = c.s0;
  float* __restrict__ v = c.s1;
  bf16_t* __restrict__ plp = static_cast<bf16_t*>(c.p_lp);

  auto upd = [&](float pv, float gv, float& mv, float& vv) -> float {
    gv = sgn * gv * gs;
    if (decoupled) pv *= decay; else gv += wd * pv;
    mv = b1 * mv + (1.f - b1) * gv;
    vv = b2 * vv + (1.f - b2) * gv * gv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    return pv - step_size * mv / denom;
  };

  const bool vec = (c.n % 4 == 0) && is_aligned16(p) && is_aligned16(m) && is_aligned16(v) &&
                   ((reinterpret_cast<uintptr_t>(g) & (sizeof(GT) * 4 - 1)) == 0) &&
                   (!LP || (reinterpret_cast<uintptr_t>(plp) & 7) == 0) &&
                   ((reinterpret_cast<uintptr_t>(p) & (sizeof(PT) * 4 - 1)) == 0);
  if (vec) {
    for (int i = threadIdx.x * 4; i < c.n; i += kOptThreads * 4) {
      float4 pv = Vec4<PT>::ld(p + i);
      float4 gv = Vec4<GT>::ld(g + i);
      float4 mv = *reinterpret_cast<const float4*>(m + i);
      float4 vv = *reinterpret_cast<const float4*>(v + i);
      pv.x = upd(pv.x, gv.x, mv.x, vv.x);
      pv.y = upd(pv.y, gv.y, mv.y, vv.y);
      pv.z = upd(pv.z, gv.z, mv.z, vv.z);
      pv.w = upd(pv.w, gv.w, mv.w, vv.w);
      Vec4<PT>::st(p + i, pv);
      *reinterpret_cast<float4*>(m + i) = mv;
      *reinterpret_cast<float4*>(v + i) = vv;
      if (LP) Vec4<bf16_t>::st(plp + i, pv);
    }
  } else {
    for (int i = threadIdx.x; i < c.n; i += kOptThreads) {
      float mv = m[i], vv = v[i];
      const float pv = upd(Elem<PT>::ld(p, i), Elem<GT>::ld(g, i), mv, vv);
      Elem<PT>::st(p, i, pv);
      m[i] = mv; v[i] = vv;
      if (LP) plp[i] = f2bf(pv);
    }
  }
}

// ----------------------------------------------------------------------------- SGD
// torch.optim.SGD semantics: g += wd*p; buf = first ? g : mom*buf + (1-damp)*g;
// g = nesterov ? g + mom*buf : buf; p -= lr*g.
template <typename PT, typename GT, bool LP, bool MOM>
__global__ void __launch_bounds__(kOptThreads)
sgd_kernel(const MTChunk* __restrict__ chunks, GroupHyper hp, const float* __restrict__ scale_ptr,
           const int32_t* __restrict__ found_inf, const float* __restrict__ step_ptr, int maximize) {
  if (found_inf != nullptr && *found_inf) return;
  const MTChunk c = chunks[blockIdx.x];
  const int grp = c.group;
  const float lr = hp.lr[grp], wd = hp.wd[grp], mom = hp.beta1[grp], damp = hp.beta2[grp];
  const bool nesterov = hp.flag[grp] != 0;
  const bool first = *step_ptr <= 1.f;
  const float gs = (scale_ptr ? *scale_ptr : 1.f) * (maximize ? -1.f : 1.f);

  PT* __restrict__ p = static_cast<PT*>(c.p);
  const GT* __restrict__ g = static_cast<const GT*>(c.g);
  float* __restrict__ buf = c.s0;
  bf16_t* __restrict__ plp = static_cast<bf16_t*>(c.p_lp);

  auto upd = [&](float pv, float gv, float& bv) -> float {
    gv = gv * gs + wd * pv;
    if (MOM) {
      bv = first ? gv : mom * bv + (1.f - damp) * gv;
      gv = nesterov ? gv + mom * bv : bv;
    }
    return pv - lr * gv;
  };

  const bool vec = (c.n % 4 == 0) && (!MOM || is_aligned16(buf)) &&
                   ((reinterpret_cast<uintptr_t>(g) & (sizeof(GT) * 4 - 1)) == 0) &&
                   ((reinterpret_cast<uintptr_t>(p) & (sizeof(PT) * 4 - 1)) == 0) &&
                   (!LP || (reinterpret_cast<uintptr_t>(plp) & 7) == 0);
  if (vec) {
    for (int i = threadIdx.x * 4; i < c.n; i += kOptThreads * 4) {
      float4 pv = Vec4<PT>::ld(p + i);
      const float4 gv = Vec4<GT>::ld(g + i);
      float4 bv = MOM ? *reinterpret_cast<const float4*>(buf + i) : make_float4(0, 0, 0, 0);
      pv.x = upd(pv.x, gv.x, bv.x);
      pv.y = upd(pv.y, gv.y, bv.y);
      pv.z = upd(pv.z, gv.z, bv.z);
      pv.w = upd(pv.w, gv.w, bv.w);
      Vec4<PT>::st(p + i, pv);
      if (MOM) *reinterpret_cast<float4*>(buf + i) = bv;
      if (LP) Vec4<bf16_t>::st(plp + i, pv);
    }
  } else {
    for (int i = threadIdx.x; i < c.n; i += kOptThreads) {
      float bv = MOM ? buf[i] : 0.f;
      const float pv = upd(Elem<PT>::ld(p, i), Elem<GT>::ld(g, i), bv);
      Elem<PT>::st(p, i, pv);
      if (MOM) buf[i] = bv;
      if (LP) plp[i] = f2bf(pv);
    }
  }
}

// ----------------------------------------------------------------------------- L2 norm
// Per-chunk sum of squares of the gradient; partial[b] = sum(g^2) of chunk b.
template <typename GT>
__global__ void __launch_bounds__(kOptThreads)
l2norm_partial_kernel(const MTChunk* __restrict__ chunks, float* __restrict__ partial) {
  __shared__ float red[kOptThreads / kWave];
  const MTChunk c = chunks[blockIdx.x];
  const GT* __restrict__ g = static_cast<const GT*>(c.g);
  float acc = 0.f;
  if ((c.n % 4 == 0) && ((reinterpret_cast<uintptr_t>(g) & (sizeof(GT) * 4 - 1)) == 0)) {
    for (int i = threadIdx.x * 4; i < c.n; i += kOptThreads * 4) {
      const float4 v = Vec4<GT>::ld(g + i);
      acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
  } else {
    for (int i = threadIdx.x; i < c.n; i += kOptThreads) {
      const float v = Elem<GT>::ld(g, i);
      acc += v * v;
    }
  }
  const float s = block_sum<kOptThreads>(acc, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}

// Single-block finalize: total norm, clip coefficient, combined grad scale, found_inf,
// and the device-side optimizer step counter (not advanced on overflow).
//   out[0] = grad scale to apply (inv_loss_scale * clip_coef)
//   out[1] = total grad norm (of unscaled grads)
__global__ void __launch_bounds__(1024)
finalize_kernel(const float* __restrict__ partial, int n_partial, float inv_loss_scale,
                const float* __restrict__ inv_scale_ptr, float max_norm, float* __restrict__ out,
                int32_t* __restrict__ found_inf, float* __restrict__ step_ptr, int check_inf) {
  __shared__ float red[1024 / kWave];
  float acc = 0.f;
  for (int i = threadIdx.x; i < n_partial; i += 1024) acc += partial[i];
  const float tot = block_sum<1024>(acc, red);
  if (threadIdx.x == 0) {
    const float inv = inv_scale_ptr ? *inv_scale_ptr : inv_loss_scale;
    const float norm = sqrtf(tot) * inv;
    const bool bad = check_inf && !isfinite(norm);
    float coef = 1.f;
    if (max_norm > 0.f && isfinite(norm)) coef = fminf(1.f, max_norm / (norm + 1e-6f));
    out[0] = inv * coef;
    out[1] = norm;
    if (found_inf) *found_inf = bad ? 1 : 0;
    if (step_ptr && !bad) *step_ptr += 1.f;
  }
}

__global__ void step_incr_kernel(float* step_ptr, const int32_t* found_inf) {
  if (found_inf == nullptr || *found_inf == 0) *step_ptr += 1.f;
}

// In-place multi-tensor scale of gradients (g *= *scale). Used for the
// non-fused-optimizer path of clip/unscale.
template <typename GT>
__global__ void __launch_bounds__(kOptThreads)
scale_kernel(const MTChunk* __restrict__ chunks, const float* __restrict__ scale_ptr) {
  const MTChunk c = chunks[blockIdx.x];
  GT* g = const_cast<GT*>(static_cast<const GT*>(c.g));
  const float s = *scale_ptr;
  for (int i = threadIdx.x; i < c.n; i += kOptThreads) Elem<GT>::st(g, i, Elem<GT>::ld(g, i) * s);
}

}  // namespace damd

// ----------------------------------------------------------------------------- launchers
using namespace damd;

void damd_adam_launch(const void* chunks, int n_chunks, const GroupHyper& hp, const float* scale_ptr,
                      const int32_t* found_inf, const float* step_ptr, int maximize, int p_dtype,
                      int g_dtype, int has_lp, hipStream_t stream) {
  if (n_chunks <= 0) return;
  const MTChunk* c = static_cast<const MTChunk*>(chunks);
#define L_ADAM(...) DAMD_LAUNCH((adam_kernel<__VA_ARGS__>), dim3(n_chunks), dim3(kOptThreads), 0, stream, c, hp, scale_ptr, found_inf, step_ptr, maximize)
  if (p_dtype == 0 && g_dtype == 0) { if (has_lp) L_ADAM(float, float, true); else L_ADAM(float, float, false); }
  else if (p_dtype == 0 && g_dtype == 1) { if (has_lp) L_ADAM(float, bf16_t, true); else L_ADAM(float, bf16_t, false); }
  else if (p_dtype == 1 && g_dtype == 1) L_ADAM(bf16_t, bf16_t, false);
  else L_ADAM(bf16_t, float, false);
#undef L_ADAM
  DAMD_CHECK_LAUNCH();
}

void damd_sgd_launch(const void* chunks, int n_chunks, const GroupHyper& hp, const float* scale_ptr,
                     const int32_t* found_inf, const float* step_ptr, int maximize, int p_dtype,
                     int g_dtype, int has_lp, int momentum, hipStream_t stream) {
  if (n_chunks <= 0) return;
  const MTChunk* c = static_cast<const MTChunk*>(chunks);
#define L_SGD(...) DAMD_LAUNCH((sgd_kernel<__VA_ARGS__>), dim3(n_chunks), dim3(kOptThreads), 0, stream, c, hp, scale_ptr, found_inf, step_ptr, maximize)
  if (momentum) {
    if (p_dtype == 0 && g_dtype == 0) { if (has_lp) L_SGD(float, float, true, true); else L_SGD(float, float, false, true); }
    else if (p_dtype == 0 && g_dtype == 1) { if (has_lp) L_SGD(float, bf16_t, true, true); else L_SGD(float, bf16_t, false, true); }
    else if (p_dtype == 1 && g_dtype == 1) L_SGD(bf16_t, bf16_t, false, true);
    else L_SGD(bf16_t, float, false, true);
  } else {
    if (p_dtype == 0 && g_dtype == 0) { if (has_lp) L_SGD(float, float, true, false); else L_SGD(float, float, false, false); }
    else if (p_dtype == 0 && g_dtype == 1) { if (has_lp) L_SGD(float, bf16_t, true, false); else L_SGD(float, bf16_t, false, false); }
    else if (p_dtype == 1 && g_dtype == 1) L_SGD(bf16_t, bf16_t, false, false);
    else L_SGD(bf16_t, float, false, false);
  }
#undef L_SGD
  DAMD_CHECK_LAUNCH();
}

void damd_l2norm_partial_launch(const void* chunks, int n_chunks, float* partial, int g_dtype,
                                hipStream_t stream) {
  if (n_chunks <= 0) return;
  const MTChunk* c = static_cast<const MTChunk*>(chunks);
  if (g_dtype == 0)
    DAMD_LAUNCH(l2norm_partial_kernel<float>, dim3(n_chunks), dim3(kOptThreads), 0, stream, c, partial);
  else
    DAMD_LAUNCH(l2norm_partial_kernel<bf16_t>, dim3(n_chunks), dim3(kOptThreads), 0, stream, c, partial);
  DAMD_CHECK_LAUNCH();
}

void damd_finalize_launch(const float* partial, int n_partial, float inv_loss_scale,
                          const float* inv_scale_ptr, float max_norm, float* out, int32_t* found_inf,
                          float* step_ptr, int check_inf, hipStream_t stream) {
  DAMD_LAUNCH(finalize_kernel, dim3(1), dim3(1024), 0, stream, partial, n_partial,
                     inv_loss_scale, inv_scale_ptr, max_norm, out, found_inf, step_ptr, check_inf);
  DAMD_CHECK_LAUNCH();
}

void damd_step_incr_launch(float* step_ptr, const int32_t* found_inf, hipStream_t stream) {
  DAMD_LAUNCH(step_incr_kernel, dim3(1), dim3(1), 0, stream, step_ptr, found_inf);
  DAMD_CHECK_LAUNCH();
}

void damd_scale_launch(const void* chunks, int n_chunks, const float* scale_ptr, int g_dtype,
                       hipStream_t stream) {
  if (n_chunks <= 0) return;
  const MTChunk* c = static_cast<const MTChunk*>(chunks);
  if (g_dtype == 0)
    DAMD_LAUNCH(scale_kernel<float>, dim3(n_chunks), dim3(kOptThreads), 0, stream, c, scale_ptr);
  else
    DAMD_LAUNCH(scale_kernel<bf16_t>, dim3(n_chunks), dim3(kOptThreads), 0, stream, c, scale_ptr);
  DAMD_CHECK_LAUNCH();
}
