// Channels-last (NHWC) BatchNorm + optional residual add + optional ReLU, fwd and bwd, for gfx950.
//
// ResNet training is bandwidth-bound on BN/ReLU/add, not on its convolutions: stock PyTorch
// runs BN stats, BN transform, residual add, ReLU, ReLU-bwd, BN-bwd-reduce and BN-bwd-elementwise
// as seven HBM passes.  Here one "BNAct" op is four passes total:
//   fwd:  stats (read x)  ->  apply  y = relu(x*scale + shift [+ res])   (read x[,res], write y)
//   bwd:  reduce (read dy, x[,res]) -> dx = A*dy' + B*x + C, dres = dy'  (read dy, x[,res]; write)
// where dy' = dy * [pre-activation > 0].  The ReLU mask is RECOMPUTED from x (and res) instead
// of reading the saved output, so the backward never touches y.
//
// Tensor view: x is [M, C] row-major (M = N*H*W).  A thread owns one 16-byte vector of
// 8 channels (bf16) and walks rows; with TPR = C/8 threads per row a 256-thread block
// covers 256/TPR rows per iteration, so every wave-instruction reads 1 KiB contiguous.
// Statistics use a per-channel shift K_c = x[0, c] ("shifted data" variance): sums of
// (x-K) and (x-K)^2 are plain sums, so block partials merge by addition with no
// E[x^2]-E[x]^2 cancellation when |mean| >> std.
// Requirements (checked on the host, torch fallback otherwise): C % 8 == 0 and C/8 a power
// of two (every ResNet width) and 16-byte aligned base pointers.

#include "common.h"

#include <math.h>

namespace damd {

constexpr int kBNThreads = 256;

template <typename T> struct V8;
template <> struct V8<bf16_t> {
  static __device__ __forceinline__ void ld(const bf16_t* p, float* o) {
    const bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = bf2f(r.v[k]);
  }
  static __device__ __forceinline__ void st(bf16_t* p, const float* o) {
    bf16x8 r;
#pragma unroll
    for (int k = 0; k < 8; k += 2) {
      const u16v2_t q = f2bf2(o[k], o[k + 1]);
      r.v[k] = q[0];
      r.v[k + 1] = q[1];
    }
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};
template <> struct V8<float> {
  static __device__ __forceinline__ void ld(const float* p, float* o) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float* o) {
    reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
};

struct Geo {
  int TPR;   // threads (8-channel vectors) per row
  int RS;    // rows per block iteration (>=1)
  int G;     // channel groups per thread (TPR > 256)
};

__device__ __forceinline__ Geo geo(int C) {
  Geo g;
  g.TPR = C / 8;
  g.RS = g.TPR <= kBNThreads ? kBNThreads / g.TPR : 1;
  g.G = g.TPR <= kBNThreads ? 1 : g.TPR / kBNThreads;
  return g;
}

// ----------------------------------------------------------------------------- fwd stats
// part: [nb][2][C]  (sum(x-K), sum((x-K)^2)) per block.
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
bn_stats_kernel(const T* __restrict__ x, int64_t M, int C, int64_t rows_per_block, float* __restrict__ part) {
  const Geo g = geo(C);
  const int tid = threadIdx.x;
  const int cg0 = g.TPR <= kBNThreads ? tid % g.TPR : tid;
  const int rsub = g.TPR <= kBNThreads ? tid / g.TPR : 0;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  __shared__ float red[kBNThreads * 8];
  for (int gi = 0; gi < g.G; ++gi) {
    const int cg = cg0 + gi * kBNThreads;
    float K[8], s[8], ss[8];
    V8<T>::ld(x + cg * 8, K);  // row 0 pilot values
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; ss[k] = 0.f; }
    int64_t r = r0 + rsub;
    for (; r + 3 * g.RS < r1; r += 4 * g.RS) {
      float a[4][8];
#pragma unroll
      for (int u = 0; u < 4; ++u) V8<T>::ld(x + (r + u * g.RS) * C + cg * 8, a[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) { const float d = a[u][k] - K[k]; s[k] += d; ss[k] += d * d; }
    }
    for (; r < r1; r += g.RS) {
      float a[8];
      V8<T>::ld(x + r * C + cg * 8, a);
#pragma unroll
      for (int k = 0; k < 8; ++k) { const float d = a[k] - K[k]; s[k] += d; ss[k] += d * d; }
    }
    // merge the RS row-lanes that share a channel group (plain sums)
    for (int which = 0; which < 2; ++which) {
      float* v = which == 0 ? s : ss;
      if (g.RS > 1) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid * 8 + k] = v[k];
        __syncthreads();
        if (rsub == 0) {
          for (int q = 1; q < g.RS; ++q)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += red[(q * g.TPR + cg0) * 8 + k];
        }
      }
      if (rsub == 0) {
        float* dst = part + (static_cast<int64_t>(blockIdx.x) * 2 + which) * C + cg * 8;
        V8<float>::st(dst, v);
      }
    }
  }
}

// ----------------------------------------------------------------------------- partial reduction
// Sums part[nb][2][C] over nb for 16 channels per block.  1024 threads = 16 channels x 64
// lanes; each lane keeps 8 independent accumulators so its loads are issued back to back
// (a serial per-thread chain over ~1000 partial rows costs ~70 us in L2 round trips).
// Result (deterministic order) lands in thread lane==0's (s, ss).
constexpr int kFinThreads = 1024;
constexpr int kFinCh = 16;                         // channels per block
constexpr int kFinLanes = kFinThreads / kFinCh;    // 64 row-lanes per channel: ~2 load rounds for nb=1024
// (finalize kernels are pure latency: 64 lanes x 8 accumulators keep the dependent rounds short)

__device__ __forceinline__ void reduce_partials(const float* __restrict__ part, int nb, int C, int c, int q,
                                                float& s, float& ss) {
  __shared__ float rs[kFinLanes][kFinCh], rq[kFinLanes][kFinCh];
  float a0[8], a1[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) { a0[u] = 0.f; a1[u] = 0.f; }
  if (c < C) {
    int bi = q;
    for (; bi + 7 * kFinLanes < nb; bi += 8 * kFinLanes) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t row = static_cast<int64_t>(bi + u * kFinLanes) * 2;
        a0[u] += part[row * C + c];
        a1[u] += part[(row + 1) * C + c];
      }
    }
    for (; bi < nb; bi += kFinLanes) {
      a0[0] += part[(static_cast<int64_t>(bi) * 2) * C + c];
      a1[0] += part[(static_cast<int64_t>(bi) * 2 + 1) * C + c];
    }
  }
  float t0 = 0.f, t1 = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) { t0 += a0[u]; t1 += a1[u]; }
  const int lane = threadIdx.x % kFinCh;
  rs[q][lane] = t0;
  rq[q][lane] = t1;
  __syncthreads();
  s = 0.f;
  ss = 0.f;
  if (q == 0) {
#pragma unroll
    for (int k = 0; k < kFinLanes; ++k) { s += rs[k][lane]; ss += rq[k][lane]; }
  }
}

// ----------------------------------------------------------------------------- fwd finalize
// Produces mean/invstd (saved for bwd), folded scale/shift (for apply) and updates the
// running statistics.  grid = ceil(C/16) blocks of 1024 threads.
template <typename WT>
__global__ void __launch_bounds__(kFinThreads)
bn_finalize_kernel(const float* __restrict__ part, int nb, int C, int64_t M, int64_t rows_per_block,
                   const void* __restrict__ xbase, int x_is_bf16, float momentum, float eps,
                   const WT* __restrict__ w, const WT* __restrict__ b, float* __restrict__ run_mean,
                   float* __restrict__ run_var, float* __restrict__ mean_out, float* __restrict__ invstd_out,
                   float* __restrict__ scale_out, float* __restrict__ shift_out) {
  const int lane = threadIdx.x % kFinCh, q = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + lane;
  float s, ss;
  reduce_partials(part, nb, C, c, q, s, ss);
  if (q == 0 && c < C) {
    // pilot: row 0 of x (bn_stats_kernel), or 0 for producer-computed plain sums (xbase null)
    const float K = xbase == nullptr ? 0.f
                    : x_is_bf16 ? bf2f(static_cast<const bf16_t*>(xbase)[c]) : static_cast<const float*>(xbase)[c];
    const float n = static_cast<float>(M);
    const float dm = s / n;
    const float var = fmaxf(ss / n - dm * dm, 0.f);
    const float mean = K + dm;
    const float invstd = rsqrtf(var + eps);
    mean_out[c] = mean;
    invstd_out[c] = invstd;
    const float wv = w ? Elem<WT>::ld(w, c) : 1.f;
    const float bv = b ? Elem<WT>::ld(b, c) : 0.f;
    scale_out[c] = wv * invstd;
    shift_out[c] = bv - mean * wv * invstd;
    if (run_mean) {
      const float unbiased = M > 1 ? var * n / (n - 1.f) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * unbiased;
    }
  }
}

// ----------------------------------------------------------------------------- fwd apply
// WMASK (residual + ReLU training path): also write one byte per 8-channel vector whose bit k is
// [output k > 0].  The backward then reads M*C/8 bytes instead of the residual tensor
// (M*C*2 bytes) in both of its passes to rebuild the ReLU mask.
template <typename T, bool RES, bool RELU, bool WMASK = false>
__global__ void __launch_bounds__(kBNThreads)
bn_apply_kernel(const T* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
                const T* __restrict__ res, T* __restrict__ y, int64_t V, int TPR, uint8_t* __restrict__ mask = nullptr) {
  const int64_t T0 = static_cast<int64_t>(blockIdx.x) * kBNThreads + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBNThreads;  // multiple of TPR
  const int cg = static_cast<int>(T0 % TPR);
  float sc[8], sh[8];
  V8<float>::ld(scale + cg * 8, sc);
  V8<float>::ld(shift + cg * 8, sh);
  for (int64_t v = T0; v < V; v += stride) {
    float a[8], r[8];
    V8<T>::ld(x + v * 8, a);
    if (RES) V8<T>::ld(res + v * 8, r);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float o = a[k] * sc[k] + sh[k];
      if (RES) o += r[k];
      if (RELU) o = fmaxf(o, 0.f);
      a[k] = o;
    }
    V8<T>::st(y + v * 8, a);
    if (WMASK) {
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) bits |= (a[k] > 0.f ? 1u : 0u) << k;
      mask[v] = static_cast<uint8_t>(bits);
    }
  }
}

// ----------------------------------------------------------------------------- bwd reduce
template <typename T>
__device__ __forceinline__ void add_v8(const T* __restrict__ p, float* d) {
  float e[8];
  V8<T>::ld(p, e);
#pragma unroll
  for (int k = 0; k < 8; ++k) d[k] += e[k];
}

// part: [nb][2][C] = (sum dy', sum dy' * (x - mean))
// MASKED: the ReLU mask comes from the forward's bit mask instead of recomputing it from
// x (and the residual), see bn_apply_kernel<..., WMASK>.
// DY2: the output fed two consumers and dy2 holds the second one's gradient; the two are
// summed on the fly instead of in a separate elementwise add (see ops/bn.py split_grad).
template <typename T, bool RES, bool RELU, bool MASKED = false, bool DY2 = false>
__global__ void __launch_bounds__(kBNThreads)
bn_bwd_reduce_kernel(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ res,
                     const float* __restrict__ mean, const float* __restrict__ scale,
                     const float* __restrict__ shift, int64_t M, int C, int64_t rows_per_block,
                     float* __restrict__ part, const uint8_t* __restrict__ mask = nullptr,
                     const T* __restrict__ dy2 = nullptr) {
  const Geo g = geo(C);
  const int tid = threadIdx.x;
  const int cg0 = g.TPR <= kBNThreads ? tid % g.TPR : tid;
  const int rsub = g.TPR <= kBNThreads ? tid / g.TPR : 0;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  __shared__ float red[kBNThreads * 8];
  for (int gi = 0; gi < g.G; ++gi) {
    const int cg = cg0 + gi * kBNThreads;
    float mu[8], sc[8], sh[8], s[8], sx[8];
    V8<float>::ld(mean + cg * 8, mu);
    if (RELU) { V8<float>::ld(scale + cg * 8, sc); V8<float>::ld(shift + cg * 8, sh); }
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; sx[k] = 0.f; }
    int64_t r = r0 + rsub;
    for (; r + g.RS < r1; r += 2 * g.RS) {
      float d[2][8], a[2][8], rr[2][8];
      uint32_t mb[2] = {0u, 0u};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int64_t off = (r + u * g.RS) * C + cg * 8;
        V8<T>::ld(dy + off, d[u]);
        if (DY2) add_v8(dy2 + off, d[u]);
        V8<T>::ld(x + off, a[u]);
        if (MASKED) mb[u] = mask[off >> 3];
        else if (RES && RELU) V8<T>::ld(res + off, rr[u]);
      }
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float dv = d[u][k];
          if (MASKED) {
            dv = (mb[u] >> k) & 1u ? dv : 0.f;
          } else if (RELU) {
            float z = a[u][k] * sc[k] + sh[k];
            if (RES) z += rr[u][k];
            dv = z > 0.f ? dv : 0.f;
          }
          s[k] += dv;
          sx[k] += dv * (a[u][k] - mu[k]);
        }
    }
    for (; r < r1; r += g.RS) {
      float d[8], a[8], rr[8];
      uint32_t mb = 0u;
      const int64_t off = r * C + cg * 8;
      V8<T>::ld(dy + off, d);
      if (DY2) add_v8(dy2 + off, d);
      V8<T>::ld(x + off, a);
      if (MASKED) mb = mask[off >> 3];
      else if (RES && RELU) V8<T>::ld(res + off, rr);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float dv = d[k];
        if (MASKED) {
          dv = (mb >> k) & 1u ? dv : 0.f;
        } else if (RELU) {
          float z = a[k] * sc[k] + sh[k];
          if (RES) z += rr[k];
          dv = z > 0.f ? dv : 0.f;
        }
        s[k] += dv;
        sx[k] += dv * (a[k] - mu[k]);
      }
    }
    for (int which = 0; which < 2; ++which) {
      float* v = which == 0 ? s : sx;
      if (g.RS > 1) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid * 8 + k] = v[k];
        __syncthreads();
        if (rsub == 0) {
          for (int q = 1; q < g.RS; ++q)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += red[(q * g.TPR + cg0) * 8 + k];
        }
      }
      if (rsub == 0) V8<float>::st(part + (static_cast<int64_t>(blockIdx.x) * 2 + which) * C + cg * 8, v);
    }
  }
}

// bwd finalize: dgamma, dbeta (fp32) and the elementwise coefficients A, B, Cc:
//   dx = A*dy' + B*x + Cc
// dgamma/dbeta are written directly in the parameter dtype (no separate cast kernels).
template <typename WT>
__global__ void __launch_bounds__(kFinThreads)
bn_bwd_finalize_kernel(const float* __restrict__ part, int nb, int C, int64_t M,
                       const float* __restrict__ mean, const float* __restrict__ invstd,
                       const float* __restrict__ scale, WT* __restrict__ dgamma, WT* __restrict__ dbeta,
                       float* __restrict__ coef /* [3][C] */) {
  const int lane = threadIdx.x % kFinCh, q = threadIdx.x / kFinCh;
  const int c = blockIdx.x * kFinCh + lane;
  float s, sx;
  reduce_partials(part, nb, C, c, q, s, sx);
  if (q == 0 && c < C) {
    const float is = invstd[c];
    const float dg = sx * is;  // sum dy' * xhat
    Elem<WT>::st(dgamma, c, dg);
    Elem<WT>::st(dbeta, c, s);
    const float n = static_cast<float>(M);
    const float sc = scale[c];
    const float A = sc;
    const float B = -sc * is * dg / n;
    const float Cc = -sc * s / n - B * mean[c];
    coef[c] = A;
    coef[C + c] = B;
    coef[2 * C + c] = Cc;
  }
}

template <typename T, bool RES, bool RELU, bool WRITE_DRES, bool MASKED = false, bool DY2 = false>
__global__ void __launch_bounds__(kBNThreads)
bn_bwd_apply_kernel(const T* __restrict__ dy, const T* __restrict__ x, const T* __restrict__ res,
                    const float* __restrict__ scale, const float* __restrict__ shift,
                    const float* __restrict__ coef, int C, T* __restrict__ dx, T* __restrict__ dres, int64_t V,
                    int TPR, const uint8_t* __restrict__ mask = nullptr, const T* __restrict__ dy2 = nullptr) {
  const int64_t T0 = static_cast<int64_t>(blockIdx.x) * kBNThreads + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBNThreads;
  const int cg = static_cast<int>(T0 % TPR);
  float A[8], B[8], Cc[8], sc[8], sh[8];
  V8<float>::ld(coef + cg * 8, A);
  V8<float>::ld(coef + C + cg * 8, B);
  V8<float>::ld(coef + 2 * C + cg * 8, Cc);
  if (RELU) { V8<float>::ld(scale + cg * 8, sc); V8<float>::ld(shift + cg * 8, sh); }
  for (int64_t v = T0; v < V; v += stride) {
    float d[8], a[8], rr[8], o[8];
    uint32_t mb = 0u;
    V8<T>::ld(dy + v * 8, d);
    if (DY2) add_v8(dy2 + v * 8, d);
    V8<T>::ld(x + v * 8, a);
    if (MASKED) mb = mask[v];
    else if (RES && RELU) V8<T>::ld(res + v * 8, rr);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float dv = d[k];
      if (MASKED) {
        dv = (mb >> k) & 1u ? dv : 0.f;
      } else if (RELU) {
        float z = a[k] * sc[k] + sh[k];
        if (RES) z += rr[k];
        dv = z > 0.f ? dv : 0.f;
      }
      d[k] = dv;
      o[k] = A[k] * dv + B[k] * a[k] + Cc[k];
    }
    V8<T>::st(dx + v * 8, o);
    if (WRITE_DRES) V8<T>::st(dres + v * 8, d);
  }
}


// ============================================================================= stem: BN+ReLU+MaxPool
// ResNet stem: y = maxpool3x3/s2/p1(relu(bn(x))).  Instead of writing relu(bn(x)) (N*H*W*C) and
// reading it back in a separate pooling pass, one kernel applies BN+ReLU on the fly while it
// pools and stores the pooled output plus the argmax (0..8, row-major in the window, first max
// wins as in PyTorch) as one byte per element.  The backward never materialises the full-size
// pooled gradient either: both BN-backward passes gather it from (dp, argmax) of the <= 4
// windows that contain each input pixel.  Traffic (bf16, C=64, 112->56): fwd reads x once and
// writes 1/4 + 1/8 of it; bwd reads x and the small (dp, argmax) twice and writes dx once.
struct PoolGeo {
  int H, W, OH, OW;
};

// (n, oh, ow) of pooled position q in 32-bit arithmetic (the host checks that the element-vector
// counts fit in 31 bits): a 64-bit division is a ~100-instruction software routine per call
__device__ __forceinline__ void pool_pos(uint32_t q, const PoolGeo& g, int64_t& n, int& oh, int& ow) {
  const uint32_t t = q / static_cast<uint32_t>(g.OW);
  ow = static_cast<int>(q - t * static_cast<uint32_t>(g.OW));
  const uint32_t nn = t / static_cast<uint32_t>(g.OH);
  oh = static_cast<int>(t - nn * static_cast<uint32_t>(g.OH));
  n = nn;
}

// window index of input (h, w) inside output window (oh, ow) (kernel 3, stride 2, pad 1)
__device__ __forceinline__ int win_pos(int h, int w, int oh, int ow) { return (h - 2 * oh + 1) * 3 + (w - 2 * ow + 1); }

template <typename T>
__global__ void __launch_bounds__(kBNThreads)
bn_relu_maxpool_fwd_kernel(const T* __restrict__ x, const float* __restrict__ scale, const float* __restrict__ shift,
                           T* __restrict__ y, uint8_t* __restrict__ idx, int64_t Vout, int TPR, PoolGeo g,
                           T* __restrict__ xarg) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBNThreads;
  const int64_t T0 = static_cast<int64_t>(blockIdx.x) * kBNThreads + threadIdx.x;
  const int cg = static_cast<int>(T0 % TPR);  // stride is a multiple of TPR
  const int C = TPR * 8;
  float sc[8], sh[8];
  V8<float>::ld(scale + cg * 8, sc);
  V8<float>::ld(shift + cg * 8, sh);
  for (int64_t v = T0; v < Vout; v += stride) {
    int64_t n;
    int oh, ow;
    pool_pos(static_cast<uint32_t>(v) / static_cast<uint32_t>(TPR), g, n, oh, ow);
    float best[8], xa[8];
    int arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; xa[k] = 0.f; }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int h = 2 * oh - 1 + kh;
      if (h < 0 || h >= g.H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int w = 2 * ow - 1 + kw;
        if (w < 0 || w >= g.W) continue;
        float a[8];
        V8<T>::ld(x + ((n * g.H + h) * g.W + w) * C + cg * 8, a);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float r = fmaxf(a[k] * sc[k] + sh[k], 0.f);
          if (r > best[k]) { best[k] = r; arg[k] = kh * 3 + kw; xa[k] = a[k]; }
        }
      }
    }
    V8<T>::st(y + v * 8, best);
    uint32_t lo = 0, hi = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) { lo |= static_cast<uint32_t>(arg[k]) << (8 * k); hi |= static_cast<uint32_t>(arg[k + 4]) << (8 * k); }
    *reinterpret_cast<uint2*>(idx + v * 8) = make_uint2(lo, hi);
    if (xarg != nullptr) V8<T>::st(xarg + v * 8, xa);
  }
}

// BN-backward reduce in the POOLED domain: every pooled gradient lands on exactly one input
// pixel (its window's argmax) and dz is linear in it, so
//   sum dz = sum_out dp [z_arg > 0],   sum dz (x - mean) = sum_out dp [z_arg > 0] (x_arg - mean)
// with x_arg the input value at the argmax (written by the forward).  Reads dp + x_arg (a
// quarter of the input each) instead of the full input plus the (dp, argmax) gathers.
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
pooled_bn_bwd_reduce_kernel(const T* __restrict__ dp, const T* __restrict__ dp2, const T* __restrict__ xarg,
                            const float* __restrict__ mean, const float* __restrict__ scale,
                            const float* __restrict__ shift, int64_t Q, int C, int64_t rows_per_block,
                            float* __restrict__ part, T* __restrict__ dzout = nullptr) {
  const Geo geo_ = geo(C);
  const int tid = threadIdx.x;
  const int cg0 = geo_.TPR <= kBNThreads ? tid % geo_.TPR : tid;
  const int rsub = geo_.TPR <= kBNThreads ? tid / geo_.TPR : 0;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(Q, r0 + rows_per_block);
  __shared__ float red[kBNThreads * 8];
  for (int gi = 0; gi < geo_.G; ++gi) {
    const int cg = cg0 + gi * kBNThreads;
    float mu[8], sc[8], sh[8], s[8], sx[8];
    V8<float>::ld(mean + cg * 8, mu);
    V8<float>::ld(scale + cg * 8, sc);
    V8<float>::ld(shift + cg * 8, sh);
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; sx[k] = 0.f; }
    for (int64_t q = r0 + rsub; q < r1; q += geo_.RS) {
      const int64_t off = q * C + cg * 8;
      float d[8], a[8];
      V8<T>::ld(dp + off, d);
      if (dp2 != nullptr) add_v8(dp2 + off, d);
      V8<T>::ld(xarg + off, a);
      float z[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float dz = (a[k] * sc[k] + sh[k]) > 0.f ? d[k] : 0.f;
        z[k] = dz;
        s[k] += dz;
        sx[k] += dz * (a[k] - mu[k]);
      }
      if (dzout != nullptr) V8<T>::st(dzout + off, z);  // the fused stem backward's routed gradient
    }
    for (int which = 0; which < 2; ++which) {
      float* v = which == 0 ? s : sx;
      if (geo_.RS > 1) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid * 8 + k] = v[k];
        __syncthreads();
        if (rsub == 0) {
          for (int qq = 1; qq < geo_.RS; ++qq)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += red[(qq * geo_.TPR + cg0) * 8 + k];
        }
      }
      if (rsub == 0) V8<float>::st(part + (static_cast<int64_t>(blockIdx.x) * 2 + which) * C + cg * 8, v);
    }
  }
}

// Pooled gradient routed back to the 2x2 input quad (2oh..2oh+1, 2ow..2ow+1) of output
// position (oh, ow): the quad's pixels lie in windows (oh..oh+1, ow..ow+1) only (stride 2), so
// the four (dp, argmax) vectors are loaded once per quad instead of once per input pixel.
// dr[2*i + j] is the gradient of input (2oh + i, 2ow + j).
template <typename T>
__device__ __forceinline__ void quad_pool_grad(const T* __restrict__ dp, const T* __restrict__ dp2,
                                               const uint8_t* __restrict__ idx, int64_t n, int oh, int ow, int cg,
                                               int C, const PoolGeo& g, float (*dr)[8]) {
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int k = 0; k < 8; ++k) dr[p][k] = 0.f;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int wh = oh + a;
    if (wh >= g.OH) continue;
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      const int ww = ow + b;
      if (ww >= g.OW) continue;
      const int64_t o = ((n * g.OH + wh) * g.OW + ww) * C + cg * 8;
      const uint2 ii = *reinterpret_cast<const uint2*>(idx + o);
      float d[8];
      V8<T>::ld(dp + o, d);
      if (dp2 != nullptr) add_v8(dp2 + o, d);  // pooled output fed two consumers
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int kh = 2 * oh + i - 2 * wh + 1;  // row of input 2oh+i inside window wh
        if (kh < 0 || kh > 2) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int kw = 2 * ow + j - 2 * ww + 1;
          if (kw < 0 || kw > 2) continue;
          const uint32_t pos = static_cast<uint32_t>(kh * 3 + kw);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            if (((ii.x >> (8 * k)) & 0xFFu) == pos) dr[2 * i + j][k] += d[k];
            if (((ii.y >> (8 * k)) & 0xFFu) == pos) dr[2 * i + j][k + 4] += d[k + 4];
          }
        }
      }
    }
  }
}

// BN-backward reduce over dz = maxpool_bwd(dp) * [bn(x) > 0]: part[nb][2][C] = (sum dz, sum dz*(x-mean)).
// Rows of this kernel are output positions (quads of 4 input pixels).
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
maxpool_bn_bwd_reduce_kernel(const T* __restrict__ dp, const T* __restrict__ dp2, const uint8_t* __restrict__ idx, const T* __restrict__ x,
                             const float* __restrict__ mean, const float* __restrict__ scale,
                             const float* __restrict__ shift, int64_t Q, int C, int64_t rows_per_block,
                             float* __restrict__ part, PoolGeo g) {
  const Geo geo_ = geo(C);
  const int tid = threadIdx.x;
  const int cg0 = geo_.TPR <= kBNThreads ? tid % geo_.TPR : tid;
  const int rsub = geo_.TPR <= kBNThreads ? tid / geo_.TPR : 0;
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * rows_per_block;
  const int64_t r1 = min(Q, r0 + rows_per_block);
  __shared__ float red[kBNThreads * 8];
  for (int gi = 0; gi < geo_.G; ++gi) {
    const int cg = cg0 + gi * kBNThreads;
    float mu[8], sc[8], sh[8], s[8], sx[8];
    V8<float>::ld(mean + cg * 8, mu);
    V8<float>::ld(scale + cg * 8, sc);
    V8<float>::ld(shift + cg * 8, sh);
#pragma unroll
    for (int k = 0; k < 8; ++k) { s[k] = 0.f; sx[k] = 0.f; }
    for (int64_t q = r0 + rsub; q < r1; q += geo_.RS) {
      int64_t n;
      int oh, ow;
      pool_pos(static_cast<uint32_t>(q), g, n, oh, ow);
      float dr[4][8];
      quad_pool_grad(dp, dp2, idx, n, oh, ow, cg, C, g, dr);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int h = 2 * oh + i;
        if (h >= g.H) continue;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int w = 2 * ow + j;
          if (w >= g.W) continue;
          float a[8];
          V8<T>::ld(x + ((n * g.H + h) * g.W + w) * C + cg * 8, a);
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const float dz = (a[k] * sc[k] + sh[k]) > 0.f ? dr[2 * i + j][k] : 0.f;
            s[k] += dz;
            sx[k] += dz * (a[k] - mu[k]);
          }
        }
      }
    }
    for (int which = 0; which < 2; ++which) {
      float* v = which == 0 ? s : sx;
      if (geo_.RS > 1) {
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 8; ++k) red[tid * 8 + k] = v[k];
        __syncthreads();
        if (rsub == 0) {
          for (int qq = 1; qq < geo_.RS; ++qq)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] += red[(qq * geo_.TPR + cg0) * 8 + k];
        }
      }
      if (rsub == 0) V8<float>::st(part + (static_cast<int64_t>(blockIdx.x) * 2 + which) * C + cg * 8, v);
    }
  }
}

// dx = A*dz + B*x + Cc over one quad of input pixels per (output position, channel group)
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
maxpool_bn_bwd_apply_kernel(const T* __restrict__ dp, const T* __restrict__ dp2, const uint8_t* __restrict__ idx, const T* __restrict__ x,
                            const float* __restrict__ scale, const float* __restrict__ shift,
                            const float* __restrict__ coef, int C, T* __restrict__ dx, int64_t VQ, int TPR, PoolGeo g) {
  const int64_t T0 = static_cast<int64_t>(blockIdx.x) * kBNThreads + threadIdx.x;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBNThreads;
  const int cg = static_cast<int>(T0 % TPR);
  float A[8], B[8], Cc[8], sc[8], sh[8];
  V8<float>::ld(coef + cg * 8, A);
  V8<float>::ld(coef + C + cg * 8, B);
  V8<float>::ld(coef + 2 * C + cg * 8, Cc);
  V8<float>::ld(scale + cg * 8, sc);
  V8<float>::ld(shift + cg * 8, sh);
  for (int64_t v = T0; v < VQ; v += stride) {
    int64_t n;
    int oh, ow;
    pool_pos(static_cast<uint32_t>(v) / static_cast<uint32_t>(TPR), g, n, oh, ow);
    float dr[4][8];
    quad_pool_grad(dp, dp2, idx, n, oh, ow, cg, C, g, dr);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int h = 2 * oh + i;
      if (h >= g.H) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int w = 2 * ow + j;
        if (w >= g.W) continue;
        const int64_t off = ((n * g.H + h) * g.W + w) * C + cg * 8;
        float a[8], o[8];
        V8<T>::ld(x + off, a);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float dz = (a[k] * sc[k] + sh[k]) > 0.f ? dr[2 * i + j][k] : 0.f;
          o[k] = A[k] * dz + B[k] * a[k] + Cc[k];
        }
        V8<T>::st(dx + off, o);
      }
    }
  }
}

}  // namespace damd

using namespace damd;

namespace {
int64_t rows_per_block_for(int64_t M, int C, int* nb_out) {
  // ~1024 blocks (4 per CU) for big tensors; at least 16 rows per block.
  int64_t nb = 1024;
  int64_t rpb = (M + nb - 1) / nb;
  const int RS = (C / 8) <= kBNThreads ? kBNThreads / (C / 8) : 1;
  if (rpb < 4 * RS) rpb = 4 * RS;
  nb = (M + rpb - 1) / rpb;
  *nb_out = static_cast<int>(nb);
  return rpb;
}

int apply_grid(int64_t V, int TPR) {
  // grid*256 must be a multiple of TPR (channel group constant per thread)
  int64_t blocks = (V + kBNThreads - 1) / kBNThreads;
  if (blocks > 2048) blocks = 2048;
  const int mult = TPR > kBNThreads ? TPR / kBNThreads : 1;
  blocks = (blocks + mult - 1) / mult * mult;
  return static_cast<int>(blocks);
}
}  // namespace

int damd_bn_num_blocks(int64_t M, int C) {
  int nb;
  rows_per_block_for(M, C, &nb);
  return nb;
}

// x_dtype/w_dtype: 0 = fp32, 1 = bf16
void damd_bn_fwd_launch(const void* x, const void* res, void* y, int64_t M, int C, const void* w, const void* b,
                        float* run_mean, float* run_var, float momentum, float eps, float* part, float* mean,
                        float* invstd, float* scale, float* shift, int relu, int x_dtype, int w_dtype,
                        hipStream_t st, uint8_t* mask, const float* pre_part, int pre_nb) {
  int nb;
  const int64_t rpb = rows_per_block_for(M, C, &nb);
  const void* pilot = x;
  if (pre_part != nullptr) {  // plain (sum, sum sq) partials from the producing convolution
    part = const_cast<float*>(pre_part);
    nb = pre_nb;
    pilot = nullptr;
  } else if (x_dtype == 1) {
    DAMD_LAUNCH(bn_stats_kernel<bf16_t>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(x), M, C, rpb, part);
  } else {
    DAMD_LAUNCH(bn_stats_kernel<float>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const float*>(x), M, C, rpb, part);
  }
  const dim3 fg((C + kFinCh - 1) / kFinCh);
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_finalize_kernel<bf16_t>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, rpb, pilot, x_dtype == 1, momentum, eps,
                       static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(b), run_mean, run_var, mean, invstd, scale, shift);
  else
    DAMD_LAUNCH(bn_finalize_kernel<float>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, rpb, pilot, x_dtype == 1, momentum, eps,
                       static_cast<const float*>(w), static_cast<const float*>(b), run_mean, run_var, mean, invstd, scale, shift);
  const int TPR = C / 8;
  const int64_t V = M * C / 8;
  const dim3 ag(apply_grid(V, TPR));
#define APPLY(T, R, A) DAMD_LAUNCH((bn_apply_kernel<T, R, A>), ag, dim3(kBNThreads), 0, st, static_cast<const T*>(x), scale, shift, static_cast<const T*>(res), static_cast<T*>(y), V, TPR, nullptr)
  if (mask != nullptr && res && relu) {
    if (x_dtype == 1)
      DAMD_LAUNCH((bn_apply_kernel<bf16_t, true, true, true>), ag, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(x), scale, shift, static_cast<const bf16_t*>(res), static_cast<bf16_t*>(y), V, TPR, mask);
    else
      DAMD_LAUNCH((bn_apply_kernel<float, true, true, true>), ag, dim3(kBNThreads), 0, st, static_cast<const float*>(x), scale, shift, static_cast<const float*>(res), static_cast<float*>(y), V, TPR, mask);
  } else if (x_dtype == 1) {
    if (res) { if (relu) APPLY(bf16_t, true, true); else APPLY(bf16_t, true, false); }
    else { if (relu) APPLY(bf16_t, false, true); else APPLY(bf16_t, false, false); }
  } else {
    if (res) { if (relu) APPLY(float, true, true); else APPLY(float, true, false); }
    else { if (relu) APPLY(float, false, true); else APPLY(float, false, false); }
  }
#undef APPLY
  DAMD_CHECK_LAUNCH();
}

// BN forward statistics from producer partials only (no apply pass): mean / invstd / folded
// scale and shift + running-statistics update, for a consumer that applies the BN itself
// (conv_igemm.hip prologue mode).
void damd_bn_finalize_launch(const float* part, int nb, int C, int64_t M, const void* w, const void* b,
                             float* run_mean, float* run_var, float momentum, float eps, float* mean, float* invstd,
                             float* scale, float* shift, int w_dtype, hipStream_t st) {
  const dim3 fg((C + kFinCh - 1) / kFinCh);
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_finalize_kernel<bf16_t>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, int64_t{0}, nullptr, 1, momentum,
                       eps, static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(b), run_mean, run_var, mean, invstd,
                       scale, shift);
  else
    DAMD_LAUNCH(bn_finalize_kernel<float>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, int64_t{0}, nullptr, 1, momentum,
                       eps, static_cast<const float*>(w), static_cast<const float*>(b), run_mean, run_var, mean, invstd,
                       scale, shift);
  DAMD_CHECK_LAUNCH();
}

void damd_bn_apply_only_launch(const void* x, const void* res, void* y, int64_t M, int C, const float* scale,
                               const float* shift, int relu, int x_dtype, hipStream_t st) {
  const int TPR = C / 8;
  const int64_t V = M * C / 8;
  const dim3 ag(apply_grid(V, TPR));
#define APPLY(T, R, A) DAMD_LAUNCH((bn_apply_kernel<T, R, A>), ag, dim3(kBNThreads), 0, st, static_cast<const T*>(x), scale, shift, static_cast<const T*>(res), static_cast<T*>(y), V, TPR)
  if (x_dtype == 1) {
    if (res) { if (relu) APPLY(bf16_t, true, true); else APPLY(bf16_t, true, false); }
    else { if (relu) APPLY(bf16_t, false, true); else APPLY(bf16_t, false, false); }
  } else {
    if (res) { if (relu) APPLY(float, true, true); else APPLY(float, true, false); }
    else { if (relu) APPLY(float, false, true); else APPLY(float, false, false); }
  }
#undef APPLY
  DAMD_CHECK_LAUNCH();
}

void damd_bn_bwd_launch(const void* dy, const void* x, const void* res, int64_t M, int C, const float* mean,
                        const float* invstd, const float* scale, const float* shift, float* part, float* coef,
                        void* dgamma, void* dbeta, void* dx, void* dres, int relu, int x_dtype, int w_dtype,
                        hipStream_t st, const uint8_t* mask, const void* dy2) {
  int nb;
  const int64_t rpb = rows_per_block_for(M, C, &nb);
  const bool has_res = res != nullptr || mask != nullptr;
  const bool masked = mask != nullptr && relu;
#define RED(T, R, A) DAMD_LAUNCH((bn_bwd_reduce_kernel<T, R, A>), dim3(nb), dim3(kBNThreads), 0, st, static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(res), mean, scale, shift, M, C, rpb, part, nullptr)
  // a second gradient (dy2) is only taken on the masked residual path (ResNet block outputs)
#define REDM(T, D2) DAMD_LAUNCH((bn_bwd_reduce_kernel<T, true, true, true, D2>), dim3(nb), dim3(kBNThreads), 0, st, static_cast<const T*>(dy), static_cast<const T*>(x), nullptr, mean, scale, shift, M, C, rpb, part, mask, static_cast<const T*>(dy2))
  if (masked) {
    if (x_dtype == 1) { if (dy2) REDM(bf16_t, true); else REDM(bf16_t, false); }
    else { if (dy2) REDM(float, true); else REDM(float, false); }
  } else if (x_dtype == 1) {
    if (has_res) { if (relu) RED(bf16_t, true, true); else RED(bf16_t, true, false); }
    else { if (relu) RED(bf16_t, false, true); else RED(bf16_t, false, false); }
  } else {
    if (has_res) { if (relu) RED(float, true, true); else RED(float, true, false); }
    else { if (relu) RED(float, false, true); else RED(float, false, false); }
  }
#undef RED
#undef REDM
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_bwd_finalize_kernel<bf16_t>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta), coef);
  else
    DAMD_LAUNCH(bn_bwd_finalize_kernel<float>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<float*>(dgamma), static_cast<float*>(dbeta), coef);
  if (dx == nullptr) {  // coefficients only: the apply pass is deferred to the consumer (bn_bwd_coef)
    DAMD_CHECK_LAUNCH();
    return;
  }
  const int TPR = C / 8;
  const int64_t V = M * C / 8;
  const dim3 ag(apply_grid(V, TPR));
  const bool wd = dres != nullptr;
#define BAP(T, R, A, W) DAMD_LAUNCH((bn_bwd_apply_kernel<T, R, A, W>), ag, dim3(kBNThreads), 0, st, static_cast<const T*>(dy), static_cast<const T*>(x), static_cast<const T*>(res), scale, shift, coef, C, static_cast<T*>(dx), static_cast<T*>(dres), V, TPR, nullptr)
#define BAPM(T, W, D2) DAMD_LAUNCH((bn_bwd_apply_kernel<T, true, true, W, true, D2>), ag, dim3(kBNThreads), 0, st, static_cast<const T*>(dy), static_cast<const T*>(x), nullptr, scale, shift, coef, C, static_cast<T*>(dx), static_cast<T*>(dres), V, TPR, mask, static_cast<const T*>(dy2))
  if (masked) {
    if (x_dtype == 1) {
      if (dy2) { if (wd) BAPM(bf16_t, true, true); else BAPM(bf16_t, false, true); }
      else { if (wd) BAPM(bf16_t, true, false); else BAPM(bf16_t, false, false); }
    } else {
      if (dy2) { if (wd) BAPM(float, true, true); else BAPM(float, false, true); }
      else { if (wd) BAPM(float, true, false); else BAPM(float, false, false); }
    }
  } else if (x_dtype == 1) {
    if (has_res) { if (relu) { if (wd) BAP(bf16_t, true, true, true); else BAP(bf16_t, true, true, false); }
                   else { if (wd) BAP(bf16_t, true, false, true); else BAP(bf16_t, true, false, false); } }
    else { if (relu) { if (wd) BAP(bf16_t, false, true, true); else BAP(bf16_t, false, true, false); }
           else { if (wd) BAP(bf16_t, false, false, true); else BAP(bf16_t, false, false, false); } }
  } else {
    if (has_res) { if (relu) { if (wd) BAP(float, true, true, true); else BAP(float, true, true, false); }
                   else { if (wd) BAP(float, true, false, true); else BAP(float, true, false, false); } }
    else { if (relu) { if (wd) BAP(float, false, true, true); else BAP(float, false, true, false); }
           else { if (wd) BAP(float, false, false, true); else BAP(float, false, false, false); } }
  }
#undef BAP
#undef BAPM
  DAMD_CHECK_LAUNCH();
}

// BN backward when the reduce partials (sum dz, sum dz*(x - mean)) already came out of the
// producer of dz (the conv input-gradient epilogue, conv_igemm.hip kEpiBnb*): dz is the gradient
// at the BN output with any ReLU mask applied, so only the finalize and one apply pass remain.
void damd_bn_bwd_finalize_launch(const float* part, int nb, int C, int64_t M, const float* mean, const float* invstd,
                                 const float* scale, float* coef, void* dgamma, void* dbeta, int w_dtype, hipStream_t st) {
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_bwd_finalize_kernel<bf16_t>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta), coef);
  else
    DAMD_LAUNCH(bn_bwd_finalize_kernel<float>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<float*>(dgamma), static_cast<float*>(dbeta), coef);
  DAMD_CHECK_LAUNCH();
}

void damd_bn_bwd_apply_coef_launch(const void* dz, const void* x, int64_t M, int C, const float* coef, void* dx,
                                   int x_dtype, hipStream_t st) {
  const int TPR = C / 8;
  const int64_t V = M * C / 8;
  const dim3 ag(apply_grid(V, TPR));
  if (x_dtype == 1)
    DAMD_LAUNCH((bn_bwd_apply_kernel<bf16_t, false, false, false>), ag, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(dz),
                       static_cast<const bf16_t*>(x), nullptr, nullptr, nullptr, coef, C, static_cast<bf16_t*>(dx), nullptr, V, TPR);
  else
    DAMD_LAUNCH((bn_bwd_apply_kernel<float, false, false, false>), ag, dim3(kBNThreads), 0, st, static_cast<const float*>(dz),
                       static_cast<const float*>(x), nullptr, nullptr, nullptr, coef, C, static_cast<float*>(dx), nullptr, V, TPR);
  DAMD_CHECK_LAUNCH();
}

void damd_bn_bwd_from_part_launch(const void* dz, const void* x, int64_t M, int C, const float* mean,
                                  const float* invstd, const float* scale, const float* part, int nb, float* coef,
                                  void* dgamma, void* dbeta, void* dx, int x_dtype, int w_dtype, hipStream_t st) {
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_bwd_finalize_kernel<bf16_t>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta), coef);
  else
    DAMD_LAUNCH(bn_bwd_finalize_kernel<float>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<float*>(dgamma), static_cast<float*>(dbeta), coef);
  const int TPR = C / 8;
  const int64_t V = M * C / 8;
  const dim3 ag(apply_grid(V, TPR));
  if (x_dtype == 1)
    DAMD_LAUNCH((bn_bwd_apply_kernel<bf16_t, false, false, false>), ag, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(dz),
                       static_cast<const bf16_t*>(x), nullptr, nullptr, nullptr, coef, C, static_cast<bf16_t*>(dx), nullptr, V, TPR);
  else
    DAMD_LAUNCH((bn_bwd_apply_kernel<float, false, false, false>), ag, dim3(kBNThreads), 0, st, static_cast<const float*>(dz),
                       static_cast<const float*>(x), nullptr, nullptr, nullptr, coef, C, static_cast<float*>(dx), nullptr, V, TPR);
  DAMD_CHECK_LAUNCH();
}

// ----------------------------------------------------------------------------- global avg-pool bwd
// dx[n, h, w, c] = g[n, c] * scale over a channels-last [N, H, W, C] output (the backward of
// x.mean((2, 3))): one vectorised write pass instead of expand + strided copy.
template <typename T>
__global__ void __launch_bounds__(kBNThreads)
hw_broadcast_kernel(const T* __restrict__ g, T* __restrict__ out, int64_t V, int TPR, int64_t HW, float scale) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kBNThreads;
  for (int64_t v = static_cast<int64_t>(blockIdx.x) * kBNThreads + threadIdx.x; v < V; v += stride) {
    const int64_t pix = v / TPR;
    const int cg = static_cast<int>(v - pix * TPR);
    const int64_t n = pix / HW;
    float d[8];
    V8<T>::ld(g + (n * TPR + cg) * 8, d);
#pragma unroll
    for (int k = 0; k < 8; ++k) d[k] *= scale;
    V8<T>::st(out + v * 8, d);
  }
}

void damd_hw_broadcast_launch(const void* g, void* out, int64_t N, int64_t HW, int C, float scale, int dtype,
                              hipStream_t st) {
  const int TPR = C / 8;
  const int64_t V = N * HW * TPR;
  const int64_t want = (V + kBNThreads - 1) / kBNThreads;
  const dim3 grid(static_cast<unsigned>(want < 8192 ? want : 8192));
  if (dtype == 1)
    DAMD_LAUNCH(hw_broadcast_kernel<bf16_t>, grid, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(g),
                       static_cast<bf16_t*>(out), V, TPR, HW, scale);
  else
    DAMD_LAUNCH(hw_broadcast_kernel<float>, grid, dim3(kBNThreads), 0, st, static_cast<const float*>(g),
                       static_cast<float*>(out), V, TPR, HW, scale);
  DAMD_CHECK_LAUNCH();
}

// ----------------------------------------------------------------------------- stem launchers
// x: [N, H, W, C] (NHWC); y / idx: [N, OH, OW, C]; 3x3 / stride 2 / pad 1 pooling.
void damd_bn_pool_fwd_launch(const void* x, void* y, uint8_t* idx, int64_t N, int H, int W, int C, int OH, int OW,
                             const void* w, const void* b, float* run_mean, float* run_var, float momentum, float eps,
                             float* part, float* mean, float* invstd, float* scale, float* shift, int x_dtype,
                             int w_dtype, hipStream_t st, const float* pre_part, int pre_nb, void* xarg) {
  const int64_t M = N * H * W;
  int nb;
  int64_t rpb = rows_per_block_for(M, C, &nb);
  const void* pilot = x;
  if (pre_part != nullptr) {  // plain (sum, sum sq) partials from the producing kernel
    part = const_cast<float*>(pre_part);
    nb = pre_nb;
    pilot = nullptr;
  } else if (x_dtype == 1) {
    DAMD_LAUNCH(bn_stats_kernel<bf16_t>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(x), M, C, rpb, part);
  } else {
    DAMD_LAUNCH(bn_stats_kernel<float>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const float*>(x), M, C, rpb, part);
  }
  const dim3 fg((C + kFinCh - 1) / kFinCh);
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_finalize_kernel<bf16_t>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, rpb, pilot, x_dtype == 1, momentum, eps,
                       static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(b), run_mean, run_var, mean, invstd, scale, shift);
  else
    DAMD_LAUNCH(bn_finalize_kernel<float>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, rpb, pilot, x_dtype == 1, momentum, eps,
                       static_cast<const float*>(w), static_cast<const float*>(b), run_mean, run_var, mean, invstd, scale, shift);
  const int TPR = C / 8;
  const int64_t Vout = N * OH * OW * TPR;
  const PoolGeo g{H, W, OH, OW};
  const dim3 ag(apply_grid(Vout, TPR));
  if (x_dtype == 1)
    DAMD_LAUNCH(bn_relu_maxpool_fwd_kernel<bf16_t>, ag, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(x), scale, shift,
                       static_cast<bf16_t*>(y), idx, Vout, TPR, g, static_cast<bf16_t*>(xarg));
  else
    DAMD_LAUNCH(bn_relu_maxpool_fwd_kernel<float>, ag, dim3(kBNThreads), 0, st, static_cast<const float*>(x), scale, shift,
                       static_cast<float*>(y), idx, Vout, TPR, g, static_cast<float*>(xarg));
  DAMD_CHECK_LAUNCH();
}

// Fused ResNet stem (conv_stem.hip stem_pool_*): the BN statistics come from the conv kernel
// (part [nb][2][C], count M = conv output pixels); the apply runs on the pooled window values
// xarg ([Q][C], Q = pooled pixels): y = relu(xarg * scale + shift), exactly the pooled output.
void damd_stem_pool_bn_fwd_launch(const float* part, int nb, int64_t M, const void* xarg, void* y, int64_t Q, int C,
                                  const void* w, const void* b, float* run_mean, float* run_var, float momentum,
                                  float eps, float* mean, float* invstd, float* scale, float* shift, int w_dtype,
                                  hipStream_t st) {
  const dim3 fg((C + kFinCh - 1) / kFinCh);
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_finalize_kernel<bf16_t>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, int64_t{0}, nullptr, 1,
                       momentum, eps, static_cast<const bf16_t*>(w), static_cast<const bf16_t*>(b), run_mean, run_var,
                       mean, invstd, scale, shift);
  else
    DAMD_LAUNCH(bn_finalize_kernel<float>, fg, dim3(kFinThreads), 0, st, part, nb, C, M, int64_t{0}, nullptr, 1,
                       momentum, eps, static_cast<const float*>(w), static_cast<const float*>(b), run_mean, run_var,
                       mean, invstd, scale, shift);
  const int TPR = C / 8;
  const int64_t V = Q * TPR;
  DAMD_LAUNCH((bn_apply_kernel<bf16_t, false, true>), dim3(apply_grid(V, TPR)), dim3(kBNThreads), 0, st,
                     static_cast<const bf16_t*>(xarg), scale, shift, nullptr, static_cast<bf16_t*>(y), V, TPR, nullptr);
  DAMD_CHECK_LAUNCH();
}

// Its backward statistics: the pooled-domain reduce over (dp [+ dp2], xarg), which also writes
// the masked pooled gradient dz for the fused weight-gradient kernel; then A, B, Cc (count M).
// part: [damd_bn_num_blocks(Q, C)][2][C].
void damd_stem_pool_bn_bwd_launch(const void* dp, const void* dp2, const void* xarg, const float* mean,
                                  const float* invstd, const float* scale, const float* shift, float* part,
                                  float* coef, void* dgamma, void* dbeta, void* dz, int64_t Q, int64_t M, int C,
                                  int w_dtype, hipStream_t st) {
  int nb;
  const int64_t rpb = rows_per_block_for(Q, C, &nb);
  DAMD_LAUNCH(pooled_bn_bwd_reduce_kernel<bf16_t>, dim3(nb), dim3(kBNThreads), 0, st,
                     static_cast<const bf16_t*>(dp), static_cast<const bf16_t*>(dp2), static_cast<const bf16_t*>(xarg),
                     mean, scale, shift, Q, C, rpb, part, static_cast<bf16_t*>(dz));
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_bwd_finalize_kernel<bf16_t>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part,
                       nb, C, M, mean, invstd, scale, static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta), coef);
  else
    DAMD_LAUNCH(bn_bwd_finalize_kernel<float>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part,
                       nb, C, M, mean, invstd, scale, static_cast<float*>(dgamma), static_cast<float*>(dbeta), coef);
  DAMD_CHECK_LAUNCH();
}

void damd_bn_pool_bwd_launch(const void* dp, const uint8_t* idx, const void* x, int64_t N, int H, int W, int C, int OH,
                             int OW, const float* mean, const float* invstd, const float* scale, const float* shift,
                             float* part, float* coef, void* dgamma, void* dbeta, void* dx, int x_dtype, int w_dtype,
                             hipStream_t st, const void* dp2, const void* xarg) {
  const int64_t M = N * H * W;      // BN statistics count
  const int64_t Q = N * OH * OW;    // quads (rows of the fused backward kernels)
  int nb;
  const int64_t rpb = rows_per_block_for(Q, C, &nb);
  const PoolGeo g{H, W, OH, OW};
  if (xarg != nullptr) {  // pooled-domain reduce (argmax input values saved by the forward)
    if (x_dtype == 1)
      DAMD_LAUNCH(pooled_bn_bwd_reduce_kernel<bf16_t>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(dp),
                         static_cast<const bf16_t*>(dp2), static_cast<const bf16_t*>(xarg), mean, scale, shift, Q, C, rpb, part);
    else
      DAMD_LAUNCH(pooled_bn_bwd_reduce_kernel<float>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const float*>(dp),
                         static_cast<const float*>(dp2), static_cast<const float*>(xarg), mean, scale, shift, Q, C, rpb, part);
  } else if (x_dtype == 1)
    DAMD_LAUNCH(maxpool_bn_bwd_reduce_kernel<bf16_t>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(dp), static_cast<const bf16_t*>(dp2), idx,
                       static_cast<const bf16_t*>(x), mean, scale, shift, Q, C, rpb, part, g);
  else
    DAMD_LAUNCH(maxpool_bn_bwd_reduce_kernel<float>, dim3(nb), dim3(kBNThreads), 0, st, static_cast<const float*>(dp), static_cast<const float*>(dp2), idx,
                       static_cast<const float*>(x), mean, scale, shift, Q, C, rpb, part, g);
  if (w_dtype == 1)
    DAMD_LAUNCH(bn_bwd_finalize_kernel<bf16_t>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta), coef);
  else
    DAMD_LAUNCH(bn_bwd_finalize_kernel<float>, dim3((C + kFinCh - 1) / kFinCh), dim3(kFinThreads), 0, st, part, nb, C, M, mean,
                       invstd, scale, static_cast<float*>(dgamma), static_cast<float*>(dbeta), coef);
  const int TPR = C / 8;
  const int64_t VQ = Q * TPR;
  const dim3 ag(apply_grid(VQ, TPR));
  if (x_dtype == 1)
    DAMD_LAUNCH(maxpool_bn_bwd_apply_kernel<bf16_t>, ag, dim3(kBNThreads), 0, st, static_cast<const bf16_t*>(dp), static_cast<const bf16_t*>(dp2), idx,
                       static_cast<const bf16_t*>(x), scale, shift, coef, C, static_cast<bf16_t*>(dx), VQ, TPR, g);
  else
    DAMD_LAUNCH(maxpool_bn_bwd_apply_kernel<float>, ag, dim3(kBNThreads), 0, st, static_cast<const float*>(dp), static_cast<const float*>(dp2), idx,
                       static_cast<const float*>(x), scale, shift, coef, C, static_cast<float*>(dx), VQ, TPR, g);
  DAMD_CHECK_LAUNCH();
}
