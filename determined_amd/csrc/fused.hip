// Fused language-model head loss and elementwise helpers for gfx950.
//
// lm_ce: next-token cross-entropy straight from the bf16 LM-head GEMM output
//   logits [B*T, Vp] (Vp = vocabulary padded for the GEMM, V = valid vocabulary),
//   labels [B*T] (int64; the label of row (b, t) is labels[b, t+1], the last position of
//   each sequence and label == ignore_index contribute nothing).
//   forward: one workgroup per row, ONE pass over the row with an online (max, sum) per
//            thread (16-byte loads), block merge -> row loss and log-sum-exp;
//   backward: dlogits = (softmax - onehot) * (dloss / n_valid), written as bf16, optionally
//            in place over the logits (they are dead after the loss), padded columns -> 0.
//   Replaces: slice + reshape + bf16->fp32 copy + softmax fwd + softmax bwd + fills.
//
// bias_grad: column sums of a [M, N] bf16 gradient (the bias gradient of a Linear) with
//   16-byte loads into row-split fp32 partials; the wide finalize of norm.hip finishes them.
//
// gelu (tanh approximation) after a Linear (GPT-2 MLP): forward g = gelu(h) as one vectorised
//   pass; backward dh = gelu'(h) * dg FUSED with the bias gradient of that Linear -- the
//   column partials of dh are accumulated while dh is written, so dh is never re-read for
//   the bias (replaces torch's GeluBackward + a separate column-sum pass).

#include "common.h"

#include <math.h>

namespace damd {
namespace fused {

constexpr int kCEThreads = 256;

__device__ __forceinline__ void online_merge(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == -INFINITY) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

__global__ void __launch_bounds__(kCEThreads)
lm_ce_fwd_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels, int T, int V, int Vp,
                 int64_t ignore_index, float* __restrict__ row_loss, float* __restrict__ lse_out) {
  const int64_t row = blockIdx.x;
  const int t = static_cast<int>(row % T);
  const bf16_t* x = logits + row * Vp;
  int64_t lab = t + 1 < T ? labels[row + 1] : ignore_index;
  if (lab == ignore_index || lab < 0 || lab >= V) lab = -1;
  float m = -INFINITY, s = 0.f;
  const int nvec = V / 8;
  for (int i = threadIdx.x; i < nvec; i += kCEThreads) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    float f[8];
    float mx = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = bf2f(v.v[j]);
      mx = fmaxf(mx, f[j]);
    }
    float ls = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) ls += __expf(f[j] - mx);
    online_merge(m, s, mx, ls);
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += kCEThreads) online_merge(m, s, bf2f(x[i]), 1.f);
  // wave merge
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o, 64), s2 = __shfl_xor(s, o, 64);
    online_merge(m, s, m2, s2);
  }
  __shared__ float sm[kCEThreads / 64], ss[kCEThreads / 64];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int k = 1; k < kCEThreads / 64; ++k) online_merge(M, S, sm[k], ss[k]);
    const float lse = M + logf(S);
    lse_out[row] = lse;
    row_loss[row] = lab >= 0 ? lse - bf2f(x[lab]) : 0.f;
  }
}

__global__ void __launch_bounds__(kCEThreads)
lm_ce_bwd_kernel(const bf16_t* __restrict__ logits, const int64_t* __restrict__ labels, const float* __restrict__ lse,
                 const float* __restrict__ scale_ptr, int T, int V, int Vp, int64_t ignore_index,
                 bf16_t* __restrict__ dlogits) {
  const int64_t row = blockIdx.x;
  const int t = static_cast<int>(row % T);
  int64_t lab = t + 1 < T ? labels[row + 1] : ignore_index;
  const bool valid = !(lab == ignore_index || lab < 0 || lab >= V);
  const bf16_t* x = logits + row * Vp;
  bf16_t* dx = dlogits + row * Vp;
  const float scale = valid ? *scale_ptr : 0.f;
  const float L = lse[row];
  const int nvec = Vp / 8;
  for (int i = threadIdx.x; i < nvec; i += kCEThreads) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(x + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = i * 8 + j;
      float g = 0.f;
      if (col < V && scale != 0.f) {
        g = __expf(bf2f(v.v[j]) - L);
        if (col == lab) g -= 1.f;
        g *= scale;
      }
      o.v[j] = f2bf(g);
    }
    *reinterpret_cast<bf16x8*>(dx + i * 8) = o;
  }
  for (int col = nvec * 8 + threadIdx.x; col < Vp; col += kCEThreads) {
    float g = 0.f;
    if (col < V && scale != 0.f) {
      g = __expf(bf2f(x[col]) - L);
      if (col == lab) g -= 1.f;
      g *= scale;
    }
    dx[col] = f2bf(g);
  }
}

// ---- bias gradient: out[n] = sum_m g[m, n] -----------------------------------------------
// Workgroup = 16 column lanes (8 columns each, one 16-byte load) x 16 row lanes; each
// workgroup sums a [rows_per_split, 128] slab; the finalize pass adds <= 32 partials/column.
constexpr int kBGCols = 128;
constexpr int kBGRowLanes = 16;

__global__ void __launch_bounds__(256)
bias_grad_partial_kernel(const bf16_t* __restrict__ g, int64_t M, int N, int64_t rows_per_split,
                         float* __restrict__ part) {
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * kBGCols + cl * 8;
  const int64_t r0 = blockIdx.y * rows_per_split;
  const int64_t r1 = min(M, r0 + rows_per_split);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    for (int64_t r = r0 + rl; r < r1; r += kBGRowLanes) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(g + r * N + col);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v.v[j]);
    }
  }
  __shared__ float red[kBGRowLanes][kBGCols + 4];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cl * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < kBGCols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kBGRowLanes; ++k) s += red[k][threadIdx.x];
    const int gc = blockIdx.x * kBGCols + threadIdx.x;
    if (gc < N) part[static_cast<int64_t>(blockIdx.y) * N + gc] = s;
  }
}

constexpr float kGeluC = 0.7978845608028654f;  // sqrt(2 / pi)
constexpr float kGeluA = 0.044715f;

__device__ __forceinline__ float tanh_fast(float u) {
  // 1 - 2 / (exp(2u) + 1): exact limits at +-inf, fp32 accuracy well below bf16 rounding
  return 1.f - 2.f / (__expf(2.f * u) + 1.f);
}

__global__ void __launch_bounds__(256)
gelu_fwd_kernel(const bf16_t* __restrict__ h, bf16_t* __restrict__ g, int64_t nvec) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * 256;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < nvec; i += stride) {
    const bf16x8 v = *reinterpret_cast<const bf16x8*>(h + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float x = bf2f(v.v[j]);
      const float t = tanh_fast(kGeluC * (x + kGeluA * x * x * x));
      o.v[j] = f2bf(0.5f * x * (1.f + t));
    }
    *reinterpret_cast<bf16x8*>(g + i * 8) = o;
  }
}

// dh = gelu'(h) * dg (bf16 out) + fp32 column partials of dh: part[blockIdx.y][N]
__global__ void __launch_bounds__(256)
gelu_bwd_bias_kernel(const bf16_t* __restrict__ dg, const bf16_t* __restrict__ h, bf16_t* __restrict__ dh, int64_t M,
                     int N, int64_t rows_per_split, float* __restrict__ part) {
  const int cl = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * kBGCols + cl * 8;
  const int64_t r0 = blockIdx.y * rows_per_split;
  const int64_t r1 = min(M, r0 + rows_per_split);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (col < N) {
    for (int64_t r = r0 + rl; r < r1; r += kBGRowLanes) {
      const int64_t off = r * N + col;
      const bf16x8 d = *reinterpret_cast<const bf16x8*>(dg + off);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(h + off);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = bf2f(v.v[j]);
        const float t = tanh_fast(kGeluC * (x + kGeluA * x * x * x));
        const float dgelu = 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * kGeluC * (1.f + 3.f * kGeluA * x * x);
        o.v[j] = f2bf(dgelu * bf2f(d.v[j]));
        acc[j] += bf2f(o.v[j]);  // the bias gradient sums the bf16 dh the weight GEMMs see
      }
      *reinterpret_cast<bf16x8*>(dh + off) = o;
    }
  }
  __shared__ float red[kBGRowLanes][kBGCols + 4];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[rl][cl * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < kBGCols) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < kBGRowLanes; ++k) s += red[k][threadIdx.x];
    const int gc = blockIdx.x * kBGCols + threadIdx.x;
    if (gc < N) part[static_cast<int64_t>(blockIdx.y) * N + gc] = s;
  }
}

}  // namespace fused
}  // namespace damd

using namespace damd;
using namespace damd::fused;

// Occupancy probe: `nblk` workgroups of 256 threads that hold their CU slots for `usec`
// microseconds (wall clock), the footprint of a collective's kernel (one workgroup per channel)
// running next to the compute stream.  Used to measure how much the persistent conv kernels lose
// when a side-stream kernel takes CUs (scripts/dev/interference.py); not on any training path.
__global__ void __launch_bounds__(256) occupy_kernel(int64_t ticks, int* sink) {
  const int64_t t0 = wall_clock64();
  int spins = 0;
  while (wall_clock64() - t0 < ticks) {
    __builtin_amdgcn_s_sleep(8);
    ++spins;
  }
  if (spins < 0) sink[threadIdx.x] = spins;  // keeps the loop; never taken
}

extern "C" {

void damd_occupy_launch(int nblk, double usec, int* sink, hipStream_t st) {
  // wall_clock64 runs at 100 MHz on gfx950
  DAMD_LAUNCH(occupy_kernel, dim3(nblk), dim3(256), 0, st, static_cast<int64_t>(usec * 100.0), sink);
}

void damd_lm_ce_fwd_launch(const void* logits, const int64_t* labels, int64_t rows, int T, int V, int Vp,
                           int64_t ignore_index, float* row_loss, float* lse, hipStream_t st) {
  if (rows <= 0) return;
  DAMD_LAUNCH(lm_ce_fwd_kernel, dim3(static_cast<unsigned>(rows)), dim3(kCEThreads), 0, st,
                     static_cast<const bf16_t*>(logits), labels, T, V, Vp, ignore_index, row_loss, lse);
  DAMD_CHECK_LAUNCH();
}

void damd_lm_ce_bwd_launch(const void* logits, const int64_t* labels, const float* lse, const float* scale,
                           int64_t rows, int T, int V, int Vp, int64_t ignore_index, void* dlogits, hipStream_t st) {
  if (rows <= 0) return;
  DAMD_LAUNCH(lm_ce_bwd_kernel, dim3(static_cast<unsigned>(rows)), dim3(kCEThreads), 0, st,
                     static_cast<const bf16_t*>(logits), labels, lse, scale, T, V, Vp, ignore_index,
                     static_cast<bf16_t*>(dlogits));
  DAMD_CHECK_LAUNCH();
}

int damd_bias_grad_splits(int64_t M, int N) {
  const int col_blocks = (N + kBGCols - 1) / kBGCols;
  int splits = static_cast<int>((1024 + col_blocks - 1) / col_blocks);  // ~1024 workgroups
  if (splits > 32) splits = 32;                                         // finalize adds <= 32
  const int64_t max_splits = (M + 127) / 128;                           // >= 128 rows per split
  if (splits > max_splits) splits = static_cast<int>(max_splits);
  return splits < 1 ? 1 : splits;
}

// Partial column sums [splits, N] (fp32); the host finishes with the wide column-sum pass
// of norm.hip (damd_norm_wgrad_finalize_launch), which writes the output dtype directly.
// (A single-launch "last block reduces" variant was measured 4-5x slower on MI355X: the
// agent-scope __threadfence each block needs before taking its ticket writes back the XCD's
// L2, so every block pays an L2 flush; the second ~5 us launch is far cheaper.)
void damd_bias_grad_launch(const void* g, int64_t M, int N, int splits, float* part, void* /*out*/,
                           int /*out_dtype*/, hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int64_t rps = (M + splits - 1) / splits;
  dim3 grid((N + kBGCols - 1) / kBGCols, splits);
  DAMD_LAUNCH(bias_grad_partial_kernel, grid, dim3(256), 0, st, static_cast<const bf16_t*>(g), M, N, rps, part);
  DAMD_CHECK_LAUNCH();
}

void damd_gelu_fwd_launch(const void* h, void* g, int64_t n, hipStream_t st) {
  const int64_t nvec = n / 8;
  if (nvec <= 0) return;
  const int64_t want = (nvec + 255) / 256;
  DAMD_LAUNCH(gelu_fwd_kernel, dim3(static_cast<unsigned>(want < 8192 ? want : 8192)), dim3(256), 0, st,
                     static_cast<const bf16_t*>(h), static_cast<bf16_t*>(g), nvec);
  DAMD_CHECK_LAUNCH();
}

// dh and bias-gradient partials [splits, N] (splits from damd_bias_grad_splits)
void damd_gelu_bwd_bias_launch(const void* dg, const void* h, void* dh, int64_t M, int N, int splits, float* part,
                               hipStream_t st) {
  if (M <= 0 || N <= 0) return;
  const int64_t rps = (M + splits - 1) / splits;
  dim3 grid((N + kBGCols - 1) / kBGCols, splits);
  DAMD_LAUNCH(gelu_bwd_bias_kernel, grid, dim3(256), 0, st, static_cast<const bf16_t*>(dg),
                     static_cast<const bf16_t*>(h), static_cast<bf16_t*>(dh), M, N, rps, part);
  DAMD_CHECK_LAUNCH();
}

}  // extern "C"

// ---- launch-check probe (tests/test_launch_check_gpu.py): fills `out` with 1.0 through a dynamic-LDS
// round trip; mode 0 = a valid launch, 1 = dynamic LDS far over the 160 KiB per-workgroup limit,
// 2 = a 2048-thread block (over the 1024-thread limit).  The invalid modes must raise, not return.
namespace damd {
__global__ void debug_fill_kernel(float* __restrict__ out, int n) {
  extern __shared__ float dbg_lds[];
  dbg_lds[threadIdx.x] = 1.f;
  __syncthreads();
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = dbg_lds[threadIdx.x];
}
}  // namespace damd

extern "C" void damd_debug_launch(float* out, int n, int mode, hipStream_t st) {
  using namespace damd;
  const int threads = mode == 2 ? 2048 : 256;
  const size_t lds = mode == 1 ? (size_t{1} << 20) : threads * sizeof(float);
  DAMD_LAUNCH(debug_fill_kernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(threads), lds, st, out, n);
}
