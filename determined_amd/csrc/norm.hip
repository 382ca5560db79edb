// LayerNorm / RMSNorm forward + backward for CDNA4 (gfx950).
//
// Layout: x is [rows, H] row-major. One 64-lane wave owns one row; lane l owns the
// 8-element (16 B for bf16) vectors l, l+64, l+128, ... so every wave-instruction moves
// a contiguous 1 KiB (bf16) / 2 KiB (fp32) span. For H <= 64*8*NV the row lives in
// registers (NV vectors per lane) and is read from HBM exactly once; the variance is a
// true two-pass over registers (no E[x^2]-E[x]^2 cancellation).
//
// Backward: dx in the same row-per-wave pass; dgamma/dbeta are accumulated in
// registers across all rows a wave visits (grid-stride) and written once per wave
// as fp32 partials, then reduced by a column kernel — no per-row atomics.
// (Reference counterpart: apex/torch fused LayerNorm used by the HF/DeepSpeed paths.)

#include "common.h"

namespace damd {

constexpr int kNormThreads = 256;  // 4 waves = 4 rows in flight per block
constexpr int kVecElems = 8;

template <typename T> struct Vec8;
template <> struct Vec8<bf16_t> {
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
template <> struct Vec8<float> {
  static __device__ __forceinline__ void ld(const float* p, float* o) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    o[0] = a.x; o[1] = a.y; o[2] = a.z; o[3] = a.w; o[4] = b.x; o[5] = b.y; o[6] = b.z; o[7] = b.w;
  }
  static __device__ __forceinline__ void st(float* p, const float* o) {
    reinterpret_cast<float4*>(p)[0] = make_float4(o[0], o[1], o[2], o[3]);
    reinterpret_cast<float4*>(p)[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
};

// ------------------------------------------------------------------ forward (register-resident)
// Residual fusion (RESID): the normalised row is s = x + dropout(branch) (the transformer's
// residual add), s is written out (it is the next residual) together with one keep-bit per
// element, and the LayerNorm runs on s from registers: one pass instead of dropout + add + LN.
struct ResidArgs {
  const void* branch;   // [rows, H]
  void* sum_out;        // [rows, H]
  uint8_t* mask;        // [rows * H / 8] keep bits
  float keep_scale;     // 1 / (1 - p)
  uint32_t seed;
  uint32_t drop_thresh; // element dropped iff hash < drop_thresh (p * 2^32); 0 = no dropout
  const int64_t* seedp; // device-side seed (graph-captured steps), or nullptr
};

__device__ __forceinline__ uint32_t drop_hash(uint32_t seed, uint64_t e) {
  uint32_t h = static_cast<uint32_t>(e) ^ (static_cast<uint32_t>(e >> 32) * 0x85EBCA6Bu) ^ (seed * 0x9E3779B9u);
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return h;
}

template <typename T, typename WT, int NV, bool RMS, bool RESID = false>
__global__ void __launch_bounds__(kNormThreads)
norm_fwd_kernel(const T* __restrict__ x, const WT* __restrict__ gamma, const WT* __restrict__ beta,
                T* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                int64_t rows, int H, float eps, ResidArgs ra = ResidArgs{}) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (kNormThreads / kWave) + threadIdx.x / kWave;
  if (row >= rows) return;
  const T* xr = x + row * H;
  float v[NV][kVecElems];
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * kWave + lane) * kVecElems;
    if (c < H) {
      Vec8<T>::ld(xr + c, v[j]);
      if (RESID) {
        float bv[kVecElems];
        Vec8<T>::ld(static_cast<const T*>(ra.branch) + row * H + c, bv);
        uint32_t bits = 0;
        const uint64_t e0 = static_cast<uint64_t>(row) * H + c;
#pragma unroll
        for (int k = 0; k < kVecElems; ++k) {
          const bool keep = ra.drop_thresh == 0u || drop_hash(ra.seedp != nullptr ? static_cast<uint32_t>(*ra.seedp) : ra.seed, e0 + k) >= ra.drop_thresh;
          bits |= (keep ? 1u : 0u) << k;
          v[j][k] += keep ? bv[k] * ra.keep_scale : 0.f;
        }
        Vec8<T>::st(static_cast<T*>(ra.sum_out) + row * H + c, v[j]);
        // normalise the value as stored (rounded to T) so forward and backward agree exactly
        if constexpr (sizeof(T) == 2) {
#pragma unroll
          for (int k = 0; k < kVecElems; ++k) v[j][k] = bf2f(f2bf(v[j][k]));
        }
        ra.mask[e0 >> 3] = static_cast<uint8_t>(bits);
      }
#pragma unroll
      for (int k = 0; k < kVecElems; ++k) s += v[j][k];
    } else {
#pragma unroll
      for (int k = 0; k < kVecElems; ++k) v[j][k] = 0.f;
    }
  }
  const float invH = 1.f / static_cast<float>(H);
  float mean = 0.f;
  if (!RMS) mean = wave_sum(s) * invH;
  float q = 0.f;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * kWave + lane) * kVecElems;
    if (c < H) {
#pragma unroll
      for (int k = 0; k < kVecElems; ++k) { const float d = v[j][k] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) * invH + eps);
  T* yr = y + row * H;
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * kWave + lane) * kVecElems;
    if (c < H) {
      float gw[kVecElems], bw[kVecElems], o[kVecElems];
      Vec8<WT>::ld(gamma + c, gw);
      if (!RMS && beta != nullptr) Vec8<WT>::ld(beta + c, bw);
#pragma unroll
      for (int k = 0; k < kVecElems; ++k) {
        o[k] = (v[j][k] - mean) * rstd * gw[k];
        if (!RMS && beta != nullptr) o[k] += bw[k];
      }
      Vec8<T>::st(yr + c, o);
    }
  }
  if (lane == 0) {
    if (!RMS && mean_out) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// ------------------------------------------------------------------ forward (generic H, 2 reads)
template <typename T, typename WT, bool RMS>
__global__ void __launch_bounds__(kNormThreads)
norm_fwd_generic_kernel(const T* __restrict__ x, const WT* __restrict__ gamma, const WT* __restrict__ beta,
                        T* __restrict__ y, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                        int64_t rows, int H, float eps) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t row = static_cast<int64_t>(blockIdx.x) * (kNormThreads / kWave) + threadIdx.x / kWave;
  if (row >= rows) return;
  const T* xr = x + row * H;
  float s = 0.f;
  for (int c = lane; c < H; c += kWave) s += Elem<T>::ld(xr, c);
  const float invH = 1.f / static_cast<float>(H);
  const float mean = RMS ? 0.f : wave_sum(s) * invH;
  float q = 0.f;
  for (int c = lane; c < H; c += kWave) { const float d = Elem<T>::ld(xr, c) - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) * invH + eps);
  T* yr = y + row * H;
  for (int c = lane; c < H; c += kWave) {
    float o = (Elem<T>::ld(xr, c) - mean) * rstd * Elem<WT>::ld(gamma, c);
    if (!RMS && beta != nullptr) o += Elem<WT>::ld(beta, c);
    Elem<T>::st(yr, c, o);
  }
  if (lane == 0) {
    if (!RMS && mean_out) mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// ------------------------------------------------------------------ backward (register-resident)
// Weight gradients: the 4 waves' column partials are reduced in LDS and each block writes one
// fp32 partial row (part_g / part_b: [gridDim.x, H]); wgrad_finalize_kernel sums the rows and
// writes dgamma / dbeta in the weight dtype.
// RESID backward: x is the saved sum s; the residual's own gradient (dres_in, from the next
// use of s) is added to the LN input-gradient, written as the residual gradient dx, and the
// branch gradient is dx * keep / (1 - p) from the saved bits.
struct ResidBwdArgs {
  const void* dres_in;  // [rows, H] (may be null: no external gradient)
  void* dbranch;        // [rows, H]
  const uint8_t* mask;
  float keep_scale;
};

template <typename T, typename WT, int NV, bool RMS, bool RESID = false>
__global__ void __launch_bounds__(kNormThreads)
norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean_in,
                const float* __restrict__ rstd_in, const WT* __restrict__ gamma, T* __restrict__ dx,
                float* __restrict__ part_g, float* __restrict__ part_b, int64_t rows, int H,
                ResidBwdArgs rb = ResidBwdArgs{}) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave_id = static_cast<int64_t>(blockIdx.x) * (kNormThreads / kWave) + threadIdx.x / kWave;
  const int64_t n_waves = static_cast<int64_t>(gridDim.x) * (kNormThreads / kWave);
  float ag[NV][kVecElems], ab[NV][kVecElems], gw[NV][kVecElems];
#pragma unroll
  for (int j = 0; j < NV; ++j) {
    const int c = (j * kWave + lane) * kVecElems;
#pragma unroll
    for (int k = 0; k < kVecElems; ++k) { ag[j][k] = 0.f; ab[j][k] = 0.f; gw[j][k] = 0.f; }
    if (c < H) Vec8<WT>::ld(gamma + c, gw[j]);
  }
  const float invH = 1.f / static_cast<float>(H);
  for (int64_t row = wave_id; row < rows; row += n_waves) {
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    float xh[NV][kVecElems], g[NV][kVecElems];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * kWave + lane) * kVecElems;
      if (c < H) {
        float xv[kVecElems];
        Vec8<T>::ld(x + row * H + c, xv);
        Vec8<T>::ld(dy + row * H + c, g[j]);
#pragma unroll
        for (int k = 0; k < kVecElems; ++k) {
          xh[j][k] = (xv[k] - mean) * rstd;
          ag[j][k] += g[j][k] * xh[j][k];
          ab[j][k] += g[j][k];
          const float wdy = g[j][k] * gw[j][k];
          s1 += wdy * xh[j][k];
          s2 += wdy;
        }
      } else {
#pragma unroll
        for (int k = 0; k < kVecElems; ++k) { xh[j][k] = 0.f; g[j][k] = 0.f; }
      }
    }
    const float c1 = wave_sum(s1) * invH;
    const float c2 = RMS ? 0.f : wave_sum(s2) * invH;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * kWave + lane) * kVecElems;
      if (c < H) {
        float o[kVecElems];
#pragma unroll
        for (int k = 0; k < kVecElems; ++k)
          o[k] = rstd * (g[j][k] * gw[j][k] - xh[j][k] * c1 - c2);
        if (RESID) {
          if (rb.dres_in != nullptr) {
            float r[kVecElems];
            Vec8<T>::ld(static_cast<const T*>(rb.dres_in) + row * H + c, r);
#pragma unroll
            for (int k = 0; k < kVecElems; ++k) o[k] += r[k];
          }
          const uint32_t bits = rb.mask[(static_cast<uint64_t>(row) * H + c) >> 3];
          float db[kVecElems];
#pragma unroll
          for (int k = 0; k < kVecElems; ++k) db[k] = (bits >> k) & 1u ? o[k] * rb.keep_scale : 0.f;
          Vec8<T>::st(static_cast<T*>(rb.dbranch) + row * H + c, db);
        }
        Vec8<T>::st(dx + row * H + c, o);
      }
    }
  }
  // block-level reduction of the 4 waves' column partials -> one partial row per block
  // (float atomics into one row from every block run ~14x below the atomic rate on MI355X,
  // so the cross-block sum is a separate wide finalize pass instead)
  constexpr int kW = kNormThreads / kWave;
  __shared__ __attribute__((aligned(16))) float red[kW][NV * kWave * kVecElems];
  const int w = threadIdx.x / kWave;
#pragma unroll
  for (int pass = 0; pass < (RMS ? 1 : 2); ++pass) {
    float* out = pass == 0 ? part_g : part_b;
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      const int c = (j * kWave + lane) * kVecElems;
      Vec8<float>::st(&red[w][c], pass == 0 ? ag[j] : ab[j]);
    }
    __syncthreads();
    if (w == 0) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        const int c = (j * kWave + lane) * kVecElems;
        if (c < H) {
          float s[kVecElems];
#pragma unroll
          for (int k = 0; k < kVecElems; ++k) s[k] = red[0][c + k] + red[1][c + k] + red[2][c + k] + red[3][c + k];
          Vec8<float>::st(out + static_cast<int64_t>(blockIdx.x) * H + c, s);
        }
      }
    }
    __syncthreads();
  }
}

template <typename T, typename WT, bool RMS>
__global__ void __launch_bounds__(kNormThreads)
norm_bwd_generic_kernel(const T* __restrict__ dy, const T* __restrict__ x, const float* __restrict__ mean_in,
                        const float* __restrict__ rstd_in, const WT* __restrict__ gamma, T* __restrict__ dx,
                        float* __restrict__ part_g, float* __restrict__ part_b, int64_t rows, int H) {
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave_id = static_cast<int64_t>(blockIdx.x) * (kNormThreads / kWave) + threadIdx.x / kWave;
  const int64_t n_waves = static_cast<int64_t>(gridDim.x) * (kNormThreads / kWave);
  for (int c = lane; c < H; c += kWave) {
    part_g[wave_id * H + c] = 0.f;
    if (!RMS) part_b[wave_id * H + c] = 0.f;
  }
  const float invH = 1.f / static_cast<float>(H);
  for (int64_t row = wave_id; row < rows; row += n_waves) {
    const float mean = RMS ? 0.f : mean_in[row];
    const float rstd = rstd_in[row];
    const T* xr = x + row * H;
    const T* dyr = dy + row * H;
    float s1 = 0.f, s2 = 0.f;
    for (int c = lane; c < H; c += kWave) {
      const float xh = (Elem<T>::ld(xr, c) - mean) * rstd;
      const float g = Elem<T>::ld(dyr, c);
      const float wdy = g * Elem<WT>::ld(gamma, c);
      s1 += wdy * xh; s2 += wdy;
      part_g[wave_id * H + c] += g * xh;
      if (!RMS) part_b[wave_id * H + c] += g;
    }
    const float c1 = wave_sum(s1) * invH;
    const float c2 = RMS ? 0.f : wave_sum(s2) * invH;
    for (int c = lane; c < H; c += kWave) {
      const float xh = (Elem<T>::ld(xr, c) - mean) * rstd;
      const float wdy = Elem<T>::ld(dyr, c) * Elem<WT>::ld(gamma, c);
      Elem<T>::st(dx + row * H, c, rstd * (wdy - xh * c1 - c2));
    }
  }
}

// Column reduction of [W, H] partials -> out[H] (fp32, pre-zeroed). grid = (ceil(H/64), S).
__global__ void __launch_bounds__(256)
col_reduce_kernel(const float* __restrict__ part, float* __restrict__ out, int W, int H) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rl = threadIdx.x >> 6;  // 0..3
  const int slice = (W + gridDim.y - 1) / gridDim.y;
  const int w0 = blockIdx.y * slice, w1 = min(W, w0 + slice);
  float acc = 0.f;
  if (col < H)
    for (int w = w0 + rl; w < w1; w += 4) acc += part[static_cast<int64_t>(w) * H + col];
  red[rl][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rl == 0 && col < H) {
    const float s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(out + col, s);
  }
}

// Column sums of [W, H] fp32 partial rows written directly in the output dtype (no atomics,
// no pre-zeroed output, no cast kernel).  Latency-bound, so it is made WIDE: grid =
// (ceil(H/32), 2: gamma | beta), 256 threads = 32 column lanes x 8 row lanes (one 128-byte
// coalesced segment per row per wave).  Also used for Linear bias gradients (part_b = null).
template <typename WT>
__global__ void __launch_bounds__(256)
wgrad_finalize_kernel(const float* __restrict__ part_g, const float* __restrict__ part_b, int W, int H,
                      WT* __restrict__ dg, WT* __restrict__ db) {
  const float* part = blockIdx.y == 0 ? part_g : part_b;
  WT* out = blockIdx.y == 0 ? dg : db;
  if (part == nullptr) return;  // no second output (uniform per block)
  const int cl = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int col = blockIdx.x * 32 + cl;
  float acc = 0.f;
  if (col < H) {
#pragma unroll 4
    for (int w = rl; w < W; w += 8) acc += part[static_cast<int64_t>(w) * H + col];
  }
  __shared__ float red[8][33];
  red[rl][cl] = acc;
  __syncthreads();
  if (threadIdx.x < 32) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += red[k][threadIdx.x];
    if (col < H) Elem<WT>::st(out, col, s);
  }
}

}  // namespace damd

using namespace damd;

namespace {
template <typename T, typename WT, bool RMS>
void fwd_dispatch(const void* x, const void* g, const void* b, void* y, float* mean, float* rstd,
                  int64_t rows, int H, float eps, hipStream_t st) {
  const dim3 grid(static_cast<unsigned>((rows + 3) / 4)), block(kNormThreads);
  const T* xp = static_cast<const T*>(x);
  const WT* gp = static_cast<const WT*>(g);
  const WT* bp = static_cast<const WT*>(b);
  T* yp = static_cast<T*>(y);
  const int nv = (H + kWave * kVecElems - 1) / (kWave * kVecElems);
  const bool vec_ok = (H % kVecElems) == 0 && nv <= 16;
#define FWD_NV(N) DAMD_LAUNCH((norm_fwd_kernel<T, WT, N, RMS>), grid, block, 0, st, xp, gp, bp, yp, mean, rstd, rows, H, eps)
  if (vec_ok) {
    switch (nv) {
      case 1: FWD_NV(1); break;
      case 2: FWD_NV(2); break;
      case 3: FWD_NV(3); break;
      case 4: FWD_NV(4); break;
      case 5: case 6: FWD_NV(6); break;
      case 7: case 8: FWD_NV(8); break;
      default: FWD_NV(16); break;
    }
  } else {
    DAMD_LAUNCH((norm_fwd_generic_kernel<T, WT, RMS>), grid, block, 0, st, xp, gp, bp, yp, mean, rstd, rows, H, eps);
  }
#undef FWD_NV
  DAMD_CHECK_LAUNCH();
}

// returns the number of partial rows written (one per block on the register-resident path,
// one per wave on the generic path)
template <typename T, typename WT, bool RMS>
int bwd_dispatch(const void* dy, const void* x, const float* mean, const float* rstd, const void* g,
                 void* dx, float* part_g, float* part_b, int64_t rows, int H, int n_blocks,
                 hipStream_t st) {
  const dim3 grid(n_blocks), block(kNormThreads);
  const T* dyp = static_cast<const T*>(dy);
  const T* xp = static_cast<const T*>(x);
  const WT* gp = static_cast<const WT*>(g);
  T* dxp = static_cast<T*>(dx);
  const int nv = (H + kWave * kVecElems - 1) / (kWave * kVecElems);
  const bool vec_ok = (H % kVecElems) == 0 && nv <= 4;  // 5*NV*8 live fp32 regs
#define BWD_NV(N) DAMD_LAUNCH((norm_bwd_kernel<T, WT, N, RMS>), grid, block, 0, st, dyp, xp, mean, rstd, gp, dxp, part_g, part_b, rows, H)
  int W = n_blocks;
  if (vec_ok) {
    switch (nv) {
      case 1: BWD_NV(1); break;
      case 2: BWD_NV(2); break;
      default: BWD_NV(4); break;
    }
  } else {
    DAMD_LAUNCH((norm_bwd_generic_kernel<T, WT, RMS>), grid, block, 0, st, dyp, xp, mean, rstd, gp, dxp, part_g, part_b, rows, H);
    W = n_blocks * (kNormThreads / kWave);
  }
#undef BWD_NV
  DAMD_CHECK_LAUNCH();
  return W;
}
}  // namespace

// dtype codes: 0 = fp32, 1 = bf16
void damd_norm_fwd_launch(const void* x, const void* gamma, const void* beta, void* y, float* mean,
                          float* rstd, int64_t rows, int H, float eps, int rms, int x_dtype,
                          int w_dtype, hipStream_t st) {
#define FD(T, WT) do { if (rms) fwd_dispatch<T, WT, true>(x, gamma, beta, y, mean, rstd, rows, H, eps, st); \
                       else fwd_dispatch<T, WT, false>(x, gamma, beta, y, mean, rstd, rows, H, eps, st); } while (0)
  if (x_dtype == 1 && w_dtype == 1) FD(bf16_t, bf16_t);
  else if (x_dtype == 1) FD(bf16_t, float);
  else if (w_dtype == 1) FD(float, bf16_t);
  else FD(float, float);
#undef FD
}

int damd_norm_bwd_blocks(int64_t rows);

// Residual-fused LayerNorm (register-resident path only: H % 8 == 0 and H <= 64*8*16 forward,
// <= 64*8*4 backward; the host checks damd_resid_norm_supported first).
int damd_resid_norm_supported(int H) {
  const int nv = (H + kWave * kVecElems - 1) / (kWave * kVecElems);
  return (H % kVecElems) == 0 && nv <= 4;
}

void damd_resid_norm_fwd_launch(const void* x, const void* branch, const void* gamma, const void* beta, void* sum_out,
                                void* y, uint8_t* mask, float* mean, float* rstd, int64_t rows, int H, float eps,
                                float p, uint32_t seed, const int64_t* seedp, int x_dtype, int w_dtype,
                                hipStream_t st) {
  ResidArgs ra;
  ra.branch = branch;
  ra.sum_out = sum_out;
  ra.mask = mask;
  ra.keep_scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  ra.seed = seed;
  ra.seedp = seedp;
  ra.drop_thresh = p > 0.f ? static_cast<uint32_t>(static_cast<double>(p) * 4294967296.0) : 0u;
  const dim3 grid(static_cast<unsigned>((rows + 3) / 4)), block(kNormThreads);
  const int nv = (H + kWave * kVecElems - 1) / (kWave * kVecElems);
#define RF(T, WT, N) DAMD_LAUNCH((norm_fwd_kernel<T, WT, N, false, true>), grid, block, 0, st, static_cast<const T*>(x), \
    static_cast<const WT*>(gamma), static_cast<const WT*>(beta), static_cast<T*>(y), mean, rstd, rows, H, eps, ra)
#define RFN(T, WT) do { switch (nv) { case 1: RF(T, WT, 1); break; case 2: RF(T, WT, 2); break; default: RF(T, WT, 4); } } while (0)
  if (x_dtype == 1 && w_dtype == 1) RFN(bf16_t, bf16_t);
  else if (x_dtype == 1) RFN(bf16_t, float);
  else if (w_dtype == 1) RFN(float, bf16_t);
  else RFN(float, float);
#undef RFN
#undef RF
  DAMD_CHECK_LAUNCH();
}

// Returns the number of partial rows (input of damd_norm_wgrad_finalize_launch).
int damd_resid_norm_bwd_launch(const void* dy, const void* dres_in, const void* s, const float* mean, const float* rstd,
                               const void* gamma, const uint8_t* mask, float p, void* dx, void* dbranch,
                               float* part_g, float* part_b, int64_t rows, int H, int x_dtype, int w_dtype,
                               hipStream_t st) {
  ResidBwdArgs rb;
  rb.dres_in = dres_in;
  rb.dbranch = dbranch;
  rb.mask = mask;
  rb.keep_scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  const int nb = damd_norm_bwd_blocks(rows);
  const dim3 grid(nb), block(kNormThreads);
  const int nv = (H + kWave * kVecElems - 1) / (kWave * kVecElems);
#define RB(T, WT, N) DAMD_LAUNCH((norm_bwd_kernel<T, WT, N, false, true>), grid, block, 0, st, static_cast<const T*>(dy), \
    static_cast<const T*>(s), mean, rstd, static_cast<const WT*>(gamma), static_cast<T*>(dx), part_g, part_b, rows, H, rb)
#define RBN(T, WT) do { switch (nv) { case 1: RB(T, WT, 1); break; case 2: RB(T, WT, 2); break; default: RB(T, WT, 4); } } while (0)
  if (x_dtype == 1 && w_dtype == 1) RBN(bf16_t, bf16_t);
  else if (x_dtype == 1) RBN(bf16_t, float);
  else if (w_dtype == 1) RBN(float, bf16_t);
  else RBN(float, float);
#undef RBN
#undef RB
  DAMD_CHECK_LAUNCH();
  return nb;
}

// Number of blocks used by the backward grid (=> partial rows = 4 * blocks).
int damd_norm_bwd_blocks(int64_t rows) {
  int64_t b = (rows + 3) / 4;
  if (b > 512) b = 512;
  if (b < 1) b = 1;
  return static_cast<int>(b);
}

// Returns the number of partial rows written to part_g / part_b (input of
// damd_norm_wgrad_finalize_launch).
int damd_norm_bwd_launch(const void* dy, const void* x, const float* mean, const float* rstd,
                         const void* gamma, void* dx, float* part_g, float* part_b, int64_t rows,
                         int H, int rms, int x_dtype, int w_dtype, hipStream_t st) {
  const int nb = damd_norm_bwd_blocks(rows);
  int W = 0;
#define BD(T, WT) do { if (rms) W = bwd_dispatch<T, WT, true>(dy, x, mean, rstd, gamma, dx, part_g, part_b, rows, H, nb, st); \
                       else W = bwd_dispatch<T, WT, false>(dy, x, mean, rstd, gamma, dx, part_g, part_b, rows, H, nb, st); } while (0)
  if (x_dtype == 1 && w_dtype == 1) BD(bf16_t, bf16_t);
  else if (x_dtype == 1) BD(bf16_t, float);
  else if (w_dtype == 1) BD(float, bf16_t);
  else BD(float, float);
#undef BD
  return W;
}

void damd_norm_wgrad_finalize_launch(const float* part_g, const float* part_b, int W, int H, void* dgamma,
                                     void* dbeta, int w_dtype, hipStream_t st) {
  const dim3 grid((H + 31) / 32, 2);
  if (w_dtype == 1)
    DAMD_LAUNCH((wgrad_finalize_kernel<bf16_t>), grid, dim3(256), 0, st, part_g, part_b, W, H,
                       static_cast<bf16_t*>(dgamma), static_cast<bf16_t*>(dbeta));
  else
    DAMD_LAUNCH((wgrad_finalize_kernel<float>), grid, dim3(256), 0, st, part_g, part_b, W, H,
                       static_cast<float*>(dgamma), static_cast<float*>(dbeta));
  DAMD_CHECK_LAUNCH();
}

void damd_col_reduce_launch(const float* part, float* out, int W, int H, hipStream_t st) {
  int S = W / 64;
  if (S < 1) S = 1;
  if (S > 32) S = 32;
  DAMD_LAUNCH(col_reduce_kernel, dim3((H + 63) / 64, S), dim3(256), 0, st, part, out, W, H);
  DAMD_CHECK_LAUNCH();
}
