// Flash attention (forward + backward) for gfx950 / MI355X: bf16 in/out, fp32 accumulate,
// online softmax, optional causal mask, head dim D in {64, 128}.
//
// MFMA: v_mfma_f32_16x16x32_bf16 (a 64-wide wave computes a 16x16 tile, K = 32).
//   A operand: lane l holds A[row l&15][k 8(l>>4)+j], B operand: B[k 8(l>>4)+j][col l&15],
//   C/D: C[row 4(l>>4)+r][col l&15], r = 0..3.
// Transposed operands come from the SAME row-major LDS tile through ds_read_b64_tr_b16
// (gfx950 hardware transpose read: per 16-lane group, lane 4q+p addresses row q, columns
// 4p..4p+3 of a 4x16 block and lane i receives column i of the 4 rows).
//
// Forward (workgroup = 4 waves = 128 query rows, a wave = 2 x 16 rows):
//   S^T = K.Q^T puts the query on the lane (col) and 4 keys per 16-key tile in the lane's
//   registers: the online-softmax row max / sum are in-lane + 2 xor shuffles, the running
//   (m, l) and the rescale of O are lane-local, and O^T = V^T.P^T consumes P^T straight from
//   the S^T accumulators: a 32-key MFMA step uses the k order key(g, j) = (j < 4 ? 4g + j :
//   16 + 4g + j - 4), and the V^T operand is read in that order with two transposed reads.
//   K/V tiles (64 keys) are staged in LDS once per workgroup; the next tile's global loads
//   are issued into registers before the current tile's MFMAs (latency hidden).
//
// Backward (workgroup = 64 keys, a wave = 16 keys; loop over 64-row query blocks):
//   S = Q.K^T and dP = dO.V^T with the key on the lane (K, V fragments of the wave's keys stay
//   in registers), P = exp2(S.scale.log2e - LSE.log2e), dS = P.(dP - delta); P / dS feed
//   dV^T = dO^T.P and dK^T = Q^T.dS directly (dO^T, Q^T by transposed reads of the row-major
//   tiles).
// dQ (separate kernel, query-major like the forward): S^T = K.Q^T and dP^T = V.dO^T, P^T from
//   the saved LSE, dS^T = P^T.(dP^T - delta), dQ^T += K^T.dS^T, written once as bf16.  Summing
//   dQ over key blocks with float atomics instead (one 64x64 fp32 tile per key/query block
//   pair: ~285 MB of atomic adds per GPT-2-medium layer at mb 8) ran at the chip's atomic rate
//   and made the backward atomic-bound; recomputing S and dP costs two extra MFMA tiles per
//   block pair and no atomics.
//
// Strides are in elements for (batch, head, token); the head dimension must be contiguous.
//
// Key padding (BERT-style batches): an optional byte mask km[b][key] (row stride kms, rows padded to
// a multiple of 64 keys with zeros) removes keys from every query's softmax; with a mask every key
// tile takes the masked body.  Dropout on the attention probabilities: keep(b, h, q, k) is a
// counter-based hash of (seed, b*H + h, q, k) compared with a threshold, recomputed identically by
// the forward, the dK/dV and the dQ kernels (no mask tensor is stored); kept probabilities are
// scaled by 1 / (1 - p).  The row sums (l, LSE) use the undropped probabilities, so the backward's
// delta = rowsum(dO . O) and dS = P . (Z . dP / (1 - p) - delta) hold unchanged.

#include "common.h"

#include <math.h>

#include <type_traits>

namespace damd {
namespace attn {

typedef short s8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

constexpr int kBlk = 64;       // kv tile (fwd) / key block (bwd) / query block (bwd)
constexpr int kThreads = 256;  // 4 waves
constexpr int kQT = 2;         // 16-row query tiles per wave in the forward
constexpr int kFwdRows = 4 * 16 * kQT;
constexpr float kLog2e = 1.4426950408889634f;
// LDS row stride of the staged K/V/Q/dO tiles: D + 16 elements makes both the row-major
// ds_read_b128 operand reads (lane groups {0-3,12-15,20-27}, ...) and the transposed
// ds_read_b64_tr_b16 reads (2 x 32 lanes) bank-conflict-free; D + 8 was 2-way on both
// (SQ_LDS_BANK_CONFLICT ~40% of LDS cycles).
constexpr int kLdsStride(int D) { return D + 16; }
constexpr float kLn2 = 0.6931471805599453f;

struct Strides {
  int64_t b, h, t;
};

struct KeyMaskDrop {
  const uint8_t* km;   // [B][kms] key validity (nullptr: every key < T is valid)
  int64_t kms;
  uint32_t seed;       // dropout stream
  uint32_t thresh;     // drop when hash < thresh (0: no dropout)
  float inv_keep;      // 1 / (1 - p)
  const int64_t* seedp;  // device-side seed (read at run time: a graph-captured step draws a new one per replay)
};

__device__ __forceinline__ uint32_t md_seed(const KeyMaskDrop& md) {
  return md.seedp != nullptr ? static_cast<uint32_t>(*md.seedp) : md.seed;
}

struct FwdArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; bf16_t* o; float* lse;
  Strides sq, sk, sv, so;
  int H, T;
  float scale_log2;  // softmax scale * log2(e)
  KeyMaskDrop md;
};

struct BwdArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* dout;
  const float* lse; const float* delta; float* dq_acc; bf16_t* dk; bf16_t* dv;
  Strides sq, sk, sv, sdo, sdk, sdv;
  int H, T;
  float scale, scale_log2;
  KeyMaskDrop md;
};

// dropout decision for (b*H + h, query, key): murmur3-style finalizer of the mixed counters
__device__ __forceinline__ bool drop_keep(uint32_t seed, uint32_t thresh, uint32_t bh, uint32_t q, uint32_t k) {
  uint32_t x = seed ^ (bh * 0x9E3779B1u) ^ (q * 0x85EBCA77u) ^ (k * 0xC2B2AE3Du);
  x ^= x >> 16;
  x *= 0x85EBCA6Bu;
  x ^= x >> 13;
  x *= 0xC2B2AE35u;
  x ^= x >> 16;
  return x >= thresh;
}

__device__ __forceinline__ f4 mfma(s8 a, s8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}

typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef short sh2 __attribute__((ext_vector_type(2)));

// gfx950 converts fp32 -> bf16 (round to nearest even) in hardware: one v_cvt_pk_bf16_f32 per
// pair instead of the ~6-instruction software rounding (the kernels are VALU-bound, not MFMA).
__device__ __forceinline__ sh2 cvt2(float a, float b) {
  return __builtin_bit_cast(sh2, __builtin_convertvector((f2{a, b}), bf2));
}
__device__ __forceinline__ short bfs(float x) { return cvt2(x, 0.f)[0]; }
// raw v_exp_f32 (softmax arguments are <= 0 or -inf; no denormal-range fixup needed)
__device__ __forceinline__ float ex2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ s8 cat4(s4 lo, s4 hi) {
  s8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// bf16 fragment from two 16-wide accumulator tiles (the permuted 32-wide k step).
__device__ __forceinline__ s8 pack_pair(f4 lo, f4 hi) {
  const sh2 a = cvt2(lo[0], lo[1]), b = cvt2(lo[2], lo[3]), c = cvt2(hi[0], hi[1]), d = cvt2(hi[2], hi[3]);
  s8 r;
  r[0] = a[0]; r[1] = a[1]; r[2] = b[0]; r[3] = b[1];
  r[4] = c[0]; r[5] = c[1]; r[6] = d[0]; r[7] = d[1];
  return r;
}

__device__ __forceinline__ s4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p));
}

// Transposed operand (rows of the image are the k index): lane c of each 16-lane group gets
// column col0 + c of image rows {r0 + q} (elements 0..3) and {r1 + q} (elements 4..7).
__device__ __forceinline__ s8 tr_pair(const bf16_t* img, int stride, int r0, int r1, int col0, int c) {
  const int q = c >> 2, p = c & 3;
  const s4 lo = tr_read(img + (r0 + q) * stride + col0 + 4 * p);
  const s4 hi = tr_read(img + (r1 + q) * stride + col0 + 4 * p);
  return cat4(lo, hi);
}

// Register-staged tile of `ROWS` x D bf16: global -> registers (issued early), registers ->
// row-major LDS image (row stride kLdsStride(D)).  Rows >= T load zeros.
template <int D, int ROWS>
struct Stage {
  static constexpr int CH = D / 8;
  static constexpr int N = ROWS * CH / kThreads;
  s8 r[N];
  __device__ __forceinline__ void load(const bf16_t* __restrict__ base, int64_t st, int r0, int T) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = threadIdx.x + i * kThreads, row = idx / CH, col = (idx % CH) * 8;
      s8 x = {0, 0, 0, 0, 0, 0, 0, 0};
      if (r0 + row < T) x = *reinterpret_cast<const s8*>(base + static_cast<int64_t>(r0 + row) * st + col);
      r[i] = x;
    }
  }
  __device__ __forceinline__ void store(bf16_t* img) const {
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int idx = threadIdx.x + i * kThreads, row = idx / CH, col = (idx % CH) * 8;
      *reinterpret_cast<s8*>(img + row * kLdsStride(D) + col) = r[i];
    }
  }
};

// ------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------
template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads) attn_fwd_kernel(FwdArgs a) {
  constexpr int KP = kLdsStride(D);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[kBlk * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[kBlk * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int T = a.T, nkb = (T + kBlk - 1) / kBlk, nqb = (T + kFwdRows - 1) / kFwdRows;
  const int qb = CAUSAL ? (nqb - 1 - static_cast<int>(blockIdx.x)) : static_cast<int>(blockIdx.x);
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = qb * kFwdRows, qw = q0 + w * 16 * kQT;  // first query row of this wave
  const bf16_t* Qp = a.q + b * a.sq.b + h * a.sq.h;
  const bf16_t* Kp = a.k + b * a.sk.b + h * a.sk.h;
  const bf16_t* Vp = a.v + b * a.sv.b + h * a.sv.h;
  const uint8_t* KMp = a.md.km ? a.md.km + b * a.md.kms : nullptr;
  const uint32_t bh32 = static_cast<uint32_t>(b * a.H + h);

  s8 qf[kQT][D / 32];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int q = qw + qt * 16 + c;
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds) {
      s8 x = {0, 0, 0, 0, 0, 0, 0, 0};
      if (q < T) x = *reinterpret_cast<const s8*>(Qp + static_cast<int64_t>(q) * a.sq.t + ds * 32 + 8 * g);
      qf[qt][ds] = x;
    }
  }
  f4 oacc[kQT][D / 16];
  float m[kQT], l[kQT];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    m[qt] = -INFINITY;
    l[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) oacc[qt][dt] = f4{0.f, 0.f, 0.f, 0.f};
  }

  const int kb_end = CAUSAL ? min(nkb, (q0 + kFwdRows - 1) / kBlk + 1) : nkb;
  Stage<D, kBlk> ks, vs;
  ks.load(Kp, a.sk.t, 0, T);
  vs.load(Vp, a.sv.t, 0, T);
  // Leading tiles that no row of the workgroup masks (all keys < T and <= q0) run a body
  // compiled without any masking code; only the <= 2 diagonal / ragged tiles carry the selects.
  // (D = 128: a single masked body -- the unmasked copy pushes it to 256 VGPRs, 1 wave / SIMD)
  const int kb_full = D == 64 && !KMp ? min(kb_end, CAUSAL ? min((q0 + 1) / kBlk, T / kBlk) : T / kBlk) : 0;
  auto tile = [&](int kb, auto masked) {
    constexpr bool MASK = decltype(masked)::value;
    const int k0 = kb * kBlk;
    __syncthreads();
    ks.store(Ks);
    vs.store(Vs);
    __syncthreads();
    if (kb + 1 < kb_end) {  // next tile's loads fly under this tile's MFMAs
      ks.load(Kp, a.sk.t, k0 + kBlk, T);
      vs.load(Vp, a.sv.t, k0 + kBlk, T);
    }
    f4 s[kQT][4];
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) s[qt][nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int ds = 0; ds < D / 32; ++ds) {
        const s8 kf = *reinterpret_cast<const s8*>(Ks + (nt * 16 + c) * KP + ds * 32 + 8 * g);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt) s[qt][nt] = mfma(kf, qf[qt][ds], s[qt][nt]);
      }
    }
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt) {
      const int myq = qw + qt * 16 + c;
      // raw scores; the softmax scale (> 0) is folded into the exp2 argument: p = 2^(s*c - m)
      if constexpr (MASK) {
        const int kmax = CAUSAL ? min(T - 1, myq) : T - 1;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            s[qt][nt][r] = (k0 + nt * 16 + 4 * g + r > kmax) ? -INFINITY : s[qt][nt][r];
        if (KMp) {  // padded keys (row padded to a multiple of 64: the word loads stay in bounds)
#pragma unroll
          for (int nt = 0; nt < 4; ++nt) {
            const uint32_t mw = *reinterpret_cast<const uint32_t*>(KMp + k0 + nt * 16 + 4 * g);
#pragma unroll
            for (int r = 0; r < 4; ++r) s[qt][nt][r] = ((mw >> (8 * r)) & 0xffu) ? s[qt][nt][r] : -INFINITY;
          }
        }
      }
      float mx = -INFINITY;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int r = 0; r < 4; ++r) mx = fmaxf(mx, s[qt][nt][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m[qt], mx * a.scale_log2);
      const float m_use = m_new == -INFINITY ? 0.f : m_new;
      const float alpha = ex2(m[qt] - m_use);
      float rs = 0.f;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float p = ex2(fmaf(s[qt][nt][r], a.scale_log2, -m_use));
          rs += p;
          if constexpr (DROP)
            s[qt][nt][r] = drop_keep(md_seed(a.md), a.md.thresh, bh32, myq, k0 + nt * 16 + 4 * g + r) ? p : 0.f;
          else
            s[qt][nt][r] = p;
        }
      }
      l[qt] = l[qt] * alpha + rs;
      m[qt] = m_new;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) oacc[qt][dt] *= alpha;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s8 pb[kQT];
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) pb[qt] = pack_pair(s[qt][2 * s2], s[qt][2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const s8 vf = tr_pair(Vs, KP, s2 * 32 + 4 * g, s2 * 32 + 16 + 4 * g, dt * 16, c);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt) oacc[qt][dt] = mfma(vf, pb[qt], oacc[qt][dt]);
      }
    }
  };
  int kb = 0;
  for (; kb < kb_full; ++kb) tile(kb, std::false_type{});
  for (; kb < kb_end; ++kb) tile(kb, std::true_type{});
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    float lt = l[qt];
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int myq = qw + qt * 16 + c;
    if (myq < T) {
      const float inv = lt > 0.f ? (DROP ? a.md.inv_keep : 1.f) / lt : 0.f;
      bf16_t* Op = a.o + b * a.so.b + h * a.so.h + static_cast<int64_t>(myq) * a.so.t;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        s4 ov;
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = bfs(oacc[qt][dt][r] * inv);
        *reinterpret_cast<s4*>(Op + dt * 16 + 4 * g) = ov;
      }
      if (g == 0)
        a.lse[(static_cast<int64_t>(b) * a.H + h) * T + myq] = lt > 0.f ? m[qt] * kLn2 + logf(lt) : -INFINITY;
    }
  }
}

// ------------------------------------------------------------------------------------------
// backward
// ------------------------------------------------------------------------------------------
// delta[b,h,t] = sum_d dO * O  (D/8 lanes per row, one 16-byte chunk each)
template <int D>
__global__ void __launch_bounds__(256) attn_delta_kernel(const bf16_t* __restrict__ o, Strides so,
                                                         const bf16_t* __restrict__ dout, Strides sd,
                                                         float* __restrict__ delta, int H, int T, int64_t rows) {
  constexpr int L = D / 8;
  const int64_t row = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) / L;
  const int part = threadIdx.x % L;
  float acc = 0.f;
  if (row < rows) {
    const int t = static_cast<int>(row % T);
    const int64_t bh = row / T;
    const int h = static_cast<int>(bh % H), b = static_cast<int>(bh / H);
    const s8 x = *reinterpret_cast<const s8*>(o + b * so.b + h * so.h + t * so.t + part * 8);
    const s8 y = *reinterpret_cast<const s8*>(dout + b * sd.b + h * sd.h + t * sd.t + part * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += bf2f(static_cast<bf16_t>(x[j])) * bf2f(static_cast<bf16_t>(y[j]));
  }
#pragma unroll
  for (int off = L / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
  if (row < rows && part == 0) delta[row] = acc;
}

template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads) attn_bwd_kernel(BwdArgs a) {
  constexpr int RP = kLdsStride(D);
  __shared__ __attribute__((aligned(16))) bf16_t Qs[kBlk * RP];
  __shared__ __attribute__((aligned(16))) bf16_t dOs[kBlk * RP];
  __shared__ float lse2[kBlk], dl[kBlk];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int T = a.T, nblk = (T + kBlk - 1) / kBlk;
  const int kb = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int k0 = kb * kBlk;
  const bf16_t* Qp = a.q + b * a.sq.b + h * a.sq.h;
  const bf16_t* Kp = a.k + b * a.sk.b + h * a.sk.h;
  const bf16_t* Vp = a.v + b * a.sv.b + h * a.sv.h;
  const bf16_t* dOp = a.dout + b * a.sdo.b + h * a.sdo.h;
  const int64_t bh = static_cast<int64_t>(b) * a.H + h;
  const int mykey = k0 + w * 16 + c;
  const uint8_t* KMp = a.md.km ? a.md.km + b * a.md.kms : nullptr;
  const bool kvalid = mykey < T && (KMp == nullptr || KMp[mykey] != 0);

  s8 kf[D / 32], vf[D / 32];
#pragma unroll
  for (int ds = 0; ds < D / 32; ++ds) {
    s8 x = {0, 0, 0, 0, 0, 0, 0, 0}, y = x;
    if (mykey < T) {
      x = *reinterpret_cast<const s8*>(Kp + static_cast<int64_t>(mykey) * a.sk.t + ds * 32 + 8 * g);
      y = *reinterpret_cast<const s8*>(Vp + static_cast<int64_t>(mykey) * a.sv.t + ds * 32 + 8 * g);
    }
    kf[ds] = x;
    vf[ds] = y;
  }
  f4 dk[D / 16], dv[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) dk[dt] = dv[dt] = f4{0.f, 0.f, 0.f, 0.f};

  const int qb0 = CAUSAL ? kb : 0;
  Stage<D, kBlk> qst, ost;
  qst.load(Qp, a.sq.t, qb0 * kBlk, T);
  ost.load(dOp, a.sdo.t, qb0 * kBlk, T);
  for (int qb = qb0; qb < nblk; ++qb) {
    const int q0 = qb * kBlk;
    __syncthreads();
    qst.store(Qs);
    ost.store(dOs);
    if (threadIdx.x < kBlk) {
      const int q = q0 + threadIdx.x;
      lse2[threadIdx.x] = q < T ? a.lse[bh * T + q] * kLog2e : INFINITY;
      dl[threadIdx.x] = q < T ? a.delta[bh * T + q] : 0.f;
    }
    __syncthreads();
    if (qb + 1 < nblk) {
      qst.load(Qp, a.sq.t, q0 + kBlk, T);
      ost.load(dOp, a.sdo.t, q0 + kBlk, T);
    }

    const bool need_mask = (k0 + kBlk > T) || (CAUSAL && q0 < k0 + kBlk) || KMp != nullptr;
    f4 P[4], dS[4];
#pragma unroll
    for (int qt = 0; qt < 4; ++qt) {
      f4 sacc = {0.f, 0.f, 0.f, 0.f}, dpacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < D / 32; ++ds) {
        const s8 qa = *reinterpret_cast<const s8*>(Qs + (qt * 16 + c) * RP + ds * 32 + 8 * g);
        const s8 oa = *reinterpret_cast<const s8*>(dOs + (qt * 16 + c) * RP + ds * 32 + 8 * g);
        sacc = mfma(qa, kf[ds], sacc);
        dpacc = mfma(oa, vf[ds], dpacc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ql = qt * 16 + 4 * g + r;
        float p = ex2(fmaf(sacc[r], a.scale_log2, -lse2[ql]));
        if (need_mask) p = (!kvalid || (CAUSAL && mykey > q0 + ql)) ? 0.f : p;
        if constexpr (DROP) {
          const bool keep = drop_keep(md_seed(a.md), a.md.thresh, static_cast<uint32_t>(bh), q0 + ql, mykey);
          P[qt][r] = keep ? p * a.md.inv_keep : 0.f;  // dV uses the dropped, rescaled probabilities
          dS[qt][r] = p * ((keep ? dpacc[r] * a.md.inv_keep : 0.f) - dl[ql]);
        } else {
          P[qt][r] = p;
          dS[qt][r] = p * (dpacc[r] - dl[ql]);
        }
      }
    }
    // dV^T += dO^T . P ; dK^T += Q^T . dS   (k = 32 queries per step, permuted order)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const s8 pb = pack_pair(P[2 * s2], P[2 * s2 + 1]);
      const s8 sb = pack_pair(dS[2 * s2], dS[2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        dv[dt] = mfma(tr_pair(dOs, RP, s2 * 32 + 4 * g, s2 * 32 + 16 + 4 * g, dt * 16, c), pb, dv[dt]);
        dk[dt] = mfma(tr_pair(Qs, RP, s2 * 32 + 4 * g, s2 * 32 + 16 + 4 * g, dt * 16, c), sb, dk[dt]);
      }
    }
  }
  if (mykey < T) {
    bf16_t* dKp = a.dk + b * a.sdk.b + h * a.sdk.h + static_cast<int64_t>(mykey) * a.sdk.t;
    bf16_t* dVp = a.dv + b * a.sdv.b + h * a.sdv.h + static_cast<int64_t>(mykey) * a.sdv.t;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) {
      s4 kv, vv;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        kv[r] = bfs(dk[dt][r] * a.scale);
        vv[r] = bfs(dv[dt][r]);
      }
      *reinterpret_cast<s4*>(dKp + dt * 16 + 4 * g) = kv;
      *reinterpret_cast<s4*>(dVp + dt * 16 + 4 * g) = vv;
    }
  }
}

struct DqArgs {
  const bf16_t* q; const bf16_t* k; const bf16_t* v; const bf16_t* dout;
  const float* lse; const float* delta; bf16_t* dq;
  Strides sq, sk, sv, sdo, sdq;
  int H, T;
  float scale, scale_log2;
  KeyMaskDrop md;
};

// dQ for a block of kFwdRows query rows (same wave / lane layout as the forward).
template <int D, bool CAUSAL, bool DROP>
__global__ void __launch_bounds__(kThreads) attn_dq_kernel(DqArgs a) {
  constexpr int KP = kLdsStride(D);
  __shared__ __attribute__((aligned(16))) bf16_t Ks[kBlk * KP];
  __shared__ __attribute__((aligned(16))) bf16_t Vs[kBlk * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, g = lane >> 4, c = lane & 15;
  const int T = a.T, nkb = (T + kBlk - 1) / kBlk, nqb = (T + kFwdRows - 1) / kFwdRows;
  const int qb = CAUSAL ? (nqb - 1 - static_cast<int>(blockIdx.x)) : static_cast<int>(blockIdx.x);
  const int h = blockIdx.y, b = blockIdx.z;
  const int q0 = qb * kFwdRows, qw = q0 + w * 16 * kQT;
  const int64_t bh = static_cast<int64_t>(b) * a.H + h;
  const bf16_t* Qp = a.q + b * a.sq.b + h * a.sq.h;
  const bf16_t* Kp = a.k + b * a.sk.b + h * a.sk.h;
  const bf16_t* Vp = a.v + b * a.sv.b + h * a.sv.h;
  const bf16_t* dOp = a.dout + b * a.sdo.b + h * a.sdo.h;
  const uint8_t* KMp = a.md.km ? a.md.km + b * a.md.kms : nullptr;

  s8 qf[kQT][D / 32], of[kQT][D / 32];
  float lse2[kQT], dl[kQT];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int q = qw + qt * 16 + c;
#pragma unroll
    for (int ds = 0; ds < D / 32; ++ds) {
      s8 x = {0, 0, 0, 0, 0, 0, 0, 0}, y = x;
      if (q < T) {
        x = *reinterpret_cast<const s8*>(Qp + static_cast<int64_t>(q) * a.sq.t + ds * 32 + 8 * g);
        y = *reinterpret_cast<const s8*>(dOp + static_cast<int64_t>(q) * a.sdo.t + ds * 32 + 8 * g);
      }
      qf[qt][ds] = x;
      of[qt][ds] = y;
    }
    lse2[qt] = q < T ? a.lse[bh * T + q] * kLog2e : INFINITY;
    dl[qt] = q < T ? a.delta[bh * T + q] : 0.f;
  }
  f4 dq[kQT][D / 16];
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt)
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) dq[qt][dt] = f4{0.f, 0.f, 0.f, 0.f};

  const int kb_end = CAUSAL ? min(nkb, (q0 + kFwdRows - 1) / kBlk + 1) : nkb;
  Stage<D, kBlk> ks, vs;
  ks.load(Kp, a.sk.t, 0, T);
  vs.load(Vp, a.sv.t, 0, T);
  for (int kb = 0; kb < kb_end; ++kb) {
    const int k0 = kb * kBlk;
    __syncthreads();
    ks.store(Ks);
    vs.store(Vs);
    __syncthreads();
    if (kb + 1 < kb_end) {
      ks.load(Kp, a.sk.t, k0 + kBlk, T);
      vs.load(Vp, a.sv.t, k0 + kBlk, T);
    }
    // S^T = K.Q^T and dP^T = V.dO^T (key on the accumulator rows, query on the lane)
    f4 s[kQT][4], dp[kQT][4];
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt)
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) s[qt][nt] = dp[qt][nt] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
#pragma unroll
      for (int ds = 0; ds < D / 32; ++ds) {
        const s8 kf = *reinterpret_cast<const s8*>(Ks + (nt * 16 + c) * KP + ds * 32 + 8 * g);
        const s8 vf = *reinterpret_cast<const s8*>(Vs + (nt * 16 + c) * KP + ds * 32 + 8 * g);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt) {
          s[qt][nt] = mfma(kf, qf[qt][ds], s[qt][nt]);
          dp[qt][nt] = mfma(vf, of[qt][ds], dp[qt][nt]);
        }
      }
    }
    const bool need_mask = (k0 + kBlk > T) || (CAUSAL && k0 + kBlk - 1 > qw);
#pragma unroll
    for (int qt = 0; qt < kQT; ++qt) {
      const int myq = qw + qt * 16 + c;
      const int kmax = CAUSAL ? min(T - 1, myq) : T - 1;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const uint32_t mw = KMp ? *reinterpret_cast<const uint32_t*>(KMp + k0 + nt * 16 + 4 * g) : 0xffffffffu;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = k0 + nt * 16 + 4 * g + r;
          float p = ex2(fmaf(s[qt][nt][r], a.scale_log2, -lse2[qt]));
          if (need_mask) p = (key > kmax) ? 0.f : p;
          p = ((mw >> (8 * r)) & 0xffu) ? p : 0.f;
          float dpv = dp[qt][nt][r];
          if constexpr (DROP)
            dpv = drop_keep(md_seed(a.md), a.md.thresh, static_cast<uint32_t>(bh), myq, key) ? dpv * a.md.inv_keep : 0.f;
          s[qt][nt][r] = p * (dpv - dl[qt]);  // dS^T
        }
      }
    }
    // dQ^T += K^T . dS^T (32 keys per step in the permuted order of the forward's V^T.P^T)
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s8 sb[kQT];
#pragma unroll
      for (int qt = 0; qt < kQT; ++qt) sb[qt] = pack_pair(s[qt][2 * s2], s[qt][2 * s2 + 1]);
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        const s8 kt = tr_pair(Ks, KP, s2 * 32 + 4 * g, s2 * 32 + 16 + 4 * g, dt * 16, c);
#pragma unroll
        for (int qt = 0; qt < kQT; ++qt) dq[qt][dt] = mfma(kt, sb[qt], dq[qt][dt]);
      }
    }
  }
#pragma unroll
  for (int qt = 0; qt < kQT; ++qt) {
    const int myq = qw + qt * 16 + c;
    if (myq < T) {
      bf16_t* Dp = a.dq + b * a.sdq.b + h * a.sdq.h + static_cast<int64_t>(myq) * a.sdq.t;
#pragma unroll
      for (int dt = 0; dt < D / 16; ++dt) {
        s4 ov;
#pragma unroll
        for (int r = 0; r < 4; ++r) ov[r] = bfs(dq[qt][dt][r] * a.scale);
        *reinterpret_cast<s4*>(Dp + dt * 16 + 4 * g) = ov;
      }
    }
  }
}

}  // namespace attn
}  // namespace damd

using namespace damd;
using namespace damd::attn;

extern "C" {

#define DAMD_ATTN_DISPATCH(KERNEL, GRID, ARGS)                                                       \
  do {                                                                                               \
    const bool drop_ = (ARGS).md.thresh != 0;                                                        \
    if (D == 64) {                                                                                   \
      if (causal) {                                                                                  \
        if (drop_) DAMD_LAUNCH((KERNEL<64, true, true>), GRID, dim3(kThreads), 0, st, ARGS);         \
        else DAMD_LAUNCH((KERNEL<64, true, false>), GRID, dim3(kThreads), 0, st, ARGS);              \
      } else {                                                                                       \
        if (drop_) DAMD_LAUNCH((KERNEL<64, false, true>), GRID, dim3(kThreads), 0, st, ARGS);        \
        else DAMD_LAUNCH((KERNEL<64, false, false>), GRID, dim3(kThreads), 0, st, ARGS);             \
      }                                                                                              \
    } else {                                                                                         \
      if (causal) {                                                                                  \
        if (drop_) DAMD_LAUNCH((KERNEL<128, true, true>), GRID, dim3(kThreads), 0, st, ARGS);        \
        else DAMD_LAUNCH((KERNEL<128, true, false>), GRID, dim3(kThreads), 0, st, ARGS);             \
      } else {                                                                                       \
        if (drop_) DAMD_LAUNCH((KERNEL<128, false, true>), GRID, dim3(kThreads), 0, st, ARGS);       \
        else DAMD_LAUNCH((KERNEL<128, false, false>), GRID, dim3(kThreads), 0, st, ARGS);            \
      }                                                                                              \
    }                                                                                                \
  } while (0)

static KeyMaskDrop make_md(const uint8_t* km, int64_t kms, uint32_t seed, const int64_t* seedp, float drop_p) {
  KeyMaskDrop md;
  md.km = km;
  md.kms = kms;
  md.seed = seed;
  md.seedp = seedp;
  const double t = static_cast<double>(drop_p) * 4294967296.0;
  md.thresh = drop_p > 0.f ? static_cast<uint32_t>(t >= 4294967295.0 ? 4294967295.0 : (t < 1.0 ? 1.0 : t)) : 0u;
  md.inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  return md;
}

// strides: 4 tensors (q, k, v, o) x (b, h, t) in elements; km: optional [B][kms] key mask
void damd_attn_fwd_launch(const void* q, const void* k, const void* v, void* o, float* lse, const int64_t* strides,
                          int B, int H, int T, int D, float scale, int causal, const uint8_t* km, int64_t kms,
                          uint32_t seed, const int64_t* seedp, float drop_p, hipStream_t st) {
  FwdArgs a;
  a.q = static_cast<const bf16_t*>(q); a.k = static_cast<const bf16_t*>(k); a.v = static_cast<const bf16_t*>(v);
  a.o = static_cast<bf16_t*>(o); a.lse = lse;
  a.sq = {strides[0], strides[1], strides[2]}; a.sk = {strides[3], strides[4], strides[5]};
  a.sv = {strides[6], strides[7], strides[8]}; a.so = {strides[9], strides[10], strides[11]};
  a.H = H; a.T = T; a.scale_log2 = scale * kLog2e;
  a.md = make_md(km, kms, seed, seedp, drop_p);
  dim3 grid((T + kFwdRows - 1) / kFwdRows, H, B);
  DAMD_ATTN_DISPATCH(attn_fwd_kernel, grid, a);
}

// strides: 8 tensors (q, k, v, o, dout, dk, dv, dq) x (b, h, t)
void damd_attn_bwd_launch(const void* q, const void* k, const void* v, const void* o, const void* dout,
                          const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                          const int64_t* s, int B, int H, int T, int D, float scale, int causal,
                          const uint8_t* km, int64_t kms, uint32_t seed, const int64_t* seedp, float drop_p,
                          hipStream_t st) {
  const Strides sq{s[0], s[1], s[2]}, sk{s[3], s[4], s[5]}, sv{s[6], s[7], s[8]}, so{s[9], s[10], s[11]},
      sdo{s[12], s[13], s[14]}, sdk{s[15], s[16], s[17]}, sdv{s[18], s[19], s[20]}, sdq{s[21], s[22], s[23]};
  const int64_t rows = static_cast<int64_t>(B) * H * T;
  (void)dq_acc;  // unused: dQ is produced by attn_dq_kernel without an fp32 accumulator
  {
    const int64_t threads = rows * (D / 8);
    const int blocks = static_cast<int>((threads + 255) / 256);
    if (D == 64)
      DAMD_LAUNCH((attn_delta_kernel<64>), dim3(blocks), dim3(256), 0, st, static_cast<const bf16_t*>(o), so,
                         static_cast<const bf16_t*>(dout), sdo, delta, H, T, rows);
    else
      DAMD_LAUNCH((attn_delta_kernel<128>), dim3(blocks), dim3(256), 0, st, static_cast<const bf16_t*>(o),
                         so, static_cast<const bf16_t*>(dout), sdo, delta, H, T, rows);
    DAMD_CHECK_LAUNCH();
  }
  BwdArgs a;
  a.q = static_cast<const bf16_t*>(q); a.k = static_cast<const bf16_t*>(k); a.v = static_cast<const bf16_t*>(v);
  a.dout = static_cast<const bf16_t*>(dout); a.lse = lse; a.delta = delta; a.dq_acc = dq_acc;
  a.dk = static_cast<bf16_t*>(dk); a.dv = static_cast<bf16_t*>(dv);
  a.sq = sq; a.sk = sk; a.sv = sv; a.sdo = sdo; a.sdk = sdk; a.sdv = sdv;
  a.H = H; a.T = T; a.scale = scale; a.scale_log2 = scale * kLog2e;
  a.md = make_md(km, kms, seed, seedp, drop_p);
  dim3 grid((T + kBlk - 1) / kBlk, H, B);
  DAMD_ATTN_DISPATCH(attn_bwd_kernel, grid, a);
  DqArgs d;
  d.q = a.q; d.k = a.k; d.v = a.v; d.dout = a.dout; d.lse = lse; d.delta = delta;
  d.dq = static_cast<bf16_t*>(dq);
  d.sq = sq; d.sk = sk; d.sv = sv; d.sdo = sdo; d.sdq = sdq;
  d.H = H; d.T = T; d.scale = scale; d.scale_log2 = scale * kLog2e;
  d.md = a.md;
  dim3 qgrid((T + kFwdRows - 1) / kFwdRows, H, B);
  DAMD_ATTN_DISPATCH(attn_dq_kernel, qgrid, d);
}

}  // extern "C"
