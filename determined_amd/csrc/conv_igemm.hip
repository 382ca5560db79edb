// Implicit-GEMM convolution for gfx950 / MI355X: bf16 NHWC activations, [K][R][S][C] weights
// (PyTorch's channels-last weight layout), fp32 accumulation on MFMA.
//
// One kernel serves the forward convolution and the stride-1 input gradient (the latter is the
// forward convolution of dY with the flipped, transposed weights), with an optional epilogue
// that emits the per-output-channel (sum, sum of squares) partials the following BatchNorm
// needs -- which removes BatchNorm's separate statistics pass over the conv output.
//
// GEMM view (C^T formulation): out^T[co][pixel] = W[co][k] . im2col^T[k][pixel], k = (r, s, c).
// Both operands are k-contiguous rows in memory (weight rows; one input pixel's 64 channels for
// one tap), so both are staged into LDS by the direct global->LDS DMA
// (`global_load_lds_dwordx4`, 16 B per lane, 8 rows of 128 B per wave-instruction) with a per-lane
// source address that does the im2col gather and points padding / tail rows at a zero page.
// MFMA v_mfma_f32_16x16x32_bf16: A = weight rows (co), B = pixel rows; lane l holds
// C[co = 4(l>>4) + r][pixel = l&15], so after permuting which weight row feeds which A row a lane
// ends with 8 consecutive output channels of one pixel and writes them as one 16-byte store.
//
// LDS image: [rows][64] bf16, 128-byte rows, 16-byte chunk c of row r stored at slot
// c ^ f(r), f(r) = ((r >> 1) ^ (r >> 3)) & 7 -- conflict-free for the ds_read_b128 lane groups of
// both the permuted weight rows and the consecutive pixel rows (checked against the gfx950
// lane-group table).  The DMA writes LDS linearly, so the swizzle is applied to the per-lane
// SOURCE address (chunk = slot ^ f(row)) and again on the read.
//
// Schedule: persistent blocks.  Block -> (co tile, pixel group) with the co tiles of one pixel
// group on one XCD (they read the same input rows through that XCD's L2); each block walks the
// pixel tiles grp, grp + groups, ...  The (tile, k-step) stream is flattened and double-buffered:
// the DMA for item i+1 is in flight while item i computes, including across tile boundaries, so
// K = 64 layers (one k-step per tile) still overlap their loads with the previous tile's MFMAs
// and stores.

#include <cstdlib>

#include "common.h"

namespace damd {
namespace igemm {

typedef short s8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void glb_void_t;

constexpr int kThreads = 256;  // 4 waves
constexpr int kBK = 64;        // k elements per stage: 64 channels of one tap

// 128 zero bytes: the DMA source of padding / out-of-range rows (read-only).
__device__ __attribute__((aligned(128))) uint4 g_zero_rows[8];

struct Geo {
  int H, W, C;       // input (C % 64 == 0)
  int OH, OW, K;     // output (K % BCO == 0)
  int R, S, stride, pad;
  int64_t M;         // N * OH * OW
  int cblk;          // C / 64
  int ksteps;        // R * S * cblk
  int ptiles, ctiles, groups;
  // output placement: ost == 0 -> output pixel m is row m of y; ost == 2 -> y is an
  // [N][OHf][OWf] grid and output pixel m = (n, i, j) of the OH x OW grid goes to (n, 2i + oa, 2j + ob)
  // (one phase of a stride-2 input gradient, conv_phase_launch)
  int ost, oa, ob, OHf, OWf;
  uint32_t xbytes;   // input tensor bytes (< 0xF0000000: 32-bit buffer offsets, damd_conv_fwd_launch)
};

__device__ __forceinline__ int64_t out_row(const Geo& g, int64_t m) {
  if (g.ost == 0) return m;
  const uint32_t u = static_cast<uint32_t>(m), t = u / static_cast<uint32_t>(g.OW);
  const uint32_t j = u - t * static_cast<uint32_t>(g.OW), n = t / static_cast<uint32_t>(g.OH);
  const uint32_t i = t - n * static_cast<uint32_t>(g.OH);
  return (static_cast<int64_t>(n) * g.OHf + 2 * i + g.oa) * g.OWf + 2 * j + g.ob;
}

__device__ __forceinline__ f4 mfma(s8 a, s8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}

__device__ __forceinline__ int swz(int row) { return ((row >> 1) ^ (row >> 3)) & 7; }

// compile-time integer tag (ring slots of the unrolled main loops)
template <int V>
struct IC {
  static constexpr int value = V;
};

__device__ __forceinline__ void dma16(const void* src, bf16_t* lds_base) {
  __builtin_amdgcn_global_load_lds((glb_void_t*)src, (lds_void_t*)lds_base, 16, 0, 0);
}

// the buffer form: 16 bytes from rsrc + voff (per lane) + soff (wave-uniform) to LDS
__device__ __forceinline__ void dma16b(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff, bf16_t* lds_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_base, 16, voff, soff, 0, 0);
}

// A-operand row (output channel within the wave's co range) of fragment i for fragment row rho:
// fragment pair (2q, 2q+1) covers 32 channels and lane group g ends with channels 8g..8g+7.
__device__ __forceinline__ int a_row(int i, int rho) {
  return 32 * (i >> 1) + 8 * (rho >> 2) + 4 * (i & 1) + (rho & 3);
}

// n / d for 0 <= n < 2^31 by multiply-high (d fixed per launch, magic built on the host)
struct FastDiv {
  uint32_t d, mul, shift;
  __device__ __forceinline__ uint32_t div(uint32_t n) const { return (__umulhi(n, mul) + n) >> shift; }
};

typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

// NW waves (64 * NW threads), NST-slot LDS ring: NST - 1 k-steps of DMA in flight ahead of the
// MFMAs, retired by counted waits (vmcnt counts loads and stores together in issue order, so a
// count of the younger DMA instructions is exact without epilogue stores and conservative with
// them) and a raw s_barrier (a __syncthreads() fence would drain the whole ring).
// Epilogue modes (EPI):
//   kEpiNone  : store out
//   kEpiStats : store out + (sum, sum sq) partials of the bf16 outputs (the next BN's statistics)
//   kEpiBnbM / kEpiBnbR : the kernel is the input gradient of a conv whose input was
//       a = relu(bn(yb) [+ residual]); it stores dz = (acc [+ d2]) * [a > 0] (the gradient at the
//       BN output, ReLU mask from the forward's bit mask (M) or recomputed as
//       yb*scale + shift > 0 (R)) and the partials (sum dz, sum dz*(yb - mean)) of that BN's
//       backward -- the BN-backward reduce pass over (dz, yb) is never run.
constexpr int kEpiNone = 0, kEpiStats = 1, kEpiBnbM = 2, kEpiBnbR = 3;

struct EpiArgs {
  const bf16_t* d2;      // second gradient of the BN output (shortcut consumer) or null
  const bf16_t* yb;      // BN input, [M][K]
  const uint8_t* mask;   // ReLU bit mask [M][K/8] (kEpiBnbM)
  const float* mean;     // BN batch mean [K]
  const float* scale;    // folded BN scale / shift [K] (kEpiBnbR)
  const float* shift;
  int d2h, d2w;          // 0, 0: d2 is on the output grid; else d2 is the compact (d2h x d2w) gradient of
                         // a 1x1 stride-2 shortcut's input: nonzero only at even (h, w) of the output grid
};

// Tile epilogue shared by the conv kernels (EPI modes above): stores the BP x BCO output tile of
// pixel tile pt / co tile ct from the accumulators, accumulating the per-lane channel sums.
// Prologue (PRO) mode of the generic kernel, 1x1 / stride 1 only: the input operand is
// a = relu(y * scale[c] + shift[c] [+ res]) computed while staging (global -> registers ->
// transform -> LDS) instead of read from a materialised `a`; the blocks of co tile 0 also write
// `a` (aout) and its ReLU bit mask (mout) for the backward / the shortcut consumer.  This fuses
// a BatchNorm(+residual)+ReLU forward apply pass into its consuming 1x1 convolution: the
// activation is read as (y, res) once instead of (y, res) by the BN pass and `a` by the conv.
// PRO == 2 is the backward counterpart: the operand is a BN backward's output
// dy = A * dz + B * y + Cc (x = dz, res = y, scale = A, rscale = B, shift = Cc, no ReLU), written to
// aout by co tile 0 for the weight gradient -- the BN backward apply pass fused into the input
// gradient of the conv that produced y.
struct ProArgs {
  const bf16_t* res;     // residual added before the ReLU (PRO 1) / BN input y (PRO 2), or null
  const float* scale;    // per input channel [C]: folded BN scale (PRO 1) / A (PRO 2)
  const float* shift;    //                         folded BN shift (PRO 1) / Cc (PRO 2)
  const float* rscale;   // PRO 2: B (scale of res); PRO 1: null (res enters with weight 1) or the
                         // residual's own folded BN scale (its shift is pre-added to `shift`)
  bf16_t* aout;          // the operand, [M][C], or null
  uint8_t* mout;         // PRO 1: ReLU bit mask of a, [M][C/8], or null
};

template <int BCO, int BP, int FI, int FJ, int EPI>
__device__ __forceinline__ void epi_store_tile(const f4 (&acc)[FI][FJ], int64_t pt, int ct, int wco0, int wp0, int lg,
                                               int rho, const Geo& g, const EpiArgs& ea, const float* prm,
                                               bf16_t* __restrict__ y, float (&st_s)[FI / 2][8],
                                               float (&st_q)[FI / 2][8]) {
  // epilogue: lane (lg, rho) holds channels wco0 + 32q + 8lg + 0..7 of pixel wp0 + 16j + rho.
  // Done in halves over j: the BN-backward operand loads of a half are all issued first
  // (unconditionally, tail rows clamped to row 0, a missing d2 replaced by yb and scaled
  // by 0) so they overlap instead of each load waiting before the next is issued.
  constexpr int JH = FJ >= 2 ? FJ / 2 : 1;
  const bf16_t* d2p = ea.d2 != nullptr ? ea.d2 : ea.yb;
  const float d2f = ea.d2 != nullptr ? 1.f : 0.f;
#pragma unroll
  for (int j0 = 0; j0 < FJ; j0 += JH) {
    bf16x8 dv[JH][FI / 2], yr[JH][FI / 2];
    uint32_t mb[JH][FI / 2];
    float d2k[JH];
    if (EPI >= kEpiBnbM) {
#pragma unroll
      for (int jj = 0; jj < JH; ++jj) {
        const int64_t m = pt * BP + wp0 + 16 * (j0 + jj) + rho;
        const int64_t ms = m < g.M ? m : 0;
        int64_t m2 = ms;  // d2's pixel
        d2k[jj] = d2f;
        if (ea.d2h > 0) {  // compact stride-2 grid: odd rows / columns of the output get no d2
          const uint32_t u = static_cast<uint32_t>(ms), t = u / static_cast<uint32_t>(g.OW);
          const uint32_t w = u - t * static_cast<uint32_t>(g.OW), n = t / static_cast<uint32_t>(g.OH);
          const uint32_t h = t - n * static_cast<uint32_t>(g.OH);
          const bool on = ((h | w) & 1u) == 0;
          m2 = on ? (static_cast<int64_t>(n) * ea.d2h + (h >> 1)) * ea.d2w + (w >> 1) : 0;
          d2k[jj] = on ? d2f : 0.f;
        }
#pragma unroll
        for (int q = 0; q < FI / 2; ++q) {
          const int64_t cof = static_cast<int64_t>(ct) * BCO + wco0 + 32 * q + 8 * lg;
          const int64_t off = ms * g.K + cof;
          yr[jj][q] = *reinterpret_cast<const bf16x8*>(ea.yb + off);
          dv[jj][q] = *reinterpret_cast<const bf16x8*>(d2p + m2 * g.K + cof);
          if (EPI == kEpiBnbM) mb[jj][q] = ea.mask[off >> 3];
        }
      }
    }
#pragma unroll
    for (int jj = 0; jj < JH; ++jj) {
      const int j = j0 + jj;
      const int64_t m = pt * BP + wp0 + 16 * j + rho;
      const bool ok = m < g.M;
#pragma unroll
      for (int q = 0; q < FI / 2; ++q) {
        const int cl = wco0 + 32 * q + 8 * lg;  // channel within the block's co tile
        const int64_t co = static_cast<int64_t>(ct) * BCO + cl;
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] = acc[2 * q][j][e]; o[4 + e] = acc[2 * q + 1][j][e]; }
        float yv[8];
        if (EPI >= kEpiBnbM) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            yv[e] = bf2f(yr[jj][q].v[e]);
            o[e] += d2k[jj] * bf2f(dv[jj][q].v[e]);
          }
          if (EPI == kEpiBnbM) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (mb[jj][q] >> e) & 1u ? o[e] : 0.f;
          } else {
            const float4 s0 = *reinterpret_cast<const float4*>(prm + BCO + cl);
            const float4 s1 = *reinterpret_cast<const float4*>(prm + BCO + cl + 4);
            const float4 h0 = *reinterpret_cast<const float4*>(prm + 2 * BCO + cl);
            const float4 h1 = *reinterpret_cast<const float4*>(prm + 2 * BCO + cl + 4);
            const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
            const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = yv[e] * sc[e] + sh[e] > 0.f ? o[e] : 0.f;
          }
        }
        bf16x8 v;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const u16v2_t pk = f2bf2(o[e], o[e + 1]);
          v.v[e] = pk[0]; v.v[e + 1] = pk[1];
        }
        if (ok) {
          *reinterpret_cast<bf16x8*>(y + out_row(g, m) * g.K + co) = v;
          if (EPI == kEpiStats) {  // statistics of the fp32 conv outputs (before the bf16 store)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              st_s[q][e] += o[e];
              st_q[q][e] += o[e] * o[e];
            }
          } else if (EPI >= kEpiBnbM) {
            const float4 u0 = *reinterpret_cast<const float4*>(prm + cl);
            const float4 u1 = *reinterpret_cast<const float4*>(prm + cl + 4);
            const float mu[8] = {u0.x, u0.y, u0.z, u0.w, u1.x, u1.y, u1.z, u1.w};
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const float f = bf2f(v.v[e]);  // the stored (rounded) dz, as the apply pass reads it
              st_s[q][e] += f;
              st_q[q][e] += f * (yv[e] - mu[e]);
            }
          }
        }
      }
    }
  }
}

// Block-level reduction of the epilogue channel sums into part[grp][2][K] (LDS reused: call
// after the last fragment read).
template <int BCO, int FI, int WCO, int NW>
__device__ __forceinline__ void epi_flush_sums(float (&st_s)[FI / 2][8], float (&st_q)[FI / 2][8], bf16_t* lds,
                                               int wave, int lg, int rho, int wco0, int grp, int ct, int K,
                                               float* __restrict__ part) {
  constexpr int NT = 64 * NW, WP = NW / WCO;
  // sum over the 16 pixel lanes of each lane group, then over the WP waves sharing a co range
#pragma unroll
  for (int q = 0; q < FI / 2; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        st_s[q][e] += __shfl_xor(st_s[q][e], o, 64);
        st_q[q][e] += __shfl_xor(st_q[q][e], o, 64);
      }
  __syncthreads();  // LDS reuse: every wave is past its last fragment read
  float* red = reinterpret_cast<float*>(lds);  // [WP][2][BCO]
  const int wpi = wave / WCO;
  if (rho == 0) {
#pragma unroll
    for (int q = 0; q < FI / 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int co = wco0 + 32 * q + 8 * lg + e;
        red[(wpi * 2) * BCO + co] = st_s[q][e];
        red[(wpi * 2 + 1) * BCO + co] = st_q[q][e];
      }
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * BCO; t += NT) {
    const int which = t / BCO, co = t - which * BCO;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WP; ++k) s += red[(k * 2 + which) * BCO + co];
    part[(static_cast<int64_t>(grp) * 2 + which) * K + static_cast<int64_t>(ct) * BCO + co] = s;
  }
}


// ============================================================================ stream-K work plans
// A persistent launch that deals whole pixel tiles round-robin ends on a partial round: with T
// tiles per co tile and G blocks, the slowest block computes ceil(T / G) tiles while the average is
// T / G (ResNet-50 at batch 512: 3.06 -> 4 rounds on the 14x14 layers, 1.53 -> 2 on 7x7).  With
// stream-K (Geo::sk) each XCD slice of the grid (G / 8 blocks, the XCD-grouped block order above)
// takes 1/8 of the pixel tiles and cuts its (tile, k-unit) stream into equal contiguous ranges, one
// per block, so a tile may be computed in segments by consecutive blocks.  A block's range is at
// most: a TAIL (the end of a tile begun by earlier blocks), whole tiles, and a HEAD (the start of a
// tile the next block finishes); it runs them as whole tiles -> HEAD -> TAIL.  A HEAD (or a MIDDLE
// segment) is published as an fp32 slab; the block owning a tile's last unit gathers the earlier
// segments' slabs into its accumulators and runs the epilogue (BN statistics etc. exactly once per
// tile).  Hand-off (MI355X agent-scope protocol): slabs are stored write-through (sc1 buffer
// stores), every storing wave drains (vmcnt(0)), a barrier, then one lane sets the block's flag with
// a relaxed agent-scope atomic store; the consumer's lane 0 polls relaxed, takes ONE agent acquire,
// resets the flag for the next launch, and after a barrier every wave reads the slabs with plain
// loads.  Every block publishes before it waits, and only waits on earlier blocks of its own XCD
// slice (dispatched before it), so the chain always drains; the poll is bounded anyway: a time-out
// counts in sk.err and fills the tile with NaN (never a silently wrong output); the host checks
// the counter (ops.conv_health_check) after tuning and at reporting boundaries, and raises.
struct SkArgs {
  float* ws;   // [nblk][BCO * BP] fp32 slabs, slot = the block's remapped id
  int* flags;  // [nblk] 0 / 1, zero between launches (the consumer resets them)
  int* err;    // poll time-outs (must stay 0)
};

struct Plan {
  int nfull, t0, ts;   // whole tiles t0 + i * ts
  int th, kh;          // HEAD: tile th, units [0, kh)
  int tt, ka, ke;      // TAIL: tile tt, units [ka, ke)
  int gpx, xs, j, p0;  // stream-K: blocks per XCD slice, slice, index in it, its first tile
  int64_t U;           // units in the slice
};

__device__ __forceinline__ Plan make_plan(int grp, int groups, int ptiles, int units, int sk) {
  Plan p{};
  p.ts = 1;
  if (!sk) {
    p.nfull = grp < ptiles ? (ptiles - grp + groups - 1) / groups : 0;
    p.t0 = grp;
    p.ts = groups;
    return p;
  }
  p.gpx = groups >> 3;
  p.xs = grp / p.gpx;
  p.j = grp - p.xs * p.gpx;
  p.p0 = static_cast<int>(static_cast<int64_t>(p.xs) * ptiles / 8);
  const int p1 = static_cast<int>(static_cast<int64_t>(p.xs + 1) * ptiles / 8);
  p.U = static_cast<int64_t>(p1 - p.p0) * units;
  const int64_t u0 = p.j * p.U / p.gpx, u1 = (p.j + 1) * p.U / p.gpx;
  if (u0 >= u1) return p;
  const int a = p.p0 + static_cast<int>(u0 / units), ka = static_cast<int>(u0 % units);
  const int b = p.p0 + static_cast<int>(u1 / units), kb = static_cast<int>(u1 % units);
  if (a == b) {  // the whole range lies in one tile
    if (ka == 0) { p.th = a; p.kh = kb; } else { p.tt = a; p.ka = ka; p.ke = kb; }
    return p;
  }
  int fs = a;
  if (ka > 0) { p.tt = a; p.ka = ka; p.ke = units; fs = a + 1; }
  p.t0 = fs;
  p.nfull = b - fs;
  if (kb > 0) { p.th = b; p.kh = kb; }
  return p;
}

// Segment cursor over a plan: run 0 = whole tiles, 1 = HEAD, 2 = TAIL, 3 = done.
struct Cursor {
  int run, i, pt, k, kend;
};

__device__ __forceinline__ void seg_enter(Cursor& c, const Plan& p, int units) {
  if (c.run == 0) {
    if (c.i < p.nfull) { c.pt = p.t0 + c.i * p.ts; c.k = 0; c.kend = units; return; }
    c.run = 1;
  }
  if (c.run == 1) {
    if (p.kh > 0) { c.pt = p.th; c.k = 0; c.kend = p.kh; return; }
    c.run = 2;
  }
  if (c.run == 2) {
    if (p.ke > p.ka) { c.pt = p.tt; c.k = p.ka; c.kend = p.ke; return; }
    c.run = 3;
  }
}

__device__ __forceinline__ void seg_next(Cursor& c, const Plan& p, int units) {
  if (c.run == 0) ++c.i; else ++c.run;
  seg_enter(c, p, units);
}

__device__ __forceinline__ int plan_units(const Plan& p, int units) { return p.nfull * units + p.kh + (p.ke - p.ka); }

typedef int v4i __attribute__((ext_vector_type(4)));

// publish this block's partial tile (slot `rid`) and set its flag
template <int FI, int FJ, int NT>
__device__ __forceinline__ void sk_publish(const f4 (&acc)[FI][FJ], const SkArgs& sk, int rid) {
  float* base = sk.ws + static_cast<int64_t>(rid) * (FI * FJ * 4 * NT);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, FI * FJ * 16 * NT, 0x00020000);
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)  // write-through (sc1): visible without a release fence
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i, acc[i][j]), rs,
                                             ((i * FJ + j) * NT + static_cast<int>(threadIdx.x)) * 16, 0, 16);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store(sk.flags + rid, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// add the slabs of every earlier block of this XCD slice that computed part of tile `pt`
template <int FI, int FJ, int NT>
__device__ __forceinline__ void sk_gather(f4 (&acc)[FI][FJ], const SkArgs& sk, const Plan& p, int pt, int units,
                                          int ctiles, int ct) {
  const int64_t t0u = static_cast<int64_t>(pt - p.p0) * units;  // the tile's first unit in the slice
  __shared__ int sk_bad;  // a hand-off that never arrived: the tile's output is poisoned (NaN)
  if (threadIdx.x == 0) {
    int bad = 0;
    for (int jj = p.j - 1; jj >= 0; --jj) {
      const int64_t r0 = jj * p.U / p.gpx, r1 = (jj + 1) * p.U / p.gpx;
      if (r1 <= t0u) break;
      if (r0 >= r1) continue;
      int* f = sk.flags + (p.xs * p.gpx + jj) * ctiles + ct;
      unsigned spins = 0;
      bool arrived = true;
      while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 20)) { arrived = false; break; }
      }
      if (arrived) {
        __hip_atomic_store(f, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // ready for the next launch
      } else {  // the flag is left as is: the host sees sk.err, resets the flags and raises
        __hip_atomic_fetch_add(sk.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bad = 1;
      }
    }
    sk_bad = bad;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (sk_bad) {  // never a silently wrong tile: NaN propagates into the loss
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = f4{__builtin_nanf(""), __builtin_nanf(""), __builtin_nanf(""),
                                                  __builtin_nanf("")};
    return;
  }
  for (int jj = p.j - 1; jj >= 0; --jj) {
    const int64_t r0 = jj * p.U / p.gpx, r1 = (jj + 1) * p.U / p.gpx;
    if (r1 <= t0u) break;
    if (r0 >= r1) continue;
    const f4* slab = reinterpret_cast<const f4*>(sk.ws + static_cast<int64_t>((p.xs * p.gpx + jj) * ctiles + ct) *
                                                            (FI * FJ * 4 * NT));
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] += slab[(i * FJ + j) * NT + threadIdx.x];
  }
}


// SCH (k-step schedule): 0 = per 32-deep half: fragment reads then its MFMAs; 1 = all fragment
// reads of the k-step issued first (the second half's reads overlap the first half's MFMAs);
// 2 = as 1 with s_setprio(1) over the MFMA block; 3 = software-pipelined across k-steps (below).
template <int BCO, int BP, int WCO, int NW, int NST, int EPI, int SCH = 0, int PRO = 0, int SK = 0>
__global__ void __launch_bounds__(64 * NW, 2)
conv_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                float* __restrict__ part, Geo g, EpiArgs ea, ProArgs pa, SkArgs sk) {
  constexpr bool SUMS = EPI != kEpiNone;
  constexpr int NT = 64 * NW;
  constexpr int WP = NW / WCO;
  constexpr int TCO = BCO / WCO, TP = BP / WP;
  constexpr int FI = TCO / 16, FJ = TP / 16;
  static_assert(WCO * WP == NW && FI % 2 == 0 && FJ >= 1 && BCO % (8 * NW) == 0 && BP % (8 * NW) == 0, "bad tile");
  static_assert(NST >= 2 && NST <= 4, "ring depth");
  constexpr int STAGE = (BCO + BP) * kBK;  // elements per stage
  constexpr int NIW = BCO / (8 * NW), NIX = BP / (8 * NW);  // DMA instructions per wave per stage
  constexpr int NL = NIW + NIX;
  static_assert(NL * (NST - 2) <= 63, "vmcnt range");
  static_assert(!PRO || (NST == 3 && (SCH == 0 || SCH == 3)), "prologue mode uses the 3-slot ring");
  // one LDS array (a second __shared__ object makes hipcc wait for every DMA before each
  // ds_read): NST ring slots, then the block's per-channel BN parameters for the BN-backward
  // epilogues (mean, scale, shift of its BCO output channels; the co tile is fixed per block)
  constexpr int PARAMS = EPI >= kEpiBnbM ? 3 * BCO * 2 : 0;  // in bf16_t units (3 x BCO floats)
  __shared__ __attribute__((aligned(16))) bf16_t lds[NST * STAGE + PARAMS];
  float* prm = reinterpret_cast<float*>(lds + NST * STAGE);

  // wave index as a provably uniform (SGPR) value: the LDS-DMA destinations derived from it go
  // to M0 without a v_readfirstlane per DMA
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int rho = lane & 15, lg = lane >> 4;
  const int wco0 = (wave % WCO) * TCO, wp0 = (wave / WCO) * TP;

  // block -> (co tile, pixel group); consecutive remapped ids share an XCD (bijective remap)
  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ct = rid % g.ctiles, grp = rid / g.ctiles;
  const Plan plan = make_plan(grp, g.groups, g.ptiles, g.ksteps, SK);
  const int items = plan_units(plan, g.ksteps);
  const int64_t Ktot = static_cast<int64_t>(g.ksteps) * kBK;
  // LDS-DMA through buffer resources (buffer_load_dwordx4 ... lds): a lane's source is a 32-bit
  // byte offset (VGPR) plus a wave-uniform k-step offset (SGPR), so a DMA costs no 64-bit VALU
  // address arithmetic; an out-of-range offset (a tap outside the image) reads zeros.  The host
  // keeps both tensors below 0xF0000000 bytes (damd_conv_fwd_launch).
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(w), 0, static_cast<int>(g.K * Ktot * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16_t*>(x), 0, static_cast<int>(g.xbytes), 0x00020000);
  if (EPI >= kEpiBnbM) {  // visible to every wave after the main loop's first barrier
    for (int t = threadIdx.x; t < BCO; t += NT) {
      const int co = ct * BCO + t;
      prm[t] = ea.mean[co];
      prm[BCO + t] = EPI == kEpiBnbR ? ea.scale[co] : 0.f;
      prm[2 * BCO + t] = EPI == kEpiBnbR ? ea.shift[co] : 0.f;
    }
  }

  // ---- DMA lane roles: lane -> (row within its 8-row piece, 16-byte slot)
  const int prow = lane >> 3, slot = lane & 7;
  uint32_t wvoff[NIW];  // byte offset of the lane's weight chunk at k-step 0
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int co = 8 * (wave + NW * i) + prow;
    wvoff[i] = static_cast<uint32_t>(((static_cast<int64_t>(ct) * BCO + co) * Ktot + ((slot ^ swz(co)) << 3)) * 2);
  }
  // pixel rows, per tile: element offset of the row's tap-(0,0) input pixel (+ its DMA chunk;
  // may lie outside the image -- only dereferenced for valid taps) and a bit mask of the taps
  // r*S + s that fall inside the image.  Per k-step the source is then one 64-bit add of a
  // wave-uniform tap/channel offset and a bit test (the per-k-step im2col arithmetic was ~4
  // VALU instructions per MFMA in the PMC counters).
  // bytes, modulo 2^32: the tap-(0,0) pixel may lie before the tensor (negative), and inputs are
  // up to 0xF0000000 bytes, so the offsets are kept unsigned and wrap by definition; for a tap
  // inside the image xbase + soff is the true (in-range) byte offset
  uint32_t xbase[NIX];
  uint32_t vmask[NIX];
  const int OHW = g.OH * g.OW;
  auto tile_rows = [&](int pt) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < NIX; ++i) {
      const int p = 8 * (wave + NW * i) + prow;
      const int m = pt * BP + p;  // M < 2^31 (host-checked)
      const int n = m / OHW;
      const int rem = m - n * OHW;
      const int oh = rem / g.OW, ow = rem - (rem / g.OW) * g.OW;
      const int ih0 = oh * g.stride - g.pad, iw0 = ow * g.stride - g.pad;
      xbase[i] = static_cast<uint32_t>((((static_cast<int64_t>(n) * g.H + ih0) * g.W + iw0) * g.C + ((slot ^ swz(p)) << 3)) * 2);
      uint32_t bits = 0;
      if (m < g.M) {
        for (int r = 0; r < g.R; ++r) {
          const bool rok = static_cast<unsigned>(ih0 + r) < static_cast<unsigned>(g.H);
          for (int s2 = 0; s2 < g.S; ++s2)
            if (rok && static_cast<unsigned>(iw0 + s2) < static_cast<unsigned>(g.W)) bits |= 1u << (r * g.S + s2);
        }
      }
      vmask[i] = bits;
    }
  };

  // PRO: register-staged input rows of one k-step (lane: channel chunk `slot`, rows
  // 8 * (wave + NW * i) + prow), their BN parameters, and the tile / channel block they belong to
  bf16x8 py[PRO ? NIX : 1], pr[PRO ? NIX : 1];
  float4 psc[2], psh[2], prs[2];
  int p_pt = 0, p_cb = 0;
  auto load_px = [&](int pt, int cb) __attribute__((always_inline)) {
    p_pt = pt;
    p_cb = cb;
    const int cofs = cb * kBK + (slot << 3);
#pragma unroll
    for (int i = 0; i < NIX; ++i) {
      const int m = pt * BP + 8 * (wave + NW * i) + prow;
      const int64_t off = static_cast<int64_t>(m < g.M ? m : 0) * g.C + cofs;
      py[i] = *reinterpret_cast<const bf16x8*>(x + off);
      if (pa.res != nullptr) pr[i] = *reinterpret_cast<const bf16x8*>(pa.res + off);
    }
    psc[0] = *reinterpret_cast<const float4*>(pa.scale + cofs);
    psc[1] = *reinterpret_cast<const float4*>(pa.scale + cofs + 4);
    psh[0] = *reinterpret_cast<const float4*>(pa.shift + cofs);
    psh[1] = *reinterpret_cast<const float4*>(pa.shift + cofs + 4);
    if (PRO == 2 || pa.rscale != nullptr) {
      prs[0] = *reinterpret_cast<const float4*>(pa.rscale + cofs);
      prs[1] = *reinterpret_cast<const float4*>(pa.rscale + cofs + 4);
    }
  };
  // transform the staged rows into LDS slot `stage` (+ a / mask stores by co tile 0)
  auto store_px = [&](int stage) __attribute__((always_inline)) {
    bf16_t* sx = lds + stage * STAGE + BCO * kBK;
    const float sc[8] = {psc[0].x, psc[0].y, psc[0].z, psc[0].w, psc[1].x, psc[1].y, psc[1].z, psc[1].w};
    const float sh[8] = {psh[0].x, psh[0].y, psh[0].z, psh[0].w, psh[1].x, psh[1].y, psh[1].z, psh[1].w};
    float rs[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) rs[e] = 1.f;
    if (PRO == 2 || pa.rscale != nullptr) {
      rs[0] = prs[0].x; rs[1] = prs[0].y; rs[2] = prs[0].z; rs[3] = prs[0].w;
      rs[4] = prs[1].x; rs[5] = prs[1].y; rs[6] = prs[1].z; rs[7] = prs[1].w;
    }
    const bool has_res = pa.res != nullptr;
#pragma unroll
    for (int i = 0; i < NIX; ++i) {
      const int row = 8 * (wave + NW * i) + prow;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = bf2f(py[i].v[e]) * sc[e] + sh[e];
        if (has_res) t += rs[e] * bf2f(pr[i].v[e]);
        v[e] = PRO == 1 ? fmaxf(t, 0.f) : t;
      }
      bf16x8 o;
      uint32_t bits = 0;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const u16v2_t pk = f2bf2(v[e], v[e + 1]);
        o.v[e] = pk[0]; o.v[e + 1] = pk[1];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) bits |= (v[e] > 0.f ? 1u : 0u) << e;
      *reinterpret_cast<bf16x8*>(sx + row * kBK + ((slot ^ swz(row)) << 3)) = o;
      const int m = p_pt * BP + row;
      if (ct == 0 && m < g.M) {
        const int64_t off = static_cast<int64_t>(m) * g.C + p_cb * kBK + (slot << 3);
        if (pa.aout != nullptr) *reinterpret_cast<bf16x8*>(pa.aout + off) = o;
        if (PRO == 1 && pa.mout != nullptr) pa.mout[off >> 3] = static_cast<uint8_t>(bits);
      }
    }
  };

  // load side: segment cursor (tile, k-step range) + the k-step's channel block and tap (r, s)
  Cursor lc{0, 0, 0, 0, 0};
  seg_enter(lc, plan, g.ksteps);
  int l_cb = 0, l_r = 0, l_s = 0;
  bool l_new = true;
  auto seed = [&]() __attribute__((always_inline)) {  // k-step lc.k = (r * S + s) * cblk + cb
    l_cb = lc.k % g.cblk;
    const int rs = lc.k / g.cblk;
    l_s = rs % g.S;
    l_r = rs / g.S;
    l_new = true;
  };
  seed();
  auto issue = [&](int stage) __attribute__((always_inline)) {
    bf16_t* sw = lds + stage * STAGE;
    const int pt = lc.pt;
    if (!PRO && l_new) tile_rows(pt);
    l_new = false;
    const int wk = lc.k * kBK * 2;  // wave-uniform byte offset of this k-step in a weight row
#pragma unroll
    for (int i = 0; i < NIW; ++i) dma16b(rs_w, wvoff[i], wk, sw + 8 * (wave + NW * i) * kBK);
    if (!PRO) {
      const int tap = l_r * g.S + l_s;
      const int soff = ((l_r * g.W + l_s) * g.C + l_cb * kBK) * 2;  // wave-uniform, bytes
#pragma unroll
      for (int i = 0; i < NIX; ++i) {
        const uint32_t off = (vmask[i] >> tap) & 1u ? xbase[i] + static_cast<uint32_t>(soff) : 0xFFFFFFF0u;
        dma16b(rs_x, off, 0, sw + (BCO + 8 * (wave + NW * i)) * kBK);
      }
    } else {
      load_px(pt, l_cb);
    }
    // advance (cb fastest, then s, then r, then the next segment)
    if (++l_cb == g.cblk) {
      l_cb = 0;
      if (++l_s == g.S) {
        l_s = 0;
        if (++l_r == g.R) l_r = 0;
      }
    }
    if (++lc.k == lc.kend) {
      seg_next(lc, plan, g.ksteps);
      seed();
    }
  };

  // per-lane LDS fragment offsets (elements) for the two 32-deep k halves of a stage
  int aoff[2][FI], boff[2][FJ];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int chunk = kk * 4 + lg;
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wco0 + a_row(i, rho);
      aoff[kk][i] = row * kBK + ((chunk ^ swz(row)) << 3);
    }
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int row = wp0 + 16 * j + rho;
      boff[kk][j] = (BCO + row) * kBK + ((chunk ^ swz(row)) << 3);
    }
  }

  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float st_s[FI / 2][8], st_q[FI / 2][8];
  if (SUMS) {
#pragma unroll
    for (int q = 0; q < FI / 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) { st_s[q][e] = 0.f; st_q[q][e] = 0.f; }
  }

  // The main loops run NST items per trip with the ring slot of each a compile-time constant
  // (step(IC<S>)): every fragment read is then `ds_read_b128 off[lane] offset:S*STAGE` with no VALU
  // address arithmetic (a runtime slot cost two VALU instructions per read -- the kernels are
  // VALU-issue-bound, profiles/conv3x3_pmc_valu_bound_b1024_1gpu.txt).
  auto tile_done = [&](Cursor& cc) __attribute__((always_inline)) {
    if (++cc.k == cc.kend) {
      const bool whole = !SK || cc.run == 0 || (cc.run == 2 && cc.kend == g.ksteps);
      if (!whole) {  // HEAD / middle segment: hand the partial tile to the block that finishes it
        sk_publish<FI, FJ, NT>(acc, sk, rid);
      } else {
        if (SK && cc.run == 2) sk_gather<FI, FJ, NT>(acc, sk, plan, cc.pt, g.ksteps, g.ctiles, ct);
        epi_store_tile<BCO, BP, FI, FJ, EPI>(acc, cc.pt, ct, wco0, wp0, lg, rho, g, ea, prm, y, st_s, st_q);
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      seg_next(cc, plan, g.ksteps);
    }
  };
  if constexpr (SCH == 3) {
    // Software-pipelined k-steps: the fragments of each k-half are read from LDS while the other
    // half's MFMAs run -- the item's second half during its first half's MFMAs, the NEXT item's
    // first half (after the one barrier per item, placed mid-item) during this item's second
    // half.  The MFMA pipe then waits on LDS only at the start of a launch, not at every k-step.
    // Ring safety: the barrier of iteration it follows every wave's wait on its reads of slot it
    // (lgkmcnt) and on the DMA / operand registers of item it+1 (vmcnt), so item it+2 may then be
    // issued into slot (it+2) % NST and item it+1's operand stored (PRO) into slot (it+1) % NST.
    s8 fa[2][FI], fb[2][FJ];
    auto read_half = [&](auto SI, int kk) __attribute__((always_inline)) {
      constexpr int S = decltype(SI)::value;
      const bf16_t* sw = lds + S * STAGE;
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[kk][i] = *reinterpret_cast<const s8*>(sw + aoff[kk][i]);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb[kk][j] = *reinterpret_cast<const s8*>(sw + boff[kk][j]);
    };
    auto mfma_half = [&](int kk) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(fa[kk][i], fb[kk][j], acc[i][j]);
    };
    if (items > 0) {
      issue(0);
      if (PRO) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store_px(0);
        if (items > 1) issue(1);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      } else {
        if (items > 1) {
          issue(1);
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      read_half(IC<0>{}, 0);
    }
    Cursor cc{0, 0, 0, 0, 0};
    seg_enter(cc, plan, g.ksteps);
    auto step = [&](auto SI, int it) __attribute__((always_inline)) {
      constexpr int S = decltype(SI)::value;
      read_half(SI, 1);
      mfma_half(0);
      if (it + 1 < items) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // item it+1: DMA (+ operand registers, PRO)
        if (PRO) store_px((S + 1) % NST);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of slot it (+ its stores)
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (it + 2 < items) issue((S + 2) % NST);
        read_half(IC<(S + 1) % NST>{}, 0);
      }
      mfma_half(1);
      tile_done(cc);
    };
    for (int it0 = 0; it0 < items; it0 += NST) {
      step(IC<0>{}, it0);
      if (it0 + 1 < items) step(IC<1>{}, it0 + 1);
      if constexpr (NST > 2) if (it0 + 2 < items) step(IC<2 % NST>{}, it0 + 2);
      if constexpr (NST > 3) if (it0 + 3 < items) step(IC<3 % NST>{}, it0 + 3);
    }
  } else {
    if (PRO) {
      // item j: weights DMA + input rows to registers at iteration j-2, transform into LDS at
      // iteration j-1, MFMAs at iteration j
      if (items > 0) {
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        store_px(0);
      }
      if (items > 1) issue(1);
    } else {
  #pragma unroll
      for (int s0 = 0; s0 < NST - 1; ++s0)
        if (s0 < items) issue(s0);
    }
    Cursor cc{0, 0, 0, 0, 0};
    seg_enter(cc, plan, g.ksteps);
    auto step = [&](auto SI, int it) __attribute__((always_inline)) {
      constexpr int S = decltype(SI)::value;
      if (PRO) {
        // weights of item it, input registers of item it+1 and this wave's LDS writes of item it
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        if (it + 1 < items) store_px((S + 1) % NST);
        if (it + 2 < items) issue((S + 2) % NST);
      } else {
        // retire slot it: the DMAs of the (at most NST - 2) later slots already issued may stay in flight
        const int ahead = items - 1 - it;
        if (NST >= 4 && ahead >= 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NL) : "memory");
        else if (NST >= 3 && ahead >= 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NL) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();  // slot it landed for every wave; slot it-1 is no longer read
        if (it + NST - 1 < items) issue((S + NST - 1) % NST);
      }
      const bf16_t* sw = lds + S * STAGE;
      if (SCH == 0) {
  #pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          s8 a[FI], b[FJ];
  #pragma unroll
          for (int i = 0; i < FI; ++i) a[i] = *reinterpret_cast<const s8*>(sw + aoff[kk][i]);
  #pragma unroll
          for (int j = 0; j < FJ; ++j) b[j] = *reinterpret_cast<const s8*>(sw + boff[kk][j]);
  #pragma unroll
          for (int i = 0; i < FI; ++i)
  #pragma unroll
            for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
        }
      } else {
        s8 a[2][FI], b[2][FJ];
  #pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
  #pragma unroll
          for (int i = 0; i < FI; ++i) a[kk][i] = *reinterpret_cast<const s8*>(sw + aoff[kk][i]);
  #pragma unroll
          for (int j = 0; j < FJ; ++j) b[kk][j] = *reinterpret_cast<const s8*>(sw + boff[kk][j]);
        }
        if (SCH == 2) __builtin_amdgcn_s_setprio(1);
  #pragma unroll
        for (int kk = 0; kk < 2; ++kk)
  #pragma unroll
          for (int i = 0; i < FI; ++i)
  #pragma unroll
            for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(a[kk][i], b[kk][j], acc[i][j]);
        if (SCH == 2) __builtin_amdgcn_s_setprio(0);
      }
      tile_done(cc);
    };
    for (int it0 = 0; it0 < items; it0 += NST) {
      step(IC<0>{}, it0);
      if (it0 + 1 < items) step(IC<1>{}, it0 + 1);
      if constexpr (NST > 2) if (it0 + 2 < items) step(IC<2 % NST>{}, it0 + 2);
      if constexpr (NST > 3) if (it0 + 3 < items) step(IC<3 % NST>{}, it0 + 3);
    }
  }

  if (SUMS) epi_flush_sums<BCO, FI, WCO, NW>(st_s, st_q, lds, wave, lg, rho, wco0, grp, ct, g.K, part);
}



// =============================================================================== 3x3 halo kernel
// 3x3 / stride 1 / pad 1 convolution (forward, or the input gradient with flipped weights).  The
// generic kernel re-gathers the im2col rows of every tap (9 x BP pixel rows per 64 channels) and
// is bound by the LDS-DMA gather rate from L2 (~52 GB/s per CU measured: 256-ch 3x3 at 14x14 in
// profiles/conv_igemm_*).  Here the pixel tile's input halo -- the BP + 2W + 2 consecutive input
// pixels m0 - W - 1 ... (stride 1 keeps the flattened input and output pixel index aligned) -- is
// staged ONCE per 64-channel block and all 9 taps read it at row offset r*W + s; a per-pixel
// 9-bit tap-validity mask zeroes the fragments whose tap falls outside the image (the flattened
// neighbour belongs to another row or image).  Weights stream per tap through a 3-slot ring.
// Halo image swizzle: chunk c of row k at slot c ^ (k & 7) -- conflict-free for 16 consecutive
// rows starting at ANY row (the taps shift the fragment rows by r*W + s).
constexpr int kHaloMaxLds = 160 * 1024;

// PRO (as in conv_fwd_kernel): the halo is register-staged -- loaded at issue time, transformed
// (PRO 1: a = relu(x * scale + shift), the consuming conv's BatchNorm+ReLU forward apply; PRO 2:
// dy = A * dz + B * y + Cc, the producing conv's deferred BatchNorm-backward apply) and written to
// LDS one iteration later; blocks of co tile 0 also store the operand for the tile's own pixels
// (aout: the activation / gradient the weight gradient needs).  Out-of-image rows stay zero.
constexpr int kHaloProRows = 6;  // register-staged halo rows per lane: HR <= 6 * 8 * NW

template <int BCO, int BP, int WCO, int NW, int EPI, int SK = 0, int PRO = 0>
__global__ void __launch_bounds__(64 * NW, 2)
conv3x3_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
               float* __restrict__ part, Geo g, EpiArgs ea, int HR, SkArgs sk, ProArgs pa) {
  constexpr bool SUMS = EPI != kEpiNone;
  constexpr int NT = 64 * NW;
  constexpr int WP = NW / WCO;
  constexpr int TCO = BCO / WCO, TP = BP / WP;
  constexpr int FI = TCO / 16, FJ = TP / 16;
  static_assert(WCO * WP == NW && FI % 2 == 0 && FJ >= 1 && BCO % (8 * NW) == 0, "bad tile");
  constexpr int NIW = BCO / (8 * NW);
  constexpr int WSLOT = BCO * kBK;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int HSLOT = HR * kBK;
  bf16_t* halo = lds;               // [2][HR][64]
  bf16_t* wts = lds + 2 * HSLOT;    // [3][BCO][64]
  float* prm = reinterpret_cast<float*>(wts + 3 * WSLOT);
  float* pprm = prm + 3 * BCO;      // PRO: [3][C] per input channel scale / shift / rscale
  // one 128-byte zero row after the parameters (host: halo_lds_bytes): the fragment source of taps
  // that fall outside the image
  bf16_t* zrow = reinterpret_cast<bf16_t*>(pprm + (PRO ? 3 * g.C : 0));
  static_assert(sizeof(bf16x8) == 16, "zero row store");
  if (threadIdx.x < 8) *reinterpret_cast<bf16x8*>(zrow + 8 * threadIdx.x) = bf16x8{};

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rho = lane & 15, lg = lane >> 4;
  const int wco0 = (wave % WCO) * TCO, wp0 = (wave / WCO) * TP;
  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ct = rid % g.ctiles, grp = rid / g.ctiles;
  // work units are 64-channel blocks (9 taps each: the halo is staged once per unit)
  const Plan plan = make_plan(grp, g.groups, g.ptiles, g.cblk, SK);
  const int items = 9 * plan_units(plan, g.cblk);  // tap fastest
  const int64_t Ktot = static_cast<int64_t>(g.ksteps) * kBK;
  if (EPI >= kEpiBnbM) {
    for (int t = threadIdx.x; t < BCO; t += NT) {
      const int co = ct * BCO + t;
      prm[t] = ea.mean[co];
      prm[BCO + t] = EPI == kEpiBnbR ? ea.scale[co] : 0.f;
      prm[2 * BCO + t] = EPI == kEpiBnbR ? ea.shift[co] : 0.f;
    }
  }
  if (PRO) {
    for (int t = threadIdx.x; t < g.C; t += NT) {
      pprm[t] = pa.scale[t];
      pprm[g.C + t] = pa.shift[t];
      pprm[2 * g.C + t] = PRO == 2 ? pa.rscale[t] : 0.f;
    }
    // the first flush() (item 0's halo, before the main loop's first barrier) reads channels
    // staged by other waves (threads t < C: with C = 64 wave 0 alone writes every parameter)
  }
  __syncthreads();  // prologue parameters and the zero row
  const int prow = lane >> 3, slot = lane & 7;
  const bf16_t* wsrc[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int co = 8 * (wave + NW * i) + prow;
    wsrc[i] = w + (static_cast<int64_t>(ct) * BCO + co) * Ktot + ((slot ^ swz(co)) << 3);
  }
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_rows) + (slot << 3);

  // PRO: the pending register-staged halo (rows 8 * wave + 8 * NW * i + prow, channel chunk slot)
  constexpr int MAXR = PRO ? kHaloProRows : 1;
  bf16x8 hx[MAXR], hr[MAXR];
  bf16_t* p_hs = nullptr;
  int64_t p_f0 = 0;
  int p_cb = 0;
  bool p_pending = false;
  auto flush = [&]() __attribute__((always_inline)) {
    if (!PRO || !p_pending) return;
    p_pending = false;
    const float* sc = pprm + p_cb * kBK + (slot << 3);
    float fs[8], fh[8], fr[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fs[e] = sc[e];
      fh[e] = sc[g.C + e];
      fr[e] = PRO == 2 ? sc[2 * g.C + e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < MAXR; ++i) {
      if (8 * wave + 8 * NW * i >= HR) break;  // wave-uniform (HR % 8 == 0)
      const int k = 8 * wave + 8 * NW * i + prow;
      const int64_t f = p_f0 + k;
      const bool valid = f >= 0 && f < g.M;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = PRO == 2 ? fs[e] * bf2f(hx[i].v[e]) + fr[e] * bf2f(hr[i].v[e]) + fh[e]
                                 : fmaxf(bf2f(hx[i].v[e]) * fs[e] + fh[e], 0.f);
        v[e] = valid ? t : 0.f;
      }
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const u16v2_t pk = f2bf2(v[e], v[e + 1]);
        o.v[e] = pk[0]; o.v[e + 1] = pk[1];
      }
      *reinterpret_cast<bf16x8*>(p_hs + k * kBK + ((slot ^ (k & 7)) << 3)) = o;
      if (pa.aout != nullptr && ct == 0 && valid && k >= g.W + 1 && k < g.W + 1 + BP)
        *reinterpret_cast<bf16x8*>(pa.aout + f * g.C + p_cb * kBK + (slot << 3)) = o;
    }
  };

  // load side: segment cursor (tile, channel-block range), tap, running halo count (slot parity)
  Cursor lc{0, 0, 0, 0, 0};
  seg_enter(lc, plan, g.cblk);
  int l_tap = 0, l_halo = 0;
  auto issue = [&](int wslot) __attribute__((always_inline)) {
    const int l_cb = lc.k;
    if (l_tap == 0) {  // stage this tile's halo for channel block l_cb
      const int64_t f0 = static_cast<int64_t>(lc.pt) * BP - g.W - 1;
      bf16_t* hs = halo + (l_halo & 1) * HSLOT;
      if (PRO) {  // registers now, LDS at the next flush()
#pragma unroll
        for (int i = 0; i < MAXR; ++i) {
          const int k = 8 * wave + 8 * NW * i + prow;
          const int64_t f = f0 + k;
          const int64_t fc = (k < HR && f >= 0 && f < g.M) ? f : 0;  // clamped: zeroed at flush
          const int64_t off = fc * g.C + l_cb * kBK + (slot << 3);
          hx[i] = *reinterpret_cast<const bf16x8*>(x + off);
          if (PRO == 2) hr[i] = *reinterpret_cast<const bf16x8*>(pa.res + off);
        }
        p_hs = hs;
        p_f0 = f0;
        p_cb = l_cb;
        p_pending = true;
      } else {
        for (int k0 = 8 * wave; k0 < HR; k0 += 8 * NW) {
          const int k = k0 + prow;
          const int64_t f = f0 + k;
          const bf16_t* src = (f >= 0 && f < g.M) ? x + f * g.C + l_cb * kBK + ((slot ^ (k & 7)) << 3) : zero;
          dma16(src, hs + k0 * kBK);
        }
      }
      ++l_halo;
    }
    bf16_t* ws = wts + wslot * WSLOT;
    const int koff = l_tap * g.C + l_cb * kBK;
#pragma unroll
    for (int i = 0; i < NIW; ++i) dma16(wsrc[i] + koff, ws + 8 * (wave + NW * i) * kBK);
    if (++l_tap == 9) {
      l_tap = 0;
      if (++lc.k == lc.kend) seg_next(lc, plan, g.cblk);
    }
  };

  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float st_s[FI / 2][8], st_q[FI / 2][8];
  if (SUMS) {
#pragma unroll
    for (int q = 0; q < FI / 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) { st_s[q][e] = 0.f; st_q[q][e] = 0.f; }
  }
  uint32_t vm[FJ];  // per fragment pixel: bit 3r+s = tap (r, s) inside the image

  if (items > 0) issue(0);
  if (PRO) {  // item 0's halo goes to LDS before the loop's first barrier
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    flush();
  }
  if (items > 1) issue(1);
  Cursor cc{0, 0, 0, 0, 0};
  seg_enter(cc, plan, g.cblk);
  int c_halo = 0;
  bool c_first = true;  // first unit of a segment: per-pixel tap masks of its tile

  // Lane-constant LDS byte addresses, computed once: the weight fragments of ring slot 0 (the slot
  // of a tap is compile-time below, so it lands in the ds_read offset field), the halo fragment rows
  // (the halo slot and the tap's row shift are wave-uniform per tap: one v_add per fragment), and the
  // zero row an out-of-image tap reads instead of selecting zeros into the fragment dwords.
  const char* lds_c = reinterpret_cast<const char*>(lds);
  const uint32_t wts_b = static_cast<uint32_t>(reinterpret_cast<const char*>(wts) - lds_c);
  const uint32_t zrow_b = static_cast<uint32_t>(reinterpret_cast<const char*>(zrow) - lds_c);
  uint32_t aoff[2][FI], zoff[2];
  int brow[FJ];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wco0 + a_row(i, rho);
      aoff[kk][i] = wts_b + 2u * static_cast<uint32_t>(row * kBK + (((kk * 4 + lg) ^ swz(row)) << 3));
    }
    zoff[kk] = zrow_b + (static_cast<uint32_t>(kk * 4 + lg) << 4);
  }
#pragma unroll
  for (int j = 0; j < FJ; ++j) brow[j] = wp0 + 16 * j + rho;
  // LDS byte offsets from the dynamic LDS base (the halo ring starts there)
  auto ld_s8 = [&](uint32_t off) __attribute__((always_inline)) {
    return *reinterpret_cast<const s8*>(lds_c + off);
  };

  // One item = one tap of one 64-channel unit; items come in units of 9 taps, so the weight ring
  // slot (item % 3) and the tap's (r, s) are compile-time in the 9-way unrolled unit body.
  auto tap = [&](auto TT, int it, int hrow0) __attribute__((always_inline)) {
    constexpr int T = decltype(TT)::value;
    // the next item's DMAs may stay in flight (a halo issued with it is over-waited: correct;
    // a register-staged halo (PRO) is waited for here and written to LDS by flush() below)
    if (PRO) {
      if (it + 1 < items) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)" :: "n"(NIW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    } else {
      if (it + 1 < items) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIW) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    flush();  // the halo of item it+1 (slot free: last read two units ago)
    if (it + 2 < items) issue((T + 2) % 3);
    const int rb = hrow0 + (T / 3) * g.W + (T % 3);  // wave-uniform row shift of this tap
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      s8 a[FI], b[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) a[i] = ld_s8(aoff[kk][i] + 2u * (T % 3) * WSLOT);
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int row = brow[j] + rb;
        const uint32_t hb = 2u * static_cast<uint32_t>(row * kBK + (((kk * 4 + lg) ^ (row & 7)) << 3));
        b[j] = ld_s8(((vm[j] >> T) & 1u) ? hb : zoff[kk]);
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
  };

  for (int it0 = 0; it0 < items; it0 += 9) {
    const int64_t pt = cc.pt;
    if (c_first) {
      c_first = false;
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int64_t m = pt * BP + wp0 + 16 * j + rho;
        uint32_t bits = 0;
        if (m < g.M) {
          const int64_t hw = m / g.W;
          const int ww = static_cast<int>(m - hw * g.W);
          const int hh = static_cast<int>(hw % g.H);
#pragma unroll
          for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int s2 = 0; s2 < 3; ++s2) {
              const bool ok = hh + r - 1 >= 0 && hh + r - 1 < g.H && ww + s2 - 1 >= 0 && ww + s2 - 1 < g.W;
              bits |= (ok ? 1u : 0u) << (3 * r + s2);
            }
        }
        vm[j] = bits;
      }
    }
    const int hrow0 = (c_halo & 1) * HR;  // halo slot as a row offset (HR % 8 == 0: same swizzle)
    tap(IC<0>{}, it0, hrow0);
    tap(IC<1>{}, it0 + 1, hrow0);
    tap(IC<2>{}, it0 + 2, hrow0);
    tap(IC<3>{}, it0 + 3, hrow0);
    tap(IC<4>{}, it0 + 4, hrow0);
    tap(IC<5>{}, it0 + 5, hrow0);
    tap(IC<6>{}, it0 + 6, hrow0);
    tap(IC<7>{}, it0 + 7, hrow0);
    tap(IC<8>{}, it0 + 8, hrow0);
    ++c_halo;
    if (++cc.k == cc.kend) {
      const bool whole = !SK || cc.run == 0 || (cc.run == 2 && cc.kend == g.cblk);
      if (!whole) {
        sk_publish<FI, FJ, NT>(acc, sk, rid);
      } else {
        if (SK && cc.run == 2) sk_gather<FI, FJ, NT>(acc, sk, plan, cc.pt, g.cblk, g.ctiles, ct);
        epi_store_tile<BCO, BP, FI, FJ, EPI>(acc, pt, ct, wco0, wp0, lg, rho, g, ea, prm, y, st_s, st_q);
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
      seg_next(cc, plan, g.cblk);
      c_first = true;
    }
  }
  if (SUMS) epi_flush_sums<BCO, FI, WCO, NW>(st_s, st_q, lds, wave, lg, rho, wco0, grp, ct, g.K, part);
}

// =============================================================================== weight gradient
// dW[co][k] = sum_p dY[p][co] . im2col[p][k], k = (r, s, c): rows co, columns k, reduction over
// the output pixels p (the MFMA K dimension).  Both operands are pixel-major in memory, so the
// LDS images keep pixel rows ([64 px][64 ch] blocks, 128-byte rows, filled by the same LDS-DMA
// gather as the forward) and the fragments are read with the hardware transpose
// ds_read_b64_tr_b16: lane c of a 16-lane group receives channel col0 + c of 4 pixel rows.
// Swizzle for these reads: chunk c of row r at slot c ^ (2 * ((r >> 1) & 3)) -- conflict-free per
// 32-lane half for the 4-row x 32-byte blocks the transposed reads take.
// Fragment k-order: elements 0..3 = pixels r0..r0+3, 4..7 = r0+16..r0+19 (r0 = 32 kk + 4 g) for
// both operands, so the permuted pixel order cancels in the product.
// The pixel range is split over `splits` blocks per output tile; each block writes an fp32 partial
// tile and wgrad_finalize_kernel sums the splits in a fixed order (deterministic).

__device__ __forceinline__ int swz_tr(int row) { return 2 * ((row >> 1) & 3); }

struct WGeo {
  int H, W, C, OH, OW, K, R, S, stride, pad;
  int M;          // pixels (output positions)
  int cotiles, ktiles, splits, chunk;  // chunk: pixels per split (multiple of 64)
  int kblk_per_tap;                    // C / BKC
  FastDiv dOHW, dOW;
};

template <int BCO, int BKC, int WCO, int NST = 2, int NW = 4>
__global__ void __launch_bounds__(64 * NW, 2)
conv_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ part, WGeo g) {
  constexpr int WK = NW / WCO;
  constexpr int TCO = BCO / WCO, TK = BKC / WK;
  constexpr int FI = TCO / 16, FJ = TK / 16;
  static_assert(WCO * WK == NW && FI >= 1 && FJ >= 1 && BCO % 64 == 0 && BKC % 64 == 0, "bad tile");
  constexpr int ACB = BCO / 64, BCB = BKC / 64;   // 64-channel blocks per operand
  constexpr int BLK = 64 * 64;                    // elements per [64 px][64 ch] block
  constexpr int STAGE = (ACB + BCB) * BLK;
  static_assert((ACB + BCB) * 8 % NW == 0, "DMA pieces per wave");
  constexpr int NI = (ACB + BCB) * 8 / NW;        // DMA instructions per wave per stage
  static_assert(NST == 2 || NST == 3, "ring depth");
  constexpr int NLW = NI;  // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) bf16_t lds[NST * STAGE];

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c16 = lane & 15, lg = lane >> 4;
  const int wco0 = (wave % WCO) * TCO, wk0 = (wave / WCO) * TK;

  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ntile = g.cotiles * g.ktiles;
  const int tile = rid % ntile, split = rid / ntile;
  const int cot = tile % g.cotiles, kt = tile / g.cotiles;
  const int tap = kt / g.kblk_per_tap;
  const int ci0 = (kt - tap * g.kblk_per_tap) * BKC;
  const int tr = tap / g.S, ts = tap - (tap / g.S) * g.S;
  const int p_begin = split * g.chunk;
  int p_end = p_begin + g.chunk;
  if (p_end > g.M) p_end = g.M;
  const int items = p_end > p_begin ? (p_end - p_begin + 63) / 64 : 0;
  const bool plain = g.R == 1 && g.S == 1 && g.stride == 1 && g.pad == 0;

  const int prow = lane >> 3, slot = lane & 7;
  auto issue = [&](int stage, int it) {
    bf16_t* base = lds + stage * STAGE;
    const int p0 = p_begin + it * 64;
#pragma unroll
    for (int n = 0; n < NI; ++n) {
      const int ins = wave + NW * n;              // 0 .. (ACB+BCB)*8-1
      const int blk = ins >> 3, row = 8 * (ins & 7) + prow;
      const int p = p0 + row;
      const int chunk = slot ^ swz_tr(row);
      const bf16_t* src = reinterpret_cast<const bf16_t*>(g_zero_rows) + (slot << 3);
      if (p < p_end) {
        if (blk < ACB) {
          src = dy + static_cast<int64_t>(p) * g.K + cot * BCO + blk * 64 + (chunk << 3);
        } else if (plain) {
          src = x + static_cast<int64_t>(p) * g.C + ci0 + (blk - ACB) * 64 + (chunk << 3);
        } else {
          const int nimg = static_cast<int>(g.dOHW.div(static_cast<uint32_t>(p)));
          const int rem = p - nimg * g.OH * g.OW;
          const int oh = static_cast<int>(g.dOW.div(static_cast<uint32_t>(rem)));
          const int ow = rem - oh * g.OW;
          const int ih = oh * g.stride - g.pad + tr, iw = ow * g.stride - g.pad + ts;
          if (static_cast<unsigned>(ih) < static_cast<unsigned>(g.H) && static_cast<unsigned>(iw) < static_cast<unsigned>(g.W))
            src = x + ((static_cast<int64_t>(nimg) * g.H + ih) * g.W + iw) * g.C + ci0 + (blk - ACB) * 64 + (chunk << 3);
        }
      }
      dma16(src, base + blk * BLK + 8 * (ins & 7) * 64);
    }
  };

  // transposed fragment: channels col0..col0+15 (lane c16 -> col0 + c16) of pixel rows r0..r0+3
  // and r0+16..r0+19 of a [64 px][64 ch] block image
  auto tr_frag = [&](const bf16_t* blkimg, int col0, int r0) {
    const int q = c16 >> 2, pp = c16 & 3;
    const int col = col0 + 4 * pp, chunk = col >> 3, within = col & 7;
    const int ra = r0 + q, rb = r0 + 16 + q;
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(blkimg + ra * 64 + ((chunk ^ swz_tr(ra)) << 3) + within));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(blkimg + rb * 64 + ((chunk ^ swz_tr(rb)) << 3) + within));
    s8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  };

  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int s0 = 0; s0 < NST - 1; ++s0)
    if (s0 < items) issue(s0, s0);
  for (int it = 0; it < items; ++it) {
    // retire slot it; with the 3-slot ring the next slot's DMAs stay in flight (counted wait,
    // raw barrier: a __syncthreads() fence would drain the ring)
    if (NST == 3 && it + 1 < items) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NLW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (it + NST - 1 < items) issue((it + NST - 1) % NST, it + NST - 1);
    const bf16_t* sa = lds + (it % NST) * STAGE;
    const bf16_t* sb = sa + ACB * BLK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = 32 * kk + 4 * lg;
      s8 a[FI], b[FJ];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int col = wco0 + 16 * i;
        a[i] = tr_frag(sa + (col >> 6) * BLK, col & 63, r0);
      }
#pragma unroll
      for (int j = 0; j < FJ; ++j) {
        const int col = wk0 + 16 * j;
        b[j] = tr_frag(sb + (col >> 6) * BLK, col & 63, r0);
      }
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
  }
  // acc[i][j][r] = partial dW[co = cot*BCO + wco0 + 16i + 4lg + r][k = kt*BKC + wk0 + 16j + c16]
  const int64_t Ktot = static_cast<int64_t>(g.R) * g.S * g.C;
  float* dst = part + static_cast<int64_t>(split) * g.K * Ktot;
  const int64_t kcol0 = static_cast<int64_t>(tap) * g.C + ci0 + wk0;
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t co = static_cast<int64_t>(cot) * BCO + wco0 + 16 * i + 4 * lg + r;
        dst[co * Ktot + kcol0 + 16 * j + c16] = acc[i][j][r];
      }
}

// =========================================================== 3x3 / stride-1 halo weight gradient
// dW[co][r][s][c] = sum_p dY[p][co] * x[p + (r-1, s-1)][c].  The generic weight gradient above
// re-stages both operands for every (tap, channel block) column tile -- 9x the pixel traffic of a
// 3x3 layer, and per-row im2col arithmetic.  Here one block owns a (BCO output channels) x (64
// input channels) x (all 9 taps) tile and walks its pixel range once: per stage of 128 pixels it
// stages the dY rows and the input halo (the 128 + 2(W+1) + 2 surrounding rows) once, and the 9
// taps read the halo at row offsets r(W+1) + s.  Pixels are indexed on a zero-padded grid of
// (H+1) x (W+1) per image (one pad column, one pad row): every out-of-image neighbour of a real
// pixel lands on a pad position, which is staged as zeros, and pad positions carry zero dY -- so
// no per-element boundary masks are needed (the cost: (H+1)(W+1)/(HW) more MFMA work, 1.15x at
// 14x14, 1.04x at 56x56).  8 waves = 2 (output channels) x 4 (16 input channels each); fragments
// by hardware-transposed LDS reads as in conv_wgrad_kernel; the pixel range is split over blocks
// and the splits are summed by wgrad_finalize_kernel (deterministic).
constexpr int kHwPB = 128;  // padded pixels per stage

struct HWGeo {
  int H, W, C, K;
  int Mp;                          // N * (H + 1) * (W + 1)
  int HR;                          // halo rows per stage (multiple of 8)
  int cotiles, cblks, splits, chunk;
  FastDiv dImg, dRow;              // (H + 1) * (W + 1), W + 1
};

template <int BCO>
__global__ void __launch_bounds__(512, 2)
conv3x3_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ part,
                     HWGeo g) {
  constexpr int NW = 8;
  constexpr int WCO = 2;                      // waves along output channels (x 4 along input channels)
  constexpr int TCO = BCO / WCO, FI = TCO / 16;
  constexpr int ACB = BCO / 64;               // 64-channel blocks of the dY image
  constexpr int BLK = 64 * 64;
  constexpr int DYS = 2 * ACB * BLK;          // dY image: [2 pixel halves][ACB][64 px][64 ch]
  constexpr int NID = 2 * ACB * 8 / NW;       // dY DMA pieces per wave per stage
  static_assert(FI >= 1 && NID >= 1, "bad tile");
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int SE = DYS + g.HR * 64;             // elements per stage

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c16 = lane & 15, lg = lane >> 4;
  const int wco0 = (wave % WCO) * TCO, wc0 = (wave / WCO) * 16;

  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ntile = g.cotiles * g.cblks;
  const int tile = rid % ntile, split = rid / ntile;
  const int cot = tile % g.cotiles, cb = tile / g.cotiles;
  const int p_begin = split * g.chunk;
  const int p_end = min(p_begin + g.chunk, g.Mp);
  const int items = p_end > p_begin ? (p_end - p_begin + kHwPB - 1) / kHwPB : 0;
  const int W1 = g.W + 1;

  const int prow = lane >> 3, slot = lane & 7;
  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_rows) + (slot << 3);
  // padded index -> element offset of the pixel in an [N][H][W] image, or -1 for a pad position
  auto pix = [&](int q) -> int64_t {
    if (q < 0 || q >= g.Mp) return -1;
    const int n = static_cast<int>(g.dImg.div(static_cast<uint32_t>(q)));
    const int rem = q - n * (g.H + 1) * W1;
    const int h = static_cast<int>(g.dRow.div(static_cast<uint32_t>(rem)));
    const int w = rem - h * W1;
    if (h >= g.H || w >= g.W) return -1;
    return (static_cast<int64_t>(n) * g.H + h) * g.W + w;
  };
  auto issue = [&](int stage, int it) {
    bf16_t* base = lds + stage * SE;
    const int q0 = p_begin + it * kHwPB;
#pragma unroll
    for (int n = 0; n < NID; ++n) {
      const int ins = wave + NW * n;
      const int blk = ins >> 3, row = 8 * (ins & 7) + prow;
      const int pxb = blk / ACB, cob = blk - pxb * ACB;
      const int q = q0 + 64 * pxb + row;
      const int64_t e = q < p_end ? pix(q) : -1;
      const bf16_t* src = e >= 0 ? dy + e * g.K + cot * BCO + cob * 64 + ((slot ^ swz_tr(row)) << 3) : zero;
      dma16(src, base + blk * BLK + 8 * (ins & 7) * 64);
    }
    bf16_t* hx = base + DYS;
    for (int k0 = 8 * wave; k0 < g.HR; k0 += 8 * NW) {
      const int row = k0 + prow;
      const int64_t e = pix(q0 - W1 - 1 + row);
      const bf16_t* src = e >= 0 ? x + e * g.C + cb * 64 + ((slot ^ swz_tr(row)) << 3) : zero;
      dma16(src, hx + k0 * 64);
    }
  };
  // transposed fragment: channels col0 + c16 of rows r0..r0+3 and r0+16..r0+19 of a 64-wide image
  auto tr_frag = [&](const bf16_t* img, int col0, int r0) {
    const int q = c16 >> 2, pp = c16 & 3;
    const int col = col0 + 4 * pp, chunk = col >> 3, within = col & 7;
    const int ra = r0 + q, rb = r0 + 16 + q;
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(img + ra * 64 + ((chunk ^ swz_tr(ra)) << 3) + within));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lds_s4*)(img + rb * 64 + ((chunk ^ swz_tr(rb)) << 3) + within));
    s8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  };

  f4 acc[9][FI];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < FI; ++i) acc[t][i] = f4{0.f, 0.f, 0.f, 0.f};

  if (items > 0) issue(0, 0);
  for (int it = 0; it < items; ++it) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // stage it landed for every wave; stage it-1 is no longer read
    if (it + 1 < items) issue((it + 1) & 1, it + 1);
    const bf16_t* sd = lds + (it & 1) * SE;
    const bf16_t* sx = sd + DYS;
#pragma unroll
    for (int kk = 0; kk < kHwPB / 32; ++kk) {
      const int r0 = 32 * (kk & 1) + 4 * lg;  // row within the 64-pixel dY block
      s8 a[FI];
#pragma unroll
      for (int i = 0; i < FI; ++i) {
        const int col = wco0 + 16 * i;
        a[i] = tr_frag(sd + ((kk >> 1) * ACB + (col >> 6)) * BLK, col & 63, r0);
      }
      const int hr0 = 32 * kk + 4 * lg;       // halo row of pixel 32kk + 4lg for tap (0, 0)
      // the tap row offsets are re-derived here from an opaque copy of W + 1: hoisted out of the
      // pixel loop, the 72 per-(kk, tap) swizzled fragment addresses would spill the accumulators
      int w1 = W1;
      asm volatile("" : "+s"(w1));
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const s8 b = tr_frag(sx, wc0, hr0 + (t / 3) * w1 + (t % 3));
#pragma unroll
        for (int i = 0; i < FI; ++i) acc[t][i] = mfma(a[i], b, acc[t][i]);
        // keep the scheduler from hoisting every tap's fragment reads (9 live fragments spill
        // the 128-channel tile's 144 accumulator registers)
        if (t % 3 == 2) __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // acc[t][i][r] = partial dW[co = cot*BCO + wco0 + 16i + 4lg + r][tap t][c = cb*64 + wc0 + c16]
  const int64_t Ktot = 9LL * g.C;
  float* dst = part + static_cast<int64_t>(split) * g.K * Ktot;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t co = static_cast<int64_t>(cot) * BCO + wco0 + 16 * i + 4 * lg + r;
        dst[co * Ktot + t * g.C + cb * 64 + wc0 + c16] = acc[t][i][r];
      }
}

// ==================================================== fused 1x1 backward (dgrad + wgrad, one pass)
// The backward of z = conv1x1(a) when z's gradient arrives as a deferred BatchNorm backward
// (dy = A*dz + B*y + Cc, ops/conv.py _LazyBNGrad) and a = relu(bn(yb)) without a residual: the
// separate kernels read (dz, y) for the input gradient, write dy for the weight gradient, and read
// dy and a again there -- on ResNet-50's 56x56 layers that is ~1.6 GB of the ~3.9 GB the two
// passes move.  Here one persistent block per CU walks 64-pixel tiles once: it forms the dy tile
// in LDS from (dz, y), computes the input gradient dX = dy . W (MFMA, the BN-backward epilogue:
// dz' = dX * [yb * scale + shift > 0] and the (sum dz', sum dz' (yb - mean)) partials) and
// accumulates dW += dy^T . a in registers; each block's dW partial is summed by
// wgrad_finalize_kernel (deterministic).  K (dz channels) = 256, C (dX channels) = 64 -- the
// 64 -> 256 bottleneck conv of ResNet-50's first stage, where the traffic is largest.
template <int K, int C>
__global__ void __launch_bounds__(512, 2)
conv1x1_bwd_fused_kernel(const bf16_t* __restrict__ dz, const bf16_t* __restrict__ yk, const float* __restrict__ coef,
                         const bf16_t* __restrict__ wt, const bf16_t* __restrict__ a, const bf16_t* __restrict__ yb,
                         const float* __restrict__ bnp, int M, bf16_t* __restrict__ dzo, float* __restrict__ part,
                         float* __restrict__ wpart) {
  constexpr int NW = 8, NT = 512, BP = 64;
  constexpr int KB = K / 64;                    // 64-channel blocks of dy
  constexpr int BLK = 64 * 64;
  static_assert(C == 64 && K % 64 == 0 && KB * 8 % NW == 0, "tile");
  // dgrad: out^T[c][px] = Wt[c][k] . dy^T[k][px]; waves 2 (c) x 4 (px): TCO 32, TP 16
  constexpr int DWCO = 2, DTCO = C / DWCO, DFI = DTCO / 16;
  // wgrad: dW[k][c] = dy^T[k][px] . a[px][c]; waves 4 (k) x 2 (c): TK = K / 4, TC 32
  constexpr int WWK = 4, WTK = K / WWK, WFI = WTK / 16, WFJ = 2;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* wimg = lds;                           // [KB][64 c][64 k]     swz
  bf16_t* dyimg = wimg + KB * BLK;              // [2][KB][64 px][64 k] swz
  bf16_t* aimg = dyimg + 2 * KB * BLK;          // [2][64 px][64 c]     swz_tr
  float* cf = reinterpret_cast<float*>(aimg + 2 * BLK);  // [3][K] A, B, Cc
  float* prm = cf + 3 * K;                      // [3][C] mean, scale, shift of the BN on yb

  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int rho = lane & 15, lg = lane >> 4, c16 = rho;
  const int prow = lane >> 3, slot = lane & 7;
  const int tiles = (M + BP - 1) / BP;
  const int G = gridDim.x, b = blockIdx.x;

  // ---- once per block: weights (LDS-DMA, swizzled source), BN-backward coefficients, BN parameters
#pragma unroll
  for (int n = 0; n < KB * 8 / NW; ++n) {
    const int piece = wave + NW * n;            // (k-block, 8-row group)
    const int kb = piece >> 3, row = 8 * (piece & 7) + prow;
    dma16(wt + static_cast<int64_t>(row) * K + kb * 64 + ((slot ^ swz(row)) << 3), wimg + kb * BLK + 8 * (piece & 7) * 64);
  }
  for (int t = threadIdx.x; t < 3 * K; t += NT) cf[t] = coef[t];
  for (int t = threadIdx.x; t < 3 * C; t += NT) prm[t] = bnp[t];

  const bf16_t* zero = reinterpret_cast<const bf16_t*>(g_zero_rows) + (slot << 3);
  // per-thread staging of one dy tile: pass kb covers k-block kb, thread -> (pixel t >> 3, chunk t & 7)
  const int spx = threadIdx.x >> 3, sch = threadIdx.x & 7;
  bf16x8 rz[KB], ry[KB], ryb;
  const int dwco0 = (wave % DWCO) * DTCO, dwp0 = (wave / DWCO) * 16;
  auto load_tile = [&](int tl, int buf) {
    const int64_t p = static_cast<int64_t>(tl) * BP + spx;
    const int64_t pc = p < M ? p : 0;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const int64_t off = pc * K + kb * 64 + (sch << 3);
      rz[kb] = *reinterpret_cast<const bf16x8*>(dz + off);
      ry[kb] = *reinterpret_cast<const bf16x8*>(yk + off);
    }
    const int64_t pe = static_cast<int64_t>(tl) * BP + dwp0 + rho;  // this lane's epilogue pixel
    ryb = *reinterpret_cast<const bf16x8*>(yb + (pe < M ? pe : 0) * C + dwco0 + 8 * lg);
    const int arow = 8 * wave + prow;
    const int64_t pa = static_cast<int64_t>(tl) * BP + arow;
    dma16(pa < M ? a + pa * C + ((slot ^ swz_tr(arow)) << 3) : zero, aimg + buf * BLK + 8 * wave * 64);
  };
  auto store_tile = [&](int tl, int buf) {  // dy = A*dz + B*y + Cc -> LDS (zero past the last pixel)
    const bool ok = static_cast<int64_t>(tl) * BP + spx < M;
#pragma unroll
    for (int kb = 0; kb < KB; ++kb) {
      const float* A = cf + kb * 64 + (sch << 3);
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e)
        v[e] = ok ? A[e] * bf2f(rz[kb].v[e]) + A[K + e] * bf2f(ry[kb].v[e]) + A[2 * K + e] : 0.f;
      bf16x8 o;
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const u16v2_t pk = f2bf2(v[e], v[e + 1]);
        o.v[e] = pk[0]; o.v[e + 1] = pk[1];
      }
      *reinterpret_cast<bf16x8*>(dyimg + (buf * KB + kb) * BLK + spx * 64 + ((sch ^ swz(spx)) << 3)) = o;
    }
  };
  // transposed fragment of a 64-wide image (rows r0..r0+3, r0+16..r0+19; column col0 + c16) under
  // swizzle f: the dy image keeps the dgrad's b128 swizzle, the a image the wgrad's
  auto tr_frag = [&](const bf16_t* img, int col0, int r0, bool dy_swz) {
    const int q = c16 >> 2, pp = c16 & 3;
    const int col = col0 + 4 * pp, chunk = col >> 3, within = col & 7;
    const int ra = r0 + q, rb = r0 + 16 + q;
    const int fa = dy_swz ? swz(ra) : swz_tr(ra), fb = dy_swz ? swz(rb) : swz_tr(rb);
    const s4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + ra * 64 + ((chunk ^ fa) << 3) + within));
    const s4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(img + rb * 64 + ((chunk ^ fb) << 3) + within));
    s8 r;
    r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
    r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
    return r;
  };

  f4 accw[WFI][WFJ];
#pragma unroll
  for (int i = 0; i < WFI; ++i)
#pragma unroll
    for (int j = 0; j < WFJ; ++j) accw[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  float st_s[DFI / 2][8], st_q[DFI / 2][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { st_s[0][e] = 0.f; st_q[0][e] = 0.f; }
  const int wk0 = (wave % WWK) * WTK, wc0 = (wave / WWK) * 32;

  int buf = 0;
  if (b < tiles) load_tile(b, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();  // coefficients / BN parameters in LDS before the first dy tile is formed
  for (int tl = b; tl < tiles; tl += G) {
    store_tile(tl, buf);
    const bf16x8 yb_cur = ryb;
    __syncthreads();  // dy tile, a tile (DMA waited by every wave), weights, coefficients visible
    if (tl + G < tiles) load_tile(tl + G, buf ^ 1);
    const bf16_t* dyb = dyimg + buf * KB * BLK;
    // ---- input gradient for the 64 pixels x 64 channels, then the BN-backward epilogue
    f4 acc[DFI];
#pragma unroll
    for (int i = 0; i < DFI; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kb = 0; kb < KB; ++kb)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + lg;
        const int prw = dwp0 + rho;
        const s8 bv = *reinterpret_cast<const s8*>(dyb + kb * BLK + prw * 64 + ((chunk ^ swz(prw)) << 3));
#pragma unroll
        for (int i = 0; i < DFI; ++i) {
          const int row = dwco0 + a_row(i, rho);
          const s8 av = *reinterpret_cast<const s8*>(wimg + kb * BLK + row * 64 + ((chunk ^ swz(row)) << 3));
          acc[i] = mfma(av, bv, acc[i]);
        }
      }
    {  // lane: channels dwco0 + 8lg .. +7 of pixel tl*64 + dwp0 + rho
      const int64_t m = static_cast<int64_t>(tl) * BP + dwp0 + rho;
      const int cl = dwco0 + 8 * lg;
      float o[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { o[e] = acc[0][e]; o[4 + e] = acc[1][e]; }
      bf16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float yv = bf2f(yb_cur.v[e]);
        o[e] = yv * prm[C + cl + e] + prm[2 * C + cl + e] > 0.f ? o[e] : 0.f;  // recomputed ReLU
      }
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const u16v2_t pk = f2bf2(o[e], o[e + 1]);
        v.v[e] = pk[0]; v.v[e + 1] = pk[1];
      }
      if (m < M) {
        *reinterpret_cast<bf16x8*>(dzo + m * C + cl) = v;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float f = bf2f(v.v[e]);  // the stored (rounded) dz', as the apply pass reads it
          st_s[0][e] += f;
          st_q[0][e] += f * (bf2f(yb_cur.v[e]) - prm[cl + e]);
        }
      }
    }
    // ---- weight gradient: dW[k][c] += dy^T . a over the tile's 64 pixels
    const bf16_t* ab = aimg + buf * BLK;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = 32 * kk + 4 * lg;
      s8 av[WFI], bv[WFJ];
#pragma unroll
      for (int i = 0; i < WFI; ++i) {
        const int col = wk0 + 16 * i;
        av[i] = tr_frag(dyb + (col >> 6) * BLK, col & 63, r0, true);
      }
#pragma unroll
      for (int j = 0; j < WFJ; ++j) bv[j] = tr_frag(ab, wc0 + 16 * j, r0, false);
#pragma unroll
      for (int i = 0; i < WFI; ++i)
#pragma unroll
        for (int j = 0; j < WFJ; ++j) accw[i][j] = mfma(av[i], bv[j], accw[i][j]);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the next tile's loads / a-tile DMA
    buf ^= 1;
  }
  // per-block partials: BN-backward sums (part[b][2][C]) and dW (wpart[b][K][C])
  epi_flush_sums<C, DFI, DWCO, NW>(st_s, st_q, lds, wave, lg, rho, dwco0, b, 0, C, part);
  float* dst = wpart + static_cast<int64_t>(b) * K * C;
#pragma unroll
  for (int i = 0; i < WFI; ++i)
#pragma unroll
    for (int j = 0; j < WFJ; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        dst[static_cast<int64_t>(wk0 + 16 * i + 4 * lg + r) * C + wc0 + 16 * j + c16] = accw[i][j][r];
}

// dW = sum over splits of part[split][n].  A 256-thread block owns 64 float4 columns; its 4 waves
// each sum every 4th split with 4 independent accumulators (16 loads in flight per wave instead
// of one dependent chain per column), then the 4 wave sums are combined in LDS in a fixed order
// (deterministic).
template <typename WT>
__global__ void __launch_bounds__(256)
wgrad_finalize_kernel(const float* __restrict__ part, int splits, int64_t n, WT* __restrict__ dw) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (static_cast<int64_t>(blockIdx.x) * 64 + lane) * 4;
  float4 a[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) a[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n) {
    int k = wv;
    for (; k + 12 < splits; k += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float4 v = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k + 4 * u) * n + i);
        a[u].x += v.x; a[u].y += v.y; a[u].z += v.z; a[u].w += v.w;
      }
    }
    for (; k < splits; k += 4) {
      const float4 v = *reinterpret_cast<const float4*>(part + static_cast<int64_t>(k) * n + i);
      a[0].x += v.x; a[0].y += v.y; a[0].z += v.z; a[0].w += v.w;
    }
  }
  float4 s = a[0];
#pragma unroll
  for (int u = 1; u < 4; ++u) { s.x += a[u].x; s.y += a[u].y; s.z += a[u].z; s.w += a[u].w; }
  red[wv][lane] = s;
  __syncthreads();
  if (wv == 0 && i < n) {
#pragma unroll
    for (int u = 1; u < 4; ++u) { s.x += red[u][lane].x; s.y += red[u][lane].y; s.z += red[u][lane].z; s.w += red[u][lane].w; }
    Elem<WT>::st(dw, i, s.x);
    Elem<WT>::st(dw, i + 1, s.y);
    Elem<WT>::st(dw, i + 2, s.z);
    Elem<WT>::st(dw, i + 3, s.w);
  }
}


}  // namespace igemm
}  // namespace damd

using namespace damd;
using namespace damd::igemm;

namespace {

struct Cfg {
  int bco, bp, wco, nw, nst, sch, sk = 0;
};
// 0-2: 4 waves, 2-slot ring; 3-5: 8 waves, 3-slot ring (the tiles that won on some ResNet-50
// layer in profiles/conv_igemm_*; 128x256 / 256x128 with 4 waves spill and never won)
// nst = 0 marks the 3x3 halo kernel (stride-1 3x3 only)
constexpr Cfg kCfgs[] = {{64, 128, 1, 4, 2, 0},  {128, 128, 2, 4, 2, 0}, {64, 256, 1, 4, 2, 0},
                         {128, 256, 2, 8, 3, 0}, {64, 256, 1, 8, 3, 0},  {256, 128, 4, 8, 3, 0},
                         {128, 256, 2, 8, 0, 0}, {64, 256, 1, 8, 0, 0},  {128, 128, 2, 4, 0, 0},
                         {256, 128, 4, 8, 0, 0}, {128, 128, 2, 4, 2, 1}, {256, 128, 4, 8, 3, 1},
                         {128, 128, 2, 4, 2, 2}, {256, 128, 4, 8, 3, 2},
                         // 14-21: stream-K work split of the generic / halo tiles above (make_plan)
                         {128, 128, 2, 4, 2, 0, 1}, {256, 128, 4, 8, 3, 0, 1}, {128, 256, 2, 8, 3, 0, 1},
                         {64, 256, 1, 8, 3, 0, 1},  {128, 256, 2, 8, 0, 0, 1}, {64, 256, 1, 8, 0, 0, 1},
                         {128, 128, 2, 4, 0, 0, 1}, {256, 128, 4, 8, 0, 0, 1},
                         // 22-25: software-pipelined k-steps (SCH 3) of the generic tiles
                         {128, 128, 2, 4, 2, 3}, {256, 128, 4, 8, 3, 3}, {128, 256, 2, 8, 3, 3}, {64, 256, 1, 8, 3, 3}};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

int halo_rows(int bp, int W) { return (bp + 2 * W + 2 + 7) / 8 * 8; }

constexpr int kSkMaxBlocks = 4096;  // flag words the host keeps per device (damd_conv_sk_flag_words)

int halo_lds_bytes(const Cfg& c, int W, int C = 0) {  // C > 0: + the prologue's per-channel parameters
  return (2 * halo_rows(c.bp, W) * kBK + 3 * c.bco * kBK) * 2 + 3 * c.bco * 4 + 3 * C * 4 + 128;  // + zero row
}

int blocks_per_cu(const Cfg& c, int W = 0) {
  const int lds = c.nst == 0 ? halo_lds_bytes(c, W) : c.nst * (c.bco + c.bp) * kBK * 2;
  int occ = (160 * 1024) / lds;
  const int by_waves = 8 / c.nw;  // __launch_bounds__(64 * NW, 2): <= 2 waves per SIMD
  if (occ > by_waves) occ = by_waves;
  return occ < 1 ? 1 : occ;
}

}  // namespace

extern "C" {

int damd_conv_num_cfgs() { return kNumCfgs; }

// stream-K configs: fp32 slab workspace (floats) a launch needs, 0 for the others; the flag words
// (kSkMaxBlocks, then one time-out counter) are a zeroed per-device buffer the caller keeps.
int64_t damd_conv_sk_ws_floats(int K, int W, int cfg) {
  if (cfg < 0 || cfg >= kNumCfgs || !kCfgs[cfg].sk) return 0;
  const Cfg c = kCfgs[cfg];
  return static_cast<int64_t>(256 * blocks_per_cu(c, W)) * c.bco * c.bp;
}
int damd_conv_sk_flag_words() { return kSkMaxBlocks + 16; }
int damd_conv_cfg_is_sk(int cfg) { return cfg >= 0 && cfg < kNumCfgs && kCfgs[cfg].sk; }
int c_is_sk(int cfg) { return damd_conv_cfg_is_sk(cfg); }

// Heuristic default config for a layer: widest co tile the channel count allows.
int damd_conv_default_cfg(int K, int64_t M) {
  (void)M;
  if (K % 256 == 0) return 5;
  if (K % 128 == 0) return 1;
  return 2;
}

// W: input width (the halo configs stage BP + 2W + 2 pixel rows per channel block)
int damd_conv_supported(int C, int K, int R, int S, int stride, int pad, int W, int cfg) {
  if (cfg < 0 || cfg >= kNumCfgs) return 0;
  const Cfg c = kCfgs[cfg];
  if (!(C % kBK == 0 && C > 0 && K % c.bco == 0 && R * S <= 32)) return 0;
  if (c.sk) {  // every XCD slice holds whole sets of co tiles: K / BCO divides the blocks per XCD
    const int nblk = 256 * blocks_per_cu(c, W), ctiles = K / c.bco;
    if (nblk % 8 != 0 || (nblk / 8) % ctiles != 0 || nblk > kSkMaxBlocks) return 0;
  }
  if (c.nst == 0)
    return R == 3 && S == 3 && stride == 1 && pad == 1 && W >= 1 && halo_lds_bytes(c, W) <= kHaloMaxLds;
  return 1;
}

// DAMD_CONV_OVERSUB=k: k x the resident grid for the (non-stream-K) persistent configs, so blocks
// displaced by a concurrent kernel (a collective on another stream) leave work the others pick up
int conv_oversub() {
  static const int k = [] {
    const char* e = getenv("DAMD_CONV_OVERSUB");
    const int v = e != nullptr ? atoi(e) : 1;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  return k;
}

// groups (pixel-tile strides) for a config; also the leading dim of the stats partials
int damd_conv_groups(int64_t M, int K, int W, int cfg, int groups_override) {
  const Cfg c = kCfgs[cfg];
  const int64_t ptiles = (M + c.bp - 1) / c.bp;
  const int ctiles = K / c.bco;
  if (c.sk) return 256 * blocks_per_cu(c, W) / ctiles;  // the resident grid; plans may leave blocks idle
  int64_t groups = groups_override > 0 ? groups_override
                                       : (256LL * blocks_per_cu(c, W) + ctiles - 1) / ctiles * conv_oversub();
  if (groups > ptiles) groups = ptiles;
  if (groups < 1) groups = 1;
  return static_cast<int>(groups);
}

// x: [N, H, W, C] bf16; w: [K, R, S, C] bf16; y: [N, OH, OW, K] bf16;
// part: null or [groups][2][K] fp32 (epi 1: sum / sum of squares of y; epi 2, 3: see EpiArgs)
// epi: 0 none, 1 stats, 2 BN-backward with bit mask, 3 BN-backward with recomputed ReLU mask
int damd_conv_pro_supported(int C, int K, int R, int S, int stride, int pad, int cfg) {
  if (cfg < 0 || cfg >= kNumCfgs) return 0;
  const Cfg c = kCfgs[cfg];
  if (c.nst == 0)  // 3x3 halo kernel: the 64-channel / 256-pixel 8-wave tiles (register-staged halo)
    return c.bco == 64 && c.bp == 256 && c.nw == 8 && R == 3 && S == 3 && stride == 1 && pad == 1 &&
           damd_conv_supported(C, K, R, S, stride, pad, 1, cfg);
  return c.nst == 3 && (c.sch == 0 || c.sch == 3) && R == 1 && S == 1 && stride == 1 && pad == 0 &&
         damd_conv_supported(C, K, R, S, stride, pad, 1, cfg);
}

// W-dependent limit of the halo prologue (the register-staged halo of one channel block)
int damd_conv_pro_supported_w(int C, int K, int R, int S, int stride, int pad, int W, int cfg) {
  if (!damd_conv_pro_supported(C, K, R, S, stride, pad, cfg)) return 0;
  const Cfg c = kCfgs[cfg];
  if (c.nst != 0) return 1;
  return halo_rows(c.bp, W) <= kHaloProRows * 8 * c.nw && halo_lds_bytes(c, W, C) <= kHaloMaxLds;
}

// pro: the input is a = relu(x * p_scale + p_shift [+ p_res]) (ProArgs), 1x1 / stride 1 only
int damd_conv_fwd_launch(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K,
                         int R, int S, int stride, int pad, int cfg, int groups, hipStream_t st, int epi,
                         const void* d2, const void* yb, const uint8_t* mask, const float* mean,
                         const float* scale, const float* shift, int pro, const void* p_res, const float* p_scale,
                         const float* p_shift, const float* p_rscale, void* p_aout, uint8_t* p_mout, float* sk_ws,
                         int* sk_flags, int d2hw, int ophase) {
  if (!damd_conv_supported(C, K, R, S, stride, pad, W, cfg)) return -1;
  if (pro < 0 || pro > 2) return -4;
  if (pro && (!damd_conv_pro_supported_w(C, K, R, S, stride, pad, W, cfg) || p_scale == nullptr || p_shift == nullptr ||
              (pro == 2 && (p_rscale == nullptr || p_res == nullptr))))
    return -4;
  const ProArgs pa{static_cast<const bf16_t*>(p_res), p_scale, p_shift, p_rscale, static_cast<bf16_t*>(p_aout), p_mout};
  if (epi < 0 || epi > 3 || (epi != 0 && part == nullptr)) return -3;
  if (epi >= 2 && (yb == nullptr || mean == nullptr || (epi == 2 && mask == nullptr) ||
                   (epi == 3 && (scale == nullptr || shift == nullptr))))
    return -3;
  const Cfg c = kCfgs[cfg];
  Geo g;
  g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.stride = stride; g.pad = pad;
  g.OH = (H + 2 * pad - R) / stride + 1;
  g.OW = (W + 2 * pad - S) / stride + 1;
  if (ophase != 0) {  // one phase of a stride-2 input gradient: output grid = input grid (taps 0 / +1)
    if (stride != 1 || pad != 0 || R > 2 || S > 2 || epi != 0 || pro != 0 || c_is_sk(cfg)) return -6;
    g.OH = H;
    g.OW = W;
  }
  g.M = static_cast<int64_t>(N) * g.OH * g.OW;
  const int64_t xbytes = static_cast<int64_t>(N) * H * W * C * 2;
  if (xbytes >= 0xF0000000LL || static_cast<int64_t>(K) * R * S * C * 2 >= 0xF0000000LL) return -7;
  g.xbytes = static_cast<uint32_t>(xbytes);
  g.cblk = C / kBK;
  g.ksteps = R * S * g.cblk;
  g.ptiles = static_cast<int>((g.M + c.bp - 1) / c.bp);
  g.ctiles = K / c.bco;
  g.groups = groups;
  g.ost = ophase != 0 ? 2 : 0; g.oa = (ophase >> 1) & 1; g.ob = ophase & 1;
  g.OHf = ophase != 0 ? 2 * g.OH : g.OH; g.OWf = ophase != 0 ? 2 * g.OW : g.OW;
  if (c.sk && (sk_ws == nullptr || sk_flags == nullptr || groups != damd_conv_groups(g.M, K, W, cfg, 0))) return -5;
  const SkArgs ska{sk_ws, sk_flags, sk_flags + kSkMaxBlocks};
  EpiArgs ea{static_cast<const bf16_t*>(d2), static_cast<const bf16_t*>(yb), mask, mean, scale, shift, d2hw >> 16,
             d2hw & 0xffff};
  if (d2hw != 0 && (d2 == nullptr || epi < 2 || ea.d2h != (g.OH + 1) / 2 || ea.d2w != (g.OW + 1) / 2)) return -3;
  const dim3 grid(static_cast<unsigned>(g.ctiles * groups));
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(w);
  bf16_t* yp = static_cast<bf16_t*>(y);
#define L1(BCO, BP, WCO, NW, NST, E, SC, K_)                                                              \
  do {                                                                                                     \
    if constexpr (NST == 3 && (SC == 0 || SC == 3)) {                                                      \
      if (pro == 1) {                                                                                      \
        DAMD_LAUNCH((conv_fwd_kernel<BCO, BP, WCO, NW, NST, E, SC, 1, K_>), grid, dim3(64 * NW), 0, st, xp, wp, yp, part, g, ea, pa, ska); \
        break;                                                                                             \
      }                                                                                                    \
      if (pro == 2) {                                                                                      \
        DAMD_LAUNCH((conv_fwd_kernel<BCO, BP, WCO, NW, NST, E, SC, 2, K_>), grid, dim3(64 * NW), 0, st, xp, wp, yp, part, g, ea, pa, ska); \
        break;                                                                                             \
      }                                                                                                    \
    }                                                                                                      \
    DAMD_LAUNCH((conv_fwd_kernel<BCO, BP, WCO, NW, NST, E, SC, 0, K_>), grid, dim3(64 * NW), 0, st, xp, wp, yp, part, g, ea, pa, ska); \
  } while (0)
#define LSK(BCO, BP, WCO, NW, NST, SC, K_)                          \
  do {                                                              \
    switch (epi) {                                                  \
      case 0: L1(BCO, BP, WCO, NW, NST, kEpiNone, SC, K_); break;   \
      case 1: L1(BCO, BP, WCO, NW, NST, kEpiStats, SC, K_); break;  \
      case 2: L1(BCO, BP, WCO, NW, NST, kEpiBnbM, SC, K_); break;   \
      default: L1(BCO, BP, WCO, NW, NST, kEpiBnbR, SC, K_); break;  \
    }                                                               \
  } while (0)
#define LS(BCO, BP, WCO, NW, NST, SC) LSK(BCO, BP, WCO, NW, NST, SC, 0)
#define L(BCO, BP, WCO, NW, NST) LS(BCO, BP, WCO, NW, NST, 0)
  const int HR = halo_rows(c.bp, W);
  const int hlds = c.nst == 0 ? halo_lds_bytes(c, W, pro ? C : 0) : 0;
#define H2(BCO, BP, WCO, NW, E, K_, P_)                                                                      \
  do {                                                                                                       \
    auto* kfn = conv3x3_kernel<BCO, BP, WCO, NW, E, K_, P_>;                                                  \
    DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, hlds)); \
    DAMD_LAUNCH(kfn, grid, dim3(64 * NW), hlds, st, xp, wp, yp, part, g, ea, HR, ska, pa);  \
  } while (0)
#define H1(BCO, BP, WCO, NW, E, K_)                        \
  do {                                                     \
    if constexpr (BCO == 64 && BP == 256 && NW == 8) {     \
      if (pro == 1) { H2(BCO, BP, WCO, NW, E, K_, 1); break; } \
      if (pro == 2) { H2(BCO, BP, WCO, NW, E, K_, 2); break; } \
    }                                                      \
    H2(BCO, BP, WCO, NW, E, K_, 0);                        \
  } while (0)
#define HK(BCO, BP, WCO, NW, K_)                            \
  do {                                                      \
    switch (epi) {                                          \
      case 0: H1(BCO, BP, WCO, NW, kEpiNone, K_); break;    \
      case 1: H1(BCO, BP, WCO, NW, kEpiStats, K_); break;   \
      case 2: H1(BCO, BP, WCO, NW, kEpiBnbM, K_); break;    \
      default: H1(BCO, BP, WCO, NW, kEpiBnbR, K_); break;   \
    }                                                       \
  } while (0)
#define H(BCO, BP, WCO, NW) HK(BCO, BP, WCO, NW, 0)
  switch (cfg) {
    case 0: L(64, 128, 1, 4, 2); break;
    case 1: L(128, 128, 2, 4, 2); break;
    case 2: L(64, 256, 1, 4, 2); break;
    case 3: L(128, 256, 2, 8, 3); break;
    case 4: L(64, 256, 1, 8, 3); break;
    case 5: L(256, 128, 4, 8, 3); break;
    case 6: H(128, 256, 2, 8); break;
    case 7: H(64, 256, 1, 8); break;
    case 8: H(128, 128, 2, 4); break;
    case 9: H(256, 128, 4, 8); break;
    case 10: LS(128, 128, 2, 4, 2, 1); break;
    case 11: LS(256, 128, 4, 8, 3, 1); break;
    case 12: LS(128, 128, 2, 4, 2, 2); break;
    case 13: LS(256, 128, 4, 8, 3, 2); break;
    case 14: LSK(128, 128, 2, 4, 2, 0, 1); break;
    case 15: LSK(256, 128, 4, 8, 3, 0, 1); break;
    case 16: LSK(128, 256, 2, 8, 3, 0, 1); break;
    case 17: LSK(64, 256, 1, 8, 3, 0, 1); break;
    case 18: HK(128, 256, 2, 8, 1); break;
    case 19: HK(64, 256, 1, 8, 1); break;
    case 20: HK(128, 128, 2, 4, 1); break;
    case 21: HK(256, 128, 4, 8, 1); break;
    case 22: LS(128, 128, 2, 4, 2, 3); break;
    case 23: LS(256, 128, 4, 8, 3, 3); break;
    case 24: LS(128, 256, 2, 8, 3, 3); break;
    default: LS(64, 256, 1, 8, 3, 3); break;
  }
#undef L
#undef LS
#undef LSK
#undef L1
#undef H
#undef HK
#undef H1
#undef H2
  DAMD_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

// ---- weight gradient
namespace {
FastDiv make_fastdiv(uint32_t d) {
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  const uint64_t mul = ((1ull << 32) * ((1ull << l) - d)) / d + 1;
  return FastDiv{d, static_cast<uint32_t>(mul), l};
}
struct WCfg {
  int bco, bkc, wco, nst, nw = 4;
};
// 0: 128x128 (2x2 waves), 1: 64x128 (1x4), 2: 128x64 (4x1), 3: 64x64 (2x2: 32x32 per wave);
// 4-7: the same tiles with a 3-slot ring; 8-11: 8-wave blocks with 256-wide tiles (1 block per CU):
// each pixel chunk staged once feeds twice the MFMA work (the re-streaming of x / dY across
// co / channel tiles through L2 is what bounds the small-spatial layers)
constexpr WCfg kWCfgs[] = {{128, 128, 2, 2}, {64, 128, 1, 2}, {128, 64, 4, 2}, {64, 64, 2, 2},
                           {128, 128, 2, 3}, {64, 128, 1, 3}, {128, 64, 4, 3}, {64, 64, 2, 3},
                           {256, 256, 2, 2, 8}, {256, 128, 4, 3, 8}, {128, 256, 2, 3, 8}, {256, 128, 2, 3, 8}};
constexpr int kNumWCfgs = sizeof(kWCfgs) / sizeof(kWCfgs[0]);
}  // namespace

extern "C" {

int damd_wgrad_num_cfgs() { return kNumWCfgs; }

int damd_wgrad_supported(int C, int K, int cfg) {
  if (cfg < 0 || cfg >= kNumWCfgs) return 0;
  return C % kWCfgs[cfg].bkc == 0 && K % kWCfgs[cfg].bco == 0;
}

// number of pixel splits (leading dim of the fp32 partials)
int damd_wgrad_splits(int64_t M, int C, int K, int R, int S, int cfg, int splits_override) {
  const WCfg c = kWCfgs[cfg];
  const int64_t tiles = static_cast<int64_t>(K / c.bco) * (R * S * C / c.bkc);
  const int64_t target = 256 * (8 / c.nw);  // resident blocks: 2 per CU at 4 waves, 1 at 8
  int64_t splits = splits_override > 0 ? splits_override : (target + tiles - 1) / tiles;
  const int64_t max_splits = (M + 255) / 256;  // at least 4 k-steps per block
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return static_cast<int>(splits);
}

// x: [N, H, W, C]; dy: [N, OH, OW, K]; part: [splits][K][R*S*C] fp32 scratch; dw: [K][R][S][C]
int damd_wgrad_launch(const void* x, const void* dy, float* part, void* dw, int w_dtype, int N, int H, int W, int C,
                      int K, int R, int S, int stride, int pad, int cfg, int splits, hipStream_t st) {
  if (!damd_wgrad_supported(C, K, cfg)) return -1;
  const WCfg c = kWCfgs[cfg];
  WGeo g;
  g.H = H; g.W = W; g.C = C; g.K = K; g.R = R; g.S = S; g.stride = stride; g.pad = pad;
  g.OH = (H + 2 * pad - R) / stride + 1;
  g.OW = (W + 2 * pad - S) / stride + 1;
  const int64_t M = static_cast<int64_t>(N) * g.OH * g.OW;
  if (M >= (int64_t{1} << 31) - 4096) return -2;
  g.M = static_cast<int>(M);
  g.cotiles = K / c.bco;
  g.kblk_per_tap = C / c.bkc;
  g.ktiles = R * S * g.kblk_per_tap;
  g.splits = splits;
  g.chunk = static_cast<int>(((M + splits - 1) / splits + 63) / 64 * 64);
  g.dOHW = make_fastdiv(static_cast<uint32_t>(g.OH * g.OW));
  g.dOW = make_fastdiv(static_cast<uint32_t>(g.OW));
  const dim3 grid(static_cast<unsigned>(g.cotiles * g.ktiles * splits));
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* dp = static_cast<const bf16_t*>(dy);
#define WG(BCO, BKC, WCO, NST) \
  DAMD_LAUNCH((conv_wgrad_kernel<BCO, BKC, WCO, NST>), grid, dim3(kThreads), 0, st, xp, dp, part, g)
#define WG8(BCO, BKC, WCO, NST) \
  DAMD_LAUNCH((conv_wgrad_kernel<BCO, BKC, WCO, NST, 8>), grid, dim3(512), 0, st, xp, dp, part, g)
  switch (cfg) {
    case 0: WG(128, 128, 2, 2); break;
    case 1: WG(64, 128, 1, 2); break;
    case 2: WG(128, 64, 4, 2); break;
    case 3: WG(64, 64, 2, 2); break;
    case 4: WG(128, 128, 2, 3); break;
    case 5: WG(64, 128, 1, 3); break;
    case 6: WG(128, 64, 4, 3); break;
    case 7: WG(64, 64, 2, 3); break;
    case 8: WG8(256, 256, 2, 2); break;
    case 9: WG8(256, 128, 4, 3); break;
    case 10: WG8(128, 256, 2, 3); break;
    default: WG8(256, 128, 2, 3); break;
  }
#undef WG
#undef WG8
  const int64_t n = static_cast<int64_t>(K) * R * S * C;  // multiple of 4 (C % 64 == 0)
  const dim3 fg(static_cast<unsigned>((n / 4 + 63) / 64));
  if (w_dtype == 1)
    DAMD_LAUNCH(wgrad_finalize_kernel<bf16_t>, fg, dim3(256), 0, st, part, splits, n, static_cast<bf16_t*>(dw));
  else
    DAMD_LAUNCH(wgrad_finalize_kernel<float>, fg, dim3(256), 0, st, part, splits, n, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"


// ---- 3x3 halo weight gradient (cfg 0: 128 output channels per block, 1: 64; cfg 2 + k: conv3x3v2.hip's
// whole-row-tile kernel, its config k)
extern "C" int damd_v2w_num_cfgs();
extern "C" int damd_v2w_supported(int C, int K, int H, int W, int cfg);
extern "C" int damd_v2w_splits(int64_t N, int H, int C, int K, int cfg);
extern "C" int damd_v2w_launch(const void* x, const void* dy, float* part, int N, int H, int W, int C, int K, int cfg,
                               int splits, hipStream_t st);
namespace {
int hw_bco(int cfg) { return cfg == 0 ? 128 : 64; }
int hw_halo_rows(int W) { return (kHwPB + 2 * (W + 1) + 2 + 7) / 8 * 8; }
int hw_lds_bytes(int bco, int W) { return 2 * (2 * (bco / 64) * 64 * 64 + hw_halo_rows(W) * 64) * 2; }
int hw_launch(const void* x, const void* dy, float* part, int N, int H, int W, int C, int K, int cfg, int splits,
              hipStream_t st);
}  // namespace

extern "C" {

int damd_wgrad3x3_num_cfgs() { return 2 + damd_v2w_num_cfgs(); }

int damd_wgrad3x3_supported(int C, int K, int H, int W, int cfg) {
  if (cfg >= 2) return damd_v2w_supported(C, K, H, W, cfg - 2);
  if (cfg < 0 || cfg > 1) return 0;
  const int bco = hw_bco(cfg);
  return C % 64 == 0 && K % bco == 0 && W >= 1 && hw_lds_bytes(bco, W) <= 160 * 1024;
}

int damd_wgrad3x3_splits(int64_t N, int H, int W, int C, int K, int cfg, int splits_override) {
  if (cfg >= 2) return damd_v2w_splits(N, H, C, K, cfg - 2);
  const int64_t tiles = static_cast<int64_t>(K / hw_bco(cfg)) * (C / 64);
  int64_t splits = splits_override > 0 ? splits_override : (256 + tiles - 1) / tiles;
  const int64_t Mp = N * (H + 1) * (W + 1);
  const int64_t max_splits = (Mp + 4 * kHwPB - 1) / (4 * kHwPB);  // at least 4 stages per block
  if (splits > max_splits) splits = max_splits;
  if (splits < 1) splits = 1;
  return static_cast<int>(splits);
}

// x: [N, H, W, C]; dy: [N, H, W, K] (stride 1, pad 1); part: [splits][K][9*C] fp32; dw: [K][3][3][C]
int damd_wgrad3x3_launch(const void* x, const void* dy, float* part, void* dw, int w_dtype, int N, int H, int W,
                         int C, int K, int cfg, int splits, hipStream_t st) {
  if (!damd_wgrad3x3_supported(C, K, H, W, cfg)) return -1;
  if (cfg >= 2) {
    const int rc = damd_v2w_launch(x, dy, part, N, H, W, C, K, cfg - 2, splits, st);
    if (rc != 0) return rc;
  } else {
    const int rc = hw_launch(x, dy, part, N, H, W, C, K, cfg, splits, st);
    if (rc != 0) return rc;
  }
  const int64_t n = static_cast<int64_t>(K) * 9 * C;
  const dim3 fg(static_cast<unsigned>((n / 4 + 63) / 64));
  if (w_dtype == 1)
    DAMD_LAUNCH(wgrad_finalize_kernel<bf16_t>, fg, dim3(256), 0, st, part, splits, n, static_cast<bf16_t*>(dw));
  else
    DAMD_LAUNCH(wgrad_finalize_kernel<float>, fg, dim3(256), 0, st, part, splits, n, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"

namespace {
int hw_launch(const void* x, const void* dy, float* part, int N, int H, int W, int C, int K, int cfg, int splits,
              hipStream_t st) {
  const int64_t Mp = static_cast<int64_t>(N) * (H + 1) * (W + 1);
  if (Mp >= (int64_t{1} << 31) - 4096) return -2;
  const int bco = hw_bco(cfg);
  HWGeo g;
  g.H = H; g.W = W; g.C = C; g.K = K;
  g.Mp = static_cast<int>(Mp);
  g.HR = hw_halo_rows(W);
  g.cotiles = K / bco;
  g.cblks = C / 64;
  g.splits = splits;
  g.chunk = static_cast<int>(((Mp + splits - 1) / splits + kHwPB - 1) / kHwPB * kHwPB);
  g.dImg = make_fastdiv(static_cast<uint32_t>((H + 1) * (W + 1)));
  g.dRow = make_fastdiv(static_cast<uint32_t>(W + 1));
  const dim3 grid(static_cast<unsigned>(g.cotiles * g.cblks * splits));
  const int lds = hw_lds_bytes(bco, W);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* dp = static_cast<const bf16_t*>(dy);
  if (cfg == 0) {
    DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_wgrad_kernel<128>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DAMD_LAUNCH(conv3x3_wgrad_kernel<128>, grid, dim3(512), lds, st, xp, dp, part, g);
  } else {
    DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(conv3x3_wgrad_kernel<64>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, lds));
    DAMD_LAUNCH(conv3x3_wgrad_kernel<64>, grid, dim3(512), lds, st, xp, dp, part, g);
  }
  return 0;
}
}  // namespace


// ---- fused 1x1 backward (K = 256 -> C = 64)
extern "C" {

int damd_conv1x1_bwd_fused_supported(int K, int C) { return K == 256 && C == 64; }

int damd_conv1x1_bwd_fused_blocks(int64_t M) {
  const int64_t tiles = (M + 63) / 64;
  return static_cast<int>(tiles < 256 ? tiles : 256);
}

// dz, y: [M][K]; coef: [3][K]; wt: [C][K] (the conv weight transposed); a, yb: [M][C]; bnp: [3][C]
// (mean, scale, shift of the BN on yb); dzo: [M][C]; part: [G][2][C]; wpart: [G][K][C]; dw: [K][C]
int damd_conv1x1_bwd_fused_launch(const void* dz, const void* y, const float* coef, const void* wt, const void* a,
                                  const void* yb, const float* bnp, int64_t M, void* dzo, float* part, float* wpart,
                                  void* dw, int w_dtype, int K, int C, hipStream_t st) {
  if (!damd_conv1x1_bwd_fused_supported(K, C) || M <= 0 || M >= (int64_t{1} << 31) - 4096) return -1;
  const int G = damd_conv1x1_bwd_fused_blocks(M);
  constexpr int kK = 256, kC = 64;
  const int lds = ((kK / 64) * 4096 * 3 + 2 * 4096) * 2 + (3 * kK + 3 * kC) * 4;
  auto* kfn = conv1x1_bwd_fused_kernel<kK, kC>;
  DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  DAMD_LAUNCH(kfn, dim3(G), dim3(512), lds, st, static_cast<const bf16_t*>(dz), static_cast<const bf16_t*>(y),
                     coef, static_cast<const bf16_t*>(wt), static_cast<const bf16_t*>(a), static_cast<const bf16_t*>(yb),
                     bnp, static_cast<int>(M), static_cast<bf16_t*>(dzo), part, wpart);
  const int64_t n = static_cast<int64_t>(K) * C;
  const dim3 fg(static_cast<unsigned>((n / 4 + 63) / 64));
  if (w_dtype == 1)
    DAMD_LAUNCH(wgrad_finalize_kernel<bf16_t>, fg, dim3(256), 0, st, wpart, G, n, static_cast<bf16_t*>(dw));
  else
    DAMD_LAUNCH(wgrad_finalize_kernel<float>, fg, dim3(256), 0, st, wpart, G, n, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
  return 0;
}

}  // extern "C"
