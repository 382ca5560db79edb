// ResNet stem convolution (3 -> 64 channels, 7x7, stride 2, pad 3) for gfx950 / MI355X, bf16
// channels-last, forward + weight gradient.  (The image input never needs a gradient.)
//
// Why a dedicated kernel: with 3 input channels the generic implicit-GEMM solvers waste most
// of their K tile (K = 147) and re-gather the image per tile; at batch 512 MIOpen's best
// forward / weight-gradient solvers take ~0.7 ms each for 0.12 TFLOP.  Here the image rows a
// workgroup needs are staged in LDS ONCE per output row with the channel dimension padded
// 3 -> 4, which makes the im2col row of output pixel ow for a fixed kernel row kh the 32
// contiguous LDS elements starting at 8*ow (k' = 4*kw + ci, kw = 7 / ci = 3 are zero pad).  So
// one MFMA k-step (K = 32) is exactly one kernel row and every im2col operand is a single
// aligned 16-byte LDS read -- no gather.
//
// MFMA: v_mfma_f32_16x16x32_bf16.  A operand: lane l holds A[row l&15][k 8(l>>4)+j]; B operand:
// B[k 8(l>>4)+j][col l&15]; C/D: C[row 4(l>>4)+r][col l&15].
//
// Forward (one output row of 112 pixels x 64 channels per iteration, persistent grid): wave w
// owns output channels 16w..16w+15 and keeps their weights (7 k-steps) in registers for the
// whole kernel; C^T[co][pixel] = W[co][k] . im2col^T[k][pixel] puts 4 consecutive channels of
// one pixel in a lane, which are staged through LDS so the row leaves as 16-byte stores.
//
// Weight gradient: dW[co][k] = sum_pixels dY[pixel][co] . im2col[pixel][k].  The pixel sum is
// the MFMA K: dY^T comes from the staged dY row by a transposed LDS read (ds_read_tr16_b64)
// and im2col by a transposed read of the same padded image rows (rows = output pixels, row
// stride 8 elements); both use the same permuted pixel order, so the product is exact.  Each
// workgroup accumulates a 64 x (7 x 32) fp32 partial over its rows; a small kernel sums the
// partials in a fixed order (deterministic) and writes dW in the weight dtype.

#include "common.h"

namespace damd {
namespace stem {

typedef short s8 __attribute__((ext_vector_type(8)));
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

constexpr int kThreads = 256;  // 4 waves
constexpr int kCo = 64;
constexpr int kKH = 7;
constexpr int kMaxOW = 112;             // output row <= 7 pixel tiles
constexpr int kPix = 128;               // pixels per row padded to 4 MFMA k-steps (wgrad)
constexpr int kImgPix = 2 * kPix + 8;   // staged image pixels per row: iw + 3 in [0, 264)
constexpr int kRowE = kImgPix * 4 + 8;  // elements per staged image row (+8: bank spread)
constexpr int kOutRS = kCo + 8;         // staged output / dY row stride (elements)
constexpr int kPartCols = kKH * 32;     // partial dW columns per output channel (kh, k')

__device__ __forceinline__ f4 mfma(s8 a, s8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}

__device__ __forceinline__ s4 tr_read(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(p));
}

// transposed operand: lane c of a 16-lane group gets column col0 + c of rows r0+{0..3}
// (elements 0..3) and r1+{0..3} (elements 4..7) of a row-major LDS image
__device__ __forceinline__ s8 tr_pair(const bf16_t* img, int stride, int r0, int r1, int col0, int c) {
  const int q = c >> 2, p = c & 3;
  const s4 lo = tr_read(img + (r0 + q) * stride + col0 + 4 * p);
  const s4 hi = tr_read(img + (r1 + q) * stride + col0 + 4 * p);
  s8 r;
  r[0] = lo[0]; r[1] = lo[1]; r[2] = lo[2]; r[3] = lo[3];
  r[4] = hi[0]; r[5] = hi[1]; r[6] = hi[2]; r[7] = hi[3];
  return r;
}

// Workgroup barrier for LDS hand-offs.  __syncthreads()'s release fence waits for every
// outstanding global access (vmcnt(0)), which would expose the register prefetch of the next
// row's image (and dY / pooled rows) at every row; only this wave's LDS accesses need to be done.
// The "memory" clobbers keep the compiler from moving LDS accesses across the barrier.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Wait for every outstanding vector-memory load (s_waitcnt vmcnt(0), as the builtin the
// compiler's wait-count pass understands).  Used once after the prologue loads (weights, BN
// coefficients): without it the pass keeps their first-iteration waits inside the row loop,
// where in steady state they wait for the just-issued prefetch of the next row instead.
__device__ __forceinline__ void drain_vm() { __builtin_amdgcn_s_waitcnt(0x0F70); }

struct Geo {
  int H, W, OH, OW;
};

// Zero the staged image once: the pad columns (iw < 0, iw >= W) are never written again.
__device__ __forceinline__ void zero_image(bf16_t* img) {
  for (int i = threadIdx.x; i < kKH * kRowE / 8; i += kThreads)
    reinterpret_cast<uint4*>(img)[i] = make_uint4(0, 0, 0, 0);
}

// Image rows ih = 2*oh - 3 + kh (kh = 0..6) of image n, 4 pixels (24 bytes) per item, at most
// kImgItems items per thread (W <= 224).  Loaded into registers one row ahead (the global
// loads of row i+1 are in flight while row i computes), then stored into LDS with channels
// padded 3 -> 4 at LDS pixel index iw + 3.  Rows outside the image are zero.
constexpr int kImgItems = 2;
struct ImgRegs {
  uint2 v[kImgItems][3];
};

__device__ __forceinline__ void load_image(const bf16_t* __restrict__ x, ImgRegs& r, int64_t n, int oh,
                                           const Geo& g) {
  const int groups = g.W / 4;
#pragma unroll
  for (int i = 0; i < kImgItems; ++i) {
    const int it = threadIdx.x + i * kThreads;
    const int kh = it / groups, q = it - kh * groups;
    const int ih = 2 * oh - 3 + kh;
    r.v[i][0] = r.v[i][1] = r.v[i][2] = make_uint2(0, 0);
    if (kh < kKH && ih >= 0 && ih < g.H) {
      const uint2* src = reinterpret_cast<const uint2*>(x + ((n * g.H + ih) * g.W + 4 * q) * 3);
      r.v[i][0] = src[0]; r.v[i][1] = src[1]; r.v[i][2] = src[2];
    }
  }
}

__device__ __forceinline__ void store_image(const ImgRegs& r, bf16_t* img, const Geo& g) {
  const int groups = g.W / 4;
#pragma unroll
  for (int i = 0; i < kImgItems; ++i) {
    const int it = threadIdx.x + i * kThreads;
    const int kh = it / groups, q = it - kh * groups;
    if (kh < kKH) {
      const uint2 v0 = r.v[i][0], v1 = r.v[i][1], v2 = r.v[i][2];
      // 12 bf16 = pixels (a0 a1 a2)(b0 b1 b2)(c0 c1 c2)(d0 d1 d2) -> 4 x (r g b 0)
      uint2* dst = reinterpret_cast<uint2*>(img + kh * kRowE + (4 * q + 3) * 4);
      dst[0] = make_uint2(v0.x, v0.y & 0xFFFFu);
      dst[1] = make_uint2((v0.y >> 16) | (v1.x << 16), v1.x >> 16);
      dst[2] = make_uint2(v1.y, v2.x & 0xFFFFu);
      dst[3] = make_uint2((v2.x >> 16) | (v2.y << 16), v2.y >> 16);
    }
  }
}

// One conv output row: acc[t][r] = y[co = 16*wave + 4*grp + r][pixel 16t + c].  The B fragments
// of kernel row kh + 1 are read while kh's MFMAs run (a read-then-use per MFMA leaves each MFMA
// waiting for its LDS read).  The forward and the fused backward's recompute share this exact
// accumulation order, so the recomputed outputs are bit-identical.
template <int TILES, bool DB = true>
__device__ __forceinline__ void conv_row(const bf16_t* img, const s8 (&wa)[kKH], int grp, int c, f4 (&acc)[TILES]) {
#pragma unroll
  for (int t = 0; t < TILES; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  s8 b[DB ? 2 : 1][TILES];
#pragma unroll
  for (int t = 0; t < TILES; ++t) b[0][t] = *reinterpret_cast<const s8*>(img + 8 * grp + 8 * (16 * t + c));
#pragma unroll
  for (int kh = 0; kh < kKH; ++kh) {
    if (DB && kh + 1 < kKH) {
#pragma unroll
      for (int t = 0; t < TILES; ++t)
        b[(kh + 1) & (DB ? 1 : 0)][t] = *reinterpret_cast<const s8*>(img + (kh + 1) * kRowE + 8 * grp + 8 * (16 * t + c));
    }
#pragma unroll
    for (int t = 0; t < TILES; ++t) acc[t] = mfma(wa[kh], b[DB ? (kh & 1) : 0][t], acc[t]);
    if (!DB && kh + 1 < kKH) {  // single-buffered (register budget): the next row's reads after these MFMAs
#pragma unroll
      for (int t = 0; t < TILES; ++t)
        b[0][t] = *reinterpret_cast<const s8*>(img + (kh + 1) * kRowE + 8 * grp + 8 * (16 * t + c));
    }
  }
}


// wk: [64][7][32] bf16 weight image (k' = 4*kw + ci, zero where kw = 7 or ci = 3; built by the
// host wrapper); y: [N][OH][OW][64] bf16, OW = 16 * TILES.  With `part` the kernel also emits
// the following BatchNorm's batch statistics: part[block][0|1][64] = (sum y, sum y^2) of the
// bf16-rounded outputs it wrote (pilot 0, consumed by bn_finalize_kernel with xbase = null),
// which saves the BN statistics pass over the 112x112x64 activation.
template <int TILES>
__global__ void __launch_bounds__(kThreads)
stem_conv_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wk, bf16_t* __restrict__ y,
                     float* __restrict__ part, int64_t rows, Geo g) {
  __shared__ __attribute__((aligned(16))) bf16_t img[kKH * kRowE];
  __shared__ __attribute__((aligned(16))) bf16_t outs[kMaxOW * kOutRS];
  const int wave = threadIdx.x / 64, lane = threadIdx.x & 63, grp = lane >> 4, c = lane & 15;
  // A operands (weights): co = 16*wave + c, k' = 8*grp + j..+7: one 16-byte load per k-step
  s8 wa[kKH];
#pragma unroll
  for (int kh = 0; kh < kKH; ++kh)
    wa[kh] = *reinterpret_cast<const s8*>(wk + ((16 * wave + c) * kKH + kh) * 32 + 8 * grp);
  zero_image(img);
  drain_vm();
  float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
  ImgRegs ir;
  if (blockIdx.x < rows) load_image(x, ir, blockIdx.x / g.OH, static_cast<int>(blockIdx.x % g.OH), g);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    lds_barrier();  // previous row's LDS reads are done
    store_image(ir, img, g);
    lds_barrier();
    const int64_t nxt = row + gridDim.x;
    if (nxt < rows) load_image(x, ir, nxt / g.OH, static_cast<int>(nxt % g.OH), g);
    f4 acc[TILES];
    conv_row<TILES>(img, wa, grp, c, acc);
    // C[co = 16*wave + 4*grp + r][pixel = 16t + c] -> outs[pixel][co]
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
      bf16x4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v.v[r] = f2bf(acc[t][r]);
        const float q = bf2f(v.v[r]);
        st_s[r] += q;
        st_q[r] += q * q;
      }
      *reinterpret_cast<bf16x4*>(outs + (16 * t + c) * kOutRS + 16 * wave + 4 * grp) = v;
    }
    lds_barrier();
    bf16_t* dst = y + row * g.OW * kCo;
    for (int v = threadIdx.x; v < g.OW * (kCo / 8); v += kThreads) {
      const int px = v >> 3, cv = v & 7;
      *reinterpret_cast<uint4*>(dst + px * kCo + cv * 8) = *reinterpret_cast<const uint4*>(outs + px * kOutRS + cv * 8);
    }
  }
  if (part != nullptr) {
    // lanes c = 0..15 of a 16-lane group hold the same 4 channels: xor-reduce inside the group
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        st_s[r] += __shfl_xor(st_s[r], o, 64);
        st_q[r] += __shfl_xor(st_q[r], o, 64);
      }
    if (c == 0) {
      float* dst = part + static_cast<int64_t>(blockIdx.x) * 2 * kCo + 16 * wave + 4 * grp;
#pragma unroll
      for (int r = 0; r < 4; ++r) { dst[r] = st_s[r]; dst[kCo + r] = st_q[r]; }
    }
  }
}

// dY row (OW x 64 bf16 = OW * 8 16-byte vectors), at most kDyItems per thread (OW <= 128)
constexpr int kDyItems = kPix * (kCo / 8) / kThreads;
__device__ __forceinline__ void load_dy(const bf16_t* __restrict__ dy, uint4* dr, int64_t row, const Geo& g) {
  const bf16_t* src = dy + row * g.OW * kCo;
#pragma unroll
  for (int i = 0; i < kDyItems; ++i) {
    const int v = threadIdx.x + i * kThreads;
    dr[i] = v < g.OW * (kCo / 8) ? *reinterpret_cast<const uint4*>(src + (v >> 3) * kCo + (v & 7) * 8)
                                 : make_uint4(0, 0, 0, 0);
  }
}

// part: [gridDim.x][64][7 * 32] fp32 partial sums of dW[co][kh][k'] over this block's rows;
// STEPS = ceil(OW / 32) pixel k-steps per row.
template <int STEPS>
__global__ void __launch_bounds__(kThreads)
stem_conv_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ part,
                       int64_t rows, Geo g) {
  __shared__ __attribute__((aligned(16))) bf16_t img[kKH * kRowE];
  __shared__ __attribute__((aligned(16))) bf16_t dys[kPix * kOutRS];
  const int wave = threadIdx.x / 64, lane = threadIdx.x & 63, grp = lane >> 4, c = lane & 15;
  zero_image(img);
  for (int i = threadIdx.x; i < kPix * kOutRS / 8; i += kThreads)
    reinterpret_cast<uint4*>(dys)[i] = make_uint4(0, 0, 0, 0);  // pixels >= OW stay zero
  f4 acc[kKH * 2];
#pragma unroll
  for (int i = 0; i < kKH * 2; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};
  ImgRegs ir;
  uint4 dr[kDyItems];
  if (blockIdx.x < rows) {
    load_image(x, ir, blockIdx.x / g.OH, static_cast<int>(blockIdx.x % g.OH), g);
    load_dy(dy, dr, blockIdx.x, g);
  }
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    lds_barrier();
    store_image(ir, img, g);
#pragma unroll
    for (int i = 0; i < kDyItems; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < g.OW * (kCo / 8)) *reinterpret_cast<uint4*>(dys + (v >> 3) * kOutRS + (v & 7) * 8) = dr[i];
    }
    lds_barrier();
    const int64_t nxt = row + gridDim.x;
    if (nxt < rows) {
      load_image(x, ir, nxt / g.OH, static_cast<int>(nxt % g.OH), g);
      load_dy(dy, dr, nxt, g);
    }
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int r0 = 32 * s + 4 * grp, r1 = r0 + 16;
      // A[co = 16*wave + c][pixel p(grp, j)] = dY^T
      const s8 a = tr_pair(dys, kOutRS, r0, r1, 16 * wave, c);
#pragma unroll
      for (int kh = 0; kh < kKH; ++kh) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          // B[pixel p(grp, j)][k' = 16*kt + c] = img[kh][8 * pixel + k']
          const s8 b = tr_pair(img + kh * kRowE, 8, r0, r1, 16 * kt, c);
          acc[kh * 2 + kt] = mfma(a, b, acc[kh * 2 + kt]);
        }
      }
    }
  }
  // acc[kh*2+kt][r] = dW[co = 16*wave + 4*grp + r][kh][k' = 16*kt + c]
  float* dst = part + static_cast<int64_t>(blockIdx.x) * kCo * kPartCols;
#pragma unroll
  for (int i = 0; i < kKH * 2; ++i) {
    const int kh = i >> 1, kt = i & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[(16 * wave + 4 * grp + r) * kPartCols + kh * 32 + 16 * kt + c] = acc[i][r];
  }
}

// dW[co][kh][kw][ci] = sum over blocks of part[b][co][kh][4*kw + ci]; 64 partial columns x 4
// block slices per workgroup, fixed summation order.
template <typename WT>
__global__ void __launch_bounds__(kThreads)
stem_wgrad_finalize_kernel(const float* __restrict__ part, int nb, WT* __restrict__ dw) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63);  // < 64 * 224
  const int slice = threadIdx.x >> 6;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int b = slice;
  for (; b + 28 < nb; b += 32) {
#pragma unroll
    for (int u = 0; u < 8; ++u) acc[u] += part[static_cast<int64_t>(b + 4 * u) * kCo * kPartCols + col];
  }
  for (; b < nb; b += 4) acc[0] += part[static_cast<int64_t>(b) * kCo * kPartCols + col];
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += acc[u];
  red[slice][threadIdx.x & 63] = s;
  __syncthreads();
  if (slice == 0) {
    s = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    const int co = col / kPartCols, rem = col - co * kPartCols;
    const int kh = rem / 32, kp = rem & 31, kw = kp >> 2, ci = kp & 3;
    if (kw < 7 && ci < 3) Elem<WT>::st(dw, ((co * 7 + kh) * 7 + kw) * 3 + ci, s);
  }
}

// ============================================== fused stem: conv -> BN -> ReLU -> MaxPool 3x3/s2/p1
// The stem conv's 112x112x64 output (1.6 GB at batch 1024) existed only to be pooled: the
// separate path writes it, reads it back for BN+ReLU+pool, reads it again in the BN backward
// apply, writes its gradient and reads that in the weight gradient -- ~7 GB of HBM traffic for a
// 0.24 TFLOP conv.  Here it is never stored:
//  * relu(s*x + b) is monotone in x (non-decreasing for s >= 0, non-increasing for s < 0) and
//    s = gamma * invstd has gamma's sign, known before the statistics are.  So
//    maxpool(relu(bn(x))) = relu(s * x_sel + b) with x_sel the window's max of the RAW conv output
//    where gamma >= 0 and its min where gamma < 0 (first extremum wins, as torch's argmax).  The
//    forward kernel pools the conv rows it computed out of a 4-row LDS ring and writes only
//    x_sel + the window position (1/4 + 1/8 of the full output) and the BN statistics partials;
//    the BN apply then runs on the pooled tensor (csrc/bn.hip damd_stem_pool_bn_fwd_launch).
//  * the backward recomputes each conv row (the same MFMA sequence, so bit-identical values),
//    routes the masked pooled gradient dz to the window arg-extrema, forms the BN input gradient
//    dx = A*dz + B*x + Cc in registers and feeds it straight to the weight-gradient MFMAs.
// Work items are bands of kPoolBand pooled rows of one image (the forward recomputes the one conv
// row a band shares with the band above; it is excluded from the statistics).
constexpr int kPoolBand = 8;
constexpr int kMaxPW = kMaxOW / 2;
constexpr int kPdzRS = 72;  // LDS row stride (elements) of a staged pooled-gradient row
constexpr int kPixRS = 80;  // LDS row stride (bytes) of a staged window-position row

struct PGeo {
  int H, W, OH, OW, PH, PW, bands;
};

// conv rows [h0, h1) of work item `item` (image n, pooled rows from oh0); `overlap`: start one
// row early (the forward's pooling window of pooled row oh0 reaches up to conv row 2*oh0 - 1)
__device__ __forceinline__ void band_rows(int64_t item, const PGeo& p, bool overlap, int64_t& n, int& h0, int& h1,
                                          int& oh0) {
  n = item / p.bands;
  const int b = static_cast<int>(item - n * p.bands);
  oh0 = b * kPoolBand;
  const int oh1 = min(oh0 + kPoolBand, p.PH);
  h0 = overlap ? max(2 * oh0 - 1, 0) : 2 * oh0;
  h1 = 2 * oh1;
}

// gamma: the BN weight (fp32 or bf16), read for its sign only.  xarg / idx: [N][PH][PW][64]
// selected raw value / window position (kh * 3 + kw); part: [gridDim.x][2][64] (sum, sum sq) of
// the bf16-rounded conv outputs, each conv row counted once.
template <int TILES>
__global__ void __launch_bounds__(kThreads, 2)
stem_pool_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wk, const void* __restrict__ gamma,
                     int gamma_bf16, bf16_t* __restrict__ xarg, uint8_t* __restrict__ idx, float* __restrict__ part,
                     int64_t items, PGeo p) {
  __shared__ __attribute__((aligned(16))) bf16_t img[kKH * kRowE];
  __shared__ __attribute__((aligned(16))) bf16_t ring[4][kMaxOW * kOutRS];  // conv row r in slot (r + 1) & 3
  const int wave = threadIdx.x / 64, lane = threadIdx.x & 63, grp = lane >> 4, c = lane & 15;
  const Geo g{p.H, p.W, p.OH, p.OW};
  s8 wa[kKH];
#pragma unroll
  for (int kh = 0; kh < kKH; ++kh)
    wa[kh] = *reinterpret_cast<const s8*>(wk + ((16 * wave + c) * kKH + kh) * 32 + 8 * grp);
  zero_image(img);
  // pooling role: channel group pcg (8 channels) of pooled pixels threadIdx.x / 8 + 32 * i
  const int pcg = threadIdx.x & 7;
  bool neg[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int ch = pcg * 8 + k;
    const float gv = gamma_bf16 ? bf2f(static_cast<const bf16_t*>(gamma)[ch]) : static_cast<const float*>(gamma)[ch];
    neg[k] = gv < 0.f;
  }
  // the ring holds pooling KEYS: the conv value, sign-flipped for gamma < 0 channels (exact for bf16), so
  // the pooling is a plain max with no per-element select; the writer's channels are 16 wave + 4 grp + r
  uint16_t kflip[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ch = 16 * wave + 4 * grp + r;
    const float gv = gamma_bf16 ? bf2f(static_cast<const bf16_t*>(gamma)[ch]) : static_cast<const float*>(gamma)[ch];
    kflip[r] = gv < 0.f ? 0x8000u : 0u;
  }
  drain_vm();
  float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
  // Iteration h of a band computes conv row h (h < h1) and pools pooled row h / 2 - 1 (even h):
  // its rows h - 3 .. h - 1 were finished by earlier iterations, so an iteration issues all its
  // global traffic (the next image prefetch, the pooled stores) BEFORE its MFMAs, which then cover
  // that traffic's latency until the next iteration's first wait.  h runs to h1 inclusive (a
  // pool-only last iteration).
  int64_t item = blockIdx.x, n = 0;
  int h = 0, h1 = 0, oh0 = 0;
  ImgRegs ir;
  if (item < items) {
    band_rows(item, p, true, n, h, h1, oh0);
    load_image(x, ir, n, h, g);
  }
  while (item < items) {
    const bool compute = h < h1;
    lds_barrier();  // the previous iteration's image and ring reads are done
    if (compute) store_image(ir, img, g);
    lds_barrier();
    int64_t nitem = item, nn = n;
    int nh = h + 1, nh1 = h1, noh0 = oh0;
    if (nh > h1) {
      nitem = item + gridDim.x;
      if (nitem < items) band_rows(nitem, p, true, nn, nh, nh1, noh0);
    }
    if (nitem < items && nh < nh1) load_image(x, ir, nn, nh, g);
    if (!(h & 1) && h >= 2 * oh0 + 2) {  // conv rows h - 3, h - 2, h - 1 complete pooled row h / 2 - 1
      const int oh = (h >> 1) - 1;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int v = threadIdx.x + i * kThreads;
        if (v >= p.PW * 8) break;
        const int ow = v >> 3;
        float best[8];
        int arg[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) { best[k] = -INFINITY; arg[k] = 0; }
#pragma unroll
        for (int kh = 0; kh < 3; ++kh) {
          const int r = 2 * oh - 1 + kh;
          if (r < 0) continue;
          const bf16_t* row = ring[(r + 1) & 3] + pcg * 8;
#pragma unroll
          for (int kw = 0; kw < 3; ++kw) {
            const int col = 2 * ow - 1 + kw;
            if (col < 0 || col >= p.OW) continue;
            const bf16x8 a = *reinterpret_cast<const bf16x8*>(row + col * kOutRS);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float key = bf2f(a.v[k]);  // the ring holds keys (see kflip)
              if (key > best[k]) { best[k] = key; arg[k] = kh * 3 + kw; }
            }
          }
        }
        bf16x8 o;
        uint32_t lo = 0, hi = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = f2bf(neg[k] ? -best[k] : best[k]);
#pragma unroll
        for (int k = 0; k < 4; ++k) { lo |= static_cast<uint32_t>(arg[k]) << (8 * k); hi |= static_cast<uint32_t>(arg[k + 4]) << (8 * k); }
        const int64_t off = ((n * p.PH + oh) * p.PW + ow) * kCo + pcg * 8;
        *reinterpret_cast<bf16x8*>(xarg + off) = o;
        *reinterpret_cast<uint2*>(idx + off) = make_uint2(lo, hi);
      }
    }
    if (compute) {
      f4 acc[TILES];
      conv_row<TILES>(img, wa, grp, c, acc);
      // slot (h + 1) & 3 last held row h - 4, whose last pooling (iteration h - 2) is done
      const bool own = h >= 2 * oh0;
      bf16_t* rs = ring[(h + 1) & 3];
#pragma unroll
      for (int t = 0; t < TILES; ++t) {
        bf16x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          v.v[r] = f2bf(acc[t][r]);
          const float q = own ? bf2f(v.v[r]) : 0.f;
          st_s[r] += q;
          st_q[r] += q * q;
          v.v[r] = static_cast<bf16_t>(v.v[r] ^ kflip[r]);  // pooling key
        }
        *reinterpret_cast<bf16x4*>(rs + (16 * t + c) * kOutRS + 16 * wave + 4 * grp) = v;
      }
    }
    item = nitem; n = nn; h = nh; h1 = nh1; oh0 = noh0;
  }
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      st_s[r] += __shfl_xor(st_s[r], o, 64);
      st_q[r] += __shfl_xor(st_q[r], o, 64);
    }
  if (c == 0) {
    float* dst = part + static_cast<int64_t>(blockIdx.x) * 2 * kCo + 16 * wave + 4 * grp;
#pragma unroll
    for (int r = 0; r < 4; ++r) { dst[r] = st_s[r]; dst[kCo + r] = st_q[r]; }
  }
}

// dpz: [N][PH][PW][64] pooled gradient with the ReLU mask applied (bn.hip pooled reduce);
// coef: [3][64] BN-backward coefficients (A, B, Cc); part: [gridDim.x][64][7 * 32] as the plain
// weight-gradient kernel (summed by stem_wgrad_finalize_kernel).
template <int TILES, int STEPS>
__global__ void __launch_bounds__(kThreads, 2)
stem_pool_bwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ wk, const bf16_t* __restrict__ dpz,
                     const uint8_t* __restrict__ idx, const float* __restrict__ coef, float* __restrict__ part,
                     int64_t items, PGeo p) {
  __shared__ __attribute__((aligned(16))) bf16_t img[kKH * kRowE];
  __shared__ __attribute__((aligned(16))) bf16_t dys[kPix * kOutRS];
  __shared__ __attribute__((aligned(16))) bf16_t pdz[2][kMaxPW * kPdzRS];
  __shared__ __attribute__((aligned(16))) uint8_t pix[2][kMaxPW * kPixRS];
  const int wave = threadIdx.x / 64, lane = threadIdx.x & 63, grp = lane >> 4, c = lane & 15;
  const Geo g{p.H, p.W, p.OH, p.OW};
  s8 wa[kKH];
#pragma unroll
  for (int kh = 0; kh < kKH; ++kh)
    wa[kh] = *reinterpret_cast<const s8*>(wk + ((16 * wave + c) * kKH + kh) * 32 + 8 * grp);
  zero_image(img);
  for (int i = threadIdx.x; i < kPix * kOutRS / 8; i += kThreads)
    reinterpret_cast<uint4*>(dys)[i] = make_uint4(0, 0, 0, 0);  // pixels >= OW stay zero
  const int co0 = 16 * wave + 4 * grp;  // this lane's 4 channels in the recomputed row
  // BN-backward coefficients in LDS, read per row (loop-invariant registers would cost 12 VGPRs
  // across the whole row loop)
  __shared__ __attribute__((aligned(16))) float cf[3 * kCo];
  for (int i = threadIdx.x; i < 3 * kCo; i += kThreads) cf[i] = coef[i];
  drain_vm();
  f4 acc[kKH * 2];
#pragma unroll
  for (int i = 0; i < kKH * 2; ++i) acc[i] = f4{0.f, 0.f, 0.f, 0.f};

  // one pooled row: PW * 8 gradient vectors + PW * 4 position vectors of 16 bytes, <= 3 per thread
  // (named registers: an indexed array here is promoted to LDS scratch by the compiler)
  uint4 pr0 = make_uint4(0, 0, 0, 0), pr1 = pr0, pr2 = pr0;
  auto pooled_src = [&](int64_t base, int v) -> const uint4* {
    return v < p.PW * 8 ? reinterpret_cast<const uint4*>(dpz + base + v * 8)
                        : reinterpret_cast<const uint4*>(idx + base + (v - p.PW * 8) * 16);
  };
  auto load_pooled = [&](int64_t nn, int oh) {
    const int64_t base = (nn * p.PH + oh) * p.PW * kCo;
    const int v0 = threadIdx.x, v1 = v0 + kThreads, v2 = v1 + kThreads;
    if (v0 < p.PW * 12) pr0 = *pooled_src(base, v0);
    if (v1 < p.PW * 12) pr1 = *pooled_src(base, v1);
    if (v2 < p.PW * 12) pr2 = *pooled_src(base, v2);
  };
  auto put_pooled = [&](int s, int v, uint4 val) {
    if (v < p.PW * 8) {
      *reinterpret_cast<uint4*>(pdz[s] + (v >> 3) * kPdzRS + (v & 7) * 8) = val;
    } else if (v < p.PW * 12) {
      const int u = v - p.PW * 8;
      *reinterpret_cast<uint4*>(pix[s] + (u >> 2) * kPixRS + (u & 3) * 16) = val;
    }
  };
  auto store_pooled = [&](int oh) {
    const int s = oh & 1;
    put_pooled(s, threadIdx.x, pr0);
    put_pooled(s, threadIdx.x + kThreads, pr1);
    put_pooled(s, threadIdx.x + 2 * kThreads, pr2);
  };

  int64_t item = blockIdx.x, n = 0;
  int h = 0, h1 = 0, oh0 = 0, pend = -1;
  ImgRegs ir;
  if (item < items) {
    band_rows(item, p, false, n, h, h1, oh0);
    load_image(x, ir, n, h, g);
    load_pooled(n, oh0);
    pend = oh0;
  }
  while (item < items) {
    // pooled row k + 1 goes into the slot of row k - 1, last read by conv row 2k - 1
    lds_barrier();
    store_image(ir, img, g);
    if (pend >= 0) store_pooled(pend);
    lds_barrier();
    int64_t nitem = item, nn = n;
    int nh = h + 1, nh1 = h1, noh0 = oh0;
    if (nh >= h1) {
      nitem = item + gridDim.x;
      if (nitem < items) band_rows(nitem, p, false, nn, nh, nh1, noh0);
    }
    pend = -1;
    if (nitem < items) {
      load_image(x, ir, nn, nh, g);
      // a band's first (even) row needs pooled row nh / 2; an odd row also needs (nh + 1) / 2
      const int need = nh == 2 * noh0 ? noh0 : ((nh & 1) && (nh + 1) / 2 < p.PH ? (nh + 1) / 2 : -1);
      if (need >= 0) {
        load_pooled(nn, need);
        pend = need;
      }
    }
    // recompute conv row h exactly as stem_pool_fwd_kernel did
    f4 xa[TILES];
    conv_row<TILES, false>(img, wa, grp, c, xa);
    // dz at (h, px): sum of the masked pooled gradients of the windows whose arg-extremum it is.
    // Row window a / column window b: h even -> window h / 2 only (at window row 1); h odd ->
    // windows (h - 1) / 2 (row 2) and (h + 1) / 2 (row 0, if it exists); likewise for px.  All four
    // (a, b) reads are issued unconditionally (a missing window re-reads window 0 and is masked), so
    // the LDS reads of a row go out back to back instead of one dependent pair per loop trip.
    const bool r2 = (h & 1) && ((h + 1) >> 1) < p.PH;
#pragma unroll
    for (int t = 0; t < TILES; ++t) {
      const int px = 16 * t + c;
      const bool c2 = (px & 1) && ((px + 1) >> 1) < p.PW;
      float dz[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const int oh = (h >> 1) + (a && r2 ? 1 : 0);
        const int prow = (h & 1) ? (a == 0 ? 2 : 0) : 1;  // row of h inside window oh
        const bf16_t* dzr = pdz[oh & 1] + co0;
        const uint8_t* pxr = pix[oh & 1] + co0;
#pragma unroll
        for (int b = 0; b < 2; ++b) {
          const bool ok = (a == 0 || r2) && (b == 0 || c2);
          const int ow = (px >> 1) + (b && c2 ? 1 : 0);
          const int pcol = (px & 1) ? (b == 0 ? 2 : 0) : 1;
          const uint32_t pos = ok ? static_cast<uint32_t>(prow * 3 + pcol) : 0xFFu;  // 0xFF: never a position
          const uint32_t ib = *reinterpret_cast<const uint32_t*>(pxr + ow * kPixRS);
          const bf16x4 dv = *reinterpret_cast<const bf16x4*>(dzr + ow * kPdzRS);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (((ib >> (8 * r)) & 0xFFu) == pos) dz[r] += bf2f(dv.v[r]);
        }
      }
      const float4 cA = *reinterpret_cast<const float4*>(cf + co0);
      const float4 cB = *reinterpret_cast<const float4*>(cf + kCo + co0);
      const float4 cC = *reinterpret_cast<const float4*>(cf + 2 * kCo + co0);
      const float fa[4] = {cA.x, cA.y, cA.z, cA.w}, fb[4] = {cB.x, cB.y, cB.z, cB.w}, fc[4] = {cC.x, cC.y, cC.z, cC.w};
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float xv = bf2f(f2bf(xa[t][r]));
        o.v[r] = f2bf(fa[r] * dz[r] + fb[r] * xv + fc[r]);
      }
      *reinterpret_cast<bf16x4*>(dys + px * kOutRS + co0) = o;
      // VGPR budget
    }
    lds_barrier();
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int r0 = 32 * s + 4 * grp, r1 = r0 + 16;
      const s8 a = tr_pair(dys, kOutRS, r0, r1, 16 * wave, c);
#pragma unroll
      for (int kh = 0; kh < kKH; ++kh) {
#pragma unroll
        for (int kt = 0; kt < 2; ++kt) {
          const s8 b = tr_pair(img + kh * kRowE, 8, r0, r1, 16 * kt, c);
          acc[kh * 2 + kt] = mfma(a, b, acc[kh * 2 + kt]);
        }
      }
    }
    item = nitem; n = nn; h = nh; h1 = nh1; oh0 = noh0;
  }
  float* dst = part + static_cast<int64_t>(blockIdx.x) * kCo * kPartCols;
#pragma unroll
  for (int i = 0; i < kKH * 2; ++i) {
    const int kh = i >> 1, kt = i & 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) dst[(16 * wave + 4 * grp + r) * kPartCols + kh * 32 + 16 * kt + c] = acc[i][r];
  }
}

}  // namespace stem
}  // namespace damd

using namespace damd;
using namespace damd::stem;

extern "C" {

// output width must be a whole number of 16-pixel tiles (ResNet at 224: OW = 112 = 7 tiles)
int damd_stem_supported(int64_t H, int64_t W) {
  const int64_t OW = (W - 1) / 2 + 1;
  return H >= 1 && W % 4 == 0 && OW % 16 == 0 && OW >= 16 && OW <= kMaxOW;
}

int damd_stem_fwd_blocks(int64_t N, int H) {
  // 4 workgroups / CU are resident: a single persistent round, each looping over its rows
  const int64_t rows = N * ((H - 1) / 2 + 1);
  return static_cast<int>(rows < 1024 ? rows : 1024);
}

// wk: [64][7][32] bf16 padded weight image; part: null or [damd_stem_fwd_blocks][2][64] fp32
void damd_stem_fwd_launch(const void* x, const void* wk, void* y, float* part, int64_t N, int H, int W,
                          hipStream_t st) {
  const Geo g{H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t rows = N * g.OH;
  const unsigned grid = static_cast<unsigned>(damd_stem_fwd_blocks(N, H));
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(wk);
  bf16_t* yp = static_cast<bf16_t*>(y);
#define FWD(T) DAMD_LAUNCH(stem_conv_fwd_kernel<T>, dim3(grid), dim3(kThreads), 0, st, xp, wp, yp, part, rows, g)
  switch (g.OW / 16) {
    case 1: FWD(1); break;
    case 2: FWD(2); break;
    case 3: FWD(3); break;
    case 4: FWD(4); break;
    case 5: FWD(5); break;
    case 6: FWD(6); break;
    default: FWD(7); break;
  }
#undef FWD
  DAMD_CHECK_LAUNCH();
}

int damd_stem_wgrad_blocks(int64_t N, int H) {
  const int64_t rows = N * ((H - 1) / 2 + 1);
  // 3 workgroups / CU fit (LDS + AGPR accumulators): one resident round over 256 CUs
  return static_cast<int>(rows < 768 ? rows : 768);
}

// part: [damd_stem_wgrad_blocks][64][224] fp32 scratch; dw: [64][7][7][3], w_dtype 0 fp32 / 1 bf16
void damd_stem_wgrad_launch(const void* x, const void* dy, float* part, void* dw, int w_dtype, int64_t N, int H,
                            int W, hipStream_t st) {
  const Geo g{H, W, (H - 1) / 2 + 1, (W - 1) / 2 + 1};
  const int64_t rows = N * g.OH;
  const int nb = damd_stem_wgrad_blocks(N, H);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* dp = static_cast<const bf16_t*>(dy);
#define WG(S) DAMD_LAUNCH(stem_conv_wgrad_kernel<S>, dim3(nb), dim3(kThreads), 0, st, xp, dp, part, rows, g)
  switch ((g.OW + 31) / 32) {
    case 1: WG(1); break;
    case 2: WG(2); break;
    case 3: WG(3); break;
    default: WG(4); break;
  }
#undef WG
  const dim3 fg(kCo * kPartCols / 64);
  if (w_dtype == 1)
    DAMD_LAUNCH(stem_wgrad_finalize_kernel<bf16_t>, fg, dim3(kThreads), 0, st, part, nb, static_cast<bf16_t*>(dw));
  else
    DAMD_LAUNCH(stem_wgrad_finalize_kernel<float>, fg, dim3(kThreads), 0, st, part, nb, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
}

// ---- fused stem conv + BN + ReLU + max-pool (3x3 / stride 2 / pad 1)
namespace {
PGeo pool_geo(int64_t H, int64_t W) {
  PGeo p;
  p.H = static_cast<int>(H); p.W = static_cast<int>(W);
  p.OH = (p.H - 1) / 2 + 1; p.OW = (p.W - 1) / 2 + 1;
  p.PH = p.OH / 2; p.PW = p.OW / 2;
  p.bands = (p.PH + kPoolBand - 1) / kPoolBand;
  return p;
}
}  // namespace

// the conv output must pool without a partial last window (even OH, OW)
int damd_stem_pool_supported(int64_t H, int64_t W) {
  const int64_t OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  return damd_stem_supported(H, W) && OH % 2 == 0 && OW % 2 == 0 && OW / 2 <= kMaxPW;
}

int damd_stem_pool_blocks(int64_t N, int64_t H, int64_t W) {
  // 2 workgroups / CU (LDS): one resident round over 256 CUs, each looping over its bands
  const int64_t items = N * pool_geo(H, W).bands;
  return static_cast<int>(items < 512 ? items : 512);
}

// wk: [64][7][32] padded weight image; gamma: BN weight (gamma_bf16: its dtype); xarg / idx:
// [N][PH][PW][64]; part: [damd_stem_pool_blocks][2][64]
void damd_stem_pool_fwd_launch(const void* x, const void* wk, const void* gamma, int gamma_bf16, void* xarg,
                               uint8_t* idx, float* part, int64_t N, int H, int W, hipStream_t st) {
  const PGeo p = pool_geo(H, W);
  const int64_t items = N * p.bands;
  const unsigned grid = static_cast<unsigned>(damd_stem_pool_blocks(N, H, W));
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(wk);
  bf16_t* ap = static_cast<bf16_t*>(xarg);
#define PF(T) DAMD_LAUNCH(stem_pool_fwd_kernel<T>, dim3(grid), dim3(kThreads), 0, st, xp, wp, gamma, gamma_bf16, ap, idx, part, items, p)
  switch (p.OW / 16) {
    case 1: PF(1); break;
    case 2: PF(2); break;
    case 3: PF(3); break;
    case 4: PF(4); break;
    case 5: PF(5); break;
    case 6: PF(6); break;
    default: PF(7); break;
  }
#undef PF
  DAMD_CHECK_LAUNCH();
}

// dpz: masked pooled gradient [N][PH][PW][64]; coef: [3][64]; part: [damd_stem_pool_blocks][64][224]
// fp32 scratch; dw: [64][7][7][3] in w_dtype (0 fp32 / 1 bf16)
void damd_stem_pool_bwd_launch(const void* x, const void* wk, const void* dpz, const uint8_t* idx, const float* coef,
                               float* part, void* dw, int w_dtype, int64_t N, int H, int W, hipStream_t st) {
  const PGeo p = pool_geo(H, W);
  const int64_t items = N * p.bands;
  const int nb = damd_stem_pool_blocks(N, H, W);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(wk);
  const bf16_t* dp = static_cast<const bf16_t*>(dpz);
#define PB(T, S) DAMD_LAUNCH((stem_pool_bwd_kernel<T, S>), dim3(nb), dim3(kThreads), 0, st, xp, wp, dp, idx, coef, part, items, p)
  switch (p.OW / 16) {
    case 1: PB(1, 1); break;
    case 2: PB(2, 1); break;
    case 3: PB(3, 2); break;
    case 4: PB(4, 2); break;
    case 5: PB(5, 3); break;
    case 6: PB(6, 3); break;
    default: PB(7, 4); break;
  }
#undef PB
  const dim3 fg(kCo * kPartCols / 64);
  if (w_dtype == 1)
    DAMD_LAUNCH(stem_wgrad_finalize_kernel<bf16_t>, fg, dim3(kThreads), 0, st, part, nb, static_cast<bf16_t*>(dw));
  else
    DAMD_LAUNCH(stem_wgrad_finalize_kernel<float>, fg, dim3(kThreads), 0, st, part, nb, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
}

}  // extern "C"
