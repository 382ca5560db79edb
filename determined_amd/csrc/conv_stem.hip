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
  float st_s[4] = {0.f, 0.f, 0.f, 0.f}, st_q[4] = {0.f, 0.f, 0.f, 0.f};
  ImgRegs ir;
  if (blockIdx.x < rows) load_image(x, ir, blockIdx.x / g.OH, static_cast<int>(blockIdx.x % g.OH), g);
  for (int64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    __syncthreads();  // previous row's LDS reads are done
    store_image(ir, img, g);
    __syncthreads();
    const int64_t nxt = row + gridDim.x;
    if (nxt < rows) load_image(x, ir, nxt / g.OH, static_cast<int>(nxt % g.OH), g);
    f4 acc[TILES];
#pragma unroll
    for (int t = 0; t < TILES; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kh = 0; kh < kKH; ++kh) {
      const bf16_t* base = img + kh * kRowE + 8 * grp;
#pragma unroll
      for (int t = 0; t < TILES; ++t) {
        const s8 b = *reinterpret_cast<const s8*>(base + 8 * (16 * t + c));
        acc[t] = mfma(wa[kh], b, acc[t]);
      }
    }
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
    __syncthreads();
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
    __syncthreads();
    store_image(ir, img, g);
#pragma unroll
    for (int i = 0; i < kDyItems; ++i) {
      const int v = threadIdx.x + i * kThreads;
      if (v < g.OW * (kCo / 8)) *reinterpret_cast<uint4*>(dys + (v >> 3) * kOutRS + (v & 7) * 8) = dr[i];
    }
    __syncthreads();
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
#define FWD(T) hipLaunchKernelGGL(stem_conv_fwd_kernel<T>, dim3(grid), dim3(kThreads), 0, st, xp, wp, yp, part, rows, g)
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
#define WG(S) hipLaunchKernelGGL(stem_conv_wgrad_kernel<S>, dim3(nb), dim3(kThreads), 0, st, xp, dp, part, rows, g)
  switch ((g.OW + 31) / 32) {
    case 1: WG(1); break;
    case 2: WG(2); break;
    case 3: WG(3); break;
    default: WG(4); break;
  }
#undef WG
  const dim3 fg(kCo * kPartCols / 64);
  if (w_dtype == 1)
    hipLaunchKernelGGL(stem_wgrad_finalize_kernel<bf16_t>, fg, dim3(kThreads), 0, st, part, nb, static_cast<bf16_t*>(dw));
  else
    hipLaunchKernelGGL(stem_wgrad_finalize_kernel<float>, fg, dim3(kThreads), 0, st, part, nb, static_cast<float*>(dw));
  DAMD_CHECK_LAUNCH();
}

}  // extern "C"
