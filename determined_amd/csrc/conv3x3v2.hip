// 3x3 / stride 1 / pad 1 convolution on a zero-padded LDS halo (gfx950 / MI355X): bf16 NHWC activations,
// [K][3][3][C] weights, fp32 accumulation on v_mfma_f32_16x16x32_bf16.  Forward, and the input gradient
// as the forward of the flipped, transposed weights; optional BatchNorm prologue (PRO) / epilogue (EPI)
// fusions with the same contracts as conv_igemm.hip's generic and halo kernels.
//
// Why a second 3x3 kernel.  conv_igemm.hip's halo kernel stages the flattened pixel run
// m0 - W - 1 ... m0 + BP + W of a tile and reads tap (r, s) at row offset r*W + s: a tap that falls
// outside the image lands on a neighbouring row / image, so every B-fragment read needs a per-pixel
// tap-validity test and a select, and its XOR-swizzled LDS address depends on (pixel + tap offset) & 7
// -- about 8 VALU instructions per B read, the kernel was VALU-issue-bound
// (profiles/conv3x3_pmc_valu_bound_b1024_1gpu.txt).  Here:
//   * a tile is TR whole image rows of ONE image (TR | H), so the pixel -> halo-slot map of a lane is
//     the same for every tile and is computed once per launch;
//   * the halo is a (TR + 2) x (W + 2) grid of slots with the image border as real zero slots, so no
//     tap ever needs a validity test;
//   * the halo is chunk-planar (16-byte channel chunk c of slot s at c * PLANE + 16 s) and the pixel
//     lanes are row-padded (W -> multiple of 16), so a fragment's 16 lanes read 16 consecutive slots of
//     one image row: the ds_read_b128 lane groups, which mix two chunks (lanes {0-3, 12-15} and {20-27}),
//     hit 16 distinct bank quads with no swizzle.  (The first version -- 144-byte pixel slots, 8 waves --
//     spent 23% of its LDS cycles in bank conflicts: profiles/conv3x3v2_pmc_b2048_1gpu.txt.)  With W a template
//     constant every tap / k-half offset is an immediate of the ds_read: a B-fragment read costs no VALU;
//   * 8 waves, 2 per SIMD (256 registers each), every wave a 64-channel x 32- or 64-pixel tile; a tap's
//     fragments are read after its barrier into one register set, and the other wave on the SIMD
//     multiplies while this one waits.  (A 4-wave variant -- 1 wave per SIMD, 64x64 wave tiles, fragments
//     double-buffered across taps -- halved the LDS reads per MFMA but left the halo staging and epilogue
//     VALU with no other wave to hide under: 3.4 VALU per MFMA, slower on every layer,
//     profiles/conv3x3v2_4wave_vs_8wave_b2048_1gpu.txt.)
// Halo staging: buffer loads from a per-unit resource whose out-of-range offsets return the zero border
// (no per-chunk address arithmetic or select).  With a BN prologue the halo is register-staged (load ->
// transform -> ds_write_b128): loaded at the first tap of a 64-channel unit and written into the other halo
// buffer at tap 5, so five taps of MFMAs cover the HBM latency; without one it goes straight to LDS by the
// buffer LDS-DMA.  The BN prologue's per-channel coefficients are staged in LDS once per launch.  Weights
// stream per tap through a 5-slot LDS ring filled 4 taps ahead by the LDS-DMA, XOR-swizzled as in
// conv_igemm.hip -- except for 64-channel layers (RES configs), whose whole filter stays resident in LDS:
// no weight traffic and no per-tap barrier, the waves meet only at unit boundaries.
// The same file holds the whole-row-tile 3x3 weight gradient (conv3x3v2_wgrad_kernel, below).
// Work split: persistent blocks (one per CU), each a contiguous run of tiles, so consecutive tiles of an
// image -- which share two halo rows -- run back to back on the same CU / XCD L2.

#include <cstdlib>

#include "common.h"

namespace damd {
namespace c3v2 {

typedef short s8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void lds_void_t;

constexpr int kBK = 64;      // channels per unit (one k-step of 64 per tap)

constexpr int kEpiNone = 0, kEpiStats = 1, kEpiBnbM = 2, kEpiBnbR = 3;  // conv_igemm.hip EPI modes

__device__ __forceinline__ f4 mfma(s8 a, s8 b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(b8, a), __builtin_bit_cast(b8, b), c, 0, 0, 0);
}
__device__ __forceinline__ int swz(int row) { return ((row >> 1) ^ (row >> 3)) & 7; }
// A-operand row of fragment i for fragment row rho (conv_igemm.hip a_row): lane group g ends with 8
// consecutive output channels, stored as one 16-byte vector
__device__ __forceinline__ int a_row(int i, int rho) { return 32 * (i >> 1) + 8 * (rho >> 2) + 4 * (i & 1) + (rho & 3); }

// 16 bytes from rsrc + voff (per lane) + soff (wave-uniform) to LDS (buffer_load_dwordx4 ... lds).  Kept out
// of the kernel's lambdas: an amdgcn builtin called directly inside them makes hipcc drop the host launch
// stub of the kernel template (declared, never defined: an undefined symbol at load time)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// bf16 element `hi` (0: low half, 1: high half) of a packed dword, as float
__device__ __forceinline__ float bf_lo(uint32_t d, int hi) {
  return __uint_as_float(hi ? (d & 0xffff0000u) : (d << 16));
}

__device__ __forceinline__ void dma16b(__amdgpu_buffer_rsrc_t rs, uint32_t voff, int soff, void* lds_dst) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void_t*)lds_dst, 16, voff, soff, 0, 0);
}

template <int V>
struct IC {
  static constexpr int value = V;
};

struct Geo {
  int N, H, C, K;
  int cblk;     // C / 64
  int ntiles;   // N * H / TR
  int ctiles;   // K / BCO
  int groups;   // blocks per co tile (persistent)
  uint32_t wbytes;
};

struct EpiArgs {
  const bf16_t* yb;      // BN input [M][K] (EPI 2, 3)
  const uint8_t* mask;   // ReLU bit mask [M][K/8] (EPI 2)
  const float* mean;     // [K]
  const float* scale;    // [K] (EPI 3)
  const float* shift;    // [K] (EPI 3)
};

struct ProArgs {
  const bf16_t* res;     // PRO 2: y
  const float* scale;    // PRO 1: folded BN scale; PRO 2: A
  const float* shift;    // PRO 1: folded BN shift; PRO 2: Cc
  const float* rscale;   // PRO 2: B
  bf16_t* aout;          // the transformed operand [M][C] (tile rows only), or null
};

// TR image rows x W pixels per tile; BCO output channels per block; 8 waves = WCO co-waves x (8 / WCO) pixel
// waves; NB halo buffers (2: the next unit's halo is written during this unit's taps; 1: between units).
// Halo layout (chunk-planar): the 16-byte channel chunk c (channels 8c .. 8c + 7 of the unit) of halo slot
// s is at c * PLANE + 16 * s.  A 16-lane fragment row covers 16 consecutive slots of ONE image row (the
// pixel lanes are row-padded to WR = W rounded up to 16), and the ds_read_b128 lane groups
// ({0-3, 12-15 | 20-27}, ...) mix two chunks of 8 + 8 slots: with PLANE a multiple of 256 bytes the 16
// addresses of a group always fall in 16 distinct bank quads -- no swizzle, no conflict.
template <int W, int TR, int BCO, int WCO, int NB, int RES>
struct Shape {
  static constexpr int NW = 8;
  static constexpr int RS = W + 2;                        // slots per halo row (zero column at both ends)
  static constexpr int HS = (TR + 2) * RS;                // halo slots
  static constexpr int WR = (W + 15) / 16 * 16;           // pixel lanes per image row
  static constexpr int XS = WR + 2 > RS ? WR + 2 - RS : 0;  // slots past HS that idle lanes read
  static constexpr int PLANE = ((HS + XS) * 16 + 255) / 256 * 256;
  static constexpr int HB = 8 * PLANE;                    // halo buffer bytes (64 channels)
  static constexpr int P = TR * WR;                       // lane pixels per tile (row-padded)
  static constexpr int PW = NW / WCO;                     // pixel waves
  static constexpr int PL = (P + 16 * PW - 1) / (16 * PW) * (16 * PW);
  static constexpr int TP = PL / PW, TCO = BCO / WCO;
  static constexpr int FI = TCO / 16, FJ = TP / 16;
  static constexpr int NT = 64 * NW;
  static constexpr int NCH = (HS * 8 + NT - 1) / NT;      // halo 16-byte chunks per thread
  static constexpr int NIW = BCO / (8 * NW);              // weight DMA instructions per wave per tap
  static constexpr int WSLOT = BCO * kBK * 2;             // bytes per weight ring slot
  // weight ring slots: 5 (DMA 4 taps ahead); RES: 9, one per tap, the 64-channel layer's whole filter
  // resident in LDS for the launch (C == 64: every unit has the same weights)
  static constexpr int RING = RES ? 9 : 5;
  static constexpr int LDS = NB * HB + RING * WSLOT + 3 * BCO * 4;  // + the PRO coefficients [2 or 3][C] fp32
  static_assert(FI % 2 == 0 && FJ >= 1 && BCO % (8 * NW) == 0 && WCO * PW == NW && (NB == 1 || NB == 2), "bad tile");
  static_assert(NT % 128 == 0 && NCH <= 16, "halo staging map");
  static_assert(4 * PLANE + ((2 * RS + 2) * 16) < 65536, "ds_read immediate offsets");
};

template <int W, int TR, int BCO, int WCO, int NB, int RES, int EPI, int PRO>
__global__ void __launch_bounds__(512, 1)
conv3x3v2_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ w, bf16_t* __restrict__ y,
                 float* __restrict__ part, Geo g, EpiArgs ea, ProArgs pa) {
  using S = Shape<W, TR, BCO, WCO, NB, RES>;
  static_assert(!RES || NB == 1, "resident weights: one halo buffer");
  constexpr int NW = S::NW;
  constexpr int FI = S::FI, FJ = S::FJ, NT = S::NT, NCH = S::NCH, NIW = S::NIW, RING = S::RING;
  constexpr bool SUMS = EPI != kEpiNone;
  constexpr int LPC = PRO == 2 ? 2 : 1;  // global loads per halo chunk
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* halo = lds;                             // [NB][HB]
  char* wts = lds + NB * S::HB;                 // [RING][BCO][64] bf16, swizzled
  float* prm = reinterpret_cast<float*>(wts + RING * S::WSLOT);  // [3][BCO]: mean, scale, shift
  float* ppar = reinterpret_cast<float*>(lds + S::LDS);           // PRO: [3][C] scale, shift, rscale

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int rho = lane & 15, lg = lane >> 4;
  const int wco0 = (wave % WCO) * S::TCO, wp0 = (wave / WCO) * S::TP;

  // block -> (co tile, contiguous tile run); remapped ids keep consecutive runs on one XCD
  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ct = rid % g.ctiles, grp = rid / g.ctiles;
  const int t_begin = static_cast<int>(static_cast<int64_t>(grp) * g.ntiles / g.groups);
  const int t_end = static_cast<int>(static_cast<int64_t>(grp + 1) * g.ntiles / g.groups);
  const int units = (t_end - t_begin) * g.cblk;
  const int nitems = units * 9;
  const int tiles_per_img = g.H / TR;

  if (EPI >= kEpiBnbM) {
    for (int t = tid; t < BCO; t += NT) {
      const int co = ct * BCO + t;
      prm[t] = ea.mean[co];
      prm[BCO + t] = EPI == kEpiBnbR ? ea.scale[co] : 0.f;
      prm[2 * BCO + t] = EPI == kEpiBnbR ? ea.shift[co] : 0.f;
    }
  }
  if (PRO) {
    for (int t = tid; t < g.C; t += NT) {
      ppar[t] = pa.scale[t];
      ppar[g.C + t] = pa.shift[t];
      if (PRO == 2) ppar[2 * g.C + t] = pa.rscale[t];
    }
  }

  // ---- halo staging roles (tile-invariant): chunk u = tid + NT * i -> channel chunk hc = (u >> 4) & 7 (the
  // same for every i), slot (u & 15) + 16 * (u >> 7): 16 consecutive lanes write 16 consecutive slots
  // Loads are buffer loads from a per-unit resource based at halo slot 0's pixel (image row h0 - 1, column
  // -1): a chunk's byte offset hoff is the same for every unit, and a chunk outside the image gets offset
  // 2^31, past the resource's range, which the hardware answers with zeros -- no address arithmetic or
  // zero-select per chunk.
  const int hc = (tid >> 4) & 7;
  uint32_t hoff[NCH];    // byte offset of the chunk from halo slot 0's pixel, channel block 0
  uint32_t ok_s = 0, top_m = 0, bot_m = 0, in_m = 0;  // bit i: chunk i inside the image columns / in halo
                                                      // row 0 / in halo row TR + 1 / a halo slot at all
  // chunk i's slot is slot0 + 2 NT / 16 * i: its LDS offset is hlds0 + 2 NT * i (an immediate)
  const uint32_t hlds0 = static_cast<uint32_t>(hc * S::PLANE + ((tid & 15) + 16 * (tid >> 7)) * 16);
#pragma unroll
  for (int i = 0; i < NCH; ++i) {
    const int u = tid + NT * i, slot = (u & 15) + 16 * (u >> 7);
    const int hr = slot / S::RS, wc = slot - (slot / S::RS) * S::RS;
    const bool in = slot < S::HS;
    const bool ok = in && wc >= 1 && wc <= W;
    hoff[i] = static_cast<uint32_t>(((hr * W + wc) * g.C + hc * 8) * 2);
    ok_s |= (ok ? 1u : 0u) << i;
    top_m |= (in && hr == 0 ? 1u : 0u) << i;
    bot_m |= (in && hr == TR + 1 ? 1u : 0u) << i;
    in_m |= (in ? 1u : 0u) << i;
  }
  // a unit resource's range: through the last pixel of halo row TR + 1 ((TR + 2) W pixels past slot 0's)
  const uint32_t hbytes = static_cast<uint32_t>(((TR + 2) * W + 1) * g.C * 2);
  // ---- PRO == 0 with two halo buffers: no transform, so the halo goes global -> LDS by the buffer LDS-DMA
  // without registers.  Wave w fills plane w (channels 8w .. 8w + 7 of the unit) in NBK blocks of 64
  // consecutive slots (1 KiB each; the last block overlaps its predecessor -- duplicate writes of the same
  // data -- so no block crosses into the next plane)
  constexpr bool HDMA = PRO == 0 && NB == 2;
  constexpr int NSL = S::PLANE / 16, NBK = (NSL + 63) / 64;
  static_assert(NSL >= 64, "halo DMA blocks");
  auto blk0 = [](int b) __attribute__((always_inline)) { return 64 * b < NSL - 64 ? 64 * b : NSL - 64; };
  uint32_t dof[NBK];
  uint32_t dok = 0, dtop = 0, dbot = 0;  // bit b: as ok_s / top_m / bot_m for the lane's slot of block b
  if (HDMA) {
#pragma unroll
    for (int b = 0; b < NBK; ++b) {
      const int slot = blk0(b) + lane;
      const int hr = slot / S::RS, wc = slot - (slot / S::RS) * S::RS;
      const bool in = slot < S::HS;
      dof[b] = static_cast<uint32_t>(((hr * W + wc) * g.C + wave * 8) * 2);
      dok |= (in && wc >= 1 && wc <= W ? 1u : 0u) << b;
      dtop |= (in && hr == 0 ? 1u : 0u) << b;
      dbot |= (in && hr == TR + 1 ? 1u : 0u) << b;
    }
  }
  // ---- B-fragment bases: lane pixel p = wp0 + 16 j + rho = (image row p / WR, column p % WR) -> slot of
  // tap (0, 0) = row * RS + column; chunk lg of k-half 0 (k-half 1: + 4 planes, an immediate)
  uint32_t bb[2][FJ];
#pragma unroll
  for (int j = 0; j < FJ; ++j) {
    const int p = wp0 + 16 * j + rho;
    const int s0 = p < S::P ? (p / S::WR) * S::RS + (p - (p / S::WR) * S::WR) : 0;
    bb[0][j] = static_cast<uint32_t>(s0 * 16 + lg * S::PLANE);
    bb[1][j] = bb[0][j] + (NB == 2 ? S::HB : 0);
  }
  // ---- A-fragment (weight) offsets in ring slot 0 (+ slot * WSLOT per item)
  const uint32_t wts_b = static_cast<uint32_t>(NB * S::HB);
  uint32_t aoff[2][FI];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < FI; ++i) {
      const int row = wco0 + a_row(i, rho);
      aoff[kk][i] = wts_b + 2u * static_cast<uint32_t>(row * kBK + (((kk * 4 + lg) ^ swz(row)) << 3));
    }
  // ---- weight DMA roles: lane -> (row within its 8-row piece, 16-byte chunk)
  const int prow = lane >> 3, dslot = lane & 7;
  const int64_t Ktot = 9LL * g.C;
  uint32_t wvoff[NIW];
#pragma unroll
  for (int i = 0; i < NIW; ++i) {
    const int co = 8 * (wave + NW * i) + prow;
    wvoff[i] = static_cast<uint32_t>(((static_cast<int64_t>(ct) * BCO + co) * Ktot + ((dslot ^ swz(co)) << 3)) * 2);
  }
  const __amdgpu_buffer_rsrc_t rs_w =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(w), 0, static_cast<int>(g.wbytes), 0x00020000);

  auto unit_tile = [&](int u) __attribute__((always_inline)) { return t_begin + u / g.cblk; };
  auto unit_cb = [&](int u) __attribute__((always_inline)) { return u - (u / g.cblk) * g.cblk; };

  // weight item = unit * 9 + tap, DMA'd into ring slot item % RING; soff: the tap's and channel block's
  // byte offset in a weight row (wave-uniform)
  auto issue_w = [&](int soff, int slot) __attribute__((always_inline)) {
    char* dst = wts + slot * S::WSLOT;
#pragma unroll
    for (int i = 0; i < NIW; ++i)
      dma16b(rs_w, wvoff[i], soff, dst + 8 * (wave + NW * i) * kBK * 2);
  };
  auto ring = [](int s0, int k) __attribute__((always_inline)) {  // (s0 + k) % RING for s0 < RING, k < 3 RING
    int r = s0 + k;
    r = r >= 2 * RING ? r - 2 * RING : r;
    return r >= RING ? r - RING : r;
  };
  static_assert(8 + RING - 1 + RING - 1 < 4 * RING, "ring(): slot + tap lookahead range");

  // ---- register-staged halo of one unit (native vectors: an aggregate select would go to scratch).  Three
  // steps: load (global -> registers), transform (PRO: BN affine / ReLU / residual, zero outside the image,
  // packed to bf16 in place) and write (registers -> LDS, plus the transformed operand to pa.aout).  NB == 2:
  // loaded at tap 0, transformed and written at tap HST.  RES: loaded and transformed in two halves during
  // the unit's taps, written at the next unit boundary (between two barriers, so only the LDS stores remain
  // there)
  constexpr int HST = 5, NH = (NCH + 1) / 2;
  u32x4 hx[NCH], hy[PRO == 2 ? NCH : 1];
  int h_tile = 0, h_cb = 0;
  uint32_t h_ok = 0;  // bit i: chunk i of the staged unit holds image data
  auto load_halo = [&](int u, auto I0, auto I1) __attribute__((always_inline)) {
    constexpr int A = decltype(I0)::value, Z = decltype(I1)::value;
    if (A == 0) {
      h_tile = unit_tile(u);
      h_cb = unit_cb(u);
    }
    const int n = h_tile / tiles_per_img, h0 = (h_tile - n * tiles_per_img) * TR;
    if (A == 0) h_ok = ok_s & (h0 == 0 ? ~top_m : ~0u) & (h0 + TR == g.H ? ~bot_m : ~0u);
    const int64_t base = ((static_cast<int64_t>(n) * g.H + h0) * W - (W + 1)) * g.C + h_cb * kBK;
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x + base), 0, static_cast<int>(hbytes), 0x00020000);
    __amdgpu_buffer_rsrc_t rr = rx;
    if (PRO == 2)
      rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(pa.res + base), 0, static_cast<int>(hbytes),
                                             0x00020000);
#pragma unroll
    for (int i = A; i < Z; ++i) {
      const uint32_t off = (h_ok >> i) & 1u ? hoff[i] : 0x80000000u;
      hx[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
      if (PRO == 2) hy[i] = __builtin_amdgcn_raw_buffer_load_b128(rr, off, 0, 0);
    }
  };
  auto dma_halo = [&](int u, int buf) __attribute__((always_inline)) {  // HDMA
    const int tile = unit_tile(u), cb = unit_cb(u);
    const int n = tile / tiles_per_img, h0 = (tile - n * tiles_per_img) * TR;
    const uint32_t okm = dok & (h0 == 0 ? ~dtop : ~0u) & (h0 + TR == g.H ? ~dbot : ~0u);
    const int64_t base = ((static_cast<int64_t>(n) * g.H + h0) * W - (W + 1)) * g.C + cb * kBK;
    const __amdgpu_buffer_rsrc_t rx =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16_t*>(x + base), 0, static_cast<int>(hbytes), 0x00020000);
    char* dst = halo + buf * S::HB + wave * S::PLANE;
#pragma unroll
    for (int b = 0; b < NBK; ++b)
      dma16b(rx, (okm >> b) & 1u ? dof[b] : 0x80000000u, 0, dst + blk0(b) * 16);
  };
  auto xform_halo = [&](auto I0, auto I1) __attribute__((always_inline)) {  // PRO only
    constexpr int A = decltype(I0)::value, Z = decltype(I1)::value;
    if (!PRO) return;
    float fs[8], fh[8], fr[8];
    const int c0 = h_cb * kBK + hc * 8;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      fs[e] = ppar[c0 + e];
      fh[e] = ppar[g.C + c0 + e];
      fr[e] = PRO == 2 ? ppar[2 * g.C + c0 + e] : 0.f;
    }
#pragma unroll
    for (int i = A; i < Z; ++i) {
      const bool ok = (h_ok >> i) & 1u;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = bf_lo(hx[i][e >> 1], e & 1);
        const float t = PRO == 2 ? fs[e] * xv + fr[e] * bf_lo(hy[i][e >> 1], e & 1) + fh[e]
                                 : fmaxf(xv * fs[e] + fh[e], 0.f);
        v[e] = ok ? t : 0.f;
      }
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const u16v2_t pk = f2bf2(v[e], v[e + 1]);
        hx[i][e >> 1] = static_cast<uint32_t>(pk[0]) | (static_cast<uint32_t>(pk[1]) << 16);
      }
    }
  };
  auto write_halo = [&](int buf) __attribute__((always_inline)) {
    const int n = h_tile / tiles_per_img, h0 = (h_tile - n * tiles_per_img) * TR;
    // slot 0's pixel, channel block h_cb (elements)
    const int64_t slot0 = ((static_cast<int64_t>(n) * g.H + h0) * W - (W + 1)) * g.C + h_cb * kBK;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      if (!((in_m >> i) & 1u)) continue;  // beyond the halo (last round of chunks)
      // PRO == 0: zeros outside the image come from the out-of-range buffer loads
      *reinterpret_cast<u32x4*>(halo + buf * S::HB + hlds0 + 2 * NT * i) = hx[i];
      // the tile's own rows: the transformed operand is an output (weight gradient / BN backward)
      if (PRO && pa.aout != nullptr && ct == 0 && ((h_ok >> i) & 1u) && !((top_m >> i) & 1u) &&
          !((bot_m >> i) & 1u))
        *reinterpret_cast<u32x4*>(reinterpret_cast<char*>(pa.aout + slot0) + hoff[i]) = hx[i];
    }
  };
  auto store_halo = [&](int buf) __attribute__((always_inline)) {
    xform_halo(IC<0>{}, IC<NCH>{});
    write_halo(buf);
  };

  f4 acc[FI][FJ];
#pragma unroll
  for (int i = 0; i < FI; ++i)
#pragma unroll
    for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  // channel sums as pairs: the accumulation is packed fp32 math (v_pk_add_f32 / v_pk_fma_f32), half the VALU
  f2 st_s[FI / 2][4], st_q[FI / 2][4];
#pragma unroll
  for (int q = 0; q < FI / 2; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) { st_s[q][e] = f2{0.f, 0.f}; st_q[q][e] = f2{0.f, 0.f}; }

  // ---- epilogue of one tile: lane (lg, rho) holds channels wco0 + 32q + 8lg + 0..7 of lane pixel p_j
  auto epilogue = [&](int tile) __attribute__((always_inline)) {
    const int n = tile / tiles_per_img, h0 = (tile - n * tiles_per_img) * TR;
    const int64_t m0 = (static_cast<int64_t>(n) * g.H + h0) * W;
#pragma unroll
    for (int j = 0; j < FJ; ++j) {
      const int p = wp0 + 16 * j + rho;
      const int pr = p / S::WR, pc = p - (p / S::WR) * S::WR;
      const bool okp = p < S::P && pc < W;
      const int64_t m = m0 + (okp ? pr * W + pc : 0);
      u32x4 yr[FI / 2];
      uint32_t mb[FI / 2];
      if (EPI >= kEpiBnbM) {
#pragma unroll
        for (int q = 0; q < FI / 2; ++q) {
          const int64_t off = m * g.K + static_cast<int64_t>(ct) * BCO + wco0 + 32 * q + 8 * lg;
          yr[q] = *reinterpret_cast<const u32x4*>(ea.yb + off);
          if (EPI == kEpiBnbM) mb[q] = ea.mask[off >> 3];
        }
      }
#pragma unroll
      for (int q = 0; q < FI / 2; ++q) {
        const int cl = wco0 + 32 * q + 8 * lg;
        float o[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) { o[e] = acc[2 * q][j][e]; o[4 + e] = acc[2 * q + 1][j][e]; }
        float yv[8];
        if (EPI >= kEpiBnbM) {
#pragma unroll
          for (int e = 0; e < 8; ++e) yv[e] = bf_lo(yr[q][e >> 1], e & 1);
          if (EPI == kEpiBnbM) {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = (mb[q] >> e) & 1u ? o[e] : 0.f;
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = yv[e] * prm[BCO + cl + e] + prm[2 * BCO + cl + e] > 0.f ? o[e] : 0.f;
          }
        }
        u32x4 v;
#pragma unroll
        for (int e = 0; e < 8; e += 2) {
          const u16v2_t pk = f2bf2(o[e], o[e + 1]);
          v[e >> 1] = static_cast<uint32_t>(pk[0]) | (static_cast<uint32_t>(pk[1]) << 16);
        }
        if (okp) {
          *reinterpret_cast<u32x4*>(y + m * g.K + static_cast<int64_t>(ct) * BCO + cl) = v;
          if (EPI == kEpiStats) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f2 ov = {o[2 * e], o[2 * e + 1]};
              st_s[q][e] += ov;
              st_q[q][e] = __builtin_elementwise_fma(ov, ov, st_q[q][e]);
            }
          } else if (EPI >= kEpiBnbM) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f2 fv = {bf_lo(v[e], 0), bf_lo(v[e], 1)};
              const f2 dv = f2{yv[2 * e], yv[2 * e + 1]} - f2{prm[cl + 2 * e], prm[cl + 2 * e + 1]};
              st_s[q][e] += fv;
              st_q[q][e] = __builtin_elementwise_fma(fv, dv, st_q[q][e]);
            }
          }
        }
      }
    }
#pragma unroll
    for (int i = 0; i < FI; ++i)
#pragma unroll
      for (int j = 0; j < FJ; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  };

  const char* lds_c = lds;
  auto ld = [&](uint32_t off) __attribute__((always_inline)) { return *reinterpret_cast<const s8*>(lds_c + off); };

  // one register set of fragments, read after the tap's barrier (the other wave on the SIMD multiplies
  // meanwhile)
  s8 fa[2][FI], fb[2][FJ];
  // load the fragments of an item (tap T, halo buffer B: compile-time; its weights in ring slot `slot`)
  auto fetch = [&](auto TT, auto BUF, int slot) __attribute__((always_inline)) {
    constexpr int T = decltype(TT)::value, B = decltype(BUF)::value;
    constexpr uint32_t toff = static_cast<uint32_t>(((T / 3) * S::RS + (T % 3)) * 16);
    const uint32_t roff = static_cast<uint32_t>(slot * S::WSLOT);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < FI; ++i) fa[kk][i] = ld(aoff[kk][i] + roff);
#pragma unroll
      for (int j = 0; j < FJ; ++j) fb[kk][j] = ld(bb[B][j] + toff + kk * 4 * S::PLANE);
    }
  };

  // ---- prologue: unit 0's halo into buffer 0, weight items 0 .. 3 in flight (RES: all 9 taps)
  constexpr int PRE = RES ? 9 : RING - 1;
  if (units > 0) {
    if constexpr (HDMA) {
      dma_halo(0, 0);
    } else {
      load_halo(0, IC<0>{}, IC<NCH>{});
      if (PRO) __syncthreads();  // ppar
      store_halo(0);
    }
    const int cb0 = unit_cb(0), cb1 = units > 1 ? unit_cb(1) : 0;
#pragma unroll
    for (int it = 0; it < PRE; ++it)
      if (it < nitems) issue_w(((it < 9 ? it : it - 9) * g.C + (it < 9 ? cb0 : cb1) * kBK) * 2, it);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }

  // one tap: item it = u * 9 + T.  rs0: ring slot of item u * 9; wo_u / wo_n: channel-block byte offsets of
  // units u and u + 1 in a weight row
  auto tap = [&](auto TT, auto BUF, int u, int it, int rs0, int wo_u, int wo_n) __attribute__((always_inline)) {
    constexpr int T = decltype(TT)::value, B = decltype(BUF)::value;
    // item it's weights landed (own DMA; the barrier makes every wave's visible).  Younger VMEM ops: the
    // DMAs of items it+1 .. it+3 and, at taps 1 .. 4, the next unit's halo loads issued at tap 0 after the
    // DMA of item it (VMEM loads complete in issue order)
    constexpr int YH = (T >= 1 && T <= 4) ? (HDMA ? NBK : NCH * LPC) : 0;
    const bool hl = YH > 0 && u + 1 < units;
    if (it + 3 < nitems) {
      if (hl) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * NIW + YH) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * NIW) : "memory");
    } else if (it + 2 < nitems) {
      if (hl) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NIW + YH) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NIW) : "memory");
    } else if (it + 1 < nitems) {
      if (hl) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIW + YH) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NIW) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // own halo stores and the last item's fragments
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (it + RING - 1 < nitems) {  // item it+4: its slot last held item it-1 (read before the barrier)
      constexpr int TN = T + RING - 1;
      issue_w(TN < 9 ? TN * 2 * g.C + wo_u : (TN - 9) * 2 * g.C + wo_n, ring(rs0, TN));
    }
    if (NB == 1 && T == 0 && u > 0) {  // this unit's halo (staged during unit u-1), once every wave is past
      store_halo(0);                     // unit u-1's last fragment reads (the barrier above)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (u + 1 < units) {  // NB == 2: halo buffer B^1 was last read by unit u-1
      if constexpr (HDMA) {
        if (T == 0) dma_halo(u + 1, B ^ 1);
      } else {
        if (T == 0) load_halo(u + 1, IC<0>{}, IC<NCH>{});
        if (NB == 2 && T == HST) store_halo(B ^ 1);
      }
    }
    fetch(TT, BUF, ring(rs0, T));
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(fa[kk][i], fb[kk][j], acc[i][j]);
  };
  // RES: no weight traffic after the prologue, so no per-tap wait or barrier -- the waves only meet at unit
  // boundaries, where the single halo buffer is rewritten
  auto tap_res = [&](auto TT, int u) __attribute__((always_inline)) {
    constexpr int T = decltype(TT)::value;
    if (T == 0 && u > 0) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is past unit u-1's fragment reads
      asm volatile("" ::: "memory");
      write_halo(0);  // transformed during unit u-1
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    if (u + 1 < units) {
      if (T == 0) load_halo(u + 1, IC<0>{}, IC<NH>{});
      if (T == 3) {
        xform_halo(IC<0>{}, IC<NH>{});
        asm volatile("" ::: "memory");  // keep the second half's loads here (register pressure)
        load_halo(u + 1, IC<NH>{}, IC<NCH>{});
      }
      if (T == 7) xform_halo(IC<NH>{}, IC<NCH>{});
    }
    fetch(TT, IC<0>{}, T);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int i = 0; i < FI; ++i)
#pragma unroll
        for (int j = 0; j < FJ; ++j) acc[i][j] = mfma(fa[kk][i], fb[kk][j], acc[i][j]);
  };
  auto unit_body = [&](auto BUF, int u) __attribute__((always_inline)) {
    if constexpr (RES) {
      tap_res(IC<0>{}, u);
      tap_res(IC<1>{}, u);
      tap_res(IC<2>{}, u);
      tap_res(IC<3>{}, u);
      tap_res(IC<4>{}, u);
      tap_res(IC<5>{}, u);
      tap_res(IC<6>{}, u);
      tap_res(IC<7>{}, u);
      tap_res(IC<8>{}, u);
      epilogue(unit_tile(u));
      return;
    }
    // BUF = u & 1: the unit's halo buffer
    const int it = u * 9;
    const int rs0 = it % RING;
    const int wo_u = unit_cb(u) * kBK * 2, wo_n = u + 1 < units ? unit_cb(u + 1) * kBK * 2 : 0;
    tap(IC<0>{}, BUF, u, it, rs0, wo_u, wo_n);
    tap(IC<1>{}, BUF, u, it + 1, rs0, wo_u, wo_n);
    tap(IC<2>{}, BUF, u, it + 2, rs0, wo_u, wo_n);
    tap(IC<3>{}, BUF, u, it + 3, rs0, wo_u, wo_n);
    tap(IC<4>{}, BUF, u, it + 4, rs0, wo_u, wo_n);
    tap(IC<5>{}, BUF, u, it + 5, rs0, wo_u, wo_n);
    tap(IC<6>{}, BUF, u, it + 6, rs0, wo_u, wo_n);
    tap(IC<7>{}, BUF, u, it + 7, rs0, wo_u, wo_n);
    tap(IC<8>{}, BUF, u, it + 8, rs0, wo_u, wo_n);
    if (unit_cb(u) == g.cblk - 1) epilogue(unit_tile(u));
  };
  for (int u = 0; u < units; u += 2) {
    unit_body(IC<0>{}, u);
    if (u + 1 < units) unit_body(IC<1>{}, u + 1);
  }

  if (SUMS) {  // block reduction of the channel sums into part[grp][2][K]
#pragma unroll
    for (int q = 0; q < FI / 2; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          st_s[q][e >> 1][e & 1] += __shfl_xor(st_s[q][e >> 1][e & 1], o, 64);
          st_q[q][e >> 1][e & 1] += __shfl_xor(st_q[q][e >> 1][e & 1], o, 64);
        }
    __syncthreads();
    constexpr int WPW = S::PW;
    float* red = reinterpret_cast<float*>(lds);  // [WPW][2][BCO]
    const int wpi = wave / WCO;
    if (rho == 0) {
#pragma unroll
      for (int q = 0; q < FI / 2; ++q)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int co = wco0 + 32 * q + 8 * lg + e;
          red[(wpi * 2) * BCO + co] = st_s[q][e >> 1][e & 1];
          red[(wpi * 2 + 1) * BCO + co] = st_q[q][e >> 1][e & 1];
        }
    }
    __syncthreads();
    for (int t = tid; t < 2 * BCO; t += NT) {
      const int which = t / BCO, co = t - which * BCO;
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < WPW; ++k) s += red[(k * 2 + which) * BCO + co];
      part[(static_cast<int64_t>(grp) * 2 + which) * g.K + static_cast<int64_t>(ct) * BCO + co] = s;
    }
  }
}

// ============================================================ 3x3 / stride-1 weight gradient
// dW[co][r][s][ci] = sum_p dY[p][co] x[p + (r - 1, s - 1)][ci] on the same whole-row tiles: a stage is TR
// image rows of one image -- the dY tile (64 output channels) and the input's zero-padded halo (64 input
// channels) -- both LDS-DMA'd as 8-channel planes (out-of-range offsets give the zero border), and each
// wave reduces the stage's pixels into all 9 taps of its (32 co x 16 ci) tile.  The MFMA's reduction
// index is the pixel, so both operands are read with ds_read_b64_tr_b16 (4 pixels x 16 channels per
// 16-lane group, delivered channel-major): a lane's address is (its pixel slot, its plane) -- a lane base
// register per 16-pixel half-step and immediates for the tap, plane and step: no VALU per read.  Plane
// pitches are 128 (mod 256) bytes, so the two planes a 32-lane half touches sit 32 banks apart.  Lane
// pixels are row-padded to a multiple of 4 (a transposed read's 4 rows stay in one image row); pad pixels
// carry zero dY.  Blocks = (64 co, 64 ci) tiles x pixel splits; every block writes its partial dW slab
// and conv_igemm.hip's wgrad_finalize_kernel sums them (deterministic).
// Reference counterpart: the cuDNN weight-gradient call in harness/determined/pytorch/_pytorch_trial.py's
// training step (backward of torch.nn.Conv2d).
typedef short s4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4 lds_s4;

constexpr int wpitch(int b) { return b <= 128 ? 128 : (b - 128 + 255) / 256 * 256 + 128; }

template <int W, int TR, int WR_>
struct WShape {
  static constexpr int WR = WR_;               // lane pixels per image row (>= W, a multiple of 4)
  static constexpr int PV = TR * WR;           // lane pixels of the stage's rows
  static constexpr int P = (PV + 31) / 32 * 32;  // lane pixels per stage (pixels >= PV: zero dY)
  static constexpr int KS = P / 32;            // k-steps per stage
  static constexpr int RS = W + 2, HS = (TR + 2) * RS;
  // slots the taps of every lane pixel read (pad pixels' reads past HS hit zeros or finite data times zero dY)
  static constexpr int XR = ((P - 1) / WR + 2) * RS + WR + 2;
  static constexpr int XPL = wpitch((XR > HS ? XR : HS) * 16);  // x halo plane pitch (8 channels)
  static constexpr int DPL = wpitch(P * 16);                // dY plane pitch
  static constexpr int XB = 8 * XPL, SB = XB + 8 * DPL;     // x image / stage bytes
  static constexpr int LDS = 2 * SB;
  static constexpr int NXS = XPL / 16, NXB = (NXS + 63) / 64;  // x plane slots, 64-slot DMA blocks
  static constexpr int NDB = (P + 63) / 64;                    // dY 64-pixel DMA blocks
  static_assert(WR >= W && WR % 4 == 0 && P % 32 == 0 && P >= 64 && NXS >= 64 && NXB <= 32 && NDB <= 32,
                "wgrad stage shape");
};

struct WGeo {
  int N, H, C, K;
  int cotiles, cblks, splits, stages;  // stages = N * H / TR
};

// RG = 0: both images by LDS-DMA (lane-linear 1 KiB writes: each lane fetches 16 bytes of a different pixel,
// 8x the cache-line traffic of the bytes used); RG = 1: register-staged with 8 consecutive lanes per pixel
// (one 128-byte line), ds_write_b128 into the planes, loaded at the top of a stage and written mid-stage.
template <int W, int TR, int WR, int RG>
__global__ void __launch_bounds__(512, 1)
conv3x3v2_wgrad_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, float* __restrict__ part,
                       WGeo g) {
  using S = WShape<W, TR, WR>;
  constexpr int KS = S::KS;
  constexpr int NXC = (S::NXS * 8 + 511) / 512, NDC = (S::P * 8 + 511) / 512;  // RG: chunks per thread
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int wco = wave >> 2, cig = wave & 3;  // 32 output channels x 16 input channels per wave

  const int nblk = gridDim.x, L = blockIdx.x;
  const int xcd = L & 7, q8 = nblk >> 3, r8 = nblk & 7;
  const int rid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (L >> 3);
  const int ntile = g.cotiles * g.cblks;
  const int tile = rid % ntile, split = rid / ntile;
  const int cot = tile % g.cotiles, cb = tile / g.cotiles;
  const int s_begin = static_cast<int>(static_cast<int64_t>(split) * g.stages / g.splits);
  const int s_end = static_cast<int>(static_cast<int64_t>(split + 1) * g.stages / g.splits);
  const int items = s_end - s_begin;
  const int tiles_per_img = g.H / TR;

  // ---- DMA roles: wave w fills x plane w (input channels 8w .. 8w + 7 of the block) and dY plane w
  // (output channels 8w .. 8w + 7) in 64-slot blocks; the last block of a plane overlaps its predecessor
  auto bx0 = [](int b) __attribute__((always_inline)) { return 64 * b < S::NXS - 64 ? 64 * b : S::NXS - 64; };
  auto bd0 = [](int b) __attribute__((always_inline)) { return 64 * b < S::P - 64 ? 64 * b : S::P - 64; };
  uint32_t xof[S::NXB], dof[S::NDB];
  uint32_t xok = 0, xtop = 0, xbot = 0, dok = 0;
#pragma unroll
  for (int b = 0; b < S::NXB; ++b) {
    const int slot = bx0(b) + lane;
    const int hr = slot / S::RS, wc = slot - (slot / S::RS) * S::RS;
    const bool in = slot < S::HS;
    xof[b] = static_cast<uint32_t>(((hr * W + wc) * g.C + wave * 8) * 2);
    xok |= (in && wc >= 1 && wc <= W ? 1u : 0u) << b;
    xtop |= (in && hr == 0 ? 1u : 0u) << b;
    xbot |= (in && hr == TR + 1 ? 1u : 0u) << b;
  }
#pragma unroll
  for (int b = 0; b < S::NDB; ++b) {
    const int p = bd0(b) + lane;
    const int row = p / S::WR, col = p - (p / S::WR) * S::WR;
    dof[b] = static_cast<uint32_t>(((row * W + col) * g.K + wave * 8) * 2);
    dok |= (p < S::PV && col < W ? 1u : 0u) << b;
  }
  const uint32_t xbytes = static_cast<uint32_t>(((TR + 2) * W + 1) * g.C * 2);
  const uint32_t dbytes = static_cast<uint32_t>(TR * W * g.K * 2);
  // ---- RG staging roles: chunk u = tid + 512 i -> (slot or pixel u >> 3, 8-channel plane u & 7)
  uint32_t rxo[RG ? NXC : 1], rdo[RG ? NDC : 1];
  uint32_t rxok = 0, rxtop = 0, rxbot = 0, rdok = 0, rxin = 0, rdin = 0;
  if (RG) {
#pragma unroll
    for (int i = 0; i < NXC; ++i) {
      const int u = tid + 512 * i, slot = u >> 3, c = u & 7;
      const int hr = slot / S::RS, wc = slot - (slot / S::RS) * S::RS;
      const bool in = slot < S::HS;
      rxo[i] = static_cast<uint32_t>(((hr * W + wc) * g.C + c * 8) * 2);
      rxok |= (in && wc >= 1 && wc <= W ? 1u : 0u) << i;
      rxtop |= (in && hr == 0 ? 1u : 0u) << i;
      rxbot |= (in && hr == TR + 1 ? 1u : 0u) << i;
      rxin |= (slot < S::NXS ? 1u : 0u) << i;
    }
#pragma unroll
    for (int i = 0; i < NDC; ++i) {
      const int u = tid + 512 * i, p = u >> 3, c = u & 7;
      const int row = p / S::WR, col = p - (p / S::WR) * S::WR;
      rdo[i] = static_cast<uint32_t>(((row * W + col) * g.K + c * 8) * 2);
      rdok |= (p < S::PV && col < W ? 1u : 0u) << i;
      rdin |= (p < S::P ? 1u : 0u) << i;
    }
  }
  const uint32_t rxl = static_cast<uint32_t>((tid & 7) * S::XPL + (tid >> 3) * 16);
  const uint32_t rdl = static_cast<uint32_t>(S::XB + (tid & 7) * S::DPL + (tid >> 3) * 16);
  u32x4 rxv[RG ? NXC : 1], rdv[RG ? NDC : 1];
  auto rg_load = [&](int st) __attribute__((always_inline)) {
    const int n = st / tiles_per_img, h0 = (st - n * tiles_per_img) * TR;
    const int64_t pix0 = (static_cast<int64_t>(n) * g.H + h0) * W;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(x + (pix0 - (W + 1)) * g.C + cb * 64), 0, static_cast<int>(xbytes), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(dy + pix0 * g.K + cot * 64), 0, static_cast<int>(dbytes), 0x00020000);
    const uint32_t okm = rxok & (h0 == 0 ? ~rxtop : ~0u) & (h0 + TR == g.H ? ~rxbot : ~0u);
#pragma unroll
    for (int i = 0; i < NXC; ++i)
      rxv[i] = __builtin_amdgcn_raw_buffer_load_b128(rx, (okm >> i) & 1u ? rxo[i] : 0x80000000u, 0, 0);
#pragma unroll
    for (int i = 0; i < NDC; ++i)
      rdv[i] = __builtin_amdgcn_raw_buffer_load_b128(rd, (rdok >> i) & 1u ? rdo[i] : 0x80000000u, 0, 0);
  };
  auto rg_write = [&](int buf) __attribute__((always_inline)) {
    char* b = lds + buf * S::SB;
#pragma unroll
    for (int i = 0; i < NXC; ++i)
      if ((rxin >> i) & 1u) *reinterpret_cast<u32x4*>(b + rxl + 1024 * i) = rxv[i];
#pragma unroll
    for (int i = 0; i < NDC; ++i)
      if ((rdin >> i) & 1u) *reinterpret_cast<u32x4*>(b + rdl + 1024 * i) = rdv[i];
  };
  auto issue = [&](int st, int buf) __attribute__((always_inline)) {
    const int n = st / tiles_per_img, h0 = (st - n * tiles_per_img) * TR;
    const int64_t pix0 = (static_cast<int64_t>(n) * g.H + h0) * W;
    const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(x + (pix0 - (W + 1)) * g.C + cb * 64), 0, static_cast<int>(xbytes), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16_t*>(dy + pix0 * g.K + cot * 64), 0, static_cast<int>(dbytes), 0x00020000);
    const uint32_t okm = xok & (h0 == 0 ? ~xtop : ~0u) & (h0 + TR == g.H ? ~xbot : ~0u);
    char* xd = lds + buf * S::SB + wave * S::XPL;
    char* dd = lds + buf * S::SB + S::XB + wave * S::DPL;
#pragma unroll
    for (int b = 0; b < S::NXB; ++b) dma16b(rx, (okm >> b) & 1u ? xof[b] : 0x80000000u, 0, xd + bx0(b) * 16);
#pragma unroll
    for (int b = 0; b < S::NDB; ++b) dma16b(rd, (dok >> b) & 1u ? dof[b] : 0x80000000u, 0, dd + bd0(b) * 16);
  };

  // ---- transposed-read lane bases: lane 4q + p of a 16-lane group addresses row (pixel) q, columns
  // (channels) 4p .. 4p + 3 = plane p >> 1, byte 8 (p & 1) of the 16-byte slot; group lg takes pixels
  // 4lg .. 4lg + 3 of each 16-pixel half-step
  const int i16 = lane & 15, qq = i16 >> 2, pp = i16 & 3, lg = lane >> 4;
  const uint32_t a_l = static_cast<uint32_t>(S::XB + (4 * wco + (pp >> 1)) * S::DPL + 8 * (pp & 1) +
                                             16 * (4 * lg + qq));
  uint32_t b_l[KS][2];  // x slot of the lane's pixel for tap (0, 0), per half-step
#pragma unroll
  for (int ks = 0; ks < KS; ++ks)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int px = 32 * ks + 16 * h + 4 * lg + qq;
      const int row = px / S::WR, col = px - (px / S::WR) * S::WR;
      b_l[ks][h] = static_cast<uint32_t>((2 * cig + (pp >> 1)) * S::XPL + 8 * (pp & 1) + 16 * (row * S::RS + col));
    }
  auto tr8 = [&](uint32_t lo, uint32_t hi) __attribute__((always_inline)) {
    const s4 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + lo));
    const s4 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(lds + hi));
    s8 r;
    r[0] = a[0]; r[1] = a[1]; r[2] = a[2]; r[3] = a[3];
    r[4] = b[0]; r[5] = b[1]; r[6] = b[2]; r[7] = b[3];
    return r;
  };

  f4 acc[9][2];
#pragma unroll
  for (int t = 0; t < 9; ++t) acc[t][0] = acc[t][1] = f4{0.f, 0.f, 0.f, 0.f};

  if (items > 0) {
    if (RG) {
      rg_load(s_begin);
      rg_write(0);
    } else {
      issue(s_begin, 0);
    }
  }
  for (int it = 0; it < items; ++it) {
    if (RG) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();  // stage it landed for every wave; stage it-1 is no longer read
    if (it + 1 < items) {
      if (RG) rg_load(s_begin + it + 1);
      else issue(s_begin + it + 1, (it + 1) & 1);
    }
    const uint32_t sb = static_cast<uint32_t>((it & 1) * S::SB);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      if (RG && ks == KS / 2 && it + 1 < items) rg_write((it + 1) & 1);  // the other buffer: free since the barrier
      s8 a[2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
        a[i] = tr8(sb + a_l + 2 * i * S::DPL + 512 * ks, sb + a_l + 2 * i * S::DPL + 512 * ks + 256);
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const uint32_t toff = static_cast<uint32_t>(((t / 3) * S::RS + (t % 3)) * 16);
        const s8 b = tr8(sb + b_l[ks][0] + toff, sb + b_l[ks][1] + toff);
        acc[t][0] = mfma(a[0], b, acc[t][0]);
        acc[t][1] = mfma(a[1], b, acc[t][1]);
      }
    }
  }
  // acc[t][i][r] = partial dW[co = cot*64 + 32 wco + 16 i + 4 lg + r][tap t][ci = cb*64 + 16 cig + i16]
  const int64_t Ktot = 9LL * g.C;
  float* dst = part + static_cast<int64_t>(split) * g.K * Ktot;
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t co = static_cast<int64_t>(cot) * 64 + 32 * wco + 16 * i + 4 * lg + r;
        dst[co * Ktot + t * g.C + cb * 64 + 16 * cig + i16] = acc[t][i][r];
      }
}

// ------------------------------------------------------------------------------------------ host
struct V2Cfg {
  int W, TR, bco, wco, nb, res;
};
// 8 waves each.  0: 56x56 layers, 4-row tiles (64 co, 64x32 wave tiles); 1: 28x28 layers, 4-row tiles (128 co,
// 2 co-waves, 64x32); 2 / 3: 14x14 layers, one image per tile (64 co / 128 co with 2 co-waves, 64x64 tiles);
// 4: 56x56, 8-row tiles with 64x64 wave tiles (2/3 of the LDS reads per MFMA; the 10-row halo fits once:
// written between units); 5: 28x28, 7-row tiles, 128 co, 64x64 wave tiles (1/8 of the lanes idle); 6: as 4
// with the 64-channel filter resident in LDS (C == 64), no per-tap barrier
constexpr V2Cfg kV2[] = {{56, 4, 64, 1, 2, 0},  {28, 4, 128, 2, 2, 0}, {14, 14, 64, 1, 2, 0}, {14, 14, 128, 2, 2, 0},
                         {56, 8, 64, 1, 1, 0}, {28, 7, 128, 2, 2, 0}, {56, 8, 64, 1, 1, 1}};
constexpr int kNumV2 = sizeof(kV2) / sizeof(kV2[0]);

template <int W, int TR, int BCO, int WCO, int NB, int RES>
int lds_bytes() {
  return Shape<W, TR, BCO, WCO, NB, RES>::LDS;
}

int v2_lds(int cfg) {  // without the PRO coefficients
  switch (cfg) {
    case 0: return lds_bytes<56, 4, 64, 1, 2, 0>();
    case 1: return lds_bytes<28, 4, 128, 2, 2, 0>();
    case 2: return lds_bytes<14, 14, 64, 1, 2, 0>();
    case 3: return lds_bytes<14, 14, 128, 2, 2, 0>();
    case 4: return lds_bytes<56, 8, 64, 1, 1, 0>();
    case 5: return lds_bytes<28, 7, 128, 2, 2, 0>();
    default: return lds_bytes<56, 8, 64, 1, 1, 1>();
  }
}

}  // namespace c3v2
}  // namespace damd

using namespace damd;
using namespace damd::c3v2;

extern "C" {

int damd_v2_num_cfgs() { return kNumV2; }

// pro: the config is asked for with a BN prologue (1 / 2) -- every v2 config has one
int damd_v2_supported(int C, int K, int R, int S, int stride, int pad, int H, int W, int cfg) {
  if (cfg < 0 || cfg >= kNumV2) return 0;
  const V2Cfg c = kV2[cfg];
  return R == 3 && S == 3 && stride == 1 && pad == 1 && W == c.W && H > 0 && H % c.TR == 0 && C % kBK == 0 &&
         C > 0 && K % c.bco == 0 && (c.res == 0 || C == kBK) && v2_lds(cfg) + 12 * C <= 160 * 1024;
}

// stats-partial rows (= blocks per co tile) of a launch
int damd_v2_groups(int N, int H, int K, int cfg) {
  const V2Cfg c = kV2[cfg];
  const int ntiles = N * (H / c.TR), ctiles = K / c.bco;
  int g = (256 + ctiles - 1) / ctiles;
  if (g > ntiles) g = ntiles;
  return g < 1 ? 1 : g;
}

// Same argument contract as damd_conv_fwd_launch (conv_igemm.hip); no stream-K, no residual operand, no
// output phase, no compact second gradient.
int damd_v2_launch(const void* x, const void* w, void* y, float* part, int N, int H, int W, int C, int K, int R,
                   int S, int stride, int pad, int cfg, int groups, hipStream_t st, int epi, const void* d2,
                   const void* yb, const uint8_t* mask, const float* mean, const float* scale, const float* shift,
                   int pro, const void* p_res, const float* p_scale, const float* p_shift, const float* p_rscale,
                   void* p_aout, uint8_t* p_mout, float* sk_ws, int* sk_flags, int d2hw, int ophase) {
  (void)sk_ws;
  (void)sk_flags;
  (void)p_mout;
  if (!damd_v2_supported(C, K, R, S, stride, pad, H, W, cfg)) return -1;
  if (d2 != nullptr || d2hw != 0 || ophase != 0) return -6;
  if (pro < 0 || pro > 2 || (pro && (p_scale == nullptr || p_shift == nullptr)) ||
      (pro == 2 && (p_res == nullptr || p_rscale == nullptr)) || (pro == 1 && p_res != nullptr))
    return -4;
  if (epi < 0 || epi > 3 || (epi != 0 && part == nullptr)) return -3;
  if (epi >= 2 && (yb == nullptr || mean == nullptr || (epi == 2 && mask == nullptr) ||
                   (epi == 3 && (scale == nullptr || shift == nullptr))))
    return -3;
  const V2Cfg c = kV2[cfg];
  const int64_t wbytes = 9LL * C * K * 2;
  if (wbytes >= 0xF0000000LL || static_cast<int64_t>(N) * H * W >= (int64_t{1} << 31) - 4096) return -7;
  if (groups != damd_v2_groups(N, H, K, cfg)) return -5;
  Geo g;
  g.N = N; g.H = H; g.C = C; g.K = K;
  g.cblk = C / kBK;
  g.ntiles = N * (H / c.TR);
  g.ctiles = K / c.bco;
  g.groups = groups;
  g.wbytes = static_cast<uint32_t>(wbytes);
  const EpiArgs ea{static_cast<const bf16_t*>(yb), mask, mean, scale, shift};
  const ProArgs pa{static_cast<const bf16_t*>(p_res), p_scale, p_shift, p_rscale, static_cast<bf16_t*>(p_aout)};
  const dim3 grid(static_cast<unsigned>(g.ctiles * groups));
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* wp = static_cast<const bf16_t*>(w);
  bf16_t* yp = static_cast<bf16_t*>(y);
  const int lds = v2_lds(cfg) + (pro == 0 ? 0 : pro == 1 ? 8 * C : 12 * C);
#define V2L(W_, TR_, BCO_, WCO_, NB_, R_, E_, P_)                                                                 \
  do {                                                                                                       \
    auto* kfn = conv3x3v2_kernel<W_, TR_, BCO_, WCO_, NB_, R_, E_, P_>;                                           \
    DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    DAMD_LAUNCH(kfn, grid, dim3(512), lds, st, xp, wp, yp, part, g, ea, pa);                              \
  } while (0)
#define V2E(W_, TR_, BCO_, WCO_, NB_, R_)                                                                         \
  do {                                                                                                       \
    if (epi == 0 && pro == 0) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiNone, 0);                                     \
    else if (epi == 1 && pro == 0) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiStats, 0);                               \
    else if (epi == 1 && pro == 1) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiStats, 1);                               \
    else if (epi == 2 && pro == 0) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiBnbM, 0);                                \
    else if (epi == 3 && pro == 0) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiBnbR, 0);                                \
    else if (epi == 2 && pro == 2) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiBnbM, 2);                                \
    else if (epi == 3 && pro == 2) V2L(W_, TR_, BCO_, WCO_, NB_, R_, kEpiBnbR, 2);                                \
    else return -4;                                                                                          \
  } while (0)
  switch (cfg) {
    case 0: V2E(56, 4, 64, 1, 2, 0); break;
    case 1: V2E(28, 4, 128, 2, 2, 0); break;
    case 2: V2E(14, 14, 64, 1, 2, 0); break;
    case 3: V2E(14, 14, 128, 2, 2, 0); break;
    case 4: V2E(56, 8, 64, 1, 1, 0); break;
    case 5: V2E(28, 7, 128, 2, 2, 0); break;
    default: V2E(56, 8, 64, 1, 1, 1); break;
  }
#undef V2E
#undef V2L
  return 0;
}

// ---- weight gradient: 224 lane pixels (7 k-steps) per stage -- cfg 0: 56x56 layers, 4-row stages; 1: 28x28,
// 7 rows padded to 32 lanes; 2: 14x14, whole images padded to 16 lanes; 6: 7x7, whole images (8-lane rows,
// 56 + 8 zero pixels: 2 k-steps)
namespace {
struct V2WCfg {
  int W, TR, WR;
};
// cfg 3 .. 5: the same with register-staged, line-coalesced loads (RG = 1)
constexpr V2WCfg kV2W[] = {{56, 4, 56}, {28, 7, 32}, {14, 14, 16}, {56, 4, 56}, {28, 7, 32}, {14, 14, 16},
                           {7, 7, 8}, {7, 7, 8}};
int v2w_lds(int cfg) {
  if (cfg >= 6) return WShape<7, 7, 8>::LDS;
  switch (cfg % 3) {
    case 0: return WShape<56, 4, 56>::LDS;
    case 1: return WShape<28, 7, 32>::LDS;
    default: return WShape<14, 14, 16>::LDS;
  }
}
}  // namespace

int damd_v2w_num_cfgs() { return static_cast<int>(sizeof(kV2W) / sizeof(kV2W[0])); }

int damd_v2w_supported(int C, int K, int H, int W, int cfg) {
  if (cfg < 0 || cfg >= damd_v2w_num_cfgs()) return 0;
  const V2WCfg c = kV2W[cfg];
  return W == c.W && H > 0 && H % c.TR == 0 && C > 0 && C % 64 == 0 && K > 0 && K % 64 == 0 &&
         v2w_lds(cfg) <= 160 * 1024;
}

// partial-sum slabs of a launch (= pixel splits): about as many blocks as fit on the 256 CUs at once (the
// small 7x7 stages leave room for up to 3 blocks per CU) over all (co, ci) tiles
int damd_v2w_splits(int64_t N, int H, int C, int K, int cfg) {
  const int64_t tiles = static_cast<int64_t>(K / 64) * (C / 64);
  const int64_t stages = N * (H / kV2W[cfg].TR);
  int per_cu = 160 * 1024 / v2w_lds(cfg);
  per_cu = per_cu < 1 ? 1 : per_cu > 3 ? 3 : per_cu;
  int64_t sp = (256 * per_cu + tiles - 1) / tiles;
  if (sp > stages / 2) sp = stages / 2;
  return static_cast<int>(sp < 1 ? 1 : sp);
}

// x: [N, H, W, C]; dy: [N, H, W, K]; part: [splits][K][9 C] fp32 (summed by the caller)
int damd_v2w_launch(const void* x, const void* dy, float* part, int N, int H, int W, int C, int K, int cfg,
                    int splits, hipStream_t st) {
  if (!damd_v2w_supported(C, K, H, W, cfg)) return -1;
  const V2WCfg c = kV2W[cfg];
  if (static_cast<int64_t>(N) * H * W * (C > K ? C : K) >= (int64_t{1} << 31) - 4096) return -7;
  if (splits != damd_v2w_splits(N, H, C, K, cfg)) return -5;
  WGeo g;
  g.N = N; g.H = H; g.C = C; g.K = K;
  g.cotiles = K / 64;
  g.cblks = C / 64;
  g.splits = splits;
  g.stages = N * (H / c.TR);
  const dim3 grid(static_cast<unsigned>(g.cotiles * g.cblks * splits));
  const int lds = v2w_lds(cfg);
  const bf16_t* xp = static_cast<const bf16_t*>(x);
  const bf16_t* dp = static_cast<const bf16_t*>(dy);
#define V2W(W_, TR_, WR_, RG_)                                                                               \
  do {                                                                                                       \
    auto* kfn = conv3x3v2_wgrad_kernel<W_, TR_, WR_, RG_>;                                                           \
    DAMD_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, lds)); \
    DAMD_LAUNCH(kfn, grid, dim3(512), lds, st, xp, dp, part, g);                                              \
  } while (0)
  switch (cfg) {
    case 0: V2W(56, 4, 56, 0); break;
    case 1: V2W(28, 7, 32, 0); break;
    case 2: V2W(14, 14, 16, 0); break;
    case 3: V2W(56, 4, 56, 1); break;
    case 4: V2W(28, 7, 32, 1); break;
    case 5: V2W(14, 14, 16, 1); break;
    case 6: V2W(7, 7, 8, 0); break;
    default: V2W(7, 7, 8, 1); break;
  }
#undef V2W
  return 0;
}

}  // extern "C"
