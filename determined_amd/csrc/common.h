// Shared device helpers for the determined_amd CDNA4 (gfx950) kernels.
//
// Everything here is written for 64-lane wavefronts: reductions use 6 xor-shuffle
// steps, block sizes are multiples of 64, and bf16 data always moves in 16-byte
// vectors (8 x bf16) so a wave-instruction covers a full 1 KiB of contiguous HBM.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace damd {

constexpr int kWave = 64;

typedef uint16_t bf16_t;  // raw bf16 bits; converted explicitly (no __hip_bfloat16 overhead)

struct __attribute__((aligned(16))) bf16x8 { bf16_t v[8]; };
struct __attribute__((aligned(8))) bf16x4 { bf16_t v[4]; };

__device__ __forceinline__ float bf2f(bf16_t x) {
  return __uint_as_float(static_cast<uint32_t>(x) << 16);
}

typedef __bf16 bf16v2_t __attribute__((ext_vector_type(2)));
typedef float f32v2_t __attribute__((ext_vector_type(2)));
typedef uint16_t u16v2_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even fp32 -> bf16 (NaN stays NaN): gfx950's v_cvt_pk_bf16_f32, one
// instruction per PAIR, instead of the 6-instruction integer rounding sequence.
__device__ __forceinline__ u16v2_t f2bf2(float a, float b) {
  return __builtin_bit_cast(u16v2_t, __builtin_convertvector((f32v2_t{a, b}), bf16v2_t));
}
__device__ __forceinline__ bf16_t f2bf(float f) { return f2bf2(f, 0.f)[0]; }

// Scalar load/store of either float or bf16 storage as float.
template <typename T> struct Elem;
template <> struct Elem<float> {
  static __device__ __forceinline__ float ld(const float* p, int64_t i) { return p[i]; }
  static __device__ __forceinline__ void st(float* p, int64_t i, float x) { p[i] = x; }
};
template <> struct Elem<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p, int64_t i) { return bf2f(p[i]); }
  static __device__ __forceinline__ void st(bf16_t* p, int64_t i, float x) { p[i] = f2bf(x); }
};

// 4-wide vector load/store as float4 (16 B for fp32, 8 B for bf16).
template <typename T> struct Vec4;
template <> struct Vec4<float> {
  static __device__ __forceinline__ float4 ld(const float* p) { return *reinterpret_cast<const float4*>(p); }
  static __device__ __forceinline__ void st(float* p, float4 v) { *reinterpret_cast<float4*>(p) = v; }
};
template <> struct Vec4<bf16_t> {
  static __device__ __forceinline__ float4 ld(const bf16_t* p) {
    bf16x4 r = *reinterpret_cast<const bf16x4*>(p);
    return make_float4(bf2f(r.v[0]), bf2f(r.v[1]), bf2f(r.v[2]), bf2f(r.v[3]));
  }
  static __device__ __forceinline__ void st(bf16_t* p, float4 v) {
    bf16x4 r;
    r.v[0] = f2bf(v.x); r.v[1] = f2bf(v.y); r.v[2] = f2bf(v.z); r.v[3] = f2bf(v.w);
    *reinterpret_cast<bf16x4*>(p) = r;
  }
};

__device__ __forceinline__ float wave_sum(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, kWave);
  return x;
}

__device__ __forceinline__ float wave_max(float x) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x = fmaxf(x, __shfl_xor(x, o, kWave));
  return x;
}

// Block-wide sum for blockDim.x = NT (multiple of 64). `smem` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float x, float* smem) {
  x = wave_sum(x);
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  if (lane == 0) smem[wid] = x;
  __syncthreads();
  float r = 0.f;
  if (wid == 0) {
    r = lane < NT / kWave ? smem[lane] : 0.f;
    r = wave_sum(r);
  }
  return r;  // valid in wave 0
}

__device__ __forceinline__ bool is_aligned16(const void* p) {
  return (reinterpret_cast<uintptr_t>(p) & 15u) == 0;
}

}  // namespace damd

// Launch checking.  Every kernel launch goes through DAMD_LAUNCH, which reads hipGetLastError() right
// after the launch; a failure (bad grid, dynamic LDS over the limit, missing code object, ...) raises
// through launch_failed (defined in the host TU, bindings.cpp) as a C++ exception that the bindings
// surface as a Python RuntimeError naming the launcher, file and line -- a kernel path never returns
// an unwritten output tensor silently.
namespace damd {
[[noreturn]] void launch_failed(hipError_t err, const char* func, const char* file, int line);
inline void check_hip(hipError_t err, const char* func, const char* file, int line) {
  if (err != hipSuccess) launch_failed(err, func, file, line);
}
}  // namespace damd

#define DAMD_CHECK(expr) ::damd::check_hip((expr), __func__, __FILE__, __LINE__)
#define DAMD_CHECK_LAUNCH() DAMD_CHECK(hipGetLastError())
#define DAMD_LAUNCH(...)          \
  do {                            \
    hipLaunchKernelGGL(__VA_ARGS__); \
    DAMD_CHECK_LAUNCH();          \
  } while (0)
