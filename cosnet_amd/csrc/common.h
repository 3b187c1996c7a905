// Shared device helpers for the CDNA4 (gfx950) kernels of libcosnet_hip.
// Activations are NHWC "pixel-major" matrices [P][C] with a row stride `ld` (elements), so
// channel slices of concat buffers are plain (ptr + offset, ld) views.  Element type T is
// float (fp32 parity path) or __bf16 (throughput path); accumulation is always fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// Measured-and-rejected kernel variants (co-attention wave pairs, GEMM tile configurations 21-25)
// are compiled only into development builds (make EXPERIMENTAL=1); the product library keeps the
// code that runs by default.
#ifndef CN_EXPERIMENTAL
#define CN_EXPERIMENTAL 0
#endif

// dtype codes shared with the C ABI (include/cosnet_hip.h)
enum { DT_F32 = 0, DT_BF16 = 1, DT_FP8 = 2, DT_FP8_E5M2 = 3 };  // DT_FP8_E5M2 GEMM: A e5m2, B e4m3

// OCP fp8 e4m3 (gfx950's e4m3fn, not MI300's fnuz), stored as raw bytes; matrix-core operand
// only (the fp8 GEMMs read it, elementwise code never computes in it)
struct f8e4m3 { unsigned char v; };
struct f8e5m2 { unsigned char v; };   // OCP e5m2 ("bf8"): gradients
typedef __attribute__((ext_vector_type(8))) int i32x8;

template <class T> struct VecOf;
template <> struct VecOf<float> { static constexpr int N = 4; };  // elements per 16-byte chunk
template <> struct VecOf<bf16> { static constexpr int N = 8; };
template <> struct VecOf<f8e4m3> { static constexpr int N = 16; };
template <> struct VecOf<f8e5m2> { static constexpr int N = 16; };

__device__ __forceinline__ float tof(float x) { return x; }
__device__ __forceinline__ float tof(bf16 x) { return (float)x; }
template <class T> __device__ __forceinline__ T fromf(float x);
template <> __device__ __forceinline__ float fromf<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 fromf<bf16>(float x) { return (bf16)x; }

// Unpack / pack one 16-byte chunk to VEC floats.
template <class T> struct Chunk;
template <> struct Chunk<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void unpack(const u32x4& v, float* f) {
    f32x4 q = __builtin_bit_cast(f32x4, v);
    f[0] = q[0]; f[1] = q[1]; f[2] = q[2]; f[3] = q[3];
  }
  __device__ __forceinline__ static u32x4 pack(const float* f) {
    f32x4 q = {f[0], f[1], f[2], f[3]};
    return __builtin_bit_cast(u32x4, q);
  }
};
template <> struct Chunk<bf16> {
  static constexpr int N = 8;
  __device__ __forceinline__ static void unpack(const u32x4& v, float* f) {
    unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __builtin_bit_cast(float, w[i] << 16);
      f[2 * i + 1] = __builtin_bit_cast(float, w[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static u32x4 pack(const float* f) {
    unsigned w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16 lo = (bf16)f[2 * i], hi = (bf16)f[2 * i + 1];
      w[i] = (unsigned)__builtin_bit_cast(unsigned short, lo) |
             ((unsigned)__builtin_bit_cast(unsigned short, hi) << 16);
    }
    u32x4 v; v.x = w[0]; v.y = w[1]; v.z = w[2]; v.w = w[3];
    return v;
  }
};

// Fast unsigned divmod by a runtime-invariant divisor (round-up multiplier method; valid for
// 0 <= n < 2^31).  mul/shift are computed on the host (see fastdiv_make in launch code).
struct FastDiv {
  int d;
  unsigned mul;
  int shift;
};
__device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  return (int)((__umulhi((unsigned)n, f.mul) + (unsigned)n) >> f.shift);
}
__device__ __forceinline__ void fdivmod(int n, const FastDiv& f, int& q, int& r) {
  q = fdiv(n, f);
  r = n - q * f.d;
}
static inline FastDiv fastdiv_make(int d) {
  FastDiv f;
  f.d = d;
  int s = 0;
  while ((1ll << s) < (long long)d) ++s;
  f.shift = s;
  f.mul = (unsigned)((((1ull << 32) * ((1ull << s) - (unsigned long long)d)) / (unsigned long long)d) + 1ull);
  return f;
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

#define CN_CHECK_LAUNCH() \
  do { hipError_t e__ = hipGetLastError(); if (e__ != hipSuccess) return (int)e__; } while (0)
