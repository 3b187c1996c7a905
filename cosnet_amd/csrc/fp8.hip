// fp8 (OCP e4m3) operand preparation for the fp8 GEMM path (BASELINE configs[4]: "fp8 MFMA
// affinity + implicit-GEMM conv").  Per-tensor scaling with a device-side state per tensor:
//   state[0] = scale  (dequantisation factor the GEMM multiplies its accumulators by)
//   state[1] = 1/scale (quantisation factor)
//   state[2] = running amax |x| since the last update (fp32 bits, atomicMax as unsigned)
// Delayed scaling (activations): quantise with the scale of the previous update while
// collecting this tensor's amax; cn_fp8_update turns the amax into the next scale.  Current
// scaling (weights): amax pass, update, quantise.  fp8 max finite = 448; |x| / scale is clamped
// there before the conversion (saturating, never NaN).
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

constexpr float FP8_MAX = 448.f;

constexpr float BF8_MAX = 57344.f;   // OCP e5m2 max finite (gradients)

__device__ __forceinline__ unsigned pack4_fp8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -FP8_MAX), FP8_MAX);
  b = fminf(fmaxf(b, -FP8_MAX), FP8_MAX);
  c = fminf(fmaxf(c, -FP8_MAX), FP8_MAX);
  d = fminf(fmaxf(d, -FP8_MAX), FP8_MAX);
  unsigned w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}
__device__ __forceinline__ unsigned pack4_bf8(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -BF8_MAX), BF8_MAX);
  b = fminf(fmaxf(b, -BF8_MAX), BF8_MAX);
  c = fminf(fmaxf(c, -BF8_MAX), BF8_MAX);
  d = fminf(fmaxf(d, -BF8_MAX), BF8_MAX);
  unsigned w = __builtin_amdgcn_cvt_pk_bf8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_bf8_f32(c, d, w, true);
}
template <int FMT>
__device__ __forceinline__ unsigned pack4(float a, float b, float c, float d) {
  return FMT ? pack4_bf8(a, b, c, d) : pack4_fp8(a, b, c, d);
}

// block max -> ONE atomic per block (same-address atomics serialise in L2)
__device__ __forceinline__ void wave_amax_atomic(float m, float* state) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[16];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) wm[w] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int i = 1; i < (int)(blockDim.x >> 6); ++i) m = fmaxf(m, wm[i]);
    if (m > 0.f) atomicMax((unsigned*)&state[2], __float_as_uint(m));
  }
}

// y8[r][c] = fp8(x[r][c] * state[1]) for a [P][C] matrix (row strides ldx / ldy, C % 8 == 0);
// amax of |x| accumulated into state[2] when `collect`.  Block = 64 chunk-columns (8 elements
// each) x 4 row groups; rows strided over gridDim.y -- no index division in the loop.
template <class T, int FMT>
__global__ __launch_bounds__(256) void quant_fp8_k(const T* __restrict__ x, long long ldx, int P, int C,
                                                   unsigned char* __restrict__ y, long long ldy,
                                                   float* state, int quantise, int collect) {
  const float inv = state[1];
  const int cc = blockIdx.x * 64 + (threadIdx.x & 63);
  const int c = cc * 8;
  float m = 0.f;
  if (c < C) {
    constexpr int U = 4;  // rows in flight per thread
    const int step = 4 * gridDim.y;
    for (int r0 = blockIdx.y * 4 + (threadIdx.x >> 6); r0 < P; r0 += U * step) {
      float f[U][8];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * step;
        if (r >= P) break;
        if constexpr (sizeof(T) == 2) {
          Chunk<bf16>::unpack(*(const u32x4*)(x + (long long)r * ldx + c), f[u]);
        } else {
          *(f32x4*)&f[u][0] = *(const f32x4*)(x + (long long)r * ldx + c);
          *(f32x4*)&f[u][4] = *(const f32x4*)(x + (long long)r * ldx + c + 4);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = r0 + u * step;
        if (r >= P) break;
#pragma unroll
        for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[u][e]));
        if (quantise) {
          u32x2 o;
          o.x = pack4<FMT>(f[u][0] * inv, f[u][1] * inv, f[u][2] * inv, f[u][3] * inv);
          o.y = pack4<FMT>(f[u][4] * inv, f[u][5] * inv, f[u][6] * inv, f[u][7] * inv);
          *(u32x2*)(y + (long long)r * ldy + c) = o;
        }
      }
    }
  }
  if (collect) wave_amax_atomic(m, state);
}

// scale = amax / (fmt max / 2^margin); a zero amax (all-zero tensor) keeps the previous scale.
// state[3] = the format's max finite value (0: e4m3's 448; 57344 for e5m2 gradient states)
__global__ void fp8_update_k(float* state, int nstates, float margin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nstates) return;
  float* s = state + 4 * i;
  const float amax = __uint_as_float(*(const unsigned*)&s[2]);
  if (amax > 0.f) {
    const float sc = amax * margin / (s[3] > 0.f ? s[3] : FP8_MAX);
    s[0] = sc;
    s[1] = 1.f / sc;
  }
  s[2] = 0.f;
}

// Multi-tensor weight preparation: one launch per pass over every fp8 weight copy.
struct Fp8Rec {
  const void* x; long long ldx; int P, C;    // x fp32, or bf16 when xbf16 (e.g. the transposed
  unsigned char* y; long long ldy;           // bf16 dgrad weight copy)
  float* state;
  long long xbf16;
};
static_assert(sizeof(Fp8Rec) == 56, "Fp8Rec layout is shared with cosnet_amd/ops.py");

__global__ __launch_bounds__(256) void quant_fp8_multi_k(const Fp8Rec* __restrict__ recs, int quantise,
                                                         int collect) {
  const Fp8Rec r = recs[blockIdx.y];
  const float inv = r.state[1];
  const int cpr = r.C / 8;
  float m = 0.f;
  // block x of gridDim.x walks rows x, x + gridDim.x, ... ; threads stride the row's chunks
  for (int row = blockIdx.x; row < r.P; row += gridDim.x) {
    for (int cc = threadIdx.x; cc < cpr; cc += blockDim.x) {
      const int c = cc * 8;
      float f[8];
      if (r.xbf16) {
        Chunk<bf16>::unpack(*(const u32x4*)((const bf16*)r.x + row * r.ldx + c), f);
      } else {
        *(f32x4*)&f[0] = *(const f32x4*)((const float*)r.x + row * r.ldx + c);
        *(f32x4*)&f[4] = *(const f32x4*)((const float*)r.x + row * r.ldx + c + 4);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
      if (quantise) {
        u32x2 o;
        o.x = pack4_fp8(f[0] * inv, f[1] * inv, f[2] * inv, f[3] * inv);
        o.y = pack4_fp8(f[4] * inv, f[5] * inv, f[6] * inv, f[7] * inv);
        *(u32x2*)(r.y + row * r.ldy + c) = o;
      }
    }
  }
  if (collect) wave_amax_atomic(m, r.state);
}

__global__ void fp8_update_list_k(const Fp8Rec* __restrict__ recs, int n, float margin) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float* s = recs[i].state;
  const float amax = __uint_as_float(*(const unsigned*)&s[2]);
  if (amax > 0.f) {
    const float sc = amax * margin / (s[3] > 0.f ? s[3] : FP8_MAX);
    s[0] = sc;
    s[1] = 1.f / sc;
  }
  s[2] = 0.f;
}

}  // namespace

extern "C" int cn_fp8_quant_fmt(int dtype, int fmt, const void* x, long long ldx, int P, int C,
                                void* y8, long long ldy, float* state, int mode, hipStream_t st) {
  if (C % 8 || ldx % 8 || ldy % 8 || !state) return CN_ERR_ALIGN;
  if (fmt != 0 && fmt != 1) return CN_ERR_UNSUPPORTED;
  if (P <= 0) return 0;
  const int gx = (C / 8 + 63) / 64;
  int gy = (P + 63) / 64;                      // >= 16 rows per thread
  const int maxy = (1024 + gx - 1) / gx;       // ~1024 blocks: 4 per CU
  if (gy > maxy) gy = maxy;
  if (gy < 1) gy = 1;
  const dim3 grid(gx, gy);
  auto launch = [&](int quantise, int collect) {
    if (dtype == DT_BF16 && fmt == 0)
      hipLaunchKernelGGL((quant_fp8_k<bf16, 0>), grid, dim3(256), 0, st, (const bf16*)x, ldx, P, C,
                         (unsigned char*)y8, ldy, state, quantise, collect);
    else if (dtype == DT_BF16)
      hipLaunchKernelGGL((quant_fp8_k<bf16, 1>), grid, dim3(256), 0, st, (const bf16*)x, ldx, P, C,
                         (unsigned char*)y8, ldy, state, quantise, collect);
    else if (fmt == 0)
      hipLaunchKernelGGL((quant_fp8_k<float, 0>), grid, dim3(256), 0, st, (const float*)x, ldx, P, C,
                         (unsigned char*)y8, ldy, state, quantise, collect);
    else
      hipLaunchKernelGGL((quant_fp8_k<float, 1>), grid, dim3(256), 0, st, (const float*)x, ldx, P, C,
                         (unsigned char*)y8, ldy, state, quantise, collect);
  };
  if (dtype != DT_BF16 && dtype != DT_F32) return CN_ERR_UNSUPPORTED;
  if (mode == 0) {          // delayed: quantise with the current scale, collect this amax
    launch(1, 1);
  } else if (mode == 1) {   // current: amax pass, scale update, quantise
    launch(0, 1);
    CN_CHECK_LAUNCH();
    hipLaunchKernelGGL(fp8_update_k, dim3(1), dim3(64), 0, st, state, 1, 1.f);
    CN_CHECK_LAUNCH();
    launch(1, 0);
  } else if (mode == 2) {   // amax only (calibration of a delayed-scaling state)
    launch(0, 1);
  } else {
    return CN_ERR_SHAPE;
  }
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_fp8_quant(int dtype, const void* x, long long ldx, int P, int C, void* y8,
                            long long ldy, float* state, int mode, hipStream_t st) {
  return cn_fp8_quant_fmt(dtype, 0, x, ldx, P, C, y8, ldy, state, mode, st);
}

// Current scaling of a list of fp32 tensors (e.g. every fp8 conv-weight copy after the SGD
// step): amax pass, scale update, quantise -- three launches for the whole list.
extern "C" int cn_fp8_quant_multi(const void* recs, int n, hipStream_t st) {
  if (n <= 0) return 0;
  const Fp8Rec* r = (const Fp8Rec*)recs;
  hipLaunchKernelGGL(quant_fp8_multi_k, dim3(128, n), dim3(256), 0, st, r, 0, 1);
  CN_CHECK_LAUNCH();
  hipLaunchKernelGGL(fp8_update_list_k, dim3((n + 63) / 64), dim3(64), 0, st, r, n, 1.f);
  CN_CHECK_LAUNCH();
  hipLaunchKernelGGL(quant_fp8_multi_k, dim3(128, n), dim3(256), 0, st, r, 1, 0);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_fp8_update(float* states, int nstates, float margin, hipStream_t st) {
  if (nstates <= 0) return 0;
  hipLaunchKernelGGL(fp8_update_k, dim3((nstates + 63) / 64), dim3(64), 0, st, states, nstates, margin);
  CN_CHECK_LAUNCH();
  return 0;
}
