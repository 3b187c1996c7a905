// Evaluation tail of test.py on the GPU: uint8 quantisation of the resized mean output
// (test.py:317, `(output1 * 255).astype(np.uint8)`) and the soft-J score of evaluation.py:3-22
// per frame:
//
//   p = uint8(trunc(x * 255))           (fp32 product, truncation toward zero like numpy)
//   g = uint8(gt * 255)                 (uint8 arithmetic, i.e. mod 256, like numpy on uint8)
//   gt all zero : J = 1 - count_nonzero(p) / (H * W)                      (:4-7)
//   otherwise   : J = sum(int16(p) & int16(g)) / sum(int16(p) | int16(g))  (:8-19)
//
// Integer byte work, HBM-bound: one workgroup per frame streams the frame once (16-byte
// loads of x, 4-byte loads of gt), writes the uint8 mask and reduces four 64-bit integer
// counts with wave shuffles + LDS -- integer sums are order-free, so the result is bit-exact
// against numpy and needs no atomics.  The final divisions are done in double like numpy's.
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

__device__ __forceinline__ unsigned quant(float x) {
  // numpy: float32 * 255 -> float32, astype(uint8) truncates; the product of a sigmoid
  // average lies in [0, 255]
  float v = __fmul_rn(x, 255.0f);
  return (unsigned)(int)v & 255u;
}

struct Acc {
  unsigned long long a, o, nz, g;
};

__device__ __forceinline__ void add_px(Acc& s, unsigned p, unsigned gt) {
  const unsigned g = (gt * 255u) & 255u;
  s.a += p & g;
  s.o += p | g;
  s.nz += p != 0;
  s.g += g != 0;
}

__global__ __launch_bounds__(512) void soft_iou_k(const float* __restrict__ x,
                                                  const unsigned char* __restrict__ gt, long long hw,
                                                  unsigned char* __restrict__ mask, double* iou,
                                                  long long* counts) {
  const long long f = blockIdx.x;
  const float* xf = x + f * hw;
  const unsigned char* gf = gt + f * hw;
  unsigned char* mf = mask + f * hw;
  Acc s{0, 0, 0, 0};
  // 4-pixel groups: x as 16 B, gt / mask as 4 B (frames are 4-element aligned when hw % 4 == 0)
  const long long n4 = (hw % 4 == 0) ? hw / 4 : 0;
  for (long long i = threadIdx.x; i < n4; i += blockDim.x) {
    const f32x4 v = *(const f32x4*)(xf + 4 * i);
    const unsigned gw = *(const unsigned*)(gf + 4 * i);
    unsigned mw = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const unsigned p = quant(v[k]);
      add_px(s, p, (gw >> (8 * k)) & 255u);
      mw |= p << (8 * k);
    }
    *(unsigned*)(mf + 4 * i) = mw;
  }
  for (long long i = 4 * n4 + threadIdx.x; i < hw; i += blockDim.x) {
    const unsigned p = quant(xf[i]);
    add_px(s, p, gf[i]);
    mf[i] = (unsigned char)p;
  }
  // block reduction: 64-lane shuffles, then one value per wave through LDS
  unsigned long long v[4] = {s.a, s.o, s.nz, s.g};
#pragma unroll
  for (int q = 0; q < 4; ++q)
    for (int off = 32; off > 0; off >>= 1) v[q] += __shfl_xor(v[q], off, 64);
  __shared__ unsigned long long red[4][8];
  const int w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int q = 0; q < 4; ++q) red[q][w] = v[q];
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t[4] = {0, 0, 0, 0};
    for (int k = 0; k < nw; ++k)
#pragma unroll
      for (int q = 0; q < 4; ++q) t[q] += red[q][k];
    double j;
    if (t[3] == 0) j = 1.0 - (double)t[2] / (double)hw;
    else j = (double)t[0] / (double)t[1];
    iou[f] = j;
    if (counts)
#pragma unroll
      for (int q = 0; q < 4; ++q) counts[4 * f + q] = (long long)t[q];
  }
}

}  // namespace

extern "C" int cn_soft_iou(const float* x, const unsigned char* gt, int nframes, long long hw,
                           unsigned char* mask, double* iou, long long* counts, hipStream_t st) {
  if (nframes < 1 || hw < 1) return CN_ERR_SHAPE;
  if (hw % 4 == 0 && (((uintptr_t)x & 15) || ((uintptr_t)gt & 3) || ((uintptr_t)mask & 3)))
    return CN_ERR_ALIGN;
  hipLaunchKernelGGL(soft_iou_k, dim3(nframes), dim3(512), 0, st, x, gt, hw, mask, iou, counts);
  CN_CHECK_LAUNCH();
  return 0;
}
