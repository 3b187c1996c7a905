// Two-direction softmax of the co-attention affinity (rgbd_segmentation_RAA.py:164-165,
// :215-216) and its backward.  S = Va_t . Vb^T is fp32 [B][HW][ld] (ld = HW rounded up to 8).
//   P_col[i][j]  = softmax_j(S[i][:])[j]   ("S_column" of the reference, transposed: it is
//                                          the row-normalised S that multiplies V_b)
//   P_rowT[j][i] = softmax_i(S[:][j])[i]   ("S_row", stored transposed so that its GEMM
//                                          with V_a reads k (= i) contiguously)
// Both are written in the compute dtype with zero padding in columns [HW, ld) so the GEMMs
// that consume them can run their K loop over the padded length.
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

__device__ __forceinline__ float block_reduce(float v, float* sh, bool is_max) {
  v = is_max ? warp_max(v) : warp_sum(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float r = sh[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) r = is_max ? fmaxf(r, sh[i]) : r + sh[i];
  return r;
}

template <class T>
__global__ __launch_bounds__(256) void softmax_rows_k(const float* __restrict__ S, int HW, int ld,
                                                      T* __restrict__ P) {
  const long long row = blockIdx.x;  // over B*HW rows
  const float* s = S + row * ld;
  T* p = P + row * ld;
  __shared__ float sh[8];
  float m = -INFINITY;
  for (int j = threadIdx.x; j < HW; j += 256) m = fmaxf(m, s[j]);
  m = block_reduce(m, sh, true);
  float l = 0.f;
  for (int j = threadIdx.x; j < HW; j += 256) l += expf(s[j] - m);
  l = block_reduce(l, sh, false);
  const float inv = 1.f / l;
  for (int j = threadIdx.x; j < ld; j += 256) p[j] = fromf<T>(j < HW ? expf(s[j] - m) * inv : 0.f);
}

// column stats: grid (ceil(HW/64), B, RS); block 256 = 64 columns x 4 row groups
__global__ __launch_bounds__(256) void col_stats_partial_k(const float* __restrict__ S, int HW, int ld,
                                                           int RS, float* __restrict__ part) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  const int b = blockIdx.y, rs = blockIdx.z;
  const int rows_per = (HW + RS - 1) / RS;
  const int i0 = rs * rows_per, i1 = min(HW, i0 + rows_per);
  float m = -INFINITY, l = 0.f;
  if (j < HW) {
    const float* s = S + (long long)b * HW * ld + j;
    for (int i = i0 + rg; i < i1; i += 4) {
      float v = s[(long long)i * ld];
      if (v > m) { l = l * expf(m - v) + 1.f; m = v; }
      else l += expf(v - m);
    }
  }
  __shared__ float sm[4][64], sl[4][64];
  sm[rg][threadIdx.x & 63] = m;
  sl[rg][threadIdx.x & 63] = l;
  __syncthreads();
  if (rg == 0 && j < HW) {
    float M = sm[0][threadIdx.x];
    for (int k = 1; k < 4; ++k) M = fmaxf(M, sm[k][threadIdx.x]);
    float L = 0.f;
    for (int k = 0; k < 4; ++k)
      if (sl[k][threadIdx.x] > 0.f) L += sl[k][threadIdx.x] * expf(sm[k][threadIdx.x] - M);
    long long o = (((long long)rs * gridDim.y + b) * ld + j) * 2;
    part[o] = M;
    part[o + 1] = L;
  }
}

__global__ void col_stats_final_k(const float* __restrict__ part, int B, int HW, int ld, int RS,
                                  float* __restrict__ cm, float* __restrict__ cl) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int b = blockIdx.y;
  if (j >= HW) return;
  float M = -INFINITY;
  for (int r = 0; r < RS; ++r) M = fmaxf(M, part[(((long long)r * B + b) * ld + j) * 2]);
  float L = 0.f;
  for (int r = 0; r < RS; ++r) {
    long long o = (((long long)r * B + b) * ld + j) * 2;
    if (part[o + 1] > 0.f) L += part[o + 1] * expf(part[o] - M);
  }
  cm[(long long)b * ld + j] = M;
  cl[(long long)b * ld + j] = 1.f / L;
}

// P_rowT[b][j][i] = exp(S[b][i][j] - cm[j]) * rcl[j]; 64x64 tiles transposed through LDS
template <class T>
__global__ __launch_bounds__(256) void prow_trans_k(const float* __restrict__ S, int HW, int ld,
                                                    const float* __restrict__ cm,
                                                    const float* __restrict__ rcl, T* __restrict__ PT) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const float* s = S + (long long)b * HW * ld;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int j = j0 + tx;
  float m = 0.f, r = 0.f;
  if (j < HW) { m = cm[(long long)b * ld + j]; r = rcl[(long long)b * ld + j]; }
  for (int ii = ty; ii < 64; ii += 4) {
    int i = i0 + ii;
    float v = 0.f;
    if (i < HW && j < HW) v = expf(s[(long long)i * ld + j] - m) * r;
    tile[ii][tx] = v;
  }
  __syncthreads();
  T* pt = PT + (long long)b * HW * ld;
  for (int jj = ty; jj < 64; jj += 4) {
    int jo = j0 + jj, io = i0 + tx;
    if (jo < HW && io < ld) pt[(long long)jo * ld + io] = fromf<T>(tile[tx][jj]);
  }
}

// dS[i][j] = Pc (dPc - d1[i]) + Pr (dPr - d2[j]),  Pr[i][j] = PT[j][i]
template <class T>
__global__ __launch_bounds__(256) void dscore_k(const T* __restrict__ Pc, const float* __restrict__ dPc,
                                                const float* __restrict__ d1, const T* __restrict__ PT,
                                                const float* __restrict__ dPr,
                                                const float* __restrict__ d2, int HW, int ld,
                                                T* __restrict__ dS) {
  __shared__ float tile[64][65];
  const int b = blockIdx.z;
  const int i0 = blockIdx.y * 64, j0 = blockIdx.x * 64;
  const long long bo = (long long)b * HW * ld;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  if (PT) {  // stage Pr tile: read PT rows j (i contiguous), store tile[i][j]
    for (int jj = ty; jj < 64; jj += 4) {
      int jr = j0 + jj, ic = i0 + tx;
      float v = 0.f;
      if (jr < HW && ic < HW) v = tof(PT[bo + (long long)jr * ld + ic]);
      tile[tx][jj] = v;
    }
  }
  __syncthreads();
  const int j = j0 + tx;
  float dj = (PT && j < HW) ? d2[(long long)b * HW + j] : 0.f;
  for (int ii = ty; ii < 64; ii += 4) {
    int i = i0 + ii;
    if (i >= HW || j >= ld) continue;
    float v = 0.f;
    if (j < HW) {
      long long o = bo + (long long)i * ld + j;
      v = tof(Pc[o]) * (dPc[o] - d1[(long long)b * HW + i]);
      if (PT) v += tile[ii][tx] * (dPr[o] - dj);
    }
    dS[bo + (long long)i * ld + j] = fromf<T>(v);
  }
}

}  // namespace

extern "C" size_t cn_coatt_workspace_floats(int B, int HW, int ld) {
  // column-stat partials (RS=16 splits) + cm + rcl
  return (size_t)16 * B * ld * 2 + (size_t)2 * B * ld;
}

extern "C" int cn_coatt_softmax(int dtype, const float* S, int B, int HW, int ld, void* Pc, void* PT,
                                float* ws, hipStream_t st) {
  if (ld % 8 || ld < HW) return CN_ERR_ALIGN;
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(softmax_rows_k<bf16>, dim3(B * HW), dim3(256), 0, st, S, HW, ld, (bf16*)Pc);
  else
    hipLaunchKernelGGL(softmax_rows_k<float>, dim3(B * HW), dim3(256), 0, st, S, HW, ld, (float*)Pc);
  CN_CHECK_LAUNCH();
  if (!PT) return 0;
  const int RS = 16;
  float* part = ws;
  float* cm = ws + (size_t)RS * B * ld * 2;
  float* rcl = cm + (size_t)B * ld;
  hipLaunchKernelGGL(col_stats_partial_k, dim3((HW + 63) / 64, B, RS), dim3(256), 0, st, S, HW, ld, RS, part);
  CN_CHECK_LAUNCH();
  hipLaunchKernelGGL(col_stats_final_k, dim3((HW + 255) / 256, B), dim3(256), 0, st, part, B, HW, ld, RS, cm, rcl);
  CN_CHECK_LAUNCH();
  dim3 grid((HW + 63) / 64, (ld + 63) / 64, B);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(prow_trans_k<bf16>, grid, dim3(256), 0, st, S, HW, ld, cm, rcl, (bf16*)PT);
  else
    hipLaunchKernelGGL(prow_trans_k<float>, grid, dim3(256), 0, st, S, HW, ld, cm, rcl, (float*)PT);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_coatt_dscore(int dtype, const void* Pc, const float* dPc, const float* d1,
                               const void* PT, const float* dPr, const float* d2, int B, int HW,
                               int ld, void* dS, hipStream_t st) {
  dim3 grid((ld + 63) / 64, (HW + 63) / 64, B);
  if (dtype == DT_BF16)
    hipLaunchKernelGGL(dscore_k<bf16>, grid, dim3(256), 0, st, (const bf16*)Pc, dPc, d1, (const bf16*)PT, dPr, d2, HW, ld, (bf16*)dS);
  else
    hipLaunchKernelGGL(dscore_k<float>, grid, dim3(256), 0, st, (const float*)Pc, dPc, d1, (const float*)PT, dPr, d2, HW, ld, (float*)dS);
  CN_CHECK_LAUNCH();
  return 0;
}
