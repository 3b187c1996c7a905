// Train/eval BatchNorm (nn.BatchNorm2d semantics: biased batch variance for normalisation,
// unbiased for running_var, momentum 0.1, eps 1e-5) over NHWC [P][C] activations, with the
// consumers' ReLU / PReLU / residual add fused into the apply pass and the activation masks
// fused into the backward passes.  Reference call sites: every BN in deeplab/residual_net.py
// (:60-68,:107,:131), deeplab/deeplabv3_encoder.py (:16-32), rgbd_segmentation_RAA.py (:32-42).
//
// Thread layout for every kernel here: a block of 256 threads = CB chunk-columns x RPB rows,
// each thread owns one 16-byte chunk of channels for the whole launch (so per-channel
// constants live in registers) and walks rows with stride RPB * gridDim.y.
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

constexpr int UNR = 4;  // rows in flight per thread in the streaming loops

struct Layout {
  int CPR, CB, RPB;
};
template <class T> __host__ __device__ inline Layout layout_of(int C) {
  Layout l;
  l.CPR = C / VecOf<T>::N;
  l.CB = l.CPR < 256 ? l.CPR : 256;
  l.RPB = 256 / l.CB;
  return l;
}

template <class T> __device__ __forceinline__ void ld_chunk(const T* p, float* f) {
  Chunk<T>::unpack(*(const u32x4*)p, f);
}
template <class T> __device__ __forceinline__ void st_chunk(T* p, const float* f) {
  *(u32x4*)p = Chunk<T>::pack(f);
}

// ---- forward statistics: shifted sums per thread -> (n, mean, M2) -> Chan merge ----------
template <class T>
__global__ __launch_bounds__(256) void bn_stats_partial(const T* __restrict__ x, long long ld, int P,
                                                        int C, float* __restrict__ ws) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  const bool act = chunk < L.CPR && ty < L.RPB;
  float sh[V], s[V], ss[V];
  int n = 0;
#pragma unroll
  for (int v = 0; v < V; ++v) { sh[v] = 0.f; s[v] = 0.f; ss[v] = 0.f; }
  if (act) {
    const int step = gridDim.y * L.RPB;
    for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
      float f[UNR][V];
#pragma unroll
      for (int u = 0; u < UNR; ++u)  // UNR independent 16-B loads in flight per thread
        if (r0 + u * step < P) ld_chunk(x + (long long)(r0 + u * step) * ld + chunk * V, f[u]);
      if (n == 0) {
#pragma unroll
        for (int v = 0; v < V; ++v) sh[v] = f[0][v];
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (r0 + u * step >= P) break;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          float d = f[u][v] - sh[v];
          s[v] += d;
          ss[v] = fmaf(d, d, ss[v]);
        }
        ++n;
      }
    }
  }
  // per-thread (mean, M2)
  __shared__ float lm[256 * 8], l2[256 * 8];
  __shared__ int ln[256];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    float mean = n ? sh[v] + s[v] / n : 0.f;
    float m2 = n ? fmaxf(ss[v] - s[v] * s[v] / n, 0.f) : 0.f;
    lm[threadIdx.x * V + v] = mean;
    l2[threadIdx.x * V + v] = m2;
  }
  ln[threadIdx.x] = n;
  __syncthreads();
  if (ty == 0 && chunk < L.CPR) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float cn = 0.f, cm = 0.f, c2 = 0.f;
      for (int k = 0; k < L.RPB; ++k) {
        int t = k * L.CB + tx;
        float nb = (float)ln[t];
        if (nb == 0.f) continue;
        float mb = lm[t * V + v], m2b = l2[t * V + v];
        float nn = cn + nb, d = mb - cm;
        cm += d * nb / nn;
        c2 += m2b + d * d * cn * nb / nn;
        cn = nn;
      }
      long long o = ((long long)blockIdx.y * C + chunk * V + v) * 3;
      ws[o] = cn; ws[o + 1] = cm; ws[o + 2] = c2;
    }
  }
}

// block = 64 channels x 16 split-lanes (1024 threads); each lane Chan-merges every 16th split
// partial, then a 16-way merge through LDS.
__global__ __launch_bounds__(1024) void bn_stats_finalize(const float* __restrict__ ws, int S, int C,
                                                          float* mean, float* invstd, float* run_mean,
                                                          float* run_var, float momentum, float eps) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  float cn = 0.f, cm = 0.f, c2 = 0.f;
  if (c < C) {
    // 4 partials loaded per round (independent loads in flight), then merged in order
    for (int s0 = lane; s0 < S; s0 += 64) {
      float pn[4], pm[4], pq[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int s = s0 + 16 * u;
        const float* w = ws + ((long long)(s < S ? s : 0) * C + c) * 3;
        pn[u] = s < S ? w[0] : 0.f;
        pm[u] = w[1];
        pq[u] = w[2];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (pn[u] == 0.f) continue;
        float nn = cn + pn[u], d = pm[u] - cm, r = pn[u] / nn;
        cm = fmaf(d, r, cm);
        c2 += pq[u] + d * d * cn * r;
        cn = nn;
      }
    }
  }
  __shared__ float sn[16][64], sm[16][64], s2[16][64];
  sn[lane][threadIdx.x & 63] = cn;
  sm[lane][threadIdx.x & 63] = cm;
  s2[lane][threadIdx.x & 63] = c2;
  __syncthreads();
  if (lane != 0 || c >= C) return;
  double n = 0, m = 0, q = 0;
  for (int k = 0; k < 16; ++k) {
    double nb = sn[k][threadIdx.x];
    if (nb == 0) continue;
    double nn = n + nb, d = sm[k][threadIdx.x] - m;
    m += d * nb / nn;
    q += s2[k][threadIdx.x] + d * d * n * nb / nn;
    n = nn;
  }
  double var = n > 0 ? q / n : 0.0;
  mean[c] = (float)m;
  invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (run_mean) {
    double unb = n > 1 ? q / (n - 1) : var;
    run_mean[c] = (float)((1.0 - momentum) * run_mean[c] + momentum * m);
    run_var[c] = (float)((1.0 - momentum) * run_var[c] + momentum * unb);
  }
}

__global__ void bn_eval_params(const float* rm, const float* rv, int C, float eps, float* mean, float* invstd) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

// ---- apply: y = act(bn(x) [+ res | + bn_r(xr)]) -----------------------------------------
template <class T>
__global__ __launch_bounds__(256) void bn_apply_k(const T* __restrict__ x, long long ldx, int P, int C,
                                                  const float* mean, const float* invstd,
                                                  const float* gamma, const float* beta,
                                                  const T* __restrict__ res, long long ldr,
                                                  const T* __restrict__ xr, long long ldxr,
                                                  const float* rmean, const float* rinvstd,
                                                  const float* rgamma, const float* rbeta, int act,
                                                  const float* prelu, T* __restrict__ y,
                                                  long long ldy) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  if (chunk >= L.CPR || ty >= L.RPB) return;
  float sc[V], sf[V], rsc[V], rsf[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    int c = chunk * V + v;
    float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
    sc[v] = g * invstd[c];
    sf[v] = b - mean[c] * sc[v];
    if (xr) {
      float rg = rgamma ? rgamma[c] : 1.f, rb = rbeta ? rbeta[c] : 0.f;
      rsc[v] = rg * rinvstd[c];
      rsf[v] = rb - rmean[c] * rsc[v];
    }
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  const int step = gridDim.y * L.RPB;
  for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
    float f[UNR][V], q[UNR][V];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = r0 + u * step;
      if (r >= P) break;
      ld_chunk(x + (long long)r * ldx + chunk * V, f[u]);
      if (res) ld_chunk(res + (long long)r * ldr + chunk * V, q[u]);
      if (xr) ld_chunk(xr + (long long)r * ldxr + chunk * V, q[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = r0 + u * step;
      if (r >= P) break;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float t = fmaf(f[u][v], sc[v], sf[v]);
        if (res) t += q[u][v];
        if (xr) t += fmaf(q[u][v], rsc[v], rsf[v]);
        if (act == 1) t = fmaxf(t, 0.f);
        else if (act == 2) t = t > 0.f ? t : a * t;
        f[u][v] = t;
      }
      st_chunk(y + (long long)r * ldy + chunk * V, f[u]);
    }
  }
}

// ---- backward reduce: sum(dz), sum(dz * xhat) [, sum(dy * pre * (pre<=0)) for PReLU] ------
// dz = dy * mask, mask = (y > 0) for act 1, 1 for act 0, (pre > 0 ? 1 : a) for act 2.
template <class T>
__global__ __launch_bounds__(256) void bn_bwd_reduce_k(const T* __restrict__ x, long long ldx,
                                                       const T* __restrict__ dy, long long lddy,
                                                       const T* __restrict__ y, long long ldy,
                                                       int P, int C, const float* mean,
                                                       const float* invstd, const float* gamma,
                                                       const float* beta, int act,
                                                       const float* prelu, float* __restrict__ ws) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  const bool on = chunk < L.CPR && ty < L.RPB;
  float s1[V], s2[V], s3[V], mu[V], is[V], g[V], b[V];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    s1[v] = s2[v] = s3[v] = 0.f;
    int c = on ? chunk * V + v : 0;
    mu[v] = mean[c]; is[v] = invstd[c];
    g[v] = gamma ? gamma[c] : 1.f; b[v] = beta ? beta[c] : 0.f;
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  if (on) {
    const int step = gridDim.y * L.RPB;
    for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
      float xf[UNR][V], d[UNR][V], yf[UNR][V];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * step;
        if (r >= P) break;
        ld_chunk(x + (long long)r * ldx + chunk * V, xf[u]);
        ld_chunk(dy + (long long)r * lddy + chunk * V, d[u]);
        if (act == 1) ld_chunk(y + (long long)r * ldy + chunk * V, yf[u]);
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        if (r0 + u * step >= P) break;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          float dd = (act == 1 && !(yf[u][v] > 0.f)) ? 0.f : d[u][v];
          float xh = (xf[u][v] - mu[v]) * is[v];
          if (act == 2) {
            float pre = fmaf(xh, g[v], b[v]);
            if (pre <= 0.f) { s3[v] = fmaf(dd, pre, s3[v]); dd *= a; }
          }
          s1[v] += dd;
          s2[v] = fmaf(dd, xh, s2[v]);
        }
      }
    }
  }
  __shared__ float r1[256 * 8], r2[256 * 8], r3[256 * 8];
#pragma unroll
  for (int v = 0; v < V; ++v) {
    r1[threadIdx.x * V + v] = s1[v]; r2[threadIdx.x * V + v] = s2[v]; r3[threadIdx.x * V + v] = s3[v];
  }
  __syncthreads();
  if (ty == 0 && chunk < L.CPR) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      float a1 = 0.f, a2 = 0.f, a3 = 0.f;
      for (int k = 0; k < L.RPB; ++k) {
        int t = (k * L.CB + tx) * V + v;
        a1 += r1[t]; a2 += r2[t]; a3 += r3[t];
      }
      long long o = ((long long)blockIdx.y * C + chunk * V + v) * 3;
      ws[o] = a1; ws[o + 1] = a2; ws[o + 2] = a3;
    }
  }
}

__global__ __launch_bounds__(1024) void bn_bwd_finalize(const float* __restrict__ ws, int S, int C,
                                                        float* sum_dz, float* sum_dzxh,
                                                        float* dprelu_c) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  float a = 0.f, b = 0.f, d = 0.f;
  if (c < C) {
    for (int s0 = lane; s0 < S; s0 += 64) {
      float pa[4], pb[4], pd[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int s = s0 + 16 * u;
        const float* w = ws + ((long long)(s < S ? s : 0) * C + c) * 3;
        const bool ok = s < S;
        pa[u] = ok ? w[0] : 0.f;
        pb[u] = ok ? w[1] : 0.f;
        pd[u] = ok ? w[2] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) { a += pa[u]; b += pb[u]; d += pd[u]; }
    }
  }
  __shared__ float ra[16][64], rb[16][64], rd[16][64];
  ra[lane][threadIdx.x & 63] = a;
  rb[lane][threadIdx.x & 63] = b;
  rd[lane][threadIdx.x & 63] = d;
  __syncthreads();
  if (lane != 0 || c >= C) return;
  const int t = threadIdx.x;
  float A = 0.f, Bs = 0.f, D = 0.f;
  for (int k = 0; k < 16; ++k) { A += ra[k][t]; Bs += rb[k][t]; D += rd[k][t]; }
  sum_dz[c] = A;
  sum_dzxh[c] = Bs;
  if (dprelu_c) dprelu_c[c] = D;
}

// dx = gamma*invstd*(dz - sum_dz/P - xhat*sum_dzxh/P);  dres = dz (optional)
template <class T>
__global__ __launch_bounds__(256) void bn_bwd_apply_k(const T* __restrict__ x, long long ldx,
                                                      const T* __restrict__ dy, long long lddy,
                                                      const T* __restrict__ y, long long ldy,
                                                      int P, int C, const float* mean,
                                                      const float* invstd, const float* gamma,
                                                      const float* beta, int act,
                                                      const float* prelu, const float* sum_dz,
                                                      const float* sum_dzxh, T* __restrict__ dx,
                                                      long long lddx, T* __restrict__ dres,
                                                      long long lddres) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  if (chunk >= L.CPR || ty >= L.RPB) return;
  float mu[V], is[V], k1[V], m1[V], m2[V], g[V], b[V];
  const float invP = 1.f / (float)P;
#pragma unroll
  for (int v = 0; v < V; ++v) {
    int c = chunk * V + v;
    mu[v] = mean[c]; is[v] = invstd[c];
    g[v] = gamma ? gamma[c] : 1.f; b[v] = beta ? beta[c] : 0.f;
    k1[v] = g[v] * is[v];
    m1[v] = sum_dz[c] * invP;
    m2[v] = sum_dzxh[c] * invP;
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  const int step = gridDim.y * L.RPB;
  for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
    float xf[UNR][V], d[UNR][V], yf[UNR][V];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = r0 + u * step;
      if (r >= P) break;
      ld_chunk(x + (long long)r * ldx + chunk * V, xf[u]);
      ld_chunk(dy + (long long)r * lddy + chunk * V, d[u]);
      if (act == 1) ld_chunk(y + (long long)r * ldy + chunk * V, yf[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = r0 + u * step;
      if (r >= P) break;
      float o[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float dd = (act == 1 && !(yf[u][v] > 0.f)) ? 0.f : d[u][v];
        float xh = (xf[u][v] - mu[v]) * is[v];
        if (act == 2) {
          float pre = fmaf(xh, g[v], b[v]);
          if (pre <= 0.f) dd *= a;
        }
        o[v] = k1[v] * (dd - m1[v] - xh * m2[v]);
        d[u][v] = dd;
      }
      st_chunk(dx + (long long)r * lddx + chunk * V, o);
      if (dres) st_chunk(dres + (long long)r * lddres + chunk * V, d[u]);
    }
  }
}

// Row blocks for a launch: ~`blocks` blocks in total, each thread walking >= min_rows rows.
// Reductions (stats, backward sums) use min_rows 8 so the split count stays small for the
// finalize pass; pure streaming passes (apply) use 2 for more parallelism.
template <class T> int grid_rows(int P, int C, int* gx, int min_rows = 8, int blocks = 1024) {
  Layout L = layout_of<T>(C);
  *gx = (L.CPR + L.CB - 1) / L.CB;
  int want = (blocks + *gx - 1) / *gx;
  int maxy = (P + min_rows * L.RPB - 1) / (min_rows * L.RPB);
  int gy = want < maxy ? want : maxy;
  return gy < 1 ? 1 : gy;
}

template <class T> int splits_for(int P, int C) {
  int gx;
  int gy = grid_rows<T>(P, C, &gx);
  return gy;
}

}  // namespace

extern "C" size_t cn_bn_workspace_floats(int dtype, int P, int C) {
  int S = dtype == DT_BF16 ? splits_for<bf16>(P, C) : splits_for<float>(P, C);
  return (size_t)S * C * 3;
}

extern "C" int cn_bn_stats(int dtype, const void* x, long long ldx, int P, int C, float* mean,
                           float* invstd, float* run_mean, float* run_var, float momentum,
                           float eps, float* ws, hipStream_t st) {
  if (C % (dtype == DT_BF16 ? 8 : 4) || ldx % (dtype == DT_BF16 ? 8 : 4)) return CN_ERR_ALIGN;
  int gx, gy;
  if (dtype == DT_BF16) {
    gy = grid_rows<bf16>(P, C, &gx);
    hipLaunchKernelGGL(bn_stats_partial<bf16>, dim3(gx, gy), dim3(256), 0, st, (const bf16*)x, ldx, P, C, ws);
  } else {
    gy = grid_rows<float>(P, C, &gx);
    hipLaunchKernelGGL(bn_stats_partial<float>, dim3(gx, gy), dim3(256), 0, st, (const float*)x, ldx, P, C, ws);
  }
  CN_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_stats_finalize, dim3((C + 63) / 64), dim3(1024), 0, st, ws, gy, C, mean,
                     invstd, run_mean, run_var, momentum, eps);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_eval_params(const float* run_mean, const float* run_var, int C, float eps,
                                 float* mean, float* invstd, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_params, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps, mean, invstd);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_apply(int dtype, const void* x, long long ldx, int P, int C, const float* mean,
                           const float* invstd, const float* gamma, const float* beta,
                           const void* res, long long ldr, const void* xr, long long ldxr,
                           const float* rmean, const float* rinvstd, const float* rgamma,
                           const float* rbeta, int act, const float* prelu, void* y,
                           long long ldy, hipStream_t st) {
  int gx, gy;
  if (dtype == DT_BF16) {
    gy = grid_rows<bf16>(P, C, &gx, UNR, 2048);
    hipLaunchKernelGGL(bn_apply_k<bf16>, dim3(gx, gy), dim3(256), 0, st, (const bf16*)x, ldx, P, C,
                       mean, invstd, gamma, beta, (const bf16*)res, ldr, (const bf16*)xr, ldxr, rmean,
                       rinvstd, rgamma, rbeta, act, prelu, (bf16*)y, ldy);
  } else {
    gy = grid_rows<float>(P, C, &gx, UNR, 2048);
    hipLaunchKernelGGL(bn_apply_k<float>, dim3(gx, gy), dim3(256), 0, st, (const float*)x, ldx, P, C,
                       mean, invstd, gamma, beta, (const float*)res, ldr, (const float*)xr, ldxr,
                       rmean, rinvstd, rgamma, rbeta, act, prelu, (float*)y, ldy);
  }
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_bwd(int dtype, const void* x, long long ldx, const void* dy, long long lddy,
                         const void* y, long long ldy, int P, int C, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int act,
                         const float* prelu, float* dgamma, float* dbeta, float* dprelu_c,
                         void* dx, long long lddx, void* dres, long long lddres, float* ws,
                         hipStream_t st) {
  int gx, gy;
  if (dtype == DT_BF16) {
    gy = grid_rows<bf16>(P, C, &gx);
    hipLaunchKernelGGL(bn_bwd_reduce_k<bf16>, dim3(gx, gy), dim3(256), 0, st, (const bf16*)x, ldx,
                       (const bf16*)dy, lddy, (const bf16*)y, ldy, P, C, mean, invstd, gamma, beta,
                       act, prelu, ws);
  } else {
    gy = grid_rows<float>(P, C, &gx);
    hipLaunchKernelGGL(bn_bwd_reduce_k<float>, dim3(gx, gy), dim3(256), 0, st, (const float*)x, ldx,
                       (const float*)dy, lddy, (const float*)y, ldy, P, C, mean, invstd, gamma,
                       beta, act, prelu, ws);
  }
  CN_CHECK_LAUNCH();
  hipLaunchKernelGGL(bn_bwd_finalize, dim3((C + 63) / 64), dim3(1024), 0, st, ws, gy, C, dbeta, dgamma, dprelu_c);
  CN_CHECK_LAUNCH();
  if (!dx) return 0;
  gy = dtype == DT_BF16 ? grid_rows<bf16>(P, C, &gx, UNR, 2048) : grid_rows<float>(P, C, &gx, UNR, 2048);
  if (dtype == DT_BF16) {
    hipLaunchKernelGGL(bn_bwd_apply_k<bf16>, dim3(gx, gy), dim3(256), 0, st, (const bf16*)x, ldx,
                       (const bf16*)dy, lddy, (const bf16*)y, ldy, P, C, mean, invstd, gamma, beta,
                       act, prelu, dbeta, dgamma, (bf16*)dx, lddx, (bf16*)dres, lddres);
  } else {
    hipLaunchKernelGGL(bn_bwd_apply_k<float>, dim3(gx, gy), dim3(256), 0, st, (const float*)x, ldx,
                       (const float*)dy, lddy, (const float*)y, ldy, P, C, mean, invstd, gamma,
                       beta, act, prelu, dbeta, dgamma, (float*)dx, lddx, (float*)dres, lddres);
  }
  CN_CHECK_LAUNCH();
  return 0;
}
