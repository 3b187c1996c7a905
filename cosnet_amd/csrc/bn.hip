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

constexpr int UNR = 4;   // rows in flight per thread in the streaming (apply) loops
constexpr int SUNR = 8;  // rows in flight per thread in the statistics pass

struct Layout {
  int CPR, CB, RPB;
};
// Reduction passes (statistics, backward sums) use at most 32 chunk columns per block, so a
// block walks >= 8 rows per step and wide layers (C = 1024..2560) need 8x fewer row splits:
// the per-split partials (written by the pass, re-read by the finalize) stay ~2 MB instead of
// ~17-25 MB per call.
template <class T> __host__ __device__ inline Layout layout_red(int C) {
  Layout l;
  l.CPR = C / VecOf<T>::N;
  l.CB = l.CPR < 32 ? l.CPR : 32;
  l.RPB = 256 / l.CB;
  return l;
}
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
// the same chunk stored write-through (sc1) at a byte offset from a buffer resource's base
template <class T> __device__ __forceinline__ void st_chunk_wt(__amdgpu_buffer_rsrc_t r, long long off,
                                                              const float* f) {
  __builtin_amdgcn_raw_buffer_store_b128(Chunk<T>::pack(f), r, (int)off, 0, 16);
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7fffffff, 0x00020000);
}
// The apply kernels store their outputs write-through (sc1) where the byte offsets from the
// output's base fit 31 bits: the lines go to memory as they are written instead of waiting dirty
// in the XCD's L2 for the end-of-kernel write-back that the next kernel's start waits on
// (+0.55 % on the step; the same for the GEMM epilogue's C stores measured -0.4 %:
// profiles/r06_write_through_ab.txt).  CN_BN_WT=0: plain stores; 2: also the ReLU-mask bytes and
// the fp8 output copy; 3: non-temporal (nt) stores instead (A/B runs).
static int bn_wt_env() {
  static const int lvl = [] { const char* e = getenv("CN_BN_WT"); return e ? atoi(e) : 1; }();
  return lvl;
}
static int bn_wt(long long rows, long long ld, int esz) {
  return rows * ld * esz < 0x7fff0000ll ? bn_wt_env() : 0;
}

// Column sums of the block's RPB rows of per-thread accumulators, written as
// out[q][blockIdx.y][c] (q < NQ planes of S x C floats).  Parallel over all 256 threads: with
// NCOL = CB*V columns, 256/NCOL partial sums per column, then one more pass.
template <int V, int NQ>
__device__ __forceinline__ void block_col_sums(const Layout& L, int tx, int ty, const float* a,
                                               const float* b, const float* c3, float* out,
                                               int S, int C) {
  __shared__ float red[NQ][256 * 8];
  const int NCOL = L.CB * V;
  if (ty < L.RPB) {
#pragma unroll
    for (int v = 0; v < V; ++v) {
      red[0][ty * NCOL + tx * V + v] = a[v];
      if (NQ > 1) red[1][ty * NCOL + tx * V + v] = b[v];
      if (NQ > 2) red[NQ > 2 ? 2 : 0][ty * NCOL + tx * V + v] = c3[v];
    }
  }
  __syncthreads();
  const int c0 = blockIdx.x * NCOL;
  const long long plane = (long long)S * C;
  float* o = out + (long long)blockIdx.y * C + c0;
  if (NCOL >= 256) {
    for (int j = threadIdx.x; j < NCOL; j += 256) {
      float acc[NQ];
#pragma unroll
      for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
      for (int k = 0; k < L.RPB; ++k)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += red[q][k * NCOL + j];
      if (c0 + j < C)
#pragma unroll
        for (int q = 0; q < NQ; ++q) o[q * plane + j] = acc[q];
    }
  } else {
    const int np = 256 / NCOL, part = threadIdx.x / NCOL, j = threadIdx.x % NCOL;
    float acc[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) acc[q] = 0.f;
    if (part < np)
      for (int k = part; k < L.RPB; k += np)
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc[q] += red[q][k * NCOL + j];
    __syncthreads();
    if (part < np)
#pragma unroll
      for (int q = 0; q < NQ; ++q) red[q][part * NCOL + j] = acc[q];
    __syncthreads();
    if (threadIdx.x < NCOL && c0 + j < C) {
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        float t = 0.f;
        for (int k = 0; k < np; ++k) t += red[q][k * NCOL + j];
        o[q * plane + j] = t;
      }
    }
  }
}

// Sum over the S splits of npl consecutive planes of S x C partials, for the FCH channels of
// this block: thread = (channel tid % FCH, lane tid / FCH), 32 lanes stride the splits, then
// shuffles over the 8 lanes of a wave and an LDS pass over the 4 waves.  tot[plane][FCH].
constexpr int FCH = 8, MAXPL = 8;
template <int NPL>
__device__ __forceinline__ void plane_sums(const float* __restrict__ ws, int S, int C, int c0,
                                           float (*tot)[FCH]) {
  constexpr int npl = NPL;  // compile-time so every plane's load is issued unconditionally
  const int ch = threadIdx.x % FCH, lane = threadIdx.x / FCH, c = c0 + ch;
  const long long plane = (long long)S * C;
  float acc[NPL];
#pragma unroll
  for (int q = 0; q < NPL; ++q) acc[q] = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int s = lane; s < S; s += 256 / FCH)
#pragma unroll
      for (int q = 0; q < NPL; ++q) acc[q] += ws[q * plane + (long long)s * C + c];
  }
  __shared__ float red[MAXPL][4][FCH];
  const int wave = threadIdx.x / 64;
#pragma unroll
  for (int q = 0; q < NPL; ++q) {
    float v = acc[q];
    v += __shfl_xor(v, FCH, 64);
    v += __shfl_xor(v, 2 * FCH, 64);
    v += __shfl_xor(v, 4 * FCH, 64);
    if ((threadIdx.x & 63) < FCH) red[q][wave][ch] = v;
  }
  __syncthreads();
  if (threadIdx.x < npl * FCH) {
    const int q = threadIdx.x / FCH;
    tot[q][ch] = red[q][0][ch] + red[q][1][ch] + red[q][2][ch] + red[q][3][ch];
  }
  __syncthreads();
}

// ---- forward statistics -------------------------------------------------------------------
// Sums shifted by a common per-channel value K = x[first row of the segment] (so partials are
// plain sums and merge by addition): partial[seg][q][split][c], q = 0: sum(x-K), 1: sum((x-K)^2).
// A block = CB chunk-columns x RPB rows; rows past P load K itself and contribute zero.
template <class T>
__global__ __launch_bounds__(256) void bn_stats_partial(const T* __restrict__ x, long long ld, int P,
                                                        int C, float* __restrict__ ws) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_red<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  const int S = gridDim.y, seg = blockIdx.z;
  const T* xs = x + (long long)seg * P * ld;
  float s[V], ss[V];
#pragma unroll
  for (int v = 0; v < V; ++v) { s[v] = 0.f; ss[v] = 0.f; }
  if (chunk < L.CPR && ty < L.RPB) {
    float K[V];
    ld_chunk(xs + chunk * V, K);
    const int step = S * L.RPB;
    for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += SUNR * step) {
      float f[SUNR][V];
      // SUNR independent 16-B loads in flight per thread: every load is issued unconditionally
      // (rows past P re-read row 0 and contribute zero), so no branch separates them -- a
      // bounds branch per load made hipcc drain vmcnt(0) after each one
#pragma unroll
      for (int u = 0; u < SUNR; ++u) {
        const int r = r0 + u * step;
        ld_chunk(xs + (long long)(r < P ? r : 0) * ld + chunk * V, f[u]);
      }
#pragma unroll
      for (int u = 0; u < SUNR; ++u) {
        const bool in = r0 + u * step < P;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          float d = in ? f[u][v] - K[v] : 0.f;
          s[v] += d;
          ss[v] = fmaf(d, d, ss[v]);
        }
      }
    }
  }
  block_col_sums<V, 2>(L, tx, ty, s, ss, nullptr, ws + (long long)seg * 2 * S * C, S, C);
}

// mean / invstd per segment; running stats updated segment after segment (the reference runs
// the encoder once per frame, so each frame's batch is one BN call).
template <class T, int NSEG>
__global__ __launch_bounds__(256) void bn_stats_finalize(const float* __restrict__ ws, int S, int C,
                                                         const T* __restrict__ x,
                                                         long long ld, int P, float* mean,
                                                         float* invstd, float* run_mean,
                                                         float* run_var, float momentum, float eps) {
  const int c0 = blockIdx.x * FCH;
  __shared__ float tot[MAXPL][FCH];
  plane_sums<2 * NSEG>(ws, S, C, c0, tot);
  const int c = c0 + threadIdx.x;
  if (threadIdx.x >= FCH || c >= C) return;
  double rm = 0, rv = 0;
  if (run_mean) { rm = run_mean[c]; rv = run_var[c]; }
  for (int seg = 0; seg < NSEG; ++seg) {
    const double n = P, K = tof(x[(long long)seg * P * ld + c]);
    const double s1 = tot[2 * seg][threadIdx.x], s2 = tot[2 * seg + 1][threadIdx.x];
    const double md = s1 / n;
    const double q = s2 - s1 * md > 0 ? s2 - s1 * md : 0.0;  // sum of squared deviations
    const double var = q / n;
    mean[seg * C + c] = (float)(K + md);
    invstd[seg * C + c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = n > 1 ? q / (n - 1) : var;
      rm = (float)((1.0 - momentum) * rm + momentum * (K + md));
      rv = (float)((1.0 - momentum) * rv + momentum * unb);
    }
  }
  if (run_mean) { run_mean[c] = (float)rm; run_var[c] = (float)rv; }
}

// ---- forward statistics from the conv epilogue (gemm.h st_mode 1) ---------------------------
// Per M-tile t and column c the GEMM wrote K (the tile's first row), and shifted sums
// [sum(c-K), sum((c-K)^2)] of the rows in the tile's first segment and of the rows in the next.
// Each tile's sums are turned into plain sum / sum of squares in double and added over the tiles
// in a fixed order (lanes stride the tiles, then a shuffle tree and the 4 waves in order):
// deterministic, and double keeps the final var = E[x^2] - mean^2 exact enough for any data
// whose per-tile spread fp32 resolves.
template <int NSEG>
__global__ __launch_bounds__(256) void bn_tile_stats_finalize(const float* __restrict__ ws, long long plane,
                                                              int mtiles, int BM, int M, int seg_rows,
                                                              int C, float* mean, float* invstd,
                                                              float* run_mean, float* run_var,
                                                              float momentum, float eps) {
  const int c0 = blockIdx.x * FCH;
  const int ch = threadIdx.x % FCH, lane = threadIdx.x / FCH, c = c0 + ch;
  double d1[NSEG], d2[NSEG];
#pragma unroll
  for (int s = 0; s < NSEG; ++s) { d1[s] = 0.0; d2[s] = 0.0; }
  if (c < C) {
    for (int t = lane; t < mtiles; t += 256 / FCH) {
      const int r0 = t * BM, r1 = min(M, r0 + BM);
      const int sA = r0 / seg_rows;
      const int endA = min(r1, (sA + 1) * seg_rows);
      const double nA = endA - r0, nB = r1 - endA;
      const long long o = (long long)t * C + c;
      const double K = ws[o];
      const double a1 = ws[o + plane], a2 = ws[o + 2 * plane];
#pragma unroll
      for (int s = 0; s < NSEG; ++s) {
        if (s == sA) { d1[s] += nA * K + a1; d2[s] += a2 + 2.0 * K * a1 + nA * K * K; }
        if (s == sA + 1 && nB > 0) {
          const double b1 = ws[o + 3 * plane], b2 = ws[o + 4 * plane];
          d1[s] += nB * K + b1;
          d2[s] += b2 + 2.0 * K * b1 + nB * K * K;
        }
      }
    }
  }
  __shared__ double red[2 * NSEG][4][FCH];
  const int wave = threadIdx.x / 64;
#pragma unroll
  for (int s = 0; s < NSEG; ++s) {
#pragma unroll
    for (int o = FCH; o < 64; o <<= 1) {
      d1[s] += __shfl_xor(d1[s], o, 64);
      d2[s] += __shfl_xor(d2[s], o, 64);
    }
    if ((threadIdx.x & 63) < FCH) { red[2 * s][wave][ch] = d1[s]; red[2 * s + 1][wave][ch] = d2[s]; }
  }
  __syncthreads();
  if (threadIdx.x >= FCH || c >= C) return;
  double rm = 0, rv = 0;
  if (run_mean) { rm = run_mean[c]; rv = run_var[c]; }
  const double n = seg_rows;
  for (int s = 0; s < NSEG; ++s) {
    const double s1 = ((red[2 * s][0][ch] + red[2 * s][1][ch]) + red[2 * s][2][ch]) + red[2 * s][3][ch];
    const double s2 = ((red[2 * s + 1][0][ch] + red[2 * s + 1][1][ch]) + red[2 * s + 1][2][ch]) + red[2 * s + 1][3][ch];
    const double md = s1 / n;
    double var = s2 / n - md * md;
    if (var < 0) var = 0;
    mean[s * C + c] = (float)md;
    invstd[s * C + c] = (float)(1.0 / sqrt(var + (double)eps));
    if (run_mean) {
      const double unb = n > 1 ? var * n / (n - 1) : var;
      rm = (float)((1.0 - momentum) * rm + momentum * md);
      rv = (float)((1.0 - momentum) * rv + momentum * unb);
    }
  }
  if (run_mean) { run_mean[c] = (float)rm; run_var[c] = (float)rv; }
}

__global__ void bn_eval_params(const float* rm, const float* rv, int C, float eps, float* mean, float* invstd) {
  int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  mean[c] = rm[c];
  invstd[c] = 1.0f / sqrtf(rv[c] + eps);
}

// fp8 e4m3 (OCP) packing of the optional fp8 output of bn_apply (cosnet_amd/fp8.py): saturating
__device__ __forceinline__ unsigned pack4_fp8_bn(float a, float b, float c, float d) {
  a = fminf(fmaxf(a, -448.f), 448.f);
  b = fminf(fmaxf(b, -448.f), 448.f);
  c = fminf(fmaxf(c, -448.f), 448.f);
  d = fminf(fmaxf(d, -448.f), 448.f);
  unsigned w = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  return __builtin_amdgcn_cvt_pk_fp8_f32(c, d, w, true);
}

// amax of the block -> one atomicMax on the state's amax slot (every thread must call)
__device__ __forceinline__ void fp8_block_amax(float m, float* state) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  __shared__ float wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    m = fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3]));
    if (m > 0.f) atomicMax((unsigned*)&state[2], __float_as_uint(m));
  }
}

// V consecutive fp32 per-channel constants (16-byte aligned; null -> dflt)
template <int V>
__device__ __forceinline__ void ld_params(const float* p, int c0, float dflt, float* o) {
  if (!p) {
#pragma unroll
    for (int v = 0; v < V; ++v) o[v] = dflt;
    return;
  }
#pragma unroll
  for (int v = 0; v < V; v += 4) {
    f32x4 q = *(const f32x4*)(p + c0 + v);
    o[v] = q[0]; o[v + 1] = q[1]; o[v + 2] = q[2]; o[v + 3] = q[3];
  }
}

// ---- apply: y = act(bn(x) [+ res | + bn_r(xr)]) per segment (blockIdx.z) -------------------
template <class T>
__global__ __launch_bounds__(256) void bn_apply_k(const T* __restrict__ x, long long ldx, int P, int C,
                                                  const float* mean, const float* invstd,
                                                  const float* gamma, const float* beta,
                                                  const T* __restrict__ res, long long ldr,
                                                  const T* __restrict__ xr, long long ldxr,
                                                  const float* rmean, const float* rinvstd,
                                                  const float* rgamma, const float* rbeta, int act,
                                                  const float* prelu, T* __restrict__ y,
                                                  long long ldy, unsigned char* __restrict__ y8,
                                                  long long ldy8, float* qstate,
                                                  unsigned char* __restrict__ mk, long long ldm,
                                                  int wt) {
  constexpr int V = VecOf<T>::N;
  // wt: y stored write-through (sc1), offsets from y (the host checked they fit 31 bits)
  const __amdgpu_buffer_rsrc_t yrs = wt_rsrc(y), mkrs = wt_rsrc(mk), y8rs = wt_rsrc(y8);
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  float qmax = 0.f;
  const float qinv = y8 ? qstate[1] : 0.f;
  if (chunk >= L.CPR || ty >= L.RPB) {
    if (y8) fp8_block_amax(qmax, qstate);
    return;
  }
  const int seg = blockIdx.z, c0 = chunk * V;
  const long long row0 = (long long)seg * P;
  float sc[V], sf[V], rsc[V], rsf[V], t0[V], t1[V];
  ld_params<V>(gamma, c0, 1.f, sc);
  ld_params<V>(beta, c0, 0.f, sf);
  ld_params<V>(invstd + seg * C, c0, 1.f, t0);
  ld_params<V>(mean + seg * C, c0, 0.f, t1);
#pragma unroll
  for (int v = 0; v < V; ++v) {
    sc[v] *= t0[v];
    sf[v] -= t1[v] * sc[v];
  }
  if (xr) {
    ld_params<V>(rgamma, c0, 1.f, rsc);
    ld_params<V>(rbeta, c0, 0.f, rsf);
    ld_params<V>(rinvstd + seg * C, c0, 1.f, t0);
    ld_params<V>(rmean + seg * C, c0, 0.f, t1);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      rsc[v] *= t0[v];
      rsf[v] -= t1[v] * rsc[v];
    }
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  const int step = gridDim.y * L.RPB;
  for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
    float f[UNR][V], q[UNR][V];
    // all loads of the UNR rows issued unconditionally (rows past P re-read the segment's first
    // row and are not stored): no bounds branch between them
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long r = row0 + (r0 + u * step < P ? r0 + u * step : 0);
      ld_chunk(x + r * ldx + c0, f[u]);
      if (res) ld_chunk(res + r * ldr + c0, q[u]);
      if (xr) ld_chunk(xr + r * ldxr + c0, q[u]);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long long r = row0 + r0 + u * step;
      if (r0 + u * step >= P) break;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float t = fmaf(f[u][v], sc[v], sf[v]);
        if (res) t += q[u][v];
        if (xr) t += fmaf(q[u][v], rsc[v], rsf[v]);
        if (act == 1) t = fmaxf(t, 0.f);
        else if (act == 2) t = t > 0.f ? t : a * t;
        f[u][v] = t;
      }
      const u32x4 pk = Chunk<T>::pack(f[u]);
      if (wt == 3)
        __builtin_nontemporal_store(pk, (u32x4*)(y + r * ldy + c0));
      else if (wt)
        __builtin_amdgcn_raw_buffer_store_b128(pk, yrs, (int)((r * ldy + c0) * (long long)sizeof(T)), 0, 16);
      else
        *(u32x4*)(y + r * ldy + c0) = pk;
      if (mk) {  // ReLU mask of the STORED values, one bit per channel (the backward's act 4)
        float sv[V];
        Chunk<T>::unpack(pk, sv);
        unsigned bits = 0;
#pragma unroll
        for (int v = 0; v < V; ++v) bits |= (sv[v] > 0.f ? 1u : 0u) << v;
        if (wt == 2)
          __builtin_amdgcn_raw_buffer_store_b8((unsigned char)bits, mkrs, (int)(r * ldm + chunk), 0, 16);
        else
          mk[r * ldm + chunk] = (unsigned char)bits;
      }
      if (y8) {  // fp8 copy of the output for an fp8 consumer conv (delayed scaling)
#pragma unroll
        for (int v = 0; v < V; ++v) qmax = fmaxf(qmax, fabsf(f[u][v]));
#pragma unroll
        for (int v = 0; v < V; v += 8) {
          u32x2 o;
          o.x = pack4_fp8_bn(f[u][v] * qinv, f[u][v + 1] * qinv, f[u][v + 2] * qinv, f[u][v + 3] * qinv);
          o.y = pack4_fp8_bn(f[u][v + 4] * qinv, f[u][v + 5] * qinv, f[u][v + 6] * qinv, f[u][v + 7] * qinv);
          if (wt == 2)
            __builtin_amdgcn_raw_buffer_store_b64(o, y8rs, (int)(r * ldy8 + c0 + v), 0, 16);
          else
            *(u32x2*)(y8 + r * ldy8 + c0 + v) = o;
        }
      }
    }
  }
  if (y8) fp8_block_amax(qmax, qstate);
}

// ---- backward reduce: planes sum(dz), sum(dz * xhat) [, sum(dz * pre * (pre<=0)) PReLU] ----
// dz = dy * mask, mask = (y > 0) for act 1, 1 for act 0, (pre > 0 ? 1 : a) for act 2.
// act 4: the ReLU mask comes as bits (bn_apply_k's mask output): mk[row * ldm + chunk], bit v.
template <class T, int NQ>
__global__ __launch_bounds__(256) void bn_bwd_reduce_k(const T* __restrict__ x, long long ldx,
                                                       const T* __restrict__ dy, long long lddy,
                                                       const T* __restrict__ y, long long ldy,
                                                       const unsigned char* __restrict__ mk,
                                                       int P, int C, const float* mean,
                                                       const float* invstd, const float* gamma,
                                                       const float* beta, int act,
                                                       const float* prelu, float* __restrict__ ws) {
  constexpr int V = VecOf<T>::N;
  const Layout L = layout_red<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  const bool on = chunk < L.CPR && ty < L.RPB;
  const int c0 = on ? chunk * V : 0;
  float s1[V], s2[V], s3[V], mu[V], is[V], g[V], b[V], sc[V], sf[V];
  ld_params<V>(mean, c0, 0.f, mu);
  ld_params<V>(invstd, c0, 1.f, is);
  ld_params<V>(gamma, c0, 1.f, g);
  ld_params<V>(beta, c0, 0.f, b);
#pragma unroll
  for (int v = 0; v < V; ++v) {
    s1[v] = s2[v] = s3[v] = 0.f;
    sc[v] = g[v] * is[v];          // the forward apply's affine (bn_apply_k): the recomputed
    sf[v] = b[v] - mu[v] * sc[v];  // ReLU mask (act 3) has exactly the forward's sign
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  if (on) {
    const int step = gridDim.y * L.RPB;
    for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
      float xf[UNR][V], d[UNR][V], yf[UNR][V];
      unsigned mb[UNR];
      // loads issued unconditionally (rows past P re-read row 0 and contribute zero); the
      // activation branch sits outside the unrolled loop so no branch separates the loads
      if (act == 1) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int r = r0 + u * step < P ? r0 + u * step : 0;
          ld_chunk(x + (long long)r * ldx + c0, xf[u]);
          ld_chunk(dy + (long long)r * lddy + c0, d[u]);
          ld_chunk(y + (long long)r * ldy + c0, yf[u]);
        }
      } else if (act == 4) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int r = r0 + u * step < P ? r0 + u * step : 0;
          ld_chunk(x + (long long)r * ldx + c0, xf[u]);
          ld_chunk(dy + (long long)r * lddy + c0, d[u]);
          mb[u] = mk[(long long)r * ldy + chunk];
        }
      } else {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int r = r0 + u * step < P ? r0 + u * step : 0;
          ld_chunk(x + (long long)r * ldx + c0, xf[u]);
          ld_chunk(dy + (long long)r * lddy + c0, d[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const bool in = r0 + u * step < P;
#pragma unroll
        for (int v = 0; v < V; ++v) {
          float dd = (!in || (act == 1 && !(yf[u][v] > 0.f))) ? 0.f : d[u][v];
          if (act == 3 && !(fmaf(xf[u][v], sc[v], sf[v]) > 0.f)) dd = 0.f;
          if (act == 4 && !((mb[u] >> v) & 1u)) dd = 0.f;
          float xh = (xf[u][v] - mu[v]) * is[v];
          if (NQ > 2) {
            float pre = fmaf(xh, g[v], b[v]);
            if (pre <= 0.f) { s3[v] = fmaf(dd, pre, s3[v]); dd *= a; }
          }
          s1[v] += dd;
          s2[v] = fmaf(dd, xh, s2[v]);
        }
      }
    }
  }
  block_col_sums<V, NQ>(L, tx, ty, s1, s2, s3, ws, gridDim.y, C);
}

template <int NQ>
__global__ __launch_bounds__(256) void bn_bwd_finalize(const float* __restrict__ ws, int S, int C,
                                                       float* sum_dz, float* sum_dzxh,
                                                       float* dprelu_c) {
  const int c0 = blockIdx.x * FCH;
  __shared__ float tot[MAXPL][FCH];
  plane_sums<NQ>(ws, S, C, c0, tot);
  const int c = c0 + threadIdx.x;
  if (threadIdx.x >= FCH || c >= C) return;
  sum_dz[c] = tot[0][threadIdx.x];
  sum_dzxh[c] = tot[1][threadIdx.x];
  if (NQ > 2) dprelu_c[c] = tot[NQ > 2 ? 2 : 0][threadIdx.x];
}

// dx = gamma*invstd*(dz - sum_dz/P - xhat*sum_dzxh/P);  dres = dz (optional)
template <class T>
__global__ __launch_bounds__(256) void bn_bwd_apply_k(const T* __restrict__ x, long long ldx,
                                                      const T* __restrict__ dy, long long lddy,
                                                      const T* __restrict__ y, long long ldy,
                                                      const unsigned char* __restrict__ mk,
                                                      int P, int C, const float* mean,
                                                      const float* invstd, const float* gamma,
                                                      const float* beta, int act,
                                                      const float* prelu, const float* sum_dz,
                                                      const float* sum_dzxh, T* __restrict__ dx,
                                                      long long lddx, T* __restrict__ dres,
                                                      long long lddres, int wt) {
  constexpr int V = VecOf<T>::N;
  const __amdgpu_buffer_rsrc_t dxr = wt_rsrc(dx), drr = wt_rsrc(dres);
  const Layout L = layout_of<T>(C);
  const int tx = threadIdx.x % L.CB, ty = threadIdx.x / L.CB;
  const int chunk = blockIdx.x * L.CB + tx;
  if (chunk >= L.CPR || ty >= L.RPB) return;
  float mu[V], is[V], k1[V], m1[V], m2[V], g[V], b[V], sf[V];
  const float invP = 1.f / (float)P;
  const int c0 = chunk * V;
  ld_params<V>(mean, c0, 0.f, mu);
  ld_params<V>(invstd, c0, 1.f, is);
  ld_params<V>(gamma, c0, 1.f, g);
  ld_params<V>(beta, c0, 0.f, b);
  ld_params<V>(sum_dz, c0, 0.f, m1);
  ld_params<V>(sum_dzxh, c0, 0.f, m2);
#pragma unroll
  for (int v = 0; v < V; ++v) {
    k1[v] = g[v] * is[v];
    sf[v] = b[v] - mu[v] * k1[v];  // forward affine: mask of act 3 = fmaf(x, k1, sf) > 0
    m1[v] *= invP;
    m2[v] *= invP;
  }
  const float a = (act == 2) ? prelu[0] : 0.f;
  const int step = gridDim.y * L.RPB;
  for (int r0 = blockIdx.y * L.RPB + ty; r0 < P; r0 += UNR * step) {
    float xf[UNR][V], d[UNR][V], yf[UNR][V];
    unsigned mb[UNR];
    // loads issued unconditionally (rows past P re-read row 0 and are not stored); the
    // activation branch sits outside the unrolled loop so no branch separates the loads
    if (act == 1) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * step < P ? r0 + u * step : 0;
        ld_chunk(x + (long long)r * ldx + chunk * V, xf[u]);
        ld_chunk(dy + (long long)r * lddy + chunk * V, d[u]);
        ld_chunk(y + (long long)r * ldy + chunk * V, yf[u]);
      }
    } else if (act == 4) {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * step < P ? r0 + u * step : 0;
        ld_chunk(x + (long long)r * ldx + chunk * V, xf[u]);
        ld_chunk(dy + (long long)r * lddy + chunk * V, d[u]);
        mb[u] = mk[(long long)r * ldy + chunk];
      }
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int r = r0 + u * step < P ? r0 + u * step : 0;
        ld_chunk(x + (long long)r * ldx + chunk * V, xf[u]);
        ld_chunk(dy + (long long)r * lddy + chunk * V, d[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int r = r0 + u * step;
      if (r >= P) break;
      float o[V];
#pragma unroll
      for (int v = 0; v < V; ++v) {
        float dd = (act == 1 && !(yf[u][v] > 0.f)) ? 0.f : d[u][v];
        if (act == 3 && !(fmaf(xf[u][v], k1[v], sf[v]) > 0.f)) dd = 0.f;
        if (act == 4 && !((mb[u] >> v) & 1u)) dd = 0.f;
        float xh = (xf[u][v] - mu[v]) * is[v];
        if (act == 2) {
          float pre = fmaf(xh, g[v], b[v]);
          if (pre <= 0.f) dd *= a;
        }
        o[v] = k1[v] * (dd - m1[v] - xh * m2[v]);
        d[u][v] = dd;
      }
      if (wt == 3) {
        __builtin_nontemporal_store(Chunk<T>::pack(o), (u32x4*)(dx + (long long)r * lddx + chunk * V));
        if (dres) __builtin_nontemporal_store(Chunk<T>::pack(d[u]), (u32x4*)(dres + (long long)r * lddres + chunk * V));
      } else if (wt) {
        st_chunk_wt<T>(dxr, ((long long)r * lddx + chunk * V) * (long long)sizeof(T), o);
        if (dres) st_chunk_wt<T>(drr, ((long long)r * lddres + chunk * V) * (long long)sizeof(T), d[u]);
      } else {
        st_chunk(dx + (long long)r * lddx + chunk * V, o);
        if (dres) st_chunk(dres + (long long)r * lddres + chunk * V, d[u]);
      }
    }
  }
}

// Row blocks for a launch: ~`blocks` blocks in total over gx x gy x nseg, each thread walking
// >= min_rows rows.  Reductions use min_rows 8 (one statistics round) so the split count the
// finalize has to sum stays small; streaming passes (apply) use UNR rows per thread.
template <class T> int grid_rows(int P, int C, int* gx, int min_rows, int blocks, int nseg = 1,
                                 bool red = false) {
  Layout L = red ? layout_red<T>(C) : layout_of<T>(C);
  *gx = (L.CPR + L.CB - 1) / L.CB;
  int want = (blocks / nseg + *gx - 1) / *gx;
  int maxy = (P + min_rows * L.RPB - 1) / (min_rows * L.RPB);
  int gy = want < maxy ? want : maxy;
  return gy < 1 ? 1 : gy;
}

int g_tune[8] = {1024, SUNR, 2048, UNR, 512, UNR, 2048, UNR};  // see cn_bn_set_tuning; bwd-reduce 512: profiles/r04_bn_tune_ab.txt
enum { T_ST_BLOCKS, T_ST_ROWS, T_AP_BLOCKS, T_AP_ROWS, T_BR_BLOCKS, T_BR_ROWS, T_BA_BLOCKS, T_BA_ROWS };

template <class T> int stat_splits(int P, int C, int nseg, int* gx) {
  return grid_rows<T>(P, C, gx, g_tune[T_ST_ROWS], g_tune[T_ST_BLOCKS], nseg, true);
}
template <class T> int bwd_splits(int P, int C, int* gx) {
  return grid_rows<T>(P, C, gx, g_tune[T_BR_ROWS], g_tune[T_BR_BLOCKS], 1, true);
}

bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

}  // namespace

extern "C" int cn_bn_set_tuning(int key, int value) {
  if (key < 0 || key >= 8 || value < 1) return CN_ERR_SHAPE;
  g_tune[key] = value;
  return 0;
}

extern "C" size_t cn_bn_workspace_floats(int dtype, int P, int C, int nseg) {
  int gx, s_st, s_bw;
  if (dtype == DT_BF16) { s_st = stat_splits<bf16>(P, C, nseg, &gx); s_bw = bwd_splits<bf16>(P, C, &gx); }
  else { s_st = stat_splits<float>(P, C, nseg, &gx); s_bw = bwd_splits<float>(P, C, &gx); }
  size_t a = (size_t)nseg * 2 * s_st, b = (size_t)3 * s_bw;
  return (a > b ? a : b) * C;
}

template <class T>
static int bn_stats_launch(const T* x, long long ldx, int P, int nseg, int C, float* mean,
                           float* invstd, float* run_mean, float* run_var, float momentum,
                           float eps, float* ws, hipStream_t st) {
  int gx, gy = stat_splits<T>(P, C, nseg, &gx);
  hipLaunchKernelGGL(bn_stats_partial<T>, dim3(gx, gy, nseg), dim3(256), 0, st, x, ldx, P, C, ws);
  CN_CHECK_LAUNCH();
  const dim3 fin((C + FCH - 1) / FCH);
#define CN_FIN(NS)                                                                                 \
  hipLaunchKernelGGL((bn_stats_finalize<T, NS>), fin, dim3(256), 0, st, ws, gy, C, x, ldx, P, mean, \
                     invstd, run_mean, run_var, momentum, eps)
  switch (nseg) {
    case 1: CN_FIN(1); break;
    case 2: CN_FIN(2); break;
    case 3: CN_FIN(3); break;
    case 4: CN_FIN(4); break;
    default: return CN_ERR_UNSUPPORTED;
  }
#undef CN_FIN
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_stats(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                           float* mean, float* invstd, float* run_mean, float* run_var,
                           float momentum, float eps, float* ws, hipStream_t st) {
  if (C % (dtype == DT_BF16 ? 8 : 4) || ldx % (dtype == DT_BF16 ? 8 : 4)) return CN_ERR_ALIGN;
  if (P < 1 || nseg < 1) return CN_ERR_SHAPE;
  if (dtype == DT_BF16)
    return bn_stats_launch<bf16>((const bf16*)x, ldx, P, nseg, C, mean, invstd, run_mean, run_var,
                                 momentum, eps, ws, st);
  return bn_stats_launch<float>((const float*)x, ldx, P, nseg, C, mean, invstd, run_mean, run_var,
                                momentum, eps, ws, st);
}

int cn_bn_tile_stats_impl(const float* ws, long long plane, int mtiles, int BM, int M, int nseg, int C,
                          float* mean, float* invstd, float* run_mean, float* run_var, float momentum,
                          float eps, hipStream_t st) {
  if (nseg < 1 || M % nseg) return CN_ERR_SHAPE;
  const int seg_rows = M / nseg;
  const dim3 fin((C + FCH - 1) / FCH);
#define CN_TF(NS)                                                                                    \
  hipLaunchKernelGGL((bn_tile_stats_finalize<NS>), fin, dim3(256), 0, st, ws, plane, mtiles, BM, M, \
                     seg_rows, C, mean, invstd, run_mean, run_var, momentum, eps)
  switch (nseg) {
    case 1: CN_TF(1); break;
    case 2: CN_TF(2); break;
    default: return CN_ERR_UNSUPPORTED;
  }
#undef CN_TF
  CN_CHECK_LAUNCH();
  return 0;
}

// Backward sums from the dgrad epilogue (gemm.h st_mode 2): planes [sum dz, sum dz*xh] per
// M-tile -> sum_dz[c], sum_dzxh[c] (bn_bwd_finalize over S = mtiles splits, same layout).
int cn_bn_tile_bwd_impl(const float* ws, int mtiles, int C, float* sum_dz, float* sum_dzxh,
                        hipStream_t st) {
  const dim3 fin((C + FCH - 1) / FCH);
  hipLaunchKernelGGL(bn_bwd_finalize<2>, fin, dim3(256), 0, st, ws, mtiles, C, sum_dz, sum_dzxh,
                     (float*)nullptr);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_bwd_apply(int dtype, const void* x, long long ldx, const void* dy, long long lddy,
                               int P, int C, const float* mean, const float* invstd,
                               const float* gamma, const float* beta, const float* sum_dz,
                               const float* sum_dzxh, void* dx, long long lddx, hipStream_t st) {
  const int vec = dtype == DT_BF16 ? 8 : 4;
  if (C % vec || ldx % vec || lddy % vec || lddx % vec) return CN_ERR_ALIGN;
  if (!aligned16(mean) || !aligned16(invstd) || !aligned16(gamma) || !aligned16(beta) ||
      !aligned16(sum_dz) || !aligned16(sum_dzxh))
    return CN_ERR_ALIGN;
  if (P < 1) return CN_ERR_SHAPE;
  int gx, gy;
  // act 3: ReLU mask recomputed from x with the forward's affine (no residual on these BNs)
  if (dtype == DT_BF16) {
    gy = grid_rows<bf16>(P, C, &gx, g_tune[T_BA_ROWS], g_tune[T_BA_BLOCKS]);
    hipLaunchKernelGGL(bn_bwd_apply_k<bf16>, dim3(gx, gy), dim3(256), 0, st, (const bf16*)x, ldx,
                       (const bf16*)dy, lddy, (const bf16*)nullptr, 0ll, (const unsigned char*)nullptr, P, C, mean, invstd, gamma,
                       beta, 3, (const float*)nullptr, sum_dz, sum_dzxh, (bf16*)dx, lddx,
                       (bf16*)nullptr, 0ll, bn_wt(P, lddx, 2));
  } else {
    gy = grid_rows<float>(P, C, &gx, g_tune[T_BA_ROWS], g_tune[T_BA_BLOCKS]);
    hipLaunchKernelGGL(bn_bwd_apply_k<float>, dim3(gx, gy), dim3(256), 0, st, (const float*)x, ldx,
                       (const float*)dy, lddy, (const float*)nullptr, 0ll, (const unsigned char*)nullptr, P, C, mean, invstd, gamma,
                       beta, 3, (const float*)nullptr, sum_dz, sum_dzxh, (float*)dx, lddx,
                       (float*)nullptr, 0ll, bn_wt(P, lddx, 4));
  }
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_eval_params(const float* run_mean, const float* run_var, int C, float eps,
                                 float* mean, float* invstd, hipStream_t st) {
  hipLaunchKernelGGL(bn_eval_params, dim3((C + 255) / 256), dim3(256), 0, st, run_mean, run_var, C, eps, mean, invstd);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_apply_fp8(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                               const float* mean, const float* invstd, const float* gamma,
                               const float* beta, const void* res, long long ldr, const void* xr,
                               long long ldxr, const float* rmean, const float* rinvstd,
                               const float* rgamma, const float* rbeta, int act, const float* prelu,
                               void* y, long long ldy, void* y8, long long ldy8, float* qstate,
                               hipStream_t st);

extern "C" int cn_bn_apply(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                           const float* mean, const float* invstd, const float* gamma,
                           const float* beta, const void* res, long long ldr, const void* xr,
                           long long ldxr, const float* rmean, const float* rinvstd,
                           const float* rgamma, const float* rbeta, int act, const float* prelu,
                           void* y, long long ldy, hipStream_t st) {
  return cn_bn_apply_fp8(dtype, x, ldx, P, nseg, C, mean, invstd, gamma, beta, res, ldr, xr, ldxr,
                         rmean, rinvstd, rgamma, rbeta, act, prelu, y, ldy, nullptr, 0, nullptr, st);
}

extern "C" int cn_bn_apply_fp8(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                               const float* mean, const float* invstd, const float* gamma,
                               const float* beta, const void* res, long long ldr, const void* xr,
                               long long ldxr, const float* rmean, const float* rinvstd,
                               const float* rgamma, const float* rbeta, int act, const float* prelu,
                               void* y, long long ldy, void* y8, long long ldy8, float* qstate,
                               hipStream_t st) {
  return cn_bn_apply_ex(dtype, x, ldx, P, nseg, C, mean, invstd, gamma, beta, res, ldr, xr, ldxr,
                        rmean, rinvstd, rgamma, rbeta, act, prelu, y, ldy, y8, ldy8, qstate, nullptr,
                        0, st);
}

extern "C" int cn_bn_apply_ex(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                              const float* mean, const float* invstd, const float* gamma,
                              const float* beta, const void* res, long long ldr, const void* xr,
                              long long ldxr, const float* rmean, const float* rinvstd,
                              const float* rgamma, const float* rbeta, int act, const float* prelu,
                              void* y, long long ldy, void* y8, long long ldy8, float* qstate,
                              unsigned char* mask, long long ldm, hipStream_t st) {
  if (y8 && (dtype != DT_BF16 || !qstate || ldy8 % 16 || ((uintptr_t)y8 & 7))) return CN_ERR_ALIGN;
  if (mask && ldm < C / (dtype == DT_BF16 ? 8 : 4)) return CN_ERR_SHAPE;
  const int vec = dtype == DT_BF16 ? 8 : 4;
  if (C % vec || ldx % vec || ldy % vec || (res && ldr % vec) || (xr && ldxr % vec)) return CN_ERR_ALIGN;
  if (!aligned16(mean) || !aligned16(invstd) || !aligned16(gamma) || !aligned16(beta) ||
      !aligned16(rmean) || !aligned16(rinvstd) || !aligned16(rgamma) || !aligned16(rbeta))
    return CN_ERR_ALIGN;
  if (P < 1 || nseg < 1) return CN_ERR_SHAPE;
  int wt = bn_wt((long long)nseg * P, ldy, dtype == DT_BF16 ? 2 : 4);
  if (wt == 2 && ((mask && !bn_wt((long long)nseg * P, ldm, 1)) || (y8 && !bn_wt((long long)nseg * P, ldy8, 1))))
    wt = 1;
  int gx, gy;
  if (dtype == DT_BF16) {
    gy = grid_rows<bf16>(P, C, &gx, g_tune[T_AP_ROWS], g_tune[T_AP_BLOCKS], nseg);
    hipLaunchKernelGGL(bn_apply_k<bf16>, dim3(gx, gy, nseg), dim3(256), 0, st, (const bf16*)x, ldx, P, C,
                       mean, invstd, gamma, beta, (const bf16*)res, ldr, (const bf16*)xr, ldxr, rmean,
                       rinvstd, rgamma, rbeta, act, prelu, (bf16*)y, ldy, (unsigned char*)y8, ldy8,
                       qstate, mask, ldm, wt);
  } else {
    gy = grid_rows<float>(P, C, &gx, g_tune[T_AP_ROWS], g_tune[T_AP_BLOCKS], nseg);
    hipLaunchKernelGGL(bn_apply_k<float>, dim3(gx, gy, nseg), dim3(256), 0, st, (const float*)x, ldx, P, C,
                       mean, invstd, gamma, beta, (const float*)res, ldr, (const float*)xr, ldxr,
                       rmean, rinvstd, rgamma, rbeta, act, prelu, (float*)y, ldy,
                       (unsigned char*)nullptr, 0ll, (float*)nullptr, mask, ldm, wt);
  }
  CN_CHECK_LAUNCH();
  return 0;
}

template <class T>
static int bn_bwd_launch(const T* x, long long ldx, const T* dy, long long lddy, const T* y,
                         long long ldy, int P, int C, const float* mean, const float* invstd,
                         const float* gamma, const float* beta, int act, const float* prelu,
                         float* dgamma, float* dbeta, float* dprelu_c, T* dx, long long lddx,
                         T* dres, long long lddres, float* ws, hipStream_t st) {
  int gx, gy = bwd_splits<T>(P, C, &gx);
  const dim3 fin((C + FCH - 1) / FCH);
  // act 4: `y` is the ReLU bit mask (bytes, row stride ldy) written by cn_bn_apply_ex
  const unsigned char* mk = act == 4 ? (const unsigned char*)y : nullptr;
  if (act == 4) y = nullptr;
  if (act == 2) {
    hipLaunchKernelGGL((bn_bwd_reduce_k<T, 3>), dim3(gx, gy), dim3(256), 0, st, x, ldx, dy, lddy, y, ldy,
                       mk, P, C, mean, invstd, gamma, beta, act, prelu, ws);
    CN_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_bwd_finalize<3>, fin, dim3(256), 0, st, ws, gy, C, dbeta, dgamma, dprelu_c);
  } else {
    hipLaunchKernelGGL((bn_bwd_reduce_k<T, 2>), dim3(gx, gy), dim3(256), 0, st, x, ldx, dy, lddy, y, ldy,
                       mk, P, C, mean, invstd, gamma, beta, act, prelu, ws);
    CN_CHECK_LAUNCH();
    hipLaunchKernelGGL(bn_bwd_finalize<2>, fin, dim3(256), 0, st, ws, gy, C, dbeta, dgamma, dprelu_c);
  }
  CN_CHECK_LAUNCH();
  if (!dx) return 0;
  gy = grid_rows<T>(P, C, &gx, g_tune[T_BA_ROWS], g_tune[T_BA_BLOCKS]);
  hipLaunchKernelGGL(bn_bwd_apply_k<T>, dim3(gx, gy), dim3(256), 0, st, x, ldx, dy, lddy, y, ldy, mk, P,
                     C, mean, invstd, gamma, beta, act, prelu, dbeta, dgamma, dx, lddx, dres, lddres,
                     bn_wt(P, lddx, (int)sizeof(T)) && (!dres || bn_wt(P, lddres, (int)sizeof(T))));
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_bn_bwd(int dtype, const void* x, long long ldx, const void* dy, long long lddy,
                         const void* y, long long ldy, int P, int C, const float* mean,
                         const float* invstd, const float* gamma, const float* beta, int act,
                         const float* prelu, float* dgamma, float* dbeta, float* dprelu_c,
                         void* dx, long long lddx, void* dres, long long lddres, float* ws,
                         hipStream_t st) {
  const int vec = dtype == DT_BF16 ? 8 : 4;
  if (C % vec || ldx % vec || lddy % vec || (y && act != 4 && ldy % vec) || (dx && lddx % vec) ||
      (dres && lddres % vec))
    return CN_ERR_ALIGN;
  if (act == 4 && (!y || ldy < C / vec)) return CN_ERR_SHAPE;
  if (!aligned16(mean) || !aligned16(invstd) || !aligned16(gamma) || !aligned16(beta) ||
      !aligned16(dgamma) || !aligned16(dbeta))
    return CN_ERR_ALIGN;
  if (P < 1) return CN_ERR_SHAPE;
  if (dtype == DT_BF16)
    return bn_bwd_launch<bf16>((const bf16*)x, ldx, (const bf16*)dy, lddy, (const bf16*)y, ldy, P, C,
                               mean, invstd, gamma, beta, act, prelu, dgamma, dbeta, dprelu_c,
                               (bf16*)dx, lddx, (bf16*)dres, lddres, ws, st);
  return bn_bwd_launch<float>((const float*)x, ldx, (const float*)dy, lddy, (const float*)y, ldy, P, C,
                              mean, invstd, gamma, beta, act, prelu, dgamma, dbeta, dprelu_c,
                              (float*)dx, lddx, (float*)dres, lddres, ws, st);
}
