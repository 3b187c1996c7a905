// C-ABI entry points of the convolution / matrix-product family.  Each maps one reference
// aten call onto the implicit-GEMM kernel in gemm.hip (see include/cosnet_hip.h).
#include "gemm.h"
#include "../../include/cosnet_hip.h"

static GemmArgs gemm_defaults() {
  GemmArgs a = {};
  a.nsplit = 1;
  a.k_chunk = 1 << 30;
  a.alpha = 1.f;
  a.cfg = -1;
  FastDiv one = fastdiv_make(1);
  a.ga.div_C = a.ga.div_KW = a.ga.div_OW = a.ga.div_OHW = one;
  a.gb = a.ga;
  a.rm_div_OW = a.rm_div_OHW = one;
  return a;
}

static ConvGeom make_geom(int N, int H, int W, int C, int OH, int OW, int KH, int KW, int st,
                          int off_y, int off_x, int step_y, int step_x) {
  ConvGeom g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.OH = OH; g.OW = OW; g.KH = KH; g.KW = KW; g.st = st;
  g.off_y = off_y; g.off_x = off_x; g.step_y = step_y; g.step_x = step_x;
  g.div_C = fastdiv_make(C);
  g.div_KW = fastdiv_make(KW);
  g.div_OW = fastdiv_make(OW);
  g.div_OHW = fastdiv_make(OH * OW);
  return g;
}

static int vec_of(int dtype) {
  return dtype == DT_BF16 ? 8 : (dtype == DT_FP8 || dtype == DT_FP8_E5M2) ? 16 : 4;
}

// zero-fill with 16-byte vector stores (a kernel, not a memset node, inside captured graphs)
__global__ void zero16_k(u32x4* p, long long n16) {
  const u32x4 z = {0u, 0u, 0u, 0u};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n16;
       i += (long long)gridDim.x * blockDim.x)
    p[i] = z;
}

extern "C" int cn_conv_fwd(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                           const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                           const float* bias, void* y, long long ldy, int OH, int OW,
                           hipStream_t st) {
  if (Cin % vec_of(dtype) || ldx % vec_of(dtype)) return CN_ERR_ALIGN;
  if (OH != (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  if (OW != (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  GemmArgs a = gemm_defaults();
  a.M = N * OH * OW; a.N = Cout; a.K = KH * KW * Cin;
  a.ka_lim = a.kb_lim = a.K;
  a.A = x; a.lda = ldx;
  a.B = w; a.ldb = a.K;
  a.C = y; a.ldc = ldy;
  a.bias = bias;
  int la = L_KC_CONV;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) la = L_KC_DENSE;
  else a.ga = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  return cn_gemm_dispatch(a, dtype, 0, la, L_KC_DENSE, 1, st);
}

// ---- deep one-round forward convs: 256x256 tiles split over K -------------------------------
// A forward conv whose 128x256 grid is a single round (<= 256 blocks) and whose K is deep (the
// ASPP bottleneck conv: M = 28 800, N = 256, K = 9 x 2560) runs every block through the whole K
// at the bytes per FLOP of a 128x256 tile.  Split over K, 256x256 tiles give as many blocks at
// half the operand bytes per FLOP; the fp32 slabs are summed in a fixed order (bitwise
// reproducible) by a reduce that adds the bias and writes the bf16 output.
static int fwd_split_plan(int dtype, int M, int N, int K, int* nsplit, int* chunk) {
  *nsplit = 1; *chunk = K;
  if (dtype != DT_BF16 || K < 16384 || N > 256 || N % 8) return 0;
  if (cn_gemm_cfg_blocks(19, M, N) > 256) return 0;
  const long long b20 = cn_gemm_cfg_blocks(20, M, N);
  int ns = (int)(256 / b20);
  if (ns < 2) ns = 2;
  if (ns > 8) ns = 8;
  const int bk = 64;
  const int ch = ((K + ns - 1) / ns + bk - 1) / bk * bk;
  *nsplit = (K + ch - 1) / ch;
  *chunk = ch;
  return *nsplit > 1;
}

__global__ __launch_bounds__(256) void splitk_reduce_bf16_k(const float* __restrict__ ws, int nsplit,
                                                            long long slab, int M, int N,
                                                            const float* __restrict__ bias,
                                                            bf16* __restrict__ y, long long ldy) {
  const int cpr = N / 8;
  const long long total = (long long)M * cpr;
  for (long long t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int r = (int)(t / cpr), c = (int)(t - (long long)r * cpr) * 8;
    const float* p = ws + (long long)r * N + c;
    f32x4 a0 = *(const f32x4*)p, a1 = *(const f32x4*)(p + 4);
    for (int sp = 1; sp < nsplit; ++sp) {
      a0 += *(const f32x4*)(p + sp * slab);
      a1 += *(const f32x4*)(p + sp * slab + 4);
    }
    float f[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    if (bias) {
#pragma unroll
      for (int v = 0; v < 8; ++v) f[v] += bias[c + v];
    }
    *(u32x4*)(y + (long long)r * ldy + c) = Chunk<bf16>::pack(f);
  }
}

extern "C" size_t cn_conv_fwd_workspace_floats(int dtype, int M, int Cout, int K) {
  int ns, ch;
  return fwd_split_plan(dtype, M, Cout, K, &ns, &ch) ? (size_t)ns * M * Cout : 0;
}

// cn_conv_fwd with a workspace: the deep one-round shapes (fwd_split_plan) run split over K into
// ws (cn_conv_fwd_workspace_floats floats, 16-byte aligned); every other shape, or a missing /
// too small workspace, is cn_conv_fwd.
extern "C" int cn_conv_fwd_ws(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                              const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                              const float* bias, void* y, long long ldy, int OH, int OW, float* ws,
                              size_t ws_floats, hipStream_t st) {
  int ns, ch;
  const int M = N * OH * OW, K = KH * KW * Cin;
  if (!ws || ((uintptr_t)ws & 15) || ((uintptr_t)y & 15) || ldy % 8 ||
      !fwd_split_plan(dtype, M, Cout, K, &ns, &ch) || ws_floats < (size_t)ns * M * Cout)
    return cn_conv_fwd(dtype, x, ldx, N, H, W, Cin, w, Cout, KH, KW, stride, pad, dil, bias, y, ldy,
                       OH, OW, st);
  if (Cin % vec_of(dtype) || ldx % vec_of(dtype)) return CN_ERR_ALIGN;
  if (OH != (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  if (OW != (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  GemmArgs a = gemm_defaults();
  a.M = M; a.N = Cout; a.K = K;
  a.ka_lim = a.kb_lim = a.K;
  a.A = x; a.lda = ldx;
  a.B = w; a.ldb = a.K;
  a.C = ws; a.ldc = Cout;
  a.c_mode = 3;
  a.nsplit = ns;
  a.k_chunk = ch;
  a.slab = (long long)M * Cout;
  a.cfg = 20;
  int la = L_KC_CONV;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) la = L_KC_DENSE;
  else a.ga = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  int rc = cn_gemm_dispatch(a, dtype, 1, la, L_KC_DENSE, 1, st);
  if (rc) return rc;
  const long long total = (long long)M * (Cout / 8);
  long long nb = (total + 255) / 256;
  if (nb > 4096) nb = 4096;
  hipLaunchKernelGGL(splitk_reduce_bf16_k, dim3((unsigned)nb), dim3(256), 0, st, ws, ns, a.slab, M,
                     Cout, bias, (bf16*)y, ldy);
  CN_CHECK_LAUNCH();
  return 0;
}

// ---- conv + BatchNorm epilogues ------------------------------------------------------------
int cn_bn_tile_stats_impl(const float* ws, long long plane, int mtiles, int BM, int M, int nseg, int C,
                          float* mean, float* invstd, float* run_mean, float* run_var, float momentum,
                          float eps, hipStream_t st);
int cn_bn_tile_bwd_impl(const float* ws, int mtiles, int C, float* sum_dz, float* sum_dzxh,
                        hipStream_t st);

static int conv_fwd_args(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                         const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                         const float* bias, void* y, long long ldy, int OH, int OW, GemmArgs& a,
                         int& la) {
  if (Cin % vec_of(dtype) || ldx % vec_of(dtype)) return CN_ERR_ALIGN;
  if (OH != (H + 2 * pad - dil * (KH - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  if (OW != (W + 2 * pad - dil * (KW - 1) - 1) / stride + 1) return CN_ERR_SHAPE;
  a = gemm_defaults();
  a.M = N * OH * OW; a.N = Cout; a.K = KH * KW * Cin;
  a.ka_lim = a.kb_lim = a.K;
  a.A = x; a.lda = ldx;
  a.B = w; a.ldb = a.K;
  a.C = y; a.ldc = ldy;
  a.bias = bias;
  la = L_KC_CONV;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) la = L_KC_DENSE;
  else a.ga = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  return 0;
}

// y (bf16) = conv2d(x8, w8) * x_scale * w_scale (+ bias): fp8 e4m3 operands (cn_fp8_quant), fp32
// accumulation on the block-scaled 16x16x128 MFMA, per-tensor dequantisation in the epilogue.
extern "C" int cn_conv_fwd_fp8(const void* x8, long long ldx, int N, int H, int W, int Cin,
                               const void* w8, int Cout, int KH, int KW, int stride, int pad, int dil,
                               const float* bias, void* y, long long ldy, int OH, int OW,
                               const float* x_state, const float* w_state, hipStream_t st) {
  if (Cin % 16 || ldx % 16 || ((uintptr_t)x8 & 15) || ((uintptr_t)w8 & 15)) return CN_ERR_ALIGN;
  GemmArgs a;
  int la;
  int rc = conv_fwd_args(DT_BF16, x8, ldx, N, H, W, Cin, w8, Cout, KH, KW, stride, pad, dil, bias, y,
                         ldy, OH, OW, a, la);
  if (rc) return rc;
  a.scale_a = x_state;   // state[0] = dequantisation scale
  a.scale_b = w_state;
  return cn_gemm_dispatch(a, DT_FP8, 0, la, L_KC_DENSE, 1, st);
}

// dx (bf16) (+)= conv_dgrad(dy8, wt8) * dy_scale * w_scale, stride 1: e5m2 output gradients
// (delayed scaling, cn_fp8_quant_fmt) x e4m3 transposed weights [Cin][KH][KW][Cout] on the
// block-scaled 16x16x128 MFMA (A format e5m2, B e4m3), fp32 accumulation.
extern "C" int cn_conv_dgrad_fp8(const void* dy8, long long lddy, int N, int OH, int OW, int Cout,
                                 const void* wt8, int Cin, int KH, int KW, int pad, int dil,
                                 void* dx, long long lddx, int H, int W, int accumulate,
                                 const float* dy_state, const float* w_state, hipStream_t st) {
  if (Cout % 16 || lddy % 16 || ((uintptr_t)dy8 & 15) || ((uintptr_t)wt8 & 15)) return CN_ERR_ALIGN;
  if (lddx % 8 || ((uintptr_t)dx & 15)) return CN_ERR_ALIGN;
  if (OH != H + 2 * pad - dil * (KH - 1) || OW != W + 2 * pad - dil * (KW - 1)) return CN_ERR_SHAPE;
  GemmArgs a = gemm_defaults();
  a.M = N * H * W; a.N = Cin; a.K = KH * KW * Cout;
  a.ka_lim = a.kb_lim = a.K;
  a.A = dy8; a.lda = lddy;
  a.B = wt8; a.ldb = a.K;
  a.C = dx; a.ldc = lddx;
  a.c_mode = accumulate ? 2 : 0;
  a.scale_a = dy_state;
  a.scale_b = w_state;
  int la = L_KC_DENSE;
  if (!(KH == 1 && KW == 1 && pad == 0)) {
    la = L_KC_CONV;
    a.ga = make_geom(N, OH, OW, Cout, H, W, KH, KW, 1, pad, pad, -dil, -dil);
  }
  return cn_gemm_dispatch(a, DT_FP8_E5M2, 0, la, L_KC_DENSE, 1, st);
}

static long long mtiles_of(int dtype, int M, int N, int K) {
  const int bm = cn_gemm_bm(dtype, M, N, K, -1);
  return (M + bm - 1) / bm;
}

extern "C" size_t cn_conv_fwd_bn_workspace_floats(int dtype, int M, int Cout, int K) {
  return (size_t)5 * mtiles_of(dtype, M, Cout, K) * Cout;
}

// y = conv2d(x, w) + bias, and the train-mode BatchNorm statistics of y computed in the GEMM
// epilogue (no separate pass over y): mean / invstd [nseg][Cout] of each of the nseg stacked
// row segments (frames), running stats updated segment after segment.
extern "C" int cn_conv_fwd_bn(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                              const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                              const float* bias, void* y, long long ldy, int OH, int OW, int nseg,
                              float* ws, float* mean, float* invstd, float* run_mean, float* run_var,
                              float momentum, float eps, hipStream_t st) {
  GemmArgs a;
  int la;
  int rc = conv_fwd_args(dtype, x, ldx, N, H, W, Cin, w, Cout, KH, KW, stride, pad, dil, bias, y,
                         ldy, OH, OW, a, la);
  if (rc) return rc;
  if (nseg < 1 || a.M % nseg || !ws) return CN_ERR_SHAPE;
  const int bm = cn_gemm_bm(dtype, a.M, a.N, a.K, -1);
  const long long mt = (a.M + bm - 1) / bm;
  a.st_mode = 1;
  a.st_ws = ws;
  a.st_plane = mt * Cout;
  a.st_seg_rows = a.M / nseg;
  rc = cn_gemm_dispatch(a, dtype, 0, la, L_KC_DENSE, 1, st);
  if (rc) return rc;
  return cn_bn_tile_stats_impl(ws, a.st_plane, (int)mt, bm, a.M, nseg, Cout, mean, invstd, run_mean,
                               run_var, momentum, eps, st);
}

// fp8 conv (cn_conv_fwd_fp8) with the BN statistics in its GEMM epilogue (cn_conv_fwd_bn's
// reduction of the stored bf16 y), for configs[4]'s long-K narrow convs.  ws:
// cn_conv_fwd_bn_workspace_floats(DT_FP8, M, Cout, K) floats.
extern "C" int cn_conv_fwd_fp8_bn(const void* x8, long long ldx, int N, int H, int W, int Cin,
                                  const void* w8, int Cout, int KH, int KW, int stride, int pad,
                                  int dil, const float* bias, void* y, long long ldy, int OH, int OW,
                                  const float* x_state, const float* w_state, int nseg, float* ws,
                                  float* mean, float* invstd, float* run_mean, float* run_var,
                                  float momentum, float eps, hipStream_t st) {
  if (Cin % 16 || ldx % 16 || ((uintptr_t)x8 & 15) || ((uintptr_t)w8 & 15)) return CN_ERR_ALIGN;
  GemmArgs a;
  int la;
  int rc = conv_fwd_args(DT_BF16, x8, ldx, N, H, W, Cin, w8, Cout, KH, KW, stride, pad, dil, bias, y,
                         ldy, OH, OW, a, la);
  if (rc) return rc;
  if (nseg < 1 || a.M % nseg || !ws) return CN_ERR_SHAPE;
  a.scale_a = x_state;
  a.scale_b = w_state;
  const int bm = cn_gemm_bm(DT_FP8, a.M, a.N, a.K, -1);
  const long long mt = (a.M + bm - 1) / bm;
  a.st_mode = 1;
  a.st_ws = ws;
  a.st_plane = mt * Cout;
  a.st_seg_rows = a.M / nseg;
  rc = cn_gemm_dispatch(a, DT_FP8, 0, la, L_KC_DENSE, 1, st);
  if (rc) return rc;
  return cn_bn_tile_stats_impl(ws, a.st_plane, (int)mt, bm, a.M, nseg, Cout, mean, invstd, run_mean,
                               run_var, momentum, eps, st);
}

// G stride-1 'same' convs of one input x and one shape that differ in dilation (pad = dil), bias
// and weights -- the ASPP's atrous branches (deeplab/deeplabv3_encoder.py:22-31, :70-76) -- as ONE
// grouped GEMM launch (blockIdx.z = branch) with the BN-statistics epilogue of cn_conv_fwd_bn per
// branch.  The branches' launches are each one round of the chip whose time the tiles without
// tap skipping set (§3.1); grouped, their tiles share the rounds.  w, bias, y, ws, mean, invstd,
// run_mean, run_var, dil: host arrays of G entries (device pointers / ints); ws[g]:
// cn_conv_fwd_bn_workspace_floats(dtype, M, Cout, K) floats each.  G <= 24.
extern "C" int cn_conv_fwd_bn_grouped(int dtype, const void* x, long long ldx, int N, int H, int W,
                                      int Cin, int G, const void* const* w, int Cout, int KH, int KW,
                                      const int* dil, const float* const* bias, void* const* y,
                                      long long ldy, int nseg, float* const* ws, float* const* mean,
                                      float* const* invstd, float* const* run_mean,
                                      float* const* run_var, float momentum, float eps, hipStream_t st) {
  if (G < 1 || G > GEMM_MAXG || KH != KW || KH % 2 == 0) return CN_ERR_SHAPE;
  GemmArgs a;
  int la;
  const int d0 = dil[0], p0 = d0 * (KH / 2);
  int rc = conv_fwd_args(dtype, x, ldx, N, H, W, Cin, w[0], Cout, KH, KW, 1, p0, d0, bias[0], y[0],
                         ldy, H, W, a, la);
  if (rc) return rc;
  if (la != L_KC_CONV || nseg < 1 || a.M % nseg) return CN_ERR_SHAPE;
  const int bm = cn_gemm_bm(dtype, a.M, a.N, a.K, -1);
  const long long mt = (a.M + bm - 1) / bm;
  a.ngroup = G;
  for (int g = 0; g < G; ++g) {
    if (dil[g] < 1 || !ws[g]) return CN_ERR_SHAPE;
    a.grp.A[g] = x;
    a.grp.B[g] = w[g];
    a.grp.C[g] = y[g];
    a.grp.bias[g] = bias[g];
    a.grp.ST[g] = ws[g];
    a.grp.dil[g] = dil[g];
  }
  a.st_mode = 1;
  a.st_ws = ws[0];
  a.st_plane = mt * Cout;
  a.st_seg_rows = a.M / nseg;
  rc = cn_gemm_dispatch(a, dtype, 0, la, L_KC_DENSE, G, st);
  if (rc) return rc;
  for (int g = 0; g < G; ++g) {
    rc = cn_bn_tile_stats_impl(ws[g], a.st_plane, (int)mt, bm, a.M, nseg, Cout, mean[g], invstd[g],
                               run_mean[g], run_var[g], momentum, eps, st);
    if (rc) return rc;
  }
  return 0;
}

extern "C" size_t cn_conv_dgrad_bn_workspace_floats(int dtype, int M, int Cin, int K) {
  return (size_t)2 * mtiles_of(dtype, M, Cin, K) * Cin;
}

// dy = conv2d input-gradient (stride 1) AND, in the GEMM epilogue, the reduction of the backward
// of the BatchNorm + ReLU that produced the conv's input: with x the BN's pre-activation input
// (same [P][Cin] rows), dz = dy * (relu mask recomputed from x with the forward affine),
// sum_dz[c] = sum dz, sum_dzxh[c] = sum dz * (x - mean) * invstd  (= the BN's dbeta / dgamma).
// cn_bn_bwd_apply then forms dx of the BN from these sums.
extern "C" int cn_conv_dgrad_bn(int dtype, const void* dy, long long lddy, int N, int OH, int OW,
                                int Cout, const void* wt, int Cin, int KH, int KW, int pad, int dil,
                                void* dx, long long lddx, int H, int W, const void* x, long long ldx,
                                const float* mean, const float* invstd, const float* gamma,
                                const float* beta, float* sum_dz, float* sum_dzxh, float* ws,
                                hipStream_t st) {
  if (Cout % vec_of(dtype) || lddy % vec_of(dtype) || ldx % vec_of(dtype)) return CN_ERR_ALIGN;
  if (!ws || !x || !mean || !invstd) return CN_ERR_SHAPE;
  GemmArgs a = gemm_defaults();
  a.N = Cin; a.K = KH * KW * Cout;
  a.ka_lim = a.kb_lim = a.K;
  a.A = dy; a.lda = lddy;
  a.B = wt; a.ldb = a.K;
  a.C = dx; a.ldc = lddx;
  a.M = N * H * W;
  int la = L_KC_DENSE;
  if (!(KH == 1 && KW == 1 && pad == 0)) {
    la = L_KC_CONV;
    a.ga = make_geom(N, OH, OW, Cout, H, W, KH, KW, 1, pad, pad, -dil, -dil);
  }
  const int bm = cn_gemm_bm(dtype, a.M, a.N, a.K, -1);
  const long long mt = (a.M + bm - 1) / bm;
  a.st_mode = 2;
  a.st_ws = ws;
  a.st_plane = mt * Cin;
  a.br_x = x; a.br_ldx = ldx;
  a.br_mean = mean; a.br_invstd = invstd; a.br_gamma = gamma; a.br_beta = beta;
  int rc = cn_gemm_dispatch(a, dtype, 0, la, L_KC_DENSE, 1, st);
  if (rc) return rc;
  return cn_bn_tile_bwd_impl(ws, (int)mt, Cin, sum_dz, sum_dzxh, st);
}

extern "C" int cn_conv_dgrad(int dtype, const void* dy, long long lddy, int N, int OH, int OW,
                             int Cout, const void* wt, int Cin, int KH, int KW, int stride,
                             int pad, int dil, void* dx, long long lddx, int H, int W,
                             int accumulate, hipStream_t st) {
  if (Cout % vec_of(dtype) || lddy % vec_of(dtype)) return CN_ERR_ALIGN;
  GemmArgs a = gemm_defaults();
  a.N = Cin; a.K = KH * KW * Cout;
  a.ka_lim = a.kb_lim = a.K;
  a.A = dy; a.lda = lddy;
  a.B = wt; a.ldb = a.K;
  a.C = dx; a.ldc = lddx;
  a.c_mode = accumulate ? 2 : 0;
  if (stride == 1) {
    a.M = N * H * W;
    int la = L_KC_DENSE;
    if (!(KH == 1 && KW == 1 && pad == 0)) {
      la = L_KC_CONV;  // dX[n,h,w] = sum_{r,s} dY[n, h + pad - r*dil, w + pad - s*dil] . W[r,s]
      a.ga = make_geom(N, OH, OW, Cout, H, W, KH, KW, 1, pad, pad, -dil, -dil);
    }
    return cn_gemm_dispatch(a, dtype, 0, la, L_KC_DENSE, 1, st);
  }
  if (KH != 1 || KW != 1 || pad != 0) return CN_ERR_UNSUPPORTED;
  if (stride != 2) return CN_ERR_UNSUPPORTED;
  // 1x1 stride 2: only input pixels (2oy, 2ox) receive gradient; zero the rest first
  // (unless accumulating into an existing gradient).
  if (!accumulate) {
    if (lddx != Cin) return CN_ERR_ALIGN;
    long long n16 = (long long)N * H * W * Cin / vec_of(dtype);
    if (((long long)Cin % vec_of(dtype)) || ((uintptr_t)dx & 15)) return CN_ERR_ALIGN;
    long long nb = (n16 + 255) / 256;
    hipLaunchKernelGGL(zero16_k, dim3(nb < 4096 ? nb : 4096), dim3(256), 0, st, (u32x4*)dx, n16);
    CN_CHECK_LAUNCH();
  }
  a.M = N * OH * OW;
  a.row_map = 1;
  a.rm_div_OW = fastdiv_make(OW);
  a.rm_div_OHW = fastdiv_make(OH * OW);
  a.rm_H = H; a.rm_W = W;
  return cn_gemm_dispatch(a, dtype, 0, L_KC_DENSE, L_KC_DENSE, 1, st);
}


// Weight-gradient plan: tile configuration and K split (M = Cout, N = KH*KW*Cin, K = pixels).
// 128x128 tiles with 8 waves (128x64 for the fp32 parity path); enough K splits to give ~2
// blocks per CU, each split keeping >= 8 K tiles.
static int g_wgrad_target = 512;

// Development hook (tuning tools only): blocks the wgrad K split aims for.
extern "C" int cn_gemm_set_wgrad_target(int blocks) {
  if (blocks < 1) return CN_ERR_SHAPE;
  g_wgrad_target = blocks;
  return 0;
}

// G > 1: the split for G problems of this shape in one launch (cn_conv_wgrad_grouped_ws), the
// block target shared by the G problems.
static void wgrad_plan(int dtype, int N, int OH, int OW, int Cout, int KH, int KW, int Cin, int* nsplit,
                       int* chunk, int* cfg, int G = 1) {
  int M = Cout, NN = KH * KW * Cin, K = N * OH * OW;
  int BK = 8 * vec_of(dtype);
  long long tiles;
  int target = g_wgrad_target;
  if (dtype == DT_FP8_E5M2) {
    // fp8 operands: 128x128 / 8 waves (the k-major fp8 reader's tile), the bf16 block target
    *cfg = 11;
    tiles = cn_gemm_cfg_blocks(11, M, NN) * G;
    if (target == 512) {
      if (tiles >= 256) target = 1024;
      else {
        long long s = 512 / tiles;
        long long maxs = K / (8 * BK);
        if (s > maxs) s = maxs;
        if (s < 1) s = 1;
        target = (int)(s * tiles);
      }
    }
  } else if (dtype == DT_BF16) {
    // 128x128 / 8 waves (tools/wgrad_sweep.sh); the narrow layer-1 products get tiles that
    // do not waste half their MFMAs: 128x64 for N <= 64, 64x128 for Cout <= 64
    *cfg = NN <= 64 ? 12 : (M <= 64 ? 17 : 11);
    tiles = cn_gemm_cfg_blocks(*cfg, M, NN) * G;
    // split count from a per-split sweep on the step's shapes (tools/wgrad_bench.py,
    // profiles/r03_wgrad_splits.txt): up to 512 blocks = two co-resident blocks per CU, never a
    // third round (layer-3 3x3: 8 -> 14 splits 44.6 -> 37.0 us, layer-4 3x3: 2 -> 3 splits
    // 117.7 -> 91.6 us, layer-3 1x1: 15 -> 28 splits -4 %); many tiles (ASPP) -> 2 per tile
    if (target == 512) {
      if (tiles >= 256) target = 1024;
      else {
        long long s = 512 / tiles;
        long long maxs = K / (8 * BK);
        if (s > maxs) s = maxs;
        if (s < 1) s = 1;
        target = (int)(s * tiles);   // want = ceil(target / tiles) = s below
      }
    }
  } else {
    *cfg = -1;
    // the fp32 parity path's 128x64 tiles; a group's G problems share the block target
    tiles = (long long)((M + 127) / 128) * ((NN + 63) / 64) * G;
  }
  long long want = (target + tiles - 1) / tiles;
  long long maxs = K / (8 * BK);
  if (maxs < 1) maxs = 1;
  if (want > maxs) want = maxs;
  if (want < 1) want = 1;
  int ns = (int)want;
  int ch = (K + ns - 1) / ns;
  ch = (ch + BK - 1) / BK * BK;
  *nsplit = (K + ch - 1) / ch;
  *chunk = ch;
}

extern "C" size_t cn_conv_wgrad_workspace_floats(int dtype, int N, int OH, int OW, int Cout, int KH,
                                                 int KW, int Cin) {
  int ns, ch, cfg;
  wgrad_plan(dtype, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg);
  return ns > 1 ? (size_t)ns * Cout * KH * KW * Cin : 0;
}

extern "C" int cn_conv_wgrad(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                             const void* dy, long long lddy, int OH, int OW, int Cout, int KH,
                             int KW, int stride, int pad, int dil, float* dw, float* ws,
                             hipStream_t st) {
  if (Cin % vec_of(dtype) || Cout % vec_of(dtype)) return CN_ERR_ALIGN;
  GemmArgs a = gemm_defaults();
  a.M = Cout; a.N = KH * KW * Cin; a.K = N * OH * OW;
  a.ka_lim = a.kb_lim = a.K;
  a.A = dy; a.lda = lddy;
  a.B = x; a.ldb = ldx;
  a.ldc = a.N;
  int lb = L_MC_DENSE;
  if (!(KH == 1 && KW == 1 && stride == 1 && pad == 0)) {
    lb = L_MC_CONV;
    a.gb = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  }
  int ns, ch, cfg;
  wgrad_plan(dtype, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg);
  a.cfg = cfg;
  a.nsplit = ns;
  a.k_chunk = ch;
  if (ns == 1) {  // whole K in one block: write dw directly
    a.C = dw;
    return cn_gemm_dispatch(a, dtype, 1, L_MC_DENSE, lb, 1, st);
  }
  if (!ws) return CN_ERR_SHAPE;
  // split-K partials into fp32 slabs (plain stores, no atomics), then a fixed-order sum
  a.C = ws;
  a.c_mode = 3;
  a.slab = (long long)a.M * a.N;
  int rc = cn_gemm_dispatch(a, dtype, 1, L_MC_DENSE, lb, 1, st);
  if (rc) return rc;
  return cn_splitk_reduce_impl(ws, ns, a.slab, a.slab, dw, 0, st);
}

// G independent weight gradients of one conv shape (the same conv of the bottlenecks of a
// layer) in ONE launch: blockIdx.z = problem, every block runs the whole K (all pixels), so there
// is no split-K slab and no reduce launch; dW[g] fp32 [Cout][KH][KW][Cin] written directly.
// The per-problem launch needs split-K to fill the chip (14-28 splits on the layer-3 shapes);
// G problems of 36 (3x3) or 16 (1x1) tiles do so on their own.
extern "C" int cn_conv_wgrad_grouped(int dtype, int G, const void* const* xs, long long ldx, int N,
                                     int H, int W, int Cin, const void* const* dys, long long lddy,
                                     int OH, int OW, int Cout, int KH, int KW, int stride, int pad,
                                     int dil, float* const* dws, hipStream_t st) {
  if (G < 1 || G > GEMM_MAXG) return CN_ERR_SHAPE;
  if (Cin % vec_of(dtype) || Cout % vec_of(dtype)) return CN_ERR_ALIGN;
  GemmArgs a = gemm_defaults();
  a.M = Cout; a.N = KH * KW * Cin; a.K = N * OH * OW;
  a.ka_lim = a.kb_lim = a.K;
  a.lda = lddy;
  a.ldb = ldx;
  a.ldc = a.N;
  int lb = L_MC_DENSE;
  if (!(KH == 1 && KW == 1 && stride == 1 && pad == 0)) {
    lb = L_MC_CONV;
    a.gb = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  }
  a.ngroup = G;
  for (int g = 0; g < G; ++g) {
    a.grp.A[g] = dys[g];
    a.grp.B[g] = xs[g];
    a.grp.C[g] = dws[g];
  }
  // the first problem's pointers for the loaders' range checks (every problem has this shape)
  a.A = dys[0]; a.B = xs[0]; a.C = dws[0];
  if (dtype == DT_BF16) {
    // 256x128 tiles (3-deep ring) when they give >= 160 blocks: every block runs the whole K,
    // so the larger tile's fewer bytes per FLOP pay wherever the grid still covers most CUs
    // (layer-3 groups 334 -> 250 us (1x1), 561 -> 471 us (3x3), tools/wgrad_grouped_bench.py,
    // profiles/r03_wgrad_grouped_cfgs.txt); else 128x128 with a 3-deep ring (the depth
    // encoder's groups of 5-6 and the layer-4 1x1s: 141 -> 130 us, 159 -> 140 us, 148 -> 130 us)
    a.cfg = (long long)cn_gemm_cfg_blocks(15, a.M, a.N) * G >= 160 ? 15 : 13;
    if (a.M <= 64) a.cfg = 17;
  }
  return cn_gemm_dispatch(a, dtype, 1, L_MC_DENSE, lb, G, st);
}

// ---- grouped weight gradients split over K --------------------------------------------------
// The small bottleneck weight gradients (layers 1-2: 8-36 tiles per problem) fill the chip
// neither one by one (100-225 blocks each, plus a reduce launch each) nor grouped without a
// split (G x 8-36 blocks running K = all pixels).  Here G problems x nsplit K chunks run as ONE
// launch (blockIdx.z = problem x split; slabs ws[g][s][Cout*KH*KW*Cin], plain stores), then ONE
// reduce launch sums every problem's slabs in split order (deterministic) into its dW.
namespace {
struct RedOut { float* out[GEMM_MAXG]; };
__global__ __launch_bounds__(256) void splitk_reduce_grouped_k(const float* __restrict__ ws, int nsplit,
                                                               long long slab, long long n4, RedOut o) {
  const int g = blockIdx.y;
  const float* wg = ws + (long long)g * nsplit * slab;
  for (long long i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 8 <= nsplit; s += 8) {
      f32x4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(wg + (long long)(s + u) * slab + 4 * i);
#pragma unroll
      for (int u = 0; u < 8; ++u) a += v[u];
    }
    for (; s < nsplit; ++s) a += *(const f32x4*)(wg + (long long)s * slab + 4 * i);
    ((f32x4*)o.out[g])[i] = a;
  }
}
}  // namespace

extern "C" size_t cn_conv_wgrad_grouped_workspace_floats(int dtype, int G, int N, int OH, int OW,
                                                         int Cout, int KH, int KW, int Cin) {
  if (G < 1) return 0;
  int ns, ch, cfg;
  wgrad_plan(dtype, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg, G);
  return ns > 1 ? (size_t)G * ns * Cout * KH * KW * Cin : 0;
}

extern "C" int cn_conv_wgrad_grouped_ws(int dtype, int G, const void* const* xs, long long ldx, int N,
                                        int H, int W, int Cin, const void* const* dys, long long lddy,
                                        int OH, int OW, int Cout, int KH, int KW, int stride, int pad,
                                        int dil, float* const* dws, float* ws, size_t ws_floats,
                                        hipStream_t st) {
  if (G < 1 || G > GEMM_MAXG) return CN_ERR_SHAPE;
  if (Cin % vec_of(dtype) || Cout % vec_of(dtype)) return CN_ERR_ALIGN;
  int ns, ch, cfg;
  wgrad_plan(dtype, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg, G);
  const long long slab = (long long)Cout * KH * KW * Cin;
  if (ns <= 1 || !ws || ws_floats < (size_t)G * ns * slab || ((uintptr_t)ws & 15) || slab % 4)
    return cn_conv_wgrad_grouped(dtype, G, xs, ldx, N, H, W, Cin, dys, lddy, OH, OW, Cout, KH, KW,
                                 stride, pad, dil, dws, st);
  for (int g = 0; g < G; ++g)
    if ((uintptr_t)dws[g] & 15) return CN_ERR_ALIGN;
  GemmArgs a = gemm_defaults();
  a.M = Cout; a.N = KH * KW * Cin; a.K = N * OH * OW;
  a.ka_lim = a.kb_lim = a.K;
  a.lda = lddy;
  a.ldb = ldx;
  a.ldc = a.N;
  int lb = L_MC_DENSE;
  if (!(KH == 1 && KW == 1 && stride == 1 && pad == 0)) {
    lb = L_MC_CONV;
    a.gb = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  }
  a.ngroup = G;
  for (int g = 0; g < G; ++g) {
    a.grp.A[g] = dys[g];
    a.grp.B[g] = xs[g];
    a.grp.C[g] = ws + (long long)g * ns * slab;   // problem g's slabs
  }
  a.A = dys[0]; a.B = xs[0]; a.C = ws;
  a.cfg = cfg;
  a.nsplit = ns;
  a.k_chunk = ch;
  a.c_mode = 3;
  a.slab = slab;
  int rc = cn_gemm_dispatch(a, dtype, 1, L_MC_DENSE, lb, G, st);
  if (rc) return rc;
  RedOut o;
  for (int g = 0; g < G; ++g) o.out[g] = dws[g];
  const long long n4 = slab / 4;
  long long bx = (n4 + 255) / 256;
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(splitk_reduce_grouped_k, dim3((unsigned)bx, G), dim3(256), 0, st, (const float*)ws,
                     ns, slab, n4, o);
  CN_CHECK_LAUNCH();
  return 0;
}

// ---- fp8 weight gradients (BASELINE configs[4]) ------------------------------------------------
// dW[g] fp32 [Cout][KH][KW][Cin] = sum over output pixels of dY8[g] (e5m2) x im2col(X8[g]) (e4m3) *
// dy_scale[g] * x_scale[g]: the weight gradients of G convs of one shape in one launch (G = 1: a
// single conv), both operands k-major (pixel rows) -- the e5m2 output gradient the fp8 dgrad
// already quantised and the e4m3 input copy the fp8 forward conv read -- on the block-scaled
// 16x16x128 MFMA (A e5m2, B e4m3, unit block scales) with transposed byte reads of the LDS tiles
// (gemm.hip read_frag_f8_mc).  Split over K into fp32 slabs when the group does not fill the chip
// (wgrad_plan), summed in split order by one reduce launch (deterministic).
extern "C" size_t cn_conv_wgrad_fp8_workspace_floats(int G, int N, int OH, int OW, int Cout, int KH,
                                                     int KW, int Cin) {
  if (G < 1) return 0;
  int ns, ch, cfg;
  wgrad_plan(DT_FP8_E5M2, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg, G);
  return ns > 1 ? (size_t)G * ns * Cout * KH * KW * Cin : 0;
}

extern "C" int cn_conv_wgrad_fp8(int G, const void* const* xs8, long long ldx, int N, int H, int W,
                                 int Cin, const void* const* dys8, long long lddy, int OH, int OW,
                                 int Cout, int KH, int KW, int stride, int pad, int dil,
                                 float* const* dws, const float* const* x_states,
                                 const float* const* dy_states, float* ws, size_t ws_floats,
                                 hipStream_t st) {
  if (G < 1 || G > GEMM_MAXG) return CN_ERR_SHAPE;
  if (Cin % 16 || Cout % 16 || ldx % 16 || lddy % 16) return CN_ERR_ALIGN;
  for (int g = 0; g < G; ++g)
    if (((uintptr_t)xs8[g] & 15) || ((uintptr_t)dys8[g] & 15) || ((uintptr_t)dws[g] & 15) ||
        !x_states[g] || !dy_states[g])
      return CN_ERR_ALIGN;
  int ns, ch, cfg;
  wgrad_plan(DT_FP8_E5M2, N, OH, OW, Cout, KH, KW, Cin, &ns, &ch, &cfg, G);
  const long long slab = (long long)Cout * KH * KW * Cin;
  const bool split = ns > 1;
  if (split && (!ws || ws_floats < (size_t)G * ns * slab || ((uintptr_t)ws & 15) || slab % 4))
    return CN_ERR_SHAPE;
  GemmArgs a = gemm_defaults();
  a.M = Cout; a.N = KH * KW * Cin; a.K = N * OH * OW;
  a.ka_lim = a.kb_lim = a.K;
  a.lda = lddy;
  a.ldb = ldx;
  a.ldc = a.N;
  int lb = L_MC_DENSE;
  if (!(KH == 1 && KW == 1 && stride == 1 && pad == 0)) {
    lb = L_MC_CONV;
    a.gb = make_geom(N, H, W, Cin, OH, OW, KH, KW, stride, -pad, -pad, dil, dil);
  }
  a.ngroup = G;
  for (int g = 0; g < G; ++g) {
    a.grp.A[g] = dys8[g];
    a.grp.B[g] = xs8[g];
    a.grp.C[g] = split ? (void*)(ws + (long long)g * ns * slab) : (void*)dws[g];
    a.grp.SA[g] = dy_states[g];   // state[0] = dequantisation scale
    a.grp.SB[g] = x_states[g];
  }
  a.A = dys8[0]; a.B = xs8[0]; a.C = a.grp.C[0];
  if (split) {
    a.cfg = 11;
    a.nsplit = ns;
    a.k_chunk = ch;
    a.c_mode = 3;
    a.slab = slab;
  } else {
    a.cfg = 13;   // every block runs the whole K: the 3-deep ring (as the bf16 groups)
  }
  int rc = cn_gemm_dispatch(a, DT_FP8_E5M2, 1, L_MC_DENSE, lb, G, st);
  if (rc || !split) return rc;
  RedOut o;
  for (int g = 0; g < G; ++g) o.out[g] = dws[g];
  const long long n4 = slab / 4;
  long long bx = (n4 + 255) / 256;
  if (bx > 1024) bx = 1024;
  hipLaunchKernelGGL(splitk_reduce_grouped_k, dim3((unsigned)bx, G), dim3(256), 0, st, (const float*)ws,
                     ns, slab, n4, o);
  CN_CHECK_LAUNCH();
  return 0;
}

extern "C" int cn_splitk_reduce(const float* ws, int nsplit, long long slab, long long n, float* out,
                                int accumulate, hipStream_t st) {
  return cn_splitk_reduce_impl(ws, nsplit, slab, n, out, accumulate, st);
}

extern "C" int cn_gemm(int dtype, int layout_a, int layout_b, int M, int N, int K, int ka_lim,
                       int kb_lim, const void* A, long long lda, long long a_bs, const void* B,
                       long long ldb, long long b_bs, void* C, long long ldc, long long c_bs,
                       int c_f32, int c_mode, float alpha, const float* bias, int batch,
                       int nsplit, long long slab, hipStream_t st) {
  GemmArgs a = gemm_defaults();
  a.M = M; a.N = N; a.K = K;
  a.ka_lim = ka_lim; a.kb_lim = kb_lim;
  a.A = A; a.lda = lda; a.a_bs = a_bs;
  a.B = B; a.ldb = ldb; a.b_bs = b_bs;
  a.C = C; a.ldc = ldc; a.c_bs = c_bs;
  a.bias = bias;
  a.alpha = alpha;
  a.c_mode = c_mode;
  a.slab = slab;
  if ((c_mode == 1 || c_mode == 3) && !c_f32) return CN_ERR_UNSUPPORTED;
  if (nsplit > 1) {
    int BK = 8 * vec_of(dtype);
    int chunk = (K + nsplit - 1) / nsplit;
    chunk = (chunk + BK - 1) / BK * BK;
    a.nsplit = (K + chunk - 1) / chunk;
    a.k_chunk = chunk;
  }
  return cn_gemm_dispatch(a, dtype, c_f32, layout_a, layout_b, batch, st);
}
