// Argument block of the generic implicit-GEMM kernel (gemm.hip).
#pragma once
#include "common.h"

enum LoadKind { L_KC_DENSE = 0, L_KC_CONV = 1, L_MC_DENSE = 2, L_MC_CONV = 3,
                L_KC_CONV_G = 4 };   // KC_CONV whose K tiles may straddle taps (C % BK != 0);
                                     // picked by cn_gemm_dispatch, callers pass L_KC_CONV

// Gather geometry.  For a KC_CONV A operand the GEMM row m is an output pixel (n, oy, ox)
// over the (OH, OW) grid and k = (r, s, ci); the source element is
//   src[n, oy*st + off_y + r*step_y, ox*st + off_x + s*step_x, ci]  (zero outside H x W).
// Forward conv:  st = stride, off = -pad, step = +dilation.
// Dgrad (stride 1): src = dY, off = +pad, step = -dilation, weights in [Cin][kh][kw][Cout].
// For an MC_CONV B operand (wgrad) k is the output pixel and n = (r, s, ci).
struct ConvGeom {
  int N, H, W, C;
  int OH, OW;
  int KH, KW;
  int st;
  int off_y, off_x, step_y, step_x;
  FastDiv div_C, div_KW, div_OW, div_OHW;
};

// Grouped launch: blockIdx.z = problem g (nsplit 1) takes its A / B / C from these arrays
// instead of the a_bs / b_bs / c_bs strides (independent products of one shape, e.g. the weight
// gradients of the bottlenecks of a layer).
constexpr int GEMM_MAXG = 24;
struct GemmGroup {
  const void* A[GEMM_MAXG];
  const void* B[GEMM_MAXG];
  void* C[GEMM_MAXG];
  // fp8 operands: per-problem dequantisation scales (null: the launch-wide scale_a / scale_b)
  const float* SA[GEMM_MAXG];
  const float* SB[GEMM_MAXG];
  // grouped convs that differ in more than their operands (round 6, the ASPP's atrous branches):
  // per-problem bias, BN-statistics workspace (EPI 1) and dilation of the A gather (> 0: the
  // gather's offset / step become -dil / +dil, 'same' padding); null / 0: the launch-wide ones
  const float* bias[GEMM_MAXG];
  float* ST[GEMM_MAXG];
  int dil[GEMM_MAXG];
};

struct GemmArgs {
  int M, N, K;
  int ka_lim, kb_lim;          // k validity bound of each operand (zero beyond)
  const void* A; long long lda, a_bs;
  const void* B; long long ldb, b_bs;
  void* C; long long ldc, c_bs;
  const float* bias;           // [N] fp32 or null
  ConvGeom ga, gb;
  int k_chunk, nsplit;         // split-K: blockIdx.z = batch * nsplit + split
  int row_map;                 // 1: stride-2 dgrad scatter of output rows
  FastDiv rm_div_OW, rm_div_OHW;
  int rm_H, rm_W;
  int c_mode;                  // 0 store, 1 fp32 atomic add, 2 read-add-store,
                               // 3 split-K slab store (C + split * slab)
  long long slab;              // elements between split-K slabs (c_mode 3)
  float alpha;
  const float* scale_a;        // fp8 operands: device per-tensor dequantisation scales (C *= sa * sb)
  const float* scale_b;
  int cfg;                     // tile configuration (gemm.hip kCfg), -1 = shape heuristic
  // BatchNorm epilogues (batch == 1, nsplit == 1, row_map == 0, c_mode 0 only):
  //  st_mode 1: per-(M-tile, column) statistics of the STORED C for train-mode BN: planes
  //             [K, sum(c-K), sum((c-K)^2)] for the tile's first segment (rows < the next
  //             multiple of st_seg_rows) and [sum, sumsq] for the second, K = the tile's first
  //             row (a per-tile shift); plane stride st_plane floats, row = M-tile, col = n.
  //  st_mode 2: BN backward reduce of the stored C (= dy of a BN + ReLU whose pre-BN input is
  //             br_x): dz = dy * (br_x * k1 + sf > 0), xh = (br_x - mu) * is;
  //             planes [sum dz, sum dz * xh].  k1 = gamma * is, sf = beta - mu * k1.
  int st_mode;
  float* st_ws;
  long long st_plane;
  int st_seg_rows;
  const void* br_x; long long br_ldx;
  const float* br_mean; const float* br_invstd; const float* br_gamma; const float* br_beta;
  int ngroup;                  // > 0: grouped launch (GemmGroup), batch = ngroup, nsplit 1
  GemmGroup grp;
  int wt;                      // C stores write-through (sc1): set by cn_gemm_dispatch
};

int cn_gemm_dispatch(const GemmArgs& a, int dtype, int c_f32, int la, int lb, int batch, hipStream_t st);
// Tile configuration the dispatcher picks for a bf16 problem, and its block count.
int cn_gemm_pick(int M, int N, int K, int batch_splits);
long long cn_gemm_cfg_blocks(int cfg, int M, int N);
// Tile rows (BM) of the configuration cn_gemm_dispatch uses for a problem (BN epilogues size
// their per-M-tile partials with it).
int cn_gemm_bm(int dtype, int M, int N, int K, int cfg_or_minus1);
int cn_splitk_reduce_impl(const float* ws, int nsplit, long long slab, long long n, float* out,
                          int accumulate, hipStream_t st);
