/* libcosnet_hip — C ABI of the MI355X (gfx950) hot path of RGBDSegmentation_RAA.
 *
 * The reference has no native code and no FFI: every entry point below
 * replaces an implicit aten call made by the reference's Python, cited per function.
 * Conventions
 *   - activations are NHWC "pixel-major" matrices [P][C] with a row stride ld (elements);
 *     a channel slice of a concat buffer is (base + offset, ld)
 *   - dtype: 0 = fp32 (parity path), 1 = bf16 (throughput path), 2 = fp8 e4m3 (OCP, matrix
 *     operands only: cn_fp8_quant / cn_conv_fwd_fp8); accumulation is fp32
 *   - conv weights are [Cout][KH][KW][Cin] (= torch channels_last of [Cout,Cin,KH,KW]);
 *     dgrad takes the transposed copy [Cin][KH][KW][Cout] (cn_weight_prep makes both)
 *   - all buffers are caller-owned device memory (the library never allocates); the
 *     *_workspace_* queries size the scratch a call needs
 *   - every call is asynchronous on `stream`, re-entrant, never synchronises the host
 *   - return 0 on success, a hipError_t (> 0) from the launch, or a negative CN_ERR_*;
 *     no C++ exception crosses this boundary
 */
#ifndef COSNET_HIP_H
#define COSNET_HIP_H
#include <stddef.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CN_ERR_SHAPE (-1)
#define CN_ERR_ALIGN (-2)
#define CN_ERR_UNSUPPORTED (-3)
#define CN_ERR_HIP (-4)

/* ---- convolution / matrix products (implicit GEMM on MFMA) ---------------------------- */

/* y = conv2d(x, w) + bias.  Replaces nn.Conv2d.forward for every conv of the path:
 * deeplab/residual_net.py:59,63-64,67,106,129 ; deeplab/deeplabv3_encoder.py:15,19,22-31 ;
 * rgbd_segmentation_RAA.py:30-31,41,43.  Cin % (4 fp32 | 8 bf16) == 0. */
int cn_conv_fwd(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                const float* bias, void* y, long long ldy, int OH, int OW, hipStream_t stream);

/* cn_conv_fwd with a workspace (bf16): a deep conv whose 128x256 grid is one round (the ASPP
 * bottleneck conv, deeplab/deeplabv3_encoder.py:31-32: K = 9 x 2560) runs on 256x256 tiles
 * split over K into `ws` fp32 slabs, summed in a fixed order with the bias by a reduce that
 * writes y.  cn_conv_fwd_workspace_floats(dtype, M = N*OH*OW, Cout, K = KH*KW*Cin) is 0 for every
 * shape that does not split; those (and a missing / small workspace) run as cn_conv_fwd. */
size_t cn_conv_fwd_workspace_floats(int dtype, int M, int Cout, int K);
int cn_conv_fwd_ws(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                   const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                   const float* bias, void* y, long long ldy, int OH, int OW, float* ws,
                   size_t ws_floats, hipStream_t stream);

/* dx = conv2d input-gradient (autograd of the calls above).  stride 1: any kernel;
 * stride 2: 1x1 / pad 0 only (deeplab/residual_net.py:59,129 of layer2 block 0). */
int cn_conv_dgrad(int dtype, const void* dy, long long lddy, int N, int OH, int OW, int Cout,
                  const void* wt, int Cin, int KH, int KW, int stride, int pad, int dil,
                  void* dx, long long lddx, int H, int W, int accumulate, hipStream_t stream);

/* dw[Cout][KH][KW][Cin] = conv2d weight-gradient (fp32).  K (= output pixels) is split over
 * workgroups; partial products go to `ws` slabs (cn_conv_wgrad_workspace_floats; may be 0)
 * and are summed in a fixed order (bitwise reproducible, no atomics). */
size_t cn_conv_wgrad_workspace_floats(int dtype, int N, int OH, int OW, int Cout, int KH, int KW,
                                      int Cin);
int cn_conv_wgrad(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                  const void* dy, long long lddy, int OH, int OW, int Cout, int KH, int KW,
                  int stride, int pad, int dil, float* dw, float* ws, hipStream_t stream);
/* G (<= 24) weight gradients of one conv shape in one launch (the same conv of the bottlenecks
 * of a layer, deeplab/residual_net.py:79-94 backward): xs / dys / dws are HOST arrays of the
 * problems' device pointers; every workgroup runs the whole K, so no workspace and no reduce
 * (fixed summation order per problem, bitwise reproducible). */
int cn_conv_wgrad_grouped(int dtype, int G, const void* const* xs, long long ldx, int N, int H, int W,
                          int Cin, const void* const* dys, long long lddy, int OH, int OW, int Cout,
                          int KH, int KW, int stride, int pad, int dil, float* const* dws,
                          hipStream_t stream);
/* The same G problems split over K as well (small layer-1/2 shapes that fill the chip neither
 * one by one nor grouped whole): one launch of G x nsplit K chunks into fp32 slabs ws[g][s][..],
 * then one reduce launch summing each problem's slabs in split order into dws[g] (16-byte
 * aligned).  ws: >= cn_conv_wgrad_grouped_workspace_floats(..) floats; 0 there, or a null /
 * short ws, runs cn_conv_wgrad_grouped. */
size_t cn_conv_wgrad_grouped_workspace_floats(int dtype, int G, int N, int OH, int OW, int Cout, int KH,
                                              int KW, int Cin);
int cn_conv_wgrad_grouped_ws(int dtype, int G, const void* const* xs, long long ldx, int N, int H,
                             int W, int Cin, const void* const* dys, long long lddy, int OH, int OW,
                             int Cout, int KH, int KW, int stride, int pad, int dil,
                             float* const* dws, float* ws, size_t ws_floats, hipStream_t stream);
/* out[i] (+)= sum_s ws[s*slab + i], s < nsplit  (split-K reduction, fp32) */
int cn_splitk_reduce(const float* ws, int nsplit, long long slab, long long n, float* out,
                     int accumulate, hipStream_t stream);

/* ---- fp8 (e4m3, OCP) operands: BASELINE configs[4] -------------------------------------- */
/* Per-tensor scaling state (4 floats, caller-owned, init {1, 1, 0, 0}): [0] dequantisation scale,
 * [1] its inverse, [2] running amax.  mode 0 (delayed scaling): y8 = fp8(x * state[1]) and amax
 * collected; mode 1 (current scaling): amax pass, update, quantise; mode 2: amax only.
 * x: [P][C] (ldx) fp32 or bf16, C % 8 == 0; y8: [P][C] bytes (ldy). */
int cn_fp8_quant(int dtype, const void* x, long long ldx, int P, int C, void* y8, long long ldy,
                 float* state, int mode, hipStream_t stream);
/* The same with the output format chosen: fmt 0 = e4m3 (max 448), 1 = e5m2 (max 57344; the
 * output gradients of the fp8 dgrad).  An e5m2 state carries state[3] = 57344 (the update's
 * format max; 0 means e4m3). */
int cn_fp8_quant_fmt(int dtype, int fmt, const void* x, long long ldx, int P, int C, void* y8,
                     long long ldy, float* state, int mode, hipStream_t stream);
/* Current scaling of n matrices in three launches (amax, update, quantise): device table of n
 * records {const void* x; long long ldx; int P, C; uint8* y; long long ldy; float* state;
 * long long x_is_bf16} (56 bytes each) -- the fp8 copies of the conv weights (fp32 masters) and
 * of the transposed dgrad weights (bf16 copies) after each SGD step. */
int cn_fp8_quant_multi(const void* recs, int n, hipStream_t stream);
/* scale = amax * margin / fmt max (state[3], default 448) for each of nstates consecutive
 * states; amax reset */
int cn_fp8_update(float* states, int nstates, float margin, hipStream_t stream);
/* dx (bf16) (+)= conv_dgrad(dy8, wt8) * dy_state[0] * w_state[0], stride 1 (replaces the
 * backward of nn.Conv2d w.r.t. its input, deeplab/residual_net.py:59-67 autograd, in fp8 mode):
 * dy8 e5m2 [N*OH*OW][Cout] (cn_fp8_quant_fmt fmt 1), wt8 e4m3 [Cin][KH][KW][Cout]; block-scaled
 * MFMA with A format e5m2, B e4m3.  Cout % 16 == 0; accumulate: dx += (else dx =). */
int cn_conv_dgrad_fp8(const void* dy8, long long lddy, int N, int OH, int OW, int Cout,
                      const void* wt8, int Cin, int KH, int KW, int pad, int dil, void* dx,
                      long long lddx, int H, int W, int accumulate, const float* dy_state,
                      const float* w_state, hipStream_t stream);

/* fp8 weight gradients (BASELINE configs[4]): for each of G convs of one shape (G <= 24),
 * dws[g] (fp32 [Cout][KH][KW][Cin], written) = sum over the N*OH*OW output pixels of
 * dys8[g] (e5m2 [P][Cout], row stride lddy; the fp8 dgrad's operand) x im2col(xs8[g]) (e4m3
 * [N*H*W][Cin], row stride ldx; the fp8 forward conv's operand), times the dequantisation scales
 * dy_states[g][0] * x_states[g][0].  Replaces the weight gradient of conv2d's backward
 * (deeplab/residual_net.py:59-67 conv2 of Bottleneck, deeplab/deeplabv3_encoder.py:22-31 the ASPP
 * convs).  ws: cn_conv_wgrad_fp8_workspace_floats floats (split-K slabs; 0 = none needed). */
size_t cn_conv_wgrad_fp8_workspace_floats(int G, int N, int OH, int OW, int Cout, int KH, int KW, int Cin);
int cn_conv_wgrad_fp8(int G, const void* const* xs8, long long ldx, int N, int H, int W, int Cin,
                      const void* const* dys8, long long lddy, int OH, int OW, int Cout, int KH,
                      int KW, int stride, int pad, int dil, float* const* dws,
                      const float* const* x_states, const float* const* dy_states, float* ws,
                      size_t ws_floats, hipStream_t stream);
/* y (bf16) = conv2d(x8, w8) * x_state[0] * w_state[0] + bias: the fp8 implicit-GEMM conv
 * (block-scaled v_mfma_scale_f32_16x16x128_f8f6f4, unit block scales).  Cin % 16 == 0. */
int cn_conv_fwd_fp8(const void* x8, long long ldx, int N, int H, int W, int Cin, const void* w8,
                    int Cout, int KH, int KW, int stride, int pad, int dil, const float* bias,
                    void* y, long long ldy, int OH, int OW, const float* x_state,
                    const float* w_state, hipStream_t stream);

/* Conv + train-mode BatchNorm statistics in ONE pass: y = conv2d(x, w) + bias as cn_conv_fwd,
 * and the GEMM epilogue reduces per-tile column partials of the stored y, so no separate pass
 * reads y for the statistics (replaces nn.Conv2d + nn.BatchNorm2d's batch-stat reduction of
 * deeplab/residual_net.py:59-68,:106-107,:129-131 and deeplab/deeplabv3_encoder.py:15-32).
 * The M = N*OH*OW rows are nseg stacked segments (frames), each its own BN batch: mean / invstd
 * [nseg][Cout]; running stats updated segment after segment (momentum, eps as nn.BatchNorm2d).
 * ws: cn_conv_fwd_bn_workspace_floats(dtype, M, Cout, KH*KW*Cin) floats. */
size_t cn_conv_fwd_bn_workspace_floats(int dtype, int M, int Cout, int K);
/* G stride-1 'same' convs (pad = dil[g]) of ONE input x and one shape, differing in weights,
 * bias and dilation -- the ASPP's atrous branches (deeplab/deeplabv3_encoder.py:22-31, :70-76)
 * -- as one grouped launch with cn_conv_fwd_bn's statistics epilogue per branch.  w, dil, bias,
 * y, ws, mean, invstd, run_mean, run_var: host arrays of G (<= 24) entries; y[g] [N*H*W][ldy];
 * ws[g]: cn_conv_fwd_bn_workspace_floats(dtype, M, Cout, KH*KW*Cin) floats. */
int cn_conv_fwd_bn_grouped(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                           int G, const void* const* w, int Cout, int KH, int KW, const int* dil,
                           const float* const* bias, void* const* y, long long ldy, int nseg,
                           float* const* ws, float* const* mean, float* const* invstd,
                           float* const* run_mean, float* const* run_var, float momentum, float eps,
                           hipStream_t stream);
/* cn_conv_fwd_fp8 with the same BN-statistics epilogue (configs[4]: the fp8 forward convs whose
 * statistics the bf16 path also takes from the epilogue); ws: cn_conv_fwd_bn_workspace_floats(
 * 2 (fp8), M, Cout, K) floats.  Replaces nn.Conv2d + nn.BatchNorm2d's batch statistics as above. */
int cn_conv_fwd_fp8_bn(const void* x8, long long ldx, int N, int H, int W, int Cin, const void* w8,
                       int Cout, int KH, int KW, int stride, int pad, int dil, const float* bias,
                       void* y, long long ldy, int OH, int OW, const float* x_state,
                       const float* w_state, int nseg, float* ws, float* mean, float* invstd,
                       float* run_mean, float* run_var, float momentum, float eps, hipStream_t stream);
int cn_conv_fwd_bn(int dtype, const void* x, long long ldx, int N, int H, int W, int Cin,
                   const void* w, int Cout, int KH, int KW, int stride, int pad, int dil,
                   const float* bias, void* y, long long ldy, int OH, int OW, int nseg, float* ws,
                   float* mean, float* invstd, float* run_mean, float* run_var, float momentum,
                   float eps, hipStream_t stream);
/* Conv input-gradient (stride 1) fused with the reduction of the backward of the BN + ReLU that
 * produced the conv's input (autograd of deeplab/residual_net.py:60-66): dx = dgrad as
 * cn_conv_dgrad; with x = that BN's input, dz = dx * relu'(bn(x)), sum_dz[c] = sum dz and
 * sum_dzxh[c] = sum dz * xhat (= the BN's dbeta, dgamma).  Finish with cn_bn_bwd_apply.
 * ws: cn_conv_dgrad_bn_workspace_floats(dtype, N*H*W, Cin, KH*KW*Cout) floats. */
size_t cn_conv_dgrad_bn_workspace_floats(int dtype, int M, int Cin, int K);
int cn_conv_dgrad_bn(int dtype, const void* dy, long long lddy, int N, int OH, int OW, int Cout,
                     const void* wt, int Cin, int KH, int KW, int pad, int dil, void* dx,
                     long long lddx, int H, int W, const void* x, long long ldx, const float* mean,
                     const float* invstd, const float* gamma, const float* beta, float* sum_dz,
                     float* sum_dzxh, float* ws, hipStream_t stream);

/* Generic batched C = alpha * A . B^T (+bias) with per-operand layouts
 * (0 = k-contiguous rows, 2 = m/n-contiguous, k-major).  Replaces the linear + bmm calls of
 * the co-attention: rgbd_segmentation_RAA.py:159-160,169-170 (RGB) and :212-213,220-221
 * (depth), and their autograd.  c_mode: 0 store, 1 fp32 atomic add, 2 accumulate,
 * 3 split-K slabs at C + split*slab (reduce with cn_splitk_reduce). */
int cn_gemm(int dtype, int layout_a, int layout_b, int M, int N, int K, int ka_lim, int kb_lim,
            const void* A, long long lda, long long a_bs, const void* B, long long ldb,
            long long b_bs, void* C, long long ldc, long long c_bs, int c_f32, int c_mode,
            float alpha, const float* bias, int batch, int nsplit, long long slab,
            hipStream_t stream);

/* ---- BatchNorm2d (train: batch stats + running update; eval: running stats) ---------- */
/* x holds nseg segments of P rows each (frames a and b of a siamese pair, each its own BN
 * batch as in the reference's two encoder calls, rgbd_segmentation_RAA.py:143-148, 198-203);
 * mean/invstd are [nseg][C]; running stats are updated segment after segment. */
size_t cn_bn_workspace_floats(int dtype, int P, int C, int nseg);
int cn_bn_stats(int dtype, const void* x, long long ldx, int P, int nseg, int C, float* mean,
                float* invstd, float* run_mean, float* run_var, float momentum, float eps,
                float* ws, hipStream_t stream);
int cn_bn_eval_params(const float* run_mean, const float* run_var, int C, float eps, float* mean,
                      float* invstd, hipStream_t stream);
/* y = act(gamma*(x-mean)*invstd + beta [+ res] [+ bn_r(xr)]); act 0 none, 1 ReLU, 2 PReLU.
 * Per-channel arrays must be 16-byte aligned. */
int cn_bn_apply(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                const float* mean, const float* invstd, const float* gamma, const float* beta,
                const void* res, long long ldr, const void* xr, long long ldxr,
                const float* rmean, const float* rinvstd, const float* rgamma, const float* rbeta,
                int act, const float* prelu, void* y, long long ldy, hipStream_t stream);
/* cn_bn_apply that also writes y8 = fp8(y * qstate[1]) (bf16 only) and collects amax|y| into
 * qstate[2] (cn_fp8_quant's delayed scaling): the producer of an fp8 conv's input quantises it
 * in the same pass. */
int cn_bn_apply_fp8(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                    const float* mean, const float* invstd, const float* gamma, const float* beta,
                    const void* res, long long ldr, const void* xr, long long ldxr,
                    const float* rmean, const float* rinvstd, const float* rgamma,
                    const float* rbeta, int act, const float* prelu, void* y, long long ldy,
                    void* y8, long long ldy8, float* qstate, hipStream_t stream);
/* cn_bn_apply_fp8 that also writes the ReLU mask of the stored y as bits (mask: bytes
 * [nseg*P][ldm >= C / (8 bf16 | 4 fp32)], bit v of byte c/vec = y[., c] > 0), which cn_bn_bwd takes
 * with act 4 instead of re-reading y (the residual BN + ReLU of each bottleneck,
 * deeplab/residual_net.py:107-109 backward). */
int cn_bn_apply_ex(int dtype, const void* x, long long ldx, int P, int nseg, int C,
                   const float* mean, const float* invstd, const float* gamma, const float* beta,
                   const void* res, long long ldr, const void* xr, long long ldxr,
                   const float* rmean, const float* rinvstd, const float* rgamma,
                   const float* rbeta, int act, const float* prelu, void* y, long long ldy,
                   void* y8, long long ldy8, float* qstate, unsigned char* mask, long long ldm,
                   hipStream_t stream);
/* launch-shape knobs (blocks / rows per thread of each BN pass), for tuning only */
int cn_bn_set_tuning(int key, int value);
/* backward of cn_bn_apply w.r.t. x (train mode), masks fused; dres <- dz for the residual.
 * act 1: ReLU mask from y; 3: from x with the forward affine (no residual); 4: y is the bit
 * mask of cn_bn_apply_ex (ldy = its row stride in bytes); 2: PReLU. */
int cn_bn_bwd(int dtype, const void* x, long long ldx, const void* dy, long long lddy,
              const void* y, long long ldy, int P, int C, const float* mean, const float* invstd,
              const float* gamma, const float* beta, int act, const float* prelu, float* dgamma,
              float* dbeta, float* dprelu_c, void* dx, long long lddx, void* dres,
              long long lddres, float* ws, hipStream_t stream);

/* dx of a train-mode BN + ReLU from precomputed sums (cn_conv_dgrad_bn):
 * dx = gamma*invstd*(dz - sum_dz/P - xhat*sum_dzxh/P), dz = dy * relu'(bn(x)). */
int cn_bn_bwd_apply(int dtype, const void* x, long long ldx, const void* dy, long long lddy, int P,
                    int C, const float* mean, const float* invstd, const float* gamma,
                    const float* beta, const float* sum_dz, const float* sum_dzxh, void* dx,
                    long long lddx, hipStream_t stream);

/* ---- co-attention softmax (rgbd_segmentation_RAA.py:164-165, :215-216) ----------------- */
size_t cn_coatt_workspace_floats(int B, int HW, int ld);
int cn_coatt_softmax(int dtype, const float* S, int B, int HW, int ld, void* Pc, void* PT,
                     float* ws, hipStream_t stream);
int cn_coatt_dscore(int dtype, const void* Pc, const float* dPc, const float* d1, const void* PT,
                    const float* dPr, const float* d2, int B, int HW, int ld, void* dS,
                    hipStream_t stream);
/* Fused inference forward of both co-attention directions, S never written to HBM:
 *   za[i] = sum_j softmax_j(S[i][:]) vb[j],  zb[j] = sum_i softmax_i(S[:][j]) va[i],  S = vat vb^T
 * Replaces rgbd_segmentation_RAA.py:160-170 (RGB) and :213-221 (depth) when no gradient is
 * needed.  bf16 only, C == 256, [B*HW][ld] pixel-major, ld_vat/ld_va/ld_vb % 8 == 0 and 16-byte
 * aligned bases; za or zb may be NULL (that direction is skipped). */
int cn_coatt_fused_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                       const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                       long long ld_z, hipStream_t stream);
/* Same product with the keys split over several workgroups per query block when one
 * workgroup per (row block, pair, direction) would leave most of the last round of CUs idle
 * (configs[3]: 5 pairs -> 290 workgroups on 256 CUs): each split writes its un-normalised
 * partial O (bf16 in the default 48-row kernel, fp32 in the 4-wave one) and fp32 row (max, sum)
 * into ws, and the partials are folded in split order (in the launch, or by a merge kernel).
 * ws_bytes >= cn_coatt_fused_workspace_bytes(B, HW, ndir) (0: no split, ws may be NULL);
 * za/zb 16-byte aligned, ld_z % 8 == 0.  A NULL / too small / misaligned ws is not an error:
 * the launch then runs unsplit (same result, slower tail). */
size_t cn_coatt_fused_workspace_bytes(int B, int HW, int ndir);
/* fp8 co-attention forward (BASELINE configs[4], rgbd_segmentation_RAA.py:160-170 / :213-221):
 * both directions of cn_coatt_flash_fwd with the affinity S = Va_t Vb^T and the gathers P V on
 * the block-scaled MFMA v_mfma_scale_f32_32x32x64_f8f6f4 -- operands in MX format (e4m3 + one
 * E8M0 exponent per 32 reduction values, written by a prepass into ws), P in e4m3 (unit
 * scale, <= 2^8 under the lazy rescale), softmax max / sum in fp32.  lse_a / lse_b optional
 * ([B][ceil32(HW)], as cn_coatt_flash_fwd).  ws: cn_coatt_f8_workspace_bytes(B, HW) bytes,
 * 256-byte aligned.  C == 256. */
size_t cn_coatt_f8_workspace_bytes(int B, int HW);
int cn_coatt_f8_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                    const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                    long long ld_z, float* lse_a, float* lse_b, void* ws, size_t ws_bytes,
                    hipStream_t stream);
/* fp8 co-attention forward for TRAINING (configs[4] "fp8 MFMA affinity", the forward whose
 * gradient cn_coatt_flash_dvat / cn_coatt_flash_pv then compute): cn_coatt_f8_fwd with lse_a /
 * lse_b required, Vb quantised with one E8M0 exponent per 32 keys x 32 channels (so its row
 * image -- the S operand -- and its V^T image -- the P V operand of Z_a -- decode to the same
 * values), and the DECODED MX operands written as bf16 (exact): vat_q (Va_t rows), va_q (Va as the
 * V of Z_b), vb_q (Vb, every role); [B*HW][ld_q], 16-byte aligned.  The flash backward run on
 * (vat_q, va_q, vb_q) and this forward's lse is the gradient of this forward (straight-through
 * for the operand and P quantisations).  ws: cn_coatt_f8_train_workspace_bytes(B, HW) bytes,
 * 256-byte aligned.  Reference: rgbd_segmentation_RAA.py:160-170, :213-221. */
size_t cn_coatt_f8_train_workspace_bytes(int B, int HW);
int cn_coatt_f8_train_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                          const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                          long long ld_z, float* lse_a, float* lse_b, void* vat_q, void* va_q,
                          void* vb_q, long long ld_q, void* ws, size_t ws_bytes, hipStream_t stream);
int cn_coatt_fused_fwd_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                          const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                          long long ld_z, void* ws, size_t ws_bytes, hipStream_t stream);

/* Flash-style co-attention for TRAINING (rgbd_segmentation_RAA.py:160-170 and its autograd),
 * S never in HBM.  Forward = cn_coatt_fused_fwd plus the per-row log2-sum-exp2 of each direction
 * (lse_a[b][i] over j of S[i][j] log2(e), lse_b[b][j] over i), [B][HWp] with HWp = HW rounded up
 * to 32 and +inf in the padding; either may be NULL. */
int cn_coatt_flash_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                       const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                       long long ld_z, float* lse_a, float* lse_b, hipStream_t stream);
/* cn_coatt_flash_fwd with a workspace of cn_coatt_fused_workspace_bytes(B, HW, 2) bytes: with the
 * 48-row kernel (variant 5) the map's key tiles are then cut across the CUs (stream-K, merged in
 * the launch); the 4-wave kernel ignores it.  Same results contract as cn_coatt_flash_fwd. */
int cn_coatt_flash_fwd_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                          const void* vb, long long ld_vb, int B, int HW, int C, void* za, void* zb,
                          long long ld_z, float* lse_a, float* lse_b, void* ws, size_t ws_bytes,
                          hipStream_t st);
/* o[q] (+)= sum_k exp2(q.k log2(e) - klse[k]) v[k]: a softmax product whose normaliser is per
 * KEY (the other direction's lse) -- the co-attention backward's dV_a = S_row dZ_b
 * (autograd of rgbd_segmentation_RAA.py:169) with q = Va_t, k = Vb, v = dZ_b, klse = lse_b.
 * bf16, C == 256; accumulate: o += result (bf16 read-add-write). */
int cn_coatt_flash_pv(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                      long long ldv, const float* klse, int B, int HW, int C, void* o, long long ldo,
                      int accumulate, hipStream_t stream);
/* Same, with a workspace (>= cn_coatt_fused_workspace_bytes(B, HW, 1)) that lets the keys of
 * an under-filled last round of workgroups be split over several workgroups (partials summed
 * in split order in fp32; bf16 partial rows in the 48-row kernel); without one (NULL / too
 * small) it runs unsplit. */
int cn_coatt_flash_pv_ws(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                         long long ldv, const float* klse, int B, int HW, int C, void* o,
                         long long ldo, int accumulate, void* ws, size_t ws_bytes, hipStream_t stream);

/* Backward of the flash co-attention: dva_t (+)= sum_j dS[i][j] vb[j] with
 *   dS = P0 (dza[i].vb[j] - d0[i]) + P1 (va[i].dzb[j] - d1[j]),
 *   P0 = exp2(S log2e - lse_a[i]), P1 = exp2(S log2e - lse_b[j]), S = vat vb^T,
 * d0 = rowdot(dza, za) [B][HW], d1 = rowdot(dzb, zb) at [B][HWp].  dza == NULL drops the P0 term,
 * dzb == NULL the P1 term (a direction that receives no gradient).  bf16, C == 256.
 * Replaces the autograd of rgbd_segmentation_RAA.py:160-170 (with cn_coatt_flash_pv for dV_a). */
int cn_coatt_flash_dvat(const void* vat, long long ld_vat, const void* va, long long ld_va,
                        const void* dza, long long ld_dza, const void* vb, long long ld_vb,
                        const void* dzb, long long ld_dzb, const float* lse_a, const float* d0,
                        const float* lse_b, const float* d1, int B, int HW, int C, void* out,
                        long long ld_out, int accumulate, hipStream_t stream);
/* Same, with a workspace (>= cn_coatt_flash_bwd_workspace_bytes(B, HW)): when the B x
 * ceil(HW/128) row blocks leave CUs idle, the keys are split over up to 8 workgroups per row
 * block whose fp32 partial sums are added in split order (out 16-byte aligned, ld_out % 8 == 0;
 * otherwise, or without a workspace, unsplit). */
size_t cn_coatt_flash_bwd_workspace_bytes(int B, int HW);
int cn_coatt_flash_dvat_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                           const void* dza, long long ld_dza, const void* vb, long long ld_vb,
                           const void* dzb, long long ld_dzb, const float* lse_a, const float* d0,
                           const float* lse_b, const float* d1, int B, int HW, int C, void* out,
                           long long ld_out, int accumulate, void* ws, size_t ws_bytes,
                           hipStream_t stream);

/* ---- memory-bound helpers -------------------------------------------------------------- */
int cn_nchw_to_nhwc(int dtype, const float* x, int N, int C, int H, int W, int Cp, void* y,
                    hipStream_t stream);
int cn_weight_prep(int dtype, const float* w, int Cout, int KHW, int Cin, int Cp, void* wf,
                   void* wt, hipStream_t stream);
/* nn.MaxPool2d(3, 2, 1, ceil_mode=True): deeplab/residual_net.py:109,160 */
int cn_maxpool_fwd(int dtype, const void* x, int N, int H, int W, int C, int OH, int OW, int k,
                   int s, int pad, void* y, unsigned char* argmax, hipStream_t stream);
int cn_maxpool_bwd(int dtype, const void* dy, const unsigned char* argmax, int N, int H, int W,
                   int C, int OH, int OW, int k, int s, int pad, void* dx, hipStream_t stream);
/* AdaptiveAvgPool2d(1) + 1x1 upsample broadcast: deeplab/deeplabv3_encoder.py:57-61 */
int cn_avgpool(int dtype, const void* x, long long ld, int N, int HW, int C, float scale, void* y,
               float* ws /* cn_avgpool_workspace_floats() */, hipStream_t stream);
size_t cn_avgpool_workspace_floats(int dtype, int N, int HW, int C);
int cn_bcast_rows(int dtype, const void* src, int N, int HW, int C, float scale, void* dst,
                  long long ld, int accumulate, hipStream_t stream);
/* gate: rgbd_segmentation_RAA.py:177-184 (RGB, no bias), :228-235 (depth, bias) */
int cn_gate_fwd(int dtype, const void* z, long long ldz, int P, int C, const float* g,
                const float* gb, void* out, long long ldo, float* mask, hipStream_t stream);
int cn_gate_bwd(int dtype, const void* z, long long ldz, const void* dout, long long lddo,
                const float* mask, int P, int C, const float* g, int through_mask, void* dz,
                long long lddz, float* dg, float* dgb,
                float* ws /* cn_colpart_workspace_floats(P, C) */, hipStream_t stream);
/* Mean of N stacked fp32 maps [N][C] -> [C] (N-reference average, test.py:287-305): the fixed-
 * order sum divided by N, like the reference's `output_sum / sample_range` (test.py:305). */
int cn_mean_rows(const float* x, int nrows, int C, float* out, hipStream_t stream);
/* Fixed-order column sums of [nrows][C] fp32 (e.g. the per-channel PReLU gradient partials of
 * deeplab/deeplabv3_encoder.py:82 -> the single PReLU weight's gradient). */
int cn_sum_rows(const float* x, int nrows, int C, float* out, hipStream_t stream);
/* x[i] *= s in place (the 1/world pre-scaling of a gradient bucket before its sum all-reduce) */
int cn_scale(float* x, long long n, float s, hipStream_t stream);
/* out[i] = x[i] * s[0], s a device scalar: chain rule of a loss gradient (autograd of
 * train.py:595-599) without a host read. */
int cn_scale_dev(const float* x, long long n, const float* s, float* out, hipStream_t stream);
/* uint8 quantisation + soft-J per frame (test.py:317, evaluation.py:3-22): x [n][hw] fp32 in
 * [0,1], gt [n][hw] uint8 {0,1} -> mask [n][hw] uint8 = trunc(255 x), iou[n] (double, bit-exact
 * with numpy), counts[n][4] (optional) = {sum(p&g), sum(p|g), nonzero(p), nonzero(g)}. */
int cn_soft_iou(const float* x, const unsigned char* gt, int nframes, long long hw,
                unsigned char* mask, double* iou, long long* counts, hipStream_t stream);
/* Workspace of the deterministic column reductions (gate/head backward, colsum). */
size_t cn_colpart_workspace_floats(int P, int C);
/* fusion + 1x1 classifier: rgbd_segmentation_RAA.py:251-261 ; deeplabv3_encoder.py:138 */
int cn_head_fwd(int dtype, const void* a, long long lda, const void* b, long long ldb, int P,
                int C, int relu, const float* w, const float* bias, void* zout, long long ldz,
                float* logit, hipStream_t stream);
int cn_head_bwd(int dtype, const void* z, long long ldz, const float* dlogit, int P, int C,
                int relu, const float* w, void* dz, long long lddz, float* dw, float* db,
                float* ws /* cn_colpart_workspace_floats(P, C) */, hipStream_t stream);
/* F.upsample(bilinear, align_corners=False) + sigmoid: rgbd_segmentation_RAA.py:262-266 */
int cn_upsample_sigmoid(const float* in, int N, int h, int w, int H, int W, int apply_sigmoid,
                        float* out, hipStream_t stream);
int cn_upsample_sigmoid_bwd(const float* dout, const float* out, int N, int h, int w, int H,
                            int W, int apply_sigmoid, float* din, hipStream_t stream);
/* loss: calc_loss_BCE + 0.8 calc_loss_L1, train.py:176-216 */
int cn_count_ge(const float* gt, long long n, float thr, unsigned long long* cnt,
                hipStream_t stream);
size_t cn_loss_workspace_floats(long long n);
int cn_bce_l1(const float* pred, const float* gt, long long n, float weight, float l1w, float* ws,
              float* loss, float* dpred, hipStream_t stream);
/* same, with the BCE weight N*H*W/#pos read from a device-side count (capturable, no sync) */
int cn_bce_l1_devcount(const float* pred, const float* gt, long long n, const long long* pos_count,
                       double total, float l1w, float* ws, float* loss, float* dpred,
                       hipStream_t stream);
/* optim.SGD(momentum, weight_decay) step over a device table of tensors: train.py:538-540,602 */
int cn_sgd(const void* tensors, int nt, const float* lrs, float wd, float momentum,
           hipStream_t stream);
int cn_rowdot(int dtype, const void* a, long long lda, const void* b, long long ldb, int P, int C,
              float* out, hipStream_t stream);
/* rowdot with the rows in segments of `seg` written at a stride of seg_ld (padded per pair) */
int cn_rowdot_seg(int dtype, const void* a, long long lda, const void* b, long long ldb, int P, int C,
                  int seg, int seg_ld, float* out, hipStream_t stream);
int cn_colsum(int dtype, const void* x, long long ld, int P, int C, float* out,
              float* ws /* cn_colpart_workspace_floats(P, C) */, hipStream_t stream);
int cn_cast2d(int dtype_in, int dtype_out, const void* x, long long ldx, int P, int C, void* y,
              long long ldy, int accumulate, hipStream_t stream);
/* ---- SBM-RGBD frame preparation (dataloaders/sbm_rgbd_loader.py:590-697, utils.py:5-55) -- */
/* dst[c][H][W] (fp32) = cv2.resize(src window - mean[c]) with mode 0 INTER_LINEAR / 1
 * INTER_NEAREST, horizontally flipped if flip; src element (c, y, x) of the window at
 * src + c*plane_stride + (y0+y)*row_stride + (x0+x)*col_stride (uint8 if src_u8, else fp32). */
int cn_frame_resize(int src_u8, const void* src, int C, long long plane_stride, long long row_stride,
                    long long col_stride, int y0, int x0, int h, int w, const float* mean,
                    float* dst, int H, int W, int mode, int flip, hipStream_t stream);

/* Build provenance: SHA-256 (16 hex digits) of the HIP sources + this header the library was
 * compiled from (stamped by csrc/Makefile). */
const char* cn_build_source_hash(void);
/* 1 if the library was built with the development variants (make EXPERIMENTAL=1: co-attention
 * kernel variants 2-4, GEMM tile configurations 21-25), else 0. */
int cn_build_experimental(void);

/* Development hook (tuning tools only): force GEMM tile configuration `cfg` for every bf16
 * launch; -1 restores the shape heuristic.  Returns the number of configurations, or -1 for a
 * configuration this build does not carry (21-25 without EXPERIMENTAL=1). */
int cn_gemm_force_config(int cfg);
/* Development hook (tuning tools only): number of blocks the wgrad K split aims for. */
int cn_gemm_set_wgrad_target(int blocks);
/* Development / test hook: co-attention flash forward and PV kernel variant (1: four waves, one
 * per SIMD, 32 query rows each; 2: eight waves in pairs that split the output channels, S computed
 * by both; 3: pairs that split the keys of S and the output channels; 4: four waves in pairs of 64
 * query rows that split the channels of S (partial S exchanged through LDS) and of the output;
 * 5: four waves of 48 query rows with Q in registers and a stream-K split of the key tiles over
 * the CUs -- the default; 0: default).  Returns the previous setting, or -1 for variants 2-4 in a
 * library built without them (cn_build_experimental() == 0).  CN_COATT_VARIANT sets the default. */
int cn_coatt_force_variant(int v);

#ifdef __cplusplus
}
#endif
#endif
