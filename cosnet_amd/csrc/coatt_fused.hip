// Fused co-attention forward: both directions of the co-attention block without ever
// materialising the HW x HW affinity (rgbd_segmentation_RAA.py:160-170 for RGB, :213-221 for
// depth, inference / no-grad path):
//
//   S[i][j] = Va_t[i] . Vb[j]                                   (:160 / :213, bmm)
//   Z_a[i]  = sum_j softmax_j(S[i][:])[j] * Vb[j]               (:165 + :170 -> "S_column")
//   Z_b[j]  = sum_i softmax_i(S[:][j])[i] * Va[i]               (:164 + :169 -> "S_row")
//
// Both are the same "flash" product  O[q] = sum_k softmax_k(Q[q].K[k]) V[k]  (no temperature)
// with (Q, K, V) = (Va_t, Vb, Vb) for Z_a and (Vb, Va_t, Va) for Z_b, so one kernel serves
// both directions (blockIdx.z) and S is recomputed per direction on the MFMA instead of
// written to HBM (51.8 MB fp32 per pair and modality at 473x473).
//
// Layout: pixel-major bf16 [B*HW][ld], channel dim D = 256 (all_channel).  One workgroup =
// 4 waves = 128 query rows (32 per wave) held as a 64 KB LDS block; key tiles of 32 rows stream
// through a 3-stage LDS ring (K and V tile, 16 KB each per stage) filled by LDS-DMA.
//   * "swapped" product S^T = K . Q^T on v_mfma_f32_32x32x16_bf16 with Q as the B operand: the accumulator has the query row on the lane and 16 keys in registers,
//     so the online-softmax row max / sum are lane-local (+ one xor-32 exchange for the max)
//   * the accumulator, packed to bf16, is directly the B operand of O^T += V^T . P^T (its k
//     order is the accumulator's row order); V^T fragments come from the [key][d] LDS image
//     via the gfx950 transpose read ds_read_b64_tr_b16
//   * K image: 16-B chunk XOR (key & 15) -> conflict-free ds_read_b128; V image: chunk XOR
//     ((key & 3) << 2) -> conflict-free transposed reads.  Swizzles are applied on the DMA
//     source address, so the DMA writes stay lane-linear.
//   * O is rescaled only when some row's running max grew (wave-uniform branch, exact).
#include "common.h"
#include <cstdlib>
#include "../../include/cosnet_hip.h"
#include "coatt_fused.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int FSTAGES = 3;           // K/V ring depth (two tiles in flight behind the one read)
constexpr int FDMA = 2 * FTILE / 4096;  // LDS-DMA instructions per thread per K/V tile
#ifndef CF_KPF
#define CF_KPF 3  // K (and Q) fragment reads issued ahead of the S MFMAs
#endif
#ifndef CF_VPF
#define CF_VPF 3  // V^T fragment reads issued ahead of the PV MFMAs (<= 7)
#endif
#ifndef RESCALE_T
#define RESCALE_T 8.0f
#endif
#ifndef CF_DMA_SPREAD
#define CF_DMA_SPREAD 1
#endif

__device__ __attribute__((aligned(16))) unsigned g_zero16_fused[4];

__device__ __forceinline__ void glds16f(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void raw_barrier_f() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// wait until at most N LDS/SMEM operations are outstanding; `v` is threaded through so the
// consumer of v cannot be scheduled above the wait
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

__device__ __forceinline__ bf16x8 pack8(const float* f) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)f[j];
  return r;
}

// MODE 0: softmax over the keys of each query row (online max / sum), O = P V / l.
// MODE 1: P[q][k] = exp2(S[q][k] log2e - klse[k]) with a per-KEY normaliser computed by an
//         earlier MODE 0 pass in the other direction (no max, no sum), O (+)= P V.  This is the
//         co-attention backward's dV_a = P_row dZ_b (rgbd_segmentation_RAA.py:169 autograd).
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void coatt_fused_fwd_k(FusedArgs a) {
  // [Q: 128 rows x 512 B][stage 0: K | V][stage 1: K | V][stage 2: K | V]   (64 + 3 x 32 KB)
  __shared__ __attribute__((aligned(16))) char lds[FQB + FSTAGES * 2 * FTILE];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  // XCD-aware work order: hardware places workgroup i on XCD i % 8, so give each XCD a
  // contiguous run of the (batch, direction)-major work list -- the row blocks of one
  // (batch, direction) then share its K/V stream (3.7 MB) in that XCD's 4 MB L2.
  const int nfull8 = (a.nfull + 7) & ~7;
  int item, split = 0;
  if ((int)blockIdx.x < nfull8) {
    const int per_xcd = nfull8 >> 3;
    item = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    if (item >= a.nfull) return;
  } else {
    const int t = blockIdx.x - nfull8;
    item = a.nfull + t / a.nsplit;
    split = t % a.nsplit;
    if (item >= a.nitems) return;
  }
  const bool part = item >= a.nfull;   // a split of a tail item
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const int HW = a.HW;
  const long long b = bd / a.ndir;
  const bf16* Q = d.q + b * HW * d.ldq;
  const bf16* K = d.k + b * HW * d.ldk;
  const bf16* V = d.v + b * HW * d.ldv;
  const int q0 = rb * FBQ;
  const int qrow = q0 + w * 32 + r;
  const void* zp = (const void*)g_zero16_fused;
  char* qlds = lds;

  // Q block DMA: chunk p of the 4096-chunk image -> row p >> 5, position p & 31, source chunk
  // position ^ (row & 15) (same swizzle as K: conflict-free ds_read_b128 of rows)
#pragma unroll
  for (int i = 0; i < FQB / 4096; ++i) {
    const int p = i * 256 + tid;
    const int row = p >> 5, cpos = p & 31;
    const bool ok = q0 + row < HW;
    const bf16* src = Q + (long long)(q0 + row) * d.ldq + ((cpos ^ (row & 15)) << 3);
    glds16f(ok ? (const void*)src : zp, qlds + (i * 256 + (tid & ~63)) * 16);
  }

  // K/V tile DMA: chunk p = 256 i + tid of the 1024-chunk image -> key row p >> 5, position
  // p & 31; the source chunk is the position XOR the image's swizzle.
  const int ntiles = (HW + FBK - 1) / FBK;
  const int tb = part ? split * a.tps : 0;   // first key tile of this work item
  // piece i (< FTILE / 4096) of tile t's K and V images: one 1-KB LDS-DMA per wave for each
  auto issue_piece = [&](int t, int stage, int i) {
    char* kb = lds + FQB + stage * 2 * FTILE;
    char* vb = kb + FTILE;
    const int key0 = (tb + t) * FBK;
    const int p = i * 256 + tid;
    const int row = p >> 5, cpos = p & 31;
    const int key = key0 + row;
    const bool ok = key < HW;
    const bf16* ks = K + (long long)key * d.ldk + ((cpos ^ (row & 15)) << 3);
    const bf16* vs = V + (long long)key * d.ldv + ((cpos ^ ((row & 3) << 2)) << 3);
    const int wb = (i * 256 + (tid & ~63)) * 16;
    glds16f(ok ? (const void*)ks : zp, kb + wb);
    glds16f(ok ? (const void*)vs : zp, vb + wb);
  };
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int i = 0; i < FTILE / 4096; ++i) issue_piece(t, stage, i);
  };

  const int nt = part ? min(ntiles - tb, a.tps) : ntiles;
  issue(0, 0);
  if (nt > 1) issue(1, 1);

  f32x16 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x16{};
  float m = -INFINITY;  // running row max, log2 domain
  float l = 0.f;        // partial row sum over this lane half's keys
  const float L2E = 1.4426950408889634f;

  // fragment geometry
  const int sw = r & 15;                                   // row swizzle of Q / K images
  const char* qrp = qlds + (w * 32 + r) * FROWB;           // this lane's Q row
  const int G = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;  // transposed V reads

#ifdef CF_QREG
  bf16x8 qreg[16];
#endif
  int st = 0, st2 = 2;  // stages of tiles t and t+2
  for (int t = 0; t < nt; ++t) {
    // tile t landed when at most the FDMA chunks of tile t+1 are still in flight
    if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(FDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_f();
    // the stage of tile t+2 was last read in iteration t-1, which every wave has finished.
    // CF_DMA_SPREAD: its pieces are issued between the PV MFMAs below (a DMA piece costs its wave
    // 60-185 issue cycles; beside the MFMAs that cost hides) instead of as a burst here.
    const bool dodma = t + 2 < nt;
    const int dst2 = st2;
#if !CF_DMA_SPREAD
    if (dodma) issue(t + 2, st2);
#endif
    const char* kb = lds + FQB + st * 2 * FTILE;
    st = st == FSTAGES - 1 ? 0 : st + 1;
    st2 = st2 == FSTAGES - 1 ? 0 : st2 + 1;
    const char* vb = kb + FTILE;

    // MODE 1: this tile's per-key normalisers (lane's keys 32t + 8q + 4h + 0..3), loaded ahead
    // of the S MFMAs so their latency hides under them
    f32x4 nk[4];
    if constexpr (MODE == 1) {
      const float* kl = d.klse + b * a.HWp + (tb + t) * FBK + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) nk[q] = *(const f32x4*)(kl + 8 * q);
    }
    // ---- S^T tile (32 keys x 32 query rows per wave) = K Q^T over 16 k-steps of d;
    // both fragments come from LDS, read KPF steps ahead
    f32x16 s = f32x16{};
#ifdef CF_QREG
    // the wave's 32 query rows stay in registers (64 VGPRs) after the first tile: only the K
    // fragments are read from LDS per tile
    if (t == 0) {
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) qreg[ks] = *(const bf16x8*)(qrp + (((2 * ks + h) ^ sw) << 4));
    }
#endif
    {
      constexpr int KPF = CF_KPF;
      const char* krp = kb + r * FROWB;
      bf16x8 kf[KPF];
#ifndef CF_QREG
      bf16x8 qf[KPF];
#endif
#pragma unroll
      for (int u = 0; u < KPF; ++u) {
        const int c = ((2 * u + h) ^ sw) << 4;
        kf[u] = *(const bf16x8*)(krp + c);
#ifndef CF_QREG
        qf[u] = *(const bf16x8*)(qrp + c);
#endif
      }
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
#ifdef CF_QREG
        const bf16x8 kc = kf[ks % KPF], qc = qreg[ks];
#else
        const bf16x8 kc = kf[ks % KPF], qc = qf[ks % KPF];
#endif
        if (ks + KPF < 16) {
          const int c = ((2 * (ks + KPF) + h) ^ sw) << 4;
          kf[ks % KPF] = *(const bf16x8*)(krp + c);
#ifndef CF_QREG
          qf[ks % KPF] = *(const bf16x8*)(qrp + c);
#endif
        }
#ifndef CF_NO_S
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qc, s, 0, 0, 0);
#else
        s[ks] += (float)kc[0] * (float)qc[1];
#endif
      }
      // keep the reads KPF steps ahead: initial reads, then {1 MFMA, NR ds_read} per step
#ifdef CF_QREG
      constexpr int NR = 1;
#else
      constexpr int NR = 2;
#endif
      __builtin_amdgcn_sched_group_barrier(0x100, NR * KPF, 0);
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (ks + KPF < 16) __builtin_amdgcn_sched_group_barrier(0x100, NR, 0);
      }
    }

    // ---- online softmax over the keys (register i: key 32t + (i&3) + 8(i>>2) + 4h)
    const int key0 = (tb + t) * FBK;
    bf16x8 pf[2];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * s2 + j;
          pv[j] = __builtin_amdgcn_exp2f(fmaf(s[i], L2E, -nk[i >> 2][i & 3]));
        }
        pf[s2] = pack8(pv);
      }
    } else {
    if (key0 + FBK > HW) {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        if (key0 + (i & 3) + 8 * (i >> 2) + 4 * h >= HW) s[i] = -INFINITY;
    }
    float mx = s[0];
#pragma unroll
    for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[i]);
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mnew = fmaxf(m, mx * L2E);
    // lazy rescale: keep the stale max while no row's max grew by more than RESCALE_T (log2
    // units), so P <= 2^RESCALE_T (fp32 O / l have the headroom; P's bf16 rounding is relative)
    if (__builtin_amdgcn_ballot_w64(mnew > m + RESCALE_T) != 0) {
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);  // m = -inf: 0 (o, l are 0)
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
      m = mnew;
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float pv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        pv[j] = __builtin_amdgcn_exp2f(fmaf(s[8 * s2 + j], L2E, -m));
        l += pv[j];
      }
      pf[s2] = pack8(pv);
    }
    }  // MODE 0

    // ---- O^T += V^T P^T: k-step sk covers keys 16 sk .. +15 in the accumulator's k order;
    // 16 (dt, sk) steps, V^T fragments read VPF steps ahead.  The transposed reads are inline
    // asm with explicit lgkmcnt waits: hipcc cannot tell the ds_read_b64_tr_b16 builtin apart
    // from the in-flight LDS-DMA of the NEXT tile (other stage) and would drain vmcnt(0) in
    // front of it, exposing the whole DMA latency every tile.
    {
      const unsigned vrow = lds_addr(vb + (4 * h + q4) * FROWB);
      auto vread = [&](int dt, int sk) {
        const int g = 8 * dt + 4 * (G & 1) + pp;  // 8-byte granule of d = 32 dt + 16 (G&1) + 4 pp
        const unsigned a1 = vrow + 16 * sk * FROWB + ((g ^ (q4 << 3)) << 3);
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a1));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(8 * FROWB));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      constexpr int VPF = CF_VPF;
      bf16x8 vf[VPF];
#pragma unroll
      for (int u = 0; u < VPF; ++u) vf[u] = vread(u >> 1, u & 1);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        bf16x8 cur = vf[it % VPF];
        if (it + VPF < 16) vf[it % VPF] = vread((it + VPF) >> 1, (it + VPF) & 1);
        const int younger = 2 * (15 - it < VPF ? 15 - it : VPF);  // reads issued after cur's
        if (younger >= 14) lgkm_wait<14>(cur);
        else if (younger == 12) lgkm_wait<12>(cur);
        else if (younger == 10) lgkm_wait<10>(cur);
        else if (younger == 8) lgkm_wait<8>(cur);
        else if (younger == 6) lgkm_wait<6>(cur);
        else if (younger == 4) lgkm_wait<4>(cur);
        else if (younger == 2) lgkm_wait<2>(cur);
        else lgkm_wait<0>(cur);
#ifndef CF_NO_PV
        o[it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[it & 1], o[it >> 1], 0, 0, 0);
#else
        o[it >> 1][it] += (float)cur[0] * (float)pf[it & 1][1];
#endif
#if CF_DMA_SPREAD
        if ((it & 1) && (it >> 1) < FTILE / 4096 && dodma) issue_piece(t + 2, dst2, it >> 1);
#endif
      }
    }
  }

  // ---- epilogue: O[qrow][d] = o / l ; register i of d tile dt holds d = 32 dt + (i&3) + 8(i>>2) + 4h
  l += __shfl_xor(l, 32, 64);
  if (part) {
    // key split: un-normalised partial O (and MODE 0: the row's (m, l)) of this split, folded by
    // coatt_merge_k
    if (qrow < HW) {
      const long long prow = ((long long)split * (a.nitems - a.nfull) + (item - a.nfull)) * FBQ + (qrow - q0);
      float* op = a.opart + prow * FD + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 8; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          *(f32x4*)(op + 32 * dt + 8 * c) = f32x4{o[dt][4 * c], o[dt][4 * c + 1], o[dt][4 * c + 2], o[dt][4 * c + 3]};
      if (MODE == 0 && h == 0) *(float2*)(a.mlpart + prow * 2) = float2{m, l};
    }
    return;
  }
  if (MODE == 0 && d.lse && h == 0 && qrow < a.HWp)
    d.lse[b * a.HWp + qrow] = qrow < HW ? m + __builtin_amdgcn_logf(l) : INFINITY;  // logf = log2
  if (qrow < HW) {
    const float inv = MODE == 0 ? 1.f / l : 1.f;
    bf16* op = d.o + (b * HW + qrow) * d.ldo + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v;
        if (a.accumulate) {
          const bf16x4 old = *(const bf16x4*)(op + 32 * dt + 8 * c);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv + (float)old[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv);
        }
        *(bf16x4*)(op + 32 * dt + 8 * c) = v;
      }
  }
}

#if CN_EXPERIMENTAL
// Measured-slower wave-pair variants (round 4): built only with CN_EXPERIMENTAL=1
// (make EXPERIMENTAL=1), selected by cn_coatt_force_variant / CN_COATT_VARIANT in such builds.
// ---------------------------------------------------------------------------------------------
// Two waves per SIMD (coatt_fused2_k): the same flash product, 8 waves = 4 wave PAIRS per
// workgroup, 128 query rows.  Both waves of a pair hold the pair's 32 query rows in registers (Q,
// 64 VGPRs) and compute the same S^T tile and softmax (identical instruction streams: identical
// bits), and each accumulates ONE half of the output channels (O^T for d in [128 hb, +128): 64
// accumulators instead of 128).  So a wave fits in 256 registers and every SIMD runs two of them:
// one wave's MFMAs overlap the other's softmax, LDS waits and LDS-DMA issue, which the 4-wave
// kernel (one wave per SIMD) serialises.  The price is the duplicated S product (1.5x the MFMAs
// of the algorithmic count).  Waves 4-7 run half a tile (one phase) behind waves 0-3 (guide: two
// waves of one program per SIMD, stagger): phase 1 = S + softmax, phase 2 = PV + refill, one
// barrier each; the K/V ring is 4 stages deep so the lagging half still reads its tile while the
// leading half refills two tiles ahead.
constexpr int F2STAGES = 4;
constexpr int F2NT = 512;
constexpr int F2NP = 2 * FTILE / (16 * F2NT);    // LDS-DMA instructions per thread per K/V tile (4)

template <int MODE>
__global__ __launch_bounds__(F2NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void coatt_fused2_k(FusedArgs a) {
  // [stage s: K 16 KB | V 16 KB] x 4, then (MODE 1) the per-key normalisers of each stage's tile
  __shared__ __attribute__((aligned(16))) char lds[F2STAGES * 2 * FTILE + F2STAGES * FBK * 4];
  constexpr int NP = F2NP + (MODE == 1);        // LDS-DMA instructions per thread per tile
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int grp = w >> 2;                       // stagger group (waves 4-7 lag one phase)
  const int pair = (w >> 1) & 1 ? 2 * grp + 1 : 2 * grp;
  const int hb = w & 1;                         // output-channel half of this wave
  const int nfull8 = (a.nfull + 7) & ~7;
  int item, split = 0;
  bool live = true;
  if ((int)blockIdx.x < nfull8) {
    const int per_xcd = nfull8 >> 3;
    item = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    live = item < a.nfull;
  } else {
    const int t = blockIdx.x - nfull8;
    item = a.nfull + t / a.nsplit;
    split = t % a.nsplit;
    live = item < a.nitems;
  }
  if (!live) return;                            // whole workgroup: uniform
  const bool part = item >= a.nfull;
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const int HW = a.HW;
  const long long b = bd / a.ndir;
  const bf16* Q = d.q + b * HW * d.ldq;
  const bf16* K = d.k + b * HW * d.ldk;
  const bf16* V = d.v + b * HW * d.ldv;
  const int q0 = rb * FBQ;
  const int qrow = q0 + pair * 32 + r;
  const bool qok = qrow < HW;
  const void* zp = (const void*)g_zero16_fused;
  const float L2E = 1.4426950408889634f;

  // the pair's query rows as B fragments of S^T = K Q^T (k-step ks: d = 16 ks + 8 h .. +7)
  bf16x8 qreg[16];
  {
    const bf16* src = Q + (long long)(qok ? qrow : 0) * d.ldq + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) qreg[ks] = qok ? *(const bf16x8*)(src + 16 * ks) : bf16x8{};
  }

  const int ntiles = (HW + FBK - 1) / FBK;
  const int tb = part ? split * a.tps : 0;
  const int nt = part ? min(ntiles - tb, a.tps) : ntiles;
  // piece i (< 2) of tile t's K and V images: chunk p = 512 i + tid -> key row p >> 5, position
  // p & 31 (the 4-wave kernel's images: K chunk ^ (row & 15), V chunk ^ ((row & 3) << 2))
  auto issue_piece = [&](int t, int i) {
    char* kb = lds + ((t & (F2STAGES - 1)) * 2) * FTILE;
    char* vb = kb + FTILE;
    const int p = i * F2NT + tid;
    const int row = p >> 5, cpos = p & 31;
    const int key = (tb + t) * FBK + row;
    const bool ok = key < HW;
    const bf16* ks = K + (long long)key * d.ldk + ((cpos ^ (row & 15)) << 3);
    const bf16* vs = V + (long long)key * d.ldv + ((cpos ^ ((row & 3) << 2)) << 3);
    const int wb = (i * F2NT + (tid & ~63)) * 16;
    glds16f(ok ? (const void*)ks : zp, kb + wb);
    glds16f(ok ? (const void*)vs : zp, vb + wb);
  };
  // MODE 1: the tile's 32 per-key normalisers (128 B, +inf padded to HWp) by lanes 0-7 of every
  // wave (same bytes to the same place), so each wave's DMA count per tile stays uniform
  auto issue_klse = [&](int t) {
    if constexpr (MODE == 1) {
      char* kl = lds + F2STAGES * 2 * FTILE + (t & (F2STAGES - 1)) * FBK * 4;
      if (lane < 8) glds16f(d.klse + b * a.HWp + (tb + t) * FBK + 4 * lane, kl);
    }
  };
  // prologue: tiles 0..2 in flight, tile 0 landed
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (t < nt) { issue_piece(t, 0); issue_piece(t, 1); issue_klse(t); }
  // vmcnt: the Q loads are older than every DMA piece, so counted waits cover them too
  if (nt >= 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NP) : "memory");
  else if (nt == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier_f();
  if (grp) raw_barrier_f();                     // the stagger: waves 4-7 one phase behind

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const int sw = r & 15;
  const int G = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;

  for (int t = 0; t < nt; ++t) {
    const char* kb = lds + ((t & (F2STAGES - 1)) * 2) * FTILE;
    const char* vb = kb + FTILE;
    f32x4 nk[4];
    if constexpr (MODE == 1) {   // lane's keys 32t + 8q + 4h + 0..3
      const float* kl = (const float*)(lds + F2STAGES * 2 * FTILE + (t & (F2STAGES - 1)) * FBK * 4) + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) nk[q] = *(const f32x4*)(kl + 8 * q);
    }
    // ---- phase 1: S^T = K Q^T (32 keys x the pair's 32 queries), softmax -> P
    f32x16 s = f32x16{};
    {
      constexpr int KPF = 3;
      const char* krp = kb + r * FROWB;
      bf16x8 kf[KPF];
#pragma unroll
      for (int u = 0; u < KPF; ++u) kf[u] = *(const bf16x8*)(krp + (((2 * u + h) ^ sw) << 4));
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        const bf16x8 kc = kf[ks % KPF];
        if (ks + KPF < 16) kf[ks % KPF] = *(const bf16x8*)(krp + (((2 * (ks + KPF) + h) ^ sw) << 4));
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qreg[ks], s, 0, 0, 0);
      }
    }
    bf16x8 pf[2];
    const int key0 = (tb + t) * FBK;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int i = 8 * s2 + j;
          pv[j] = __builtin_amdgcn_exp2f(fmaf(s[i], L2E, -nk[i >> 2][i & 3]));
        }
        pf[s2] = pack8(pv);
      }
    } else {
      if (key0 + FBK > HW) {
#pragma unroll
        for (int i = 0; i < 16; ++i)
          if (key0 + (i & 3) + 8 * (i >> 2) + 4 * h >= HW) s[i] = -INFINITY;
      }
      float mx = s[0];
#pragma unroll
      for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[i]);
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mnew = fmaxf(m, mx * L2E);
      if (__builtin_amdgcn_ballot_w64(mnew > m + RESCALE_T) != 0) {
        const float alpha = __builtin_amdgcn_exp2f(m - mnew);
        l *= alpha;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        m = mnew;
      }
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        float pv[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pv[j] = __builtin_amdgcn_exp2f(fmaf(s[8 * s2 + j], L2E, -m));
          l += pv[j];
        }
        pf[s2] = pack8(pv);
      }
    }
    // end of phase 1: tile t+1 landed (this wave's pieces; tile t+2's may stay in flight)
    if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_f();

    // ---- phase 2: O^T[this half] += V^T P^T over the tile's 32 keys; refill tile t+3
    const bool dodma = t + 3 < nt;
    {
      const unsigned vrow = lds_addr(vb + (4 * h + q4) * FROWB);
      auto vread = [&](int dt, int sk) {
        const int g = 8 * (4 * hb + dt) + 4 * (G & 1) + pp;
        const unsigned a1 = vrow + 16 * sk * FROWB + ((g ^ (q4 << 3)) << 3);
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a1));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(8 * FROWB));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      constexpr int VPF = 3;
      bf16x8 vf[VPF];
#pragma unroll
      for (int u = 0; u < VPF; ++u) vf[u] = vread(u >> 1, u & 1);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        bf16x8 cur = vf[it % VPF];
        if (it + VPF < 8) vf[it % VPF] = vread((it + VPF) >> 1, (it + VPF) & 1);
        const int younger = 2 * (7 - it < VPF ? 7 - it : VPF);
        if (younger >= 6) lgkm_wait<6>(cur);
        else if (younger == 4) lgkm_wait<4>(cur);
        else if (younger == 2) lgkm_wait<2>(cur);
        else lgkm_wait<0>(cur);
        o[it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[it & 1], o[it >> 1], 0, 0, 0);
        if ((it & 3) == 1 && dodma) issue_piece(t + 3, it >> 2);
      }
      if (dodma) issue_klse(t + 3);
    }
    // end of phase 2: tile t+1 landed (tiles t+2, t+3 may stay in flight)
    if (t + 3 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NP) : "memory");
    else if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_f();
  }
  if (!grp) raw_barrier_f();                    // equal barrier counts for both halves

  // ---- epilogue: this wave's half of O; register i of tile dt: d = 128 hb + 32 dt + (i&3) + 8(i>>2) + 4h
  l += __shfl_xor(l, 32, 64);
  if (part) {
    if (qok) {
      const long long prow = ((long long)split * (a.nitems - a.nfull) + (item - a.nfull)) * FBQ + (qrow - q0);
      float* op = a.opart + prow * FD + 128 * hb + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          *(f32x4*)(op + 32 * dt + 8 * c) = f32x4{o[dt][4 * c], o[dt][4 * c + 1], o[dt][4 * c + 2], o[dt][4 * c + 3]};
      if (MODE == 0 && h == 0 && hb == 0) *(float2*)(a.mlpart + prow * 2) = float2{m, l};
    }
    return;
  }
  if (MODE == 0 && d.lse && h == 0 && hb == 0 && qrow < a.HWp)
    d.lse[b * a.HWp + qrow] = qok ? m + __builtin_amdgcn_logf(l) : INFINITY;
  if (qok) {
    const float inv = MODE == 0 ? 1.f / l : 1.f;
    bf16* op = d.o + (b * HW + qrow) * d.ldo + 128 * hb + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v;
        if (a.accumulate) {
          const bf16x4 old = *(const bf16x4*)(op + 32 * dt + 8 * c);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv + (float)old[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv);
        }
        *(bf16x4*)(op + 32 * dt + 8 * c) = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Wave pairs WITHOUT the duplicated S product (coatt_fused3_k): both waves of a pair hold the
// pair's 32 query rows (Q, 64 VGPRs) but split each 32-key tile -- wave hb computes S^T for keys
// [16 hb, +16) on v_mfma_f32_16x16x32_bf16 (8 values per lane: 4 keys x 2 queries) -- and the
// output channels [128 hb, +128) of O.  Per tile the pair exchanges through LDS its partial row
// maxima (128 B per wave) and its half of P (bf16, 1 KB per wave, [query][32 keys in the PV
// operand's k order] with a 16-B chunk XOR (q >> 2) & 3), so each wave runs the PV product over
// all 32 keys for its channels.
// Three phases per tile, one barrier each: [S + partial max] [pair max, rescale, P] [PV + refill];
// waves 4-7 lag one phase.  The row sums stay per wave (own keys) and are added once at the end.
// Algorithmic MFMA count (no duplicated S); S is summed in a different order than the 4-wave
// kernel's 32x32x16 product (not bitwise equal to it).
constexpr int F3PB = 32 * 32 * 2;        // P of one pair: [32 queries][32 keys] bf16

template <int MODE>
__global__ __launch_bounds__(F2NT) __attribute__((amdgpu_waves_per_eu(2, 2)))
void coatt_fused3_k(FusedArgs a) {
  constexpr int RING = F2STAGES * 2 * FTILE;
  constexpr int KLB = F2STAGES * FBK * 4;
  // [K/V ring 128 KB][klse ring][P of 4 pairs 8 KB][row max / sum exchange: 8 waves x 32 floats]
  __shared__ __attribute__((aligned(16))) char lds[RING + KLB + 4 * F3PB + 8 * 32 * 4];
  constexpr int NP = F2NP + (MODE == 1);
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;            // O layout (32x32 accumulators)
  const int c16 = lane & 15, g4 = lane >> 4;         // S layout (16x16 accumulators)
  const int grp = w >> 2;
  const int pair = (w >> 1) & 1 ? 2 * grp + 1 : 2 * grp;
  const int hb = w & 1;
  const int nfull8 = (a.nfull + 7) & ~7;
  int item, split = 0;
  bool live = true;
  if ((int)blockIdx.x < nfull8) {
    const int per_xcd = nfull8 >> 3;
    item = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
    live = item < a.nfull;
  } else {
    const int t = blockIdx.x - nfull8;
    item = a.nfull + t / a.nsplit;
    split = t % a.nsplit;
    live = item < a.nitems;
  }
  if (!live) return;
  const bool part = item >= a.nfull;
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const int HW = a.HW;
  const long long b = bd / a.ndir;
  const bf16* Q = d.q + b * HW * d.ldq;
  const bf16* K = d.k + b * HW * d.ldk;
  const bf16* V = d.v + b * HW * d.ldv;
  const int q0 = rb * FBQ;
  const int qrow = q0 + pair * 32 + r;
  const bool qok = qrow < HW;
  const void* zp = (const void*)g_zero16_fused;
  const float L2E = 1.4426950408889634f;
  char* pbuf = lds + RING + KLB + pair * F3PB;
  float* xch = (float*)(lds + RING + KLB + 4 * F3PB);       // [8][32]
  float* xmine = xch + w * 32;
  const float* xpart = xch + (w ^ 1) * 32;

  // Q as B fragments of S^T = K Q^T (16x16x32): q-block qb, d chunk ks -> query 16 qb + c16,
  // d = 32 ks + 8 g4 + 0..7
  bf16x8 qreg[2][8];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int row = q0 + pair * 32 + 16 * qb + c16;
    const bool ok = row < HW;
    const bf16* src = Q + (long long)(ok ? row : 0) * d.ldq + 8 * g4;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qreg[qb][ks] = ok ? *(const bf16x8*)(src + 32 * ks) : bf16x8{};
  }

  const int ntiles = (HW + FBK - 1) / FBK;
  const int tb = part ? split * a.tps : 0;
  const int nt = part ? min(ntiles - tb, a.tps) : ntiles;
  auto issue_piece = [&](int t, int i) {
    char* kb = lds + ((t & (F2STAGES - 1)) * 2) * FTILE;
    char* vb = kb + FTILE;
    const int p = i * F2NT + tid;
    const int row = p >> 5, cpos = p & 31;
    const int key = (tb + t) * FBK + row;
    const bool ok = key < HW;
    const bf16* ks = K + (long long)key * d.ldk + ((cpos ^ (row & 15)) << 3);
    const bf16* vs = V + (long long)key * d.ldv + ((cpos ^ ((row & 3) << 2)) << 3);
    const int wb = (i * F2NT + (tid & ~63)) * 16;
    glds16f(ok ? (const void*)ks : zp, kb + wb);
    glds16f(ok ? (const void*)vs : zp, vb + wb);
  };
  auto issue_klse = [&](int t) {
    if constexpr (MODE == 1) {
      char* kl = lds + RING + (t & (F2STAGES - 1)) * FBK * 4;
      if (lane < 8) glds16f(d.klse + b * a.HWp + (tb + t) * FBK + 4 * lane, kl);
    }
  };
#pragma unroll
  for (int t = 0; t < 3; ++t)
    if (t < nt) { issue_piece(t, 0); issue_piece(t, 1); issue_klse(t); }
  if (nt >= 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NP) : "memory");
  else if (nt == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  raw_barrier_f();
  if (grp) raw_barrier_f();

  f32x16 o[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) o[dt] = f32x16{};
  float ms[2] = {-INFINITY, -INFINITY}, ls[2] = {0.f, 0.f};   // S layout: queries 16 qb + c16
  float mo = -INFINITY;                                       // O layout: query r
  const int G = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
  const int krow = 16 * hb + c16;                             // this lane's key row of the tile

  auto wait_t1 = [&](int t, bool after_refill) {   // tile t+1 landed (this wave's pieces)
    if (after_refill && t + 3 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * NP) : "memory");
    else if (t + 2 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };

  for (int t = 0; t < nt; ++t) {
    const char* kb = lds + ((t & (F2STAGES - 1)) * 2) * FTILE;
    const char* vb = kb + FTILE;
    const int key0 = (tb + t) * FBK;
    // ---- phase A: S^T for this wave's 16 keys x the pair's 32 queries; partial row max
    f32x4 s[2] = {f32x4{}, f32x4{}};
    {
      constexpr int KPF = 3;
      const char* kr = kb + krow * FROWB;
      bf16x8 kf[KPF];
#pragma unroll
      for (int u = 0; u < KPF; ++u) kf[u] = *(const bf16x8*)(kr + (((4 * u + g4) ^ c16) << 4));
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 kc = kf[ks % KPF];
        if (ks + KPF < 8) kf[ks % KPF] = *(const bf16x8*)(kr + (((4 * (ks + KPF) + g4) ^ c16) << 4));
        s[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kc, qreg[0][ks], s[0], 0, 0, 0);
        s[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kc, qreg[1][ks], s[1], 0, 0, 0);
      }
    }
    // register i of s[qb]: key key0 + 16 hb + 4 g4 + i, query 16 qb + c16
    if constexpr (MODE == 0) {
      if (key0 + FBK > HW) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (key0 + 16 * hb + 4 * g4 + i >= HW) s[qb][i] = -INFINITY;
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        float mx = fmaxf(fmaxf(s[qb][0], s[qb][1]), fmaxf(s[qb][2], s[qb][3]));
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        if (g4 == 0) xmine[16 * qb + c16] = mx;
      }
    }
    wait_t1(t, false);
    // the partner reads these LDS words after the barrier: the stores must have completed
    // (s_barrier does not wait for them)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier_f();

    // ---- phase B: pair row max, lazy rescale, P of this wave's keys -> the pair's P buffer
    float pv[2][4];
    if constexpr (MODE == 1) {
      const f32x4 nk = *(const f32x4*)(lds + RING + (t & (F2STAGES - 1)) * FBK * 4 + (16 * hb + 4 * g4) * 4);
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i) pv[qb][i] = __builtin_amdgcn_exp2f(fmaf(s[qb][i], L2E, -nk[i]));
    } else {
      float mn[2];
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
        mn[qb] = fmaxf(ms[qb], fmaxf(xmine[16 * qb + c16], xpart[16 * qb + c16]) * L2E);
      const float mno = fmaxf(mo, fmaxf(xmine[r], xpart[r]) * L2E);
      if (__builtin_amdgcn_ballot_w64(mn[0] > ms[0] + RESCALE_T || mn[1] > ms[1] + RESCALE_T) != 0) {
#pragma unroll
        for (int qb = 0; qb < 2; ++qb) {
          ls[qb] *= __builtin_amdgcn_exp2f(ms[qb] - mn[qb]);
          ms[qb] = mn[qb];
        }
        const float alpha = __builtin_amdgcn_exp2f(mo - mno);
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int i = 0; i < 16; ++i) o[dt][i] *= alpha;
        mo = mno;
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          pv[qb][i] = __builtin_amdgcn_exp2f(fmaf(s[qb][i], L2E, -ms[qb]));
          ls[qb] += pv[qb][i];
        }
    }
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
      bf16x4 v4;
#pragma unroll
      for (int i = 0; i < 4; ++i) v4[i] = (bf16)pv[qb][i];
      // the PV B operand's k order (the V^T fragments' key order, as the 4-wave kernel's P
      // registers): k-step sk, lane half h, element 4a + i <-> key 16 sk + 8 a + 4 h + i.  So
      // key 16 hb + 4 g4 + i lands in chunk 2 hb + (g4 & 1), element 4 (g4 >> 1) + i.
      const int q = 16 * qb + c16;
      const int chunk = (2 * hb + (g4 & 1)) ^ ((q >> 2) & 3);
      *(bf16x4*)(pbuf + q * 64 + (chunk << 4) + 8 * (g4 >> 1)) = v4;
    }
    wait_t1(t, false);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier_f();

    // ---- phase C: O^T[this half] += V^T P^T over all 32 keys; refill tile t+3
    bf16x8 pf[2];
#pragma unroll
    for (int sk = 0; sk < 2; ++sk)
      pf[sk] = *(const bf16x8*)(pbuf + r * 64 + (((2 * sk + h) ^ ((r >> 2) & 3)) << 4));
    const bool dodma = t + 3 < nt;
    {
      const unsigned vrow = lds_addr(vb + (4 * h + q4) * FROWB);
      auto vread = [&](int dt, int sk) {
        const int g = 8 * (4 * hb + dt) + 4 * (G & 1) + pp;
        const unsigned a1 = vrow + 16 * sk * FROWB + ((g ^ (q4 << 3)) << 3);
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a1));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(8 * FROWB));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      constexpr int VPF = 3;
      bf16x8 vf[VPF];
#pragma unroll
      for (int u = 0; u < VPF; ++u) vf[u] = vread(u >> 1, u & 1);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        bf16x8 cur = vf[it % VPF];
        if (it + VPF < 8) vf[it % VPF] = vread((it + VPF) >> 1, (it + VPF) & 1);
        const int younger = 2 * (7 - it < VPF ? 7 - it : VPF);
        if (younger >= 6) lgkm_wait<6>(cur);
        else if (younger == 4) lgkm_wait<4>(cur);
        else if (younger == 2) lgkm_wait<2>(cur);
        else lgkm_wait<0>(cur);
        o[it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[it & 1], o[it >> 1], 0, 0, 0);
        if ((it & 3) == 1 && dodma) issue_piece(t + 3, it >> 2);
      }
      if (dodma) issue_klse(t + 3);
    }
    wait_t1(t, true);
    raw_barrier_f();
  }
  if (!grp) raw_barrier_f();

  // ---- row sums: this wave's keys (S layout) -> per query, + the partner's (O layout)
  float lo = 0.f;
  if constexpr (MODE == 0) {
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float v = ls[qb];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (g4 == 0) xmine[16 * qb + c16] = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier_f();
    lo = xmine[r] + xpart[r];
  }

  if (part) {
    if (qok) {
      const long long prow = ((long long)split * (a.nitems - a.nfull) + (item - a.nfull)) * FBQ + (qrow - q0);
      float* op = a.opart + prow * FD + 128 * hb + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          *(f32x4*)(op + 32 * dt + 8 * c) = f32x4{o[dt][4 * c], o[dt][4 * c + 1], o[dt][4 * c + 2], o[dt][4 * c + 3]};
      if (MODE == 0 && h == 0 && hb == 0) *(float2*)(a.mlpart + prow * 2) = float2{mo, lo};
    }
    return;
  }
  if (MODE == 0 && d.lse && h == 0 && hb == 0 && qrow < a.HWp)
    d.lse[b * a.HWp + qrow] = qok ? mo + __builtin_amdgcn_logf(lo) : INFINITY;
  if (qok) {
    const float inv = MODE == 0 ? 1.f / lo : 1.f;
    bf16* op = d.o + (b * HW + qrow) * d.ldo + 128 * hb + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v;
        if (a.accumulate) {
          const bf16x4 old = *(const bf16x4*)(op + 32 * dt + 8 * c);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv + (float)old[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] * inv);
        }
        *(bf16x4*)(op + 32 * dt + 8 * c) = v;
      }
  }
}
#endif  // CN_EXPERIMENTAL

// Fold the key-split partials of one row of a tail item: O = sum_s 2^(m_s - M) O_s /
// sum_s 2^(m_s - M) l_s, splits in order (deterministic).  One thread = 8 channels of one row.
// MODE 1 (per-key normaliser, linear in the keys): O (+)= sum_s O_s.
template <int MODE>
__global__ __launch_bounds__(256) void coatt_merge_k(FusedArgs a) {
  const long long t = blockIdx.x * 256ll + threadIdx.x;
  const long long rows = (long long)(a.nitems - a.nfull) * FBQ;   // rows per split slab
  if (t >= rows * (FD / 8)) return;
  const long long row = t / (FD / 8);
  const int c0 = (int)(t % (FD / 8)) * 8;
  const int item = a.nfull + (int)(row / FBQ);
  const int rb = item % a.nrb, bd = item / a.nrb;
  const int q = rb * FBQ + (int)(row % FBQ);
  if (q >= a.HW) return;
  const FusedDir d = a.dir[bd % a.ndir];
  const long long b = bd / a.ndir;
  const long long sstride = rows;
  if constexpr (MODE == 1) {
    float acc[8];
    bf16* op = d.o + (b * a.HW + q) * d.ldo + c0;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = a.accumulate ? (float)op[e] : 0.f;
    for (int s = 0; s < a.nsplit; ++s) {
      const float* p = a.opart + (s * sstride + row) * FD + c0;
      const f32x4 v0 = *(const f32x4*)p, v1 = *(const f32x4*)(p + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { acc[e] += v0[e]; acc[4 + e] += v1[e]; }
    }
    bf16x8 outv;
#pragma unroll
    for (int e = 0; e < 8; ++e) outv[e] = (bf16)acc[e];
    *(bf16x8*)op = outv;
    return;
  }
  float M = -INFINITY;
  for (int s = 0; s < a.nsplit; ++s) M = fmaxf(M, a.mlpart[(s * sstride + row) * 2]);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  float L = 0.f;
  for (int s = 0; s < a.nsplit; ++s) {
    const float2 ml = *(const float2*)(a.mlpart + (s * sstride + row) * 2);
    const float wgt = ml.y > 0.f ? __builtin_amdgcn_exp2f(ml.x - M) : 0.f;
    L = fmaf(ml.y, wgt, L);
    const float* op = a.opart + (s * sstride + row) * FD + c0;
    const f32x4 v0 = *(const f32x4*)op, v1 = *(const f32x4*)(op + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[e] = fmaf(v0[e], wgt, acc[e]);
      acc[4 + e] = fmaf(v1[e], wgt, acc[4 + e]);
    }
  }
  const float inv = 1.f / L;
  bf16x8 outv;
#pragma unroll
  for (int e = 0; e < 8; ++e) outv[e] = (bf16)(acc[e] * inv);
  *(bf16x8*)(d.o + (b * a.HW + q) * d.ldo + c0) = outv;
  if (d.lse && c0 == 0) d.lse[b * a.HWp + q] = M + __builtin_amdgcn_logf(L);
}

}  // namespace

static bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Tail split for `items` workgroup-sized work items at one workgroup per CU: the items of the
// last, partial round of 256 (all of them when there are fewer) are split over up to
// 256 / tail workgroups each (>= 16 key tiles per split).
static void plan_split(int items, int ntiles, int* nfull, int* nsplit) {
  *nfull = items;
  *nsplit = 1;
  const int rem = items % 256;   // the partial round (all of it when items < 256)
  if (rem == 0) return;
  int s = 256 / rem;
  if (s > 8) s = 8;
  while (s > 1 && ntiles / s < 16) --s;
  if (s < 2) return;
  *nfull = items - rem;
  *nsplit = s;
}

// Kernel variant: 1 = coatt_fused_fwd_k (4 waves, one per SIMD, 32 rows per wave), 2 =
// coatt_fused2_k (wave pairs, duplicated S), 3 = coatt_fused3_k (wave pairs splitting the keys),
// 4 = coatt_dsplit_k (coatt_dsplit.hip: wave pairs splitting the channels, 64 query rows per
// pair), 5 = coatt_q48_k (coatt_q48.hip: 48 rows per wave, Q in registers, 16x16x32 tiles,
// stream-K work split; the default since round 5: 183 vs 224 us at configs[3], 139 vs 165 us for
// the training forward at 4 pairs, the PV kernel even).  CN_COATT_VARIANT picks the default;
// cn_coatt_force_variant overrides it (tests, A/B tools).
static int g_coatt_variant = 0;
static bool variant_built(int x) { return x == 1 || x == 5 || (CN_EXPERIMENTAL && x >= 2 && x <= 4); }
static int coatt_variant() {
  static const int v = [] {
    const char* e = getenv("CN_COATT_VARIANT");
    const int x = e ? atoi(e) : 5;
    return variant_built(x) ? x : 5;
  }();
  return g_coatt_variant ? g_coatt_variant : v;
}

// Development / test hook: force the forward / PV kernel variant (1..5 as above; 0: default).
// Returns the previous setting.
// Variants 2-4 exist only in CN_EXPERIMENTAL builds (-1 otherwise, nothing changed).
extern "C" int cn_coatt_force_variant(int v) {
  if (v != 0 && !variant_built(v)) return -1;
  const int old = g_coatt_variant;
  g_coatt_variant = v;
  return old;
}

// The variant-5 launch of one co-attention call (coatt_q48.hip): work cut across the CUs when the
// outputs take the merge's 16-byte rows (merge_ok) and the workspace holds the partials.
static int q48_launch(int mode, FusedArgs& a, int B, int nd, bool merge_ok, void* ws,
                      size_t ws_bytes, hipStream_t st) {
  return coatt_q48_launch(mode, a, B, nd, merge_ok, ws, ws_bytes, st);
}

static int fused_launch(int mode, FusedArgs& a, int B, int nd, hipStream_t st) {
  a.ndir = nd;
  a.nrb = (a.HW + FBQ - 1) / FBQ;
  a.nitems = a.nrb * B * nd;
  if (a.nsplit < 2) { a.nsplit = 1; a.nfull = a.nitems; }
  const int ntiles = (a.HW + FBK - 1) / FBK;
  a.tps = (ntiles + a.nsplit - 1) / a.nsplit;
  const int nfull8 = (a.nfull + 7) & ~7;
  a.nwork = nfull8 + (a.nitems - a.nfull) * a.nsplit;
  dim3 grid(a.nwork);
  const int var = coatt_variant();
#if CN_EXPERIMENTAL
  if (var == 2) {
    if (mode == 0) hipLaunchKernelGGL(coatt_fused2_k<0>, grid, dim3(F2NT), 0, st, a);
    else hipLaunchKernelGGL(coatt_fused2_k<1>, grid, dim3(F2NT), 0, st, a);
  } else if (var == 3) {
    if (mode == 0) hipLaunchKernelGGL(coatt_fused3_k<0>, grid, dim3(F2NT), 0, st, a);
    else hipLaunchKernelGGL(coatt_fused3_k<1>, grid, dim3(F2NT), 0, st, a);
  } else if (var == 4) {
    const int rc = coatt_dsplit_launch(mode, a, grid, st);
    if (rc) return rc;
  } else
#endif
  {
    (void)var;
    if (mode == 0) hipLaunchKernelGGL(coatt_fused_fwd_k<0>, grid, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(coatt_fused_fwd_k<1>, grid, dim3(256), 0, st, a);
  }
  CN_CHECK_LAUNCH();
  if (a.nsplit > 1) {
    const long long threads = (long long)(a.nitems - a.nfull) * FBQ * (FD / 8);
    const dim3 g((unsigned)((threads + 255) / 256));
    if (mode == 0) hipLaunchKernelGGL(coatt_merge_k<0>, g, dim3(256), 0, st, a);
    else hipLaunchKernelGGL(coatt_merge_k<1>, g, dim3(256), 0, st, a);
    CN_CHECK_LAUNCH();
  }
  return 0;
}

extern "C" size_t cn_coatt_fused_workspace_bytes(int B, int HW, int ndir) {
  if (coatt_variant() == 5) {
    const int rb = coatt_q48_rows();
    return coatt_q48_workspace_bytes((HW + rb - 1) / rb * B * ndir, (HW + FBK - 1) / FBK);
  }
  const int nrb = (HW + FBQ - 1) / FBQ;
  int nfull, s;
  plan_split(nrb * B * ndir, (HW + FBK - 1) / FBK, &nfull, &s);
  if (s == 1) return 0;
  return (size_t)s * (nrb * B * ndir - nfull) * FBQ * (FD + 2) * sizeof(float);
}

static int fused_check(const void* q, long long ldq, const void* k, long long ldk, const void* v,
                       long long ldv, long long ldo, int C) {
  if (C != FD) return CN_ERR_SHAPE;
  if (ldq % 8 || ldk % 8 || ldv % 8 || ldo % 4 || ldq < C || ldk < C || ldv < C || ldo < C)
    return CN_ERR_ALIGN;
  if (!aligned16(q) || !aligned16(k) || !aligned16(v)) return CN_ERR_ALIGN;
  return 0;
}

extern "C" int cn_coatt_fused_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                  const void* vb, long long ld_vb, int B, int HW, int C, void* za,
                                  void* zb, long long ld_z, hipStream_t st) {
  return cn_coatt_flash_fwd(vat, ld_vat, va, ld_va, vb, ld_vb, B, HW, C, za, zb, ld_z, nullptr,
                            nullptr, st);
}

extern "C" int cn_coatt_fused_fwd_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                     const void* vb, long long ld_vb, int B, int HW, int C, void* za,
                                     void* zb, long long ld_z, void* ws, size_t ws_bytes, hipStream_t st) {
  if (B <= 0 || HW <= 0) return CN_ERR_SHAPE;
  int rc = fused_check(vat, ld_vat, vb, ld_vb, va, ld_va, ld_z, C);
  if (rc) return rc;
  if (((uintptr_t)za & 7) || ((uintptr_t)zb & 7)) return CN_ERR_ALIGN;
  FusedArgs a = {};
  int nd = 0;
  if (za) a.dir[nd++] = FusedDir{(const bf16*)vat, (const bf16*)vb, (const bf16*)vb, (bf16*)za, ld_vat, ld_vb, ld_vb, ld_z, nullptr, nullptr};
  if (zb) a.dir[nd++] = FusedDir{(const bf16*)vb, (const bf16*)vat, (const bf16*)va, (bf16*)zb, ld_vb, ld_vat, ld_va, ld_z, nullptr, nullptr};
  if (nd == 0) return CN_ERR_SHAPE;
  a.HW = HW;
  a.HWp = (HW + 31) / 32 * 32;
  // the merge writes 16-byte rows: unsplit when the outputs are not laid out for that
  const bool merge_ok = !(((uintptr_t)za & 15) || ((uintptr_t)zb & 15) || (ld_z % 8));
  if (coatt_variant() == 5) return q48_launch(0, a, B, nd, merge_ok, ws, ws_bytes, st);
  const int nrb = (HW + FBQ - 1) / FBQ;
  plan_split(nrb * B * nd, (HW + FBK - 1) / FBK, &a.nfull, &a.nsplit);
  if (!merge_ok) a.nsplit = 1;
  if (a.nsplit > 1) {
    const size_t tail_rows = (size_t)a.nsplit * (nrb * B * nd - a.nfull) * FBQ;
    // no (or a too small / misaligned) workspace: the unsplit launch, as the _ws siblings do
    if (!ws || ws_bytes < tail_rows * (FD + 2) * sizeof(float) || !aligned16(ws)) {
      a.nsplit = 1;
    } else {
      a.opart = (float*)ws;
      a.mlpart = a.opart + tail_rows * FD;
    }
  }
  return fused_launch(0, a, B, nd, st);
}

extern "C" int cn_coatt_flash_fwd(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                  const void* vb, long long ld_vb, int B, int HW, int C, void* za,
                                  void* zb, long long ld_z, float* lse_a, float* lse_b,
                                  hipStream_t st) {
  if (B <= 0 || HW <= 0) return CN_ERR_SHAPE;
  int rc = fused_check(vat, ld_vat, vb, ld_vb, va, ld_va, ld_z, C);
  if (rc) return rc;
  if (((uintptr_t)za & 7) || ((uintptr_t)zb & 7)) return CN_ERR_ALIGN;
  FusedArgs a = {};
  int nd = 0;
  // direction 0: Z_a = softmax_j(S) Vb  (queries i: Va_t; keys j: Vb; values Vb)
  if (za) a.dir[nd++] = FusedDir{(const bf16*)vat, (const bf16*)vb, (const bf16*)vb, (bf16*)za, ld_vat, ld_vb, ld_vb, ld_z, lse_a, nullptr};
  // direction 1: Z_b = softmax_i(S)^T Va  (queries j: Vb; keys i: Va_t; values Va)
  if (zb) a.dir[nd++] = FusedDir{(const bf16*)vb, (const bf16*)vat, (const bf16*)va, (bf16*)zb, ld_vb, ld_vat, ld_va, ld_z, lse_b, nullptr};
  if (nd == 0) return CN_ERR_SHAPE;
  a.HW = HW;
  a.HWp = (HW + 31) / 32 * 32;
  a.accumulate = 0;
  if (coatt_variant() == 5) return q48_launch(0, a, B, nd, false, nullptr, 0, st);
  return fused_launch(0, a, B, nd, st);
}

extern "C" int cn_coatt_flash_fwd_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                     const void* vb, long long ld_vb, int B, int HW, int C, void* za,
                                     void* zb, long long ld_z, float* lse_a, float* lse_b, void* ws,
                                     size_t ws_bytes, hipStream_t st) {
  if (coatt_variant() != 5)   // the 4-wave kernel runs the training forward unsplit
    return cn_coatt_flash_fwd(vat, ld_vat, va, ld_va, vb, ld_vb, B, HW, C, za, zb, ld_z, lse_a, lse_b, st);
  if (B <= 0 || HW <= 0) return CN_ERR_SHAPE;
  int rc = fused_check(vat, ld_vat, vb, ld_vb, va, ld_va, ld_z, C);
  if (rc) return rc;
  if (((uintptr_t)za & 7) || ((uintptr_t)zb & 7)) return CN_ERR_ALIGN;
  FusedArgs a = {};
  int nd = 0;
  if (za) a.dir[nd++] = FusedDir{(const bf16*)vat, (const bf16*)vb, (const bf16*)vb, (bf16*)za, ld_vat, ld_vb, ld_vb, ld_z, lse_a, nullptr};
  if (zb) a.dir[nd++] = FusedDir{(const bf16*)vb, (const bf16*)vat, (const bf16*)va, (bf16*)zb, ld_vb, ld_vat, ld_va, ld_z, lse_b, nullptr};
  if (nd == 0) return CN_ERR_SHAPE;
  a.HW = HW;
  a.HWp = (HW + 31) / 32 * 32;
  const bool merge_ok = !(((uintptr_t)za & 15) || ((uintptr_t)zb & 15) || (ld_z % 8));
  return q48_launch(0, a, B, nd, merge_ok, ws, ws_bytes, st);
}

extern "C" int cn_coatt_flash_pv_ws(const void* q, long long ldq, const void* k, long long ldk,
                                    const void* v, long long ldv, const float* klse, int B, int HW,
                                    int C, void* o, long long ldo, int accumulate, void* ws,
                                    size_t ws_bytes, hipStream_t st) {
  if (B <= 0 || HW <= 0 || !klse || !o) return CN_ERR_SHAPE;
  int rc = fused_check(q, ldq, k, ldk, v, ldv, ldo, C);
  if (rc) return rc;
  if (((uintptr_t)o & 7) || ((uintptr_t)klse & 15)) return CN_ERR_ALIGN;
  FusedArgs a = {};
  a.dir[0] = FusedDir{(const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, ldq, ldk, ldv, ldo, nullptr, klse};
  a.HW = HW;
  a.HWp = (HW + 31) / 32 * 32;
  a.accumulate = accumulate;
  const bool merge_ok = !(((uintptr_t)o & 15) || (ldo % 8));
  if (coatt_variant() == 5) return q48_launch(1, a, B, 1, merge_ok, ws, ws_bytes, st);
  const int nrb = (HW + FBQ - 1) / FBQ;
  plan_split(nrb * B, (HW + FBK - 1) / FBK, &a.nfull, &a.nsplit);
  if (!merge_ok) a.nsplit = 1;
  if (a.nsplit > 1) {
    const size_t tail_rows = (size_t)a.nsplit * (nrb * B - a.nfull) * FBQ;
    if (!ws || ws_bytes < tail_rows * FD * sizeof(float) || !aligned16(ws)) a.nsplit = 1;
    a.opart = (float*)ws;
  }
  return fused_launch(1, a, B, 1, st);
}

extern "C" int cn_coatt_flash_pv(const void* q, long long ldq, const void* k, long long ldk,
                                 const void* v, long long ldv, const float* klse, int B, int HW,
                                 int C, void* o, long long ldo, int accumulate, hipStream_t st) {
  return cn_coatt_flash_pv_ws(q, ldq, k, ldk, v, ldv, klse, B, HW, C, o, ldo, accumulate, nullptr, 0, st);
}
