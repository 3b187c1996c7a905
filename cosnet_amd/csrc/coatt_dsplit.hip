// Flash co-attention forward / PV, kernel variant 4: d-split wave PAIRS with 64 query rows each
// (rgbd_segmentation_RAA.py:160-170 for RGB, :213-221 for depth; the product of
// coatt_fused_fwd_k, same arguments, work items, key splits and outputs).
//
// One workgroup = 4 waves = 2 pairs x 64 query rows (128 rows, as the 4-wave kernel).  Wave hd of
// a pair owns the channel half d in [128 hd, +128):
//   * S^T partial over its half: K (LDS, its 128 channels) x Q^T (the pair's 64 query rows of its
//     half, in 64 VGPRs, loaded once) -- each K fragment feeds TWO 32x32x16 MFMAs (two 32-row
//     query blocks), so a wave reads half the K bytes per MFMA of the 4-wave kernel;
//   * the two partial S (8 KB per wave) are exchanged through LDS and added (a + b == b + a, so
//     both waves hold bitwise the same S and run the same softmax: no second exchange);
//   * O^T for its 128 channels x 64 rows (128 accumulators) += V^T P^T -- each V^T fragment also
//     feeds two MFMAs.
// Per wave and 32-key tile: 32 MFMAs (as the 4-wave kernel) against 8 KB K + 8 KB V^T fragment
// reads + 8 KB exchange write + 8 KB exchange read = 32 KB of LDS traffic instead of 48 KB (K, Q
// and V^T fragments), the bound DESIGN.md section 3.2 measures.  The price: the softmax of 64
// rows per wave (duplicated in the pair) and a second barrier per tile.
// Built with -amdgpu-mfma-vgpr-form (as coatt_fused.hip): the accumulators stay in arch VGPRs
// and the allocator parks MFMA source operands in AGPRs (318 registers, no copies in the key
// loop; without the flag it copies the 128 O accumulators AGPR -> VGPR every tile).
#include "common.h"
#include "coatt_fused.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int DSTAGES = 3;                    // K/V ring depth (as the 4-wave kernel)
constexpr int DDMA = 2 * FTILE / 4096;        // LDS-DMA instructions per thread per K/V tile
constexpr int DXB = 4 * 2 * 4 * 1024;         // exchange: [wave][query block][4 regs][64 lanes][16 B]
constexpr int DKPF = 3;                       // K fragment reads ahead of the S MFMAs
constexpr int DVPF = 3;                       // V^T fragment reads ahead of the PV MFMAs
constexpr float DRESCALE_T = 8.0f;            // lazy rescale threshold (log2), as the 4-wave kernel

__device__ __attribute__((aligned(16))) unsigned g_zero16_ds[4];

__device__ __forceinline__ void glds16d(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void raw_barrier_d() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned lds_addr_d(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N>
__device__ __forceinline__ void lgkm_wait_d(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

__device__ __forceinline__ bf16x8 pack8d(const float* f) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)f[j];
  return r;
}

// MODE 0: online softmax over the keys, O = P V / l (+ optional LSE); MODE 1: per-key
// normaliser, O (+)= P V (coatt_fused_fwd_k's modes).
template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void coatt_dsplit_k(FusedArgs a) {
  // [stage s: K 16 KB | V 16 KB] x 3, then the S exchange (32 KB)
  __shared__ __attribute__((aligned(16))) char lds[DSTAGES * 2 * FTILE + DXB];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int pr = w >> 1, hd = w & 1;          // pair (query rows 64 pr ..), channel half
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
  const bool part = item >= a.nfull;
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const int HW = a.HW;
  const long long b = bd / a.ndir;
  const bf16* Q = d.q + b * HW * d.ldq;
  const bf16* K = d.k + b * HW * d.ldk;
  const bf16* V = d.v + b * HW * d.ldv;
  const int q0 = rb * FBQ;
  const void* zp = (const void*)g_zero16_ds;
  char* xb = lds + DSTAGES * 2 * FTILE;

  const int ntiles = (HW + FBK - 1) / FBK;
  const int tb = part ? split * a.tps : 0;
  auto issue_piece = [&](int t, int stage, int i) {
    char* kb = lds + stage * 2 * FTILE;
    char* vb = kb + FTILE;
    const int key0 = (tb + t) * FBK;
    const int p = i * 256 + tid;
    const int row = p >> 5, cpos = p & 31;
    const int key = key0 + row;
    const bool ok = key < HW;
    const bf16* ks = K + (long long)key * d.ldk + ((cpos ^ (row & 15)) << 3);
    const bf16* vs = V + (long long)key * d.ldv + ((cpos ^ ((row & 3) << 2)) << 3);
    const int wb = (i * 256 + (tid & ~63)) * 16;
    glds16d(ok ? (const void*)ks : zp, kb + wb);
    glds16d(ok ? (const void*)vs : zp, vb + wb);
  };
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int i = 0; i < FTILE / 4096; ++i) issue_piece(t, stage, i);
  };

  const int nt = part ? min(ntiles - tb, a.tps) : ntiles;
  issue(0, 0);
  if (nt > 1) issue(1, 1);

  // the pair's query rows of this wave's channel half as B fragments: query block qb, k-step ks
  // (16 channels), lane half h -> row q0 + 64 pr + 32 qb + r, channels 128 hd + 16 ks + 8 h ..
  bf16x8 qreg[2][8];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int row = q0 + 64 * pr + 32 * qb + r;
    const bool ok = row < HW;
    const bf16* src = Q + (long long)(ok ? row : 0) * d.ldq + 128 * hd + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qreg[qb][ks] = ok ? *(const bf16x8*)(src + 16 * ks) : bf16x8{};
  }

  f32x16 o[2][4];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[qb][dt] = f32x16{};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  const float L2E = 1.4426950408889634f;
  const int sw = r & 15;
  const int G = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;

  int st = 0, st2 = 2;
  for (int t = 0; t < nt; ++t) {
    if (t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_d();
    const bool dodma = t + 2 < nt;
    const int dst2 = st2;
    const char* kb = lds + st * 2 * FTILE;
    st = st == DSTAGES - 1 ? 0 : st + 1;
    st2 = st2 == DSTAGES - 1 ? 0 : st2 + 1;
    const char* vb = kb + FTILE;

    f32x4 nk[4];
    if constexpr (MODE == 1) {
      const float* kl = d.klse + b * a.HWp + (tb + t) * FBK + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) nk[q] = *(const f32x4*)(kl + 8 * q);
    }

    // ---- partial S^T over this wave's 128 channels, both query blocks
    f32x16 s[2] = {f32x16{}, f32x16{}};
    {
      const char* krp = kb + r * FROWB;
      bf16x8 kf[DKPF];
#pragma unroll
      for (int u = 0; u < DKPF; ++u) kf[u] = *(const bf16x8*)(krp + (((16 * hd + 2 * u + h) ^ sw) << 4));
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const bf16x8 kc = kf[ks % DKPF];
        if (ks + DKPF < 8) kf[ks % DKPF] = *(const bf16x8*)(krp + (((16 * hd + 2 * (ks + DKPF) + h) ^ sw) << 4));
        s[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qreg[0][ks], s[0], 0, 0, 0);
        s[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qreg[1][ks], s[1], 0, 0, 0);
      }
    }
    // ---- exchange: write this wave's partial, read the partner's, add (both waves: same bits)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *(f32x4*)(xb + (((w * 2 + qb) * 4 + g) * 64 + lane) * 16) =
            f32x4{s[qb][4 * g], s[qb][4 * g + 1], s[qb][4 * g + 2], s[qb][4 * g + 3]};
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier_d();
#pragma unroll
    for (int qb = 0; qb < 2; ++qb)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 x = *(const f32x4*)(xb + ((((w ^ 1) * 2 + qb) * 4 + g) * 64 + lane) * 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) s[qb][4 * g + e] += x[e];
      }

    // ---- softmax (register i: key 32t + (i&3) + 8(i>>2) + 4h), both query blocks
    const int key0 = (tb + t) * FBK;
    bf16x8 pf[2][2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      if constexpr (MODE == 1) {
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          float pv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int i = 8 * s2 + j;
            pv[j] = __builtin_amdgcn_exp2f(fmaf(s[qb][i], L2E, -nk[i >> 2][i & 3]));
          }
          pf[qb][s2] = pack8d(pv);
        }
      } else {
        if (key0 + FBK > HW) {
#pragma unroll
          for (int i = 0; i < 16; ++i)
            if (key0 + (i & 3) + 8 * (i >> 2) + 4 * h >= HW) s[qb][i] = -INFINITY;
        }
        float mx = s[qb][0];
#pragma unroll
        for (int i = 1; i < 16; ++i) mx = fmaxf(mx, s[qb][i]);
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        const float mnew = fmaxf(m[qb], mx * L2E);
        if (__builtin_amdgcn_ballot_w64(mnew > m[qb] + DRESCALE_T) != 0) {
          const float alpha = __builtin_amdgcn_exp2f(m[qb] - mnew);
          l[qb] *= alpha;
#pragma unroll
          for (int dt = 0; dt < 4; ++dt)
#pragma unroll
            for (int i = 0; i < 16; ++i) o[qb][dt][i] *= alpha;
          m[qb] = mnew;
        }
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          float pv[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            pv[j] = __builtin_amdgcn_exp2f(fmaf(s[qb][8 * s2 + j], L2E, -m[qb]));
            l[qb] += pv[j];
          }
          pf[qb][s2] = pack8d(pv);
        }
      }
    }

    // ---- O^T (this wave's 4 channel tiles) += V^T P^T; one V^T fragment, two MFMAs.  Transposed
    // reads as inline asm with counted lgkmcnt waits (see coatt_fused_fwd_k)
    {
      const unsigned vrow = lds_addr_d(vb + (4 * h + q4) * FROWB);
      auto vread = [&](int dt, int sk) {
        const int g = 8 * (4 * hd + dt) + 4 * (G & 1) + pp;
        const unsigned a1 = vrow + 16 * sk * FROWB + ((g ^ (q4 << 3)) << 3);
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a1));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(8 * FROWB));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      bf16x8 vf[DVPF];
#pragma unroll
      for (int u = 0; u < DVPF; ++u) vf[u] = vread(u >> 1, u & 1);
#pragma unroll
      for (int it = 0; it < 8; ++it) {
        bf16x8 cur = vf[it % DVPF];
        if (it + DVPF < 8) vf[it % DVPF] = vread((it + DVPF) >> 1, (it + DVPF) & 1);
        const int younger = 2 * (7 - it < DVPF ? 7 - it : DVPF);
        if (younger >= 6) lgkm_wait_d<6>(cur);
        else if (younger == 4) lgkm_wait_d<4>(cur);
        else if (younger == 2) lgkm_wait_d<2>(cur);
        else lgkm_wait_d<0>(cur);
        o[0][it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[0][it & 1], o[0][it >> 1], 0, 0, 0);
        o[1][it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[1][it & 1], o[1][it >> 1], 0, 0, 0);
        if ((it & 1) && (it >> 1) < FTILE / 4096 && dodma) issue_piece(t + 2, dst2, it >> 1);
      }
    }
  }

  // ---- epilogue: register i of channel tile dt holds d = 128 hd + 32 dt + (i&3) + 8(i>>2) + 4h
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const float lq = l[qb] + __shfl_xor(l[qb], 32, 64);
    const int qrow = q0 + 64 * pr + 32 * qb + r;
    if (part) {
      if (qrow < HW) {
        const long long prow = ((long long)split * (a.nitems - a.nfull) + (item - a.nfull)) * FBQ + (qrow - q0);
        float* op = a.opart + prow * FD + 128 * hd + 4 * h;
#pragma unroll
        for (int dt = 0; dt < 4; ++dt)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            *(f32x4*)(op + 32 * dt + 8 * c) =
                f32x4{o[qb][dt][4 * c], o[qb][dt][4 * c + 1], o[qb][dt][4 * c + 2], o[qb][dt][4 * c + 3]};
        if (MODE == 0 && hd == 0 && h == 0) *(float2*)(a.mlpart + prow * 2) = float2{m[qb], lq};
      }
      continue;
    }
    if (MODE == 0 && d.lse && hd == 0 && h == 0 && qrow < a.HWp)
      d.lse[b * a.HWp + qrow] = qrow < HW ? m[qb] + __builtin_amdgcn_logf(lq) : INFINITY;
    if (qrow < HW) {
      const float inv = MODE == 0 ? 1.f / lq : 1.f;
      bf16* op = d.o + (b * HW + qrow) * d.ldo + 128 * hd + 4 * h;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
          bf16x4 v;
          if (a.accumulate) {
            const bf16x4 old = *(const bf16x4*)(op + 32 * dt + 8 * c);
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[qb][dt][4 * c + j] * inv + (float)old[j]);
          } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[qb][dt][4 * c + j] * inv);
          }
          *(bf16x4*)(op + 32 * dt + 8 * c) = v;
        }
    }
  }
}

}  // namespace

int coatt_dsplit_launch(int mode, const FusedArgs& a, dim3 grid, hipStream_t st) {
  if (mode == 0) hipLaunchKernelGGL(coatt_dsplit_k<0>, grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL(coatt_dsplit_k<1>, grid, dim3(256), 0, st, a);
  CN_CHECK_LAUNCH();
  return 0;
}
