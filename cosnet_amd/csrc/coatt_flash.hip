// Flash-style co-attention BACKWARD for training: the gradient of V_a W^T (the "query" side of
// S = Va_t Vb^T) without the HW x HW affinity, its softmaxes or their gradients ever written to
// HBM (autograd of rgbd_segmentation_RAA.py:160-170 for RGB, :213-221 for depth).
//
// With the forward's per-row normalisers (coatt_fused.hip, log2 units)
//   P0[i][j] = exp2(S[i][j] log2e - lse_a[i])   (softmax over j: "S_column", Z_a = P0 Vb)
//   P1[i][j] = exp2(S[i][j] log2e - lse_b[j])   (softmax over i: "S_row",    Z_b = P1^T Va)
// and D0[i] = dZa[i] . Za[i], D1[j] = dZb[j] . Zb[j]:
//   dS[i][j] = P0 (dZa[i] . Vb[j] - D0[i]) + P1 (Va[i] . dZb[j] - D1[j])
//   dVa_t[i] = sum_j dS[i][j] Vb[j]                       <- this kernel
// (dV_a's other term, sum_j P1[i][j] dZb[j], is cn_coatt_flash_pv; dVb is not needed: frame b
// carries no gradient in the reference, :144-148.)
//
// Structure (the forward kernel's): one workgroup = 4 waves = 128 query rows i; Va_t rows in a
// 64 KB LDS block (the B operand of S^T = Vb Va_t^T), dZa and Va rows of the wave's 32 queries
// in registers (B operands of dP0^T = Vb dZa^T and dP1^T = dZb Va^T); per 32-key tile, Vb (row
// image and transposed image) and dZb (row image) stream through a 2-stage LDS-DMA ring.  The
// three 32x32 products put the query on the lane and 16 keys in registers, so dS^T is formed
// lane-locally and, packed to bf16, is directly the B operand of dVa_t^T += Vb^T dS^T (Vb^T
// fragments by ds_read_b64_tr_b16 from the transposed image).
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int BD = 256;              // channels (all_channel)
constexpr int BQ = 128;              // query rows per workgroup
constexpr int BK = 32;               // keys per tile
constexpr int ROWB = BD * 2;         // bytes per row in LDS
constexpr int TILE = BK * ROWB;      // 16 KB per image
constexpr int QB = BQ * ROWB;        // 64 KB query block
constexpr int KPF = 2;               // K-fragment reads ahead of the product MFMAs
constexpr int VPF = 3;               // V^T fragment reads ahead of the dS V MFMAs

__device__ __attribute__((aligned(16))) unsigned g_zero16_bwd[4];

__device__ __forceinline__ void glds16b(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void blds16b(__amdgpu_buffer_rsrc_t r, unsigned voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base,
                                           16, (int)voff, 0, 0, 0);
}

__device__ __forceinline__ void raw_barrier_b() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ unsigned lds_addr_b(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N>
__device__ __forceinline__ void lgkm_wait_b(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

__device__ __forceinline__ bf16x8 pack8b(const float* f) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)f[j];
  return r;
}

struct BwdArgs {
  const bf16* vat; const bf16* va; const bf16* dza;   // query side (rows i)
  const bf16* vb; const bf16* dzb;                    // key side (rows j)
  long long ld_vat, ld_va, ld_dza, ld_vb, ld_dzb;
  const float* lse_a; const float* d0;                // per query row  [B][HWp] / [B][HW]
  const float* lse_b; const float* d1;                // per key        [B][HWp] (+inf padded), [B][HWp]
  bf16* out; long long ld_out;                        // dVa_t rows i
  int HW, HWp, nrb, nwork, accumulate;
  // key split (fewer row blocks than CUs): split s sums keys of tiles [s tps, (s+1) tps) into
  // fp32 partials part[s][B*HW][256]; dvat_sum_k adds them in split order
  int nsplit, tps;
  float* part;
};

// T0: the P0 (softmax over j) term, T1: the P1 (softmax over i) term.
template <bool T0, bool T1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void coatt_flash_dvat_k(BwdArgs a) {
  constexpr int NIMG = T1 ? 3 : 2;                 // Vb rows, Vb transposed, [dZb rows]
  constexpr int NST = T1 ? 2 : 3;                  // ring depth within the 160 KB of LDS
  constexpr int STG = NIMG * TILE;
  constexpr int FDMA = NIMG * TILE / 4096;         // LDS-DMA instructions per thread per tile
  __shared__ __attribute__((aligned(16))) char lds[QB + NST * STG];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int per_xcd = (a.nwork + 7) >> 3;
  const int work = (blockIdx.x & 7) * per_xcd + (blockIdx.x >> 3);
  if (work >= a.nwork) return;
  const int rb = work % a.nrb, rest = work / a.nrb;
  const int split = rest % a.nsplit;
  const long long b = rest / a.nsplit;
  const int HW = a.HW;
  const int q0 = rb * BQ;
  const int qrow = q0 + w * 32 + r;
  const bool qok = qrow < HW;
  const void* zp = (const void*)g_zero16_bwd;
  const float L2E = 1.4426950408889634f;

  // per-row scalars and the wave's query rows of dZa / Va as B fragments (16 k-steps of 16 d:
  // lane holds d = 16 ks + 8 h .. +7 of row qrow)
  float lsea = 0.f, dd0 = 0.f;
  bf16x8 q2[T0 ? 16 : 1], q3[T1 ? 16 : 1];
  if constexpr (T0) {
    lsea = qok ? a.lse_a[b * a.HWp + qrow] : 0.f;
    dd0 = qok ? a.d0[b * HW + qrow] : 0.f;
    const bf16* src = a.dza + (b * HW + (qok ? qrow : 0)) * a.ld_dza + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      q2[ks] = qok ? *(const bf16x8*)(src + 16 * ks) : bf16x8{};
  }
  if constexpr (T1) {
    const bf16* src = a.va + (b * HW + (qok ? qrow : 0)) * a.ld_va + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      q3[ks] = qok ? *(const bf16x8*)(src + 16 * ks) : bf16x8{};
  }

  // Va_t block DMA (row image: 16-B chunk position ^ (row & 15))
  const bf16* Q = a.vat + b * HW * a.ld_vat;
#pragma unroll
  for (int i = 0; i < QB / 4096; ++i) {
    const int p = i * 256 + tid;
    const int row = p >> 5, cpos = p & 31;
    const bool ok = q0 + row < HW;
    const bf16* src = Q + (long long)(q0 + row) * a.ld_vat + ((cpos ^ (row & 15)) << 3);
    glds16b(ok ? (const void*)src : zp, lds + (i * 256 + (tid & ~63)) * 16);
  }
  const bf16* KV = a.vb + b * HW * a.ld_vb;
  const bf16* K2 = T1 ? a.dzb + b * HW * a.ld_dzb : nullptr;
  // per tile: [Vb rows | Vb transposed | dZb rows], in buffer form: one resource per tile and
  // image (base = the tile's first row, range = the rows left: rows past HW land as zeros) and a
  // 32-bit lane offset -- cheaper to issue than global_load_lds with 64-bit lane addresses.
  // Piece i covers rows 8 i + (tid >> 5); the chunk swizzle row & 15 alternates with i's parity.
  const int ntiles = (HW + BK - 1) / BK;
  const int tb = split * a.tps;   // first key tile of this work item
  const unsigned ldb2 = (unsigned)a.ld_vb * 2, ld22 = T1 ? (unsigned)a.ld_dzb * 2 : 0u;
  const int lrow = tid >> 5, lpos = tid & 31;
  const unsigned ksw[2] = {(unsigned)((lpos ^ lrow) << 4), (unsigned)((lpos ^ (lrow + 8)) << 4)};
  const unsigned kof[2] = {lrow * ldb2 + ksw[0], lrow * ldb2 + ksw[1]};
  const unsigned vof = lrow * ldb2 + (unsigned)((lpos ^ ((lrow & 3) << 2)) << 4);
  const unsigned k2of[2] = {lrow * ld22 + ksw[0], lrow * ld22 + ksw[1]};
  auto issue = [&](int t, int stage) {
    char* kb = lds + QB + stage * STG;
    const int key0 = (tb + t) * BK;
    const int left = HW - key0;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<bf16*>(KV + (long long)key0 * a.ld_vb), 0, left * (int)ldb2, 0x00020000);
    __amdgpu_buffer_rsrc_t r2 = rk;
    if constexpr (T1)
      r2 = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(K2 + (long long)key0 * a.ld_dzb), 0,
                                             left * (int)ld22, 0x00020000);
#pragma unroll
    for (int i = 0; i < TILE / 4096; ++i) {
      const int wb = (i * 256 + (tid & ~63)) * 16;
      blds16b(rk, kof[i & 1] + 8 * i * ldb2, kb + wb);
      blds16b(rk, vof + 8 * i * ldb2, kb + TILE + wb);
      if constexpr (T1) blds16b(r2, k2of[i & 1] + 8 * i * ld22, kb + 2 * TILE + wb);
    }
  };

  const int nt = min(ntiles - tb, a.tps);
  issue(0, 0);
  if (NST > 2 && nt > 1) issue(1, 1);

  f32x16 o[8];
#pragma unroll
  for (int dt = 0; dt < 8; ++dt) o[dt] = f32x16{};

  const int sw = r & 15;
  const char* qrp = lds + (w * 32 + r) * ROWB;
  const int G = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;

  int st = 0;
  for (int t = 0; t < nt; ++t) {
    // tile t landed (NST 3: the DMA of tile t+1 may stay in flight)
    if (NST > 2 && t + 1 < nt) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(FDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    raw_barrier_b();
    // per-key normaliser and D1 of this tile (lane's keys 32t + 8q + 4h + 0..3), loaded BEFORE
    // the next DMA so their wait does not drain it
    f32x4 nk[4], nd[4];
    if constexpr (T1) {
      const int kt = tb + t;
      const float* kl = a.lse_b + b * a.HWp + kt * BK + 4 * h;
      const float* kd = a.d1 + b * a.HWp + kt * BK + 4 * h;
#pragma unroll
      for (int q = 0; q < 4; ++q) { nk[q] = *(const f32x4*)(kl + 8 * q); nd[q] = *(const f32x4*)(kd + 8 * q); }
      if ((kt + 1) * BK > HW) {  // D1's padding is not written: zero it (lse_b's is +inf)
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (kt * BK + 8 * q + 4 * h + j >= HW) nd[q][j] = 0.f;
      }
    }
    // the stage of tile t + NST - 1 was last read in iteration t-1, which every wave has passed
    if (t + NST - 1 < nt) issue(t + NST - 1, (st + NST - 1) % NST);
    const char* kb = lds + QB + st * STG;
    const char* vtb = kb + TILE;
    const char* k2b = kb + 2 * TILE;
    st = st + 1 == NST ? 0 : st + 1;

    // ---- S^T = Vb Va_t^T, dP0^T = Vb dZa^T, dP1^T = dZb Va^T (keys on registers, query on lane)
    f32x16 s = f32x16{}, p0 = f32x16{}, p1 = f32x16{};
    {
      const char* krp = kb + r * ROWB;
      const char* k2p = k2b + r * ROWB;
      bf16x8 kf[KPF], qf[KPF], k2f[T1 ? KPF : 1];
#pragma unroll
      for (int u = 0; u < KPF; ++u) {
        const int c = ((2 * u + h) ^ sw) << 4;
        kf[u] = *(const bf16x8*)(krp + c);
        qf[u] = *(const bf16x8*)(qrp + c);
        if constexpr (T1) k2f[u] = *(const bf16x8*)(k2p + c);
      }
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        const bf16x8 kc = kf[ks % KPF], qc = qf[ks % KPF];
        bf16x8 k2c;
        if constexpr (T1) k2c = k2f[ks % KPF];
        if (ks + KPF < 16) {
          const int c = ((2 * (ks + KPF) + h) ^ sw) << 4;
          kf[ks % KPF] = *(const bf16x8*)(krp + c);
          qf[ks % KPF] = *(const bf16x8*)(qrp + c);
          if constexpr (T1) k2f[ks % KPF] = *(const bf16x8*)(k2p + c);
        }
        s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, qc, s, 0, 0, 0);
        if constexpr (T0) p0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kc, q2[ks], p0, 0, 0, 0);
        if constexpr (T1) p1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(k2c, q3[ks], p1, 0, 0, 0);
      }
    }

    // ---- dS^T (register i: key 32t + (i&3) + 8(i>>2) + 4h) -> bf16 B operand.  Keys past HW
    // have zero Vb rows in the transposed image, so whatever dS they get contributes nothing.
    bf16x8 pf[2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      float dv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int i = 8 * s2 + j;
        float x = 0.f;
        if constexpr (T0) x = __builtin_amdgcn_exp2f(fmaf(s[i], L2E, -lsea)) * (p0[i] - dd0);
        if constexpr (T1)
          x = fmaf(__builtin_amdgcn_exp2f(fmaf(s[i], L2E, -nk[i >> 2][i & 3])), p1[i] - nd[i >> 2][i & 3], x);
        dv[j] = x;
      }
      pf[s2] = pack8b(dv);
    }

    // ---- dVa_t^T += Vb^T dS^T over the tile's 32 keys (as the forward's O^T += V^T P^T)
    {
      const unsigned vrow = lds_addr_b(vtb + (4 * h + q4) * ROWB);
      auto vread = [&](int dt, int sk) {
        const int g = 8 * dt + 4 * (G & 1) + pp;
        const unsigned a1 = vrow + 16 * sk * ROWB + ((g ^ (q4 << 3)) << 3);
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(a1));
        asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(8 * ROWB));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      bf16x8 vf[VPF];
#pragma unroll
      for (int u = 0; u < VPF; ++u) vf[u] = vread(u >> 1, u & 1);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        bf16x8 cur = vf[it % VPF];
        if (it + VPF < 16) vf[it % VPF] = vread((it + VPF) >> 1, (it + VPF) & 1);
        const int younger = 2 * (15 - it < VPF ? 15 - it : VPF);
        if (younger >= 6) lgkm_wait_b<6>(cur);
        else if (younger == 4) lgkm_wait_b<4>(cur);
        else if (younger == 2) lgkm_wait_b<2>(cur);
        else lgkm_wait_b<0>(cur);
        o[it >> 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(cur, pf[it & 1], o[it >> 1], 0, 0, 0);
      }
    }
  }

  // ---- epilogue: dVa_t[qrow][d]; register i of d tile dt holds d = 32 dt + (i&3) + 8(i>>2) + 4h
  if (qok && a.nsplit > 1) {   // fp32 partial of this key split
    float* op = a.part + (((long long)split * (a.nwork / (a.nrb * a.nsplit)) + b) * HW + qrow) * BD + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        *(f32x4*)(op + 32 * dt + 8 * c) = f32x4{o[dt][4 * c], o[dt][4 * c + 1], o[dt][4 * c + 2], o[dt][4 * c + 3]};
  } else if (qok) {
    bf16* op = a.out + (b * HW + qrow) * a.ld_out + 4 * h;
#pragma unroll
    for (int dt = 0; dt < 8; ++dt)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
        bf16x4 v;
        if (a.accumulate) {
          const bf16x4 old = *(const bf16x4*)(op + 32 * dt + 8 * c);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][4 * c + j] + (float)old[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)o[dt][4 * c + j];
        }
        *(bf16x4*)(op + 32 * dt + 8 * c) = v;
      }
  }
}

// out[row][c..c+7] (+)= sum_s part[s][row][c..c+7], splits in order.  One thread = 8 channels.
__global__ __launch_bounds__(256) void dvat_sum_k(const float* __restrict__ part, int nsplit, long long rows,
                                                  bf16* out, long long ld_out, int accumulate) {
  const long long t = blockIdx.x * 256ll + threadIdx.x;
  if (t >= rows * (BD / 8)) return;
  const long long row = t / (BD / 8);
  const int c0 = (int)(t % (BD / 8)) * 8;
  float acc[8];
  bf16* op = out + row * ld_out + c0;
  if (accumulate) {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = (float)op[e];
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
  }
  for (int s = 0; s < nsplit; ++s) {
    const float* p = part + ((long long)s * rows + row) * BD + c0;
    const f32x4 v0 = *(const f32x4*)p, v1 = *(const f32x4*)(p + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { acc[e] += v0[e]; acc[4 + e] += v1[e]; }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) op[e] = (bf16)acc[e];
}

bool al16(const void* p) { return ((uintptr_t)p & 15) == 0; }

// Key splits for `items` workgroups when they leave CUs idle (one workgroup per CU): up to
// 256 / items splits of >= 16 key tiles each.
int bwd_nsplit(int items, int ntiles) {
  if (items >= 256) return 1;
  int s = 256 / items;
  if (s > 8) s = 8;
  while (s > 1 && ntiles / s < 16) --s;
  return s;
}

}  // namespace

extern "C" size_t cn_coatt_flash_bwd_workspace_bytes(int B, int HW) {
  const int s = bwd_nsplit(((HW + BQ - 1) / BQ) * B, (HW + BK - 1) / BK);
  return s > 1 ? (size_t)s * B * HW * BD * sizeof(float) : 0;
}

extern "C" int cn_coatt_flash_dvat_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                      const void* dza, long long ld_dza, const void* vb, long long ld_vb,
                                      const void* dzb, long long ld_dzb, const float* lse_a,
                                      const float* d0, const float* lse_b, const float* d1, int B,
                                      int HW, int C, void* out, long long ld_out, int accumulate,
                                      void* ws, size_t ws_bytes, hipStream_t st);

extern "C" int cn_coatt_flash_dvat(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                   const void* dza, long long ld_dza, const void* vb, long long ld_vb,
                                   const void* dzb, long long ld_dzb, const float* lse_a,
                                   const float* d0, const float* lse_b, const float* d1, int B,
                                   int HW, int C, void* out, long long ld_out, int accumulate,
                                   hipStream_t st) {
  return cn_coatt_flash_dvat_ws(vat, ld_vat, va, ld_va, dza, ld_dza, vb, ld_vb, dzb, ld_dzb, lse_a,
                                d0, lse_b, d1, B, HW, C, out, ld_out, accumulate, nullptr, 0, st);
}

extern "C" int cn_coatt_flash_dvat_ws(const void* vat, long long ld_vat, const void* va, long long ld_va,
                                      const void* dza, long long ld_dza, const void* vb, long long ld_vb,
                                      const void* dzb, long long ld_dzb, const float* lse_a,
                                      const float* d0, const float* lse_b, const float* d1, int B,
                                      int HW, int C, void* out, long long ld_out, int accumulate,
                                      void* ws, size_t ws_bytes, hipStream_t st) {
  if (C != BD || B <= 0 || HW <= 0 || !out) return CN_ERR_SHAPE;
  const bool t0 = dza != nullptr, t1 = dzb != nullptr;
  if (!t0 && !t1) return CN_ERR_SHAPE;
  if ((t0 && (!lse_a || !d0)) || (t1 && (!lse_b || !d1 || !va))) return CN_ERR_SHAPE;
  for (long long ld : {ld_vat, ld_vb, t0 ? ld_dza : (long long)C, t1 ? ld_dzb : (long long)C, t1 ? ld_va : (long long)C})
    if (ld % 8 || ld < C) return CN_ERR_ALIGN;
  if (ld_out % 4 || ld_out < C) return CN_ERR_ALIGN;
  if (!al16(vat) || !al16(vb) || (t0 && !al16(dza)) || (t1 && (!al16(dzb) || !al16(va) || !al16(lse_b) || !al16(d1))) ||
      ((uintptr_t)out & 7))
    return CN_ERR_ALIGN;
  BwdArgs a;
  a.vat = (const bf16*)vat; a.va = (const bf16*)va; a.dza = (const bf16*)dza;
  a.vb = (const bf16*)vb; a.dzb = (const bf16*)dzb;
  a.ld_vat = ld_vat; a.ld_va = ld_va; a.ld_dza = ld_dza; a.ld_vb = ld_vb; a.ld_dzb = ld_dzb;
  a.lse_a = lse_a; a.d0 = d0; a.lse_b = lse_b; a.d1 = d1;
  a.out = (bf16*)out; a.ld_out = ld_out;
  a.HW = HW; a.HWp = (HW + 31) / 32 * 32;
  a.nrb = (HW + BQ - 1) / BQ;
  const int ntiles = (HW + BK - 1) / BK;
  a.nsplit = bwd_nsplit(a.nrb * B, ntiles);
  // the split sum writes 16-byte rows; without a workspace run unsplit
  const size_t need = (size_t)a.nsplit * B * HW * BD * sizeof(float);
  if (a.nsplit > 1 && (!ws || ws_bytes < need || !al16(ws) || ((uintptr_t)out & 15) || ld_out % 8))
    a.nsplit = 1;
  a.tps = (ntiles + a.nsplit - 1) / a.nsplit;
  a.part = (float*)ws;
  a.nwork = a.nrb * B * a.nsplit;
  a.accumulate = accumulate;
  dim3 grid(((a.nwork + 7) / 8) * 8);
  if (t0 && t1) hipLaunchKernelGGL((coatt_flash_dvat_k<true, true>), grid, dim3(256), 0, st, a);
  else if (t0) hipLaunchKernelGGL((coatt_flash_dvat_k<true, false>), grid, dim3(256), 0, st, a);
  else hipLaunchKernelGGL((coatt_flash_dvat_k<false, true>), grid, dim3(256), 0, st, a);
  CN_CHECK_LAUNCH();
  if (a.nsplit > 1) {
    const long long rows = (long long)B * HW;
    hipLaunchKernelGGL(dvat_sum_k, dim3((unsigned)((rows * (BD / 8) + 255) / 256)), dim3(256), 0, st,
                       (const float*)ws, a.nsplit, rows, (bf16*)out, ld_out, accumulate);
    CN_CHECK_LAUNCH();
  }
  return 0;
}
