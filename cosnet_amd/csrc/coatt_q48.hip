// Flash co-attention forward / PV with 48 query rows per wave on 16x16x32 MFMA tiles
// (kernel variant 5; rgbd_segmentation_RAA.py:160-170, :213-221).
//
//   MODE 0:  O[q] = sum_k softmax_k(Q[q].K[k]) V[k]                    (+ log2-sum-exp2 per row)
//   MODE 1:  O[q] (+)= sum_k exp2(Q[q].K[k] log2e - klse[k]) V[k]      (the backward's P_row dZ_b)
//
// The 32-row kernel (coatt_fused_fwd_k) reads, per 32-key tile and wave, the whole K tile, the
// whole V tile and its 32 Q rows from LDS and issues a quarter of the tile's LDS-DMA pieces for
// 32 MFMAs of 32x32x16; its measured bounds are exactly those.  A 64-row wave would
// halve them but does not fit the register file at D = 256 (profiles/r05_coatt_q64_isa.txt).  Here
// a wave owns 48 query rows = three 16-row tiles, with their Q fragments in REGISTERS (96 VGPRs):
// every K fragment read feeds three S MFMAs and every V^T fragment three PV MFMAs, no Q is read
// from LDS, and the tile's DMA pieces are spread over 96 MFMAs (16x16x32) instead of 32 (32x32x16)
// -- per FLOP a third of the K / V reads and of the DMA issue, no Q reads.  Accumulators: O = 16
// channel tiles x 3 row tiles x 4 = 192 registers, S^T = 2 key tiles x 3 row tiles x 4 = 24, both
// within the 256 accumulation registers.
//
// Operand maps (16x16x32 bf16 MFMA: A lane l = row (l & 15), k = 8 (l >> 4) + j; B lane l =
// column (l & 15), same k; C lane l = rows 4 (l >> 4) + i, column l & 15):
//   S^T[key][q] = K Q^T: A = K (16 keys x 32 channels, a ds_read_b128 of the K image), B = Q.
//   The S^T accumulators of the tile's two 16-key halves leave lane (q = l & 15, g = l >> 4) the
//   keys {4g + i, 16 + 4g + i}: packed to bf16 in that order they ARE the B operand of
//   O^T[d][q] += V^T P^T with k slot 8g + j <-> key (j < 4 ? 4g + j : 16 + 4g + j - 4), and the A
//   operand V^T takes the same order from two ds_read_b64_tr_b16 (keys 4g..4g+3 and 16+4g..+3,
//   lane i receiving channel i of the 16-channel tile).
// Work split (stream-K): 48-row waves leave a 4-wave workgroup 192 query rows, so a 60 x 60 map
// of 5 pairs x 2 directions is 190 such items -- 74 % of 256 CUs for one round, 59 % at 4 pairs.
// Instead the items' key tiles are laid end to end (item-major) and cut into nwork equal ranges,
// one workgroup each (nwork = 256: every CU busy for the same number of tile steps).  A range
// covering a whole item writes its output directly; a segment of a cut item writes its
// un-normalised fp32 O and per-row (reference, sum) to the item's partial slot and bumps the
// item's arrival counter; the LAST segment to arrive (no workgroup ever waits for another, so no
// co-residency is assumed) merges the item's slots in segment order and writes the output.
// The merge order is fixed (slots 0, 1, ...), so results do not depend on arrival order.
// LDS images (one 3-stage ring, 2 x 16 KB per stage) are FRAGMENT-MAJOR: the K image is 16
// blocks of 1 KB, block 2 ds + kt holding at lane slot L the 16 bytes lane L feeds the MFMA
// (key 16 kt + (L & 15), channels 32 ds + 8 (L >> 4) ..); the V image is 32 blocks of 512 B,
// block (dt, hi) at (dt >> 1) 2048 + (dt & 1) 512 + hi 1024 holding at 8-byte slot L what lane L
// addresses in its transposed read.  Every fragment read is then one contiguous block at (lane
// base + immediate offset): no swizzle arithmetic in the loop.  The LDS-DMA fills them with
// 16-byte chunks gathered from 16 key rows per 1-KB piece.  Where K = V (the Z_a direction: both
// Vb) the V^T reads address the K image at the same immediates and no V image is loaded.
#include "common.h"
#include "coatt_fused.h"
#include <algorithm>
#include <type_traits>
#include "../../include/cosnet_hip.h"

namespace {

constexpr int RW = 48;                 // query rows per wave (3 tiles of 16)
constexpr int RB = 4 * RW;             // query rows per workgroup (4 waves)
constexpr int Q48ST = 3;               // K / V ring stages
// Bound on a lane's partial softmax sum under the first tile's reference: every P it added is
// <= 2^100 (bf16 max ~2^128) and the fp32 O sums <= HW 2^100 |V| -- 2^15 of headroom for
// |V| x HW / 4096; an overflow to inf also fails it.  The training step's own features
// (tools/probes/q48_step_inputs.py) grow by 42 (median) / 71 (p99) / 92 (max) log2 units over the
// first tile, so no workgroup redoes its keys on them.
constexpr float Q48_LMAX = 0x1p100f;

// Development timing (make EXTRA_Q48=-DQ48_PROF=1 style builds only): per-phase shader-clock sums
// of every wave -- [0] DMA wait + barrier, [1] S MFMAs issued, [2] softmax, [3] PV, [4] tiles.
#ifndef Q48_PROF
#define Q48_PROF 0
#endif
#if Q48_PROF
__device__ unsigned long long g_q48_prof[8];
#define Q48_STAMP(k)                                                                          \
  do {                                                                                        \
    unsigned long long t_;                                                                    \
    asm volatile("s_memtime %0\n s_waitcnt lgkmcnt(0)" : "=s"(t_) :: "memory");             \
    if (k) prof_[(k) - 1] += t_ - prev_;                                                      \
    prev_ = t_;                                                                               \
  } while (0)
#else
#define Q48_STAMP(k) do {} while (0)
#endif

__device__ __forceinline__ void blds16q(__amdgpu_buffer_rsrc_t r, unsigned voff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base,
                                           16, (int)voff, 0, 0, 0);
}

// maximum over the four 16-lane groups holding one row's keys: VALU row swaps (no LDS round trip)
__device__ __forceinline__ float row_max_r(float x) {
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

__device__ __forceinline__ void raw_barrier_r() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Partial rows cross workgroups (and XCDs, each with its own L2): written through to memory and
// read past the L2 (cache policy sc0 sc1, system coherence) instead of device-wide fences, which
// write back and invalidate the whole L2 -- the K / V stream the XCD's other workgroups share.
constexpr int CP_SYS = 1 | 16;   // sc0 | sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t part_rsrc(const float* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), 0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ unsigned lds_addr_r(const void* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N>
__device__ __forceinline__ void lgkm_wait_r(bf16x8& v) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(v) : "n"(N));
}

// The workgroup whose range holds key-tile step u of the item-major list (ranges [w U / G,
// (w+1) U / G), U = nitems x ntiles, G = nwork): the largest w with floor(w U / G) <= u.
__device__ __forceinline__ int q48_owner(long long u, long long U, int G) {
  return (int)(((u + 1) * G + U - 1) / U) - 1;
}

// One segment: key tiles [tb, tb + nt) of `item`; `slot` < 0: the whole item, output directly,
// else the partial slot it writes.
template <int MODE>
__device__ __forceinline__ void q48_segment(const FusedArgs& a, char* lds, int* wg_ovf, int item,
                                            int tb, int nt, int slot) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int col = lane & 15, g = lane >> 4;
  const bool part = slot >= 0;
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const int HW = a.HW;
  const long long b = bd / a.ndir;
  const bf16* Q = d.q + b * HW * d.ldq;
  const bf16* K = d.k + b * HW * d.ldk;
  const bf16* V = d.v + b * HW * d.ldv;
  const int qw0 = rb * RB + w * RW;          // this wave's first query row
#if Q48_PROF
  unsigned long long prof_[5] = {0, 0, 0, 0, 0}, prev_ = 0;
#endif

  // LDS-DMA: piece i of a tile is, for wave w, block index kbi = 4 i + w of both images.
  // Both images have one layout: block kbi = 2 m + h (m = channel block of 32, h = key half of 16)
  // holds at 16-byte lane slot L = (c = (L >> 1) & 15, j = 2 (L >> 5) + (L & 1))
  //   X[key0 + 16 h + c][32 m + 8 j .. +8]        (X = K or V)
  // so K's S-fragment (kt, ds) is block 2 ds + kt and V's transposed-read block (dt, hi) is at
  // (dt >> 1) 2048 + (dt & 1) 512 + hi 1024 -- read at lane * 8 from either image (K = V: the
  // K image, below).
  // A lane's global offset is a tile-invariant per-lane part plus a uniform part.
  const unsigned ldk2 = (unsigned)d.ldk * 2, ldv2 = (unsigned)d.ldv * 2;
  const int vkey = (lane >> 1) & 15;   // + 16 h
  // The K image has the V image's layout: slot L holds key (L >> 1) & 15, channel group
  // 2 (L >> 5) + (L & 1).  The S reads (lane = key col, group g) then take slot
  // 32 (g >> 1) + 2 col + (g & 1) -- conflict-free in the ds_read_b128 lane groups
  // {0-3,12-15,20-27} / {4-11,16-19,28-31} -- and, when K = V, the V^T reads are the V image's
  // own lane * 8 pattern on the K image
  const int kcol = (lane >> 1) & 15;
  const unsigned koff = kcol * ldk2 + (2 * (lane >> 5) + (lane & 1)) * 16;
  const unsigned voff = vkey * ldv2 + (2 * (lane >> 5) + (lane & 1)) * 16;
  const int wq = __builtin_amdgcn_readfirstlane(w);
  // Z_a's direction has K = V = Vb: its V^T fragments are read from the K image and no V image is
  // loaded -- half the global / L2 traffic of those tiles' LDS-DMA
  const bool kvs = d.v == d.k && d.ldv == d.ldk;
  // one buffer resource per tile (uniform) plus a 32-bit per-lane offset: the buffer form issues
  // cheaper than global_load_lds with 64-bit lane addresses (PV phase 1620 -> 1452 clocks per
  // wave-tile); the piece's block offset is folded into the per-lane offset
  auto issue_piece = [&](int t, int stage, int i) {
    const int kbi = 4 * i + wq;
    char* kb = lds + stage * 2 * FTILE + kbi * 1024;
    char* vb = lds + stage * 2 * FTILE + FTILE + kbi * 1024;
    const int key0 = (tb + t) * FBK;
    const char* kt = (const char*)K + (size_t)((unsigned)key0 * ldk2);
    // buffer-form LDS-DMA: the tile's rows as one buffer resource (base = the tile's first row,
    // range = the rows left), a 32-bit per-lane offset -- rows past HW are out of range and land
    // as zeros (no partial-tile branch); K = V: the V resource is empty (all zeros, no fetch),
    // so the DMA issue stays branch-free and interleaved with the PV MFMAs
    const int left = HW - key0;
    const __amdgpu_buffer_rsrc_t rk = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(kt), 0, left * (int)ldk2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(kvs ? kt : (const char*)V + (size_t)((unsigned)key0 * ldv2)), 0,
        kvs ? 0 : left * (int)ldv2, 0x00020000);
    const unsigned ko = koff + (unsigned)(16 * (kbi & 1)) * ldk2 + (kbi >> 1) * 64;
    const unsigned vo = voff + (unsigned)(16 * (kbi & 1)) * ldv2 + (kbi >> 1) * 64;
    blds16q(rk, ko, kb);
    blds16q(rv, vo, vb);
  };
  auto issue = [&](int t, int stage) {
#pragma unroll
    for (int i = 0; i < FTILE / 4096; ++i) issue_piece(t, stage, i);
  };

  // Q fragments (B operand of S^T = K Q^T), straight from global memory, issued before the K / V
  // prologue (older than every DMA piece, so the loop's counted waits cover them):
  // qf[qt][ds] = Q[qw0 + 16 qt + col][32 ds + 8 g .. +8]  (rows past HW: zero)
  bf16x8 qf[3][8];
#pragma unroll
  for (int qt = 0; qt < 3; ++qt) {
    const int row = qw0 + 16 * qt + col;
    const bf16* qp = Q + (long long)(row < HW ? row : 0) * d.ldq + 8 * g;
#pragma unroll
    for (int ds = 0; ds < 8; ++ds) qf[qt][ds] = *(const bf16x8*)(qp + 32 * ds);
    if (row >= HW) {
#pragma unroll
      for (int ds = 0; ds < 8; ++ds) qf[qt][ds] = bf16x8{};
    }
  }
  f32x4 o[16][3];
  float m[3] = {-INFINITY, -INFINITY, -INFINITY};
  float mt[3] = {-INFINITY, -INFINITY, -INFINITY};   // running maxima (pass 0)
  __attribute__((ext_vector_type(2))) float l[3];   // per-lane partial sums (pairs)
  bool ovf = false;
  const float L2E = 1.4426950408889634f;

  // pass 0: reference = each row's maximum over its first tile; only when a lane's partial sum
  // ends above Q48_LMAX (a logit outgrew the reference; an overflow lands there as inf) does the
  // workgroup run pass 2 (S only: the exact row maxima) and pass 1 (again, with those maxima)
  auto run = [&](auto passc) {
  constexpr int pass = decltype(passc)::value;
  if (pass == 1) {
#pragma unroll
    for (int qt = 0; qt < 3; ++qt) m[qt] = row_max_r(mt[qt]);   // the lanes' maxima, per row
  }
#pragma unroll
  for (int dt = 0; dt < 16; ++dt)
#pragma unroll
    for (int qt = 0; qt < 3; ++qt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int qt = 0; qt < 3; ++qt) l[qt] = 0.f;
  issue(0, 0);
  if (nt > 1) issue(1, 1);

  int st = 0, st2 = 2;
  bf16x8 vlast1 = {}, vlast2 = {};   // the last two V fragments handed to MFMAs
  for (int t = 0; t < nt; ++t) {
    Q48_STAMP(0);
    if (t + 1 < nt) {   // tile t landed, tile t+1 (4 or 8 pieces per thread) may be in flight
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * FTILE / 4096) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    raw_barrier_r();
    Q48_STAMP(1);
    const bool dodma = t + 2 < nt;
    const int dst2 = st2;
    const char* kb = lds + st * 2 * FTILE;
    st = st == Q48ST - 1 ? 0 : st + 1;
    st2 = st2 == Q48ST - 1 ? 0 : st2 + 1;
    const char* vb = kb + FTILE;
    const int key0 = (tb + t) * FBK;
    // the fragment-major images: every fragment read is this lane's slot of one contiguous block
    // V^T read base: lane * 8 in the V image, or (K = V) in the K image, which is laid out alike
    const unsigned kla = lds_addr_r(kb) + (32 * (g >> 1) + 2 * col + (g & 1)) * 16;
    const unsigned vla = lds_addr_r(kvs ? kb : vb) + lane * 8;

    // MODE 1: the per-key normalisers of the lane's 8 keys {4g + i, 16 + 4g + i}
    f32x4 nk[2];
    if constexpr (MODE == 1) {
      const float* kl = d.klse + b * a.HWp + key0 + 4 * g;
      nk[0] = *(const f32x4*)kl;
      nk[1] = *(const f32x4*)(kl + 16);
    }
    // ---- S^T tiles: s[kt][qt] = K[16 kt .. +16] Q[16 qt .. +16]^T over 8 channel steps of 32
    f32x4 s[2][3];
#pragma unroll
    for (int kt = 0; kt < 2; ++kt)
#pragma unroll
      for (int qt = 0; qt < 3; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
    {
      // K fragment (A): key 16 kt + col, channels 32 ds + 8 g .. +8 = block 2 ds + kt, swizzled slot.
      // The fragment loads are inline asm with early-clobber outputs that also take the two
      // fragments consumed last as inputs: an MFMA queued behind its predecessors reads its A / B
      // registers when it starts, not when it issues, and an LDS load returning into those
      // registers before that corrupts it (seen as wrong S on the third row tile when the
      // compiler reloaded a register right behind the MFMA that read it).  Waits are counted here.
      auto kread = [&](int kt, int ds, const bf16x8& g0, const bf16x8& g1) {
        bf16x8 r;
        asm volatile("ds_read_b128 %0, %1 offset:%2"
                     : "=&v"(r) : "v"(kla), "n"((2 * ds + kt) * 1024), "v"(g0), "v"(g1));
        return r;
      };
      bf16x8 kf[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) kf[u] = kread(u & 1, u >> 1, vlast1, vlast2);
      bf16x8 kprev = vlast1, kprev2 = vlast2;
#pragma unroll
      for (int it = 0; it < 16; ++it) {          // it = 2 ds + kt
        const int kt = it & 1, ds = it >> 1;
        bf16x8 kc = kf[it & 3];
        if (it + 4 < 16) kf[it & 3] = kread((it + 4) & 1, (it + 4) >> 1, kprev, kprev2);
        const int younger = 15 - it < 4 ? 15 - it : 4;
        if (younger == 4) lgkm_wait_r<4>(kc);
        else if (younger == 3) lgkm_wait_r<3>(kc);
        else if (younger == 2) lgkm_wait_r<2>(kc);
        else if (younger == 1) lgkm_wait_r<1>(kc);
        else lgkm_wait_r<0>(kc);
#pragma unroll
        for (int qt = 0; qt < 3; ++qt)
          s[kt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kc, qf[qt][ds], s[kt][qt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);   // this step's MFMAs stay ahead of the next loads
        kprev2 = kprev;
        kprev = kc;
      }
    }

    Q48_STAMP(2);
    // ---- softmax per row tile: the lane's row q = 16 qt + col, its keys {4g + i, 16 + 4g + i}
    // (pairs of values in packed fp32 FMAs / adds; the partial last tile's key mask as its own
    // copy of the code, not selects on every tile)
    typedef __attribute__((ext_vector_type(2))) float f32x2;
    bf16x8 pf[3];
    auto soft = [&](auto qtc, auto maskc) {
      constexpr int qt = decltype(qtc)::value;
      constexpr bool MASK = decltype(maskc)::value;
      f32x2 v[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        v[i] = f32x2{s[0][qt][2 * i], s[0][qt][2 * i + 1]};
        v[2 + i] = f32x2{s[1][qt][2 * i], s[1][qt][2 * i + 1]};
      }
      const f32x2 l2e = {L2E, L2E};
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x2 nkp = {nk[i >> 1][2 * (i & 1)], nk[i >> 1][2 * (i & 1) + 1]};
          v[i] = v[i] * l2e - nkp;
          v[i] = f32x2{__builtin_amdgcn_exp2f(v[i].x), __builtin_amdgcn_exp2f(v[i].y)};
        }
      } else {
        if constexpr (MASK) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (key0 + (j < 4 ? 4 * g + j : 16 + 4 * g + j - 4) >= HW) v[j >> 1][j & 1] = -INFINITY;
        }
        // fixed reference: the row's maximum over its first key tile (O is still zero there, so
        // nothing is rescaled); later tiles are not checked one by one -- the lanes' partial sums
        // bound every P they added, and a sum above Q48_LMAX at the end makes the workgroup redo
        // its keys.  Pass 2 only tracks this lane's running maximum.
        auto lane_max = [&]() {
          return fmaxf(fmaxf(fmaxf(v[0].x, v[0].y), fmaxf(v[1].x, v[1].y)),
                       fmaxf(fmaxf(v[2].x, v[2].y), fmaxf(v[3].x, v[3].y)));
        };
        if constexpr (pass == 0) {
          if (t == 0) m[qt] = row_max_r(lane_max()) * L2E;
        } else if constexpr (pass == 2) {
          mt[qt] = fmaxf(mt[qt], lane_max() * L2E);
          return;
        }
        const f32x2 nm = {-m[qt], -m[qt]};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[i] = v[i] * l2e + nm;
          v[i] = f32x2{__builtin_amdgcn_exp2f(v[i].x), __builtin_amdgcn_exp2f(v[i].y)};
        }
        l[qt] += (v[0] + v[1]) + (v[2] + v[3]);
      }
      bf16x8 r;
#pragma unroll
      for (int j = 0; j < 8; ++j) r[j] = (bf16)v[j >> 1][j & 1];
      pf[qt] = r;
    };
    if (MODE == 0 && key0 + FBK > HW) {
      soft(std::integral_constant<int, 0>{}, std::true_type{});
      soft(std::integral_constant<int, 1>{}, std::true_type{});
      soft(std::integral_constant<int, 2>{}, std::true_type{});
    } else {
      soft(std::integral_constant<int, 0>{}, std::false_type{});
      soft(std::integral_constant<int, 1>{}, std::false_type{});
      soft(std::integral_constant<int, 2>{}, std::false_type{});
    }

    Q48_STAMP(3);
    // ---- O^T[16 dt .. +16][q] += V^T P^T: the V^T fragment (A) of channel tile dt in the k order
    // of P: two transposed reads, keys 4g .. 4g+3 and 16 + 4g .. +3; lane 4q4 + p4 of a 16-lane
    // group addresses key row (base + q4), channels 16 dt + 4 p4 .. +3 (8 bytes)
    if constexpr (pass == 2) {   // S only: tile t + 2's DMA pieces, no PV
      if (dodma) {
#pragma unroll
        for (int i = 0; i < FTILE / 4096; ++i) issue_piece(t + 2, dst2, i);
      }
    } else {
      // block (dt, hi) holds, at lane 16 G + 4 q4 + p4, V[16 hi + 4 G + q4][16 dt + 4 p4 .. +3]
      // (loads guarded as the K fragments': never into the registers of the last two fragments)
      auto vread = [&](int dt, const bf16x8& g0, const bf16x8& g1) {
        u32x2 lo, hi;
        asm volatile("ds_read_b64_tr_b16 %0, %2 offset:%3\n\tds_read_b64_tr_b16 %1, %2 offset:%4"
                     : "=&v"(lo), "=&v"(hi)
                     : "v"(vla), "n"((dt >> 1) * 2048 + (dt & 1) * 512),
                       "n"((dt >> 1) * 2048 + (dt & 1) * 512 + 1024), "v"(g0), "v"(g1));
        u32x4 v = {lo.x, lo.y, hi.x, hi.y};
        return __builtin_bit_cast(bf16x8, v);
      };
      constexpr int VPF = 5;
      bf16x8 vf[VPF];
#pragma unroll
      for (int u = 0; u < VPF; ++u) vf[u] = vread(u, vlast1, vlast2);
      bf16x8 vprev = vlast1, vprev2 = vlast2;
#pragma unroll
      for (int dt = 0; dt < 16; ++dt) {
        bf16x8 cur = vf[dt % VPF];
        if (dt + VPF < 16) vf[dt % VPF] = vread(dt + VPF, vprev, vprev2);
        const int younger = 2 * (15 - dt < VPF ? 15 - dt : VPF);
        if (younger >= 10) lgkm_wait_r<10>(cur);
        else if (younger == 8) lgkm_wait_r<8>(cur);
        else if (younger == 6) lgkm_wait_r<6>(cur);
        else if (younger == 4) lgkm_wait_r<4>(cur);
        else if (younger == 2) lgkm_wait_r<2>(cur);
        else lgkm_wait_r<0>(cur);
#pragma unroll
        for (int qt = 0; qt < 3; ++qt)
          o[dt][qt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(cur, pf[qt], o[dt][qt], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        vprev2 = vprev;
        vprev = cur;
        if ((dt & 3) == 3 && dodma) issue_piece(t + 2, dst2, dt >> 2);
      }
      vlast1 = vprev;    // the next tile's K loads stay clear of these
      vlast2 = vprev2;
    }
    Q48_STAMP(4);
#if Q48_PROF
    prof_[4] += 1;
#endif
  }
  };
  run(std::integral_constant<int, 0>{});
  if constexpr (MODE == 0) {
    // any lane's partial sum past Q48_LMAX in the workgroup?  (the barrier also retires every
    // wave's reads of the ring before the redo's DMA refills it)
#pragma unroll
    for (int qt = 0; qt < 3; ++qt) ovf |= fmaxf(l[qt].x, l[qt].y) > Q48_LMAX;
    const bool wave_ovf = __builtin_amdgcn_ballot_w64(ovf) != 0;   // all lanes vote
    if (lane == 0) wg_ovf[w] = wave_ovf;
    raw_barrier_r();
    if (wg_ovf[0] | wg_ovf[1] | wg_ovf[2] | wg_ovf[3]) {
#if Q48_PROF
      if (tid == 0) atomicAdd(&g_q48_prof[5], 1ull);
#endif
      run(std::integral_constant<int, 2>{});   // the exact row maxima
      raw_barrier_r();                          // every wave done with the ring before the refill
      run(std::integral_constant<int, 1>{});
    }
  }

  // ---- epilogue: o[dt][qt][i] = O^T[16 dt + 4 g + i][16 qt + col]
#pragma unroll
  for (int qt = 0; qt < 3; ++qt) {
    float lt = l[qt].x + l[qt].y;
    lt += __shfl_xor(lt, 16, 64);
    lt += __shfl_xor(lt, 32, 64);
    const int qrow = qw0 + 16 * qt + col;
    if (part) {
      if (qrow < HW) {
        const unsigned prow = (unsigned)slot * RB + (unsigned)(qrow - rb * RB);
        const __amdgpu_buffer_rsrc_t ro = part_rsrc(a.opart);
        // partial O in bf16 (half the write-through bytes; the merge folds <= 8 slots in fp32),
        // 16-byte chunk 4 p + g of the row = channels 32 p + 4 g .. +3 and 32 p + 16 + 4 g .. +3
        // (one dwordx4 store per channel-tile pair)
#pragma unroll
        for (int pp = 0; pp < 8; ++pp) {
          bf16x8 h;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            h[j] = (bf16)o[2 * pp][qt][j];
            h[4 + j] = (bf16)o[2 * pp + 1][qt][j];
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(f32x4, h), ro,
                                                 (prow * FD + 8 * (4 * pp + g)) * 2, 0, CP_SYS);
        }
        if (MODE == 0 && g == 0) {
          typedef __attribute__((ext_vector_type(2))) float f32x2;
          __builtin_amdgcn_raw_buffer_store_b64(f32x2{m[qt], lt}, part_rsrc(a.mlpart), prow * 8, 0, CP_SYS);
        }
      }
      continue;
    }
    if (MODE == 0 && d.lse && g == 0 && qrow < a.HWp)
      d.lse[b * a.HWp + qrow] = qrow < HW ? m[qt] + __builtin_amdgcn_logf(lt) : INFINITY;
    if (qrow < HW) {
      const float inv = MODE == 0 ? 1.f / lt : 1.f;
      bf16* op = d.o + (b * HW + qrow) * d.ldo + 4 * g;
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
#pragma unroll
      for (int dt = 0; dt < 16; ++dt) {
        bf16x4 v;
        if (a.accumulate) {
          const bf16x4 old = *(const bf16x4*)(op + 16 * dt);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][qt][j] * inv + (float)old[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[j] = (bf16)(o[dt][qt][j] * inv);
        }
        *(bf16x4*)(op + 16 * dt) = v;
      }
    }
  }
#if Q48_PROF
  if (lane == 0)
    for (int k = 0; k < 5; ++k) atomicAdd(&g_q48_prof[k], prof_[k]);
#endif
}

// Merge of a cut item (by its last-arriving segment): slots slot0 .. slot0 + nseg - 1 in order,
// an online (max, sum) fold per row.  A thread owns MB (row, 8-channel) chunks at once and issues
// the loads of one slot for all of them together: nseg x 2 round trips to memory per thread, not
// one per chunk and slot (the partial rows are read past the L2, ~1-2 us each).
template <int MODE>
__device__ __forceinline__ void q48_merge(const FusedArgs& a, int item, int nseg, int slot0) {
  constexpr int MB = 6;                                   // chunks per thread and batch
  constexpr int NCH = RB * (FD / 8);                      // 6144 chunks = 4 batches of 256 x 6
  static_assert(NCH % (256 * MB) == 0, "merge batches");
  const int rb = item % a.nrb, bd = item / a.nrb;
  const FusedDir d = a.dir[bd % a.ndir];
  const long long b = bd / a.ndir;
  typedef __attribute__((ext_vector_type(2))) float f32x2;
  const __amdgpu_buffer_rsrc_t ro = part_rsrc(a.opart), rml = part_rsrc(a.mlpart);
  for (int base = 0; base < NCH; base += 256 * MB) {
    float acc[MB][8], M[MB], L[MB];
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      M[j] = -INFINITY;
      L[j] = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[j][e] = 0.f;
    }
    for (int s = 0; s < nseg; ++s) {
      bf16x8 pv[MB];
      f32x2 ml[MB];
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        const int idx = base + j * 256 + threadIdx.x;
        const unsigned prow = (unsigned)(slot0 + s) * RB + idx / (FD / 8);
        const unsigned off = (prow * FD + (idx % (FD / 8)) * 8) * 2;   // bf16 partial rows
        pv[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ro, off, 0, CP_SYS));
        if constexpr (MODE == 0) ml[j] = __builtin_amdgcn_raw_buffer_load_b64(rml, prow * 8, 0, CP_SYS);
      }
#pragma unroll
      for (int j = 0; j < MB; ++j) {
        float ws = 1.f, wo = 1.f;
        if constexpr (MODE == 0) {
          const float mn = fmaxf(M[j], ml[j].x);
          wo = __builtin_amdgcn_exp2f(M[j] - mn);          // 0 on the first slot (M = -inf)
          ws = ml[j].y > 0.f ? __builtin_amdgcn_exp2f(ml[j].x - mn) : 0.f;
          M[j] = mn;
          L[j] = fmaf(ml[j].y, ws, L[j] * wo);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[j][e] = fmaf((float)pv[j][e], ws, acc[j][e] * wo);
      }
    }
#pragma unroll
    for (int j = 0; j < MB; ++j) {
      const int idx = base + j * 256 + threadIdx.x;
      const int row = idx / (FD / 8), k = idx % (FD / 8);
      // chunk k = 4 p + g of a partial row: channels 32 p + 4 g .. +3 and 32 p + 16 + 4 g .. +3
      const int c0 = 32 * (k >> 2) + 4 * (k & 3);
      const int q = rb * RB + row;
      if (q >= a.HW) {
        if (MODE == 0 && d.lse && k == 0 && q < a.HWp) d.lse[b * a.HWp + q] = INFINITY;
        continue;
      }
      bf16* op = d.o + (b * a.HW + q) * d.ldo + c0;
      const float inv = MODE == 0 ? 1.f / L[j] : 1.f;
      typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4m;
      bf16x4m lo, hi;
      if (MODE == 1 && a.accumulate) {
        const bf16x4m olo = *(const bf16x4m*)op, ohi = *(const bf16x4m*)(op + 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo[e] = (bf16)(acc[j][e] + (float)olo[e]);
          hi[e] = (bf16)(acc[j][4 + e] + (float)ohi[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          lo[e] = (bf16)(acc[j][e] * inv);
          hi[e] = (bf16)(acc[j][4 + e] * inv);
        }
      }
      *(bf16x4m*)op = lo;
      *(bf16x4m*)(op + 16) = hi;
      if (MODE == 0 && d.lse && k == 0) d.lse[b * a.HWp + q] = M[j] + __builtin_amdgcn_logf(L[j]);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1)))
void coatt_q48_k(FusedArgs a) {
  __shared__ __attribute__((aligned(16))) char lds[Q48ST * 2 * FTILE];   // 96 KB
  __shared__ int wg_ovf[4];
  __shared__ int wg_last;
  const int G = a.nwork;
  // XCD-aware: hardware places workgroup i on XCD i % 8, so XCD x runs the x-th eighth of the
  // item-major list (the row blocks of one (pair, direction) share its K / V stream in that L2)
  const int lw = (G & 7) ? (int)blockIdx.x : ((int)blockIdx.x & 7) * (G >> 3) + ((int)blockIdx.x >> 3);
  const int ntiles = a.ntiles;
  const long long U = (long long)a.nitems * ntiles;
  long long u = (long long)lw * U / G;
  const long long u1 = (long long)(lw + 1) * U / G;
  bool first = true;
#if Q48_PROF
  const unsigned long long k0_ = __builtin_amdgcn_s_memtime();
  unsigned long long mg_ = 0;
#endif
  while (u < u1) {
    const int item = (int)(u / ntiles), tb = (int)(u % ntiles);
    const int nt = (int)min((long long)(ntiles - tb), u1 - u);
    const long long ib = (long long)item * ntiles;
    const int w0 = q48_owner(ib, U, G), w1 = q48_owner(ib + ntiles - 1, U, G);
    const bool whole = w0 == w1;
    if (!first) raw_barrier_r();   // every wave is done with the ring (and the last merge)
    first = false;
    q48_segment<MODE>(a, lds, wg_ovf, item, tb, nt, whole ? -1 : item * a.smax + (lw - w0));
    if (!whole) {
      // every thread's write-through partial stores acknowledged, then one arrival per segment
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0)
        wg_last = __hip_atomic_fetch_add(a.cnt + item, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == w1 - w0;
      __syncthreads();
      if (wg_last) {
#if Q48_PROF
        const unsigned long long m0_ = __builtin_amdgcn_s_memtime();
#endif
        q48_merge<MODE>(a, item, w1 - w0 + 1, item * a.smax);
#if Q48_PROF
        mg_ += __builtin_amdgcn_s_memtime() - m0_;
#endif
        if (threadIdx.x == 0)    // ready for the next launch
          __hip_atomic_exchange(a.cnt + item, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    u += nt;
  }
#if Q48_PROF
  if (threadIdx.x == 0) {   // whole-workgroup clocks and merge clocks
    atomicAdd(&g_q48_prof[6], __builtin_amdgcn_s_memtime() - k0_);
    atomicAdd(&g_q48_prof[7], mg_);
  }
#endif
}

}  // namespace

__global__ __launch_bounds__(256) void q48_zero_cnt_k(int* cnt, int n) {
  for (int i = threadIdx.x; i < n; i += 256) cnt[i] = 0;
}

int coatt_q48_rows() { return RB; }

// Workgroups and partial slots per item for `items` items of `ntiles` key tiles: 256 ranges
// (one per CU) of >= 8 tile steps each; `cut` false: one workgroup per item, nothing cut.
static void q48_plan(int items, int ntiles, bool cut, int* nwork, int* smax) {
  const long long U = (long long)items * ntiles;
  long long G = items;              // uncut: one workgroup per item
  if (cut) {
    // 256 equal ranges (also when there are more items than CUs: a range then covers one item
    // and parts of its neighbours -- one round of 1.2 items beats two rounds of one at 8 pairs)
    G = std::min<long long>(256, std::max<long long>(1, U / 8));
    if ((ntiles + U / G - 1) / (U / G) + 1 > 8)   // the merge holds <= 8 slots per item
      G = std::max<long long>(1, U / ((ntiles + 6) / 7));
  }
  const long long L = U / G;        // shortest range (tile steps)
  *nwork = (int)G;
  *smax = (int)((ntiles + L - 1) / L + 1);
}

size_t coatt_q48_workspace_bytes(int items, int ntiles) {
  int G, smax;
  q48_plan(items, ntiles, true, &G, &smax);
  if (G == items) return 0;
  // bf16 partial O rows, fp32 (reference, sum) pairs, the arrival counters
  return (size_t)items * smax * RB * (FD * sizeof(bf16) + 2 * sizeof(float)) + (size_t)items * sizeof(int) + 16;
}

int coatt_q48_launch(int mode, FusedArgs& a, int B, int nd, bool merge_ok, void* ws,
                     size_t ws_bytes, hipStream_t st) {
  a.ndir = nd;
  a.nrb = (a.HW + RB - 1) / RB;
  a.nitems = a.nrb * B * nd;
  a.ntiles = (a.HW + FBK - 1) / FBK;
  const size_t need = coatt_q48_workspace_bytes(a.nitems, a.ntiles);
  const bool cut = merge_ok && need && ws && ws_bytes >= need && ((uintptr_t)ws & 15) == 0;
  q48_plan(a.nitems, a.ntiles, cut, &a.nwork, &a.smax);
  if (a.nwork != a.nitems) {
    const size_t rows = (size_t)a.nitems * a.smax * RB;
    a.opart = (float*)ws;                  // bf16 rows of FD channels
    a.mlpart = a.opart + rows * FD / 2;
    a.cnt = (int*)(a.mlpart + rows * 2);
    // zeroed by hipMemsetAsync (the merge resets each counter too).  Round 6 measured the
    // alternative the advisor suggested -- a one-workgroup zeroing kernel, a kernel node instead
    // of a memset node in the recorded step -- at 2.7 % of the whole training step: 132.1 vs 135.7
    // frame-pairs/s, the training co-attention 0.16 vs 0.21 of peak, each forward launch ~70 us
    // longer in HIP events (profiles/r06_q48_counter_zero_ab.txt).  CN_Q48_ZERO_KERNEL=1 selects
    // the kernel (A/B runs).
    static const bool use_kernel = [] { const char* e = getenv("CN_Q48_ZERO_KERNEL"); return e && e[0] == '1'; }();
    if (!use_kernel) {
      const hipError_t e = hipMemsetAsync(a.cnt, 0, (size_t)a.nitems * sizeof(int), st);
      if (e != hipSuccess) return (int)e;
    } else {
      hipLaunchKernelGGL(q48_zero_cnt_k, dim3(1), dim3(256), 0, st, a.cnt, a.nitems);
      CN_CHECK_LAUNCH();
    }
  }
  if (mode == 0) hipLaunchKernelGGL(coatt_q48_k<0>, dim3(a.nwork), dim3(256), 0, st, a);
  else hipLaunchKernelGGL(coatt_q48_k<1>, dim3(a.nwork), dim3(256), 0, st, a);
  CN_CHECK_LAUNCH();
  return 0;
}

#if Q48_PROF
extern "C" int cn_q48_prof_read(unsigned long long* out) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_q48_prof), sizeof(unsigned long long) * 8);
  if (e != hipSuccess) return (int)e;
  unsigned long long z[8] = {};
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_q48_prof), z, sizeof(z));
}
#endif
