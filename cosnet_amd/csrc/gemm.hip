// Generic implicit-GEMM on MFMA for gfx950 (CDNA4).
//
//   C[m][n] = alpha * sum_k A[m][k] * B[n][k]  (+ bias[n])   with fp32 accumulation
//
// Every matrix product on the hot path is an instance of this one kernel; the operands are
// produced by "loaders" that gather straight from NHWC activations, so no im2col buffer is
// ever materialised:
//   KC_DENSE : A/B row-major with k contiguous (weights [Cout][kh][kw][Cin], features [HW][C])
//   KC_CONV  : rows = output pixels, k = (r, s, ci) gathered from an NHWC tensor
//              (conv forward; conv dgrad with stride 1 is the same gather with negated taps)
//   MC_DENSE : k-major source, m/n contiguous (dY [P][Cout] in wgrad, V [HW][C] in attention)
//   MC_CONV  : k = output pixel, n = (r, s, ci) gathered from NHWC input (wgrad B operand)
// KC tiles live in LDS as [rows][128 B] with a (row & 7) XOR swizzle of the 16-B chunks, read
// with ds_read_b128; MC tiles live as [k][cols] and are read with the gfx950 hardware
// transpose read ds_read_b64_tr_b16 (bf16) or scalar reads (fp32 parity path).
// Block = 256 threads = 4 waves in a 2x2 grid, each wave owning a (BM/2)x(BN/2) C tile of
// 16x16 MFMA blocks (v_mfma_f32_16x16x32_bf16, or v_mfma_f32_16x16x4_f32 for fp32).
// K step = 128 bytes of k (64 bf16 / 32 fp32); register-staged double-buffered LDS.
#include "common.h"
#include "gemm.h"
#include "../../include/cosnet_hip.h"

#include <cstdlib>
#include <type_traits>

namespace {

template <class T> struct Frag;
template <> struct Frag<bf16> { typedef bf16x8 type; };
template <> struct Frag<float> { typedef f32x4 type; };

__device__ __forceinline__ int mc_swz(int k, int granules_per_row) {
  // granule (8 B) XOR so that a transposed read's 32-lane half hits 32 distinct granules
  int h = (k & 3) | (((k >> 3) & 1) << 2);
  return (granules_per_row >= 32 ? h : (h & 3)) << 2;
}

// fp8 MC tiles ([k][128 columns] bytes, eight 16-byte column chunks per k-row): chunk c of k-row k
// sits in slot c ^ mc_swz8(k).  A ds_read_b64_tr_b8 of one 16-lane group reads eight consecutive
// k-rows of one chunk (read_frag_f8_mc): k & 7 spreads them over eight slots, and (k >> 5) & 1
// moves the group reading k + 32 to the other eight 16-byte bank groups of the 256-byte window,
// so the two groups of a half-wave cover all 64 banks once.
__device__ __forceinline__ int mc_swz8(int k) { return (k & 7) ^ ((k >> 5) & 1); }

// 16 zero bytes in global memory: out-of-bounds lanes of an LDS-DMA fill read from here.
__device__ __attribute__((aligned(16))) unsigned g_zero16[4];

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// Buffer-descriptor form of the same LDS-DMA (buffer_load_dwordx4 ... lds): address = base +
// soffset (SGPR, wave-uniform: the K position of the tile) + voffset (VGPR, constant per chunk
// over a whole tap / the whole K loop).  The hardware range check covers voffset only (not
// soffset): a chunk with no source (padding row / column, conv tap outside the image, k past the
// end) gets voffset = BUF_OOB and reads zeros -- no zero page, no per-chunk select, no 64-bit
// address arithmetic in the K loop.
constexpr unsigned BUF_OOB = 0x80000000u;   // = num_records of every operand descriptor
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)BUF_OOB, 0x00020000);
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff,
                                       char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base,
                                           16, (int)voff, (int)soff, 0, 0);
}

// -------------------------------------------------------------------------------------
// Operand loader: LDS-DMA fill of one ROWS x 128-byte K tile per call, NCH = ROWS*8/NT 16-byte
// chunks per thread.  Everything that does not change along K is computed once in init().
//
// KC_DENSE, KC_CONV (C % BK == 0) and MC_DENSE use the buffer-descriptor DMA (blds16): each
// chunk keeps a 32-bit byte offset that is constant over the whole K loop (KC_DENSE, MC_DENSE)
// or over one conv tap (KC_CONV), and the K position of the tile goes into the wave-uniform
// soffset -- so a K step costs no vector address arithmetic at all: the tap and channel base of
// a tile are scalars (a K tile never straddles taps when C % BK == 0) and a missing source
// (padding row, tap outside the image, k past the end) is the out-of-range offset BUF_OOB,
// which the hardware reads as zeros.  KC_CONV_G (conv gathers with C % BK != 0: the stems,
// fp8 on 64-channel layers) and MC_CONV (weight-gradient B operand) keep per-thread pointers and
// the flat global_load_lds.  Tiles are issued strictly in order, starting at kbeg.
// -------------------------------------------------------------------------------------
template <class T, int ROWS, int KIND, int NT> struct Loader {
  static constexpr int VEC = VecOf<T>::N;
  static constexpr int BK = 8 * VEC;
  static constexpr int NCH = ROWS * 8 / NT;       // chunks per thread
  static constexpr int RSTEP = NT / 8;            // KC: rows between a thread's chunks
  static_assert(NCH >= 1 && NCH * NT == ROWS * 8, "tile rows must fill whole chunk rounds");
  static constexpr bool MC = (KIND == L_MC_DENSE || KIND == L_MC_CONV);
  static constexpr bool BUF = (KIND == L_KC_DENSE || KIND == L_KC_CONV || KIND == L_MC_DENSE);
  static constexpr int CPR = ROWS / VEC;          // MC: chunks per k-row
  static constexpr int KROW_STEP = NT / CPR;      // MC: k-rows between a thread's chunks
  static constexpr int RB = ROWS * (int)sizeof(T);  // MC: bytes per k-row of the LDS image
  static constexpr unsigned SZ = sizeof(T);
  static_assert(!(MC && sizeof(T) == 1) || CPR == 8, "fp8 MC tiles are 128 columns wide (mc_swz8)");

  long long ld;
  int klim;             // k bound (zero beyond)
  int kbeg;
  int kcol;             // KC: this thread's k offset within a tile (swizzled chunk * VEC)
  bool ok[NCH];         // row / column / pixel validity
  // buffer path
  __amdgpu_buffer_rsrc_t rsrc;
  unsigned voff[NCH];   // byte offset of chunk i (BUF_OOB: no source)
  // KC_CONV / KC_CONV_G
  int img[NCH], by[NCH], bx[NCH];
  int ctap;             // tap whose offsets / pointers are cached (-1: none)
  // flat path (KC_CONV_G, MC_CONV)
  const T* base;
  const T* ptr[NCH];    // KC_CONV_G: pixel pointer of the cached tap
  // MC_CONV: per-chunk column (tap offsets, channel) and output-pixel coordinates
  int ry[NCH], sx[NCH], cic[NCH];
  int pim[NCH], poy[NCH], pox[NCH], pp[NCH];
  int ax, ay, aim;      // advance of (ox, oy, im) per K tile
  ConvGeom g;

  __device__ __forceinline__ void init(const T* b, long long ld_, int lim, int klim_,
                                       const ConvGeom& geo, int origin, int tid, int kbeg_) {
    ld = ld_; klim = klim_; kbeg = kbeg_;
    base = b;
    if (!MC) {
      const int pos = tid & 7;
      kcol = (pos ^ ((tid >> 3) & 7)) * VEC;  // row & 7 == (tid >> 3) & 7 for every chunk
      if (KIND == L_KC_DENSE) rsrc = buf_rsrc(b + (long long)origin * ld);   // block-rebased
      if (KIND == L_KC_CONV) rsrc = buf_rsrc(b);
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int rl = (tid >> 3) + RSTEP * i;   // row within the tile
        const int row = origin + rl;
        ok[i] = row < lim;
        const int rr = ok[i] ? row : 0;
        if (KIND == L_KC_DENSE) {
          voff[i] = ok[i] ? (unsigned)((rl * ld + kcol) * SZ) : BUF_OOB;
        } else {
          int q, rem, oy, ox;
          fdivmod(rr, geo.div_OHW, q, rem);
          fdivmod(rem, geo.div_OW, oy, ox);
          img[i] = ok[i] ? q : -1;
          by[i] = oy * geo.st + geo.off_y;
          bx[i] = ox * geo.st + geo.off_x;
        }
      }
      if (KIND == L_KC_CONV || KIND == L_KC_CONV_G) {
        g = geo;
        ctap = -1;
      }
    } else {
      const int pos = tid % CPR;
      if (KIND == L_MC_DENSE) rsrc = buf_rsrc(b + (long long)kbeg_ * ld + origin);   // block-rebased
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int krl = tid / CPR + KROW_STEP * i;  // k-row within the tile
        const int cchunk = (sizeof(T) == 2) ? (pos ^ (mc_swz(krl, RB / 8) >> 1))
                         : (sizeof(T) == 1) ? (pos ^ mc_swz8(krl)) : pos;
        const int col = origin + cchunk * VEC;
        ok[i] = col < lim;
        if (KIND == L_MC_DENSE) {
          voff[i] = ok[i] ? (unsigned)((krl * ld + cchunk * VEC) * SZ) : BUF_OOB;
        } else {
          const int nn = ok[i] ? col : 0;
          int tap, r, s2;
          fdivmod(nn, geo.div_C, tap, cic[i]);
          fdivmod(tap, geo.div_KW, r, s2);
          ry[i] = r * geo.step_y + geo.off_y;
          sx[i] = s2 * geo.step_x + geo.off_x;
          pp[i] = kbeg_ + krl;
          int q, rem, oy, ox;
          fdivmod(pp[i] < klim ? pp[i] : 0, geo.div_OHW, q, rem);
          fdivmod(rem, geo.div_OW, oy, ox);
          pim[i] = q; poy[i] = oy; pox[i] = ox;
        }
      }
      if (KIND == L_MC_CONV) {
        g = geo;
        int q, rem, oy, ox;
        fdivmod(BK, geo.div_OHW, q, rem);
        fdivmod(rem, geo.div_OW, oy, ox);
        aim = q; ay = oy; ax = ox;
      }
    }
  }

  // Fill of one K tile: chunk q = tid + NT i lands at byte 16 q of the tile (lane-linear per
  // wave instruction); the XOR swizzle lives in the SOURCE address so the image is the swizzled
  // layout the fragment readers expect.
  __device__ __forceinline__ void issue(int k0, char* lds, int tid) {
    char* wbase = lds + __builtin_amdgcn_readfirstlane((tid & ~63) * 16);
    // k0 is wave-uniform: whole-tile bounds and the tap / offset arithmetic below are scalar
    const bool tail = k0 + BK > klim;
    if constexpr (KIND == L_KC_DENSE) {
      if (!tail) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) blds16(rsrc, voff[i], (unsigned)k0 * SZ, wbase + i * NT * 16);
      } else {
        const bool kok = k0 + kcol < klim;
#pragma unroll
        for (int i = 0; i < NCH; ++i) blds16(rsrc, kok ? voff[i] : BUF_OOB, (unsigned)k0 * SZ, wbase + i * NT * 16);
      }
    } else if constexpr (KIND == L_KC_CONV) {
      const int tap = __builtin_amdgcn_readfirstlane(fdiv(k0, g.div_C));
#ifdef CN_PROBE_A_ONCE
      // TIMING PROBE ONLY (results are wrong): the A tile of tap 0 stands in for every tap -- the
      // upper bound of an input-halo loader that fills A once per channel chunk instead of per tap
      if (tap != 0) return;
#endif
      if (tap != ctap) {   // new tap (uniform branch): the chunks' pixel offsets
        int r, ss;
        fdivmod(tap, g.div_KW, r, ss);
        const int oy = r * g.step_y, ox = ss * g.step_x;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
          const int y = by[i] + oy, x = bx[i] + ox;
          const bool v = img[i] >= 0 && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
          const unsigned pix = (unsigned)((img[i] * g.H + y) * g.W + x);
          voff[i] = v ? (pix * (unsigned)ld + (unsigned)kcol) * SZ : BUF_OOB;
        }
        ctap = tap;
      }
      const unsigned soff = (unsigned)(k0 - tap * g.C) * SZ;
      if (!tail) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) blds16(rsrc, voff[i], soff, wbase + i * NT * 16);
      } else {
        const bool kok = k0 + kcol < klim;
#pragma unroll
        for (int i = 0; i < NCH; ++i) blds16(rsrc, kok ? voff[i] : BUF_OOB, soff, wbase + i * NT * 16);
      }
    } else if constexpr (KIND == L_MC_DENSE) {
      const unsigned soff = (unsigned)(k0 - kbeg) * (unsigned)ld * SZ;
      if (!tail) {
#pragma unroll
        for (int i = 0; i < NCH; ++i) blds16(rsrc, voff[i], soff, wbase + i * NT * 16);
      } else {
        const int kr0 = k0 + tid / CPR;
#pragma unroll
        for (int i = 0; i < NCH; ++i)
          blds16(rsrc, kr0 + KROW_STEP * i < klim ? voff[i] : BUF_OOB, soff, wbase + i * NT * 16);
      }
    } else if constexpr (KIND == L_KC_CONV_G) {
      const void* zp = (const void*)g_zero16;
      const int k = k0 + kcol;
      const bool kok = k < klim;
      int tap, cc;
      fdivmod(kok ? k : 0, g.div_C, tap, cc);
      if (tap != ctap) {  // new tap: recompute the pixel pointers
        int r, ss;
        fdivmod(tap, g.div_KW, r, ss);
        const int oy = r * g.step_y, ox = ss * g.step_x;
#pragma unroll
        for (int i = 0; i < NCH; ++i) {
          const int y = by[i] + oy, x = bx[i] + ox;
          const bool v = img[i] >= 0 && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
          ok[i] = v;
          const unsigned pix = v ? (unsigned)((img[i] * g.H + y) * g.W + x) : 0u;
          ptr[i] = base + (unsigned long long)pix * (unsigned)ld;
        }
        ctap = tap;
      }
#pragma unroll
      for (int i = 0; i < NCH; ++i)
        glds16((ok[i] && kok) ? (const void*)(ptr[i] + cc) : zp, wbase + i * NT * 16);
    } else {  // L_MC_CONV: k = output pixel, n = (tap, ci) fixed per chunk
      const void* zp = (const void*)g_zero16;
#pragma unroll
      for (int i = 0; i < NCH; ++i) {
        const int y = poy[i] * g.st + ry[i], x = pox[i] * g.st + sx[i];
        const bool v = ok[i] && pp[i] < klim && (unsigned)y < (unsigned)g.H && (unsigned)x < (unsigned)g.W;
        const unsigned pix = (unsigned)((pim[i] * g.H + y) * g.W + x);
        const T* src = base + ((unsigned long long)pix * (unsigned)ld + (unsigned)cic[i]);
        glds16(v ? (const void*)src : zp, wbase + i * NT * 16);
        // advance the pixel by one K tile
        pp[i] += BK;
        pox[i] += ax;
        poy[i] += ay;
        pim[i] += aim;
        if (pox[i] >= g.OW) { pox[i] -= g.OW; poy[i] += 1; }
        if (poy[i] >= g.OH) { poy[i] -= g.OH; pim[i] += 1; }
      }
    }
  }
};

// Fragment readers ------------------------------------------------------------------------
// bf16: fragment for k-piece p (32 k values): lane l -> row/col (l&15), k = 32p + 8(l>>4) + j
template <int ROWS, bool MC>
__device__ __forceinline__ bf16x8 read_frag_bf16(const char* lds, int rowbase, int p, int lane) {
  int g = lane >> 4;
  if (!MC) {
    int row = rowbase + (lane & 15);
    int c = 4 * p + g;
    return *(const bf16x8*)(lds + row * 128 + ((c ^ (row & 7)) << 4));
  } else {
    constexpr int RB = ROWS * 2;
    int q = (lane & 15) >> 2, pp = lane & 3;
    int gm = (rowbase >> 2) + pp;  // granule of columns rowbase + 4pp .. +3
    int k1 = 32 * p + 8 * g + q, k2 = k1 + 4;
    const char* a1 = lds + k1 * RB + ((gm ^ mc_swz(k1, RB / 8)) << 3);
    const char* a2 = lds + k2 * RB + ((gm ^ mc_swz(k2, RB / 8)) << 3);
    s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a1));
    s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, a2));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 r = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, r);
  }
}

// fp8 (KC only): one 16x16x128 MFMA per 128-byte K tile; lane l supplies row/col (l & 15) and the
// 32 bytes of chunks 2g, 2g+1 (g = l >> 4).  The hardware's k order within the operand is the
// same for A and B, so reading both operands at the same byte offsets sums the right products.
__device__ __forceinline__ i32x8 read_frag_f8(const char* lds, int rowbase, int lane) {
  const int row = rowbase + (lane & 15), g = lane >> 4;
  const u32x4 lo = *(const u32x4*)(lds + row * 128 + (((2 * g) ^ (row & 7)) << 4));
  const u32x4 hi = *(const u32x4*)(lds + row * 128 + (((2 * g + 1) ^ (row & 7)) << 4));
  i32x8 r;
  r[0] = lo.x; r[1] = lo.y; r[2] = lo.z; r[3] = lo.w; r[4] = hi.x; r[5] = hi.y; r[6] = hi.z; r[7] = hi.w;
  return r;
}

// fp8 MC (k-major [k][128 B] tile, the weight-gradient operands dY and X): the same operand as
// read_frag_f8 -- lane l supplies column (l & 15) of the 16 at colbase and the 32 k of group
// g = l >> 4, byte b = k 32g + b -- assembled from four ds_read_b64_tr_b8: in each, the group's
// lane 2q + p addresses k-row 32g + 8j + q, bytes 8p..8p+7 of the column chunk, and lane i
// receives column i of those eight k-rows (byte q = k-row q; profiles/r04_tr_b8_probe.txt).
typedef __attribute__((ext_vector_type(2))) int i32x2;
__device__ __forceinline__ i32x8 read_frag_f8_mc(const char* lds, int colbase, int lane) {
  const int i = lane & 15, g = lane >> 4, q = i >> 1, pp = i & 1;
  const int cb = colbase >> 4;
  i32x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int k = 32 * g + 8 * j + q;
    const char* a = lds + k * 128 + ((cb ^ mc_swz8(k)) << 4) + 8 * pp;
    const i32x2 v = __builtin_amdgcn_ds_read_tr8_b64_v2i32(LDS_PTR(i32x2, a));
    r[2 * j] = v.x;
    r[2 * j + 1] = v.y;
  }
  return r;
}

// fp32: piece p, step j -> k = 16p + 4(l>>4) + j ; returns the 4 floats of (p) for KC,
// or the scalar for MC (per j).
template <int ROWS>
__device__ __forceinline__ f32x4 read_frag_f32_kc(const char* lds, int rowbase, int p, int lane) {
  int row = rowbase + (lane & 15);
  int c = 4 * p + (lane >> 4);
  return *(const f32x4*)(lds + row * 128 + ((c ^ (row & 7)) << 4));
}
template <int ROWS>
__device__ __forceinline__ float read_frag_f32_mc(const char* lds, int rowbase, int p, int j, int lane) {
  int k = 16 * p + 4 * (lane >> 4) + j;
  int col = rowbase + (lane & 15);
  return *(const float*)(lds + k * (ROWS * 4) + col * 4);
}

template <class CT> __device__ __forceinline__ void store_c(CT* c, float v, int mode);
template <> __device__ __forceinline__ void store_c<float>(float* c, float v, int mode) {
  if (mode == 1) atomicAdd(c, v);
  else if (mode == 2) *c += v;
  else *c = v;
}
template <> __device__ __forceinline__ void store_c<bf16>(bf16* c, float v, int mode) {
  if (mode == 2) v += (float)*c;
  *c = (bf16)v;
}

}  // namespace

// Counted wait on this wave's vector-memory queue: all but the n*G youngest LDS-DMA chunks
// have landed (n = tiles left in flight, G = chunks per thread per tile; immediates only).
template <int G>
__device__ __forceinline__ void wait_tiles(int n) {
  if (n <= 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if (n == 1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(G) : "memory");
  else if (n == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * G) : "memory");
  else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(3 * G) : "memory");
}

// Workgroup barrier that does NOT drain the LDS-DMA queue (unlike __syncthreads(), whose
// fence emits vmcnt(0)); the asm memory clobbers keep the compiler from moving LDS accesses
// across it.
__device__ __forceinline__ void raw_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------------------------------
// The kernel.  Tile BM x BN, WM x WN waves (each a (BM/WM) x (BN/WN) block of 16x16 MFMA
// tiles), S-deep ring of LDS stages filled by LDS-DMA: the DMA of tile kt+S-1 is issued while
// tile kt is consumed, and each K step ends with a COUNTED wait for tile kt+1 only (the
// younger S-2 tiles stay in flight across the barrier) -- one barrier per K step.
// ---------------------------------------------------------------------------------------
#ifndef CN_GEMM_GROUP_M
#define CN_GEMM_GROUP_M 8
#endif
#ifndef CN_GEMM_PRIO
#define CN_GEMM_PRIO 0
#endif
#ifndef CN_GEMM_ZREMAP
#define CN_GEMM_ZREMAP 1
#endif

// BN-epilogue variants of the 128-row tiles keep <= 128 VGPRs (4 waves per SIMD = two 512-thread
// blocks per CU, the
// occupancy the plain kernel has from its LDS footprint; HIP's 2nd bound is waves per SIMD).
//
// PP (ping-pong, 8 waves, KC bf16 operands only): the waves form two groups of four -- one wave
// of each group per SIMD -- and group 1 runs one barrier behind group 0, so between any two
// barriers one group issues its MFMAs (one 32-deep k piece of its wave tile) while the other
// reads its next fragments and issues the LDS-DMA refill.  Each K step is four barrier phases
// per group: [frags pc0] | [MFMA pc0] | [frags pc1, refill, counted wait for tile kt+1] |
// [MFMA pc1].  A phase's fragment reads are waited for (lgkmcnt) by its MFMA phase, after the
// barrier, so the read latency overlaps the other group's MFMAs.  RAW: every wave's wait for
// tile kt+1 precedes its third barrier of step kt, and both groups read tile kt+1 only after the
// barrier that follows the later group's wait.  WAR: the stage of tile kt-1 is refilled in the
// third phase of step kt, after the barrier that ends either group's MFMA phase of pc1 of step
// kt-1 -- the phase whose lgkmcnt wait retired that group's last reads of tile kt-1 (a 2-stage
// ring refills in the first phase instead, and retires the third phase's reads before its
// barrier).
//
// PP == 2 (KSG, K-split wave groups; bf16 KC operands): 2 x WM x WN waves.  Group g (waves
// g*WM*WN ..) runs k-piece g (32 of the tile's 64 k) of every K step on the WHOLE WM x WN tile
// layout, i.e. each wave owns a wave tile twice the size it would have with 8 waves splitting the
// block tile, and reads half as many fragments per MFMA: LDS fragment bytes per FLOP scale as
// 1/TM + 1/TN (the DMA-write / ds_read contention the fill probe measures), while
// two waves per SIMD remain.  The groups' partial accumulators are summed once, in the epilogue
// (group 1 stages its tile in LDS, group 0 adds its own before the stores).
template <class T, class CT, int BM, int BN, int WM, int WN, int S, int LA, int LB, int EPI = 0, int PP = 0>
__global__ __launch_bounds__(WM * WN * 64 * (PP == 2 ? 2 : 1), (EPI && sizeof(T) == 2 && BM * BN <= 128 * 128 && S == 2) ? 4 : 1) void gemm_kernel(GemmArgs p) {
  constexpr bool KSG = PP == 2;
  constexpr int NT = WM * WN * 64 * (KSG ? 2 : 1);
  constexpr int VEC = VecOf<T>::N;
  constexpr int BK = 8 * VEC;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128;
  constexpr int STAGE = ABYTES + BBYTES;
  constexpr int TM = BM / WM, TN = BN / WN;  // wave tile
  constexpr int RM = TM / 16, RN = TN / 16;  // 16x16 blocks per wave in m / n
  constexpr bool AMC = (LA == L_MC_DENSE || LA == L_MC_CONV);
  constexpr bool BMC = (LB == L_MC_DENSE || LB == L_MC_CONV);
  typedef Loader<T, BM, LA, NT> LdA;
  typedef Loader<T, BN, LB, NT> LdB;
  constexpr int G = LdA::NCH + LdB::NCH;
  static_assert(S >= 2 && S <= 4, "2..4 stages");
  __shared__ __attribute__((aligned(16))) char smem[S * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int kg = KSG ? wave / (WM * WN) : 0;            // KSG: this wave's k piece
  const int wl = KSG ? wave % (WM * WN) : wave;
  const int wm = wl / WN, wn = wl % WN;
  static_assert(!KSG || (sizeof(T) == 2 && !AMC && !BMC), "KSG: bf16 k-contiguous operands");
  // XCD-aware tile order (guide §5.5 T1, bijective form): blocks are dealt round-robin over
  // the 8 XCDs, so remap the linear id to give every XCD a contiguous run of M-tiles that
  // share the same B (weight) panel in its private L2.
  // The remap runs over the whole grid, z (batch / K split) included, z-major: the blocks of one
  // K split (or batch entry) land on one XCD, which then streams that split's A and B slices
  // through its L2 once (split-K weight gradients: 16-36 tiles per split, 1-2.3 MB per slice)
  // instead of every XCD re-reading every split's panels.
  int tm, tn, bz;
  {
    const int nwg = gridDim.x * gridDim.y;
#if CN_GEMM_ZREMAP
    const int all = nwg * gridDim.z;
    const int orig = blockIdx.x + blockIdx.y * gridDim.x + blockIdx.z * nwg;
#else
    const int all = nwg;
    const int orig = blockIdx.x + blockIdx.y * gridDim.x;
#endif
    int glin = orig;
    if (all >= 16) {
      const int xcd = orig & 7, q = all >> 3, r = all & 7;
      glin = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
    }
#if CN_GEMM_ZREMAP
    bz = glin / nwg;
#else
    bz = blockIdx.z;
#endif
    const int lin = glin - (glin / nwg) * nwg;
#if CN_GEMM_GROUP_M > 0
    // grouped order: each run of GROUP_M M-tiles walks all its N-tiles before the next run,
    // so the blocks resident on one XCD share A panels (and the B panel) in its L2
    {
      const int gm = CN_GEMM_GROUP_M;
      const int per = gm * gridDim.y;
      const int grp = lin / per, first = grp * gm;
      const int gsz = min((int)gridDim.x - first, gm);
      const int r = lin - grp * per;
      tm = first + r % gsz;
      tn = r / gsz;
    }
#else
    tm = lin % gridDim.x;
    tn = lin / gridDim.x;
#endif
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int batch = bz / p.nsplit, split = bz - batch * p.nsplit;
  int kbeg = split * p.k_chunk;
  int kend = min(p.K, kbeg + p.k_chunk);
  // the A gather's geometry: per problem in a grouped launch of convs of different dilations
  ConvGeom gA = p.ga;
  if constexpr (LA == L_KC_CONV) {
    if (p.ngroup && p.grp.dil[batch] > 0) {
      const int dl = p.grp.dil[batch];
      gA.off_y = gA.off_x = -dl;
      gA.step_y = gA.step_x = dl;
    }
  }
  const float* bias = (p.ngroup && p.grp.bias[batch]) ? p.grp.bias[batch] : p.bias;
  if constexpr (LA == L_KC_CONV) {
    // Vertical tap skipping (conv forward / stride-1 dgrad gathers; k = (r, s, ci), r-major): the
    // taps r whose source rows y = oy st + off_y + r step_y miss the image for EVERY row of this
    // tile contribute exact zeros, and the valid r form one interval, so the block runs only the
    // K range of taps [r_lo, r_hi] -- e.g. the ASPP's dilation-12 / 18 convs on the 60 x 60 map,
    // where a 256-row tile (~4 image rows) near the top or bottom edge has a whole tap row of
    // padding.  Uniform per block (the tile's first / last row); a tile spanning two images
    // keeps every tap.
    const ConvGeom& g = gA;
    if (g.KH > 1) {
      int i0, i1, rm0, rm1, oy0, oy1, ox;
      fdivmod(m0, g.div_OHW, i0, rm0);
      fdivmod(min(m0 + BM, p.M) - 1, g.div_OHW, i1, rm1);
      fdivmod(rm0, g.div_OW, oy0, ox);
      fdivmod(rm1, g.div_OW, oy1, ox);
      if (i0 != i1) { oy0 = 0; oy1 = g.OH - 1; }
      const int ylo = oy0 * g.st + g.off_y, yhi = oy1 * g.st + g.off_y;
      int rlo = g.KH, rhi = -1;
      for (int r = 0; r < g.KH; ++r) {
        const int a = ylo + r * g.step_y, b = yhi + r * g.step_y;
        if (max(min(a, b), 0) <= min(max(a, b), g.H - 1)) { rlo = min(rlo, r); rhi = r; }
      }
      const int kt0 = rlo * g.KW * g.C, kt1 = (rhi + 1) * g.KW * g.C;
      kbeg = max(kbeg, kt0);
      kend = min(kend, kt1);
    }
  }
  const int nt = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  const T* Abase = p.ngroup ? (const T*)p.grp.A[batch] : (const T*)p.A + (long long)batch * p.a_bs;
  const T* Bbase = p.ngroup ? (const T*)p.grp.B[batch] : (const T*)p.B + (long long)batch * p.b_bs;

  LdA la;
  LdB lb;
  la.init(Abase, p.lda, p.M, min(p.ka_lim, kend), gA, m0, tid, kbeg);
  lb.init(Bbase, p.ldb, p.N, min(p.kb_lim, kend), p.gb, n0, tid, kbeg);

  // Epilogue geometry (below) and the epilogue operands that do not depend on the product,
  // loaded BEFORE the K loop so their latency hides behind it (the pass loop then prefetches
  // pass p + 1's rows during pass p): EPI 2 (BN-backward reduce) -- the per-column affine of the
  // forward apply and the pre-BN input rows; EPI 3 (read-add-store, c_mode 2: dgrad accumulating
  // into the residual gradient) -- the old C rows.  Loaded at the epilogue (round 5 and before),
  // their HBM latency sat exposed at the end of every block (~8-10 us per launch in the step).
  constexpr int LDC = BN + 4;
  constexpr int HR = (BM * LDC * 4 <= S * STAGE) ? BM
                   : ((BM / 2) * LDC * 4 <= S * STAGE) ? BM / 2
                   : ((BM / 4) * LDC * 4 <= S * STAGE) ? BM / 4 : BM / 8;
  static_assert(HR % 16 == 0 && HR * LDC * 4 <= S * STAGE, "epilogue staging must fit in the LDS image");
  static_assert(!KSG || HR == BM, "KSG sums the two groups' tiles in one staging pass");
  constexpr int GPR = BN / 8;            // 8-column groups per row
  constexpr int RPP = NT / GPR;          // rows per pass
  constexpr int IT = HR / RPP;           // rows per thread per pass
  static_assert(IT * RPP == HR, "epilogue rows per pass must be a multiple of the row stride");
  constexpr int smode = EPI == 3 ? 0 : EPI;   // BN epilogue (compile-time: its registers would
                                              // otherwise cost every plain GEMM occupancy)
  constexpr bool PFC = EPI == 3;
  constexpr int PQ = (int)sizeof(CT) / 2;     // 16-B chunks per 8 elements of C
  static_assert(!PFC || sizeof(CT) == 2, "EPI 3: bf16 C");
  const int c0t = (tid % GPR) * 8;            // this thread's columns within the tile (fixed)
  CT* Cb = (p.ngroup ? (CT*)p.grp.C[batch] : (CT*)p.C + (long long)batch * p.c_bs) +
           (p.c_mode == 3 ? (long long)split * p.slab : 0);
  u32x4 xnx[(smode == 2 || PFC) ? IT * PQ : 1];   // the next staging pass's rows
  // write-through C stores (p.wt): the block's rows from its first one, 32-bit offsets
  const __amdgpu_buffer_rsrc_t crs = buf_rsrc(Cb + (long long)m0 * p.ldc);
  auto epi_fetch = [&](int pass) {
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int row = m0 + pass * HR + tid / GPR + it * RPP;
      const int col = n0 + c0t;
      if constexpr (smode == 2) {
        const bool ok = row < p.M && col + 8 <= p.N;
        const u32x4* src = (const u32x4*)((const CT*)p.br_x + (long long)(ok ? row : m0) * p.br_ldx + (ok ? col : 0));
#pragma unroll
        for (int q = 0; q < PQ; ++q) xnx[it * PQ + q] = src[q];
      } else if constexpr (PFC) {
        const CT* dst = Cb + (long long)row * p.ldc + col;
        const bool ok = row < p.M && col + 8 <= p.N && ((uintptr_t)dst % 16 == 0);
        xnx[it] = ok ? *(const u32x4*)dst : u32x4{0u, 0u, 0u, 0u};
      }
    }
  };
  // EARLY: the prefetch registers stay live across the K loop -- only where that costs no spill
  // (tiles without the 128-VGPR occupancy bound of the 2-stage BN-epilogue kernels and below
  // 256 x 256, whose accumulators fill the register file; tools/kernel_resources.py checks)
  constexpr bool EARLY = PFC || (smode == 2 && S >= 3 && BM * BN <= 128 * 128);
  float bk1[8], bsf[8], bmu[8];
  auto epi_affine = [&]() {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = n0 + c0t + e;
      const bool in = c < p.N;
      const float g = in ? (p.br_gamma ? p.br_gamma[c] : 1.f) : 0.f;
      const float b = in ? (p.br_beta ? p.br_beta[c] : 0.f) : 0.f;
      const float is = in ? p.br_invstd[c] : 0.f;
      bmu[e] = in ? p.br_mean[c] : 0.f;
      bk1[e] = g * is;                  // the forward apply's affine (bn.hip bn_apply_k): the
      bsf[e] = b - bmu[e] * bk1[e];     // recomputed ReLU mask has exactly the forward's sign
    }
  };
  if constexpr (EARLY) {
    if constexpr (smode == 2) epi_affine();
    epi_fetch(0);
  }

  f32x4 acc[RM][RN];
#pragma unroll
  for (int i = 0; i < RM; ++i)
#pragma unroll
    for (int j = 0; j < RN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  // prologue: tiles 0 .. S-2 in flight, wait for tile 0
#pragma unroll
  for (int s = 0; s < S - 1; ++s) {
    if (s < nt) {
      la.issue(kbeg + s * BK, smem + s * STAGE, tid);
      lb.issue(kbeg + s * BK, smem + s * STAGE + ABYTES, tid);
    }
  }
  wait_tiles<G>(min(nt - 1, S - 2));
  raw_barrier();

#if CN_GEMM_PRIO == 2
  if (__builtin_amdgcn_readfirstlane(tid) >= NT / 2) __builtin_amdgcn_s_setprio(1);
#endif
  auto mma_tile = [&](const char* As, const char* Bs) {
    if constexpr (sizeof(T) == 1 && (AMC || BMC)) {
      return;   // fp8 k-major operands: kstep's own path (read_frag_f8_mc)
    } else if constexpr (sizeof(T) == 1) {
      i32x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i) af[i] = read_frag_f8(As, wm * TM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j) bfr[j] = read_frag_f8(Bs, wn * TN + j * 16, lane);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)  // e4m3 x e4m3, unit block scales (E8M0 127 = 2^0)
          // A format: 0 = e4m3 (forward activations), 1 = e5m2 (gradients, dgrad); B: e4m3 weights
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              af[i], bfr[j], acc[i][j], std::is_same<T, f8e5m2>::value ? 1 : 0, 0, 0, 127, 0, 127);
      return;
    }
#pragma unroll
    for (int pcl = 0; pcl < (KSG ? 1 : 2); ++pcl) {
      const int pc = KSG ? kg : pcl;
      if constexpr (sizeof(T) == 2) {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = read_frag_bf16<BM, AMC>(As, wm * TM + i * 16, pc, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = read_frag_bf16<BN, BMC>(Bs, wn * TN + j * 16, pc, lane);
#if CN_GEMM_PRIO == 1
        __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
#if CN_GEMM_PRIO == 1
        __builtin_amdgcn_s_setprio(0);
#endif
      } else if constexpr (sizeof(T) == 4) {
        f32x4 af[RM], bfr[RN];
        if (!AMC) {
#pragma unroll
          for (int i = 0; i < RM; ++i) af[i] = read_frag_f32_kc<BM>(As, wm * TM + i * 16, pc, lane);
        } else {
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) af[i][j] = read_frag_f32_mc<BM>(As, wm * TM + i * 16, pc, j, lane);
        }
        if (!BMC) {
#pragma unroll
          for (int i = 0; i < RN; ++i) bfr[i] = read_frag_f32_kc<BN>(Bs, wn * TN + i * 16, pc, lane);
        } else {
#pragma unroll
          for (int i = 0; i < RN; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) bfr[i][j] = read_frag_f32_mc<BN>(Bs, wn * TN + i * 16, pc, j, lane);
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int j = 0; j < RN; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][s4], bfr[j][s4], acc[i][j], 0, 0, 0);
      }
    }
  };

  // One K step on compile-time stage STG (tile kt lives in stage kt % S; the refill goes to the
  // stage consumed one step earlier, which every wave has passed the barrier of).
  auto kstep = [&](int kt, auto stg_c) {
    constexpr int STG = decltype(stg_c)::value;
    constexpr int NXT = (STG + S - 1) % S;
    const char* As = smem + STG * STAGE;
    const char* Bs = As + ABYTES;
    if constexpr (sizeof(T) == 1 && (AMC || BMC)) {
      // fp8 weight gradient (e5m2 dY x e4m3 X, both k-major): transposed byte reads, so -- as
      // for bf16 below -- the whole tile's fragments are read before the refill is issued
      i32x8 af[RM], bfr[RN];
#pragma unroll
      for (int i = 0; i < RM; ++i)
        af[i] = AMC ? read_frag_f8_mc(As, wm * TM + i * 16, lane) : read_frag_f8(As, wm * TM + i * 16, lane);
#pragma unroll
      for (int j = 0; j < RN; ++j)
        bfr[j] = BMC ? read_frag_f8_mc(Bs, wn * TN + j * 16, lane) : read_frag_f8(Bs, wn * TN + j * 16, lane);
      if (kt + S - 1 < nt) {
        la.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE, tid);
        lb.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE + ABYTES, tid);
      }
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              af[i], bfr[j], acc[i][j], std::is_same<T, f8e5m2>::value ? 1 : 0, 0, 0, 127, 0, 127);
    } else if constexpr (sizeof(T) == 2 && (AMC || BMC) && (RM + RN) <= 8 && !KSG) {
      // Transposed (MC) fragments are read with ds_read_b64_tr_b16, which hipcc cannot
      // disambiguate from an in-flight LDS-DMA: a DMA issued before these reads would cost a
      // full vmcnt(0) drain in front of them.  So read the whole tile's fragments FIRST, then
      // issue the refill, then run the MFMAs on registers (tiles whose fragments fit in
      // 64 VGPRs; the 256x256 tile keeps the refill-first order).
      bf16x8 af[2][RM], bfr[2][RN];
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
#pragma unroll
        for (int i = 0; i < RM; ++i) af[pc][i] = read_frag_bf16<BM, AMC>(As, wm * TM + i * 16, pc, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[pc][j] = read_frag_bf16<BN, BMC>(Bs, wn * TN + j * 16, pc, lane);
      }
      if (kt + S - 1 < nt) {
        la.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE, tid);
        lb.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE + ABYTES, tid);
      }
#pragma unroll
      for (int pc = 0; pc < 2; ++pc)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
          for (int j = 0; j < RN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[pc][i], bfr[pc][j], acc[i][j], 0, 0, 0);
    } else {
      if (kt + S - 1 < nt) {
        la.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE, tid);
        lb.issue(kbeg + (kt + S - 1) * BK, smem + NXT * STAGE + ABYTES, tid);
      }
      mma_tile(As, Bs);
    }
    // tile kt+1 must have landed (for every wave: counted wait, then the barrier); the
    // min(nt-1, kt+S-1) - (kt+1) younger tiles stay in flight
    wait_tiles<G>(min(nt - 1, kt + S - 1) - (kt + 1));
    raw_barrier();
  };
  constexpr bool PPK = PP == 1 && sizeof(T) == 2 && !AMC && !BMC && WM * WN == 8;
  if constexpr (PPK) {
    const bool g1 = __builtin_amdgcn_readfirstlane(wave) >= 4;   // waves w, w + 4 share a SIMD
    auto phase_mma = [&](const bf16x8 (&af)[RM], const bf16x8 (&bfr)[RN]) {
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      __builtin_amdgcn_sched_barrier(0);
      raw_barrier();
    };
    auto refill = [&](int kt, int nxt) {
      la.issue(kbeg + (kt + S - 1) * BK, smem + nxt * STAGE, tid);
      lb.issue(kbeg + (kt + S - 1) * BK, smem + nxt * STAGE + ABYTES, tid);
    };
    auto kstep_pp = [&](int kt, auto stg_c) {
      constexpr int STG = decltype(stg_c)::value;
      constexpr int NXT = (STG + S - 1) % S;
      const char* As = smem + STG * STAGE;
      const char* Bs = As + ABYTES;
      {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = read_frag_bf16<BM, false>(As, wm * TM + i * 16, 0, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = read_frag_bf16<BN, false>(Bs, wn * TN + j * 16, 0, lane);
        if (S == 2 && kt + S - 1 < nt) refill(kt, NXT);
        phase_mma(af, bfr);
      }
      {
        bf16x8 af[RM], bfr[RN];
#pragma unroll
        for (int i = 0; i < RM; ++i) af[i] = read_frag_bf16<BM, false>(As, wm * TM + i * 16, 1, lane);
#pragma unroll
        for (int j = 0; j < RN; ++j) bfr[j] = read_frag_bf16<BN, false>(Bs, wn * TN + j * 16, 1, lane);
        if (S > 2 && kt + S - 1 < nt) refill(kt, NXT);
        wait_tiles<G>(min(nt - 1, kt + S - 1) - (kt + 1));
        // 2-stage ring: the next step's first phase refills this tile's stage, so this phase's
        // reads must have retired before the barrier (the deeper rings refill two barriers later)
        if constexpr (S == 2) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        phase_mma(af, bfr);
      }
    };
    if (g1) raw_barrier();
    for (int kt = 0; kt < nt; kt += S) {
      kstep_pp(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nt) kstep_pp(kt + 1, std::integral_constant<int, 1>{});
      if constexpr (S > 2) { if (kt + 2 < nt) kstep_pp(kt + 2, std::integral_constant<int, (S > 2 ? 2 : 0)>{}); }
      if constexpr (S > 3) { if (kt + 3 < nt) kstep_pp(kt + 3, std::integral_constant<int, (S > 3 ? 3 : 0)>{}); }
    }
    if (!g1) raw_barrier();
  } else {
    for (int kt = 0; kt < nt; kt += S) {
      kstep(kt, std::integral_constant<int, 0>{});
      if (kt + 1 < nt) kstep(kt + 1, std::integral_constant<int, 1>{});
      if constexpr (S > 2) { if (kt + 2 < nt) kstep(kt + 2, std::integral_constant<int, (S > 2 ? 2 : 0)>{}); }
      if constexpr (S > 3) { if (kt + 3 < nt) kstep(kt + 3, std::integral_constant<int, (S > 3 ? 3 : 0)>{}); }
    }
  }

  // Epilogue: stage alpha*acc (fp32) through LDS, HR tile rows per pass, as [HR][BN+4]; then
  // every thread writes 8 consecutive columns of a row (16-B bf16 / 2x16-B fp32 stores, or 8
  // contiguous atomics).  Lane holds C[4g + r][l & 15] of each 16x16 block.
  // BN epilogues (st_mode, gemm.h) accumulate per-column partials of the stored values in the
  // same loop (registers), reduced over the block in a fixed order at the end.
  float* cs = (float*)smem;
  float alpha = p.alpha;
  {
    const float* sa = p.scale_a;
    const float* sb = p.scale_b;
    if (p.ngroup && p.grp.SA[batch]) { sa = p.grp.SA[batch]; sb = p.grp.SB[batch]; }
    if (sa) alpha *= *sa;
    if (sb) alpha *= *sb;
  }
  const int cmode = p.c_mode == 3 ? 0 : p.c_mode;
  float sk[8], sa1[8], sa2[8], sb1[8], sb2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { sk[e] = 0.f; sa1[e] = sa2[e] = sb1[e] = sb2[e] = 0.f; }
  int segA_end = 0x7fffffff;
  if constexpr (smode == 1) segA_end = (m0 / p.st_seg_rows + 1) * p.st_seg_rows;
  if constexpr (smode == 2 && !EARLY) epi_affine();
#pragma unroll 1
  for (int pass = 0; pass < BM / HR; ++pass) {
    // EARLY: this pass's rows were prefetched (before the K loop / during the previous pass) and
    // the next pass's loads go out now.  Otherwise this pass's loads go out now, in flight while
    // the accumulators are staged through LDS.
    u32x4 xpf[(smode == 2 || PFC) ? IT * PQ : 1];
    if constexpr (EARLY) {
#pragma unroll
      for (int i = 0; i < IT * PQ; ++i) xpf[i] = xnx[i];
      if (pass + 1 < BM / HR) epi_fetch(pass + 1);
    } else if constexpr (smode == 2) {
      epi_fetch(pass);
#pragma unroll
      for (int i = 0; i < IT * PQ; ++i) xpf[i] = xnx[i];
    }
    {
      const int g = lane >> 4;
      // KSG: group 1 stages its partial tile, group 0 adds its own on top (one pass: HR == BM)
#pragma unroll
      for (int grp = 0; grp < (KSG ? 2 : 1); ++grp) {
        if (!KSG || kg == 1 - grp) {
#pragma unroll
          for (int i = 0; i < RM; ++i) {
            const int rb = wm * TM + i * 16 - pass * HR;  // block's first row within this pass
            if (rb < 0 || rb >= HR) continue;
#pragma unroll
            for (int j = 0; j < RN; ++j)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                float* c = &cs[(rb + 4 * g + r) * LDC + wn * TN + j * 16 + (lane & 15)];
                if (KSG && grp == 1) *c += acc[i][j][r] * alpha;
                else *c = acc[i][j][r] * alpha;
              }
          }
        }
        if (KSG && grp == 0) __syncthreads();
      }
    }
    __syncthreads();
    if (smode == 1 && pass == 0) {  // per-tile shift: the tile's first row (with bias)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int c = n0 + c0t + e;
        sk[e] = cs[c0t + e] + ((bias && c < p.N) ? bias[c] : 0.f);
      }
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      const int rr = tid / GPR + it * RPP;
      const int row = m0 + pass * HR + rr;
      if (row >= p.M) continue;
      long long drow = row;
      if (p.row_map == 1) {  // stride-2 dgrad scatter: row over (n, oy, ox) -> (n, 2oy, 2ox)
        int im, rem, oy, ox;
        fdivmod(row, p.rm_div_OHW, im, rem);
        fdivmod(rem, p.rm_div_OW, oy, ox);
        drow = ((long long)im * p.rm_H + 2 * oy) * p.rm_W + 2 * ox;
      }
      const int c0 = c0t;
      const int col = n0 + c0;
      if (col >= p.N) continue;
      float v[8];
      *(f32x4*)&v[0] = *(const f32x4*)&cs[rr * LDC + c0];
      *(f32x4*)&v[4] = *(const f32x4*)&cs[rr * LDC + c0 + 4];
      CT* dst = Cb + drow * p.ldc + col;
      const bool full = col + 8 <= p.N && ((uintptr_t)dst % 16 == 0);
      if (bias) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += (col + e < p.N) ? bias[col + e] : 0.f;
      }
      if (cmode == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < p.N) store_c<CT>(dst + e, v[e], 1);
      } else if (full) {
        if constexpr (sizeof(CT) == 2) {
          if (cmode == 2) {
            float q[8];
            if constexpr (PFC) Chunk<bf16>::unpack(xpf[it], q);   // prefetched (same condition)
            else Chunk<bf16>::unpack(*(const u32x4*)dst, q);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] += q[e];
          }
          const u32x4 pk = Chunk<bf16>::pack(v);
          if (p.wt == 4)
            __builtin_nontemporal_store(pk, (u32x4*)dst);
          else if (p.wt)
            __builtin_amdgcn_raw_buffer_store_b128(pk, crs, (int)(((long long)(row - m0) * p.ldc + col) * 2), 0, 16);
          else
            *(u32x4*)dst = pk;
          if (smode) Chunk<bf16>::unpack(pk, v);  // statistics of the values as stored
        } else {
          if (cmode == 2) {
            f32x4 q0 = *(const f32x4*)dst, q1 = *(const f32x4*)(dst + 4);
#pragma unroll
            for (int e = 0; e < 4; ++e) { v[e] += q0[e]; v[4 + e] += q1[e]; }
          }
          if (p.wt == 4) {
            __builtin_nontemporal_store(*(f32x4*)&v[0], (f32x4*)dst);
            __builtin_nontemporal_store(*(f32x4*)&v[4], (f32x4*)(dst + 4));
          } else if (p.wt) {
            const int off = (int)(((long long)(row - m0) * p.ldc + col) * 4);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *(f32x4*)&v[0]), crs, off, 0, 16);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, *(f32x4*)&v[4]), crs, off + 16, 0, 16);
          } else {
            *(f32x4*)dst = *(f32x4*)&v[0];
            *(f32x4*)(dst + 4) = *(f32x4*)&v[4];
          }
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (col + e < p.N) {
            store_c<CT>(dst + e, v[e], cmode);
            v[e] = tof((CT)v[e]);
          }
      }
#ifndef CN_EPI_NOACC
      if constexpr (smode == 1) {
        const bool inA = row < segA_end;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = (col + e < p.N) ? v[e] - sk[e] : 0.f;
          if (inA) { sa1[e] += d; sa2[e] = fmaf(d, d, sa2[e]); }
          else { sb1[e] += d; sb2[e] = fmaf(d, d, sb2[e]); }
        }
      } else if constexpr (smode == 2) {
        float xv[8];
        if (full) {
          if constexpr (sizeof(CT) == 2) Chunk<bf16>::unpack(xpf[it], xv);
          else { *(u32x4*)&xv[0] = xpf[2 * it]; *(u32x4*)&xv[4] = xpf[2 * it + 1]; }
        } else {
          const CT* xs = (const CT*)p.br_x + (long long)row * p.br_ldx + col;
#pragma unroll
          for (int e = 0; e < 8; ++e) xv[e] = (col + e < p.N) ? tof(xs[e]) : 0.f;
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // sum dz * (x - mu); the invstd factor of xh is applied once per column at the end
          float dd = (col + e < p.N && fmaf(xv[e], bk1[e], bsf[e]) > 0.f) ? v[e] : 0.f;
          sa1[e] += dd;
          sa2[e] = fmaf(dd, xv[e] - bmu[e], sa2[e]);
        }
      }
#endif
    }
    __syncthreads();
  }
#ifdef CN_EPI_NORED
  if constexpr (false) {
#else
  if constexpr (smode != 0) {
#endif
    // Column partials: lanes sharing this thread's column group (lane ^ GPR, ^2 GPR, ...) by
    // shuffles, then the waves in order through LDS; one row of each plane per M-tile.
    constexpr int NW = NT / 64;
    const int nq = smode == 1 ? 4 : 2;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
#pragma unroll
      for (int o = GPR; o < 64; o <<= 1) {
        sa1[e] += __shfl_xor(sa1[e], o, 64);
        sa2[e] += __shfl_xor(sa2[e], o, 64);
        if (smode == 1) {
          sb1[e] += __shfl_xor(sb1[e], o, 64);
          sb2[e] += __shfl_xor(sb2[e], o, 64);
        }
      }
    }
    float* red = cs;  // [NW][4][BN]
    if (lane < GPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(wave * 4 + 0) * BN + c0t + e] = sa1[e];
        red[(wave * 4 + 1) * BN + c0t + e] = sa2[e];
        red[(wave * 4 + 2) * BN + c0t + e] = sb1[e];
        red[(wave * 4 + 3) * BN + c0t + e] = sb2[e];
      }
    }
    __syncthreads();
    float* ws = ((p.ngroup && p.grp.ST[batch]) ? p.grp.ST[batch] : p.st_ws) + (long long)tm * p.N;
    for (int t = tid; t < nq * BN; t += NT) {
      const int q = t / BN, c = t % BN;
      float a = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) a += red[(w * 4 + q) * BN + c];
      if (smode == 2 && q == 1 && n0 + c < p.N) a *= p.br_invstd[n0 + c];
      if (n0 + c < p.N) ws[(long long)(smode == 1 ? q + 1 : q) * p.st_plane + n0 + c] = a;
    }
    if (smode == 1 && tid < GPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (n0 + c0t + e < p.N) ws[n0 + c0t + e] = sk[e];
    }
  }
}

// ---------------------------------------------------------------------------------------
// Tile configurations and dispatch.  grid = (ceil(M/BM), ceil(N/BN), batch * nsplit)
// ---------------------------------------------------------------------------------------
struct TileCfg { int bm, bn, wm, wn, s, pp; };
// bf16 configurations (index = config id); fp32 (parity path) always uses id 1's tile with S=2
static constexpr TileCfg kCfg[] = {
    {128, 64, 2, 2, 2},   // 0: small grids
    {128, 128, 2, 2, 2},  // 1
    {128, 128, 2, 2, 3},  // 2
    {256, 128, 4, 2, 3},  // 3
    {128, 256, 2, 4, 3},  // 4
    {256, 256, 2, 4, 2},  // 5
    {128, 64, 2, 2, 4},   // 6
    {128, 128, 2, 2, 4},  // 7
    {256, 128, 4, 2, 2},  // 8
    {128, 256, 2, 4, 2},  // 9
    {256, 256, 4, 2, 2},  // 10
    {128, 128, 4, 2, 2},  // 11: 8 waves of 32x64
    {128, 64, 4, 2, 2},   // 12: 8 waves of 32x32
    {128, 128, 4, 2, 3},  // 13: 8 waves, 3-deep ring
    {128, 128, 4, 2, 4},  // 14: 8 waves, 4-deep ring
    {256, 128, 4, 2, 3},  // 15
    {128, 64, 4, 2, 4},   // 16
    {64, 128, 2, 4, 2},   // 17: 8 waves of 32x32, for 64-row products (Cout = 64 wgrad)
    {256, 128, 4, 2, 3, 1},  // 18: ping-pong, 8 waves of 64x64
    {128, 256, 2, 4, 3, 1},  // 19: ping-pong, 8 waves of 64x64
    {256, 256, 2, 4, 2, 1},  // 20: ping-pong, 8 waves of 128x64
    // round 4: 4 waves (one per SIMD) with larger wave tiles -- fewer LDS fragment bytes per FLOP
    // (1/TM + 1/TN), the contention the fill probe measures
    {128, 256, 2, 2, 3},  // 21: 4 waves of 64x128
    {256, 128, 2, 2, 3},  // 22: 4 waves of 128x64
    {256, 256, 2, 2, 2},  // 23: (4 waves of 128x128 spill 36-151 VGPRs; launches config 10)
    {128, 256, 1, 4, 3, 2},  // 24: KSG, 2 groups x 4 waves of 128x64
    {128, 256, 2, 2, 3, 2},  // 25: KSG, 2 groups x 4 waves of 64x128
};
constexpr int kNumCfg = sizeof(kCfg) / sizeof(kCfg[0]);
static int g_force_cfg = -1;

static long long cfg_blocks(int c, const GemmArgs& a, int batch) {
  return (long long)((a.M + kCfg[c].bm - 1) / kCfg[c].bm) * ((a.N + kCfg[c].bn - 1) / kCfg[c].bn) *
         batch * a.nsplit;
}

// Shape heuristic (tools/fwd_sweep.sh / wgrad_sweep.sh / gemm_cold.py on the step's conv
// shapes, operands cold in HBM as in the step): 128x64 for N <= 64; 256x256 for wide, deep
// products (N >= 512 and K >= 2048: the ASPP atrous convs, layer-4) when that still gives ~200+
// blocks (the frame-batch layer-4 dgrad at 114 blocks runs 76 vs 120 us on 128x128); where
// 128x128 leaves at most one block per CU (frame-batch layer-3 dgrads: 226 blocks) the 3-deep
// ring hides the HBM latency a second resident block would (29 vs 38 us, 16 vs 21 us);
// 128x128 with 8 waves (32x64 per wave) everywhere else.
static long long tiles_of(int c, int M, int N) {
  return (long long)((M + kCfg[c].bm - 1) / kCfg[c].bm) * ((N + kCfg[c].bn - 1) / kCfg[c].bn);
}
// Round 3 (profiles/r03_gemm_cold_pingpong*.txt): the ping-pong tiles take the wide deep products
// (256x256, ASPP / layer-4 3x3: -2..-4 %) and the N = 256 frame-pair products with K >= 1024
// (128x256: layer-3 3x3 fwd -7 %, 1x1 1024->256 fwd -9 %); 256x256 (8 waves of 64x128) also
// takes the shallow N >= 1024 products (256->1024 fwd -7 %).  Transposed-operand (MC) products
// picked for a ping-pong tile run its plain twin (launch_tile).  CN_GEMM_HEUR=1 selects the
// round-2 rules (A/B runs).
static int heuristic_cfg(int M, int N, int K, int bz) {
  static const int v1 = [] { const char* e = getenv("CN_GEMM_HEUR"); return e && e[0] == '1'; }();
  if (N <= 64) return 12;
  if (v1) {
    if (N >= 512 && K >= 2048 && tiles_of(10, M, N) * bz >= 200) return 10;
    if (tiles_of(11, M, N) * bz <= 256 && K >= 512) return 13;
    return 11;
  }
  if (N >= 512 && K >= 2048 && tiles_of(10, M, N) * bz >= 200) return 20;
  if (tiles_of(11, M, N) * bz <= 256 && K >= 512) return 13;
  // Round 4: 128x128 / 8 waves for these products (layer-3 3x3 fwd 38 vs 46 us, 1x1 fwd 22 vs 25
  // us isolated; whole step +0.2 %: profiles/r04_gemm_n256_tiles_ab.txt).  CN_GEMM_N256 overrides
  // it for A/B runs (19 = the round-3 128x256 ping-pong, 24 / 25 = K-split wave groups).
  static const int n256 = [] { const char* e = getenv("CN_GEMM_N256"); const int v = e ? atoi(e) : 11; return (v >= 21 && !CN_EXPERIMENTAL) ? 11 : v; }();
  if (N == 256 && K >= 1024 && tiles_of(19, M, N) * bz >= 200) return n256;
  // shallow wide products (1x1 convs with K <= 512 into >= 1024 channels): 256x256 by the
  // round-3 isolated sweep; CN_GEMM_SHALLOW overrides it for in-step A/B runs
  static const int shallow = [] { const char* e = getenv("CN_GEMM_SHALLOW"); return e ? atoi(e) : 10; }();
  if (N >= 1024 && K <= 512 && tiles_of(10, M, N) * bz >= 200) return shallow;
  return 11;
}

static int pick_cfg(const GemmArgs& a, int batch) {
  if (g_force_cfg >= 0 && g_force_cfg < kNumCfg) return g_force_cfg;
  if (a.cfg >= 0 && a.cfg < kNumCfg) return a.cfg;
  return heuristic_cfg(a.M, a.N, a.K, batch * a.nsplit);
}

template <class T, class CT, int C, int LA, int LB, int EPI = 0>
static int launch_c(const GemmArgs& a, int batch, hipStream_t st) {
  constexpr TileCfg c = kCfg[C];
  dim3 grid((a.M + c.bm - 1) / c.bm, (a.N + c.bn - 1) / c.bn, batch * a.nsplit);
  hipLaunchKernelGGL((gemm_kernel<T, CT, c.bm, c.bn, c.wm, c.wn, c.s, LA, LB, EPI, c.pp>), grid,
                     dim3(c.wm * c.wn * 64 * (c.pp == 2 ? 2 : 1)), 0, st, a);
  CN_CHECK_LAUNCH();
  return 0;
}

// BN-epilogue GEMMs (conv fwd with statistics, stride-1 dgrad with the BN backward reduce):
// only the tiles the shape heuristic picks for conv fwd / dgrad are instantiated.
template <class T, int LA, int EPI>
static int launch_epi(const GemmArgs& a, int batch, hipStream_t st) {
  if constexpr (sizeof(T) == 4) {
    if (a.N <= 64 || cfg_blocks(1, a, batch) < 384) return launch_c<T, T, 0, LA, L_KC_DENSE, EPI>(a, batch, st);
    return launch_c<T, T, 1, LA, L_KC_DENSE, EPI>(a, batch, st);
  } else {
    switch (pick_cfg(a, batch)) {
      case 10: return launch_c<T, T, 10, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 11: return launch_c<T, T, 11, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 12: return launch_c<T, T, 12, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 13: return launch_c<T, T, 13, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 18: return launch_c<T, T, 18, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 19: return launch_c<T, T, 19, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 20: return launch_c<T, T, 20, LA, L_KC_DENSE, EPI>(a, batch, st);
#if CN_EXPERIMENTAL
      case 21: return launch_c<T, T, 21, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 22: return launch_c<T, T, 22, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 24: return launch_c<T, T, 24, LA, L_KC_DENSE, EPI>(a, batch, st);
      case 25: return launch_c<T, T, 25, LA, L_KC_DENSE, EPI>(a, batch, st);
#endif
      default: return CN_ERR_UNSUPPORTED;
    }
  }
}

// Read-add-store launches (c_mode 2, bf16 C: a dgrad accumulating into the residual gradient)
// take the EPI 3 epilogue, whose old C rows are prefetched before the K loop.  CN_GEMM_PFC=0
// keeps the plain epilogue (A/B runs).
static bool pfc_on() {
  static const bool on = [] { const char* e = getenv("CN_GEMM_PFC"); return !(e && e[0] == '0'); }();
  return on;
}

template <class T, class CT, int LA, int LB>
static int launch_tile(const GemmArgs& a, int batch, hipStream_t st) {
  if constexpr (sizeof(T) == 2 && sizeof(CT) == 2 && (LA == L_KC_DENSE || LA == L_KC_CONV) &&
                LB == L_KC_DENSE) {
    if (a.c_mode == 2 && !a.row_map && !a.ngroup && pfc_on()) {
      switch (pick_cfg(a, batch)) {
        case 10: return launch_c<T, CT, 10, LA, LB, 3>(a, batch, st);
        case 11: return launch_c<T, CT, 11, LA, LB, 3>(a, batch, st);
        case 12: return launch_c<T, CT, 12, LA, LB, 3>(a, batch, st);
        case 13: return launch_c<T, CT, 13, LA, LB, 3>(a, batch, st);
        case 20: return launch_c<T, CT, 20, LA, LB, 3>(a, batch, st);
        default: break;
      }
    }
  }
  if constexpr (sizeof(T) == 4) {
    if (a.N <= 64 || cfg_blocks(1, a, batch) < 384) return launch_c<T, CT, 0, LA, LB>(a, batch, st);
    return launch_c<T, CT, 1, LA, LB>(a, batch, st);
  } else {
    switch (pick_cfg(a, batch)) {
      case 0: return launch_c<T, CT, 0, LA, LB>(a, batch, st);
      case 1: return launch_c<T, CT, 1, LA, LB>(a, batch, st);
      case 2: return launch_c<T, CT, 2, LA, LB>(a, batch, st);
      case 3: return launch_c<T, CT, 3, LA, LB>(a, batch, st);
      case 4: return launch_c<T, CT, 4, LA, LB>(a, batch, st);
      case 5: return launch_c<T, CT, 5, LA, LB>(a, batch, st);
      case 6: return launch_c<T, CT, 6, LA, LB>(a, batch, st);
      case 7: return launch_c<T, CT, 7, LA, LB>(a, batch, st);
      case 8: return launch_c<T, CT, 8, LA, LB>(a, batch, st);
      case 9: return launch_c<T, CT, 9, LA, LB>(a, batch, st);
      case 10: return launch_c<T, CT, 10, LA, LB>(a, batch, st);
      case 11: return launch_c<T, CT, 11, LA, LB>(a, batch, st);
      case 13: return launch_c<T, CT, 13, LA, LB>(a, batch, st);
      case 14: return launch_c<T, CT, 14, LA, LB>(a, batch, st);
      case 15: return launch_c<T, CT, 15, LA, LB>(a, batch, st);
      case 16: return launch_c<T, CT, 16, LA, LB>(a, batch, st);
      case 17: return launch_c<T, CT, 17, LA, LB>(a, batch, st);
#if CN_EXPERIMENTAL
      case 21: return launch_c<T, CT, 21, LA, LB>(a, batch, st);
      case 22: return launch_c<T, CT, 22, LA, LB>(a, batch, st);
      case 23: return launch_c<T, CT, 10, LA, LB>(a, batch, st);   // 4 waves of 128x128 spill: not built
      case 24: case 25: {  // K-split wave groups: k-contiguous operands only
        constexpr bool kc = LA != L_MC_DENSE && LA != L_MC_CONV && LB != L_MC_DENSE && LB != L_MC_CONV;
        if constexpr (kc) {
          if (pick_cfg(a, batch) == 24) return launch_c<T, CT, 24, LA, LB>(a, batch, st);
          return launch_c<T, CT, 25, LA, LB>(a, batch, st);
        } else {
          return launch_c<T, CT, 11, LA, LB>(a, batch, st);
        }
      }
#endif
      case 18: case 19: case 20: {  // ping-pong tiles: k-contiguous operands only
        constexpr bool kc = LA != L_MC_DENSE && LA != L_MC_CONV && LB != L_MC_DENSE && LB != L_MC_CONV;
        if constexpr (kc) {
          const int c = pick_cfg(a, batch);
          if (c == 18) return launch_c<T, CT, 18, LA, LB>(a, batch, st);
          if (c == 19) return launch_c<T, CT, 19, LA, LB>(a, batch, st);
          return launch_c<T, CT, 20, LA, LB>(a, batch, st);
        } else {
          if (pick_cfg(a, batch) == 20) return launch_c<T, CT, 10, LA, LB>(a, batch, st);
          return launch_c<T, CT, 11, LA, LB>(a, batch, st);
        }
      }
      default: return launch_c<T, CT, 12, LA, LB>(a, batch, st);
    }
  }
}

// conv gathers whose K tiles straddle taps (C % BK != 0: the 8-channel padded stems): the
// tiles the heuristic picks for those shapes only
template <class T, class CT>
static int launch_conv_g(const GemmArgs& a, int batch, hipStream_t st) {
  if constexpr (sizeof(T) == 4) {
    if (a.N <= 64 || cfg_blocks(1, a, batch) < 384) return launch_c<T, CT, 0, L_KC_CONV_G, L_KC_DENSE>(a, batch, st);
    return launch_c<T, CT, 1, L_KC_CONV_G, L_KC_DENSE>(a, batch, st);
  } else {
    const int c = pick_cfg(a, batch);
    if (c == 12) return launch_c<T, CT, 12, L_KC_CONV_G, L_KC_DENSE>(a, batch, st);
    if (c == 13) return launch_c<T, CT, 13, L_KC_CONV_G, L_KC_DENSE>(a, batch, st);
    return launch_c<T, CT, 11, L_KC_CONV_G, L_KC_DENSE>(a, batch, st);
  }
}

template <class T, class CT>
static int launch_kinds(const GemmArgs& a, int la, int lb, int batch, hipStream_t st) {
#define CN_CASE(A_, B_) \
  if (la == A_ && lb == B_) return launch_tile<T, CT, A_, B_>(a, batch, st);
  if (la == L_KC_CONV_G && lb == L_KC_DENSE) return launch_conv_g<T, CT>(a, batch, st);
  CN_CASE(L_KC_DENSE, L_KC_DENSE)
  CN_CASE(L_KC_CONV, L_KC_DENSE)
  CN_CASE(L_KC_DENSE, L_MC_DENSE)
  CN_CASE(L_MC_DENSE, L_MC_DENSE)
  CN_CASE(L_MC_DENSE, L_MC_CONV)
#undef CN_CASE
  return -10;  // unsupported loader combination
}

// fp8 (e4m3) operands: k-contiguous loaders only (conv forward / dgrad / dense products), the
// three tiles the shape heuristic uses; 128 fp8 per 128-byte K tile, one scaled MFMA per tile.
template <class CT, int LA, class T8 = f8e4m3>
static int launch_f8(const GemmArgs& a, int batch, hipStream_t st) {
  // (the 256x256 tile would spill its fp8 fragments: 128x128 serves the wide products too).
  // Round 6: CN_GEMM_F8BIG = 8 (256x128) or 9 (128x256), 8 waves of 64x64 -- a quarter fewer LDS
  // fill bytes per FLOP than 128x128 -- for the products with >= 256 such tiles (A/B runs).
  static const int big = [] { const char* e = getenv("CN_GEMM_F8BIG"); return e ? atoi(e) : 0; }();
  const int c = pick_cfg(a, batch);
  if constexpr (sizeof(CT) == 2 && std::is_same<T8, f8e4m3>::value) {
    // fp8 conv forward with the BN-statistics epilogue (round 6; the bf16 path's EPI 1)
    if (a.st_mode == 1) {
      if (c == 12) return launch_c<T8, CT, 12, LA, L_KC_DENSE, 1>(a, batch, st);
      if (c == 13) return launch_c<T8, CT, 13, LA, L_KC_DENSE, 1>(a, batch, st);
      return launch_c<T8, CT, 11, LA, L_KC_DENSE, 1>(a, batch, st);
    }
  }
  if (a.st_mode) return CN_ERR_UNSUPPORTED;
  if ((big == 8 || big == 9) && c != 12 && tiles_of(big, a.M, a.N) * batch >= 256) {
    if (big == 8) return launch_c<T8, CT, 8, LA, L_KC_DENSE>(a, batch, st);
    return launch_c<T8, CT, 9, LA, L_KC_DENSE>(a, batch, st);
  }
  if (c == 12) return launch_c<T8, CT, 12, LA, L_KC_DENSE>(a, batch, st);
  if (c == 13) return launch_c<T8, CT, 13, LA, L_KC_DENSE>(a, batch, st);
  return launch_c<T8, CT, 11, LA, L_KC_DENSE>(a, batch, st);
}

// fp8 weight gradients (e5m2 dY MC_DENSE x e4m3 X MC_DENSE / MC_CONV, fp32 dW or split-K slabs):
// 128x128 tiles (the MC fp8 reader's 128-byte k-rows), 2- or 3-deep ring (cfg 11 / 13).
template <int LB>
static int launch_f8_mc(const GemmArgs& a, int batch, hipStream_t st) {
  if (a.cfg == 13) return launch_c<f8e5m2, float, 13, L_MC_DENSE, LB>(a, batch, st);
  return launch_c<f8e5m2, float, 11, L_MC_DENSE, LB>(a, batch, st);
}

// 32-bit byte-offset limits of the buffer-descriptor loaders (Loader, BUF path)
static bool buf_ok(int kind, const GemmArgs& a, bool is_a, int esz) {
  const long long ld = is_a ? a.lda : a.ldb;
  const ConvGeom& g = is_a ? a.ga : a.gb;
  const long long kspan = a.nsplit > 1 ? a.k_chunk : a.K;
  if (kind == L_KC_DENSE) return 256 * ld * esz < 0x80000000ll && (long long)a.K * esz < 0xFFFF0000ll;
  if (kind == L_KC_CONV) return (long long)g.N * g.H * g.W * ld * esz < 0x80000000ll;
  if (kind == L_MC_DENSE) return (kspan + 128) * ld * esz < 0xFFFF0000ll && 128 * ld * esz < 0x80000000ll;
  return true;
}

// C store policy.  Default (CN_GEMM_WT=4): non-temporal (nt) stores of C -- the split-K slabs,
// which the reduce kernel reads back, excepted -- +0.5 % on the step (profiles/r06_write_through_ab.txt:
// the lines leave the L2 early instead of waiting dirty for the end-of-launch write-back).  A/B
// variants: 0 plain stores; 1 write-through (sc1) for every C store (-0.4 %); 3 write-through for the
// split-K slabs only (-1.4 %).
static int wt_on() {
  static const int lvl = [] { const char* e = getenv("CN_GEMM_WT"); return e ? atoi(e) : 4; }();
  return lvl;
}

int cn_gemm_dispatch(const GemmArgs& a_in, int dtype, int c_f32, int la, int lb, int batch, hipStream_t st) {
  GemmArgs a = a_in;
  // per-block 32-bit offsets from the block's first row: not for the stride-2 row scatter
  a.wt = wt_on() == 4 ? (a.c_mode != 1 && a.c_mode != 3 ? 4 : 0)
                      : !a.row_map && a.c_mode != 1 && (wt_on() == 1 || (wt_on() == 3 && a.c_mode == 3));
  if (a.M <= 0 || a.N <= 0 || batch <= 0) return 0;
  const int esz = (dtype == DT_FP8 || dtype == DT_FP8_E5M2) ? 1 : dtype == DT_BF16 ? 2 : 4;
  const int bk = 128 / esz;
  // conv gathers whose K tiles can straddle taps, or too large for 32-bit offsets: per-thread
  // pointer loader
  if (la == L_KC_CONV && (a.ga.C % bk != 0 || !buf_ok(L_KC_CONV, a, true, esz))) la = L_KC_CONV_G;
  if (!buf_ok(la, a, true, esz) || !buf_ok(lb, a, false, esz)) return CN_ERR_SHAPE;
  if (dtype == DT_FP8) {
    if (lb != L_KC_DENSE || a.nsplit != 1) return CN_ERR_UNSUPPORTED;
    if (a.st_mode && (a.st_mode != 1 || batch != 1 || a.row_map || a.c_mode || c_f32)) return CN_ERR_UNSUPPORTED;
    if (la == L_KC_DENSE) return c_f32 ? launch_f8<float, L_KC_DENSE>(a, batch, st) : launch_f8<bf16, L_KC_DENSE>(a, batch, st);
    if (la == L_KC_CONV) return c_f32 ? launch_f8<float, L_KC_CONV>(a, batch, st) : launch_f8<bf16, L_KC_CONV>(a, batch, st);
    if (la == L_KC_CONV_G) return c_f32 ? launch_f8<float, L_KC_CONV_G>(a, batch, st) : launch_f8<bf16, L_KC_CONV_G>(a, batch, st);
    return CN_ERR_UNSUPPORTED;
  }
  if (dtype == DT_FP8_E5M2 && la == L_MC_DENSE) {   // wgrad: e5m2 dY (k-major) x e4m3 X, fp32 dW
    if (!c_f32 || a.st_mode || a.row_map || a.c_mode == 1 || a.c_mode == 2) return CN_ERR_UNSUPPORTED;
    if (lb == L_MC_DENSE) return launch_f8_mc<L_MC_DENSE>(a, batch, st);
    if (lb == L_MC_CONV) return launch_f8_mc<L_MC_CONV>(a, batch, st);
    return CN_ERR_UNSUPPORTED;
  }
  if (dtype == DT_FP8_E5M2) {   // dgrad: e5m2 output gradients x e4m3 transposed weights, bf16 dX
    if (lb != L_KC_DENSE || a.st_mode || a.nsplit != 1 || c_f32) return CN_ERR_UNSUPPORTED;
    if (la == L_KC_DENSE) return launch_f8<bf16, L_KC_DENSE, f8e5m2>(a, batch, st);
    if (la == L_KC_CONV) return launch_f8<bf16, L_KC_CONV, f8e5m2>(a, batch, st);
    if (la == L_KC_CONV_G) return launch_f8<bf16, L_KC_CONV_G, f8e5m2>(a, batch, st);
    return CN_ERR_UNSUPPORTED;
  }
  if (a.st_mode) {
    // grouped (EPI 1 only): one problem per blockIdx.z, each with its own statistics workspace
    if ((batch != 1 && !(a.ngroup == batch && a.st_mode == 1)) || a.nsplit != 1 || a.row_map || a.c_mode ||
        lb != L_KC_DENSE || (la != L_KC_DENSE && la != L_KC_CONV && la != L_KC_CONV_G))
      return CN_ERR_UNSUPPORTED;
#define CN_EPI(T_, M_) \
    return la == L_KC_DENSE ? launch_epi<T_, L_KC_DENSE, M_>(a, batch, st) : \
           la == L_KC_CONV ? launch_epi<T_, L_KC_CONV, M_>(a, batch, st) : launch_epi<T_, L_KC_CONV_G, M_>(a, batch, st)
    if (dtype == DT_BF16) {
      if (a.st_mode == 1) CN_EPI(bf16, 1); else CN_EPI(bf16, 2);
    } else {
      if (a.st_mode == 1) CN_EPI(float, 1); else CN_EPI(float, 2);
    }
#undef CN_EPI
  }
  if (dtype == DT_BF16) {
    return c_f32 ? launch_kinds<bf16, float>(a, la, lb, batch, st)
                 : launch_kinds<bf16, bf16>(a, la, lb, batch, st);
  } else if (dtype == DT_F32) {
    return launch_kinds<float, float>(a, la, lb, batch, st);
  }
  return -11;
}

int cn_gemm_bm(int dtype, int M, int N, int K, int cfg) {
  if (dtype != DT_BF16) return kCfg[1].bm;  // the fp32 path: configs 0 / 1 (both 128 rows)
  if (g_force_cfg >= 0 && g_force_cfg < kNumCfg) return kCfg[g_force_cfg].bm;
  if (cfg >= 0 && cfg < kNumCfg) return kCfg[cfg].bm;
  return kCfg[heuristic_cfg(M, N, K, 1)].bm;
}

int cn_gemm_pick(int M, int N, int K, int batch_splits) {
  if (g_force_cfg >= 0 && g_force_cfg < kNumCfg) return g_force_cfg;
  return heuristic_cfg(M, N, K, batch_splits);
}

long long cn_gemm_cfg_blocks(int cfg, int M, int N) {
  GemmArgs a = {};
  a.M = M; a.N = N; a.nsplit = 1;
  return cfg_blocks(cfg, a, 1);
}

// Development hook: force one tile configuration for every bf16 launch (-1 = heuristic).
extern "C" int cn_gemm_force_config(int cfg) {
  if (cfg >= kNumCfg || (!CN_EXPERIMENTAL && cfg >= 21)) return -1;
  g_force_cfg = cfg;
  return kNumCfg;
}

// Split-K reduction: out[i] (+)= sum_s ws[s * slab + i]  (fp32, float4-vectorised).  A block
// = (256 / G) float4 outputs x G slab groups: group g sums slabs g, g + G, ... (8 loads in
// flight), then the G partials are added in group order through LDS -- a fixed order, so the
// result is bitwise reproducible.  G grows when the output is small and the slabs many (the
// layer-1 weight gradients: 16 K outputs x 110 slabs), so the chip is not left latency-bound.
template <int G>
__global__ __launch_bounds__(256) void splitk_reduce_k(const float* __restrict__ ws, int nsplit,
                                                       long long slab, long long n4,
                                                       float* __restrict__ out, int accumulate) {
  constexpr int OPB = 256 / G;  // float4 outputs per block
  __shared__ f32x4 red[G][OPB];
  const int o = threadIdx.x % OPB, g = threadIdx.x / OPB;
  for (long long base = (long long)blockIdx.x * OPB; base < n4; base += (long long)gridDim.x * OPB) {
    const long long i = base + o;
    f32x4 a = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
      int s = g;
      for (; s + 7 * G < nsplit; s += 8 * G) {
        f32x4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = *(const f32x4*)(ws + (long long)(s + u * G) * slab + 4 * i);
#pragma unroll
        for (int u = 0; u < 8; ++u) a += v[u];
      }
      for (; s < nsplit; s += G) a += *(const f32x4*)(ws + (long long)s * slab + 4 * i);
    }
    if (G > 1) {
      red[g][o] = a;
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int q = 1; q < G; ++q) a += red[q][o];
      }
      __syncthreads();
    }
    if (g == 0 && i < n4) {
      if (accumulate) a += ((const f32x4*)out)[i];
      ((f32x4*)out)[i] = a;
    }
  }
}

int cn_splitk_reduce_impl(const float* ws, int nsplit, long long slab, long long n, float* out,
                          int accumulate, hipStream_t st) {
  if (n % 4 || slab % 4) return -2;
  const long long n4 = n / 4;
  // slab groups: enough threads to cover the chip (~512 K), at most the number of slabs
  int G = 1;
  while (G < 16 && 2 * G <= nsplit && n4 * G < (512ll << 10)) G *= 2;
  const int opb = 256 / G;
  long long b = (n4 + opb - 1) / opb;
  if (b > 4096) b = 4096;
#define CN_RED(GG) \
  hipLaunchKernelGGL(splitk_reduce_k<GG>, dim3((unsigned)b), dim3(256), 0, st, ws, nsplit, slab, n4, out, accumulate)
  switch (G) {
    case 1: CN_RED(1); break;
    case 2: CN_RED(2); break;
    case 4: CN_RED(4); break;
    case 8: CN_RED(8); break;
    default: CN_RED(16); break;
  }
#undef CN_RED
  CN_CHECK_LAUNCH();
  return 0;
}
