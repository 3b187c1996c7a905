// Probe: per-CU LDS-DMA fill rate (buffer_load_dwordx4 ... lds, the GEMM loaders' instruction)
// as a function of the ring geometry: tile bytes per stage, ring depth (tiles in flight), threads
// per block, and where the bytes come from (one small buffer every block reads = weights in L2;
// a block-private region of a large buffer = activations from the Infinity Cache / HBM).
// One block per CU (dynamic LDS >= 96 KB), grid = 256 blocks.  Each K step: barrier, refill the
// stage consumed one step earlier, R ds_read_b128 per wave from the current stage (the fragment
// reads of a GEMM), counted vmcnt wait for the next tile -- the gemm.hip loop without the MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, char* lds) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff,
                                           (int)soff, 0, 0);
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

template <int TILE, int NS, int NT, bool DMA = true>
__global__ __launch_bounds__(NT) void fill_k(const char* src, long long span, long long bstride, int ntiles,
                                             int R, float* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int CH = TILE / (16 * NT);   // 16-B chunks per thread per tile
  static_assert(CH * 16 * NT == TILE, "tile must be whole chunk rounds");
  const int tid = threadIdx.x;
  const long long base = ((long long)blockIdx.x * bstride) % span;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
  char* wb = lds + __builtin_amdgcn_readfirstlane((tid & ~63) * 16);
  auto issue = [&](int t, int stage) {
    if (!DMA) return;
    const long long off = (base + (long long)t * TILE) % (span - TILE + 1);
    const unsigned soff = (unsigned)(off & ~15ll);
#pragma unroll
    for (int i = 0; i < CH; ++i) blds16(rs, (unsigned)((tid + i * NT) * 16), soff, wb + stage * TILE + i * NT * 16);
  };
#pragma unroll
  for (int s = 0; s < NS - 1; ++s) issue(s, s);
  wait_vm<CH * (NS - 2)>();
  __builtin_amdgcn_s_barrier();
  u32x4 acc = {0, 0, 0, 0};
  const int lane = tid & 63;
  for (int t = 0; t < ntiles; ++t) {
    const int st = t % NS;
    if (t + NS - 1 < ntiles) issue(t + NS - 1, (t + NS - 1) % NS);
    const char* sp = lds + st * TILE;
    // fragment-like reads: 8 in flight, then folded (a GEMM's prefetched fragment reads)
    for (int r0 = 0; r0 < R; r0 += 8) {
      u32x4 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = *(const u32x4*)(sp + (((r0 + q) * 64 + lane) * 16) % TILE);
#pragma unroll
      for (int q = 0; q < 8; ++q) if (r0 + q < R) acc ^= v[q];
    }
    if (t + NS - 1 < ntiles) wait_vm<CH * (NS - 2)>();
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  if (acc.x == 0x12345678u) sink[blockIdx.x] = (float)acc.y;   // keep the reads
}

// Register path for comparison: every thread streams its chunks of the same tiles with
// global_load_dwordx4 into VGPRs (U tiles of loads in flight per thread), optionally stores them
// to an LDS ring with ds_write_b128 (register staging, STAGE_LDS); nothing is computed.
template <int TILE, int U, int NT, bool STAGE_LDS>
__global__ __launch_bounds__(NT) void vgpr_k(const char* src, long long span, long long bstride, int ntiles,
                                             float* sink) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  constexpr int CH = TILE / (16 * NT);
  const int tid = threadIdx.x;
  const long long base = ((long long)blockIdx.x * bstride) % span;
  u32x4 acc = {0, 0, 0, 0};
  for (int t0 = 0; t0 < ntiles; t0 += U) {
    u32x4 v[U][CH];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long off = (base + (long long)(t0 + u) * TILE) % (span - TILE + 1);
      const char* p = src + (off & ~15ll);
#pragma unroll
      for (int i = 0; i < CH; ++i) v[u][i] = *(const u32x4*)(p + (tid + i * NT) * 16);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int i = 0; i < CH; ++i) {
        if (STAGE_LDS) *(u32x4*)(lds + ((u & 1) * TILE) + (tid + i * NT) * 16) = v[u][i];
        else acc ^= v[u][i];
      }
    if (STAGE_LDS) __syncthreads();
  }
  if (acc.x == 0x12345678u) sink[blockIdx.x] = (float)acc.y;
}

template <int TILE, int U, int NT, bool STAGE_LDS>
void run_vgpr(const char* name, const char* src, long long span, long long bstride, int ntiles, float* sink) {
  const size_t shm = 98304;
  hipFuncSetAttribute((const void*)vgpr_k<TILE, U, NT, STAGE_LDS>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((vgpr_k<TILE, U, NT, STAGE_LDS>), dim3(256), dim3(NT), shm, 0, src, span, bstride, ntiles, sink);
  hipEventRecord(e0, 0);
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep)
    hipLaunchKernelGGL((vgpr_k<TILE, U, NT, STAGE_LDS>), dim3(256), dim3(NT), shm, 0, src, span, bstride, ntiles, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps;
  const double bytes = 256.0 * ntiles * TILE;
  printf("%-10s VGPR%s tile %3d KB x %d in flight (%3d KB) %4d thr       : %7.1f us  %6.1f GB/s per CU  %5.2f TB/s chip\n",
         name, STAGE_LDS ? "+ds_write" : "         ", TILE / 1024, U, U * TILE / 1024, NT, us,
         bytes / us / 1e3 / 256, bytes / us / 1e6);
}

template <int TILE, int NS, int NT, bool DMA = true>
void run(const char* name, const char* src, long long span, long long bstride, int ntiles, int R, float* sink) {
  const size_t shm = (size_t)NS * TILE < 98304 ? 98304 : (size_t)NS * TILE;
  hipFuncSetAttribute((const void*)fill_k<TILE, NS, NT, DMA>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 2; ++rep)
    hipLaunchKernelGGL((fill_k<TILE, NS, NT, DMA>), dim3(256), dim3(NT), shm, 0, src, span, bstride, ntiles, R, sink);
  hipEventRecord(e0, 0);
  const int reps = 5;
  for (int rep = 0; rep < reps; ++rep)
    hipLaunchKernelGGL((fill_k<TILE, NS, NT, DMA>), dim3(256), dim3(NT), shm, 0, src, span, bstride, ntiles, R, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double us = ms * 1e3 / reps;
  const double bytes = 256.0 * ntiles * TILE;
  printf("%-10s %s tile %3d KB x %d stages (%3d KB in flight) %4d thr  R=%2d : %7.1f us  %6.1f GB/s per CU  %5.2f TB/s chip  %.3f us/tile\n",
         name, DMA ? "dma" : "---", TILE / 1024, NS, (NS - 1) * TILE / 1024, NT, R, us, bytes / us / 1e3 / 256,
         bytes / us / 1e6, us / ntiles);
}

int main(int argc, char** argv) {
  const long long big = 1ll << 30;
  char* src;
  float* sink;
  hipMalloc(&src, big);
  hipMalloc(&sink, 256 * sizeof(float));
  hipMemset(src, 1, big);
  struct Src { const char* name; long long span, bstride; };
  // weights: every block streams the same 1.2 MB (layer-3 3x3 weights); activations: block-private
  // runs of a 60 MB tensor (MALL) and of a 1 GB buffer (HBM)
  const Src srcs[] = {{"shared1M", 1179648, 0}, {"priv60M", 60ll << 20, 240 << 10}, {"priv1G", big, 4ll << 20}};
  // round 4b: DMA only / reads only / both, shared (L2-resident) source; R = ds_read_b128 per wave
  // per tile (the 128x256 GEMM tile reads 16 per wave per K step, 256x256: 24)
  if (argc > 1) {
    const Src& s = srcs[0];
    for (int R : {0, 8, 16, 24}) {
      run<49152, 3, 512, true>(s.name, src, s.span, s.bstride, 36, R, sink);
      run<49152, 3, 512, false>(s.name, src, s.span, s.bstride, 36, R, sink);
      run<65536, 2, 512, true>(s.name, src, s.span, s.bstride, 36, R, sink);
    }
    hipFree(src);
    hipFree(sink);
    return 0;
  }
  for (const Src& s : srcs) {
    const int nt48 = 36;   // K steps of the layer-3 3x3 conv
    run<49152, 3, 512>(s.name, src, s.span, s.bstride, nt48, 0, sink);
    run<49152, 3, 512>(s.name, src, s.span, s.bstride, nt48, 16, sink);
    run<49152, 2, 512>(s.name, src, s.span, s.bstride, nt48, 16, sink);
    run<24576, 6, 512>(s.name, src, s.span, s.bstride, 2 * nt48, 8, sink);
    run<16384, 8, 512>(s.name, src, s.span, s.bstride, 3 * nt48, 5, sink);
    run<32768, 4, 512>(s.name, src, s.span, s.bstride, 36, 0, sink);
    run<32768, 3, 256>(s.name, src, s.span, s.bstride, 36, 0, sink);
    run<65536, 2, 512>(s.name, src, s.span, s.bstride, 36, 0, sink);
    run<16384, 8, 256>(s.name, src, s.span, s.bstride, 108, 0, sink);
    run<8192, 16, 256>(s.name, src, s.span, s.bstride, 216, 0, sink);
    run_vgpr<16384, 2, 512, false>(s.name, src, s.span, s.bstride, 108, sink);
    run_vgpr<16384, 4, 512, false>(s.name, src, s.span, s.bstride, 108, sink);
    run_vgpr<32768, 4, 512, false>(s.name, src, s.span, s.bstride, 56, sink);
    run_vgpr<16384, 4, 512, true>(s.name, src, s.span, s.bstride, 108, sink);
  }
  hipFree(src);
  hipFree(sink);
  return 0;
}
