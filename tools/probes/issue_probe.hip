// Probe: what an operand-fill instruction costs the MFMA stream of the wave that issues it.
// Every wave runs ITER iterations of {D fill instructions (16 B per lane each, from an L2-resident
// 1 MB buffer) + M independent v_mfma_f32_16x16x32_bf16}, the fills of iteration i waited for in
// iteration i+1 (counted vmcnt), 1 or 2 waves per SIMD, one workgroup per CU, 256 workgroups.
// Fill kinds: 0 none, 1 LDS-DMA (buffer_load_dwordx4 ... lds, the GEMM loaders), 2 global_load_
// dwordx4 into VGPRs, 3 global_load_dwordx4 + ds_write_b128 of the previous iteration's data
// (register staging).  Reports ns per iteration and the MFMA rate against the bare loop.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <int KIND, int D, int M, int NT>
__global__ __launch_bounds__(NT) void issue_k(const char* src, int iters, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[D * NT * 16 + 16];
  const int tid = threadIdx.x, lane = tid & 63;
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, 0x7fffffff, 0x00020000);
  char* wb = lds + __builtin_amdgcn_readfirstlane((tid & ~63) * 16);
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(0.001f * (lane + j)); b[j] = (__bf16)(0.002f * (lane - j)); }
  f32x4 acc[M];
  for (int m = 0; m < M; ++m) acc[m] = f32x4{0.f, 0.f, 0.f, 0.f};
  u32x4 st[D > 0 ? D : 1];
  u32x4 x = {0, 0, 0, 0};
  for (int d = 0; d < (D > 0 ? D : 1); ++d) st[d] = u32x4{0, 0, 0, 0};
  const unsigned span = 1u << 20;
  for (int it = 0; it < iters; ++it) {
    const unsigned base = (unsigned)((it * 97 + blockIdx.x * 13) * 16384) & (span / 2 - 1);   // + voff < span
    if constexpr (KIND == 1) {
#pragma unroll
      for (int d = 0; d < D; ++d)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(wb + d * NT * 16), 16,
                                                 (int)(tid * 16 + d * 4096), (int)base, 0, 0);
    } else if constexpr (KIND == 2 || KIND == 3) {
      // consume the previous iteration's data (its loads had the MFMAs to land), then reload
#pragma unroll
      for (int d = 0; d < D; ++d) {
        if constexpr (KIND == 3) *(u32x4*)(lds + (d * NT + tid) * 16) = st[d];
        else x ^= st[d];
      }
#pragma unroll
      for (int d = 0; d < D; ++d) st[d] = *(const u32x4*)(src + ((base + tid * 16 + d * 4096) & (span - 1)));
    }
#pragma unroll
    for (int m = 0; m < M; ++m) acc[m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[m], 0, 0, 0);
    if constexpr (KIND == 1) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(D) : "memory");
    }
  }
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += acc[m][0] + acc[m][3];
  for (int d = 0; d < (D > 0 ? D : 1); ++d) x ^= st[d];
  if (s == 12345.f || x.x == 0x12345u) sink[blockIdx.x] = s + (float)x.y + (float)lds[tid];
}

template <int KIND, int D, int M, int NT>
double run(const char* src, float* sink, double base_ns) {
  const int iters = 4000;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((issue_k<KIND, D, M, NT>), dim3(256), dim3(NT), 0, 0, src, iters, sink);
  hipEventRecord(e0, 0);
  hipLaunchKernelGGL((issue_k<KIND, D, M, NT>), dim3(256), dim3(NT), 0, 0, src, iters, sink);
  hipEventRecord(e1, 0);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  const double ns = ms * 1e6 / iters;
  static const char* kn[] = {"none", "lds-dma", "vgpr-load", "vgpr+ds_write"};
  printf("%-14s D=%d M=%2d waves/SIMD=%d : %7.1f ns/iter  MFMA rate %.2f of the bare loop  (%.0f GB/s per CU filled)\n",
         kn[KIND], D, M, NT / 256, ns, base_ns > 0 ? base_ns / ns : 1.0, KIND ? D * NT * 16 / ns : 0.0);
  return ns;
}

int main() {
  char* src;
  float* sink;
  hipMalloc(&src, 1 << 20);
  hipMalloc(&sink, 256 * sizeof(float));
  hipMemset(src, 1, 1 << 20);
  // M = 16 MFMAs (256 cycles per wave) per iteration ~ one 64x64 wave tile's k-piece
  for (int pass = 0; pass < 2; ++pass) {
    const double b1 = run<0, 0, 16, 256>(src, sink, 0);
    run<1, 2, 16, 256>(src, sink, b1);
    run<1, 4, 16, 256>(src, sink, b1);
    run<2, 2, 16, 256>(src, sink, b1);
    run<2, 4, 16, 256>(src, sink, b1);
    run<3, 2, 16, 256>(src, sink, b1);
    run<3, 4, 16, 256>(src, sink, b1);
    const double b2 = run<0, 0, 16, 512>(src, sink, 0);
    run<1, 2, 16, 512>(src, sink, b2);
    run<1, 4, 16, 512>(src, sink, b2);
    run<2, 2, 16, 512>(src, sink, b2);
    run<2, 4, 16, 512>(src, sink, b2);
    run<3, 2, 16, 512>(src, sink, b2);
    run<3, 4, 16, 512>(src, sink, b2);
  }
  hipFree(src);
  hipFree(sink);
  return 0;
}
