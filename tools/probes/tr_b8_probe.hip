// Probe: the lane / byte mapping of gfx950's ds_read_b64_tr_b8 (the 8-bit transposed LDS read an
// fp8 weight-gradient loader would use; DESIGN.md section 3.5 route (ii)).  LDS holds byte
// value = (offset mod 256) in pass 0 and (offset / 256) in pass 1, so every returned byte names
// its source offset.  Lane l supplies address 8 * l (its own 8-byte chunk).  Prints, for the
// first 16-lane group, the source offset of each of the 8 bytes each lane receives.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

__global__ void probe_k(unsigned* out, int pass) {
  __shared__ __attribute__((aligned(16))) unsigned char lds[4096];
  const int l = threadIdx.x;
  for (int i = l; i < 4096; i += 64) lds[i] = (unsigned char)(pass == 0 ? (i & 255) : (i >> 8));
  __syncthreads();
  const unsigned a = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)(lds + 8 * l);
  u32x2 v;
  asm volatile("ds_read_b64_tr_b8 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a));
  out[2 * l] = v.x;
  out[2 * l + 1] = v.y;
}

int main() {
  unsigned* d;
  hipMalloc(&d, 2 * 64 * sizeof(unsigned));
  unsigned h[2][128];
  for (int pass = 0; pass < 2; ++pass) {
    hipLaunchKernelGGL(probe_k, dim3(1), dim3(64), 0, 0, d, pass);
    hipMemcpy(h[pass], d, sizeof(h[pass]), hipMemcpyDeviceToHost);
  }
  printf("lane: source byte offsets of the 8 bytes received (lane l supplied address 8*l)\n");
  for (int l = 0; l < 64; ++l) {
    printf("lane %2d:", l);
    for (int b = 0; b < 8; ++b) {
      const unsigned lo = (h[0][2 * l + b / 4] >> (8 * (b % 4))) & 255;
      const unsigned hi = (h[1][2 * l + b / 4] >> (8 * (b % 4))) & 255;
      printf(" %4u", hi * 256 + lo);
    }
    printf("\n");
  }
  hipFree(d);
  return 0;
}
