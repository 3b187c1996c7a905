// Probe: which reduction indices (k) the 32 bytes of a lane hold in
// v_mfma_scale_f32_32x32x64_f8f6f4 (e4m3), relative to the per-lane E8M0 scale blocks.
// A: lane (r, h) byte j = 1.0 (0x38) if j in [lo, hi), else 0; B all 1.0; scale_a of lane half 1
// = 2 (128), half 0 = 1 (127); scale_b = 1.  C[0][0] = sum of sa over the k's set in A.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(8))) int i32x8;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__global__ void probe(float* out, int lo, int hi, int sel) {
  const int lane = threadIdx.x, h = lane >> 5;
  unsigned char a[32], b[32];
  for (int j = 0; j < 32; ++j) {
    a[j] = (j >= lo && j < hi && (sel < 0 || h == sel)) ? 0x38 : 0;
    b[j] = 0x38;
  }
  i32x8 av, bv;
  for (int q = 0; q < 8; ++q) {
    av[q] = a[4 * q] | (a[4 * q + 1] << 8) | (a[4 * q + 2] << 16) | (a[4 * q + 3] << 24);
    bv[q] = b[4 * q] | (b[4 * q + 1] << 8) | (b[4 * q + 2] << 16) | (b[4 * q + 3] << 24);
  }
  const int sa = h ? 128 : 127;
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(av, bv, c, 0, 0, 0, sa, 0, 127);
  out[lane * 16 + 0] = c[0];
}

int main() {
  float* d;
  hipMalloc(&d, 64 * 16 * 4);
  float h[64 * 16];
  const int cases[][3] = {{0, 32, -1}, {0, 16, -1}, {16, 32, -1}, {0, 16, 0}, {0, 16, 1},
                          {16, 32, 0}, {16, 32, 1}, {0, 8, 0}, {8, 16, 0}};
  for (auto& cs : cases) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, cs[0], cs[1], cs[2]);
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("A bytes [%2d,%2d) of half %2d set: C[0][0] = %g\n", cs[0], cs[1], cs[2], h[0]);
  }
  return 0;
}
