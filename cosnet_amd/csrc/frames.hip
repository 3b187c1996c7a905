// Frame preparation for the SBM-RGBD input pipeline:
// dataloaders/sbm_rgbd_loader.py:590-697 (_load_images) and dataloaders/utils.py:5-55.
// One kernel does a windowed resize with OpenCV's cv2.resize coordinate rules, optional
// per-channel mean subtraction of the source values and a horizontal flip of the output:
//   * ROI crop / random crop  = the source window (y0, x0, h, w), no copy;
//   * cv2.resize INTER_LINEAR = half-pixel source coordinate fx = (dx + 0.5) * w / W - 0.5,
//     taps floor(fx), floor(fx) + 1 with weights (1 - a, a), a forced to 0 when the left tap
//     falls before 0 or at/after the last column (same for rows); row pass then column pass in
//     fp32, as OpenCV's float path computes it;
//   * cv2.resize INTER_NEAREST = source index min(floor(dx * w / W), w - 1);
//   * np.fliplr               = output column W - 1 - dx.
// Sources are uint8 HWC (decoded frames) or fp32 planar; the output is fp32 CHW.
#include "common.h"
#include "../../include/cosnet_hip.h"

namespace {

template <class S>
__global__ void frame_resize_k(const S* __restrict__ src, int C, long long sp, long long sr, long long sc,
                               int y0, int x0, int h, int w, const float* __restrict__ mean,
                               float* __restrict__ dst, int H, int W, int mode, int flip,
                               double scale_y, double scale_x) {
  const long long total = (long long)C * H * W;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int dx = (int)(i % W);
    const long long q = i / W;
    const int dy = (int)(q % H), c = (int)(q / H);
    const int ox = flip ? W - 1 - dx : dx;
    const S* plane = src + (long long)c * sp + (long long)y0 * sr + (long long)x0 * sc;
    const float m = mean ? mean[c] : 0.f;
    float v;
    if (mode == 1) {  // INTER_NEAREST
      int sy = (int)floor(dy * scale_y), sx = (int)floor(ox * scale_x);
      sy = min(sy, h - 1);
      sx = min(sx, w - 1);
      v = (float)plane[sy * sr + sx * sc] - m;
    } else {          // INTER_LINEAR
      float fy = (float)((dy + 0.5) * scale_y - 0.5);
      int sy = (int)floorf(fy);
      fy -= sy;
      if (sy < 0) { fy = 0.f; sy = 0; }
      if (sy >= h - 1) { fy = 0.f; sy = h - 1; }
      float fx = (float)((ox + 0.5) * scale_x - 0.5);
      int sx = (int)floorf(fx);
      fx -= sx;
      if (sx < 0) { fx = 0.f; sx = 0; }
      if (sx >= w - 1) { fx = 0.f; sx = w - 1; }
      const int sy1 = min(sy + 1, h - 1), sx1 = min(sx + 1, w - 1);
      const float a00 = (float)plane[sy * sr + sx * sc] - m, a01 = (float)plane[sy * sr + sx1 * sc] - m;
      const float a10 = (float)plane[sy1 * sr + sx * sc] - m, a11 = (float)plane[sy1 * sr + sx1 * sc] - m;
      const float r0 = a00 * (1.f - fx) + a01 * fx;
      const float r1 = a10 * (1.f - fx) + a11 * fx;
      v = r0 * (1.f - fy) + r1 * fy;
    }
    dst[i] = v;
  }
}

}  // namespace

extern "C" int cn_frame_resize(int src_u8, const void* src, int C, long long plane_stride,
                               long long row_stride, long long col_stride, int y0, int x0, int h,
                               int w, const float* mean, float* dst, int H, int W, int mode,
                               int flip, hipStream_t st) {
  if (C < 1 || h < 1 || w < 1 || H < 1 || W < 1 || y0 < 0 || x0 < 0) return CN_ERR_SHAPE;
  if (mode != 0 && mode != 1) return CN_ERR_UNSUPPORTED;
  const long long total = (long long)C * H * W;
  long long nb = (total + 255) / 256;
  if (nb > 8192) nb = 8192;
  // OpenCV: inv_scale = dsize / ssize, scale = 1 / inv_scale (both double)
  const double sy = 1.0 / ((double)H / h), sx = 1.0 / ((double)W / w);
  if (src_u8)
    hipLaunchKernelGGL(frame_resize_k<unsigned char>, dim3((unsigned)nb), dim3(256), 0, st,
                       (const unsigned char*)src, C, plane_stride, row_stride, col_stride, y0, x0, h, w,
                       mean, dst, H, W, mode, flip, sy, sx);
  else
    hipLaunchKernelGGL(frame_resize_k<float>, dim3((unsigned)nb), dim3(256), 0, st, (const float*)src, C,
                       plane_stride, row_stride, col_stride, y0, x0, h, w, mean, dst, H, W, mode, flip,
                       sy, sx);
  CN_CHECK_LAUNCH();
  return 0;
}
