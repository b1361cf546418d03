// Clip assembly on the device (first step): the per-frame arithmetic of
// load_video_frames after decode (ravdess.py:352 cv2.resize INTER_LINEAR, :363 /255, :386-389 ImageNet
// normalisation + HWC->CHW) and the waveform pad/crop of load_audio_wav (ravdess.py:505-513).
// Decoded uint8 frames cross PCIe (37 KB per 112x112 frame instead of 150 KB of fp32) and the batch is built in HBM.
//
// Resize follows OpenCV's scalar fixed-point INTER_LINEAR path: per output index the source index and two
// 11-bit weights (rounded to nearest even), an int horizontal pass, an int vertical pass rounded with
// (v + 2^21) >> 22 and saturated to uint8; an exact 2x downscale is OpenCV's INTER_AREA 2x2 average.
// Integer arithmetic end to end until the fp32 normalisation, so results are bit-exact against
// oracle/clips_ref.py.  HBM-bound: one thread per output pixel (3 channels), coalesced along x.
#include "common.h"
#include "mer.h"

namespace {

struct LinTap {
  int s0, s1, a0, a1;
};

// OpenCV's coefficient table entry for destination index d (resize.cpp, INTER_LINEAR, ksize 2)
__device__ __forceinline__ LinTap lin_tap(int d, int src, double scale) {
  float f = (float)((d + 0.5) * scale - 0.5);
  int s = (int)floorf(f);
  f -= (float)s;
  if (s < 0) { f = 0.f; s = 0; }
  if (s >= src - 1) { f = 0.f; s = src - 1; }
  LinTap t;
  t.s0 = s;
  t.s1 = min(s + 1, src - 1);
  t.a0 = __float2int_rn((1.f - f) * 2048.f);
  t.a1 = __float2int_rn(f * 2048.f);
  return t;
}

// cv2.resize(frame, (S, S), INTER_LINEAR) of one output pixel's 3 channels (uint8 values)
__device__ __forceinline__ void resize_pixel(const uint8_t* f, int H0, int W0, int S, int x, int y, double scale_y,
                                             double scale_x, int v[3]) {
  if (H0 == 2 * S && W0 == 2 * S) {  // INTER_AREA fast path for an exact 2x downscale
    const uint8_t* p0 = f + ((long)(2 * y) * W0 + 2 * x) * 3;
    const uint8_t* p1 = p0 + (long)W0 * 3;
    for (int c = 0; c < 3; ++c) v[c] = (p0[c] + p0[3 + c] + p1[c] + p1[3 + c] + 2) >> 2;
  } else {
    const LinTap tx = lin_tap(x, W0, scale_x), ty = lin_tap(y, H0, scale_y);
    const uint8_t* r0 = f + (long)ty.s0 * W0 * 3;
    const uint8_t* r1 = f + (long)ty.s1 * W0 * 3;
    for (int c = 0; c < 3; ++c) {
      const int h0 = r0[tx.s0 * 3 + c] * tx.a0 + r0[tx.s1 * 3 + c] * tx.a1;
      const int h1 = r1[tx.s0 * 3 + c] * tx.a0 + r1[tx.s1 * 3 + c] * tx.a1;
      const int w = (h0 * ty.a0 + h1 * ty.a1 + (1 << 21)) >> 22;
      v[c] = w < 0 ? 0 : (w > 255 ? 255 : w);
    }
  }
}

__global__ __launch_bounds__(256) void frames_resize_normalize_kernel(int H0, int W0, int S, const uint8_t* __restrict__ src,
                                                                      long frame_stride, double scale_y, double scale_x,
                                                                      float m0, float m1, float m2, float sd0,
                                                                      float sd1, float sd2, float* __restrict__ dst) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= S) return;
  int v[3];
  resize_pixel(src + (long)n * frame_stride, H0, W0, S, x, y, scale_y, scale_x, v);
  // (x / 255 - mean) / std in fp32 with the reference's operation order (numpy float32, ravdess.py:363,388)
  const long plane = (long)S * S, o = (long)n * 3 * plane + (long)y * S + x;
  dst[o] = ((float)v[0] / 255.f - m0) / sd0;
  dst[o + plane] = ((float)v[1] / 255.f - m1) / sd1;
  dst[o + 2 * plane] = ((float)v[2] / 255.f - m2) / sd2;
}

__global__ __launch_bounds__(256) void frames_resize_u8_kernel(int H0, int W0, int S, const uint8_t* __restrict__ src,
                                                               long frame_stride, double scale_y, double scale_x,
                                                               uint8_t* __restrict__ dst) {
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= S) return;
  int v[3];
  resize_pixel(src + (long)n * frame_stride, H0, W0, S, x, y, scale_y, scale_x, v);
  uint8_t* o = dst + (((long)n * S + y) * S + x) * 3;
  o[0] = (uint8_t)v[0];
  o[1] = (uint8_t)v[1];
  o[2] = (uint8_t)v[2];
}

// cv::borderInterpolate(p, n, BORDER_REFLECT_101) (cv2.GaussianBlur's default border): gfedcb|abcdefgh|gfedcba
__device__ __forceinline__ int reflect101(int p, int n) {
  if (n == 1) return 0;
  while (p < 0 || p >= n) p = p < 0 ? -p : 2 * n - 2 - p;
  return p;
}

// The train-split augmentation of load_video_frames (ravdess.py:366-384) on one output pixel of a resized uint8
// frame, then ImageNet normalisation (:386-389).  Per clip (params[clip] = factor, noise_scale, ksize):
//   img  = (frames * 255).astype(uint8)         -- frames = u8 / 255 in fp32: trunc(fl(fl(u / 255) * 255)) == u for
//                                                  every u in 0..255 (tests/test_clips_cpu.py), so the blur reads u
//   img  = cv2.GaussianBlur(img, (k, k), 0)     -- sigma 0 and k <= 7: OpenCV's fixed binomial table (w / 2^m per axis,
//                                                  getGaussianKernelBitExact), its 8U fixed-point path is exact, then
//                                                  rounds half up: (sum + 2^(2m-1)) >> 2m; BORDER_REFLECT_101
//   img  = img / 255 * factor + N(0, noise_scale)   (fp32, no contraction)   -> clip [0, 1] -> (x - mean) / std
// The Gaussian draw is z = ztable[mer_hash(clip seed, element) >> 16] (the 65,536-entry inverse normal CDF at
// (i + 0.5) / 65536), noise = fl(noise_scale * z): reproducible per (seed, element), bit-exact to the restatement.
__global__ __launch_bounds__(256) void frames_augment_normalize_kernel(int S, int T, const uint8_t* __restrict__ src,
                                                                       const float* __restrict__ params,
                                                                       const unsigned long long* __restrict__ seeds,
                                                                       const float* __restrict__ ztable, float m0,
                                                                       float m1, float m2, float sd0, float sd1, float sd2,
                                                                       float* __restrict__ dst) {
#pragma clang fp contract(off)  // the noise term is fl(fl(x * factor) + fl(sigma * z)), never an fma (numpy order)
  const int x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y, n = blockIdx.z;
  if (x >= S) return;
  const int clip = n / T;
  const float factor = params[clip * 3], sigma = params[clip * 3 + 1];
  const int k = (int)params[clip * 3 + 2];
  // OpenCV small_gaussian_tab rows as integers over 2^m: k = 1 / 3 / 5 / 7
  int w[7], m;
  if (k == 3) { w[0] = 1; w[1] = 2; w[2] = 1; m = 2; }
  else if (k == 5) { w[0] = 1; w[1] = 4; w[2] = 6; w[3] = 4; w[4] = 1; m = 4; }
  else if (k == 7) { w[0] = 2; w[1] = 7; w[2] = 14; w[3] = 18; w[4] = 14; w[5] = 7; w[6] = 2; m = 6; }
  else { w[0] = 1; m = 0; }
  const int kk = (k == 3 || k == 5 || k == 7) ? k : 1, r = kk / 2;
  const uint8_t* f = src + (long)n * S * S * 3;
  int acc[3] = {0, 0, 0};
  for (int dy = 0; dy < kk; ++dy) {
    const uint8_t* row = f + (long)reflect101(y + dy - r, S) * S * 3;
    int h[3] = {0, 0, 0};
    for (int dx = 0; dx < kk; ++dx) {
      const uint8_t* px = row + reflect101(x + dx - r, S) * 3;
      for (int c = 0; c < 3; ++c) h[c] += w[dx] * px[c];
    }
    for (int c = 0; c < 3; ++c) acc[c] += w[dy] * h[c];
  }
  const float mean[3] = {m0, m1, m2}, sd[3] = {sd0, sd1, sd2};
  const unsigned long long seed = seeds[clip];
  const long plane = (long)S * S, o = (long)n * 3 * plane + (long)y * S + x;
  const long e0 = (((long)(n - clip * T) * S + y) * S + x) * 3;  // element index inside the clip, HWC order
  for (int c = 0; c < 3; ++c) {
    const int b = m ? (acc[c] + (1 << (2 * m - 1))) >> (2 * m) : acc[c];
    float v = (float)b / 255.f * factor;
    if (sigma > 0.f) v = v + sigma * ztable[mer_hash(seed, (uint64_t)(e0 + c)) >> 16];
    v = fminf(fmaxf(v, 0.f), 1.f);
    dst[o + c * plane] = (v - mean[c]) / sd[c];
  }
}

__global__ __launch_bounds__(256) void wav_pad_crop_kernel(int target, const float* __restrict__ src,
                                                           const long long* __restrict__ offsets,
                                                           const long long* __restrict__ lengths, float* __restrict__ out) {
  const int b = blockIdx.y;
  const long long off = offsets[b], len = lengths[b];
  for (int t = blockIdx.x * 256 + threadIdx.x; t < target; t += gridDim.x * 256)
    out[(long)b * target + t] = t < len ? src[off + t] : 0.f;
}

}  // namespace

MER_API int mer_frames_resize_normalize(int N, int H0, int W0, const void* frames, long frame_stride, int S, float mean0,
                                        float mean1, float mean2, float std0, float std1, float std2, float* out,
                                        void* stream) {
  if (N <= 0) return 0;
  if (H0 <= 0 || W0 <= 0 || S <= 0 || frame_stride < (long)H0 * W0 * 3) return (int)hipErrorInvalidValue;
  const double sy = 1.0 / ((double)S / H0), sx = 1.0 / ((double)S / W0);  // cv::resize: 1 / inv_scale
  hipLaunchKernelGGL(frames_resize_normalize_kernel, dim3((S + 255) / 256, S, N), dim3(256), 0, (hipStream_t)stream,
                     H0, W0, S, (const uint8_t*)frames, frame_stride, sy, sx, mean0, mean1, mean2, std0, std1, std2,
                     out);
  MER_LAUNCH_CHECK();
}

MER_API int mer_frames_resize_u8(int N, int H0, int W0, const void* frames, long frame_stride, int S, void* out,
                                 void* stream) {
  if (N <= 0) return 0;
  if (H0 <= 0 || W0 <= 0 || S <= 0 || frame_stride < (long)H0 * W0 * 3) return (int)hipErrorInvalidValue;
  const double sy = 1.0 / ((double)S / H0), sx = 1.0 / ((double)S / W0);
  hipLaunchKernelGGL(frames_resize_u8_kernel, dim3((S + 255) / 256, S, N), dim3(256), 0, (hipStream_t)stream, H0, W0,
                     S, (const uint8_t*)frames, frame_stride, sy, sx, (uint8_t*)out);
  MER_LAUNCH_CHECK();
}

MER_API int mer_frames_augment_normalize(int N, int S, int T, const void* frames_u8, const float* clip_params,
                                         const unsigned long long* clip_seeds, const float* ztable, float mean0,
                                         float mean1, float mean2, float std0, float std1, float std2, float* out,
                                         void* stream) {
  if (N <= 0) return 0;
  if (S <= 0 || T <= 0 || N % T) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(frames_augment_normalize_kernel, dim3((S + 255) / 256, S, N), dim3(256), 0, (hipStream_t)stream,
                     S, T, (const uint8_t*)frames_u8, clip_params, clip_seeds, ztable, mean0, mean1, mean2, std0, std1,
                     std2, out);
  MER_LAUNCH_CHECK();
}

MER_API int mer_wav_pad_crop(int B, int target, const float* packed, const long long* offsets,
                             const long long* lengths, float* out, void* stream) {
  if (B <= 0) return 0;
  if (target <= 0) return (int)hipErrorInvalidValue;
  const int gx = (target + 255) / 256 < 64 ? (target + 255) / 256 : 64;
  hipLaunchKernelGGL(wav_pad_crop_kernel, dim3(gx, B), dim3(256), 0, (hipStream_t)stream, target, packed, offsets,
                     lengths, out);
  MER_LAUNCH_CHECK();
}
