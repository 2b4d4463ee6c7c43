// Input normalisation on the device: the two per-clip transforms the reference
// runs on the host inside its data path.
//
//  * frame normalisation — T.ToTensor() + T.Normalize(mean, std) of data/data_process.py:55-69 applied to
//    the decoded RGB frames of extract_frames (src/utils.py:22-39): uint8 [N, H, W, 3] (HWC, as decoded)
//    -> fp32 [N, 3, H, W], y = (x / 255 - mean[c]) / std[c] with the same fp32 operations (bit-exact).
//    HBM-bound: 1 byte read + 4 bytes written per element.
//  * waveform normalisation — Wav2Vec2FeatureExtractor.zero_mean_unit_var_norm (transformers
//    feature_extraction_wav2vec2.py:94-95, called at src/trainer.py:258): each (zero-padded, Q13) row
//    y = (x - mean) / sqrt(var + 1e-7), one workgroup per clip, fp32 two-pass statistics.
#include "common.h"

namespace {

// one thread per 4 consecutive pixels of one frame row: 12 bytes in, 3 x 16 bytes out (one per channel)
__global__ __launch_bounds__(256) void frame_norm_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst,
                                                         long npix4, int HW, float m0, float m1, float m2,
                                                         float s0, float s1, float s2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;   // group of 4 pixels
  if (i >= npix4) return;
  const long p = i * 4;                                          // first pixel (frame-major)
  const long f = p / HW, o = p % HW;
  const uint32_t* s = reinterpret_cast<const uint32_t*>(src + p * 3);
  const uint32_t w0 = s[0], w1 = s[1], w2 = s[2];              // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
  const uint8_t b[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                         (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                         (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
  const float mean[3] = {m0, m1, m2}, stdv[3] = {s0, s1, s2};
  float* out = dst + f * 3 * (long)HW + o;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    float4 v;
    v.x = ((float)b[c] / 255.f - mean[c]) / stdv[c];
    v.y = ((float)b[3 + c] / 255.f - mean[c]) / stdv[c];
    v.z = ((float)b[6 + c] / 255.f - mean[c]) / stdv[c];
    v.w = ((float)b[9 + c] / 255.f - mean[c]) / stdv[c];
    *reinterpret_cast<float4*>(out + (long)c * HW) = v;
  }
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(1024) void wave_norm_kernel(const float* __restrict__ x, float* __restrict__ y, long S,
                                                         float eps) {
  __shared__ float red[16];
  const float* xr = x + (long)blockIdx.x * S;
  float* yr = y + (long)blockIdx.x * S;
  float s = 0.f;
  for (long i = threadIdx.x; i < S; i += blockDim.x) s += xr[i];
  const float mean = block_sum(s, red) / (float)S;
  float q = 0.f;
  for (long i = threadIdx.x; i < S; i += blockDim.x) {
    const float d = xr[i] - mean;
    q += d * d;
  }
  const float var = block_sum(q, red) / (float)S;
  const float inv = 1.f / sqrtf(var + eps);
  for (long i = threadIdx.x; i < S; i += blockDim.x) yr[i] = (xr[i] - mean) * inv;
}

}  // namespace

extern "C" int dfk_frame_normalize(const uint8_t* src, float* dst, int64_t frames, int32_t H, int32_t W,
                                   const float* mean3, const float* std3, hipStream_t s) {
  if (!src || !dst || !mean3 || !std3 || frames < 0 || H <= 0 || W <= 0) return DFK_EINVAL;
  const long HW = (long)H * W;
  if (HW % 4 || (reinterpret_cast<uintptr_t>(src) & 3) || (reinterpret_cast<uintptr_t>(dst) & 15)) return DFK_EINVAL;
  const long n4 = frames * HW / 4;
  if (n4 == 0) return 0;
  hipLaunchKernelGGL(frame_norm_kernel, dim3((unsigned)dfk_cdiv(n4, 256)), dim3(256), 0, s, src, dst, n4, (int)HW,
                     mean3[0], mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_wave_normalize(const float* x, float* y, int64_t B, int64_t S, float eps, hipStream_t s) {
  if (!x || !y || B < 0 || S <= 0) return DFK_EINVAL;
  if (B == 0) return 0;
  hipLaunchKernelGGL(wave_norm_kernel, dim3((unsigned)B), dim3(1024), 0, s, x, y, (long)S, eps);
  DFK_CHECK_LAUNCH();
  return 0;
}
