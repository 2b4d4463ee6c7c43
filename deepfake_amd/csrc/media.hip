// Media front end on the device: the per-clip transforms the reference runs on the host
// before the model sees a batch.
//
//  * mel-spectrogram image — generate_mel_spectrogram (src/utils.py:63-87):
//      librosa.feature.melspectrogram(y, sr, n_mels) (n_fft 2048, hop 512, periodic Hann, center=True with zero
//      padding, power 2, Slaney-normalised Slaney-scale filterbank) -> librosa.power_to_db(S, ref=np.max)
//      (amin 1e-10, top_db 80) -> cv2.normalize(NORM_MINMAX, 0, 255) -> astype(uint8) (truncation) ->
//      cv2.resize(target, INTER_LINEAR) (uint8 fixed point, 11-bit coefficients).
//    The STFT runs as one fp32 MFMA GEMM per batch (dfk_gemm: frames of the padded waveform, a strided
//    overlapping view with row stride = hop, times a window-folded cos | -sin basis); power, filterbank and dB
//    in mel_power_kernel; per-clip min/max, quantisation and the resize in mel_image_kernel (image in LDS).
//    The JPEG round trip of the reference's cached images (data_process.py:83-93,162) is not reproduced (a
//    lossy codec outside the hot path), nor librosa.load's resampling to 22.05 kHz (the caller passes the
//    waveform at the rate the filterbank was built for).
//  * gray image -> model input — Image.convert('RGB') + T.ToTensor() + T.Normalize (data_process.py:55-69,162):
//    uint8 [N, H, W] -> fp32 [N, 3, H, W], (x / 255 - mean[c]) / std[c].
//  * frame / mel-image transform — torchvision's T.Resize / RandomHorizontalFlip / RandomVerticalFlip /
//    RandomRotation(90) / ToTensor / Normalize as the reference runs them, on PIL images (data_process.py:55-69,
//    162; src/utils.py:32-33): PIL's antialiased BILINEAR resize (width pass, then height pass fused with the flips,
//    the NEAREST rotation's fixed-point inverse map and the normalisation).  Random flips / angles are per image.
#include "common.h"

namespace {

__global__ __launch_bounds__(256) void mel_pad_kernel(const float* __restrict__ y, long S, int half, long Lp,
                                                      float* __restrict__ yp) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long b = blockIdx.y;
  if (i >= Lp) return;
  const long s = i - half;
  yp[b * Lp + i] = (s >= 0 && s < S) ? y[b * S + s] : 0.f;
}

// one workgroup per (clip, frame): |X[f]|^2 into LDS, then mel[m] = sum_f fb[m][f] |X[f]|^2 (fp32, the
// filterbank row streamed once per frame), written [clip][m][frame] (the reference's S layout)
__global__ __launch_bounds__(256) void mel_power_kernel(const float* __restrict__ X, long ldx, int nbin, int T,
                                                        const float* __restrict__ fb, int n_mels,
                                                        float* __restrict__ S) {
  extern __shared__ float pw[];
  const int t = blockIdx.x, b = blockIdx.y;
  const float* xr = X + ((long)b * T + t) * ldx;
  for (int f = threadIdx.x; f < nbin; f += blockDim.x) {
    const float re = xr[f], im = xr[nbin + f];
    pw[f] = re * re + im * im;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  for (int m = w; m < n_mels; m += nw) {   // one wave per mel band: lanes stride the bins, then a wave sum
    const float* row = fb + (long)m * nbin;
    float acc = 0.f;
    for (int f = lane; f < nbin; f += 64) acc += row[f] * pw[f];
    acc = wave_sum(acc);
    if (lane == 0) S[((long)b * n_mels + m) * T + t] = acc;
  }
}

__device__ __forceinline__ float block_max(float v, float* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
  for (int i = 1; i < (int)(blockDim.x >> 6); ++i) t = fmaxf(t, red[i]);
  return t;
}

// cv2 INTER_LINEAR tap for destination index d: (source index, 11-bit weights)
__device__ __forceinline__ void cv_tap(int d, double scale, int sn, int& s0, int& a0, int& a1) {
  float fx = (float)((d + 0.5) * scale - 0.5);
  int sx = (int)floorf(fx);
  fx -= (float)sx;
  if (sx < 0) { fx = 0.f; sx = 0; }
  if (sx >= sn - 1) { fx = 0.f; sx = sn - 1; }
  s0 = sx;
  a0 = (int)rintf((1.f - fx) * 2048.f);
  a1 = (int)rintf(fx * 2048.f);
}

// one workgroup per clip: power_to_db(ref=max, top_db 80), cv2 min-max to [0, 255], uint8 truncation into an
// LDS image [n_mels][T], then the cv2 fixed-point bilinear resize to [oh][ow]
__global__ __launch_bounds__(1024) void mel_image_kernel(const float* __restrict__ S, int n_mels, int T, int oh, int ow,
                                                         uint8_t* __restrict__ out) {
  extern __shared__ uint8_t img[];
  __shared__ float red[16];
  const int b = blockIdx.x;
  const float* s = S + (long)b * n_mels * T;
  const long n = (long)n_mels * T;
  float mx = -INFINITY;
  for (long i = threadIdx.x; i < n; i += blockDim.x) mx = fmaxf(mx, s[i]);
  mx = block_max(mx, red);
  const float amin = 1e-10f;
  const float refdb = 10.f * log10f(fmaxf(amin, mx));
  // dB values, their max (0 up to rounding) and min after the top_db floor
  float dmx = -INFINITY, dmn = INFINITY;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    const float v = 10.f * log10f(fmaxf(amin, s[i])) - refdb;
    dmx = fmaxf(dmx, v);
    dmn = fminf(dmn, v);
  }
  dmx = block_max(dmx, red);
  dmn = -block_max(-dmn, red);
  const float floor_db = dmx - 80.f;
  const float lo = fmaxf(dmn, floor_db), hi = dmx;
  const double scale = hi > lo ? 255.0 / ((double)hi - (double)lo) : 0.0;
  const double shift = -(double)lo * scale;
  for (long i = threadIdx.x; i < n; i += blockDim.x) {
    float v = 10.f * log10f(fmaxf(amin, s[i])) - refdb;
    v = fmaxf(v, floor_db);
    const float q = (float)((double)v * scale + shift);   // cv2 convertTo (double scale / shift), float result
    img[i] = (uint8_t)fminf(fmaxf(q, 0.f), 255.f);        // astype(np.uint8): truncation
  }
  __syncthreads();
  const double sx = (double)T / ow, sy = (double)n_mels / oh;
  for (int p = threadIdx.x; p < oh * ow; p += blockDim.x) {
    const int dy = p / ow, dx = p % ow;
    int x0, ax0, ax1, y0, by0, by1;
    cv_tap(dx, sx, T, x0, ax0, ax1);
    cv_tap(dy, sy, n_mels, y0, by0, by1);
    const int x1 = min(x0 + 1, T - 1), y1 = min(y0 + 1, n_mels - 1);
    const int r0 = img[y0 * T + x0] * ax0 + img[y0 * T + x1] * ax1;
    const int r1 = img[y1 * T + x0] * ax0 + img[y1 * T + x1] * ax1;
    const int v = (by0 * r0 + by1 * r1 + (1 << 21)) >> 22;
    out[(long)b * oh * ow + p] = (uint8_t)min(max(v, 0), 255);
  }
}

// gray uint8 [N, HW] -> fp32 [N, 3, HW]: the RGB conversion replicates the channel, then ToTensor + Normalize
__global__ __launch_bounds__(256) void gray_norm_kernel(const uint8_t* __restrict__ src, float* __restrict__ dst, long n,
                                                        int HW, float m0, float m1, float m2, float s0, float s1,
                                                        float s2) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const long f = i / HW, o = i % HW;
  const float x = (float)src[i] / 255.f;
  float* out = dst + f * 3 * (long)HW + o;
  out[0] = (x - m0) / s0;
  out[HW] = (x - m1) / s1;
  out[2 * (long)HW] = (x - m2) / s2;
}

// ---- train-time frame transform, PIL semantics (data_process.py:62-69 on PIL images, src/utils.py:32-33) ----
// T.Resize((h, w)) on a PIL image is Image.resize(BILINEAR): PIL's two-pass separable resampling — a triangle
// filter whose support grows with the downscale factor (antialiased), coefficients normalised per output
// pixel and rounded to 22-bit fixed point (precompute_coeffs + normalize_coeffs_8bpc; built on the host,
// media.pil_bilinear_coeffs), the width pass first into uint8, then the height pass, each output rounded
// (+2^21) and clipped to uint8.  Flips are exact; T.RandomRotation on a PIL image is Image.rotate(NEAREST,
// fill 0): the 16.16 fixed-point inverse affine walk of PIL's affine_fixed (matrix built on the host exactly as
// PIL builds it, media.pil_rotate_fixed).  Then ToTensor + Normalize.
struct PilArgs {
  int H, W, cin, oh, ow, kx, ky;
  float m[3], sd[3];
};

// width pass: src [f][H][W][cin] -> tmp [f][H][ow][cin] (uint8); one thread per output pixel of a row
__global__ __launch_bounds__(256) void pil_resize_w_kernel(const uint8_t* __restrict__ src, long frames, PilArgs a,
                                                           const int* __restrict__ xb, const int* __restrict__ xk,
                                                           uint8_t* __restrict__ tmp) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long n = frames * a.H * a.ow;
  if (i >= n) return;
  const int x = (int)(i % a.ow);
  const long fr = i / a.ow;   // (frame, row)
  const int x0 = xb[2 * x], cnt = xb[2 * x + 1];
  const int* k = xk + (long)x * a.kx;
  const uint8_t* row = src + fr * a.W * a.cin;
  int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
  for (int t = 0; t < cnt; ++t) {
    const uint8_t* px = row + (long)(x0 + t) * a.cin;
    s0 += (int)px[0] * k[t];
    if (a.cin == 3) {
      s1 += (int)px[1] * k[t];
      s2 += (int)px[2] * k[t];
    }
  }
  uint8_t* o = tmp + i * a.cin;
  o[0] = (uint8_t)min(max(s0 >> 22, 0), 255);
  if (a.cin == 3) {
    o[1] = (uint8_t)min(max(s1 >> 22, 0), 255);
    o[2] = (uint8_t)min(max(s2 >> 22, 0), 255);
  }
}

// height pass of the resized pixel (y, x) fused with flips, rotation, ToTensor and Normalize
__global__ __launch_bounds__(256) void pil_augment_kernel(const uint8_t* __restrict__ tmp, long frames, PilArgs a,
                                                          const int* __restrict__ yb, const int* __restrict__ yk,
                                                          const int* __restrict__ flips, const int* __restrict__ aff,
                                                          float* __restrict__ dst) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per = (long)a.oh * a.ow;
  if (i >= frames * per) return;
  const long f = i / per;
  const int p = (int)(i % per), y = p / a.ow, x = p % a.ow;
  int iy = y, ix = x;
  bool in = true;
  if (aff && aff[8 * f]) {   // PIL affine_fixed: xx = a2 + x a0 + y a1, yy = a5 + x a3 + y a4 (16.16), >> 16
    const int* m = aff + 8 * f;
    const int xx = m[3] + x * m[1] + y * m[2], yy = m[6] + x * m[4] + y * m[5];
    ix = xx >> 16;
    iy = yy >> 16;
    in = ix >= 0 && ix < a.ow && iy >= 0 && iy < a.oh;
  }
  const int fl = flips ? flips[f] : 0;
  if (fl & 2) iy = a.oh - 1 - iy;   // vertical flip (applied before the rotation)
  if (fl & 1) ix = a.ow - 1 - ix;   // horizontal flip (first)
  float* out = dst + f * 3 * per + p;
  int v[3] = {0, 0, 0};
  if (in) {
    const int y0 = yb[2 * iy], cnt = yb[2 * iy + 1];
    const int* k = yk + (long)iy * a.ky;
    const uint8_t* col = tmp + (f * a.H * a.ow + ix) * a.cin;
    int s0 = 1 << 21, s1 = 1 << 21, s2 = 1 << 21;
    for (int t = 0; t < cnt; ++t) {
      const uint8_t* px = col + (long)(y0 + t) * a.ow * a.cin;
      s0 += (int)px[0] * k[t];
      if (a.cin == 3) {
        s1 += (int)px[1] * k[t];
        s2 += (int)px[2] * k[t];
      }
    }
    v[0] = min(max(s0 >> 22, 0), 255);
    v[1] = a.cin == 3 ? min(max(s1 >> 22, 0), 255) : v[0];
    v[2] = a.cin == 3 ? min(max(s2 >> 22, 0), 255) : v[0];
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) out[(long)c * per] = ((float)v[c] / 255.f - a.m[c]) / a.sd[c];
}

}  // namespace

extern "C" int64_t dfk_mel_workspace(int64_t B, int64_t S, int32_t n_fft, int32_t hop, int32_t n_mels) {
  if (B <= 0 || S <= 0 || n_fft <= 0 || hop <= 0 || n_mels <= 0) return -1;
  const long T = 1 + S / hop, Lp = S + n_fft, ldx = ((2 * (n_fft / 2 + 1) + 3) / 4) * 4;
  return 4 * (B * Lp + B * T * ldx + B * (long)n_mels * T) + 64;
}

extern "C" int dfk_mel_image(const float* wave, int64_t B, int64_t S, const float* basis, const float* fbank,
                             int32_t n_fft, int32_t hop, int32_t n_mels, int32_t out_h, int32_t out_w, void* ws,
                             int64_t ws_bytes, uint8_t* out, hipStream_t s) {
  if (!wave || !basis || !fbank || !ws || !out || B <= 0 || S <= 0 || n_fft <= 0 || n_fft % 4 || hop <= 0 ||
      hop % 4 || n_mels <= 0 || out_h <= 0 || out_w <= 0)
    return DFK_EINVAL;
  if (ws_bytes < dfk_mel_workspace(B, S, n_fft, hop, n_mels)) return DFK_EINVAL;
  const long T = 1 + S / hop, Lp = S + n_fft, nbin = n_fft / 2 + 1, ldx = ((2 * nbin + 3) / 4) * 4;
  if ((long)n_mels * T > 160 * 1024 - 256) return DFK_EINVAL;   // the uint8 image lives in LDS
  float* yp = reinterpret_cast<float*>(ws);
  float* X = yp + B * Lp;
  float* Sm = X + B * T * ldx;
  hipLaunchKernelGGL(mel_pad_kernel, dim3((unsigned)dfk_cdiv(Lp, 256), (unsigned)B), dim3(256), 0, s, wave, (long)S,
                     n_fft / 2, Lp, yp);
  DFK_CHECK_LAUNCH();
  // STFT: X[b][t][j] = sum_n yp[b][t*hop + n] basis[n][j]  (rows overlap: a strided view with ld = hop)
  dfk_gemm_args g = {};
  g.a.ptr = yp; g.a.ld = hop; g.a.bs0 = Lp;
  g.b.ptr = basis; g.b.ld = ldx;
  g.c = X; g.ldc = ldx; g.cbs0 = T * ldx;
  g.M = (int)T; g.N = (int)ldx; g.K = n_fft;
  g.dtype = DFK_F32; g.a_kmajor = 0; g.b_kmajor = 1; g.c_f32 = 1;
  g.nz0 = (int)B; g.nz1 = 1; g.splitk = 1;
  const int r = dfk_gemm(&g, s);
  if (r) return r;
  hipLaunchKernelGGL(mel_power_kernel, dim3((unsigned)T, (unsigned)B), dim3(256), 4 * nbin, s, X, ldx, (int)nbin,
                     (int)T, fbank, n_mels, Sm);
  static bool lds_attr = false;   // the uint8 image may take up to 160 KB of dynamic LDS (clips past ~12 s)
  if (!lds_attr) {
    // (160 KB minus the kernel's static reduction scratch: the attribute counts dynamic LDS only)
    (void)hipFuncSetAttribute((const void*)mel_image_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024 - 256);
    lds_attr = true;
  }
  hipLaunchKernelGGL(mel_image_kernel, dim3((unsigned)B), dim3(1024), (size_t)n_mels * T, s, Sm, n_mels, (int)T,
                     out_h, out_w, out);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_gray_normalize(const uint8_t* src, float* dst, int64_t n_img, int32_t H, int32_t W, const float* mean3,
                                  const float* std3, hipStream_t s) {
  if (!src || !dst || !mean3 || !std3 || H <= 0 || W <= 0) return DFK_EINVAL;
  const long n = n_img * (long)H * W;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(gray_norm_kernel, dim3((unsigned)dfk_cdiv(n, 256)), dim3(256), 0, s, src, dst, n, H * W, mean3[0],
                     mean3[1], mean3[2], std3[0], std3[1], std3[2]);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_frame_augment(const uint8_t* src, int64_t frames, const dfk_pil_resize* rs, const int32_t* flips,
                                 const int32_t* affine, const float* mean3, const float* std3, uint8_t* tmp, float* dst,
                                 hipStream_t s) {
  if (!src || !rs || !dst || !tmp || !mean3 || !std3) return DFK_EINVAL;
  const dfk_pil_resize& r = *rs;
  if (r.H <= 0 || r.W <= 0 || r.out_h <= 0 || r.out_w <= 0 || (r.cin != 1 && r.cin != 3)) return DFK_EINVAL;
  if (!r.xb || !r.xk || !r.yb || !r.yk || r.kx <= 0 || r.ky <= 0) return DFK_EINVAL;
  if (frames <= 0) return 0;
  PilArgs a;
  a.H = r.H; a.W = r.W; a.cin = r.cin; a.oh = r.out_h; a.ow = r.out_w; a.kx = r.kx; a.ky = r.ky;
  for (int c = 0; c < 3; ++c) { a.m[c] = mean3[c]; a.sd[c] = std3[c]; }
  const long nw = frames * (long)r.H * r.out_w;
  hipLaunchKernelGGL(pil_resize_w_kernel, dim3((unsigned)dfk_cdiv(nw, 256)), dim3(256), 0, s, src, (long)frames, a,
                     r.xb, r.xk, tmp);
  const long n = frames * (long)r.out_h * r.out_w;
  hipLaunchKernelGGL(pil_augment_kernel, dim3((unsigned)dfk_cdiv(n, 256)), dim3(256), 0, s, tmp, (long)frames, a,
                     r.yb, r.yk, flips, affine, dst);
  DFK_CHECK_LAUNCH();
  return 0;
}
