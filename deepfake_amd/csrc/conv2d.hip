// 2-D convolution support for the Inception-ResNet-v2 video branch (SURVEY.md §8f f4:
// src/models/InceptionResV2.py + IResNet.py): channels-last (NHWC) activations viewed as [N*H*W, C] rows with a
// row stride (so a branch can read / write a channel slice of a concat buffer in place).
//   im2col2d / col2im2d : the implicit-GEMM staging of k x k / strided convs (1x1 stride-1 convs need none)
//   bn2d                : BatchNorm2d in training mode (batch statistics over N*H*W, running-stat update),
//                         fused with the ReLU of the reference's Conv2d block; backward through both
//   pool2d              : MaxPool2d(3, s) and AvgPool2d(3, 1, 1, count_include_pad=False), forward / backward
// All reductions are fp32; activations bf16 or fp32.
#include "common.h"

namespace {

// out[(n*Ho + oh)*Wo + ow][(ky*kw + kx)*C + c] = x[n, oh*sh - ph + ky, ow*sw - pw + kx, c]  (0 outside)
template <typename T>
__global__ __launch_bounds__(256) void im2col2d_kernel(const T* __restrict__ x, long ldx, T* __restrict__ out,
                                                       int N, int H, int W, int C, int kh, int kw, int sh, int sw,
                                                       int ph, int pw, int Ho, int Wo) {
  const long cols = (long)kh * kw * C;
  const int VEC = (C % 8 == 0 && ldx % 8 == 0) ? 8 : 1;
  const long per_row = cols / VEC;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * Ho * Wo * per_row) return;
  const long r = idx / per_row;
  const long j = (idx % per_row) * VEC;
  const int tap = (int)(j / C), c = (int)(j % C);
  const int ky = tap / kw, kx = tap % kw;
  const int ow = (int)(r % Wo), oh = (int)((r / Wo) % Ho), n = (int)(r / ((long)Wo * Ho));
  const int y = oh * sh - ph + ky, xx = ow * sw - pw + kx;
  const bool ok = y >= 0 && y < H && xx >= 0 && xx < W;
  T* dst = out + r * cols + j;
  const T* src = x + (ok ? (((long)n * H + y) * W + xx) * ldx + c : 0);
  if (VEC == 8) {   // 8 channels: one bf16 / two fp32 16-B vectors
    if constexpr (sizeof(T) == 2) {
      const uint4 v = ok ? *reinterpret_cast<const uint4*>(src) : make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      reinterpret_cast<float4*>(dst)[0] = ok ? reinterpret_cast<const float4*>(src)[0] : z;
      reinterpret_cast<float4*>(dst)[1] = ok ? reinterpret_cast<const float4*>(src)[1] : z;
    }
  } else {
    *dst = ok ? x[(((long)n * H + y) * W + xx) * ldx + c] : (T)0;
  }
}

// dx[n, y, x, c] (+)= sum over the taps / output pixels that read it of dcols  (gather: no atomics)
template <typename T>
__global__ __launch_bounds__(256) void col2im2d_kernel(const T* __restrict__ dcols, T* __restrict__ dx, long ldx,
                                                       int N, int H, int W, int C, int kh, int kw, int sh, int sw,
                                                       int ph, int pw, int Ho, int Wo, int accumulate) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * H * W * C) return;
  const int c = (int)(idx % C);
  const long p = idx / C;
  const int xx = (int)(p % W), y = (int)((p / W) % H), n = (int)(p / ((long)W * H));
  const long cols = (long)kh * kw * C;
  float s = 0.f;
  for (int ky = 0; ky < kh; ++ky) {
    const int t = y + ph - ky;
    if (t < 0 || t % sh) continue;
    const int oh = t / sh;
    if (oh >= Ho) continue;
    for (int kx = 0; kx < kw; ++kx) {
      const int u = xx + pw - kx;
      if (u < 0 || u % sw) continue;
      const int ow = u / sw;
      if (ow >= Wo) continue;
      s += ldf<T>(dcols + (((long)n * Ho + oh) * Wo + ow) * cols + (ky * kw + kx) * C + c);
    }
  }
  T* d = dx + p * ldx + c;
  stf<T>(d, accumulate ? ldf<T>(d) + s : s);
}

// per-channel statistics over rows in two passes (fp32 atomics per block and channel): pass 0 sums x into
// acc[0:C]; pass 1 sums (x - mean)^2 into acc[C:2C] with mean = acc[c] / rows (no E[x^2] - m^2 cancellation)
template <typename T>
__global__ __launch_bounds__(256) void bn_stats_kernel(const T* __restrict__ x, long ldx, long rows, int C,
                                                       long rows_per, float* __restrict__ acc, int pass) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  const float m = pass ? acc[c] / (float)rows : 0.f;
  float s = 0.f;
  for (long r = r0; r < r1; ++r) {
    const float v = ldf<T>(x + r * ldx + c) - m;
    s += pass ? v * v : v;
  }
  atomicAdd(acc + pass * C + c, s);
}

// mean / rstd from the sums; running stats (momentum, unbiased variance) as nn.BatchNorm2d.train()
__global__ void bn_finalize_kernel(const float* __restrict__ acc, long n, int C, float eps, float momentum,
                                   float* __restrict__ mean, float* __restrict__ rstd, float* __restrict__ rmean,
                                   float* __restrict__ rvar) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float m = acc[c] / n;
  const float var = acc[C + c] / n;
  mean[c] = m;
  rstd[c] = rsqrtf(var + eps);
  if (rmean) {
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * m;
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * var * (n > 1 ? (float)n / (float)(n - 1) : 1.f);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void bn_apply_kernel(const T* __restrict__ x, long ldx, T* __restrict__ y, long ldy,
                                                       long rows, int C, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ g,
                                                       const float* __restrict__ b, int relu) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * C) return;
  const long r = idx / C;
  const int c = (int)(idx % C);
  float v = (ldf<T>(x + r * ldx + c) - mean[c]) * rstd[c] * g[c] + b[c];
  if (relu) v = fmaxf(v, 0.f);
  stf<T>(y + r * ldy + c, v);
}

// backward sums: s1 = sum dy', s2 = sum dy' * xhat with dy' = dy * (y > 0) under ReLU
template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_stats_kernel(const T* __restrict__ dy, long lddy, const T* __restrict__ y,
                                                           long ldy, const T* __restrict__ x, long ldx, long rows, int C,
                                                           long rows_per, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, int relu,
                                                           float* __restrict__ acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const long r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  const float m = mean[c], rs = rstd[c];
  float s1 = 0.f, s2 = 0.f;
  for (long r = r0; r < r1; ++r) {
    float d = ldf<T>(dy + r * lddy + c);
    if (relu && !(ldf<T>(y + r * ldy + c) > 0.f)) d = 0.f;
    s1 += d;
    s2 += d * (ldf<T>(x + r * ldx + c) - m) * rs;
  }
  atomicAdd(acc + c, s1);
  atomicAdd(acc + C + c, s2);
}

template <typename T>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const T* __restrict__ dy, long lddy, const T* __restrict__ y,
                                                           long ldy, const T* __restrict__ x, long ldx, T* __restrict__ dx,
                                                           long lddx, long rows, int C, const float* __restrict__ mean,
                                                           const float* __restrict__ rstd, const float* __restrict__ g,
                                                           int relu, const float* __restrict__ acc) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * C) return;
  const long r = idx / C;
  const int c = (int)(idx % C);
  float d = ldf<T>(dy + r * lddy + c);
  if (relu && !(ldf<T>(y + r * ldy + c) > 0.f)) d = 0.f;
  const float xh = (ldf<T>(x + r * ldx + c) - mean[c]) * rstd[c];
  const float inv_n = 1.f / (float)rows;
  stf<T>(dx + r * lddx + c, g[c] * rstd[c] * (d - acc[c] * inv_n - xh * acc[C + c] * inv_n));
}

// pooling, 3 x 3 windows: mode 0 = max (no padding), mode 1 = average with padding excluded from the count
template <typename T>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const T* __restrict__ x, long ldx, T* __restrict__ y, long ldy,
                                                       int N, int H, int W, int C, int k, int s, int p, int Ho, int Wo,
                                                       int mode) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * Ho * Wo * C) return;
  const int c = (int)(idx % C);
  const long o = idx / C;
  const int ow = (int)(o % Wo), oh = (int)((o / Wo) % Ho), n = (int)(o / ((long)Wo * Ho));
  float acc = mode == 0 ? -INFINITY : 0.f;
  int cnt = 0;
  for (int ky = 0; ky < k; ++ky) {
    const int yy = oh * s - p + ky;
    if (yy < 0 || yy >= H) continue;
    for (int kx = 0; kx < k; ++kx) {
      const int xx = ow * s - p + kx;
      if (xx < 0 || xx >= W) continue;
      const float v = ldf<T>(x + (((long)n * H + yy) * W + xx) * ldx + c);
      acc = mode == 0 ? fmaxf(acc, v) : acc + v;
      ++cnt;
    }
  }
  stf<T>(y + o * ldy + c, mode == 0 ? acc : acc / (float)max(cnt, 1));
}

// gather backward: input pixel (n, yy, xx, c) collects from every output window containing it (max: only when
// it is that window's first maximum, as PyTorch's max-pool index)
template <typename T>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const T* __restrict__ x, long ldx, const T* __restrict__ dy,
                                                       long lddy, T* __restrict__ dx, long lddx, int N, int H, int W,
                                                       int C, int k, int s, int p, int Ho, int Wo, int mode,
                                                       int accumulate) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (long)N * H * W * C) return;
  const int c = (int)(idx % C);
  const long pix = idx / C;
  const int xx = (int)(pix % W), yy = (int)((pix / W) % H), n = (int)(pix / ((long)W * H));
  float g = 0.f;
  for (int ky = 0; ky < k; ++ky) {
    const int t = yy + p - ky;
    if (t < 0 || t % s) continue;
    const int oh = t / s;
    if (oh >= Ho) continue;
    for (int kx = 0; kx < k; ++kx) {
      const int u = xx + p - kx;
      if (u < 0 || u % s) continue;
      const int ow = u / s;
      if (ow >= Wo) continue;
      const float d = ldf<T>(dy + (((long)n * Ho + oh) * Wo + ow) * lddy + c);
      if (mode == 1) {
        int cnt = 0;
        for (int a = 0; a < k; ++a)
          for (int bb = 0; bb < k; ++bb) {
            const int y2 = oh * s - p + a, x2 = ow * s - p + bb;
            cnt += (y2 >= 0 && y2 < H && x2 >= 0 && x2 < W) ? 1 : 0;
          }
        g += d / (float)max(cnt, 1);
      } else {   // first maximum of the window (row-major scan), as at::max_pool2d's index
        float best = -INFINITY;
        int by = -1, bx = -1;
        for (int a = 0; a < k; ++a)
          for (int bb = 0; bb < k; ++bb) {
            const int y2 = oh * s - p + a, x2 = ow * s - p + bb;
            if (y2 < 0 || y2 >= H || x2 < 0 || x2 >= W) continue;
            const float v = ldf<T>(x + (((long)n * H + y2) * W + x2) * ldx + c);
            if (v > best || by < 0) { best = v; by = y2; bx = x2; }
          }
        if (by == yy && bx == xx) g += d;
      }
    }
  }
  T* dp = dx + pix * lddx + c;
  stf<T>(dp, accumulate ? ldf<T>(dp) + g : g);
}

__global__ void acc_add_kernel(const float* __restrict__ src, float* __restrict__ dst, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] += src[i];
}

long rows_per_block(long rows) { return rows < 256 ? rows : std::max<long>(64, rows / 512); }

}  // namespace

extern "C" int dfk_im2col2d(const void* x, int64_t ldx, void* out, const dfk_conv2d_geo* g, int dtype, hipStream_t s) {
  if (!x || !out || !g || g->C <= 0 || g->kh <= 0 || g->kw <= 0 || g->sh <= 0 || g->sw <= 0) return DFK_EINVAL;
  const long cols = (long)g->kh * g->kw * g->C;
  const int vec = (g->C % 8 == 0 && ldx % 8 == 0) ? 8 : 1;
  const long n = (long)g->N * g->Ho * g->Wo * (cols / vec);
  if (n <= 0) return 0;
  const dim3 grid((unsigned)dfk_cdiv(n, 256));
#define IM2COL(T) hipLaunchKernelGGL(im2col2d_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (T*)out, g->N, \
                                     g->H, g->W, g->C, g->kh, g->kw, g->sh, g->sw, g->ph, g->pw, g->Ho, g->Wo)
  if (dtype == DFK_BF16) IM2COL(bf16raw); else IM2COL(float);
#undef IM2COL
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_col2im2d(const void* dcols, void* dx, int64_t ldx, const dfk_conv2d_geo* g, int accumulate,
                            int dtype, hipStream_t s) {
  if (!dcols || !dx || !g || g->C <= 0) return DFK_EINVAL;
  const long n = (long)g->N * g->H * g->W * g->C;
  if (n <= 0) return 0;
  const dim3 grid((unsigned)dfk_cdiv(n, 256));
#define COL2IM(T) hipLaunchKernelGGL(col2im2d_kernel<T>, grid, dim3(256), 0, s, (const T*)dcols, (T*)dx, (long)ldx, g->N, \
                                     g->H, g->W, g->C, g->kh, g->kw, g->sh, g->sw, g->ph, g->pw, g->Ho, g->Wo, accumulate)
  if (dtype == DFK_BF16) COL2IM(bf16raw); else COL2IM(float);
#undef COL2IM
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_bn2d_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t rows, int32_t C,
                            const float* gamma, const float* beta, float eps, float momentum, int relu, float* mean,
                            float* rstd, float* running_mean, float* running_var, float* ws, int dtype, hipStream_t s) {
  if (!x || !y || !gamma || !beta || !mean || !rstd || !ws || C <= 0 || (!running_mean != !running_var))
    return DFK_EINVAL;
  if (rows <= 0) return 0;
  (void)hipMemsetAsync(ws, 0, 2 * (size_t)C * 4, s);
  const long rpb = rows_per_block(rows);
  {
    const dim3 grid(dfk_cdiv(C, 256), (unsigned)dfk_cdiv(rows, rpb));
#define BNS(T, P) hipLaunchKernelGGL(bn_stats_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (long)rows, \
                                     (int)C, rpb, ws, P)
    if (dtype == DFK_BF16) { BNS(bf16raw, 0); BNS(bf16raw, 1); } else { BNS(float, 0); BNS(float, 1); }
#undef BNS
  }
  hipLaunchKernelGGL(bn_finalize_kernel, dim3(dfk_cdiv(C, 256)), dim3(256), 0, s, ws, (long)rows, (int)C, eps, momentum,
                     mean, rstd, running_mean, running_var);
  const dim3 grid((unsigned)dfk_cdiv(rows * C, 256));
#define BNA(T) hipLaunchKernelGGL(bn_apply_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (T*)y, (long)ldy, \
                                  (long)rows, (int)C, mean, rstd, gamma, beta, relu)
  if (dtype == DFK_BF16) BNA(bf16raw); else BNA(float);
#undef BNA
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_bn2d_apply(const void* x, int64_t ldx, void* y, int64_t ldy, int64_t rows, int32_t C,
                              const float* mean, const float* rstd, const float* gamma, const float* beta, int relu,
                              int dtype, hipStream_t s) {
  if (!x || !y || !mean || !rstd || !gamma || !beta || C <= 0) return DFK_EINVAL;
  if (rows <= 0) return 0;
  const dim3 grid((unsigned)dfk_cdiv(rows * C, 256));
#define BNA(T) hipLaunchKernelGGL(bn_apply_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (T*)y, (long)ldy, \
                                  (long)rows, (int)C, mean, rstd, gamma, beta, relu)
  if (dtype == DFK_BF16) BNA(bf16raw); else BNA(float);
#undef BNA
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_bn2d_bwd(const void* dy, int64_t lddy, const void* y, int64_t ldy, const void* x, int64_t ldx,
                            void* dx, int64_t lddx, int64_t rows, int32_t C, const float* mean, const float* rstd,
                            const float* gamma, int relu, float* dgamma, float* dbeta, float* ws, int dtype,
                            hipStream_t s) {
  if (!dy || !x || !dx || !mean || !rstd || !gamma || !ws || C <= 0 || (relu && !y)) return DFK_EINVAL;
  if (rows <= 0) return 0;
  (void)hipMemsetAsync(ws, 0, 2 * (size_t)C * 4, s);
  const long rpb = rows_per_block(rows);
  const dim3 grid(dfk_cdiv(C, 256), (unsigned)dfk_cdiv(rows, rpb));
#define BBS(T) hipLaunchKernelGGL(bn_bwd_stats_kernel<T>, grid, dim3(256), 0, s, (const T*)dy, (long)lddy, (const T*)y, \
                                  (long)ldy, (const T*)x, (long)ldx, (long)rows, (int)C, rpb, mean, rstd, relu, ws)
  if (dtype == DFK_BF16) BBS(bf16raw); else BBS(float);
#undef BBS
  if (dgamma) hipLaunchKernelGGL(acc_add_kernel, dim3(dfk_cdiv(C, 256)), dim3(256), 0, s, ws + C, dgamma, (int)C);
  if (dbeta) hipLaunchKernelGGL(acc_add_kernel, dim3(dfk_cdiv(C, 256)), dim3(256), 0, s, ws, dbeta, (int)C);
  const dim3 g2((unsigned)dfk_cdiv(rows * C, 256));
#define BBA(T) hipLaunchKernelGGL(bn_bwd_apply_kernel<T>, g2, dim3(256), 0, s, (const T*)dy, (long)lddy, (const T*)y, \
                                  (long)ldy, (const T*)x, (long)ldx, (T*)dx, (long)lddx, (long)rows, (int)C, mean, rstd, \
                                  gamma, relu, ws)
  if (dtype == DFK_BF16) BBA(bf16raw); else BBA(float);
#undef BBA
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_pool2d_fwd(const void* x, int64_t ldx, void* y, int64_t ldy, const dfk_conv2d_geo* g, int mode,
                              int dtype, hipStream_t s) {
  if (!x || !y || !g || g->C <= 0 || g->kh != g->kw || g->sh != g->sw || g->ph != g->pw || (mode != 0 && mode != 1))
    return DFK_EINVAL;
  const long n = (long)g->N * g->Ho * g->Wo * g->C;
  if (n <= 0) return 0;
  const dim3 grid((unsigned)dfk_cdiv(n, 256));
#define PF(T) hipLaunchKernelGGL(pool_fwd_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (T*)y, (long)ldy, g->N, \
                                 g->H, g->W, g->C, g->kh, g->sh, g->ph, g->Ho, g->Wo, mode)
  if (dtype == DFK_BF16) PF(bf16raw); else PF(float);
#undef PF
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_pool2d_bwd(const void* x, int64_t ldx, const void* dy, int64_t lddy, void* dx, int64_t lddx,
                              const dfk_conv2d_geo* g, int mode, int accumulate, int dtype, hipStream_t s) {
  if (!x || !dy || !dx || !g || g->C <= 0 || g->kh != g->kw || g->sh != g->sw || g->ph != g->pw) return DFK_EINVAL;
  const long n = (long)g->N * g->H * g->W * g->C;
  if (n <= 0) return 0;
  const dim3 grid((unsigned)dfk_cdiv(n, 256));
#define PB(T) hipLaunchKernelGGL(pool_bwd_kernel<T>, grid, dim3(256), 0, s, (const T*)x, (long)ldx, (const T*)dy, (long)lddy, \
                                 (T*)dx, (long)lddx, g->N, g->H, g->W, g->C, g->kh, g->sh, g->ph, g->Ho, g->Wo, mode, accumulate)
  if (dtype == DFK_BF16) PB(bf16raw); else PB(float);
#undef PB
  DFK_CHECK_LAUNCH();
  return 0;
}
