// LayerNorm forward/backward over the channel (last) dim — one wave per row.
// Rows are channels-last token vectors ([B,D,H,W,C] / [B,T,C]), so a row is a
// contiguous C-vector: 16-byte vector loads, two-pass statistics in registers.
#include "common.h"

namespace {

constexpr int MAXV = 8;  // up to 8 vectors of 8 per lane -> C <= 4096

template <typename T>
__device__ __forceinline__ void load8(const T* p, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const bf16raw* e = reinterpret_cast<const bf16raw*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bf2f(e[i]);
  } else {
    float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__device__ __forceinline__ void store8(T* p, const float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    uint4 u;
    bf16raw* e = reinterpret_cast<bf16raw*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) e[i] = f2bf(v[i]);
    *reinterpret_cast<uint4*>(p) = u;
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_fwd(const T* __restrict__ x, const T* __restrict__ w,
                                              const T* __restrict__ b, T* __restrict__ y, float* mean_out,
                                              float* rstd_out, long rows, int C, float eps) {
  const int lane = threadIdx.x & 63;
  const long row = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nv = C / 8;
  const T* xr = x + row * C;
  float v[MAXV][8];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      load8<T>(xr + vi * 8, v[i]);
#pragma unroll
      for (int e = 0; e < 8; ++e) s += v[i][e];
    }
  }
  const float mean = wave_sum(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    if (lane + i * 64 < nv) {
#pragma unroll
      for (int e = 0; e < 8; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
  }
  const float rstd = rsqrtf(wave_sum(q) / C + eps);
#pragma unroll
  for (int i = 0; i < MAXV; ++i) {
    const int vi = lane + i * 64;
    if (vi < nv) {
      float wv[8], bv[8], o[8];
      load8<T>(w + vi * 8, wv);
      load8<T>(b + vi * 8, bv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * wv[e] + bv[e];
      store8<T>(y + row * C + vi * 8, o);
    }
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g*xhat)),  g = dy*w ; dw += dy*xhat ; db += dy
// Two passes over the row (the second re-reads x/dy from L1/L2) keep only the
// per-lane dw/db partials live across rows.
constexpr int MAXVB = 6;  // C <= 3072 in the backward
template <typename T>
__global__ __launch_bounds__(256) void ln_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                              const T* __restrict__ w, const float* __restrict__ mean,
                                              const float* __restrict__ rstd, T* __restrict__ dx, float* dw,
                                              float* db, long rows, int C, int accumulate) {
  __shared__ float red[2][8 * 64 * MAXVB];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nv = C / 8;
  for (int i = threadIdx.x; i < C; i += 256) { red[0][i] = 0.f; red[1][i] = 0.f; }
  __syncthreads();
  float pw[MAXVB][8], pb[MAXVB][8];
#pragma unroll
  for (int i = 0; i < MAXVB; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { pw[i][e] = 0.f; pb[i][e] = 0.f; }
  const long stride = (long)gridDim.x * 4;
  for (long row = (long)blockIdx.x * 4 + wave; row < rows; row += stride) {
    const float mu = mean[row], rs = rstd[row];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < MAXVB; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        float xv[8], dv[8], wv[8];
        load8<T>(x + row * C + vi * 8, xv);
        load8<T>(dy + row * C + vi * 8, dv);
        load8<T>(w + vi * 8, wv);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (xv[e] - mu) * rs, g = dv[e] * wv[e];
          s1 += g;
          s2 += g * xh;
          pw[i][e] += dv[e] * xh;
          pb[i][e] += dv[e];
        }
      }
    }
    const float m1 = wave_sum(s1) / C, m2 = wave_sum(s2) / C;
#pragma unroll
    for (int i = 0; i < MAXVB; ++i) {
      const int vi = lane + i * 64;
      if (vi < nv) {
        float xv[8], dv[8], wv[8], o[8];
        load8<T>(x + row * C + vi * 8, xv);
        load8<T>(dy + row * C + vi * 8, dv);
        load8<T>(w + vi * 8, wv);
        if (accumulate) load8<T>(dx + row * C + vi * 8, o);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (xv[e] - mu) * rs;
          const float d = rs * (dv[e] * wv[e] - m1 - xh * m2);
          o[e] = accumulate ? o[e] + d : d;
        }
        store8<T>(dx + row * C + vi * 8, o);
      }
    }
  }
  for (int wv = 0; wv < 4; ++wv) {
    if (wave == wv) {
#pragma unroll
      for (int i = 0; i < MAXVB; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
#pragma unroll
          for (int e = 0; e < 8; ++e) { red[0][vi * 8 + e] += pw[i][e]; red[1][vi * 8 + e] += pb[i][e]; }
        }
      }
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < C; i += 256) {
    if (dw) atomicAdd(dw + i, red[0][i]);
    if (db) atomicAdd(db + i, red[1][i]);
  }
}

}  // namespace

extern "C" int dfk_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                                 int64_t rows, int32_t C, float eps, int dtype, hipStream_t s) {
  if (!x || !w || !b || !y || C % 8 || C > 8 * 64 * MAXV) return DFK_EINVAL;
  if (rows <= 0) return 0;
  dim3 grid(dfk_cdiv(rows, 4));
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(ln_fwd<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)x, (const bf16raw*)w,
                       (const bf16raw*)b, (bf16raw*)y, mean, rstd, (long)rows, C, eps);
  else
    hipLaunchKernelGGL(ln_fwd<float>, grid, dim3(256), 0, s, (const float*)x, (const float*)w, (const float*)b,
                       (float*)y, mean, rstd, (long)rows, C, eps);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                                 void* dx, float* dw, float* db, int64_t rows, int32_t C, int accumulate, int dtype,
                                 hipStream_t s) {
  if (!dy || !x || !w || !mean || !rstd || !dx || C % 8 || C > 8 * 64 * MAXVB) return DFK_EINVAL;
  if (rows <= 0) return 0;
  const int blocks = (int)std::min<int64_t>(1024, (rows + 3) / 4);
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(ln_bwd<bf16raw>, dim3(blocks), dim3(256), 0, s, (const bf16raw*)dy, (const bf16raw*)x,
                       (const bf16raw*)w, mean, rstd, (bf16raw*)dx, dw, db, (long)rows, C, accumulate);
  else
    hipLaunchKernelGGL(ln_bwd<float>, dim3(blocks), dim3(256), 0, s, (const float*)dy, (const float*)x,
                       (const float*)w, mean, rstd, (float*)dx, dw, db, (long)rows, C, accumulate);
  DFK_CHECK_LAUNCH();
  return 0;
}
