// wav2vec2 feature-encoder layer 0 (HF modeling_wav2vec2.py:302-323):
//   y[b,t,c] = sum_k w[c,k] x[b,5t+k]          Conv1d(1->512, k10, s5, no bias)
//   z = GroupNorm(512 groups = per channel over time, affine)(y)
//   out = gelu(z)   written channels-last [B, T0, 512] for the implicit-GEMM conv1
// GroupNorm needs whole-time statistics per (clip, channel), so the forward is
// two passes that both recompute the 10-tap conv from the waveform (the
// waveform is 0.26 MB/clip; y is never stored), and the backward likewise.
// The conv itself is VALU work (10 MACs / output) — the pass is HBM-bound on
// the 13 MB/clip output (bf16).
#include "common.h"

namespace {

constexpr int TB = 64;    // time steps per workgroup
constexpr int CH = 512;   // channels (conv_dim[0])
constexpr int KW = 10, KS = 5;

// stage the waveform segment of this time block and the conv weights into LDS
__device__ __forceinline__ void stage(const float* __restrict__ x, const float* __restrict__ w, long S, int b, int t0,
                                      float* xs, float* ws) {
  const long base = (long)b * S + (long)t0 * KS;
  for (int i = threadIdx.x; i < TB * KS + KW; i += 256) {
    const long j = base + i;
    xs[i] = ((long)t0 * KS + i < S) ? x[j] : 0.f;
  }
  for (int i = threadIdx.x; i < CH * KW; i += 256) ws[i] = w[i];
  __syncthreads();
}

__device__ __forceinline__ float conv_at(const float* xs, const float* ws, int tl, int c) {
  float y = 0.f;
#pragma unroll
  for (int k = 0; k < KW; ++k) y += ws[c * KW + k] * xs[tl * KS + k];
  return y;
}

// pass 1: per (b, time block, c) partial sum and sum of squares of y -> the partial slab [b][block][c][2]
__global__ __launch_bounds__(256) void conv0_stats(const float* __restrict__ x, const float* __restrict__ w, long S,
                                                   int T0, float* __restrict__ part) {
  __shared__ float xs[TB * KS + KW];
  __shared__ float ws[CH * KW];
  const int b = blockIdx.y, t0 = blockIdx.x * TB;
  stage(x, w, S, b, t0, xs, ws);
  const int nt = min(TB, T0 - t0);
  for (int c = threadIdx.x; c < CH; c += 256) {
    float s = 0.f, q = 0.f;
    for (int tl = 0; tl < nt; ++tl) {
      const float y = conv_at(xs, ws, tl, c);
      s += y;
      q += y * y;
    }
    float* dst = part + (((long)b * gridDim.x + blockIdx.x) * CH + c) * 2;
    dst[0] = s;
    dst[1] = q;
  }
}

// pass 1b: stats[b][c][2] = sum over the time blocks of the partials, in a fixed order (4 interleaved row phases,
// then (p0 + p1) + (p2 + p3)): the forward's GroupNorm statistics, and so the loss, are bitwise reproducible
__global__ __launch_bounds__(256) void conv0_stats_sum(const float* __restrict__ part, int nblk,
                                                       float* __restrict__ stats) {
  __shared__ float red[4][64];
  const int b = blockIdx.y, lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;   // column of the [CH][2] row
  const float* src = part + (long)b * nblk * CH * 2 + j;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  int r = ph;
  for (; r + 12 < nblk; r += 16) {
#pragma unroll
    for (int u = 0; u < 4; ++u) a[u] += src[(long)(r + 4 * u) * CH * 2];
  }
  for (; r < nblk; r += 4) a[0] += src[(long)r * CH * 2];
  red[ph][lane] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (ph == 0) stats[(long)b * CH * 2 + j] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

// pass 2: out = gelu(gn(y)); one thread per (t, channel pair) -> coalesced channels-last stores
template <typename T>
__global__ __launch_bounds__(256) void conv0_apply(const float* __restrict__ x, const float* __restrict__ w, long S,
                                                   int T0, const float* __restrict__ stats, const float* __restrict__ gamma,
                                                   const float* __restrict__ beta, float eps, T* __restrict__ out) {
  __shared__ float xs[TB * KS + KW];
  __shared__ float ws[CH * KW];
  __shared__ float mu[CH], rs[CH];
  const int b = blockIdx.y, t0 = blockIdx.x * TB;
  stage(x, w, S, b, t0, xs, ws);
  for (int c = threadIdx.x; c < CH; c += 256) {
    const float s = stats[((long)b * CH + c) * 2], q = stats[((long)b * CH + c) * 2 + 1];
    const float m = s / T0;
    mu[c] = m;
    rs[c] = rsqrtf(fmaxf(q / T0 - m * m, 0.f) + eps);
  }
  __syncthreads();
  const int nt = min(TB, T0 - t0);
  for (int i = threadIdx.x; i < nt * CH; i += 256) {
    const int tl = i / CH, c = i % CH;
    const float y = conv_at(xs, ws, tl, c);
    const float z = (y - mu[c]) * rs[c] * gamma[c] + beta[c];
    stf<T>(out + ((long)b * T0 + t0 + tl) * CH + c, (sizeof(T) == 2 ? gelu_bf(z) : gelu_f(z)));
  }
}

// backward pass 1: per (b,c) A = sum_t dz*yhat, Bs = sum_t dz   (dz = dout * gelu'(z))
template <typename T>
__global__ __launch_bounds__(256) void conv0_bwd_stats(const float* __restrict__ x, const float* __restrict__ w, long S,
                                                       int T0, const float* __restrict__ stats,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, const T* __restrict__ dout, float* __restrict__ red) {
  __shared__ float xs[TB * KS + KW];
  __shared__ float ws[CH * KW];
  const int b = blockIdx.y, t0 = blockIdx.x * TB;
  stage(x, w, S, b, t0, xs, ws);
  const int nt = min(TB, T0 - t0);
  for (int c = threadIdx.x; c < CH; c += 256) {
    const float s = stats[((long)b * CH + c) * 2], q = stats[((long)b * CH + c) * 2 + 1];
    const float m = s / T0, r = rsqrtf(fmaxf(q / T0 - m * m, 0.f) + eps);
    float A = 0.f, Bs = 0.f;
    for (int tl = 0; tl < nt; ++tl) {
      const float yh = (conv_at(xs, ws, tl, c) - m) * r;
      const float dz = ldf<T>(dout + ((long)b * T0 + t0 + tl) * CH + c) * (sizeof(T) == 2 ? dgelu_bf(yh * gamma[c] + beta[c]) : dgelu_f(yh * gamma[c] + beta[c]));
      A += dz * yh;
      Bs += dz;
    }
    atomicAdd(red + ((long)b * CH + c) * 2, A);
    atomicAdd(red + ((long)b * CH + c) * 2 + 1, Bs);
  }
}

// backward pass 2: dy = rstd*(gamma*dz - gamma*Bs/T0 - yhat*gamma*A/T0);  dw[c,k] += sum_t dy x[5t+k]
template <typename T>
__global__ __launch_bounds__(256) void conv0_bwd_dw(const float* __restrict__ x, const float* __restrict__ w, long S,
                                                    int T0, const float* __restrict__ stats,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    float eps, const T* __restrict__ dout, const float* __restrict__ red,
                                                    float* __restrict__ part) {
  // each workgroup sweeps a strided set of time blocks and keeps its dw partials in registers, then writes
  // them once to its slab row (four workgroups per CU: the recompute of conv + GroupNorm + GELU' is VALU work
  // that one wave per SIMD left latency-bound)
  __shared__ float xs[TB * KS + KW];
  __shared__ float ws[CH * KW];
  const int b = blockIdx.y;
  for (int i = threadIdx.x; i < CH * KW; i += 256) ws[i] = w[i];
  constexpr int CPT = CH / 256;   // channels per thread
  float acc[CPT][KW], m[CPT], r[CPT], g[CPT], be[CPT], A[CPT], Bm[CPT];
#pragma unroll
  for (int j = 0; j < CPT; ++j) {
    const int c = threadIdx.x + j * 256;
    const float s = stats[((long)b * CH + c) * 2], q = stats[((long)b * CH + c) * 2 + 1];
    m[j] = s / T0;
    r[j] = rsqrtf(fmaxf(q / T0 - m[j] * m[j], 0.f) + eps);
    g[j] = gamma[c];
    be[j] = beta[c];
    A[j] = red[((long)b * CH + c) * 2] * g[j] / T0;
    Bm[j] = red[((long)b * CH + c) * 2 + 1] * g[j] / T0;
#pragma unroll
    for (int k = 0; k < KW; ++k) acc[j][k] = 0.f;
  }
  const int ntb = (T0 + TB - 1) / TB;
  for (int tb = blockIdx.x; tb < ntb; tb += gridDim.x) {
    const int t0 = tb * TB;
    __syncthreads();
    const long base = (long)b * S + (long)t0 * KS;
    for (int i = threadIdx.x; i < TB * KS + KW; i += 256) xs[i] = ((long)t0 * KS + i < S) ? x[base + i] : 0.f;
    __syncthreads();
    const int nt = min(TB, T0 - t0);
    for (int tl = 0; tl < nt; ++tl) {
#pragma unroll
      for (int j = 0; j < CPT; ++j) {
        const int c = threadIdx.x + j * 256;
        const float yh = (conv_at(xs, ws, tl, c) - m[j]) * r[j];
        const float dz = ldf<T>(dout + ((long)b * T0 + t0 + tl) * CH + c) * (sizeof(T) == 2 ? dgelu_bf(yh * g[j] + be[j]) : dgelu_f(yh * g[j] + be[j]));
        const float dy = r[j] * (g[j] * dz - Bm[j] - yh * A[j]);
#pragma unroll
        for (int k = 0; k < KW; ++k) acc[j][k] += dy * xs[tl * KS + k];
      }
    }
  }
  // this workgroup's partial -> its slab row (summed by dw_slab_sum: no same-address atomics across the
  // workgroups of the grid)
  float* row = part + ((long)blockIdx.y * gridDim.x + blockIdx.x) * (CH * KW);
#pragma unroll
  for (int j = 0; j < CPT; ++j)
#pragma unroll
    for (int k = 0; k < KW; ++k) row[(threadIdx.x + j * 256) * KW + k] = acc[j][k];
}

// dw[i] += sum over the slab rows of part[r][i]  (i < CH*KW): workgroup = 64 columns x one 128-row chunk,
// 4 row phases x 8 loads in flight per lane, one atomic per column and chunk
__global__ __launch_bounds__(256) void dw_slab_sum(const float* __restrict__ part, int rows, float* __restrict__ dw) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * 128, r1 = min(rows, r0 + 128);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (i < CH * KW) {
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const int r = r0 + ph + 4 * u;
      if (r < r1) s[u & 7] += part[(long)r * (CH * KW) + i];
    }
  }
  red[ph][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (ph == 0 && i < CH * KW) atomicAdd(dw + i, (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]));
}

// dgamma[c] += sum_b A[b,c] ; dbeta[c] += sum_b Bs[b,c]
__global__ void gn_affine_grad(const float* __restrict__ red, int B, float* dgamma, float* dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= CH) return;
  float a = 0.f, bs = 0.f;
  for (int b = 0; b < B; ++b) { a += red[((long)b * CH + c) * 2]; bs += red[((long)b * CH + c) * 2 + 1]; }
  if (dgamma) dgamma[c] += a;
  if (dbeta) dbeta[c] += bs;
}

// workgroups per clip of the dw pass: about four per CU over the batch
int conv0_dw_blocks(long B, int T0) { return std::min(dfk_cdiv(T0, TB), std::max(1, (int)(1024 / B))); }

}  // namespace

extern "C" int64_t dfk_w2v_conv0_bwd_workspace(int64_t B, int64_t S) {
  if (B <= 0 || S < KW) return 0;
  const int T0 = (int)((S - KW) / KS + 1);
  return (int64_t)4 * (B * CH * 2 + B * conv0_dw_blocks(B, T0) * (int64_t)(CH * KW));
}

extern "C" int64_t dfk_w2v_conv0_fwd_workspace(int64_t B, int64_t S) {
  if (B <= 0 || S < KW) return 0;
  const int T0 = (int)((S - KW) / KS + 1);
  return (int64_t)4 * B * dfk_cdiv(T0, TB) * CH * 2;
}

extern "C" int dfk_w2v_conv0_fwd(const float* wave, int64_t B, int64_t S, const float* w, const float* gamma,
                                 const float* beta, float eps, float* stats, void* out, int dtype, float* ws,
                                 hipStream_t s) {
  if (!wave || !w || !gamma || !beta || !stats || !out || !ws || S < KW) return DFK_EINVAL;
  const int T0 = (int)((S - KW) / KS + 1);
  const dim3 grid(dfk_cdiv(T0, TB), (unsigned)B);
  static_assert((CH * 2) % 64 == 0, "stats columns per workgroup");
  hipLaunchKernelGGL(conv0_stats, grid, dim3(256), 0, s, wave, w, (long)S, T0, ws);
  hipLaunchKernelGGL(conv0_stats_sum, dim3(CH * 2 / 64, (unsigned)B), dim3(256), 0, s, ws, (int)grid.x, stats);
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(conv0_apply<bf16raw>, grid, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (bf16raw*)out);
  else
    hipLaunchKernelGGL(conv0_apply<float>, grid, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (float*)out);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_w2v_conv0_bwd(const float* wave, int64_t B, int64_t S, const float* w, const float* gamma,
                                 const float* beta, float eps, const float* stats, const void* dout, int dtype,
                                 float* scratch, int64_t scratch_bytes, float* dw, float* dgamma, float* dbeta,
                                 hipStream_t s) {
  if (!wave || !w || !gamma || !beta || !stats || !dout || !scratch || !dw || S < KW) return DFK_EINVAL;
  if (scratch_bytes < dfk_w2v_conv0_bwd_workspace(B, S)) return DFK_EINVAL;   // the dw slab is sized per launch
  const int T0 = (int)((S - KW) / KS + 1);
  const dim3 grid(dfk_cdiv(T0, TB), (unsigned)B);
  const dim3 gdw(conv0_dw_blocks(B, T0), (unsigned)B);
  float* part = scratch + B * CH * 2;   // [B * gdw.x][CH * KW] slab after the [B, CH, 2] reductions
  (void)hipMemsetAsync(scratch, 0, sizeof(float) * B * CH * 2, s);
  if (dtype == DFK_BF16) {
    hipLaunchKernelGGL(conv0_bwd_stats<bf16raw>, grid, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (const bf16raw*)dout, scratch);
    hipLaunchKernelGGL(conv0_bwd_dw<bf16raw>, gdw, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (const bf16raw*)dout, scratch, part);
  } else {
    hipLaunchKernelGGL(conv0_bwd_stats<float>, grid, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (const float*)dout, scratch);
    hipLaunchKernelGGL(conv0_bwd_dw<float>, gdw, dim3(256), 0, s, wave, w, (long)S, T0, stats, gamma, beta, eps,
                       (const float*)dout, scratch, part);
  }
  hipLaunchKernelGGL(dw_slab_sum, dim3(dfk_cdiv(CH * KW, 64), dfk_cdiv(B * gdw.x, 128)), dim3(256), 0, s, part,
                     (int)(B * gdw.x), dw);
  if (dgamma || dbeta)
    hipLaunchKernelGGL(gn_affine_grad, dim3(dfk_cdiv(CH, 256)), dim3(256), 0, s, scratch, (int)B, dgamma, dbeta);
  DFK_CHECK_LAUNCH();
  return 0;
}
