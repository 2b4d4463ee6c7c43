// SwinV2 continuous position bias (swin_transformer2d.py:99-100,159-162): the cpb_mlp over the
// relative_coords_table and 16*sigmoid, forward and backward, in fp32 straight from the parameters.
// The reference runs this as Linear -> ReLU -> Linear -> sigmoid -> mul (and their backward) per block and
// step; here it is one small launch each way (L = 169 coordinates, hidden 512, <= 32 heads).
#include "common.h"

namespace {

constexpr int kMaxHeads = 32;

// one workgroup per coordinate row l; thread t owns hidden units t, t + 256, ...
__global__ __launch_bounds__(256) void cpb_fwd_kernel(const float* __restrict__ c, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      float* __restrict__ out, int hidden, int heads) {
  __shared__ float part[4][kMaxHeads];
  const int l = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float c0 = c[2 * l], c1 = c[2 * l + 1];
  float acc[kMaxHeads];
#pragma unroll
  for (int h = 0; h < kMaxHeads; ++h) acc[h] = 0.f;
  for (int j = tid; j < hidden; j += blockDim.x) {
    const float hid = fmaxf(w1[2 * j] * c0 + w1[2 * j + 1] * c1 + b1[j], 0.f);
#pragma unroll
    for (int h = 0; h < kMaxHeads; ++h)
      if (h < heads) acc[h] += w2[(long)h * hidden + j] * hid;
  }
#pragma unroll
  for (int h = 0; h < kMaxHeads; ++h) {
    if (h < heads) {
      const float v = wave_sum(acc[h]);
      if (lane == 0) part[wave][h] = v;
    }
  }
  __syncthreads();
  if (tid < heads) {
    const float z = part[0][tid] + part[1][tid] + part[2][tid] + part[3][tid];
    out[(long)l * heads + tid] = 16.f / (1.f + __expf(-z));
  }
}

// workgroup b sums coordinate rows [b*kRows, b*kRows + kRows); thread t owns hidden units t, t + blockDim.x, ...;
// partial sums are added with fp32 atomics (43 workgroups per parameter element at L = 169: with 16 rows per
// workgroup the launch ran on 11 CUs)
constexpr int kRows = 4;
__global__ __launch_bounds__(512) void cpb_bwd_kernel(const float* __restrict__ c, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      const float* __restrict__ out, const float* __restrict__ dout,
                                                      float* __restrict__ dw1, float* __restrict__ db1,
                                                      float* __restrict__ dw2, int L, int hidden, int heads) {
  __shared__ float g[kRows * kMaxHeads];   // [rows][heads]: d(pre-sigmoid) = dout * 16 s (1 - s), s = out / 16
  const int l0 = blockIdx.x * kRows, nl = min(kRows, L - l0);
  for (int i = threadIdx.x; i < nl * heads; i += blockDim.x) {
    const float s = out[(long)l0 * heads + i] * (1.f / 16.f);
    g[i] = dout[(long)l0 * heads + i] * 16.f * s * (1.f - s);
  }
  __syncthreads();
  for (int j = threadIdx.x; j < hidden; j += blockDim.x) {
    const float wa = w1[2 * j], wb = w1[2 * j + 1], bj = b1[j];
    float w2j[kMaxHeads], dw2j[kMaxHeads];
#pragma unroll
    for (int h = 0; h < kMaxHeads; ++h) { w2j[h] = h < heads ? w2[(long)h * hidden + j] : 0.f; dw2j[h] = 0.f; }
    float da = 0.f, dbb = 0.f, dbias = 0.f;
    for (int l = 0; l < nl; ++l) {
      const float c0 = c[2 * (l0 + l)], c1 = c[2 * (l0 + l) + 1];
      const float pre = wa * c0 + wb * c1 + bj;
      if (pre <= 0.f) continue;   // ReLU: no gradient, no contribution to dW2
      float dh = 0.f;
#pragma unroll
      for (int h = 0; h < kMaxHeads; ++h) {
        if (h < heads) {
          const float gl = g[l * heads + h];
          dw2j[h] += gl * pre;
          dh += gl * w2j[h];
        }
      }
      da += dh * c0;
      dbb += dh * c1;
      dbias += dh;
    }
#pragma unroll
    for (int h = 0; h < kMaxHeads; ++h)
      if (h < heads) atomicAdd(dw2 + (long)h * hidden + j, dw2j[h]);
    atomicAdd(dw1 + 2 * j, da);
    atomicAdd(dw1 + 2 * j + 1, dbb);
    atomicAdd(db1 + j, dbias);
  }
}

}  // namespace

extern "C" int dfk_cpb_bias_fwd(const float* coords, const float* w1, const float* b1, const float* w2, float* out,
                                int32_t L, int32_t hidden, int32_t heads, hipStream_t s) {
  if (!coords || !w1 || !b1 || !w2 || !out || hidden <= 0 || heads <= 0 || heads > kMaxHeads) return DFK_EINVAL;
  if (L <= 0) return 0;
  hipLaunchKernelGGL(cpb_fwd_kernel, dim3(L), dim3(256), 0, s, coords, w1, b1, w2, out, (int)hidden, (int)heads);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_cpb_bias_bwd(const float* coords, const float* w1, const float* b1, const float* w2,
                                const float* out, const float* dout, float* dw1, float* db1, float* dw2, int32_t L,
                                int32_t hidden, int32_t heads, hipStream_t s) {
  if (!coords || !w1 || !b1 || !w2 || !out || !dout || !dw1 || !db1 || !dw2 || hidden <= 0 || heads <= 0 ||
      heads > kMaxHeads)
    return DFK_EINVAL;
  if (L <= 0) return 0;
  hipLaunchKernelGGL(cpb_bwd_kernel, dim3(dfk_cdiv(L, kRows)), dim3(512), 0, s, coords, w1, b1, w2, out, dout, dw1,
                     db1, dw2, (int)L, (int)hidden, (int)heads);
  DFK_CHECK_LAUNCH();
  return 0;
}
