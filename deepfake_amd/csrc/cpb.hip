// SwinV2 continuous position bias (swin_transformer2d.py:99-100,159-162): the cpb_mlp over the
// relative_coords_table and 16*sigmoid, forward and backward, in fp32 straight from the parameters.
// The reference runs this as Linear -> ReLU -> Linear -> sigmoid -> mul (and their backward) per block and
// step; here it is one small launch each way (L = 169 coordinates, hidden 512, <= 32 heads).
#include "common.h"

namespace {

constexpr int kMaxHeads = 32;

// one workgroup per coordinate row l; thread t owns hidden units t, t + 256, ...
__device__ __forceinline__ void cpb_fwd_row(const float* __restrict__ c, const float* __restrict__ w1,
                                            const float* __restrict__ b1, const float* __restrict__ w2,
                                            float* __restrict__ out, int hidden, int heads, int l) {
  __shared__ float part[4][kMaxHeads];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
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

__global__ __launch_bounds__(256) void cpb_fwd_kernel(const float* __restrict__ c, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      float* __restrict__ out, int hidden, int heads) {
  cpb_fwd_row(c, w1, b1, w2, out, hidden, heads, blockIdx.x);
}

// every SwinV2 block's table in one launch: blockIdx.y = block (descriptor), blockIdx.x = coordinate row
struct CpbDesc {
  int64_t c, w1, b1, w2, dw1, db1, dw2, off, L, hidden, heads, pad;
};

__global__ __launch_bounds__(256) void cpb_fwd_many_kernel(const CpbDesc* __restrict__ desc, float* __restrict__ out) {
  const CpbDesc d = desc[blockIdx.y];
  if ((int)blockIdx.x >= (int)d.L) return;
  cpb_fwd_row(reinterpret_cast<const float*>(d.c), reinterpret_cast<const float*>(d.w1),
              reinterpret_cast<const float*>(d.b1), reinterpret_cast<const float*>(d.w2), out + d.off, (int)d.hidden,
              (int)d.heads, blockIdx.x);
}

// workgroup b sums coordinate rows [b*kRows, b*kRows + kRows); thread t owns hidden units t, t + blockDim.x, ...;
// partial sums are added with fp32 atomics (43 workgroups per parameter element at L = 169: with 16 rows per
// workgroup the launch ran on 11 CUs)
constexpr int kRows = 4;
__device__ __forceinline__ void cpb_bwd_rows(const float* __restrict__ c, const float* __restrict__ w1,
                                             const float* __restrict__ b1, const float* __restrict__ w2,
                                             const float* __restrict__ out, const float* __restrict__ dout,
                                             float* __restrict__ dw1, float* __restrict__ db1,
                                             float* __restrict__ dw2, int L, int hidden, int heads, int blk) {
  __shared__ float g[kRows * kMaxHeads];   // [rows][heads]: d(pre-sigmoid) = dout * 16 s (1 - s), s = out / 16
  const int l0 = blk * kRows, nl = min(kRows, L - l0);
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

__global__ __launch_bounds__(512) void cpb_bwd_kernel(const float* __restrict__ c, const float* __restrict__ w1,
                                                      const float* __restrict__ b1, const float* __restrict__ w2,
                                                      const float* __restrict__ out, const float* __restrict__ dout,
                                                      float* __restrict__ dw1, float* __restrict__ db1,
                                                      float* __restrict__ dw2, int L, int hidden, int heads) {
  cpb_bwd_rows(c, w1, b1, w2, out, dout, dw1, db1, dw2, L, hidden, heads, blockIdx.x);
}

__global__ __launch_bounds__(512) void cpb_bwd_many_kernel(const CpbDesc* __restrict__ desc,
                                                           const float* __restrict__ out,
                                                           const float* __restrict__ dout) {
  const CpbDesc d = desc[blockIdx.y];
  if ((int)blockIdx.x * kRows >= (int)d.L) return;
  cpb_bwd_rows(reinterpret_cast<const float*>(d.c), reinterpret_cast<const float*>(d.w1),
               reinterpret_cast<const float*>(d.b1), reinterpret_cast<const float*>(d.w2), out + d.off,
               dout + d.off, reinterpret_cast<float*>(d.dw1), reinterpret_cast<float*>(d.db1),
               reinterpret_cast<float*>(d.dw2), (int)d.L, (int)d.hidden, (int)d.heads, blockIdx.x);
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

// Batched forms: n tables (every SwinV2 block of a model) in one launch each way.  desc: DEVICE array of n
// records of 12 int64 {coords, w1, b1, w2, dw1, db1, dw2 (device pointers), off (float offset of the block's
// [L, heads] table in out / dout), L, hidden, heads (<= 32), 0}; max_L >= every record's L.
extern "C" int dfk_cpb_bias_fwd_many(const int64_t* desc, int32_t n, int32_t max_L, float* out, hipStream_t s) {
  if (!desc || !out || n < 0 || max_L < 0) return DFK_EINVAL;
  if (n == 0 || max_L == 0) return 0;
  hipLaunchKernelGGL(cpb_fwd_many_kernel, dim3(max_L, n), dim3(256), 0, s, reinterpret_cast<const CpbDesc*>(desc),
                     out);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_cpb_bias_bwd_many(const int64_t* desc, int32_t n, int32_t max_L, const float* out,
                                     const float* dout, hipStream_t s) {
  if (!desc || !out || !dout || n < 0 || max_L < 0) return DFK_EINVAL;
  if (n == 0 || max_L == 0) return 0;
  hipLaunchKernelGGL(cpb_bwd_many_kernel, dim3(dfk_cdiv(max_L, kRows), n), dim3(512), 0, s,
                     reinterpret_cast<const CpbDesc*>(desc), out, dout);
  DFK_CHECK_LAUNCH();
  return 0;
}
