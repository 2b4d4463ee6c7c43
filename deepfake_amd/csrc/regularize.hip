// Training-mode regularisers on the device: standalone dropout / DropPath passes (and the backward of
// every dropout fused into a GEMM or LayerNorm epilogue), LayerDrop coins and SpecAugment time masking.
// Every mask comes from the counter-based hash of common.h (drop_ctx / drop_mul), keyed by the device
// [seed, step] counter, so forward and backward agree and a replayed HIP graph draws fresh masks.
#include "common.h"

namespace {

// y = x * mask: 8 consecutive columns per thread (16-B vectors when the row layout allows)
template <typename T>
__global__ __launch_bounds__(256) void dropout_kernel(const T* __restrict__ x, T* __restrict__ y, long rows, int cols,
                                                      long ld, const dfk_drop d, int vec) {
  const int cg = (cols + 7) / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cg) return;
  const long row = idx / cg;
  const int c0 = (int)(idx % cg) * 8;
  const DropCtx dc = drop_ctx(d);
  const T* xp = x + row * ld + c0;
  T* yp = y + row * ld + c0;
  if (vec && c0 + 8 <= cols) {
    float v[8];
    ld8<T>(xp, v);
    const float g = dc.mode == 2 ? drop_mul(dc, row, 0) : 1.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] *= dc.mode == 2 ? g : drop_mul(dc, row, c0 + e);
    st8<T>(yp, v);
  } else {
    for (int e = 0; e < 8 && c0 + e < cols; ++e) stf<T>(yp + e, ldf<T>(xp + e) * drop_mul(dc, row, c0 + e));
  }
}

__global__ void bernoulli_kernel(const dfk_drop d, int n, float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DropCtx dc = drop_ctx(d);
  dc.mode = 1;
  out[i] = drop_mul(dc, i, 0) != 0.f ? 1.f : 0.f;
}

// LayerDrop coins of one micro-step (keep) folded into the accumulation window's "ever kept" flags (used):
// the SGD gate of a layer is the OR of its coins since the last zero_grad
__global__ void layerdrop_kernel(const dfk_drop d, int n, float* __restrict__ keep, float* __restrict__ used) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  DropCtx dc = drop_ctx(d);
  dc.mode = 1;
  const float k = drop_mul(dc, i, 0) != 0.f ? 1.f : 0.f;
  keep[i] = k;
  used[i] = fmaxf(used[i], k);
}

// uniform [0, 1) from a draw
__device__ __forceinline__ float unit_u(uint32_t h) { return (float)(h >> 8) * (1.f / 16777216.f); }

constexpr int kSpecSlices = 16;   // workgroups per clip in the SpecAugment forward

// HF _compute_mask_indices (modeling_wav2vec2.py:101-218) for one clip of T frames, no attention mask
template <typename T>
__global__ __launch_bounds__(256) void spec_aug_fwd_kernel(const T* __restrict__ h, T* __restrict__ out,
                                                           uint8_t* __restrict__ mask, const T* __restrict__ embed,
                                                           int Tn, int C, float mask_prob, int mlen, int min_masks,
                                                           const dfk_drop d, int vec) {
  extern __shared__ int sm[];
  int* cand = sm;              // [Tn] candidate span starts (partial Fisher-Yates)
  int* msk = sm + Tn;          // [Tn] masked flags
  const int b = blockIdx.x, tid = threadIdx.x;
  DropCtx dc = drop_ctx(d);
  dc.mode = 1;
  for (int t = tid; t < Tn; t += blockDim.x) { cand[t] = t; msk[t] = 0; }
  __syncthreads();
  if (tid == 0) {
    // one epsilon per call (the whole batch), as np.random.rand(1) in HF
    const float eps = unit_u(drop_hash(dc, 0x7fffffffL, 0));
    auto num_spans = [&](int len) {
      int n = (int)(mask_prob * len / mlen + eps);
      n = max(n, min_masks);
      if (n * mlen > Tn) n = Tn / mlen;
      if (len - (mlen - 1) < n) n = max(len - (mlen - 1), 0);
      return n;
    };
    const int n = num_spans(Tn);
    const int R = Tn - (mlen - 1);   // candidate starts [0, R)
    for (int i = 0; i < n; ++i) {    // n distinct starts, uniformly without replacement
      const uint32_t hsh = drop_hash(dc, b, i);
      const int j = i + (int)(hsh % (uint32_t)(R - i));
      const int tmp = cand[i]; cand[i] = cand[j]; cand[j] = tmp;
      for (int o = 0; o < mlen; ++o) msk[min(cand[i] + o, Tn - 1)] = 1;
    }
  }
  __syncthreads();
  // every workgroup of the clip redraws the (cheap) span starts and writes its slice of rows: the B-workgroup
  // element-wise copy took 213 us for 8 x 199 x 768
  if (blockIdx.y == 0)
    for (int t = tid; t < Tn; t += blockDim.x) mask[(long)b * Tn + t] = (uint8_t)msk[t];
  const int rows = (Tn + gridDim.y - 1) / gridDim.y, t0 = blockIdx.y * rows, t1 = min(Tn, t0 + rows);
  const long base = (long)b * Tn * C;
  constexpr int VEC = 16 / sizeof(T);
  if (vec) {   // 16-B vectors along the channels (host: C % VEC == 0, 16-B aligned h / out / embed)
    const int cv = C / VEC;
    for (int i = tid; i < (t1 - t0) * cv; i += blockDim.x) {
      const int t = t0 + i / cv, c = (i % cv) * VEC;
      const long o = base + (long)t * C + c;
      *reinterpret_cast<uint4*>(out + o) = msk[t] ? *reinterpret_cast<const uint4*>(embed + c)
                                                  : *reinterpret_cast<const uint4*>(h + o);
    }
  } else {
    for (int i = tid; i < (t1 - t0) * C; i += blockDim.x) {
      const int t = t0 + i / C, c = i % C;
      out[base + (long)t * C + c] = msk[t] ? embed[c] : h[base + (long)t * C + c];
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void spec_aug_bwd_kernel(const T* __restrict__ dy, T* __restrict__ dx,
                                                           const uint8_t* __restrict__ mask, float* __restrict__ dembed,
                                                           int Tn, int C) {
  const int b = blockIdx.x;
  const long base = (long)b * Tn * C;
  const uint8_t* mk = mask + (long)b * Tn;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float s = 0.f;
    for (int t = 0; t < Tn; ++t) {
      const long i = base + (long)t * C + c;
      const T g = dy[i];
      if (mk[t]) { s += ldf<T>(&g); stf<T>(dx + i, 0.f); }
      else dx[i] = g;
    }
    if (s != 0.f) atomicAdd(dembed + c, s);
  }
}

bool drop_args_ok(const dfk_drop* d) { return d && d->rng && d->p >= 0.f && d->p < 1.f; }

}  // namespace

extern "C" int dfk_dropout(const void* x, void* y, int64_t rows, int32_t cols, int64_t ld, const dfk_drop* d, int dtype,
                           hipStream_t s) {
  if (!x || !y || cols <= 0 || ld < cols || !drop_args_ok(d) || (d->mode != 1 && d->mode != 2)) return DFK_EINVAL;
  if (rows <= 0) return 0;
  const long threads = rows * ((cols + 7) / 8);
  const int es = dtype == DFK_BF16 ? 2 : 4;
  const int vec = ld % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                  (reinterpret_cast<uintptr_t>(y) & 15) == 0 && es > 0;
  const dim3 grid((unsigned)dfk_cdiv(threads, 256));
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(dropout_kernel<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)x, (bf16raw*)y, (long)rows,
                       (int)cols, (long)ld, *d, vec);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (float*)y, (long)rows, (int)cols,
                       (long)ld, *d, vec);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_bernoulli_flags(const dfk_drop* d, int32_t n, float* out, hipStream_t s) {
  if (!out || !drop_args_ok(d)) return DFK_EINVAL;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(bernoulli_kernel, dim3(dfk_cdiv(n, 256)), dim3(256), 0, s, *d, (int)n, out);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_layerdrop_flags(const dfk_drop* d, int32_t n, float* keep, float* used, hipStream_t s) {
  if (!keep || !used || !drop_args_ok(d)) return DFK_EINVAL;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(layerdrop_kernel, dim3(dfk_cdiv(n, 256)), dim3(256), 0, s, *d, (int)n, keep, used);
  DFK_CHECK_LAUNCH();
  return 0;
}

// LayerDrop output select (forward): out = keep > 0 ? y : x, and its backward in the same form: gy = keep > 0 ? g : 0,
// gx = keep > 0 ? 0 : g (x's other gradient is added by the caller); 16-B vectors, one launch each way
__global__ __launch_bounds__(256) void layer_select_kernel(const uint4* __restrict__ y, const uint4* __restrict__ x,
                                                           const float* __restrict__ keep, uint4* __restrict__ out,
                                                           uint4* __restrict__ out2, long nv) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= nv) return;
  const bool k = *keep > 0.f;
  const uint4 z = make_uint4(0, 0, 0, 0);
  if (out2) {   // backward: y = g
    const uint4 g = y[i];
    out[i] = k ? g : z;
    out2[i] = k ? z : g;
  } else {
    out[i] = k ? y[i] : x[i];
  }
}

extern "C" int dfk_layer_select(const void* y, const void* x, const float* keep, void* out, void* out2,
                                int64_t nbytes, hipStream_t s) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (!y || !keep || !out || (!out2 && !x) || nbytes % 16 || !al(y) || !al(out) || (x && !al(x)) || (out2 && !al(out2)))
    return DFK_EINVAL;
  const long nv = nbytes / 16;
  if (nv <= 0) return 0;
  hipLaunchKernelGGL(layer_select_kernel, dim3((unsigned)dfk_cdiv(nv, 256)), dim3(256), 0, s, (const uint4*)y,
                     (const uint4*)x, keep, (uint4*)out, (uint4*)out2, nv);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_spec_augment_fwd(const void* h, void* out, uint8_t* mask, const void* embed, int32_t B, int32_t T,
                                    int32_t C, float mask_prob, int32_t mask_length, int32_t min_masks,
                                    const dfk_drop* d, int dtype, hipStream_t s) {
  if (!h || !out || !mask || !embed || !d || !d->rng || mask_length <= 0 || C <= 0 || T > 16384) return DFK_EINVAL;
  if (B <= 0 || T <= 0) return 0;
  const size_t lds = 8 * (size_t)T;
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  const int vec = C % (dtype == DFK_BF16 ? 8 : 4) == 0 && al(h) && al(out) && al(embed);
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(spec_aug_fwd_kernel<bf16raw>, dim3(B, kSpecSlices), dim3(256), lds, s, (const bf16raw*)h, (bf16raw*)out, mask,
                       (const bf16raw*)embed, (int)T, (int)C, mask_prob, (int)mask_length, (int)min_masks, *d, vec);
  else
    hipLaunchKernelGGL(spec_aug_fwd_kernel<float>, dim3(B, kSpecSlices), dim3(256), lds, s, (const float*)h, (float*)out, mask,
                       (const float*)embed, (int)T, (int)C, mask_prob, (int)mask_length, (int)min_masks, *d, vec);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_spec_augment_bwd(const void* dy, void* dx, const uint8_t* mask, float* dembed, int32_t B, int32_t T,
                                    int32_t C, int dtype, hipStream_t s) {
  if (!dy || !dx || !mask || !dembed || C <= 0) return DFK_EINVAL;
  if (B <= 0 || T <= 0) return 0;
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(spec_aug_bwd_kernel<bf16raw>, dim3(B), dim3(256), 0, s, (const bf16raw*)dy, (bf16raw*)dx, mask,
                       dembed, (int)T, (int)C);
  else
    hipLaunchKernelGGL(spec_aug_bwd_kernel<float>, dim3(B), dim3(256), 0, s, (const float*)dy, (float*)dx, mask, dembed,
                       (int)T, (int)C);
  DFK_CHECK_LAUNCH();
  return 0;
}
