// Data-movement kernels around the GEMMs: patch im2col (Conv3d/Conv2d with
// kernel == stride), PatchMerging 2x2 gather / scatter, per-clip row means,
// dtype casts and the fused SGD step.  All HBM-bound, 16-B vectorised where
// the layout allows.
#include "common.h"

namespace {

// out[row][k], row = ((b*Do+d)*Ho+h)*Wo+w, k = ((c*pd+kd)*ph+kh)*pw+kw ; zero beyond the input (pad)
template <typename TI, typename TO>
__global__ void im2col_kernel(const TI* __restrict__ x, TO* __restrict__ out, dfk_im2col_args a, long total) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total) return;
  const int K = a.cin * a.pd * a.ph * a.pw;
  const long row = idx / K;
  const int k = (int)(idx - row * K);
  const int kw = k % a.pw, kh = (k / a.pw) % a.ph, kd = (k / (a.pw * a.ph)) % a.pd, c = k / (a.pw * a.ph * a.pd);
  const int w = (int)(row % a.Wo), h = (int)((row / a.Wo) % a.Ho), d = (int)((row / ((long)a.Wo * a.Ho)) % a.Do);
  const long b = row / ((long)a.Wo * a.Ho * a.Do);
  const int t = d * a.pd + kd, y = h * a.ph + kh, xx = w * a.pw + kw;
  float v = 0.f;
  if (t < a.T && y < a.H && xx < a.W) v = ldf<TI>(x + b * a.sb + c * a.sc + t * a.st + (long)y * a.sh + (long)xx * a.sw);
  stf<TO>(out + idx, v);
}

// Row-staged im2col for fp32 input with unit W stride and 16-B aligned rows (the clip / mel-image
// PatchEmbed inputs): one workgroup per output row of tokens (b, d, h).  The cin*pd*ph input rows those
// tokens cover are staged into LDS with coalesced 16-B loads (zero beyond T / H / W), then every lane
// writes 16-B chunks of the token-major [Wo][K] output, so both HBM streams move whole lines.
template <typename TO>
__global__ __launch_bounds__(256) void im2col_rows_kernel(const float* __restrict__ x, TO* __restrict__ out,
                                                          dfk_im2col_args a) {
  extern __shared__ __attribute__((aligned(16))) float slab[];   // [cin*pd*ph][Ws]
  const int Wp = a.Wo * a.pw, Ws = Wp + 4;   // +4 floats: a token's rows spread over the banks
  long r = blockIdx.x;
  const int h = (int)(r % a.Ho);
  r /= a.Ho;
  const int d = (int)(r % a.Do);
  const long b = r / a.Do;
  const int nrows = a.cin * a.pd * a.ph, q4 = Wp / 4;
  for (int i = threadIdx.x; i < nrows * q4; i += blockDim.x) {
    const int sr = i / q4, x0 = (i - sr * q4) * 4;
    const int c = sr / (a.pd * a.ph), kd = (sr / a.ph) % a.pd, kh = sr % a.ph;
    const int t = d * a.pd + kd, y = h * a.ph + kh;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t < a.T && y < a.H) {
      const float* p = x + b * a.sb + c * a.sc + (long)t * a.st + (long)y * a.sh + x0;
      if (x0 + 4 <= a.W) {
        v = *reinterpret_cast<const float4*>(p);
      } else {
        float e[4] = {0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < 4; ++j)
          if (x0 + j < a.W) e[j] = p[j];
        v = make_float4(e[0], e[1], e[2], e[3]);
      }
    }
    *reinterpret_cast<float4*>(slab + sr * Ws + x0) = v;
  }
  __syncthreads();
  const int K = nrows * a.pw, kc = K / 8;
  TO* o = out + (long)blockIdx.x * a.Wo * K;
  for (int j = threadIdx.x; j < a.Wo * kc; j += blockDim.x) {
    const int w = j / kc, k0 = (j - w * kc) * 8;
    float v[8];
    if (a.pw == 4) {   // the chunk is 4 columns of two consecutive staged rows: two 16-B LDS reads
      const int sr = k0 / 4;
      const float4 lo = *reinterpret_cast<const float4*>(slab + sr * Ws + w * 4);
      const float4 hi = *reinterpret_cast<const float4*>(slab + (sr + 1) * Ws + w * 4);
      v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w; v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e, sr = k / a.pw;
        v[e] = slab[sr * Ws + w * a.pw + (k - sr * a.pw)];
      }
    }
    st8<TO>(o + (long)w * K + k0, v);
  }
}

// PatchMerging (video_swin_transformer.py:300-311 / swin_transformer2d.py:349-358):
// out[(b,d,h2,w2)][q*C + c] = x[b,d,2h2+i,2w2+j,c], (i,j) = (0,0),(1,0),(0,1),(1,1) for q = 0..3
template <typename T>
__global__ void merge_kernel(const T* __restrict__ src, T* __restrict__ dst, int B, int D, int H, int W, int C,
                             int reverse, long total_vec) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= total_vec) return;
  constexpr int VEC = 16 / sizeof(T);
  const int H2 = (H + 1) / 2, W2 = (W + 1) / 2;
  const int cv = C / VEC;
  const int c = (int)(idx % cv) * VEC;
  long r = idx / cv;
  const int q = (int)(r % 4);
  r /= 4;  // merged row
  const int w2 = (int)(r % W2), h2 = (int)((r / W2) % H2);
  const long bd = r / ((long)W2 * H2);
  const int i = q & 1, j = q >> 1;
  const int h = 2 * h2 + i, w = 2 * w2 + j;
  const bool ok = h < H && w < W;
  const long xoff = ((bd * H + h) * W + w) * C + c;
  const long moff = r * 4L * C + (long)q * C + c;
  if (!reverse) {
    *reinterpret_cast<uint4*>(dst + moff) = ok ? *reinterpret_cast<const uint4*>(src + xoff) : make_uint4(0, 0, 0, 0);
  } else if (ok) {
    *reinterpret_cast<uint4*>(dst + xoff) = *reinterpret_cast<const uint4*>(src + moff);
  }
}

// out[g][c] = mean_r x[g*R + r][c]   (fp32 accumulation)
template <typename T, typename TO>
__global__ __launch_bounds__(256) void rowmean_kernel(const T* __restrict__ x, TO* __restrict__ out, int R, int C) {
  // workgroup = (64 columns, group): 4 row phases x 64 coalesced columns, 8 independent partial sums per lane
  // (a thread walking all R rows serially was a chain of R dependent-latency loads: 116 us at R = 784)
  __shared__ float red[4][64];
  const int g = blockIdx.y, lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  const bool ok = c < C;
  const T* p = x + (long)g * R * C + (ok ? c : 0);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int r = ph;
  for (; r + 28 < R; r += 32)
#pragma unroll
    for (int u = 0; u < 8; ++u) s[u] += ldf<T>(p + (long)(r + 4 * u) * C);
  for (; r < R; r += 4) s[0] += ldf<T>(p + (long)r * C);
  red[ph][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (ph == 0 && ok)
    stf<TO>(out + (long)g * C + c, ((red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane])) / R);
}

template <typename T>
__global__ void gelu_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ pre, T* __restrict__ dx, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stf<T>(dx + i, ldf<T>(dy + i) * (sizeof(T) == 2 ? dgelu_bf(ldf<T>(pre + i)) : dgelu_f(ldf<T>(pre + i))));
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* __restrict__ y, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) stf<TO>(y + i, ldf<TI>(x + i));
}

// torch.optim.SGD semantics (momentum, dampening 0, weight decay, no nesterov):
//   g = grad + wd*p ; buf = first ? g : mom*buf + g ; p -= lr*buf ; shadow = bf16(p)
// NT: the parameter / momentum / shadow stores are non-temporal (streamed to HBM, not left dirty in L2 / MALL),
// so that their write-back does not land on the first kernels of the next step (the clip-batch patch embedding)
// Data-parallel fold (gscale, gbf): the gradient read is the all-reduced SUM — the fp32 buffer itself, or the
// bf16 bucket copy RCCL summed (gbf != NULL) — times gscale = 1 / world, so no separate averaging / cast-back
// pass over the flat gradient runs between the last all-reduce and the step (ddp.py GradBucketer.finish(fold)).
template <bool NT>
__global__ void sgd_kernel(float* __restrict__ p, const float* __restrict__ grad, float* __restrict__ buf,
                           bf16raw* __restrict__ shadow, long n, const float* __restrict__ lr_dev, float lr_host,
                           float mom, float wd, int first, const float* __restrict__ gate, float gscale,
                           const bf16raw* __restrict__ gbf) {
  const long i0 = ((long)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i0 >= n) return;
  if (gate && *gate == 0.f) return;   // LayerDrop-skipped layer: torch's SGD skips grad=None parameters
  const float lr = lr_dev ? *lr_dev : lr_host;
  if (i0 + 4 <= n) {
    float4 pv = *reinterpret_cast<float4*>(p + i0);
    float4 gv;
    if (gbf) {
      const uint2 u = *reinterpret_cast<const uint2*>(gbf + i0);
      gv = make_float4(__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u), __uint_as_float(u.y << 16),
                       __uint_as_float(u.y & 0xffff0000u));
    } else {
      gv = *reinterpret_cast<const float4*>(grad + i0);
    }
    float4 bv = first ? make_float4(0, 0, 0, 0) : *reinterpret_cast<float4*>(buf + i0);
    float* pp = reinterpret_cast<float*>(&pv);
    const float* gg = reinterpret_cast<const float*>(&gv);
    float* bb = reinterpret_cast<float*>(&bv);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float g = gg[k] * gscale + wd * pp[k];
      bb[k] = first ? g : mom * bb[k] + g;
      pp[k] -= lr * bb[k];
    }
    if constexpr (NT) {
      __builtin_nontemporal_store(__builtin_bit_cast(f32x4, pv), reinterpret_cast<f32x4*>(p + i0));
      __builtin_nontemporal_store(__builtin_bit_cast(f32x4, bv), reinterpret_cast<f32x4*>(buf + i0));
    } else {
      *reinterpret_cast<float4*>(p + i0) = pv;
      *reinterpret_cast<float4*>(buf + i0) = bv;
    }
    if (shadow) {
      uint2 u;
      bf16raw* e = reinterpret_cast<bf16raw*>(&u);
#pragma unroll
      for (int k = 0; k < 4; ++k) e[k] = f2bf(pp[k]);
      typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
      if constexpr (NT) __builtin_nontemporal_store(__builtin_bit_cast(u32x2, u), reinterpret_cast<u32x2*>(shadow + i0));
      else *reinterpret_cast<uint2*>(shadow + i0) = u;
    }
  } else {
    for (long i = i0; i < n; ++i) {
      const float g = (gbf ? bf2f(gbf[i]) : grad[i]) * gscale + wd * p[i];
      buf[i] = first ? g : mom * buf[i] + g;
      p[i] -= lr * buf[i];
      if (shadow) shadow[i] = f2bf(p[i]);
    }
  }
}

// All runs of one step in one launch (dfk_sgd_step_runs): the run table travels by value in the kernel
// arguments (no device table to keep alive across graph replays); a workgroup owns kSgdRunBlock consecutive
// elements of one run (two float4 per thread, so each wave keeps 2x the bytes of the one-run kernel in flight).
constexpr int kSgdRunBlock = 2048;
constexpr int kSgdMaxRuns = 64;
struct SgdRuns {
  int64_t start[kSgdMaxRuns], n[kSgdMaxRuns];
  const float* gate[kSgdMaxRuns];
  int32_t prefix[kSgdMaxRuns + 1];    // first workgroup of each run; prefix[nruns] = the grid
  uint64_t first;                     // bit r: run r takes its first momentum step
  int32_t nruns;
};

__global__ __launch_bounds__(256) void sgd_runs_kernel(float* __restrict__ P, const float* __restrict__ G,
                                                       float* __restrict__ Bf, bf16raw* __restrict__ S,
                                                       const SgdRuns R, const float* __restrict__ lr_dev,
                                                       float lr_host, float mom, float wd, float gscale,
                                                       const bf16raw* __restrict__ GB) {
  const int b = blockIdx.x;
  int lo = 0, hi = R.nruns - 1;                   // the run with prefix[lo] <= b < prefix[lo + 1]
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (R.prefix[mid] <= b) lo = mid; else hi = mid - 1;
  }
  const long start = R.start[lo], n = R.n[lo];
  const float* gate = R.gate[lo];
  const int first = (int)((R.first >> lo) & 1);
  if (gate && *gate == 0.f) return;
  const float lr = lr_dev ? *lr_dev : lr_host;
  const long base = (long)(b - R.prefix[lo]) * kSgdRunBlock;
  float* p = P + start;
  float* buf = Bf + start;
  const float* grad = G + start;
  const bf16raw* gbf = GB ? GB + start : nullptr;
  bf16raw* shadow = S ? S + start : nullptr;
  long idx[2] = {base + threadIdx.x * 4, base + 1024 + threadIdx.x * 4};
  float4 pv[2], gv[2], bv[2];
  bool full[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    full[u] = idx[u] + 4 <= n;
    if (!full[u]) continue;
    pv[u] = *reinterpret_cast<const float4*>(p + idx[u]);
    if (gbf) {
      const uint2 w = *reinterpret_cast<const uint2*>(gbf + idx[u]);
      gv[u] = make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u),
                          __uint_as_float(w.y << 16), __uint_as_float(w.y & 0xffff0000u));
    } else {
      gv[u] = *reinterpret_cast<const float4*>(grad + idx[u]);
    }
    bv[u] = first ? make_float4(0, 0, 0, 0) : *reinterpret_cast<const float4*>(buf + idx[u]);
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    if (full[u]) {
      float* pp = reinterpret_cast<float*>(&pv[u]);
      const float* gg = reinterpret_cast<const float*>(&gv[u]);
      float* bb = reinterpret_cast<float*>(&bv[u]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float g = gg[k] * gscale + wd * pp[k];
        bb[k] = first ? g : mom * bb[k] + g;
        pp[k] -= lr * bb[k];
      }
      *reinterpret_cast<float4*>(p + idx[u]) = pv[u];
      *reinterpret_cast<float4*>(buf + idx[u]) = bv[u];
      if (shadow) {
        uint2 w;
        bf16raw* e = reinterpret_cast<bf16raw*>(&w);
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = f2bf(pp[k]);
        *reinterpret_cast<uint2*>(shadow + idx[u]) = w;
      }
    } else {
      for (long i = idx[u]; i < n; ++i) {        // the run's last < 4 elements
        const float g = (gbf ? bf2f(gbf[i]) : grad[i]) * gscale + wd * p[i];
        buf[i] = first ? g : mom * buf[i] + g;
        p[i] -= lr * buf[i];
        if (shadow) shadow[i] = f2bf(p[i]);
      }
    }
  }
}

// SwinV2 cosine attention prologue (swin_transformer2d.py:154-157): per (row, head)
//   q' = q / max(|q|, 1e-12) * scale[h] ;  k' = k / max(|k|, 1e-12) ;  v' = v
// G = hd/8 consecutive lanes per (row, head), 8 elements (16 B) of q, k and v each; the norms reduce
// across the lane group by xor shuffles.
template <int G>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = 1; o < G; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int G>
__global__ __launch_bounds__(256) void cosine_fwd_kernel(const T* __restrict__ qkv, T* __restrict__ out,
                                                         const float* __restrict__ logit, float max_log, long rows,
                                                         int heads) {
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long grp = idx / G;
  const int l = (int)(idx % G);
  const bool ok = grp < rows * heads;
  const long r = ok ? grp / heads : 0;
  const int h = (int)(grp % heads);
  const int C = heads * G * 8;
  const long off = r * 3 * C + h * G * 8 + l * 8;
  float q[8], k[8], v[8];
  ld8<T>(qkv + off, q);
  ld8<T>(qkv + off + C, k);
  ld8<T>(qkv + off + 2 * C, v);
  float nq = 0.f, nk = 0.f;
#pragma unroll
  for (int e = 0; e < 8; ++e) { nq += q[e] * q[e]; nk += k[e] * k[e]; }
  nq = group_sum<G>(nq);
  nk = group_sum<G>(nk);
  const float iq = __expf(fminf(logit[h], max_log)) / fmaxf(sqrtf(nq), 1e-12f), ik = 1.f / fmaxf(sqrtf(nk), 1e-12f);
#pragma unroll
  for (int e = 0; e < 8; ++e) { q[e] *= iq; k[e] *= ik; }
  if (ok) {
    st8<T>(out + off, q);
    st8<T>(out + off + C, k);
    st8<T>(out + off + 2 * C, v);
  }
}

// backward: dq = (s*dq' - qh*(qh . s*dq'))/|q| ; dk likewise (s = 1) ; dv = dv' ;
// dlogit[h] += (qh . dq') * s * [logit <= max_log]   (s = exp(clamp(logit, max=max_log)))
template <typename T, int G>
__global__ __launch_bounds__(256) void cosine_bwd_kernel(const T* __restrict__ qkv, const T* __restrict__ dout,
                                                         T* __restrict__ dqkv, const float* __restrict__ logit,
                                                         float max_log, float* __restrict__ dlogit, long rows,
                                                         int heads, float* __restrict__ dscore) {
  __shared__ float red[64];
  if (threadIdx.x < 64) red[threadIdx.x] = 0.f;
  __syncthreads();
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long grp = idx / G;
  const int l = (int)(idx % G);
  const bool ok = grp < rows * heads;
  const long r = ok ? grp / heads : 0;
  const int h = (int)(grp % heads);
  const int C = heads * G * 8;
  const long base = r * 3 * C + h * G * 8 + l * 8;
  float dsq = 0.f;
#pragma unroll
  for (int part = 0; part < 2; ++part) {
    float x[8], d[8];
    ld8<T>(qkv + base + part * C, x);
    ld8<T>(dout + base + part * C, d);
    float n2 = 0.f, xd = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) { n2 += x[e] * x[e]; xd += x[e] * d[e]; }
    n2 = group_sum<G>(n2);
    xd = group_sum<G>(xd);
    const float n = sqrtf(n2), inv = 1.f / fmaxf(n, 1e-12f);
    const float sc = part == 0 ? __expf(fminf(logit[h], max_log)) : 1.f;
    const float dot = xd * inv;   // xhat . dq'
    if (part == 0) dsq = dot;
    const bool clamped = n <= 1e-12f;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float g = sc * d[e];
      o[e] = clamped ? g * inv : (g - x[e] * inv * sc * dot) * inv;
    }
    if (ok) st8<T>(dqkv + base + part * C, o);
  }
  if (ok) {
    float dv[8];
    ld8<T>(dout + base + 2 * C, dv);
    st8<T>(dqkv + base + 2 * C, dv);
    if (l == 0 && !dscore) atomicAdd(&red[h & 63], dsq);
  }
  if (dscore) {   // the attention backward took sum dS * score in fp32 (dfk_wattn_bwd_args.dscore): use it, re-zero it
    if (blockIdx.x == 0 && threadIdx.x < heads) {
      const float v = dscore[threadIdx.x];
      dscore[threadIdx.x] = 0.f;
      if (logit[threadIdx.x] <= max_log) atomicAdd(dlogit + threadIdx.x, v);
    }
    return;
  }
  __syncthreads();
  if (threadIdx.x < heads && threadIdx.x < 64 && red[threadIdx.x] != 0.f) {
    const float lg = logit[threadIdx.x];
    if (lg <= max_log) atomicAdd(dlogit + threadIdx.x, red[threadIdx.x] * __expf(lg));
  }
}

}  // namespace

extern "C" int dfk_cosine_qk_fwd(const void* qkv, void* out, const float* logit_scale, float max_log, int64_t rows,
                                 int heads, int hd, int dtype, hipStream_t s) {
  if (!qkv || !out || !logit_scale || heads <= 0 || heads > 64 || (hd != 32 && hd != 64)) return DFK_EINVAL;
  if (reinterpret_cast<uintptr_t>(qkv) % 16 || reinterpret_cast<uintptr_t>(out) % 16) return DFK_EINVAL;
  const long n = rows * heads * (hd / 8);
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 255) / 256));
#define COS_F(T, G) hipLaunchKernelGGL((cosine_fwd_kernel<T, G>), grid, dim3(256), 0, s, (const T*)qkv, (T*)out, \
                                       logit_scale, max_log, (long)rows, heads)
  if (dtype == DFK_BF16) { if (hd == 32) COS_F(bf16raw, 4); else COS_F(bf16raw, 8); }
  else { if (hd == 32) COS_F(float, 4); else COS_F(float, 8); }
#undef COS_F
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_cosine_qk_bwd(const void* qkv, const void* dout, void* dqkv, const float* logit_scale, float max_log,
                                 float* dlogit_scale, int64_t rows, int heads, int hd, int dtype, float* dscore,
                                 hipStream_t s) {
  if (!qkv || !dout || !dqkv || !logit_scale || !dlogit_scale || heads <= 0 || heads > 64 || (hd != 32 && hd != 64))
    return DFK_EINVAL;
  if (reinterpret_cast<uintptr_t>(qkv) % 16 || reinterpret_cast<uintptr_t>(dout) % 16 ||
      reinterpret_cast<uintptr_t>(dqkv) % 16)
    return DFK_EINVAL;
  const long n = rows * heads * (hd / 8);
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 255) / 256));
#define COS_B(T, G) hipLaunchKernelGGL((cosine_bwd_kernel<T, G>), grid, dim3(256), 0, s, (const T*)qkv, (const T*)dout, \
                                       (T*)dqkv, logit_scale, max_log, dlogit_scale, (long)rows, heads, dscore)
  if (dtype == DFK_BF16) { if (hd == 32) COS_B(bf16raw, 4); else COS_B(bf16raw, 8); }
  else { if (hd == 32) COS_B(float, 4); else COS_B(float, 8); }
#undef COS_B
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_patch_im2col(const void* x, int x_dtype, void* out, int out_dtype, const dfk_im2col_args* a,
                                hipStream_t s) {
  if (!x || !out || !a || a->pd <= 0 || a->ph <= 0 || a->pw <= 0) return DFK_EINVAL;
  const long rows = (long)a->B * a->Do * a->Ho * a->Wo;
  const long total = rows * a->cin * a->pd * a->ph * a->pw;
  if (total <= 0) return 0;
  {
    const int K = a->cin * a->pd * a->ph * a->pw, Wp = a->Wo * a->pw;
    const size_t slab = (size_t)a->cin * a->pd * a->ph * (Wp + 4) * sizeof(float);
    const bool rows_ok = x_dtype == DFK_F32 && a->sw == 1 && a->sb % 4 == 0 && a->sc % 4 == 0 && a->st % 4 == 0 &&
                         a->sh % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 &&
                         (reinterpret_cast<uintptr_t>(out) & 15) == 0 && Wp % 4 == 0 && K % 8 == 0 &&
                         slab <= 64 * 1024 && (out_dtype == DFK_BF16 || out_dtype == DFK_F32);
    if (rows_ok) {
      const dim3 g((unsigned)((long)a->B * a->Do * a->Ho));
      if (out_dtype == DFK_BF16)
        hipLaunchKernelGGL(im2col_rows_kernel<bf16raw>, g, dim3(256), slab, s, (const float*)x, (bf16raw*)out, *a);
      else
        hipLaunchKernelGGL(im2col_rows_kernel<float>, g, dim3(256), slab, s, (const float*)x, (float*)out, *a);
      DFK_CHECK_LAUNCH();
      return 0;
    }
  }
  const dim3 grid((unsigned)((total + 255) / 256));
  if (x_dtype == DFK_F32 && out_dtype == DFK_BF16)
    hipLaunchKernelGGL((im2col_kernel<float, bf16raw>), grid, dim3(256), 0, s, (const float*)x, (bf16raw*)out, *a, total);
  else if (x_dtype == DFK_F32 && out_dtype == DFK_F32)
    hipLaunchKernelGGL((im2col_kernel<float, float>), grid, dim3(256), 0, s, (const float*)x, (float*)out, *a, total);
  else if (x_dtype == DFK_BF16 && out_dtype == DFK_BF16)
    hipLaunchKernelGGL((im2col_kernel<bf16raw, bf16raw>), grid, dim3(256), 0, s, (const bf16raw*)x, (bf16raw*)out, *a,
                       total);
  else
    return DFK_EINVAL;
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_patch_merge(const void* src, void* dst, int B, int D, int H, int W, int C, int reverse, int dtype,
                               hipStream_t s) {
  const int vec = dtype == DFK_BF16 ? 8 : 4;
  if (!src || !dst || C % vec) return DFK_EINVAL;
  const long rows = (long)B * D * ((H + 1) / 2) * ((W + 1) / 2);
  const long total = rows * 4 * (C / vec);
  if (total <= 0) return 0;
  const dim3 grid((unsigned)((total + 255) / 256));
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(merge_kernel<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)src, (bf16raw*)dst, B, D, H, W, C,
                       reverse, total);
  else
    hipLaunchKernelGGL(merge_kernel<float>, grid, dim3(256), 0, s, (const float*)src, (float*)dst, B, D, H, W, C,
                       reverse, total);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_rowmean(const void* x, void* out, int groups, int R, int C, int dtype, int out_f32, hipStream_t s) {
  if (!x || !out || R <= 0) return DFK_EINVAL;
  const dim3 grid(dfk_cdiv(C, 64), groups);
  if (dtype == DFK_BF16) {
    if (out_f32) hipLaunchKernelGGL((rowmean_kernel<bf16raw, float>), grid, dim3(256), 0, s, (const bf16raw*)x, (float*)out, R, C);
    else hipLaunchKernelGGL((rowmean_kernel<bf16raw, bf16raw>), grid, dim3(256), 0, s, (const bf16raw*)x, (bf16raw*)out, R, C);
  } else {
    hipLaunchKernelGGL((rowmean_kernel<float, float>), grid, dim3(256), 0, s, (const float*)x, (float*)out, R, C);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_gelu_bwd(const void* dy, const void* pre, void* dx, int64_t n, int dtype, hipStream_t s) {
  if (!dy || !pre || !dx) return DFK_EINVAL;
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(gelu_bwd_kernel<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)dy, (const bf16raw*)pre,
                       (bf16raw*)dx, (long)n);
  else
    hipLaunchKernelGGL(gelu_bwd_kernel<float>, grid, dim3(256), 0, s, (const float*)dy, (const float*)pre, (float*)dx,
                       (long)n);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_cast(const void* x, int x_dtype, void* y, int y_dtype, int64_t n, hipStream_t s) {
  if (!x || !y) return DFK_EINVAL;
  if (n <= 0) return 0;
  const dim3 grid((unsigned)((n + 255) / 256));
  if (x_dtype == DFK_F32 && y_dtype == DFK_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16raw>), grid, dim3(256), 0, s, (const float*)x, (bf16raw*)y, (long)n);
  else if (x_dtype == DFK_BF16 && y_dtype == DFK_F32)
    hipLaunchKernelGGL((cast_kernel<bf16raw, float>), grid, dim3(256), 0, s, (const bf16raw*)x, (float*)y, (long)n);
  else
    return DFK_EINVAL;
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_sgd_step(float* param, const float* grad, float* momentum_buf, void* bf16_shadow, int64_t n,
                            const float* lr_dev, float lr, float momentum, float weight_decay, int first_step,
                            const float* gate, float grad_scale, const void* grad_bf16, hipStream_t s) {
  if (!param || !grad || !momentum_buf) return DFK_EINVAL;
  if ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
       reinterpret_cast<uintptr_t>(momentum_buf)) & 15)
    return DFK_EINVAL;
  if (reinterpret_cast<uintptr_t>(grad_bf16) & 7) return DFK_EINVAL;
  if (n <= 0) return 0;
  const long threads = (n + 3) / 4;
  // DFK_SGD_NT=1: non-temporal stores (A/B runs; no measurable effect on the step or on the next step's patch
  // embedding, profiles/step/r4p_conv3d_instep_diagnosis.txt)
  static const bool nt = getenv("DFK_SGD_NT") && atoi(getenv("DFK_SGD_NT")) != 0;
  auto kfn = nt ? sgd_kernel<true> : sgd_kernel<false>;
  hipLaunchKernelGGL(kfn, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, param, grad, momentum_buf,
                     (bf16raw*)bf16_shadow, (long)n, lr_dev, lr, momentum, weight_decay, first_step, gate, grad_scale,
                     (const bf16raw*)grad_bf16);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_sgd_step_runs(float* param, const float* grad, float* momentum_buf, void* bf16_shadow,
                                 const int64_t* runs, int32_t nruns, const float* lr_dev, float lr, float momentum,
                                 float weight_decay, float grad_scale, const void* grad_bf16, hipStream_t s) {
  if (!param || !grad || !momentum_buf || !runs || nruns <= 0) return DFK_EINVAL;
  if (nruns > kSgdMaxRuns) return DFK_ENOTSUP;
  if ((reinterpret_cast<uintptr_t>(param) | reinterpret_cast<uintptr_t>(grad) |
       reinterpret_cast<uintptr_t>(momentum_buf)) & 15)
    return DFK_EINVAL;
  if ((reinterpret_cast<uintptr_t>(grad_bf16) | reinterpret_cast<uintptr_t>(bf16_shadow)) & 7) return DFK_EINVAL;
  SgdRuns R{};
  R.nruns = nruns;
  int64_t blocks = 0;
  for (int r = 0; r < nruns; ++r) {
    const int64_t* e = runs + 4 * r;          // {start, n, gate pointer, first}
    if (e[1] <= 0 || e[0] < 0 || (e[0] & 3)) return DFK_EINVAL;
    R.start[r] = e[0];
    R.n[r] = e[1];
    R.gate[r] = reinterpret_cast<const float*>(e[2]);
    if (e[3]) R.first |= 1ull << r;
    R.prefix[r] = (int32_t)blocks;
    blocks += (e[1] + kSgdRunBlock - 1) / kSgdRunBlock;
    if (blocks > 0x7fffffffL) return DFK_EINVAL;
  }
  R.prefix[nruns] = (int32_t)blocks;
  hipLaunchKernelGGL(sgd_runs_kernel, dim3((unsigned)blocks), dim3(256), 0, s, param, grad, momentum_buf,
                     (bf16raw*)bf16_shadow, R, lr_dev, lr, momentum, weight_decay, grad_scale,
                     (const bf16raw*)grad_bf16);
  DFK_CHECK_LAUNCH();
  return 0;
}

// ---- wav2vec2 positional-conv weight norm (HF weight_norm(dim=2), modeling_wav2vec2.py:336-350) ----
// v [C][Cg][k] fp32, g [k]: w = g v / ||v[:, :, kk]||.  The forward writes w straight into the two GEMM operand
// layouts the conv uses (w2: forward, w3: the transposed conv of its input gradient); the backward turns the dW GEMM's
// fp32 output (w2's layout) into dv / dg.  Each workgroup owns one output row of C (its Cg x k slice, 24 KB at the
// wav2vec2-base shape, staged in LDS so both the [Cg][k] and the [k][Cg] walks are coalesced); the per-kk sums go
// through [C][k] partials and one fixed-order reduce (deterministic).
namespace {

// part[o][kk] = sum_i v[o][i][kk]^2 (dw2 == nullptr) or sum_i v[o][i][kk] dw[o][i][kk], dw[o][i][kk] = dw2[o][kk*Cg+i]
__global__ __launch_bounds__(256) void wn_partial_kernel(const float* __restrict__ v, const float* __restrict__ dw2,
                                                         int Cg, int k, float* __restrict__ part) {
  extern __shared__ float wsm[];   // dw2 row o (k * Cg)
  const int o = blockIdx.x, n = Cg * k;
  const float* vo = v + (long)o * n;
  if (dw2) {
    for (int p = threadIdx.x; p < n; p += blockDim.x) wsm[p] = dw2[(long)o * n + p];
    __syncthreads();
  }
  for (int kk = threadIdx.x; kk < k; kk += blockDim.x) {
    float s = 0.f;
    for (int i = 0; i < Cg; ++i) {
      const float x = vo[i * k + kk];
      s += dw2 ? x * wsm[kk * Cg + i] : x * x;
    }
    part[(long)o * k + kk] = s;
  }
}

// fwd (dg == nullptr): norm[kk] = sqrt(sum_o part[o][kk]); bwd: dg[kk] += (sum_o part[o][kk]) / norm[kk], and the sum
// itself is left in part[0][kk] for the dv pass.  One workgroup per kk: 256 strided partial sums, then a fixed-order
// tree in LDS (one thread per kk walking all C partials took 170 us)
__global__ __launch_bounds__(256) void wn_reduce_kernel(float* __restrict__ part, int C, int k, float* __restrict__ norm,
                                                        float* __restrict__ dg) {
  __shared__ float red[256];
  const int kk = blockIdx.x, t = threadIdx.x;
  float s = 0.f;
  for (int o = t; o < C; o += 256) s += part[(long)o * k + kk];
  red[t] = s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if (t < h) red[t] += red[t + h];
    __syncthreads();
  }
  if (t == 0) {
    const float tot = red[0];
    if (dg) {
      dg[kk] += tot / norm[kk];
      part[kk] = tot;   // part[0][kk]: every workgroup has read its own column before this write (same kk only)
    } else {
      norm[kk] = sqrtf(tot);
    }
  }
}

// blockIdx.y 0: w2 row o = blockIdx.x, w2[o][kk*Cg+i] = g v[o][i][kk] / norm; 1: w3 row r = gr*Cg+ci,
// w3[r][u*Cg+co] = w[gr*Cg+co][ci][k-1-u]
template <typename T>
__global__ __launch_bounds__(256) void wn_apply_fwd_kernel(const float* __restrict__ v, const float* __restrict__ g,
                                                           const float* __restrict__ norm, int Cg, int k,
                                                           T* __restrict__ w2, T* __restrict__ w3) {
  extern __shared__ float vsm[];   // [Cg][k]: v[o] (w2) or v[gr*Cg+co][ci][:] for co = 0..Cg-1 (w3)
  const int row = blockIdx.x, n = Cg * k;
  const bool t3 = blockIdx.y == 1;
  const int gr = row / Cg, ci = row % Cg;
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int a = p / k, kk = p % k;   // a = i (w2) or co (w3)
    const long src = t3 ? ((long)(gr * Cg + a) * Cg + ci) * k + kk : (long)row * n + p;
    vsm[p] = v[src] * (g[kk] / norm[kk]);
  }
  __syncthreads();
  T* out = (t3 ? w3 : w2) + (long)row * n;
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int u = p / Cg, a = p % Cg;
    stf<T>(out + p, t3 ? vsm[a * k + (k - 1 - u)] : vsm[a * k + u]);
  }
}

// dv[o][i][kk] += g/norm dw - g s / norm^3 v  (s = part[0][kk] from wn_reduce_kernel)
__global__ __launch_bounds__(256) void wn_apply_bwd_kernel(const float* __restrict__ v, const float* __restrict__ g,
                                                           const float* __restrict__ norm, const float* __restrict__ s,
                                                           const float* __restrict__ dw2, int Cg, int k,
                                                           float* __restrict__ dv) {
  extern __shared__ float wsm[];   // dw2 row o
  const int o = blockIdx.x, n = Cg * k;
  for (int p = threadIdx.x; p < n; p += blockDim.x) wsm[p] = dw2[(long)o * n + p];
  __syncthreads();
  for (int p = threadIdx.x; p < n; p += blockDim.x) {
    const int i = p / k, kk = p % k;
    const float nk = norm[kk], gk = g[kk];
    dv[(long)o * n + p] += gk / nk * wsm[kk * Cg + i] - gk * s[kk] / (nk * nk * nk) * v[(long)o * n + p];
  }
}

}  // namespace

extern "C" int dfk_posconv_wnorm_fwd(const float* v, const float* g, int32_t C, int32_t Cg, int32_t k, float* norm,
                                     float* ws, void* w2, void* w3, int dtype, hipStream_t s) {
  if (!v || !g || !norm || !ws || !w2 || !w3 || C <= 0 || Cg <= 0 || k <= 0 || C % Cg) return DFK_EINVAL;
  if (dtype != DFK_BF16 && dtype != DFK_F32) return DFK_EINVAL;
  const size_t lds = sizeof(float) * (size_t)Cg * k;
  if (lds > 64 * 1024) return DFK_EINVAL;
  hipLaunchKernelGGL(wn_partial_kernel, dim3(C), dim3(256), 0, s, v, nullptr, Cg, k, ws);
  hipLaunchKernelGGL(wn_reduce_kernel, dim3(k), dim3(256), 0, s, ws, C, k, norm, nullptr);
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(wn_apply_fwd_kernel<bf16raw>, dim3(C, 2), dim3(256), lds, s, v, g, norm, Cg, k, (bf16raw*)w2,
                       (bf16raw*)w3);
  else
    hipLaunchKernelGGL(wn_apply_fwd_kernel<float>, dim3(C, 2), dim3(256), lds, s, v, g, norm, Cg, k, (float*)w2,
                       (float*)w3);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_posconv_wnorm_bwd(const float* v, const float* g, const float* norm, const float* dw2, int32_t C,
                                     int32_t Cg, int32_t k, float* ws, float* dv, float* dg, hipStream_t s) {
  if (!v || !g || !norm || !dw2 || !ws || !dv || !dg || C <= 0 || Cg <= 0 || k <= 0 || C % Cg) return DFK_EINVAL;
  const size_t lds = sizeof(float) * (size_t)Cg * k;
  if (lds > 64 * 1024) return DFK_EINVAL;
  hipLaunchKernelGGL(wn_partial_kernel, dim3(C), dim3(256), lds, s, v, dw2, Cg, k, ws);
  hipLaunchKernelGGL(wn_reduce_kernel, dim3(k), dim3(256), 0, s, ws, C, k, const_cast<float*>(norm), dg);
  hipLaunchKernelGGL(wn_apply_bwd_kernel, dim3(C), dim3(256), lds, s, v, g, norm, ws, dw2, Cg, k, dv);
  DFK_CHECK_LAUNCH();
  return 0;
}
