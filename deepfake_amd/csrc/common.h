// Shared device helpers for the DeepFake MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include "../../include/dfk.h"

typedef uint16_t bf16raw;  // bf16 storage (upper half of an fp32)

typedef __attribute__((ext_vector_type(8))) short short8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

__device__ __forceinline__ float bf2f(bf16raw v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ bf16raw f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (bf16raw)0x7fc0;  // keep NaN a NaN
  u += 0x7fffu + ((u >> 16) & 1u);                               // round to nearest even
  return (bf16raw)(u >> 16);
}

template <typename T> __device__ __forceinline__ float ldf(const T* p);
template <> __device__ __forceinline__ float ldf<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ldf<bf16raw>(const bf16raw* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ void stf(T* p, float v);
template <> __device__ __forceinline__ void stf<float>(float* p, float v) { *p = v; }
template <> __device__ __forceinline__ void stf<bf16raw>(bf16raw* p, float v) { *p = f2bf(v); }

// DFK_ST_NT: bf16 st8 stores carry the non-temporal hint (streaming outputs; experiment builds)
#ifndef DFK_ST_NT
#define DFK_ST_NT 0
#endif

// 8 consecutive elements <-> fp32 (16-B aligned: one bf16 vector / two f32 vectors)
template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* v) {
  if constexpr (sizeof(T) == 2) {
    const uint4 u = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* v) {
  if constexpr (sizeof(T) == 2) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (uint32_t)f2bf(v[2 * i]) | ((uint32_t)f2bf(v[2 * i + 1]) << 16);
#if DFK_ST_NT
    typedef unsigned int u32x4nt __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(u32x4nt{w[0], w[1], w[2], w[3]}, reinterpret_cast<u32x4nt*>(p));
#else
    *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
#endif
  } else {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  }
}

// GELU in the erf form, as torch.nn.GELU() / HF ACT2FN["gelu"].
// Standard normal CDF Phi(x) = erfc(-x / sqrt 2) / 2, branch-free (GELU epilogues run it per output element,
// and ocml's erff is a branchy piecewise evaluation that doubled the cost of a GELU GEMM epilogue).
// With t = |x| / sqrt 2:  t <= 1: erf(t) = t * PA(t^2);  t > 1: erfc(t) = exp(PB(t) - t^2) (PB fitted to
// log erfc(t) + t^2 on [1, 4]; t clamped to 4, where erfc < 2e-8).  Least-squares fits in float64, checked
// in float32 arithmetic: |erf error| <= 1.6e-7, erfc relative error <= 3.0e-6 (so Phi keeps its relative
// accuracy far into the negative tail).
__device__ __forceinline__ float phi_cdf(float x) {
  const float t = fabsf(x) * 0.70710678118654752f;
  const float s = t * t;
  float pa = 8.006874122656882e-05f;
  pa = fmaf(pa, s, -0.0008053751080296934f);
  pa = fmaf(pa, s, 0.005192957818508148f);
  pa = fmaf(pa, s, -0.0268560703843832f);
  pa = fmaf(pa, s, 0.11283634603023529f);
  pa = fmaf(pa, s, -0.3761262893676758f);
  pa = fmaf(pa, s, 1.128379225730896f);
  const float tb = fminf(fmaxf(t, 1.f), 4.f);
  float pb = -7.109802879767813e-08f;
  pb = fmaf(pb, tb, 3.2261048090731492e-06f);
  pb = fmaf(pb, tb, -6.147683598101139e-05f);
  pb = fmaf(pb, tb, 0.0006819369154982269f);
  pb = fmaf(pb, tb, -0.005053868982940912f);
  pb = fmaf(pb, tb, 0.027080601081252098f);
  pb = fmaf(pb, tb, -0.11103697121143341f);
  pb = fmaf(pb, tb, 0.36903998255729675f);
  pb = fmaf(pb, tb, -1.1306767463684082f);
  pb = fmaf(pb, tb, 0.0004179477400612086f);
  const float ecb = __builtin_amdgcn_exp2f(fmaf(-tb, tb, pb) * 1.4426950408889634f);
  const float ec = t <= 1.f ? fmaf(-t, pa, 1.f) : ecb;   // erfc(t)
  return x >= 0.f ? fmaf(-0.5f, ec, 1.f) : 0.5f * ec;
}
// GELU (erf form, nn.GELU default) and its derivative Phi(x) + x phi(x)
__device__ __forceinline__ float gelu_f(float x) { return x * phi_cdf(x); }

// The bf16 epilogues' Phi: erfc(t) = k P5(k) exp(-t^2), k = 1 / (1 + 0.3275911 t) (Abramowitz & Stegun
// 7.1.26, |erf error| <= 1.5e-7): one reciprocal, one exp and five FMAs instead of the two fitted
// polynomials above — GELU relative error <= 1.3e-5 wherever |GELU| > 1e-2 (0.08 % of bf16 outputs above
// 1e-3 move by one ulp), far inside bf16's 3.9e-3 spacing; fp32 parity mode keeps phi_cdf.  `e` returns
// exp(-x^2 / 2), the Gaussian factor GELU' needs as well.
__device__ __forceinline__ float phi_cdf_bf(float x, float& e) {
  const float t = fabsf(x) * 0.70710678118654752f;
  const float k = __builtin_amdgcn_rcpf(fmaf(0.3275911f, t, 1.f));
  float y = fmaf(k, 1.061405429f, -1.453152027f);
  y = fmaf(k, y, 1.421413741f);
  y = fmaf(k, y, -0.284496736f);
  y = fmaf(k, y, 0.254829592f);
  e = __builtin_amdgcn_exp2f(-1.4426950408889634f * t * t);
  const float ec = k * y * e;   // erfc(t)
  return x >= 0.f ? fmaf(-0.5f, ec, 1.f) : 0.5f * ec;
}
__device__ __forceinline__ float gelu_bf(float x) { float e; return x * phi_cdf_bf(x, e); }

// The same on a pair of values in packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: two elements per VALU issue;
// the reciprocal and the exp stay per element)
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f32x2 phi_cdf_bf2(f32x2 x, f32x2& e) {
  const f32x2 t = f32x2{fabsf(x.x), fabsf(x.y)} * 0.70710678118654752f;
  const f32x2 den = t * 0.3275911f + 1.f;
  const f32x2 k = f32x2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 y = k * 1.061405429f - 1.453152027f;
  y = k * y + 1.421413741f;
  y = k * y - 0.284496736f;
  y = k * y + 0.254829592f;
  const f32x2 tt = t * t * -1.4426950408889634f;
  e = f32x2{__builtin_amdgcn_exp2f(tt.x), __builtin_amdgcn_exp2f(tt.y)};
  const f32x2 ec = k * y * e;   // erfc(t)
  const f32x2 hi = ec * -0.5f + 1.f, lo = ec * 0.5f;
  return f32x2{x.x >= 0.f ? hi.x : lo.x, x.y >= 0.f ? hi.y : lo.y};
}
__device__ __forceinline__ f32x2 gelu_bf2(f32x2 x) { f32x2 e; return x * phi_cdf_bf2(x, e); }
__device__ __forceinline__ f32x2 dgelu_bf2(f32x2 x) {
  f32x2 e;
  const f32x2 p = phi_cdf_bf2(x, e);
  return x * 0.3989422804014327f * e + p;
}
__device__ __forceinline__ float dgelu_bf(float x) {
  float e;
  const float p = phi_cdf_bf(x, e);
  return fmaf(x * 0.3989422804014327f, e, p);
}
__device__ __forceinline__ float dgelu_f(float x) {
  return phi_cdf(x) + x * 0.3989422804014327f * __builtin_amdgcn_exp2f(-0.72134752044448170f * x * x);
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- dropout masks (dfk_drop, include/dfk.h): counter-based hash of (seed, step, site, row, col) ----
__device__ __forceinline__ uint32_t dfk_fmix(uint32_t h) {   // murmur3 finaliser
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
struct DropCtx {
  uint32_t key, thr;   // per-launch key; drop iff (hash >> 8) < thr
  float scale;         // 1 / (1 - p)
  int mode, grows;
};
__device__ __forceinline__ DropCtx drop_ctx(const dfk_drop& d) {
  DropCtx c;
  c.mode = d.rng ? d.mode : 0;
  c.key = 0; c.thr = 0; c.scale = 1.f; c.grows = d.group_rows > 0 ? d.group_rows : 1;
  if (c.mode) {
    const uint64_t seed = (uint64_t)d.rng[d.shared ? 2 : 0], step = (uint64_t)d.rng[1];
    uint32_t h = dfk_fmix((uint32_t)seed ^ 0x9e3779b9u);
    h = dfk_fmix(h ^ (uint32_t)(seed >> 32));
    h = dfk_fmix(h + (uint32_t)step * 0x85ebca77u);
    h = dfk_fmix(h ^ (uint32_t)(step >> 32));
    c.key = dfk_fmix(h + (uint32_t)d.site * 0xc2b2ae3du);
    c.thr = (uint32_t)(d.p * 16777216.f);
    c.scale = 1.f / (1.f - d.p);
  }
  return c;
}
// element (row, col) draw of mode 1; group draw (row / grows) of mode 2
__device__ __forceinline__ uint32_t drop_hash(const DropCtx& c, long row, long col) {
  if (c.mode == 2) return dfk_fmix(c.key ^ dfk_fmix((uint32_t)(row / c.grows) + 0x6a09e667u));
  const uint32_t h = dfk_fmix(c.key + (uint32_t)row * 0x9e3779b1u);
  return dfk_fmix(h ^ ((uint32_t)col * 0x85ebca77u + 0x165667b1u));
}
__device__ __forceinline__ float drop_mul(const DropCtx& c, long row, long col) {
  if (!c.mode) return 1.f;
  return (drop_hash(c, row, col) >> 8) >= c.thr ? c.scale : 0.f;
}

#define DFK_CHECK_LAUNCH() \
  do { hipError_t e_ = hipGetLastError(); if (e_ != hipSuccess) return (int)e_; } while (0)

static inline int dfk_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// weight-resident streaming GEMM (wres.hip): 1 = launched, 0 = not applicable, < 0 = launch error
int dfk_wres_try(const dfk_gemm_args& g, hipStream_t s);
int dfk_wgrad_try(const dfk_gemm_args& g, hipStream_t s);
// zeroed arrival-ticket slice of n counters for an in-launch combine (gemm.hip), nullptr if unavailable
uint32_t* dfk_ticket_slice(long n, hipStream_t s);
