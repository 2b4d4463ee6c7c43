// LayerNorm forward/backward over the channel (last) dim of channels-last token
// rows ([B,D,H,W,C] / [B,T,C]): every row is a contiguous C-vector.
//
// A row is owned by a group of L lanes (L = 16 / 32 / 64, the smallest power of
// two covering C/8 16-byte vectors), so a wave handles 64/L rows at once: the
// Swin stage-1 rows (C = 96 -> 12 vectors) keep 48 of 64 lanes busy instead of
// 12.  Each lane holds V vectors of 8 channels; row statistics are shuffle
// reductions inside the group.  Loads are branch-free (out-of-range vectors
// read the row start and are masked), so every load of a row is in flight at
// once.  The backward keeps x / dy in registers between its two sweeps when
// V <= 4, and reduces the dw / db partials group -> wave -> block in LDS with
// one atomic per channel per block.
#include "common.h"

namespace {

template <typename T>
__device__ __forceinline__ void load8m(const T* base, long off, bool ok, float (&v)[8]) {
  const T* p = base + (ok ? off : 0);
  if constexpr (sizeof(T) == 2) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    const bf16raw* e = reinterpret_cast<const bf16raw*>(&u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ok ? bf2f(e[i]) : 0.f;
  } else {
    const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ok ? v[i] : 0.f;
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

// raw 8-element vectors: the loads of a row group are issued as early as possible and converted when used
template <typename T> struct Raw8;
template <> struct Raw8<bf16raw> { uint4 u; };
template <> struct Raw8<float> { float4 a, b; };

template <typename T>
__device__ __forceinline__ Raw8<T> ld_raw(const T* base, long off, bool ok) {
  const T* p = base + (ok ? off : 0);
  Raw8<T> r;
  if constexpr (sizeof(T) == 2) {
    r.u = *reinterpret_cast<const uint4*>(p);
  } else {
    r.a = *reinterpret_cast<const float4*>(p);
    r.b = *reinterpret_cast<const float4*>(p + 4);
  }
  return r;
}

template <typename T>
__device__ __forceinline__ void unraw(const Raw8<T>& r, bool ok, float (&v)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16raw* e = reinterpret_cast<const bf16raw*>(&r.u);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ok ? bf2f(e[i]) : 0.f;
  } else {
    const float t[8] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = ok ? t[i] : 0.f;
  }
}

template <int L>
__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = L / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int L, int V>
__global__ __launch_bounds__(256) void ln_fwd(const T* __restrict__ x, const T* __restrict__ w,
                                              const T* __restrict__ b, T* __restrict__ y, float* mean_out,
                                              float* rstd_out, long rows, int C, float eps, const T* __restrict__ res,
                                              const dfk_drop drop) {
  constexpr int RPW = 64 / L;  // rows per wave
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane % L;
  const long row = ((long)blockIdx.x * 4 + wave) * RPW + lane / L;
  const bool rok = row < rows;
  const int nv = C / 8;
  const long roff = rok ? row * C : 0;
  float v[V][8];
  float s = 0.f;
  // the residual rows are loaded with x (one HBM round trip per row group, not two)
  Raw8<T> rr[V];
  if (res) {
#pragma unroll
    for (int i = 0; i < V; ++i) rr[i] = ld_raw<T>(res, roff + (li + i * L) * 8, rok && li + i * L < nv);
  }
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int vi = li + i * L;
    load8m<T>(x, roff + vi * 8, rok && vi < nv, v[i]);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += v[i][e];
  }
  const float mean = group_sum<L>(s) / C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const bool ok = li + i * L < nv;
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float d = ok ? v[i][e] - mean : 0.f; q += d * d; }
  }
  const float rstd = rsqrtf(group_sum<L>(q) / C + eps);
  const DropCtx dc = drop_ctx(drop);
  const float gmul = dc.mode == 2 ? drop_mul(dc, row, 0) : 1.f;
#pragma unroll
  for (int i = 0; i < V; ++i) {
    const int vi = li + i * L;
    const bool ok = vi < nv;
    float wv[8], bv[8], o[8];
    load8m<T>(w, vi * 8, ok, wv);
    load8m<T>(b, vi * 8, ok, bv);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * wv[e] + bv[e];
    if (dc.mode == 2) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= gmul;
    } else if (dc.mode == 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] *= drop_mul(dc, row, vi * 8 + e);
    }
    if (res) {
      float rv[8];
      unraw<T>(rr[i], rok && ok, rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] += rv[e];
    }
    if (rok && ok) store8<T>(y + row * C + vi * 8, o);
  }
  if (rok && li == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// dx = rstd * (g - mean(g) - xhat * mean(g*xhat)),  g = dy*w ; dw += dy*xhat ; db += dy
template <typename T, int L, int V, bool TWO>
__global__ __launch_bounds__(256) void ln_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                              const T* __restrict__ w, const float* __restrict__ mean,
                                              const float* __restrict__ rstd, T* __restrict__ dx, float* dw,
                                              float* db, long rows, int C, int accumulate, float* __restrict__ part,
                                              const dfk_drop drop, uint32_t* cnt, int gs, const T* __restrict__ addend) {
  constexpr int RPW = 64 / L;
  extern __shared__ float red[];  // [2][C] block partials of dw, db
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int li = lane % L;
  const int nv = C / 8;
  for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) red[i] = 0.f;
  float wv[V][8];
#pragma unroll
  for (int i = 0; i < V; ++i) load8m<T>(w, (li + i * L) * 8, li + i * L < nv, wv[i]);
  float pw[V][8], pb[V][8];
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { pw[i][e] = 0.f; pb[i][e] = 0.f; }
  __syncthreads();
  const DropCtx dc = drop_ctx(drop);   // the forward's mask on dy (gradient of drop(LN(x)))
  const long step = (long)gridDim.x * 4 * RPW;
  const bool add = addend || accumulate;
  const T* aptr = addend ? addend : dx;
  // A row group's operands — x, dy, the addend (or dx when accumulating), mean, rstd — as raw registers, all
  // loaded at once.  Narrow rows (bf16, V <= 2: every Swin stage-1/2 and SwinV2 LayerNorm) keep two groups in
  // flight: the wave's next-but-one group is loaded right after the current one is consumed (two register sets,
  // the loop unrolled by two, no copy of a register with a load in flight).
  struct Grp {
    Raw8<T> x[V], d[V], a[V];
    float mu, rs;
  };
  auto fetch = [&](Grp& gp, long r0) __attribute__((always_inline)) {
    const long row = r0 + lane / L;
    const bool rok = row < rows;
    const long roff = rok ? row * C : 0;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int vi = li + i * L;
      const bool ok = rok && vi < nv;
      gp.x[i] = ld_raw<T>(x, roff + vi * 8, ok);
      gp.d[i] = ld_raw<T>(dy, roff + vi * 8, ok);
      if (add) gp.a[i] = ld_raw<T>(aptr, roff + vi * 8, ok);
    }
    gp.mu = mean[rok ? row : 0];
    gp.rs = rstd[rok ? row : 0];
  };
  auto process = [&](const Grp& gp, long r0) __attribute__((always_inline)) {
    const long row = r0 + lane / L;
    const bool rok = row < rows;
    const float mu = gp.mu, rs = gp.rs;
    const float gmul = dc.mode == 2 ? drop_mul(dc, row, 0) : 1.f;
    float xs[V][8], ds[V][8];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int vi = li + i * L;
      const bool ok = rok && vi < nv;
      unraw<T>(gp.x[i], ok, xs[i]);
      unraw<T>(gp.d[i], ok, ds[i]);
      if (dc.mode == 2) {
#pragma unroll
        for (int e = 0; e < 8; ++e) ds[i][e] *= gmul;
      } else if (dc.mode == 1) {
#pragma unroll
        for (int e = 0; e < 8; ++e) ds[i][e] *= drop_mul(dc, row, vi * 8 + e);
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (xs[i][e] - mu) * rs, g = ds[i][e] * wv[i][e];
        s1 += g;
        s2 += g * xh;
        pw[i][e] += ok ? ds[i][e] * xh : 0.f;
        pb[i][e] += ds[i][e];
      }
    }
    const float m1 = group_sum<L>(s1) / C, m2 = group_sum<L>(s2) / C;
#pragma unroll
    for (int i = 0; i < V; ++i) {
      const int vi = li + i * L;
      const bool ok = rok && vi < nv;
      float o[8];
      if (add) unraw<T>(gp.a[i], ok, o);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xh = (xs[i][e] - mu) * rs;
        const float d = rs * (ds[i][e] * wv[i][e] - m1 - xh * m2);
        o[e] = add ? o[e] + d : d;
      }
      if (ok) store8<T>(dx + row * C + vi * 8, o);
    }
  };
  long r0 = ((long)blockIdx.x * 4 + wave) * RPW;
  if constexpr (TWO) {   // two groups in flight (a separate instantiation: its registers cost the one-group form occupancy)
    Grp ga, gb;
    fetch(ga, r0);
    fetch(gb, r0 + step);
    while (r0 < rows) {
      process(ga, r0);
      fetch(ga, r0 + 2 * step);   // past the end: clamped to row 0, masked
      r0 += step;
      if (r0 >= rows) break;
      process(gb, r0);
      fetch(gb, r0 + 2 * step);
      r0 += step;
    }
  } else {
    for (; r0 < rows; r0 += step) {
      Grp gp;
      fetch(gp, r0);
      process(gp, r0);
    }
  }
  // dw / db partials: sum the RPW row groups of the wave, then the waves of the block through LDS
#pragma unroll
  for (int i = 0; i < V; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int o = L; o < 64; o <<= 1) {
        pw[i][e] += __shfl_xor(pw[i][e], o, 64);
        pb[i][e] += __shfl_xor(pb[i][e], o, 64);
      }
  for (int wv2 = 0; wv2 < 4; ++wv2) {   // waves in turn: plain read-modify-write, distinct channels per lane
    if (wave == wv2 && lane < L) {
#pragma unroll
      for (int i = 0; i < V; ++i) {
        const int vi = li + i * L;
        if (vi < nv)
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[vi * 8 + e] += pw[i][e];
            red[C + vi * 8 + e] += pb[i][e];
          }
      }
    }
    __syncthreads();
  }
  if (part) {   // block partials -> [blocks][2C] slab (no same-address atomics from every block)
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) part[(long)blockIdx.x * 2 * C + i] = red[i];
    if (!cnt) return;   // slab_colsum sums the slab
    // in-launch combine per group of gs blocks: publish (drain, barrier, agent release), ticket; the group's last
    // arriver acquires, sums the group's rows in block order and adds the group sum (groups-way atomics)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    const int grp = blockIdx.x / gs, g0 = grp * gs, gn = min(gs, (int)gridDim.x - g0);
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t = __hip_atomic_fetch_add(cnt + grp, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = t == (uint32_t)(gn - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(cnt + grp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      red[0] = last ? 1.f : 0.f;
    }
    __syncthreads();
    if (red[0] == 0.f) return;
    for (int i = threadIdx.x; i < 2 * C; i += blockDim.x) {
      const float* src = part + (long)g0 * 2 * C + i;
      float a[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      int r = 0;
      for (; r + 8 <= gn; r += 8)
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] += src[(long)(r + u) * 2 * C];
      for (; r < gn; ++r) a[0] += src[(long)r * 2 * C];   // ragged last group
      const float t = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
      float* out = i < C ? dw : db;
      if (out) atomicAdd(out + (i < C ? i : i - C), t);
    }
    return;
  }
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    if (dw) atomicAdd(dw + i, red[i]);
    if (db) atomicAdd(db + i, red[C + i]);
  }
}

// dw[j] += sum_r part[r][j], db[j] += sum_r part[r][C + j]: one launch for both halves of the [rows][2C]
// slab; a workgroup sums 256 slab rows of 64 columns (4 row phases x 64 coalesced columns, 8 loads in
// flight per lane), folds the phases through LDS and adds once per column (rows/256-way atomics)
__global__ __launch_bounds__(256) void slab_colsum(const float* __restrict__ part, int rows, int C,
                                                   float* __restrict__ dw, float* __restrict__ db) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  const int r0 = blockIdx.y * 256;
  const bool ok = j < 2 * C;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < 64; i += 8)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = r0 + ph + 4 * (i + u);
      s[u] += (ok && r < rows) ? part[(long)r * 2 * C + j] : 0.f;
    }
  red[ph][lane] = ((s[0] + s[1]) + (s[2] + s[3])) + ((s[4] + s[5]) + (s[6] + s[7]));
  __syncthreads();
  if (ph == 0 && ok) {
    const float t = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    float* out = j < C ? dw : db;
    if (out) atomicAdd(out + (j < C ? j : j - C), t);
  }
}

constexpr long kLnSmallRows = 4096;   // kernels.py _LN_SMALL_ROWS

long bwd_blocks(long rows, int C) {
  const int nv = C / 8;
  const int L = nv <= 16 ? 16 : (nv <= 32 ? 32 : 64);
  // at most 2048 workgroups, 512 from C = 512 up: their [blocks][2C] partial slab, summed by slab_colsum, grows
  // with C (tools/ln_bench.py, profiles/r4/r4s_ln_bwd_block_cap.txt: [6272, 768] 46 -> 25 us at 512, while the
  // narrow stage-1/2 rows need the 2048 workgroups: [401408, 96] 65 -> 84 us at 512)
  static const long env = getenv("DFK_LN_BWD_BLOCKS") ? atol(getenv("DFK_LN_BWD_BLOCKS")) : 0;   // tuning runs
  const long cap = env > 0 ? env : (C >= 512 ? 512 : 2048);
  // small LayerNorms (rows <= kLnSmallRows: the SwinV2 stage-3/4 and wav2vec2 ones): at most 128 workgroups adding
  // their dw/db partials atomically, no slab pass (r6b: 1568 x 512 14.1 -> 11.5 us, 1592 x 768 17.8 -> 15.9,
  // 392 x 1024 16.5 -> 12.5; from 6k rows the slab + column pass stays faster).  DFK_LN_SMALL=n: n workgroups (A/B)
  static const long small = getenv("DFK_LN_SMALL") ? atol(getenv("DFK_LN_SMALL")) : 128;
  if (small > 0 && rows <= kLnSmallRows) return std::min<long>(small, dfk_cdiv(rows, 4L * (64 / L)));
  return std::min<long>(cap, dfk_cdiv(rows, 4L * (64 / L)));
}

template <typename T, int L, int V>
void fwd_launch(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, long rows, int C,
                float eps, const void* res, dfk_drop drop, hipStream_t s) {
  const long per_block = 4L * (64 / L);
  hipLaunchKernelGGL((ln_fwd<T, L, V>), dim3((unsigned)dfk_cdiv(rows, per_block)), dim3(256), 0, s, (const T*)x,
                     (const T*)w, (const T*)b, (T*)y, mean, rstd, rows, C, eps, (const T*)res, drop);
}

template <typename T, int L, int V>
void bwd_launch(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx, float* dw,
                float* db, long rows, int C, int accumulate, float* ws, dfk_drop drop, const void* addend,
                hipStream_t s) {
  const int blocks = (int)bwd_blocks(rows, C);
  float* part = ws && (dw || db) ? ws : nullptr;
  // in-launch combine groups: about 48 KB of partials per group's reducer, 8-64 blocks
  int gs = 64;
  while (gs > 8 && (long)gs * 8 * C > 49152) gs >>= 1;
  uint32_t* cnt = part ? dfk_ticket_slice(dfk_cdiv(blocks, gs), s) : nullptr;
  // two row groups in flight when the waves loop (bf16 rows of at most 2 x 64 x 8 channels)
  const bool two = sizeof(T) == 2 && V <= 2 && rows > (long)blocks * 4 * (64 / L);
  if (two)
    hipLaunchKernelGGL((ln_bwd<T, L, V, (sizeof(T) == 2 && V <= 2)>), dim3(blocks), dim3(256), 2 * C * sizeof(float), s,
                       (const T*)dy, (const T*)x, (const T*)w, mean, rstd, (T*)dx, dw, db, rows, C, accumulate, part,
                       drop, cnt, gs, (const T*)addend);
  else
    hipLaunchKernelGGL((ln_bwd<T, L, V, false>), dim3(blocks), dim3(256), 2 * C * sizeof(float), s, (const T*)dy,
                       (const T*)x, (const T*)w, mean, rstd, (T*)dx, dw, db, rows, C, accumulate, part, drop, cnt, gs,
                       (const T*)addend);
  if (part && !cnt)
    hipLaunchKernelGGL(slab_colsum, dim3(dfk_cdiv(2 * C, 64), dfk_cdiv(blocks, 256)), dim3(256), 0, s, part, blocks, C,
                       dw, db);
}

// (L, V) for C: L = lanes per row, V = 8-channel vectors per lane
template <typename T, template <typename, int, int> class F, typename... Args>
bool pick(int C, Args... args) {
  const int nv = C / 8;
  if (nv <= 16) { F<T, 16, 1>::run(args...); return true; }
  if (nv <= 32) { F<T, 32, 1>::run(args...); return true; }
  switch ((nv + 63) / 64) {
    case 1: F<T, 64, 1>::run(args...); return true;
    case 2: F<T, 64, 2>::run(args...); return true;
    case 3: F<T, 64, 3>::run(args...); return true;
    case 4: F<T, 64, 4>::run(args...); return true;
    case 5: F<T, 64, 5>::run(args...); return true;
    case 6: F<T, 64, 6>::run(args...); return true;
    case 7: F<T, 64, 7>::run(args...); return true;
    case 8: F<T, 64, 8>::run(args...); return true;
    default: return false;
  }
}

template <typename T, int L, int V>
struct Fwd {
  static void run(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd, long rows, int C,
                  float eps, const void* res, dfk_drop drop, hipStream_t s) {
    fwd_launch<T, L, V>(x, w, b, y, mean, rstd, rows, C, eps, res, drop, s);
  }
};

template <typename T, int L, int V>
struct Bwd {
  static void run(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, void* dx,
                  float* dw, float* db, long rows, int C, int accumulate, float* ws, dfk_drop drop, const void* addend,
                  hipStream_t s) {
    bwd_launch<T, L, V>(dy, x, w, mean, rstd, dx, dw, db, rows, C, accumulate, ws, drop, addend, s);
  }
};

dfk_drop drop_or_none(const dfk_drop* d) {
  dfk_drop z = {nullptr, 0, 0, 0.f, 1, 0};
  return d && d->rng && d->mode ? *d : z;
}

bool drop_ok(const dfk_drop* d) { return !d || !d->mode || (d->rng && d->p >= 0.f && d->p < 1.f); }

}  // namespace

extern "C" int dfk_layernorm_fwd(const void* x, const void* w, const void* b, void* y, float* mean, float* rstd,
                                 int64_t rows, int32_t C, float eps, int dtype, const void* residual,
                                 const dfk_drop* drop, hipStream_t s) {
  if (!x || !w || !b || !y || C <= 0 || C % 8 || C > 4096 || !drop_ok(drop)) return DFK_EINVAL;
  if (rows <= 0) return 0;
  const dfk_drop d = drop_or_none(drop);
  const bool ok = dtype == DFK_BF16
                      ? pick<bf16raw, Fwd>(C, x, w, b, y, mean, rstd, (long)rows, (int)C, eps, residual, d, s)
                      : pick<float, Fwd>(C, x, w, b, y, mean, rstd, (long)rows, (int)C, eps, residual, d, s);
  if (!ok) return DFK_EINVAL;
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t dfk_layernorm_bwd_workspace(int64_t rows, int32_t C) {
  if (rows <= 0 || C <= 0) return 0;
  return bwd_blocks(rows, C) * 2 * (int64_t)C * (int64_t)sizeof(float);
}

extern "C" int dfk_layernorm_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd,
                                 void* dx, float* dw, float* db, int64_t rows, int32_t C, int accumulate, int dtype,
                                 float* ws, const dfk_drop* drop, const void* addend, hipStream_t s) {
  if (!dy || !x || !w || !mean || !rstd || !dx || C <= 0 || C % 8 || C > 4096 || !drop_ok(drop)) return DFK_EINVAL;
  if (rows <= 0) return 0;
  const dfk_drop d = drop_or_none(drop);
  const bool ok = dtype == DFK_BF16
                      ? pick<bf16raw, Bwd>(C, dy, x, w, mean, rstd, dx, dw, db, (long)rows, (int)C, accumulate, ws, d, addend, s)
                      : pick<float, Bwd>(C, dy, x, w, mean, rstd, dx, dw, db, (long)rows, (int)C, accumulate, ws, d, addend, s);
  if (!ok) return DFK_EINVAL;
  DFK_CHECK_LAUNCH();
  return 0;
}
