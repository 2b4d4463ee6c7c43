// Generic MFMA GEMM for gfx950 with operand views (plain / transposed /
// implicit-conv), batching, split-K and fused epilogues.  See include/dfk.h.
//
// Tile 128x128 per 256-thread workgroup (4 waves, 2x2, 64x64 each).
//   bf16: v_mfma_f32_16x16x32_bf16, BK = 64 (2 MFMA k-steps per staged tile)
//   f32 : v_mfma_f32_16x16x4_f32   (exact fp32, parity mode), BK = 32
// Staging: global -> registers (16-B vectors along the contiguous dim of each
// view) -> LDS tile stored [row][k] (k contiguous); the next tile's global
// loads are issued before the current tile's MFMAs (register prefetch).
#include "common.h"

namespace {

constexpr int BM = 128, BN = 128, NT = 256;

template <typename T> struct GT;
template <> struct GT<bf16raw> { static constexpr int BK = 64, VEC = 8, PAD = 8; };
template <> struct GT<float> { static constexpr int BK = 32, VEC = 4, PAD = 4; };

// element offset of V(r, c), or -1 when it lies in the conv view's zero padding
__device__ __forceinline__ long view_off(const dfk_view& v, long r, long c) {
  if (v.conv_cg > 0) {
    const long kk = c / v.conv_cg;
    const long row = r * v.conv_stride + kk - v.conv_pad;
    if (row < 0 || row >= v.conv_rows) return -1;
    return row * v.ld + (c - kk * v.conv_cg);
  }
  return r * v.ld + c;
}

// 16-byte load of VEC contiguous elements V(r, c .. c+VEC-1); zero outside the
// view (rok false, c >= climit, conv padding).  `vec` (host-checked alignment of
// ptr/ld/batch strides/conv group) selects the vector load; otherwise (odd
// shapes such as the out_dim=1 classifier) element-wise loads.
template <typename T>
__device__ __forceinline__ uint4 view_load(const T* base, const dfk_view& v, long r, long c, bool rok, long climit,
                                           bool vec) {
  constexpr int VEC = 16 / sizeof(T);
  uint4 z = make_uint4(0, 0, 0, 0);
  if (!rok || c >= climit) return z;
  if (vec && c + VEC <= climit) {
    const long o = view_off(v, r, c);
    return o < 0 ? z : *reinterpret_cast<const uint4*>(base + o);
  }
  T* e = reinterpret_cast<T*>(&z);
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    if (c + i < climit) {
      const long o = view_off(v, r, c + i);
      if (o >= 0) e[i] = base[o];
    }
  }
  return z;
}

template <typename T>
__device__ __forceinline__ void scatter_col(T* lds, int stride, int r0, int kcol, uint4 val) {
  // write VEC elements (consecutive rows r0.., fixed k column) — transposed staging
  const T* e = reinterpret_cast<const T*>(&val);
#pragma unroll
  for (int i = 0; i < GT<T>::VEC; ++i) lds[(r0 + i) * stride + kcol] = e[i];
}

template <typename T, bool KMAJ, int ROWS>
__device__ __forceinline__ void load_tile(const T* base, const dfk_view& v, int row0, int rowlim, int k0, int klim,
                                          int tid, bool vec, uint4 (&r)[4]) {
  constexpr int TBK = GT<T>::BK, VEC = GT<T>::VEC;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int idx = tid + s * NT;
    if (!KMAJ) {  // view rows = tile rows, contiguous along k
      const int i = idx / (TBK / VEC), kc = idx % (TBK / VEC);
      const int gr = row0 + i, gk = k0 + kc * VEC;
      r[s] = view_load<T>(base, v, gr, gk, gr < rowlim, klim, vec);
    } else {      // view rows = k, contiguous along tile rows
      const int k = idx / (ROWS / VEC), ic = idx % (ROWS / VEC);
      const int gk = k0 + k, gr = row0 + ic * VEC;
      r[s] = view_load<T>(base, v, gk, gr, gk < klim, rowlim, vec);
    }
  }
}

template <typename T, bool KMAJ, int ROWS>
__device__ __forceinline__ void store_tile(T* lds, int tid, const uint4 (&r)[4]) {
  constexpr int TBK = GT<T>::BK, VEC = GT<T>::VEC, S = TBK + GT<T>::PAD;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int idx = tid + s * NT;
    if (!KMAJ) {
      const int i = idx / (TBK / VEC), kc = idx % (TBK / VEC);
      *reinterpret_cast<uint4*>(lds + i * S + kc * VEC) = r[s];
    } else {
      const int k = idx / (ROWS / VEC), ic = idx % (ROWS / VEC);
      scatter_col<T>(lds, S, ic * VEC, k, r[s]);
    }
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <typename T, bool AK, bool BK>
__global__ __launch_bounds__(256) void gemm_kernel(const dfk_gemm_args g, int kchunk, int avec, int bvec) {
  constexpr int TBK = GT<T>::BK, S = TBK + GT<T>::PAD;
  __shared__ __attribute__((aligned(16))) T As[BM * S];
  __shared__ __attribute__((aligned(16))) T Bs[BN * S];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int bn = blockIdx.x * BN, bm = blockIdx.y * BM;
  int z = blockIdx.z;
  const int split = z % g.splitk;
  z /= g.splitk;
  const int z0 = z / g.nz1, z1 = z % g.nz1;
  const T* A = reinterpret_cast<const T*>(g.a.ptr) + z0 * g.a.bs0 + z1 * g.a.bs1;
  const T* B = reinterpret_cast<const T*>(g.b.ptr) + z0 * g.b.bs0 + z1 * g.b.bs1;
  const int kbeg = split * kchunk;
  const int kend = min(g.K, kbeg + kchunk);

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  uint4 ra[4], rb[4];
  if (kbeg < kend) {
    load_tile<T, AK, BM>(A, g.a, bm, g.M, kbeg, kend, tid, avec, ra);
    load_tile<T, BK, BN>(B, g.b, bn, g.N, kbeg, kend, tid, bvec, rb);
    store_tile<T, AK, BM>(As, tid, ra);
    store_tile<T, BK, BN>(Bs, tid, rb);
  }
  __syncthreads();
  for (int k0 = kbeg; k0 < kend; k0 += TBK) {
    const bool more = k0 + TBK < kend;
    if (more) {
      load_tile<T, AK, BM>(A, g.a, bm, g.M, k0 + TBK, kend, tid, avec, ra);
      load_tile<T, BK, BN>(B, g.b, bn, g.N, k0 + TBK, kend, tid, bvec, rb);
    }
    if constexpr (sizeof(T) == 2) {
#pragma unroll
      for (int ks = 0; ks < TBK / 32; ++ks) {
        bf16x8 af[4], bfr[4];
        const int kof = ks * 32 + (lane >> 4) * 8;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
          af[mi] = *reinterpret_cast<const bf16x8*>(As + (wm * 64 + mi * 16 + (lane & 15)) * S + kof);
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          bfr[ni] = *reinterpret_cast<const bf16x8*>(Bs + (wn * 64 + ni * 16 + (lane & 15)) * S + kof);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < TBK / 4; ++ks) {
        float af[4], bfr[4];
        const int kof = ks * 4 + (lane >> 4);
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) af[mi] = As[(wm * 64 + mi * 16 + (lane & 15)) * S + kof];
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) bfr[ni] = Bs[(wn * 64 + ni * 16 + (lane & 15)) * S + kof];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      }
    }
    __syncthreads();
    if (more) {
      store_tile<T, AK, BM>(As, tid, ra);
      store_tile<T, BK, BN>(Bs, tid, rb);
      __syncthreads();
    }
  }

  // ---- epilogue
  const T* bias = g.bias ? reinterpret_cast<const T*>(g.bias) + z1 * g.bias_bs1 : nullptr;
  const T* res = g.residual ? reinterpret_cast<const T*>(g.residual) + z0 * g.rbs0 + z1 * g.rbs1 : nullptr;
  const long coff = z0 * g.cbs0 + z1 * g.cbs1;
  T* aux = g.aux ? reinterpret_cast<T*>(g.aux) + coff : nullptr;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni) {
      const int col = bn + wn * 64 + ni * 16 + (lane & 15);
      if (col >= g.N) continue;
      const float bv = bias ? ldf<T>(bias + col) : 0.f;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm + wm * 64 + mi * 16 + (lane >> 4) * 4 + r;
        if (row >= g.M) continue;
        float v = acc[mi][ni][r] + bv;
        if (g.act == 1) {
          if (aux) stf<T>(aux + (long)row * g.ldaux + col, v);
          v = gelu_f(v);
        } else if (g.act == 2) {
          v *= dgelu_f(ldf<T>(aux + (long)row * g.ldaux + col));
        }
        if (res) v += ldf<T>(res + (long)row * g.ldr + col);
        const long ci = coff + (long)row * g.ldc + col;
        if (g.atomic) {
          atomicAdd(reinterpret_cast<float*>(g.c) + ci, v);
        } else if (g.c_f32) {
          float* C = reinterpret_cast<float*>(g.c) + ci;
          *C = g.beta != 0.f ? v + g.beta * *C : v;
        } else {
          T* C = reinterpret_cast<T*>(g.c) + ci;
          stf<T>(C, g.beta != 0.f ? v + g.beta * ldf<T>(C) : v);
        }
      }
    }
  }
}

template <typename T>
__global__ void colsum_kernel(const T* __restrict__ x, long rows, int cols, long ld, long rows_per, float* out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= cols) return;
  const long r0 = blockIdx.y * rows_per, r1 = min(rows, r0 + rows_per);
  float s = 0.f;
  for (long r = r0; r < r1; ++r) s += ldf<T>(x + r * ld + j);
  atomicAdd(out + j, s);
}

// 16-byte vector loads are legal for this view (else the element-wise path runs)
bool view_vec(const dfk_view& v, int vec) {
  if (v.ld % vec || v.bs0 % vec || v.bs1 % vec) return false;
  if ((reinterpret_cast<uintptr_t>(v.ptr) & 15) != 0) return false;
  if (v.conv_cg > 0 && v.conv_cg % vec) return false;
  return true;
}

template <typename T>
int launch(const dfk_gemm_args& g, hipStream_t s) {
  constexpr int VEC = GT<T>::VEC, TBK = GT<T>::BK;
  if (!g.a.ptr || !g.b.ptr || !g.c) return DFK_EINVAL;
  if ((g.a.conv_cg > 0 && g.a.conv_stride <= 0) || (g.b.conv_cg > 0 && g.b.conv_stride <= 0)) return DFK_EINVAL;
  const int avec = view_vec(g.a, VEC), bvec = view_vec(g.b, VEC);
  if (g.splitk < 1 || g.nz0 < 1 || g.nz1 < 1) return DFK_EINVAL;
  if (g.splitk > 1 && !g.atomic) return DFK_EINVAL;
  if (g.atomic && (!g.c_f32 || g.bias || g.residual || g.act)) return DFK_EINVAL;
  if (g.act && g.act != 1 && !g.aux) return DFK_EINVAL;
  if (g.M <= 0 || g.N <= 0) return 0;
  int kchunk = dfk_cdiv(g.K, g.splitk);
  kchunk = dfk_cdiv(kchunk, TBK) * TBK;
  dim3 grid(dfk_cdiv(g.N, BN), dfk_cdiv(g.M, BM), g.nz0 * g.nz1 * g.splitk);
  if (grid.y > 65535 || grid.z > 65535) return DFK_EINVAL;
  if (g.a_kmajor) {
    if (g.b_kmajor) hipLaunchKernelGGL((gemm_kernel<T, true, true>), grid, dim3(NT), 0, s, g, kchunk, avec, bvec);
    else hipLaunchKernelGGL((gemm_kernel<T, true, false>), grid, dim3(NT), 0, s, g, kchunk, avec, bvec);
  } else {
    if (g.b_kmajor) hipLaunchKernelGGL((gemm_kernel<T, false, true>), grid, dim3(NT), 0, s, g, kchunk, avec, bvec);
    else hipLaunchKernelGGL((gemm_kernel<T, false, false>), grid, dim3(NT), 0, s, g, kchunk, avec, bvec);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int dfk_gemm(const dfk_gemm_args* g, hipStream_t s) {
  if (!g) return DFK_EINVAL;
  return g->dtype == DFK_BF16 ? launch<bf16raw>(*g, s) : launch<float>(*g, s);
}

extern "C" int dfk_colsum(const void* x, int dtype, int64_t rows, int64_t cols, int64_t ld, float* out,
                          hipStream_t s) {
  if (!x || !out || cols <= 0) return DFK_EINVAL;
  if (rows <= 0) return 0;
  long chunks = rows < 64 ? 1 : std::min<long>(1024, (rows + 63) / 64);
  long rows_per = (rows + chunks - 1) / chunks;
  chunks = (rows + rows_per - 1) / rows_per;
  dim3 grid(dfk_cdiv(cols, 256), (unsigned)chunks);
  if (dtype == DFK_BF16)
    hipLaunchKernelGGL(colsum_kernel<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)x, (long)rows, (int)cols,
                       (long)ld, rows_per, out);
  else
    hipLaunchKernelGGL(colsum_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (long)rows, (int)cols,
                       (long)ld, rows_per, out);
  DFK_CHECK_LAUNCH();
  return 0;
}
