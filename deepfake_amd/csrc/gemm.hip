// Generic MFMA GEMM for gfx950 with operand views (plain / k-major / implicit
// conv), batching, split-K and fused epilogues.  See include/dfk.h.
//
// Tile 128x128 (or 64x64 for grids too small to fill the chip) per 256-thread workgroup (4 waves, 2x2).
//   bf16: v_mfma_f32_16x16x32_bf16, BK = 64 (2 MFMA k-steps per staged tile)
//   f32 : v_mfma_f32_16x16x4_f32   (exact fp32, parity mode), BK = 32
// Staging: global -> registers (16-B vectors along each view's contiguous dim)
// -> LDS in the view's NATURAL orientation:
//   k-contiguous operand  -> tile [row][k]  : fragments by ds_read_b128
//   k-major operand       -> tile [k][row]  : bf16 fragments by two
//                            ds_read_b64_tr_b16 (hardware transpose), so the
//                            dX / dW GEMMs of every Linear never scatter.
// LDS is double-buffered: the next tile's global loads are in flight during
// the current tile's MFMAs, one barrier per k-tile.
// bf16 launches with plain views take the LDS-DMA kernel instead (gemm_dma_kernel, below): the same tiles
// and MFMAs, operands moved HBM -> LDS by buffer_load ... lds with source-swizzled, conflict-free images.
// The register-staged kernel remains for fp32 parity mode and the implicit-conv views.
#include <mutex>

#include "common.h"

namespace {

constexpr int NT = 256;   // 4 waves (2 x 2), wave tile WT x WT, workgroup tile 2WT x 2WT

// split-K state of a launch: fp32 partial slabs [z][split][M][N] and (in-launch combine) one arrival ticket per
// output tile; cnt == nullptr: the partials are combined by splitk_reduce_kernel instead
struct SplitK {
  float* slab;
  uint32_t* cnt;
};

template <typename T> struct GT;
template <> struct GT<bf16raw> { static constexpr int BK = 64, VEC = 8, PADR = 8, PADK = 16; };
template <> struct GT<float> { static constexpr int BK = 32, VEC = 4, PADR = 4, PADK = 4; };

// LDS tile geometry for one operand (ROWS x BK): [row][k] or [k][row]
template <typename T, bool KMAJ, int ROWS>
struct Tile {
  static constexpr int TBK = GT<T>::BK;
  static constexpr int STRIDE = KMAJ ? ROWS + GT<T>::PADK : TBK + GT<T>::PADR;   // elements
  static constexpr int ELEMS = KMAJ ? TBK * STRIDE : ROWS * STRIDE;
};

// element offset of V(r, c), or -1 when it lies in the conv view's zero padding
template <bool CONV>
__device__ __forceinline__ long view_off(const dfk_view& v, long r, long c) {
  if constexpr (CONV) {
    if (v.conv_cg > 0) {
      const long kk = c / v.conv_cg;
      const long row = r * v.conv_stride + kk - v.conv_pad;
      if (row < 0 || row >= v.conv_rows) return -1;
      return row * v.ld + (c - kk * v.conv_cg);
    }
  }
  return r * v.ld + c;
}

// VEC contiguous elements V(r, c..c+VEC-1); zeros outside the view.
// VECOK: host guarantees 16-B alignment and whole-vector extents -> one vector load.
// Otherwise elements are assembled in registers (odd shapes, e.g. out_dim=1).
template <typename T, bool VECOK, bool CONV>
__device__ __forceinline__ uint4 view_load(const T* base, const dfk_view& v, long r, long c, bool rok, long climit) {
  constexpr int VEC = 16 / sizeof(T);
  uint4 z = make_uint4(0, 0, 0, 0);
  if constexpr (VECOK) {
    // branch-free: an out-of-range element loads from the view base and is masked to zero, so the
    // compiler keeps every tile load in flight (a branch around a load makes it wait vmcnt(0) there)
    const long o = view_off<CONV>(v, r, c);
    const bool ok = rok && c < climit && o >= 0;
    uint4 x = *reinterpret_cast<const uint4*>(base + (ok ? o : 0));
    const uint32_t m = ok ? 0xffffffffu : 0u;
    x.x &= m; x.y &= m; x.z &= m; x.w &= m;
    return x;
  } else {
    if (!rok || c >= climit) return z;
    uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      if (c + i < climit) {
        const long o = view_off<CONV>(v, r, c + i);
        if (o >= 0) {
          if constexpr (sizeof(T) == 2) {
            w[i >> 1] |= (uint32_t)(*reinterpret_cast<const uint16_t*>(base + o)) << (16 * (i & 1));
          } else {
            w[i] = *reinterpret_cast<const uint32_t*>(base + o);
          }
        }
      }
    }
    return make_uint4(w[0], w[1], w[2], w[3]);
  }
}

// stage one ROWS x BK operand tile: global -> 4 x 16-B registers per thread
template <typename T, int ROWS> constexpr int tile_vecs() { return ROWS * GT<T>::BK / (NT * GT<T>::VEC); }

template <typename T, bool KMAJ, int ROWS, bool VECOK, bool CONV>
__device__ __forceinline__ void load_tile(const T* base, const dfk_view& v, int row0, int rowlim, int k0, int klim,
                                          int tid, uint4 (&r)[tile_vecs<T, ROWS>()]) {
  constexpr int TBK = GT<T>::BK, VEC = GT<T>::VEC;
#pragma unroll
  for (int s = 0; s < tile_vecs<T, ROWS>(); ++s) {
    const int idx = tid + s * NT;
    if constexpr (!KMAJ) {   // view rows = tile rows, contiguous along k
      const int i = idx / (TBK / VEC), kc = idx % (TBK / VEC);
      const int gr = row0 + i, gk = k0 + kc * VEC;
      r[s] = view_load<T, VECOK, CONV>(base, v, gr, gk, gr < rowlim, klim);
    } else {                 // view rows = k, contiguous along tile rows
      const int k = idx / (ROWS / VEC), ic = idx % (ROWS / VEC);
      const int gk = k0 + k, gr = row0 + ic * VEC;
      r[s] = view_load<T, VECOK, CONV>(base, v, gk, gr, gk < klim, rowlim);
    }
  }
}

template <typename T, bool KMAJ, int ROWS>
__device__ __forceinline__ void store_tile(T* lds, int tid, const uint4 (&r)[tile_vecs<T, ROWS>()]) {
  using TL = Tile<T, KMAJ, ROWS>;
  constexpr int TBK = GT<T>::BK, VEC = GT<T>::VEC;
#pragma unroll
  for (int s = 0; s < tile_vecs<T, ROWS>(); ++s) {
    const int idx = tid + s * NT;
    if constexpr (!KMAJ) {
      const int i = idx / (TBK / VEC), kc = idx % (TBK / VEC);
      *reinterpret_cast<uint4*>(lds + i * TL::STRIDE + kc * VEC) = r[s];
    } else {
      const int k = idx / (ROWS / VEC), ic = idx % (ROWS / VEC);
      *reinterpret_cast<uint4*>(lds + k * TL::STRIDE + ic * VEC) = r[s];
    }
  }
}

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;

// bf16 MFMA fragment: 8 consecutive k (kb..kb+7) of tile row r (lane&15 within a 16-row block)
template <bool KMAJ, int ROWS>
__device__ __forceinline__ bf16x8 frag_bf16(const bf16raw* lds, int r0, int kb, int lane) {
  using TL = Tile<bf16raw, KMAJ, ROWS>;
  if constexpr (!KMAJ) {
    return *reinterpret_cast<const bf16x8*>(lds + (r0 + (lane & 15)) * TL::STRIDE + kb + (lane >> 4) * 8);
  } else {
    // ds_read_b64_tr_b16: lane 4q+p of each 16-lane group addresses row (k) q, columns 4p..4p+3;
    // lane i of the group receives column i of the 4 rows.
    const int li = lane & 15, q = li >> 2, p = li & 3;
    const int k = kb + (lane >> 4) * 8 + q;
    const bf16raw* a0 = lds + k * TL::STRIDE + r0 + 4 * p;
    const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0));
    const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0 + 4 * TL::STRIDE));
    short8 u = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, u);
  }
}

// fp32 MFMA (16x16x4) operand: element [row r0+(lane&15)][k = kb + (lane>>4)]
template <bool KMAJ, int ROWS>
__device__ __forceinline__ float frag_f32(const float* lds, int r0, int kb, int lane) {
  using TL = Tile<float, KMAJ, ROWS>;
  if constexpr (!KMAJ) return lds[(r0 + (lane & 15)) * TL::STRIDE + kb + (lane >> 4)];
  else return lds[(kb + (lane >> 4)) * TL::STRIDE + r0 + (lane & 15)];
}

// Epilogue for 8 consecutive columns col0.. of output row `row` (batch z0, z1), fp32 sums in v:
// +bias; act 1: aux <- v, v = gelu(v); act 2: v *= gelu'(aux); +residual; store (beta: += beta*C_old).
template <typename T>
__device__ __forceinline__ void epilogue8(const dfk_gemm_args& g, int z0, int z1, int row, int col0, float (&v)[8],
                                          int evec) {
  const T* bias = g.bias ? reinterpret_cast<const T*>(g.bias) + z1 * g.bias_bs1 : nullptr;
  const T* res = g.residual ? reinterpret_cast<const T*>(g.residual) + z0 * g.rbs0 + z1 * g.rbs1 : nullptr;
  const long coff = z0 * g.cbs0 + z1 * g.cbs1;
  T* aux = g.aux ? reinterpret_cast<T*>(g.aux) + coff : nullptr;
  const bool full = evec && col0 + 8 <= g.N;
  // partial groups loop over all 8 slots with a predicate: a loop bounded by ncol would index v[] dynamically
  // and demote it (for every epilogue, full-vector path included) to scratch / LDS
  const int ncol = min(8, g.N - col0);
  if (bias) {
    if (full) { float b8[8]; ld8<T>(bias + col0, b8); for (int e = 0; e < 8; ++e) v[e] += b8[e]; }
    else for (int e = 0; e < 8; ++e) if (e < ncol) v[e] += ldf<T>(bias + col0 + e);
  }
  if (g.act == 1) {
    T* ap = aux ? aux + (long)row * g.ldaux + col0 : nullptr;
    if (ap) { if (full) st8<T>(ap, v); else for (int e = 0; e < 8; ++e) if (e < ncol) stf<T>(ap + e, v[e]); }
    if constexpr (sizeof(T) == 2) {
      for (int e = 0; e < 8; e += 2) {
        const f32x2 r = gelu_bf2(f32x2{v[e], v[e + 1]});
        v[e] = r.x;
        v[e + 1] = r.y;
      }
    } else {
      for (int e = 0; e < 8; ++e) v[e] = gelu_f(v[e]);
    }
  } else if (g.act == 2) {
    const T* ap = aux + (long)row * g.ldaux + col0;
    float a8[8];
    if (full) ld8<T>(ap, a8); else for (int e = 0; e < 8; ++e) if (e < ncol) a8[e] = ldf<T>(ap + e);
    if constexpr (sizeof(T) == 2) {
      for (int e = 0; e < 8; e += 2) {
        const f32x2 d = dgelu_bf2(f32x2{a8[e], a8[e + 1]});
        v[e] *= d.x;
        v[e + 1] *= d.y;
      }
    } else {
      for (int e = 0; e < 8; ++e) v[e] *= dgelu_f(a8[e]);
    }
  }
  if (g.drop.mode && g.drop.rng) {   // dropout / DropPath of the branch output (before the residual add)
    const DropCtx dc = drop_ctx(g.drop);
    const long rr = row + (long)(z0 * g.nz1 + z1) * g.M;
    if (dc.mode == 2) {
      const float m = drop_mul(dc, rr, 0);
      for (int e = 0; e < 8; ++e) v[e] *= m;
    } else {
      for (int e = 0; e < 8; ++e) v[e] *= drop_mul(dc, rr, col0 + e);
    }
  }
  if (g.alpha != 0.f && g.alpha != 1.f)   // Inception residual scale (0 reads as 1)
    for (int e = 0; e < 8; ++e) v[e] *= g.alpha;
  if (res) {
    const T* rp = res + (long)row * g.ldr + col0;
    if (full) { float r8[8]; ld8<T>(rp, r8); for (int e = 0; e < 8; ++e) v[e] += r8[e]; }
    else for (int e = 0; e < 8; ++e) if (e < ncol) v[e] += ldf<T>(rp + e);
  }
  if (g.act == 3)   // ReLU after the residual add
    for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  const long ci = coff + (long)row * g.ldc + col0;
  if (g.atomic) {
    float* C = reinterpret_cast<float*>(g.c) + ci;
    for (int e = 0; e < 8; ++e) if (e < ncol) atomicAdd(C + e, v[e]);
  } else if (g.c_f32) {
    float* C = reinterpret_cast<float*>(g.c) + ci;
    for (int e = 0; e < 8; ++e) if (e < ncol) C[e] = g.beta != 0.f ? v[e] + g.beta * C[e] : v[e];
  } else {
    T* C = reinterpret_cast<T*>(g.c) + ci;
    if (g.beta != 0.f) {
      if (full) { float c8v[8]; ld8<T>(C, c8v); for (int e = 0; e < 8; ++e) v[e] += g.beta * c8v[e]; }
      else for (int e = 0; e < 8; ++e) if (e < ncol) v[e] += g.beta * ldf<T>(C + e);
    }
    if (full) st8<T>(C, v);
    else for (int e = 0; e < 8; ++e) if (e < ncol) stf<T>(C + e, v[e]);
  }
}

template <typename T, int WT, bool MXO = false>
__device__ __forceinline__ void tile_epilogue(const dfk_gemm_args& g, float* smem, const f32x4 (&acc)[WT / 16][WT / 16],
                                              int lane, int wave, int wm, int wn, int bm, int bn, int z, int split,
                                              int tile, int evec, SplitK sk);
__device__ __forceinline__ int mx_scale_byte(float am);
__device__ __forceinline__ uint2 mx_pack8(const float (&v)[8], int e);

template <typename T, int WT, bool AK, bool BKM, bool VECOK, bool CONV, bool RS = false>
__global__ __launch_bounds__(256) void gemm_kernel(const dfk_gemm_args g, int kchunk, int evec, SplitK sk) {
  constexpr int BM = 2 * WT, BN = 2 * WT, MI = WT / 16;
  constexpr int VA = tile_vecs<T, BM>(), VB = tile_vecs<T, BN>();
  using TA = Tile<T, AK, BM>;
  using TB = Tile<T, BKM, BN>;
  constexpr int TBK = GT<T>::BK;
  constexpr int BUF = TA::ELEMS + TB::ELEMS;
  constexpr int ES = WT + 4;                      // epilogue staging row stride (fp32)
  constexpr int SMEM_T = 2 * BUF > (4 * WT * ES * 4) / (int)sizeof(T) ? 2 * BUF : (4 * WT * ES * 4) / (int)sizeof(T);
  __shared__ __attribute__((aligned(16))) T smem[SMEM_T];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order (blocks b and b+8 share an XCD's L2): consecutive remapped ids —
  // the N-tiles of one M-panel — land on one XCD and re-read A from its L2.
  int tn, tmi;
  {
    const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int nid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    tn = nid % gridDim.x;
    tmi = nid / gridDim.x;
  }
  const int bn = tn * BN, bm = tmi * BM;
  int z = blockIdx.z;
  const int split = z % g.splitk;
  z /= g.splitk;
  const int z0 = z / g.nz1, z1 = z % g.nz1;
  const T* A = reinterpret_cast<const T*>(g.a.ptr) + z0 * g.a.bs0 + z1 * g.a.bs1;
  const T* B = reinterpret_cast<const T*>(g.b.ptr) + z0 * g.b.bs0 + z1 * g.b.bs1;
  const int kbeg = split * kchunk;
  const int kend = min(g.K, kbeg + kchunk);

  f32x4 acc[MI][MI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused row sums of A (bias gradients): one wave column of the first N-tile multiplies A by ones
  const bool do_rs = RS && tn == 0 && wn == 0;   // RS: instantiated only for the dW (k-major x k-major) GEMM
  f32x4 accr[MI];
#pragma unroll
  for (int i = 0; i < MI; ++i) accr[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // register ring of PF staged k-tiles in flight (loads are unconditional: past kend they are masked
  // to zero by the view bounds), LDS double buffer: tile t is computed from LDS[t&1] while tile t+1
  // moves from its registers into LDS[(t+1)&1] and tile t+1+PF is requested into the freed registers.
#ifndef DFK_GEMM_PF64
#define DFK_GEMM_PF64 1
#endif
  constexpr int PF = WT == 32 ? 4 : DFK_GEMM_PF64;
  uint4 ra[PF][VA], rb[PF][VB];
  const int ntile = kend > kbeg ? (kend - kbeg + TBK - 1) / TBK : 0;
#pragma unroll
  for (int d = 0; d < PF; ++d) {
    const int kd = kbeg + max(0, min(d, ntile - 1)) * TBK;
    load_tile<T, AK, BM, VECOK, CONV>(A, g.a, bm, g.M, kd, kend, tid, ra[d]);
    load_tile<T, BKM, BN, VECOK, CONV>(B, g.b, bn, g.N, kd, kend, tid, rb[d]);
  }
  store_tile<T, AK, BM>(smem, tid, ra[0]);
  store_tile<T, BKM, BN>(smem + TA::ELEMS, tid, rb[0]);
  {
    const int kd = kbeg + max(0, min(PF, ntile - 1)) * TBK;
    load_tile<T, AK, BM, VECOK, CONV>(A, g.a, bm, g.M, kd, kend, tid, ra[0]);
    load_tile<T, BKM, BN, VECOK, CONV>(B, g.b, bn, g.N, kd, kend, tid, rb[0]);
  }
  __syncthreads();
  for (int t0 = 0; t0 < ntile; t0 += PF) {
#pragma unroll
    for (int d = 0; d < PF; ++d) {
      const int t = t0 + d;
      if (t >= ntile) break;
      const T* As = smem + (t & 1) * BUF;
      const T* Bs = As + TA::ELEMS;
      if constexpr (sizeof(T) == 2) {
#pragma unroll
        for (int ks = 0; ks < TBK / 32; ++ks) {
          bf16x8 af[MI], bfr[MI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) af[mi] = frag_bf16<AK, BM>(As, wm * WT + mi * 16, ks * 32, lane);
#pragma unroll
          for (int ni = 0; ni < MI; ++ni) bfr[ni] = frag_bf16<BKM, BN>(Bs, wn * WT + ni * 16, ks * 32, lane);
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
          if (RS && do_rs) {
            bf16x8 ones;
#pragma unroll
            for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) accr[mi] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], ones, accr[mi], 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < TBK / 4; ++ks) {
          float af[MI], bfr[MI];
#pragma unroll
          for (int mi = 0; mi < MI; ++mi) af[mi] = frag_f32<AK, BM>(As, wm * WT + mi * 16, ks * 4, lane);
#pragma unroll
          for (int ni = 0; ni < MI; ++ni) bfr[ni] = frag_f32<BKM, BN>(Bs, wn * WT + ni * 16, ks * 4, lane);
#pragma unroll
          for (int mi = 0; mi < MI; ++mi)
#pragma unroll
            for (int ni = 0; ni < MI; ++ni)
              acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
          if (RS && do_rs)
#pragma unroll
            for (int mi = 0; mi < MI; ++mi) accr[mi] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[mi], 1.0f, accr[mi], 0, 0, 0);
        }
      }
      const int nx = (d + 1) % PF;   // static after the full unroll
      if (PF == 1 && t + 1 >= ntile) break;   // single stage: no trailing re-request (uniform)
      store_tile<T, AK, BM>(smem + ((t + 1) & 1) * BUF, tid, ra[nx]);
      store_tile<T, BKM, BN>(smem + ((t + 1) & 1) * BUF + TA::ELEMS, tid, rb[nx]);
      __syncthreads();
      const int kn = kbeg + min(t + 1 + PF, ntile - 1) * TBK;   // past the end: re-request the last tile (L2 hit)
      load_tile<T, AK, BM, VECOK, CONV>(A, g.a, bm, g.M, kn, kend, tid, ra[nx]);
      load_tile<T, BKM, BN, VECOK, CONV>(B, g.b, bn, g.N, kn, kend, tid, rb[nx]);
    }
  }

  if (RS && do_rs && (lane & 15) == 0) {   // every column of A*ones is the row sum: lanes of column 0 publish it
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = bm + wm * WT + mi * 16 + (lane >> 4) * 4 + r;
        if (row < g.M) atomicAdd(g.rowsum + row, accr[mi][r]);
      }
  }
  __syncthreads();   // every wave is done reading the last k-tile before the staging overwrites it
  tile_epilogue<T, WT>(g, reinterpret_cast<float*>(smem), acc, lane, wave, wm, wn, bm, bn, z, split,
                       (z * (int)gridDim.y + tmi) * (int)gridDim.x + tn, evec, sk);
}

// Epilogue shared by the GEMM kernels: stage each wave's WT x WT fp32 tile through LDS (the 16x16 MFMA C/D
// layout is col = lane&15, row = (lane>>4)*4 + r), then every lane owns 8 consecutive columns of a row:
// 16-B loads of bias/residual/aux and 16-B stores.  The caller has passed a barrier after its last LDS read.
template <typename T, int WT, bool MXO>
__device__ __forceinline__ void tile_epilogue(const dfk_gemm_args& g, float* smem, const f32x4 (&acc)[WT / 16][WT / 16],
                                              int lane, int wave, int wm, int wn, int bm, int bn, int z, int split,
                                              int tile, int evec, SplitK sk) {
  constexpr int MI = WT / 16, ES = WT + 4;   // staging row stride (fp32)
  const int z0 = z / g.nz1, z1 = z % g.nz1;
  float* es = smem + wave * WT * ES;
#pragma unroll
  for (int mi = 0; mi < MI; ++mi)
#pragma unroll
    for (int ni = 0; ni < MI; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) es[(mi * 16 + (lane >> 4) * 4 + r) * ES + ni * 16 + (lane & 15)] = acc[mi][ni][r];
  __syncthreads();
  const T* bias = g.bias ? reinterpret_cast<const T*>(g.bias) + z1 * g.bias_bs1 : nullptr;
  const T* res = g.residual ? reinterpret_cast<const T*>(g.residual) + z0 * g.rbs0 + z1 * g.rbs1 : nullptr;
  const long coff = z0 * g.cbs0 + z1 * g.cbs1;
  T* aux = g.aux ? reinterpret_cast<T*>(g.aux) + coff : nullptr;
  if (sk.slab) {
    // split-K partial: raw fp32 sums to this split's slab, one row per wave instruction
    constexpr int RPI = 64 / WT;   // rows per wave instruction
    const int cl = lane % WT, col = bn + wn * WT + cl;
    const long MN = (long)g.M * g.N;
    float* S = sk.slab + (long)(z * g.splitk + split) * MN;
#pragma unroll 4
    for (int rl = lane / WT; rl < WT; rl += RPI) {
      const int row = bm + wm * WT + rl;
      if (row < g.M && col < g.N) S[(long)row * g.N + col] = es[rl * ES + cl];
    }
    if (!sk.cnt) return;   // splitk_reduce_kernel combines
    // in-launch combine: publish the slab (drain, barrier, one agent-scope release), draw a ticket; the tile's
    // last arriver acquires, sums the splits and runs the epilogue.  "Last" is broadcast through the kernel's one
    // LDS array (every wave has finished reading its staging tile at the barrier).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint32_t t = __hip_atomic_fetch_add(sk.cnt + tile, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const bool last = t == (uint32_t)(g.splitk - 1);
      if (last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(sk.cnt + tile, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // the slice's next use
      }
      smem[0] = last ? 1.f : 0.f;
    }
    __syncthreads();
    if (smem[0] == 0.f) return;
    // splits summed in split order (as splitk_reduce_kernel), 8 columns per lane of this wave's WT x WT part
    constexpr int CPR = WT / 8;
    const float* S0 = sk.slab + (long)z * g.splitk * MN;
    for (int it = lane; it < WT * CPR; it += 64) {
      const int row = bm + wm * WT + it / CPR, col0 = bn + wn * WT + (it % CPR) * 8;
      if (row >= g.M || col0 >= g.N) continue;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      const int ncol = min(8, g.N - col0);
      const bool vec = (g.N % 4) == 0 && ncol == 8;
      const float* src = S0 + (long)row * g.N + col0;
      for (int sidx = 0; sidx < g.splitk; ++sidx, src += MN) {
        if (vec) {
          const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
          v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
          v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
        } else {
          for (int e = 0; e < 8; ++e) if (e < ncol) v[e] += src[e];
        }
      }
      epilogue8<T>(g, z0, z1, row, col0, v, evec);
    }
    return;
  }
  if (g.atomic || g.c_f32) {
    // fp32 output (weight gradients): one row per wave instruction = 256 contiguous bytes
    constexpr int RPI = 64 / WT;
    const int cl = lane % WT, col = bn + wn * WT + cl;
    float* Cb = reinterpret_cast<float*>(g.c) + coff;
#pragma unroll 4
    for (int rl = lane / WT; rl < WT; rl += RPI) {
      const int row = bm + wm * WT + rl;
      if (row >= g.M || col >= g.N) continue;
      float v = es[rl * ES + cl];
      if (bias) v += ldf<T>(bias + col);
      if (res) v += ldf<T>(res + (long)row * g.ldr + col);
      float* C = Cb + (long)row * g.ldc + col;
      if (g.atomic) atomicAdd(C, v);
      else *C = g.beta != 0.f ? v + g.beta * *C : v;
    }
    return;
  }
  constexpr int CPR = WT / 8, RPP = 64 / CPR;   // lanes per row (8 columns each), rows per pass
  const int c8 = (lane % CPR) * 8;
  const int col0 = bn + wn * WT + c8;
#pragma unroll 1
  for (int pass = 0; pass < WT / RPP; ++pass) {
    const int rl = pass * RPP + lane / CPR;
    const int row = bm + wm * WT + rl;
    if constexpr (MXO) {
      // MX copy of the stored bf16 C along N: lanes 4q..4q+3 hold the 32 columns of one block of this row
      const bool ok = row < g.M && col0 < g.N;
      float v[8];
      *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(es + rl * ES + c8);
      *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(es + rl * ES + c8 + 4);
      if (ok) epilogue8<T>(g, z0, z1, row, col0, v, evec);
      float am = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[e] = ok ? bf2f(f2bf(v[e])) : 0.f;
        am = fmaxf(am, fabsf(v[e]));
      }
      am = fmaxf(am, __shfl_xor(am, 1, 64));
      am = fmaxf(am, __shfl_xor(am, 2, 64));
      const int eb = mx_scale_byte(am);
      const uint2 w = mx_pack8(v, eb);
      if (ok) {
        *reinterpret_cast<uint2*>(g.mx_q + (long)row * g.mx_ldq + col0) = w;
        if ((lane & 3) == 0)
          reinterpret_cast<uint8_t*>(g.mx_s)[((long)(col0 >> 7) * g.mx_lds + row) * 4 + ((col0 & 127) >> 5)] = (uint8_t)eb;
      }
    } else {
      if (row >= g.M || col0 >= g.N) continue;
      float v[8];
      *reinterpret_cast<float4*>(v) = *reinterpret_cast<const float4*>(es + rl * ES + c8);
      *reinterpret_cast<float4*>(v + 4) = *reinterpret_cast<const float4*>(es + rl * ES + c8 + 4);
      epilogue8<T>(g, z0, z1, row, col0, v, evec);
    }
  }
}

// ---------------------------------------------------------------------------------------------------
// LDS-DMA GEMM (bf16, plain views, 16-B aligned extents): the operand tiles go HBM -> LDS by
// buffer_load_dwordx4 ... lds (16 B per lane, lane-linear 1 KB per wave-instruction) with no VGPR
// staging and no ds_write pass — on gfx950 the register-staged ds_write_b128 (~79 B/clk/CU) costs more
// LDS cycles per k-tile than the fragment reads, so the register-staged kernel above is LDS-bound
// before it is MFMA-bound.  The swizzle lives on the SOURCE address (the LDS image stays lane-linear):
//   k-contiguous operand: image [ROWS][64] (128-B rows), 16-B chunk c of row r stored at c ^ ((r>>1)&7)
//                         -> the ds_read_b128 fragment reads are conflict-free;
//   k-major operand     : image [64][ROWS] (k rows), chunk c of k-row k stored at c ^ kmaj_swz(k)
//                         -> the ds_read_b64_tr_b16 transposed reads are conflict-free
// (screened against the LDS lane-group/bank model of the microarchitecture guide).  Out-of-range chunks
// (rows past M/N, k past the split's end) get a voffset past the descriptor's range: the hardware
// returns zeros, so the loop has no branches around loads.  S LDS stages: tile t+S-1 is requested
// right after the barrier that retires tile t, one raw s_barrier per k-tile, counted vmcnt waits
// (an LDS-DMA is a VM-counter load; __syncthreads() would drain it with vmcnt(0)).
typedef __attribute__((address_space(3))) void lds_void;

template <int ROWS>
__device__ __forceinline__ int kmaj_swz(int k) {   // 16-B chunk XOR of k-row k in a [64][ROWS] bf16 image
  // (ROWS = 256: a k-row spans two bank rows; the XOR stays below 16, the same bank pattern as 128)
  if constexpr (ROWS >= 128) return ((k & 3) | ((k >> 1) & 4)) << 1;
  else return (((k >> 1) & 1) | ((k >> 2) & 2)) << 1;
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// One operand's DMA for k-tile k0: NI wave-instructions per wave, each 64 lanes x 16 B into 1 KB of the
// image.  Offsets are recomputed per call in 32-bit arithmetic (the host keeps every operand below 2 GB):
// per-lane arrays of them were demoted to scratch / LDS by the compiler.
template <bool KM, int ROWS, int NWV, bool CONV>
struct Dma {
  static constexpr int NI = ROWS / (8 * NWV);   // ROWS x 64 bf16 = ROWS/8 KB per tile over NWV waves
  __device__ static __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, const dfk_view& v, int row0, int rowlim,
                                               int k0, int kend, bf16raw* img, int wave, int lane) {
    const uint32_t ld = (uint32_t)v.ld;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int sl = (wave * NI + i) * 64 + lane;   // 16-B slot of the tile image
      int vr, vc;                                   // view row / first view column of the lane's 8 elements
      bool in;
      if constexpr (!KM) {
        const int r = sl >> 3, c = (sl & 7) ^ ((r >> 1) & 7);
        vr = row0 + r;
        vc = k0 + c * 8;
        in = vr < rowlim && vc < kend;
      } else {
        constexpr int CPR = ROWS / 8;
        const int k = sl / CPR, c = (sl % CPR) ^ kmaj_swz<ROWS>(k);
        vr = k0 + k;
        vc = row0 + c * 8;
        in = vc < rowlim && vr < kend;
      }
      uint32_t off = ((uint32_t)vr * ld + (uint32_t)vc) * 2u;
      if constexpr (CONV) {   // implicit-conv view: column vc = tap * cg + channel of input row vr*stride + tap - pad
        if (v.conv_cg > 0) {
          const int tap = vc / v.conv_cg;
          const int sr = vr * v.conv_stride + tap - v.conv_pad;
          in = in && sr >= 0 && sr < v.conv_rows;
          off = ((uint32_t)sr * ld + (uint32_t)(vc - tap * v.conv_cg)) * 2u;
        }
      }
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wave * NI + i) * 512), 16,
                                               in ? off : 0x80000000u, 0, 0, 0);
    }
  }
};

// MFMA fragment (8 consecutive k of tile row r0 + (lane&15)) from a DMA-filled image
template <bool KM, int ROWS>
__device__ __forceinline__ bf16x8 frag_dma(const bf16raw* img, int r0, int kb, int lane) {
  if constexpr (!KM) {
    const int r = r0 + (lane & 15), c = (kb >> 3) + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * 64 + ((c ^ ((r >> 1) & 7)) << 3));
  } else {
    const int li = lane & 15, q = li >> 2, p = li & 3;
    const int k = kb + (lane >> 4) * 8 + q, c = (r0 >> 3) + (p >> 1);
    const bf16raw* lo = img + k * ROWS + ((c ^ kmaj_swz<ROWS>(k)) << 3) + (p & 1) * 4;
    const bf16raw* hi = img + (k + 4) * ROWS + ((c ^ kmaj_swz<ROWS>(k + 4)) << 3) + (p & 1) * 4;
    const short4v a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(lo));
    const short4v b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(hi));
    short8 u = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return __builtin_bit_cast(bf16x8, u);
  }
}

// bytes a view can touch (the buffer descriptor's range): rows x cols, or an implicit-conv view's input rows
__host__ __device__ __forceinline__ long view_extent(const dfk_view& v, long rows, long cols) {
  if (v.conv_cg > 0) return ((long)(v.conv_rows - 1) * v.ld + v.conv_cg) * 2;
  return ((rows - 1) * v.ld + cols) * 2;
}

// Workgroup tile (NWM * 64/... ) = BM x BN from NWM x NWN waves of WT x WT each: 64x64 (2x2 waves of 32),
// 128x128 (2x2 waves of 64) and 256x128 (4x2 waves of 64, 512 threads: twice the MFMA work per k-tile for
// 1.5x the staged bytes, so one DMA in flight covers more of its latency).
// splits from which a dW's fused bias gradient goes through per-split partials + rowsum_reduce_kernel instead of
// atomics (the same-address atomics serialise only when many splits add; below this, one more launch costs more)
constexpr int kRsPartialMin = 32;

template <int WT, int NWM, int NWN, bool AK, bool BKM, int S, bool RS, bool CONV = false>
__global__ __launch_bounds__(NWM * NWN * 64) void gemm_dma_kernel(const dfk_gemm_args g, int kchunk, int evec,
                                                                  SplitK sk) {
  constexpr int NWV = NWM * NWN, BM = NWM * WT, BN = NWN * WT, MI = WT / 16, BK = 64;
  constexpr int STAGE = (BM + BN) * BK;                         // elements per LDS stage
  constexpr int ES = WT + 4;
  constexpr int SMEM = S * STAGE * 2 > NWV * WT * ES * 4 ? S * STAGE * 2 : NWV * WT * ES * 4;   // bytes
  constexpr int LPT = Dma<AK, BM, NWV, CONV>::NI + Dma<BKM, BN, NWV, CONV>::NI;   // DMA instructions per wave per tile
  __shared__ __attribute__((aligned(16))) float smem_f[SMEM / 4];   // the ONE LDS object (staging + epilogue)
  bf16raw* smem = reinterpret_cast<bf16raw*>(smem_f);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  int tn, tmi, z;
  const int nwg = gridDim.x * gridDim.y;
  if (g.atomic && g.splitk % 8 == 0 && (int)gridDim.z == g.splitk && nwg > 1) {
    // atomic split-K weight gradients: all nwg output tiles of one split on one XCD (the dispatcher deals
    // workgroups of the linear order to the 8 XCDs round robin), so the token range of the operand every tile
    // of that split reads (x: the whole narrow dW row block) comes from that XCD's L2 after the first tile
    const int lin = blockIdx.z * nwg + blockIdx.y * gridDim.x + blockIdx.x;
    const int j = lin >> 3, i = j % nwg;
    z = (j / nwg) * 8 + (lin & 7);
    tn = i % gridDim.x;
    tmi = i / gridDim.x;
  } else {
    const int bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int nid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    tn = nid % gridDim.x;
    tmi = nid / gridDim.x;
    z = blockIdx.z;
  }
  const int bn = tn * BN, bm = tmi * BM;
  const int split = z % g.splitk;
  z /= g.splitk;
  const int z0 = z / g.nz1, z1 = z % g.nz1;
  const bf16raw* A = reinterpret_cast<const bf16raw*>(g.a.ptr) + z0 * g.a.bs0 + z1 * g.a.bs1;
  const bf16raw* B = reinterpret_cast<const bf16raw*>(g.b.ptr) + z0 * g.b.bs0 + z1 * g.b.bs1;
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16raw*>(A), (short)0, (int)(AK ? view_extent(g.a, g.K, g.M) : view_extent(g.a, g.M, g.K)), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16raw*>(B), (short)0, (int)(BKM ? view_extent(g.b, g.K, g.N) : view_extent(g.b, g.N, g.K)), 0x00020000);
  const int kbeg = split * kchunk;
  const int kend = min(g.K, kbeg + kchunk);
  const int ntile = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;

  auto issue = [&](int kt, bf16raw* st) {
    Dma<AK, BM, NWV, CONV>::issue(ra, g.a, bm, g.M, kt, kend, st, wave, lane);
    Dma<BKM, BN, NWV, CONV>::issue(rb, g.b, bn, g.N, kt, kend, st + BM * BK, wave, lane);
  };

  f32x4 acc[MI][MI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // fused row sums of A (bias gradients) in the first column of tiles, shared by the wave columns: wave column wn
  // takes fragments mi = h NWN + wn (one wave column doing all of them held every k-tile's barrier for its extra
  // MFMAs: stage-1 dW + db 120 -> 137 us)
  constexpr int MH = (MI + NWN - 1) / NWN;
  const bool do_rs = RS && tn == 0;
  f32x4 accr[MH];
#pragma unroll
  for (int i = 0; i < MH; ++i) accr[i] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int d = 0; d < S - 1; ++d)
    if (d < ntile) {
      issue(kbeg + d * BK, smem + d * STAGE);
    }
  for (int t = 0; t < ntile; ++t) {
    // retire tile t: S-2 later tiles may stay in flight (fewer near the end)
    if constexpr (S == 4) {
      if (t + 2 < ntile) wait_vm<2 * LPT>(); else if (t + 1 < ntile) wait_vm<LPT>(); else wait_vm<0>();
    } else if constexpr (S == 3) {
      if (t + 1 < ntile) wait_vm<LPT>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // this wave's reads of tile t-1 are complete
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + S - 1 < ntile) {   // refill the stage every wave finished reading at t-1
      issue(kbeg + (t + S - 1) * BK, smem + ((t + S - 1) % S) * STAGE);
    }
    const bf16raw* As = smem + (t % S) * STAGE;
    const bf16raw* Bs = As + BM * BK;
#pragma unroll
    for (int ks = 0; ks < BK / 32; ++ks) {
      bf16x8 af[MI], bfr[MI];
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) af[mi] = frag_dma<AK, BM>(As, wm * WT + mi * 16, ks * 32, lane);
#pragma unroll
      for (int ni = 0; ni < MI; ++ni) bfr[ni] = frag_dma<BKM, BN>(Bs, wn * WT + ni * 16, ks * 32, lane);
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < MI; ++ni)
          acc[mi][ni] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0);
      if (RS && do_rs) {
        bf16x8 ones;
#pragma unroll
        for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
        for (int h = 0; h < MH; ++h) {
          bf16x8 a = af[h * NWN < MI ? h * NWN : MI - 1];
#pragma unroll
          for (int c = 1; c < NWN; ++c)
            if (wn == c && h * NWN + c < MI) a = af[h * NWN + c];
          accr[h] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, ones, accr[h], 0, 0, 0);
        }
      }
    }
  }
  if (RS && do_rs && (lane & 15) == 0) {
    // atomic split-K (the workspace holds [splitk][M] partials): one plain store per (split, row), summed by
    // rowsum_reduce_kernel — the splits' same-address atomics on the few cache lines of the bias gradient
    // serialised (stage-1 dW + db 120 -> 137 us, proj 41 -> 66 us)
    float* rsp = g.splitk >= kRsPartialMin && g.ws
                     ? reinterpret_cast<float*>(g.ws) + (g.atomic ? 0L : (long)g.splitk * g.M * g.N) + (long)split * g.M
                     : nullptr;
#pragma unroll
    for (int h = 0; h < MH; ++h) {
      const int mi = h * NWN + wn;
      if (mi < MI)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = bm + wm * WT + mi * 16 + (lane >> 4) * 4 + r;
          if (row < g.M) {
            if (rsp) rsp[row] = accr[h][r];
            else atomicAdd(g.rowsum + row, accr[h][r]);
          }
        }
    }
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  tile_epilogue<bf16raw, WT>(g, smem_f, acc, lane, wave, wm, wn, bm, bn, z, split,
                             (z * (int)gridDim.y + tmi) * (int)gridDim.x + tn, evec, sk);
}

// rowsum[row] += sum over splits of part[split][row] (the bias gradient of an atomic split-K dW, fixed order):
// 64 rows per workgroup, 16 split phases (each thread sums every 16th split, 4 loads in flight), folded in LDS
__global__ __launch_bounds__(1024) void rowsum_reduce_kernel(const float* __restrict__ part, int splitk, int M,
                                                             float* __restrict__ rowsum) {
  __shared__ float red[16][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const int row = blockIdx.x * 64 + c;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (row < M) {
    int sp = ph;
    for (; sp + 48 < splitk; sp += 64)
#pragma unroll
      for (int u = 0; u < 4; ++u) a[u] += part[(long)(sp + 16 * u) * M + row];
    for (; sp < splitk; sp += 16) a[0] += part[(long)sp * M + row];
  }
  red[ph][c] = (a[0] + a[1]) + (a[2] + a[3]);
  __syncthreads();
  if (ph == 0 && row < M) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += red[i][c];
    rowsum[row] += t;
  }
}

// fp32 C (+)= the sum of many split slabs (the weight gradients' split-K when not atomic): 64 threads x 4
// columns per workgroup row segment, 8 split phases (each thread sums every 8th split), folded in LDS
__global__ __launch_bounds__(512) void slab_sum_f32_kernel(const dfk_gemm_args g, const float* __restrict__ slab,
                                                           int splitk) {
  __shared__ f32x4 red[8][64];
  const int c = threadIdx.x & 63, ph = threadIdx.x >> 6;
  const long MN = (long)g.M * g.N;
  const long i = ((long)blockIdx.x * 64 + c) * 4;   // element index in [M][N] (N % 4 == 0)
  f32x4 a = {0.f, 0.f, 0.f, 0.f}, b2 = {0.f, 0.f, 0.f, 0.f};
  if (i < MN) {
    int sp = ph;
    for (; sp + 8 < splitk; sp += 16) {
      a += *reinterpret_cast<const f32x4*>(slab + (long)sp * MN + i);
      b2 += *reinterpret_cast<const f32x4*>(slab + (long)(sp + 8) * MN + i);
    }
    if (sp < splitk) a += *reinterpret_cast<const f32x4*>(slab + (long)sp * MN + i);
  }
  red[ph][c] = a + b2;
  __syncthreads();
  if (ph == 0 && i < MN) {
    f32x4 t = red[0][c];
#pragma unroll
    for (int k = 1; k < 8; ++k) t += red[k][c];
    const long row = i / g.N, col = i % g.N;
    float* C = reinterpret_cast<float*>(g.c) + row * g.ldc + col;
#pragma unroll
    for (int e = 0; e < 4; ++e) C[e] = g.beta != 0.f ? t[e] + g.beta * C[e] : t[e];
  }
}

// split-K slabs [z][split][M][N] fp32 -> sum -> epilogue (8 columns per thread)
template <typename T>
__global__ __launch_bounds__(256) void splitk_reduce_kernel(const dfk_gemm_args g, const float* __restrict__ slab,
                                                            int splitk, int evec) {
  const int cg = (g.N + 7) / 8;
  const long idx = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long per_z = (long)g.M * cg;
  const int z = (int)(idx / per_z);
  if (z >= g.nz0 * g.nz1) return;
  const long rem = idx - (long)z * per_z;
  const int row = (int)(rem / cg), col0 = (int)(rem % cg) * 8;
  const long MN = (long)g.M * g.N;
  const float* src = slab + (long)z * splitk * MN + (long)row * g.N + col0;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int ncol = min(8, g.N - col0);
  const bool vec = (g.N % 4) == 0 && ncol == 8;
  for (int sidx = 0; sidx < splitk; ++sidx, src += MN) {
    if (vec) {
      const float4 x0 = *reinterpret_cast<const float4*>(src), x1 = *reinterpret_cast<const float4*>(src + 4);
      v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
      v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
    } else {
      for (int e = 0; e < 8; ++e) if (e < ncol) v[e] += src[e];
    }
  }
  epilogue8<T>(g, z / g.nz1, z % g.nz1, row, col0, v, evec);
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

// 16-byte vector loads are legal for this view (else the element-wise instantiation runs)
bool view_vec(const dfk_view& v, int vec) {
  if (v.ld % vec || v.bs0 % vec || v.bs1 % vec) return false;
  if ((reinterpret_cast<uintptr_t>(v.ptr) & 15) != 0) return false;
  if (v.conv_cg > 0 && v.conv_cg % vec) return false;
  return true;
}

template <typename T, int WT, bool VECOK, bool CONV>
void dispatch_wt(const dfk_gemm_args& g, dim3 grid, int kchunk, int evec, SplitK sk, hipStream_t s) {
  if (g.a_kmajor) {
    if (g.b_kmajor) {
      if (g.rowsum) hipLaunchKernelGGL((gemm_kernel<T, WT, true, true, VECOK, CONV, true>), grid, dim3(NT), 0, s, g, kchunk, evec, sk);
      else hipLaunchKernelGGL((gemm_kernel<T, WT, true, true, VECOK, CONV>), grid, dim3(NT), 0, s, g, kchunk, evec, sk);
    }
    else hipLaunchKernelGGL((gemm_kernel<T, WT, true, false, VECOK, CONV>), grid, dim3(NT), 0, s, g, kchunk, evec, sk);
  } else {
    if (g.b_kmajor) hipLaunchKernelGGL((gemm_kernel<T, WT, false, true, VECOK, CONV>), grid, dim3(NT), 0, s, g, kchunk, evec, sk);
    else hipLaunchKernelGGL((gemm_kernel<T, WT, false, false, VECOK, CONV>), grid, dim3(NT), 0, s, g, kchunk, evec, sk);
  }
}

// implicit-conv views (wav2vec2 conv1-6 and their weight gradients): 2 LDS stages, 64x64 / 128x128 tiles
template <int WT>
void dispatch_dma_conv(const dfk_gemm_args& g, dim3 grid, int kchunk, int evec, SplitK sk, hipStream_t s) {
  const dim3 blk(256);
  if (g.a_kmajor) {
    if (g.b_kmajor) {
      if (g.rowsum) hipLaunchKernelGGL((gemm_dma_kernel<WT, 2, 2, true, true, 2, true, true>), grid, blk, 0, s, g, kchunk, evec, sk);
      else hipLaunchKernelGGL((gemm_dma_kernel<WT, 2, 2, true, true, 2, false, true>), grid, blk, 0, s, g, kchunk, evec, sk);
    }
    else hipLaunchKernelGGL((gemm_dma_kernel<WT, 2, 2, true, false, 2, false, true>), grid, blk, 0, s, g, kchunk, evec, sk);
  } else {
    if (g.b_kmajor) hipLaunchKernelGGL((gemm_dma_kernel<WT, 2, 2, false, true, 2, false, true>), grid, blk, 0, s, g, kchunk, evec, sk);
    else hipLaunchKernelGGL((gemm_dma_kernel<WT, 2, 2, false, false, 2, false, true>), grid, blk, 0, s, g, kchunk, evec, sk);
  }
}

template <int WT, int NWM, int NWN, int S>
void dispatch_dma_s(const dfk_gemm_args& g, dim3 grid, int kchunk, int evec, SplitK sk, hipStream_t s) {
  const dim3 blk(NWM * NWN * 64);
  if (g.a_kmajor) {
    if (g.b_kmajor) {
      if (g.rowsum) hipLaunchKernelGGL((gemm_dma_kernel<WT, NWM, NWN, true, true, S, true>), grid, blk, 0, s, g, kchunk, evec, sk);
      else hipLaunchKernelGGL((gemm_dma_kernel<WT, NWM, NWN, true, true, S, false>), grid, blk, 0, s, g, kchunk, evec, sk);
    }
    else hipLaunchKernelGGL((gemm_dma_kernel<WT, NWM, NWN, true, false, S, false>), grid, blk, 0, s, g, kchunk, evec, sk);
  } else {
    if (g.b_kmajor) hipLaunchKernelGGL((gemm_dma_kernel<WT, NWM, NWN, false, true, S, false>), grid, blk, 0, s, g, kchunk, evec, sk);
    else hipLaunchKernelGGL((gemm_dma_kernel<WT, NWM, NWN, false, false, S, false>), grid, blk, 0, s, g, kchunk, evec, sk);
  }
}

// LDS-DMA kernel stages (tuning runs may override): 2 for both tile sizes (C2 sweep: occupancy hides the
// DMA latency better than a deeper ring; 128x128: 69 KB -> two workgroups per CU)
int dma_stages(int wt) {
  static const int s128 = getenv("DFK_DMA_S128") ? atoi(getenv("DFK_DMA_S128")) : 2;
  if (wt == 128) return s128;
  static const int s64 = getenv("DFK_DMA_S64") ? atoi(getenv("DFK_DMA_S64")) : 2;
  static const int s32 = getenv("DFK_DMA_S32") ? atoi(getenv("DFK_DMA_S32")) : 2;
  return wt == 64 ? s64 : s32;
}

// wt: 32 -> 64x64 tiles, 64 -> 128x128, 128 -> 256x128 (8 waves)
void dispatch_dma(const dfk_gemm_args& g, int wt, dim3 grid, int kchunk, int evec, SplitK sk, hipStream_t s) {
  if (g.a.conv_cg > 0 || g.b.conv_cg > 0) {
    if (wt == 32) dispatch_dma_conv<32>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_conv<64>(g, grid, kchunk, evec, sk, s);
    return;
  }
  // weight gradients (k-major A: the token dimension is the reduction) on 128x128 tiles: tuning knob for their ring
  // depth (3 stages measured slower: dW 116 -> 119 us, C2 256.8 -> 247.7 clips/s, profiles/gemm/r4sdw_*)
  static const int sdw = getenv("DFK_DMA_SDW") ? atoi(getenv("DFK_DMA_SDW")) : 2;
  static const int sdw32 = getenv("DFK_DMA_SDW32") ? atoi(getenv("DFK_DMA_SDW32")) : 2;   // their 64x64 tiles (A/B)
  const int st = g.a_kmajor && wt == 64 ? sdw : (g.a_kmajor && wt == 32 ? sdw32 : dma_stages(wt));
  static const int s8w = getenv("DFK_DMA_S8W") ? atoi(getenv("DFK_DMA_S8W")) : 2;   // A/B: ring depth of the 8-wave tiles
  if (wt == 33) {   // 128 x 64 (8 waves of 32 x 32)
    if (s8w == 3) dispatch_dma_s<32, 4, 2, 3>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_s<32, 4, 2, 2>(g, grid, kchunk, evec, sk, s);
    return;
  }
  if (wt == 34) {   // 64 x 128
    if (s8w == 3) dispatch_dma_s<32, 2, 4, 3>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_s<32, 2, 4, 2>(g, grid, kchunk, evec, sk, s);
    return;
  }
  if (wt == 128) {
    if (st == 3) dispatch_dma_s<64, 4, 2, 3>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_s<64, 4, 2, 2>(g, grid, kchunk, evec, sk, s);
  } else if (wt == 64) {
    if (st == 2) dispatch_dma_s<64, 2, 2, 2>(g, grid, kchunk, evec, sk, s);
    else if (st == 4) dispatch_dma_s<64, 2, 2, 4>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_s<64, 2, 2, 3>(g, grid, kchunk, evec, sk, s);
  } else {
    if (st == 2) dispatch_dma_s<32, 2, 2, 2>(g, grid, kchunk, evec, sk, s);
    else if (st == 4) dispatch_dma_s<32, 2, 2, 4>(g, grid, kchunk, evec, sk, s);
    else dispatch_dma_s<32, 2, 2, 3>(g, grid, kchunk, evec, sk, s);
  }
}

// the LDS-DMA kernel addresses each operand through a buffer descriptor with 32-bit byte offsets
bool dma_ok(const dfk_gemm_args& g) {
  static const int off = getenv("DFK_GEMM_DMA") ? atoi(getenv("DFK_GEMM_DMA")) == 0 : 0;   // A/B runs only
  if (off || g.dtype != DFK_BF16) return false;
  const long ea = g.a_kmajor ? view_extent(g.a, g.K, g.M) : view_extent(g.a, g.M, g.K);
  const long eb = g.b_kmajor ? view_extent(g.b, g.K, g.N) : view_extent(g.b, g.N, g.K);
  return ea < 0x7fffffffL && eb < 0x7fffffffL;
}

template <typename T, bool VECOK, bool CONV>
void dispatch(const dfk_gemm_args& g, int wt, dim3 grid, int kchunk, int evec, SplitK sk, hipStream_t s) {
  if (wt == 32) dispatch_wt<T, 32, VECOK, CONV>(g, grid, kchunk, evec, sk, s);
  else dispatch_wt<T, 64, VECOK, CONV>(g, grid, kchunk, evec, sk, s);
}

// wave tile: 64 (128 x 128 workgroup tiles) unless that grid has fewer than eight tiles per CU: then 32
// (64 x 64 tiles, four times the workgroups, half the LDS, a 4-deep register ring of k-tiles in flight)
int pick_wt(const dfk_gemm_args& g) {
  // caller-planned split-K grids (weight gradients): 128x128 tiles (A/B knob DFK_DW_WT=32: 64x64 tiles, whose
  // smaller LDS stages let three workgroups per CU keep more bytes in flight)
  static const int dw_wt = getenv("DFK_DW_WT") ? atoi(getenv("DFK_DW_WT")) : 64;
  if (g.atomic || g.splitk > 1) return dw_wt == 32 ? 32 : 64;
  static const int force = getenv("DFK_GEMM_WT") ? atoi(getenv("DFK_GEMM_WT")) : 0;   // tuning runs only
  if (force == 32 || force == 64) return force;
  // measured on the C2 Linear shapes (tools/gemm_bench.py, both tile shapes): below 2048 128x128 tiles (eight
  // per CU) the 64x64 tiles with the k-tile ring win or tie at every K (e.g. [25088,1536]x[1536,384] 98 -> 73
  // us, [6272,3072]x[3072,768] 86 -> 77 us), above it the 128x128 tiles win
  const long tiles128 = (long)dfk_cdiv(g.N, 128) * dfk_cdiv(g.M, 128) * g.nz0 * g.nz1;
  // LDS-DMA kernel (below): 128x128 tiles from 1024 of them (C2 sweep: [6272,768]x[768,3072] 74 -> 58 us,
  // the M ~ 1.6k wav2vec2 / SwinV2-stage-3 shapes stay faster on 64x64 tiles)
  if (dma_ok(g)) return tiles128 < 1024 ? 32 : 64;
  return tiles128 < 2048 ? 32 : 64;
}

// automatic K split for grids that cannot fill the chip (caller asked for no split, no atomics)
template <typename T>
int auto_splitk(const dfk_gemm_args& g) {
  constexpr int TBK = GT<T>::BK;
  if (g.atomic || g.splitk != 1 || g.M <= 0 || g.N <= 0) return 1;
  const int wt = pick_wt(g);
  const long tiles = (long)dfk_cdiv(g.N, 2 * wt) * dfk_cdiv(g.M, 2 * wt) * g.nz0 * g.nz1;
  if (tiles >= 384) return 1;
  static const int nosplit = getenv("DFK_GEMM_NOSPLIT") ? atoi(getenv("DFK_GEMM_NOSPLIT")) : 0;   // tuning runs only
  if (nosplit) return 1;
  // at least 12 k-tiles per split: below that the fp32 slab round trip and the reduce launch cost more than
  // the shorter k-loop saves (C2 sweep of the LDS-DMA kernel: K = 512-2048 run fastest unsplit, K >= 2304
  // with 3-4 splits)
  const int maxs = g.K / (12 * TBK);
  static const int target = getenv("DFK_GEMM_SPLIT_TARGET") ? atoi(getenv("DFK_GEMM_SPLIT_TARGET")) : 768;   // tuning runs only
  const int want = (int)dfk_cdiv(target, tiles);
  return std::max(1, std::min(maxs, want));
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }


template <typename T>
int launch(const dfk_gemm_args& g, hipStream_t s) {
  constexpr int VEC = GT<T>::VEC, TBK = GT<T>::BK;
  if (!g.a.ptr || !g.b.ptr || !g.c) return DFK_EINVAL;
  if ((g.a.conv_cg > 0 && g.a.conv_stride <= 0) || (g.b.conv_cg > 0 && g.b.conv_stride <= 0)) return DFK_EINVAL;
  if (g.splitk < 1 || g.nz0 < 1 || g.nz1 < 1) return DFK_EINVAL;
  if (g.splitk > 1 && !g.atomic && !g.ws) return DFK_EINVAL;   // explicit split-K: fp32 slabs in ws
  if (g.atomic && (!g.c_f32 || g.bias || g.residual || g.act)) return DFK_EINVAL;
  if (g.act == 2 && !g.aux) return DFK_EINVAL;
  if (g.act < 0 || g.act > 3 || (g.act == 3 && (g.c_f32 || g.atomic))) return DFK_EINVAL;
  if (g.rowsum && (g.nz0 != 1 || g.nz1 != 1 || !g.a_kmajor || !g.b_kmajor)) return DFK_EINVAL;
  if (g.drop.mode && (g.c_f32 || g.atomic || !g.drop.rng || !(g.drop.p >= 0.f && g.drop.p < 1.f))) return DFK_EINVAL;
  if (g.M <= 0 || g.N <= 0) return 0;
  if constexpr (sizeof(T) == 2) {
    const int w = dfk_wres_try(g, s);     // huge-M / small-weight Linears: weight-resident streaming kernel
    if (w != 0) return w > 0 ? 0 : w;
    const int d = dfk_wgrad_try(g, s);    // their weight gradients: token-streaming, output slice in registers
    if (d != 0) return d > 0 ? 0 : d;
  }
  // split-K through fp32 slabs + a reduce/epilogue kernel: caller-chosen (splitk > 1, no atomics) or
  // automatic for grids too small to fill the chip
  const int autos = g.splitk > 1 && !g.atomic ? g.splitk : (g.ws ? auto_splitk<T>(g) : 1);
  dfk_gemm_args gg = g;
  if (autos > 1) gg.splitk = autos;
  int kchunk = dfk_cdiv(g.K, gg.splitk);
  kchunk = dfk_cdiv(kchunk, TBK) * TBK;
  int wt = pick_wt(g);
  const bool dma = sizeof(T) == 2 && dma_ok(g);
  const bool conv = g.a.conv_cg > 0 || g.b.conv_cg > 0;
  // vector path also needs the contiguous extents to be whole vectors (else tails load element-wise)
  const bool vec = view_vec(g.a, VEC) && view_vec(g.b, VEC) && (g.a_kmajor ? g.M : g.K) % VEC == 0 &&
                   (g.b_kmajor ? g.N : g.K) % VEC == 0;
  if (dma && vec && wt == 64 && !conv) {   // 256x128 tiles (8 waves) when the grid still covers the chip (tuning knob for now)
    static const long t256 = getenv("DFK_GEMM_T256") ? atol(getenv("DFK_GEMM_T256")) : (1L << 40);
    const long tiles256 = (long)dfk_cdiv(g.N, 128) * dfk_cdiv(g.M, 256) * g.nz0 * g.nz1 * gg.splitk;
    if (tiles256 >= t256) wt = 128;
  }
  if (dma && vec && wt == 32 && !conv) {
    // small grids, forward and dX: 8-wave 128x64 / 64x128 workgroups of 32x32 waves, the longer side along the
    // larger of M / N (each staged tile feeds twice the MFMA work of a 4-wave 64x64 one; r4u: C2 247.1 -> 250.6
    // clips/s, vst4.fc1 dX 69 -> 49 us); the dW GEMMs (k-major A) keep 64x64 (their fp32 epilogue lost there)
    static const int t32x = getenv("DFK_GEMM_T32X") ? atoi(getenv("DFK_GEMM_T32X")) : -1;   // A/B: 0 / 1 / 2
    if (t32x == 1 || (t32x < 0 && !g.a_kmajor && g.M >= g.N)) wt = 33;
    else if (t32x == 2 || (t32x < 0 && !g.a_kmajor)) wt = 34;
  }
  const int bm = wt == 128 ? 256 : (wt == 33 ? 128 : (wt == 34 ? 64 : 2 * wt));
  const int bn = wt == 128 ? 128 : (wt == 33 ? 64 : (wt == 34 ? 128 : 2 * wt));
  dim3 grid(dfk_cdiv(g.N, bn), dfk_cdiv(g.M, bm), g.nz0 * g.nz1 * gg.splitk);
  if (grid.y > 65535 || grid.z > 65535) return DFK_EINVAL;
  // epilogue 16-B path: 8-element groups of C / residual / aux / bias rows stay 16-B aligned
  const bool evec = !g.c_f32 && aligned16(g.c) && g.ldc % 8 == 0 && g.cbs0 % 8 == 0 && g.cbs1 % 8 == 0 &&
                    (!g.bias || (aligned16(g.bias) && g.bias_bs1 % 8 == 0)) &&
                    (!g.residual || (aligned16(g.residual) && g.ldr % 8 == 0 && g.rbs0 % 8 == 0 && g.rbs1 % 8 == 0)) &&
                    (!g.aux || (aligned16(g.aux) && g.ldaux % 8 == 0));
  float* slab = autos > 1 ? reinterpret_cast<float*>(g.ws) : nullptr;
  const SplitK sk{slab, slab ? dfk_ticket_slice((long)grid.x * grid.y * g.nz0 * g.nz1, s) : nullptr};
  if (vec) {
    if (dma) dispatch_dma(gg, wt, grid, kchunk, evec, sk, s);
    else if (conv) dispatch<T, true, true>(gg, wt, grid, kchunk, evec, sk, s);
    else dispatch<T, true, false>(gg, wt, grid, kchunk, evec, sk, s);
  } else {
    dispatch<T, false, true>(gg, wt, grid, kchunk, evec, sk, s);
  }
  // the bias-gradient partials (after the slab, if any): only gemm_dma_kernel writes them (dma && vec); the
  // register-staged kernels add the bias gradient atomically into rowsum and leave the workspace untouched
  if (dma && vec && g.rowsum && gg.splitk >= kRsPartialMin && g.ws)
    hipLaunchKernelGGL(rowsum_reduce_kernel, dim3(dfk_cdiv(g.M, 64)), dim3(1024), 0, s,
                       reinterpret_cast<const float*>(g.ws) + (g.atomic ? 0L : (long)gg.splitk * g.M * g.N), gg.splitk,
                       g.M, g.rowsum);
  if (slab && !sk.cnt && g.c_f32 && autos >= 8 && g.N % 4 == 0 && g.nz0 == 1 && g.nz1 == 1 && !g.bias &&
      !g.residual && !g.act) {   // many fp32 splits (weight gradients): the split loop spread over 8 phases
    hipLaunchKernelGGL(slab_sum_f32_kernel, dim3((unsigned)dfk_cdiv((long)g.M * g.N, 256)), dim3(512), 0, s, g,
                       slab, autos);
  } else if (slab && !sk.cnt) {   // no ticket arena: the reduce / epilogue launch combines the splits
    const long threads = (long)g.nz0 * g.nz1 * g.M * dfk_cdiv(g.N, 8);
    hipLaunchKernelGGL(splitk_reduce_kernel<T>, dim3((unsigned)dfk_cdiv(threads, 256)), dim3(256), 0, s, g, slab,
                       autos, evec ? 1 : 0);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}


// ---------------------------------------------------------------------------------------------------
// MX-fp8 GEMM (include/dfk.h dfk_gemm_mx): C = A B^T with A [M][K], B [N][K] OCP e4m3 + E8M0 block scales, on
// v_mfma_scale_f32_16x16x128_f8f6f4 — one MFMA covers a whole 128-k tile, at twice the bf16 rate per clock.
// Lane map of that instruction, decoded on the hardware (tools/mx_probe.hip, profiles/fp8/r4_mx_lane_map_probe.txt):
// lane l holds row (col) l&15 of A (B); its 32 bytes are two 16-byte halves, half h = k [64h + 16(l>>4), +16); the
// E8M0 scale of row i's k-block kb (k in [32kb, 32kb+32)) is byte 0 of lane (i + 16kb)'s scale VGPR.  So a k-tile
// image [ROWS][128 B] is the bf16 kernel's [ROWS][64 bf16] image byte for byte: same source-side XOR swizzle, and
// the two 16-B fragment reads of lane l are chunks (l>>4) and 4 + (l>>4) of its row (conflict-free, as the bf16
// kernel's k-steps 0 and 1).  Scales: per k-tile one dword per row (the 4 block scales), DMA'd 4 B per lane into a
// per-stage scale image; lane l shifts its row's dword right by 8(l>>4) (the instruction reads byte 0 only).
// The accumulator must stay loop-carried (dst tied to srcC): with a fresh zero C, hipcc once placed the destination
// over srcA and the hardware result was wrong (r4a probe).
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int ROWS, int NWV>
struct Dma8 {   // one operand's [ROWS][128 B] k-tile image: chunk c of row r stored at c ^ ((r>>1)&7)
  static constexpr int NI = ROWS / (8 * NWV);
  __device__ static __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, uint32_t ld, int row0, int rowlim, int k0,
                                               uint8_t* img, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int sl = (wave * NI + i) * 64 + lane;
      const int r = sl >> 3, c = (sl & 7) ^ ((r >> 1) & 7);
      const int vr = row0 + r;
      const uint32_t off = (uint32_t)vr * ld + (uint32_t)(k0 + c * 16);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + (wave * NI + i) * 1024), 16,
                                               vr < rowlim ? off : 0x80000000u, 0, 0, 0);
    }
  }
};

__device__ __forceinline__ i32x8 frag_mx(const uint8_t* img, int r0, int lane) {
  const int r = r0 + (lane & 15), g = lane >> 4, sw = (r >> 1) & 7;
  const uint4 lo = *reinterpret_cast<const uint4*>(img + r * 128 + ((g ^ sw) << 4));
  const uint4 hi = *reinterpret_cast<const uint4*>(img + r * 128 + (((4 + g) ^ sw) << 4));
  return i32x8{(int)lo.x, (int)lo.y, (int)lo.z, (int)lo.w, (int)hi.x, (int)hi.y, (int)hi.z, (int)hi.w};
}

template <int WT, int NWM, int NWN, int S, bool MXO>
__global__ __launch_bounds__(NWM * NWN * 64) void gemm_mx_kernel(const dfk_gemm_args g, const dfk_mx_operand ma,
                                                                 const dfk_mx_operand mb, int evec) {
  constexpr int NWV = NWM * NWN, BM = NWM * WT, BN = NWN * WT, MI = WT / 16, BK = 128;
  constexpr int RW = (BM + BN) / NWV;                 // scale rows DMA'd per wave (one 4-B-per-lane instruction)
  static_assert(RW <= 64 && BM % RW == 0, "scale DMA split");
  constexpr int STAGE = (BM + BN) * BK + NWV * 256;   // operand images + per-wave 256-B scale slots (bytes)
  constexpr int ES = WT + 4;
  constexpr int SMEM = S * STAGE > NWV * WT * ES * 4 ? S * STAGE : NWV * WT * ES * 4;
  constexpr int LPT = Dma8<BM, NWV>::NI + Dma8<BN, NWV>::NI + 1;   // DMA instructions per wave per k-tile
  __shared__ __attribute__((aligned(16))) float smem_f[SMEM / 4];   // the one LDS object (staging + epilogue)
  uint8_t* smem = reinterpret_cast<uint8_t*>(smem_f);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / NWN, wn = wave % NWN;
  int tn, tmi;
  {
    const int nwg = gridDim.x * gridDim.y, bid = blockIdx.y * gridDim.x + blockIdx.x;
    const int xcd = bid & 7, q = nwg >> 3, rr = nwg & 7;
    const int nid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + (bid >> 3);
    tn = nid % gridDim.x;
    tmi = nid / gridDim.x;
  }
  const int bn = tn * BN, bm = tmi * BM;
  const int ntile = g.K / BK;
  const uint32_t lda = (uint32_t)ma.ld, ldb = (uint32_t)mb.ld;
  const __amdgpu_buffer_rsrc_t rqa = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(ma.q), (short)0, (int)((long)(g.M - 1) * ma.ld + g.K), 0x00020000);
  const __amdgpu_buffer_rsrc_t rqb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(mb.q), (short)0, (int)((long)(g.N - 1) * mb.ld + g.K), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(ma.s), (short)0, (int)(((long)(ntile - 1) * ma.lds + g.M) * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint32_t*>(mb.s), (short)0, (int)(((long)(ntile - 1) * mb.lds + g.N) * 4), 0x00020000);
  // this wave's scale rows: entries [wave*RW, wave*RW + RW) of (A tile rows ++ B tile rows) — all of one operand
  const bool sc_a = wave * RW < BM;
  const int sc_row = (sc_a ? bm + wave * RW : bn + wave * RW - BM) + lane;
  const bool sc_in = lane < RW && sc_row < (sc_a ? g.M : g.N);
  const uint32_t sc_ld = (uint32_t)(sc_a ? ma.lds : mb.lds);

  auto issue = [&](int t, uint8_t* st) {
    Dma8<BM, NWV>::issue(rqa, lda, bm, g.M, t * BK, st, wave, lane);
    Dma8<BN, NWV>::issue(rqb, ldb, bn, g.N, t * BK, st + BM * BK, wave, lane);
    const uint32_t off = ((uint32_t)t * sc_ld + (uint32_t)sc_row) * 4u;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(sc_a ? rsa : rsb, (lds_void*)(st + (BM + BN) * BK + wave * 256), 4,
                                             sc_in ? off : 0x80000000u, 0, 0, 0);
  };

  f32x4 acc[MI][MI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < MI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
  for (int d = 0; d < S - 1; ++d)
    if (d < ntile) issue(d, smem + d * STAGE);
  for (int t = 0; t < ntile; ++t) {
    if constexpr (S == 3) {
      if (t + 1 < ntile) wait_vm<LPT>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + S - 1 < ntile) issue(t + S - 1, smem + ((t + S - 1) % S) * STAGE);
    const uint8_t* As = smem + (t % S) * STAGE;
    const uint8_t* Bs = As + BM * BK;
    const uint32_t* Ss = reinterpret_cast<const uint32_t*>(As + (BM + BN) * BK);
    i32x8 af[MI], bfr[MI];
    int sa[MI], sb[MI];
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      af[mi] = frag_mx(As, wm * WT + mi * 16, lane);
      const int i = wm * WT + mi * 16 + (lane & 15);
      sa[mi] = (int)(Ss[(i / RW) * 64 + i % RW] >> (8 * (lane >> 4)));
    }
#pragma unroll
    for (int ni = 0; ni < MI; ++ni) {
      bfr[ni] = frag_mx(Bs, wn * WT + ni * 16, lane);
      const int i = BM + wn * WT + ni * 16 + (lane & 15);
      sb[ni] = (int)(Ss[(i / RW) * 64 + i % RW] >> (8 * (lane >> 4)));
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi)
#pragma unroll
      for (int ni = 0; ni < MI; ++ni)
        acc[mi][ni] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[mi], bfr[ni], acc[mi][ni], 0, 0, 0, sa[mi],
                                                                        0, sb[ni]);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __syncthreads();
  tile_epilogue<bf16raw, WT, MXO>(g, smem_f, acc, lane, wave, wm, wn, bm, bn, 0, 0, 0, evec, SplitK{nullptr, nullptr});
}

// ---- MX quantisation (dfk_mx_quant) ----
// E8M0 scale byte of a 32-element block with max |x| = am: the smallest e with am / 2^(e-127) <= 448
// (am = 1.m * 2^(E-127): e = E - 8, or E - 7 when 1.m > 1.75), clamped so 2^(127-e) is a normal float
__device__ __forceinline__ int mx_scale_byte(float am) {
  const uint32_t b = __float_as_uint(am);
  int e = (int)((b >> 23) & 0xff) - 8 + ((b & 0x7fffffu) > 0x600000u ? 1 : 0);
  e = am == 0.f ? 127 : e;
  return min(max(e, 1), 253);
}
// 8 values -> 8 e4m3 bytes (x * 2^(127-e), rounded to nearest even)
__device__ __forceinline__ uint2 mx_pack8(const float (&v)[8], int e) {
  const float inv = __uint_as_float((uint32_t)(254 - e) << 23);
  int w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
  w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
  int w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
  w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
  return make_uint2((uint32_t)w0, (uint32_t)w1);
}
// the 4 block scales of a 16-lane k-tile group -> one dword (valid in the group's first lane)
__device__ __forceinline__ uint32_t mx_gather_scales(int e, int lane) {
  const int base = lane & ~15;
  const uint32_t b0 = (uint32_t)__shfl(e, base, 64), b1 = (uint32_t)__shfl(e, base + 4, 64);
  const uint32_t b2 = (uint32_t)__shfl(e, base + 8, 64), b3 = (uint32_t)__shfl(e, base + 12, 64);
  return b0 | (b1 << 8) | (b2 << 16) | (b3 << 24);
}

// along the rows' contiguous dim: one thread per 8 elements, 4 lanes per 32-block, 16 lanes per 128-k tile
template <typename T>
__global__ __launch_bounds__(256) void mx_quant_kernel(const T* __restrict__ x, long rows, int cols, long ldx,
                                                       uint8_t* __restrict__ q, long ldq, uint32_t* __restrict__ s) {
  const long t = (long)blockIdx.x * 256 + threadIdx.x;
  const int lane = threadIdx.x & 63;
  const int cpr = cols >> 3;
  const long r = t / cpr;
  const int c8 = (int)(t - r * cpr);
  const bool ok = r < rows;
  float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (ok) ld8<T>(x + r * ldx + c8 * 8, v);
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[i]));
  am = fmaxf(am, __shfl_xor(am, 1, 64));
  am = fmaxf(am, __shfl_xor(am, 2, 64));
  const int e = mx_scale_byte(am);
  const uint2 w = mx_pack8(v, e);
  const uint32_t sd = mx_gather_scales(e, lane);
  if (ok) {
    *reinterpret_cast<uint2*>(q + r * ldq + c8 * 8) = w;
    if ((c8 & 15) == 0) s[(long)(c8 >> 4) * rows + r] = sd;
  }
}

// x^T along x's rows: a 128 (r) x 64 (c) tile through LDS; output row c = 16 lanes x 8 consecutive r.
// Full tiles (vec: 16-B aligned rows) load 8-element chunks, all four of a thread in flight at once (the
// weights' dX operand: grids of 32-128 workgroups, so the per-workgroup latency is the kernel time; the
// element-wise loop ran 17 us per Swin-B stage-3 weight); the column tail keeps the element-wise loop
template <typename T>
__global__ __launch_bounds__(256) void mx_quant_t_kernel(const T* __restrict__ x, int R, int C, long ldx,
                                                         uint8_t* __restrict__ q, long ldq, uint32_t* __restrict__ s,
                                                         int vec) {
  __shared__ float tile[128][65];
  const int c0 = blockIdx.x * 64, r0 = blockIdx.y * 128, tid = threadIdx.x, lane = tid & 63;
  if (vec && c0 + 64 <= C) {
    float v[4][8];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256;
      ld8<T>(x + (long)(r0 + (i >> 3)) * ldx + c0 + (i & 7) * 8, v[j]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = tid + j * 256;
#pragma unroll
      for (int e = 0; e < 8; ++e) tile[i >> 3][(i & 7) * 8 + e] = v[j][e];
    }
  } else {
#pragma unroll 4
    for (int i = tid; i < 128 * 64; i += 256) {
      const int rr = i >> 6, cc = i & 63;
      tile[rr][cc] = c0 + cc < C ? ldf<T>(x + (long)(r0 + rr) * ldx + c0 + cc) : 0.f;
    }
  }
  __syncthreads();
  const int ch = tid & 15;
#pragma unroll
  for (int it = 0; it < 4; ++it) {
    const int cc = (tid >> 4) + 16 * it, c = c0 + cc;
    float v[8];
    float am = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      v[i] = tile[ch * 8 + i][cc];
      am = fmaxf(am, fabsf(v[i]));
    }
    am = fmaxf(am, __shfl_xor(am, 1, 64));
    am = fmaxf(am, __shfl_xor(am, 2, 64));
    const int e = mx_scale_byte(am);
    const uint2 w = mx_pack8(v, e);
    const uint32_t sd = mx_gather_scales(e, lane);
    if (c < C) {
      *reinterpret_cast<uint2*>(q + (long)c * ldq + r0 + ch * 8) = w;
      if (ch == 0) s[(long)(r0 >> 7) * C + c] = sd;
    }
  }
}

// epilogue 16-B path legal for g (8-element groups of C / residual / aux / bias rows stay 16-B aligned)
bool epi_vec(const dfk_gemm_args& g) {
  return !g.c_f32 && aligned16(g.c) && g.ldc % 8 == 0 && g.cbs0 % 8 == 0 && g.cbs1 % 8 == 0 &&
         (!g.bias || (aligned16(g.bias) && g.bias_bs1 % 8 == 0)) &&
         (!g.residual || (aligned16(g.residual) && g.ldr % 8 == 0 && g.rbs0 % 8 == 0 && g.rbs1 % 8 == 0)) &&
         (!g.aux || (aligned16(g.aux) && g.ldaux % 8 == 0));
}

}  // namespace

// Arrival tickets of the in-launch split-K combine: one zeroed arena of counters per device, handed out in
// consecutive slices (a launch's tiles), round robin.  Every ticket returns to 0 when its tile's last arriver
// resets it, so a slice is zero whenever it is handed out again; launches that can run concurrently (other
// streams, one captured graph) hold disjoint slices as long as fewer than kTickets tiles are in flight.
// nullptr: no arena (first use inside a stream capture, or allocation failure): the caller combines in a
// separate launch (splitk_reduce_kernel, slab_colsum).  Shared by the GEMM split-K and LayerNorm dγ/dβ partials.
constexpr long kTickets = 1L << 20;
uint32_t* dfk_ticket_slice(long n, hipStream_t s) {
  // opt-in (DFK_INLAUNCH_COMBINE=1): measured slower than the separate combine launch in the C2 step (the last
  // arriver reads every split's slab serially: w2v dX 22 -> 43 us, LN backward 17 -> 45 us;
  // profiles/gemm/r4o_inlaunch_combine_rejected.txt)
  const char* env = getenv("DFK_INLAUNCH_COMBINE");   // read per call: tests switch it inside one process
  if (!env || atoi(env) == 0 || n <= 0 || n > kTickets) return nullptr;
  // never inside a graph capture: a slice baked into a graph stays in use at every replay, and the round-robin
  // cursor would later hand it to another launch (two launches miscounting one slice's arrivals); captured
  // launches take the separate combine launch instead
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(s, &cap) != hipSuccess || cap != hipStreamCaptureStatusNone) return nullptr;
  static std::mutex mu;
  static uint32_t* arena[64] = {};
  static long cursor[64] = {};
  std::lock_guard<std::mutex> lock(mu);
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!arena[dev]) {
    void* p = nullptr;
    if (hipMalloc(&p, kTickets * 4) != hipSuccess) return nullptr;
    if (hipMemsetAsync(p, 0, kTickets * 4, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) {
      (void)hipFree(p);
      return nullptr;
    }
    arena[dev] = static_cast<uint32_t*>(p);
  }
  if (cursor[dev] + n > kTickets) cursor[dev] = 0;
  uint32_t* t = arena[dev] + cursor[dev];
  cursor[dev] += (n + 63) & ~63L;
  return t;
}

extern "C" int dfk_gemm(const dfk_gemm_args* g, hipStream_t s) {
  if (!g || g->mx_q) return DFK_EINVAL;   // the MX copy of C is a dfk_gemm_mx epilogue
  return g->dtype == DFK_BF16 ? launch<bf16raw>(*g, s) : launch<float>(*g, s);
}

extern "C" int64_t dfk_gemm_workspace(const dfk_gemm_args* g) {
  if (!g) return -1;
  const int autos = g->splitk > 1 && !g->atomic ? g->splitk
                    : (g->dtype == DFK_BF16 ? auto_splitk<bf16raw>(*g) : auto_splitk<float>(*g));
  // per-split bias-gradient partials (gemm_dma_kernel RS, i.e. the LDS-DMA vector path only), after the split
  // slabs if there are any
  const bool dmav = g->dtype == DFK_BF16 && dma_ok(*g) && view_vec(g->a, 8) && view_vec(g->b, 8) &&
                    (g->a_kmajor ? g->M : g->K) % 8 == 0 && (g->b_kmajor ? g->N : g->K) % 8 == 0;
  const int64_t rs = !dmav || !g->rowsum ? 0
                     : (g->atomic && g->splitk >= kRsPartialMin ? (int64_t)g->splitk * g->M * 4
                                                                : (autos >= kRsPartialMin ? (int64_t)autos * g->M * 4 : 0));
  if (autos <= 1) return rs;
  return (int64_t)autos * g->nz0 * g->nz1 * g->M * g->N * 4 + rs;
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

extern "C" int dfk_gemm_mx(const dfk_gemm_args* gp, const dfk_mx_operand* a, const dfk_mx_operand* b, hipStream_t s) {
  if (!gp || !a || !b) return DFK_EINVAL;
  const dfk_gemm_args& g = *gp;
  if (!a->q || !a->s || !b->q || !b->s || !g.c) return DFK_EINVAL;
  if (g.dtype != DFK_BF16 || g.splitk != 1 || g.atomic || g.c_f32 || g.rowsum || g.nz0 != 1 || g.nz1 != 1)
    return DFK_EINVAL;
  if (g.K <= 0 || g.K % 128 || a->ld % 16 || b->ld % 16 || a->ld < g.K || b->ld < g.K) return DFK_EINVAL;
  if (a->lds < g.M || b->lds < g.N) return DFK_EINVAL;
  if (g.act < 0 || g.act > 2 || (g.act == 2 && !g.aux)) return DFK_EINVAL;
  if (g.drop.mode && (!g.drop.rng || !(g.drop.p >= 0.f && g.drop.p < 1.f))) return DFK_EINVAL;
  if (g.M <= 0 || g.N <= 0) return 0;
  if ((long)(g.M - 1) * a->ld + g.K >= 0x7fffffffL || (long)(g.N - 1) * b->ld + g.K >= 0x7fffffffL) return DFK_EINVAL;
  const bool mxo = g.mx_q != nullptr;
  if (mxo && (!g.mx_s || g.N % 128 || g.mx_ldq % 16 || g.mx_ldq < g.N || g.mx_lds < g.M ||
              (reinterpret_cast<uintptr_t>(g.mx_q) & 15)))
    return DFK_EINVAL;
  const long tiles128 = (long)dfk_cdiv(g.N, 128) * dfk_cdiv(g.M, 128);
  const int evec = epi_vec(g) ? 1 : 0;
  if (tiles128 < 1024) {   // 64 x 64 tiles for grids that 128 x 128 tiles cannot spread over the chip
    dim3 grid(dfk_cdiv(g.N, 64), dfk_cdiv(g.M, 64));
    if (grid.y > 65535) return DFK_EINVAL;
    if (mxo) hipLaunchKernelGGL((gemm_mx_kernel<32, 2, 2, 2, true>), grid, dim3(256), 0, s, g, *a, *b, evec);
    else hipLaunchKernelGGL((gemm_mx_kernel<32, 2, 2, 2, false>), grid, dim3(256), 0, s, g, *a, *b, evec);
  } else {
    dim3 grid(dfk_cdiv(g.N, 128), dfk_cdiv(g.M, 128));
    if (grid.y > 65535) return DFK_EINVAL;
    if (mxo) hipLaunchKernelGGL((gemm_mx_kernel<64, 2, 2, 2, true>), grid, dim3(256), 0, s, g, *a, *b, evec);
    else hipLaunchKernelGGL((gemm_mx_kernel<64, 2, 2, 2, false>), grid, dim3(256), 0, s, g, *a, *b, evec);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_mx_quant(const void* x, int dtype, int64_t rows, int64_t cols, int64_t ldx, int transpose,
                            uint8_t* q, int64_t ldq, uint32_t* sc, hipStream_t s) {
  if (!x || !q || !sc || rows < 0 || cols < 0 || (dtype != DFK_BF16 && dtype != DFK_F32)) return DFK_EINVAL;
  if (ldq % 16 || (reinterpret_cast<uintptr_t>(q) & 15)) return DFK_EINVAL;
  if (rows == 0 || cols == 0) return 0;
  if (!transpose) {
    if (cols % 128 || ldq < cols || ldx < cols || ldx % 8 || (reinterpret_cast<uintptr_t>(x) & 15)) return DFK_EINVAL;
    const long threads = rows * (cols / 8);
    const unsigned blocks = (unsigned)dfk_cdiv(threads, 256);
    if (dtype == DFK_BF16)
      hipLaunchKernelGGL(mx_quant_kernel<bf16raw>, dim3(blocks), dim3(256), 0, s, (const bf16raw*)x, (long)rows,
                         (int)cols, (long)ldx, q, (long)ldq, sc);
    else
      hipLaunchKernelGGL(mx_quant_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, (long)rows, (int)cols,
                         (long)ldx, q, (long)ldq, sc);
  } else {
    if (rows % 128 || ldq < rows || ldx < cols || rows > 0x7fffffff || cols > 0x7fffffff) return DFK_EINVAL;
    dim3 grid(dfk_cdiv(cols, 64), (unsigned)(rows / 128));
    if (grid.y > 65535) return DFK_EINVAL;
    const int vec = (reinterpret_cast<uintptr_t>(x) & 15) == 0 && ldx % 8 == 0;
    if (dtype == DFK_BF16)
      hipLaunchKernelGGL(mx_quant_t_kernel<bf16raw>, grid, dim3(256), 0, s, (const bf16raw*)x, (int)rows, (int)cols,
                         (long)ldx, q, (long)ldq, sc, vec);
    else
      hipLaunchKernelGGL(mx_quant_t_kernel<float>, grid, dim3(256), 0, s, (const float*)x, (int)rows, (int)cols,
                         (long)ldx, q, (long)ldq, sc, vec);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}
