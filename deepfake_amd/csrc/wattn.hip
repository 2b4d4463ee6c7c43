// Shifted-window multi-head attention core for gfx950 (forward + backward).
//
// One workgroup = one (clip, window, head); the window's tokens are gathered
// straight from the token-major qkv buffer: padding, cyclic roll and
// window_partition / window_reverse (video_swin_transformer.py:224-252) are
// pure index arithmetic, so no permuted copy of the activations ever exists.
// Relative-position bias: token ids decoded with the FULL window geometry
// (Q3) so idx(q,k) = pos(q) - pos(k) + C0 with pos() precomputed per token.
// Shift mask: region labels per token, -100 when they differ (Q4, :319-333).
//
// Forward (per wave, 16 queries): S^T = K Q^T on MFMA with the QUERY on the
// lane, online softmax over 32-key blocks (row statistics are per-lane
// scalars), O^T += V^T P^T with P^T taken straight from the accumulators.
#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

// This file is built with IEEE mode off and no-NaN semantics (build.py FILE_FLAGS).  The device library's ockl
// functions behind threadIdx / blockIdx / __umulhi carry the default attributes, so hipcc does not inline them
// here: each use compiled to an s_swappc call (346 in this object, inside the K / V / Q gather loops of every
// attention kernel).  The work-item / work-group ids and the multiply-high below are inline instructions.
#ifdef DFK_OCKL_ALL
__device__ __forceinline__ int dfk_tid() { return threadIdx.x; }
__device__ __forceinline__ int dfk_bid_x() { return blockIdx.x; }
__device__ __forceinline__ int dfk_bid_y() { return blockIdx.y; }
__device__ __forceinline__ int dfk_bid_z() { return blockIdx.z; }
__device__ __forceinline__ uint32_t dfk_umulhi(uint32_t a, uint32_t b) { return __umulhi(a, b); }
#else
__device__ __forceinline__ int dfk_tid() { return (int)__builtin_amdgcn_workitem_id_x(); }
__device__ __forceinline__ int dfk_bid_x() { return (int)__builtin_amdgcn_workgroup_id_x(); }
__device__ __forceinline__ int dfk_bid_y() { return (int)__builtin_amdgcn_workgroup_id_y(); }
__device__ __forceinline__ int dfk_bid_z() { return (int)__builtin_amdgcn_workgroup_id_z(); }
__device__ __forceinline__ uint32_t dfk_umulhi(uint32_t a, uint32_t b) { return (uint32_t)(((uint64_t)a * b) >> 32); }
#endif
// blockDim / gridDim stay HIP's: the dispatch-packet builtins (__builtin_amdgcn_workgroup_size_x / grid_size_x)
// measured slower in every attention kernel (mel1 forward 13.8 -> 36.5 us, vst3 52.9 -> 76.3 us: r4 A/B,
// profiles/attn/r4h_builtin_dims_ab.txt)
__device__ __forceinline__ int dfk_bdim() { return blockDim.x; }
__device__ __forceinline__ int dfk_gdim_x() { return gridDim.x; }
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

struct TokInfo {
  int row;     // token row index into the token-major buffers; -1: padded position; -2: beyond N
  int pos;     // RPB position (full-window decode)
  int lab;     // region label (shift mask)
};

struct Geo {
  int nwd, nwh, nww, nW;   // windows per dim
  int Dp, Hp, Wp;          // padded dims
  int N;                   // tokens per window (clamped)
  int Np;                  // N rounded up to 32
  int L;                   // rpb table rows
  int C0;                  // rpb index offset
  int use_mask;
  uint32_t m_hw, m_w;      // fast-division multipliers for wh*ww and ww (0: divisor 1), exact for i < 2^16
};

// floor(x / n) for x < 2^16, n < 2^16 with m = floor((2^32-1)/n) + 1 (m = 0 encodes n = 1): the error of
// x*m/2^32 is below x/2^32 < 1/n, so the floor is exact; one v_mul_hi_u32 instead of a division sequence
__device__ __forceinline__ int fdiv16(int x, uint32_t m) { return m ? (int)dfk_umulhi((uint32_t)x, m) : x; }

__device__ __forceinline__ int region(int p, int P, int w, int s) {
  if (s == 0) return 2;
  return p < P - w ? 0 : (p < P - s ? 1 : 2);
}

// token i of window `win` of clip b
__device__ __forceinline__ TokInfo token_info(const dfk_wattn_args& a, const Geo& g, int b, int win, int i) {
  TokInfo t;
  if (i >= g.N) { t.row = -2; t.pos = 0; t.lab = -1; return t; }
  const int wwi = win % g.nww, whi = (win / g.nww) % g.nwh, wdi = win / (g.nww * g.nwh);
  const int td = i / (a.wh * a.ww), th = (i / a.ww) % a.wh, tw = i % a.ww;
  const int pd = wdi * a.wd + td, ph = whi * a.wh + th, pw = wwi * a.ww + tw;   // shifted frame
  const int od = (pd + a.sd) % g.Dp, oh = (ph + a.sh) % g.Hp, ow = (pw + a.sw) % g.Wp;  // roll(-shift)
  t.row = (od < a.D && oh < a.H && ow < a.W) ? ((b * a.D + od) * a.H + oh) * a.W + ow : -1;
  const int fd = i / (a.fh * a.fw), fh = (i / a.fw) % a.fh, fw = i % a.fw;        // Q3 decode
  t.pos = (fd * (2 * a.fh - 1) + fh) * (2 * a.fw - 1) + fw;
  t.lab = region(pd, g.Dp, a.wd, a.sd) * 9 + region(ph, g.Hp, a.wh, a.sh) * 3 + region(pw, g.Wp, a.ww, a.sw);
  return t;
}

// only the row of token i (the forward's Q/K/V gathers): window origin from uniform values, token
// offsets by multiply-high divisions, cyclic roll by one conditional subtract (coordinate < 2 * padded dim)
__device__ __forceinline__ int token_info_row(const dfk_wattn_args& a, const Geo& g, int b, int win, int i) {
  if (i >= g.N) return -2;
  const int wwi = win % g.nww, whi = (win / g.nww) % g.nwh, wdi = win / (g.nww * g.nwh);
  const int td = fdiv16(i, g.m_hw), r = i - td * (a.wh * a.ww);
  const int th = fdiv16(r, g.m_w), tw = r - th * a.ww;
  int od = wdi * a.wd + a.sd + td, oh = whi * a.wh + a.sh + th, ow = wwi * a.ww + a.sw + tw;
  od -= od >= g.Dp ? g.Dp : 0;
  oh -= oh >= g.Hp ? g.Hp : 0;
  ow -= ow >= g.Wp ? g.Wp : 0;
  return (od < a.D && oh < a.H && ow < a.W) ? ((b * a.D + od) * a.H + oh) * a.W + ow : -1;
}

// address of element e of head h for token info row (or the pad vector / zero)
template <typename T>
__device__ __forceinline__ const T* tok_ptr(const void* base, const void* pad, int row, long ld, int off) {
  if (row >= 0) return reinterpret_cast<const T*>(base) + (long)row * ld + off;
  if (row == -1 && pad) return reinterpret_cast<const T*>(pad) + off;
  return nullptr;
}

template <typename T>
__device__ __forceinline__ uint4 ld16(const T* p) {
  return p ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
}

// Branch-free token loads: the address is always valid (invalid tokens read the buffer base) and the
// value is masked afterwards, so no branch (and no vmcnt(0) wait inside it) surrounds the load.
template <typename T>
__device__ __forceinline__ const T* tok_src(const void* base, const void* pad, int row, long ld, int off, bool& ok) {
  const bool real = row >= 0, padded = row == -1 && pad != nullptr;
  ok = real || padded;
  const T* pr = reinterpret_cast<const T*>(base) + (real ? (long)row * ld + off : 0);
  const T* pp = reinterpret_cast<const T*>(padded ? pad : base) + (padded ? off : 0);
  return real ? pr : pp;
}

template <typename T>
__device__ __forceinline__ uint4 tok_ld16(const void* base, const void* pad, int row, long ld, int off) {
  bool ok;
  const T* p = tok_src<T>(base, pad, row, ld, off, ok);
  uint4 x = *reinterpret_cast<const uint4*>(p);
  const uint32_t m = ok ? 0xffffffffu : 0u;
  x.x &= m; x.y &= m; x.z &= m; x.w &= m;
  return x;
}

template <typename T>
__device__ __forceinline__ T tok_ld1(const void* base, const void* pad, int row, long ld, int off) {
  bool ok;
  const T* p = tok_src<T>(base, pad, row, ld, off, ok);
  const T x = *p;
  return ok ? x : (T)0;
}

typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;

constexpr float kLog2e = 1.4426950408889634f;
constexpr int kBwdWaves = 8;
constexpr int kSdStride = 40;  // bf16 row stride of the per-wave dS^T scratch [32 keys][32 queries]

// element offset of (row, col) in a [rows][HD] bf16 tile with 16-B chunks XOR-swizzled by row.  HD 32:
// chunk ^= (-(row >> 2)) & 3 makes the three access shapes conflict-free on the gfx950 lane groups (16-B
// A-operand row reads: lanes 16 rows x 4 chunks; 8-B tr16 reads: 8 rows x 4 column pairs; 16-B staging
// writes) — checked by brute force over the lane groups; HD 64: 2-way on the row and tr16 reads.
template <int HD>
__device__ __forceinline__ int swz(int row, int col) {
  const int f = HD == 32 ? ((4 - ((row >> 2) & 3)) & 3) : (((row & 3) << 1) | ((row >> 2) & 1));
  return row * HD + (((col >> 3) ^ f) << 3) + (col & 7);
}

// fp32 [rows][HD] accumulator: the 4 rows a C fragment touches land in two bank halves
template <int HD>
__device__ __forceinline__ int dq_off(int row, int col) {
  return row * HD + (col ^ (((row >> 2) & 1) << 4));
}

__device__ __forceinline__ bf16x8 tr16x2(const bf16raw* p0, const bf16raw* p1) {
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(p0));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(p1));
  short8 u = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, u);
}

__device__ __forceinline__ float dot8_bf16(uint4 x, uint4 y) {
  const bf16raw* a = reinterpret_cast<const bf16raw*>(&x);
  const bf16raw* b = reinterpret_cast<const bf16raw*>(&y);
  float d = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) d += bf2f(a[j]) * bf2f(b[j]);
  return d;
}

// ---------------------------------------------------------------- forward
template <typename T, int HD>
__global__ __launch_bounds__(256) void wattn_fwd_kernel(const dfk_wattn_args a, const Geo g, int qsplit) {
  constexpr bool BF = sizeof(T) == 2;
  constexpr int VEC = 16 / sizeof(T);
  extern __shared__ __attribute__((aligned(16))) char smem[];
  // layout: tok[Np] | rpb[L] | K[Np][HD] | V (bf16: Vt[HD][Np+8], f32: V[Np][HD])
  TokInfo* tok = reinterpret_cast<TokInfo*>(smem);
  float* rpb = reinterpret_cast<float*>(smem + sizeof(TokInfo) * g.Np);
  const int Lal = (g.L + 3) & ~3;
  T* Ks = reinterpret_cast<T*>(smem + sizeof(TokInfo) * g.Np + 4 * Lal);
  T* Vs = Ks + g.Np * HD;
  const int VTS = g.Np + 8;  // bf16 transposed-V row stride

  const int tid = dfk_tid(), lane = tid & 63, wave = tid >> 6;
  int unit = dfk_bid_x();
  const int head = unit % a.heads;
  unit /= a.heads;
  const int win = unit % g.nW, b = unit / g.nW;
  const float* mrow = a.mask ? a.mask + (((long)b * g.nW + win) % a.mask_nw) * g.N * g.N : nullptr;

  for (int i = tid; i < g.Np; i += 256) tok[i] = token_info(a, g, b, win, i);
  if (a.rpb)
    for (int l = tid; l < g.L; l += 256) rpb[l] = a.rpb[(long)l * a.heads + head];
  __syncthreads();
  // K, V of the window -> LDS
  const int hoff = head * HD;
  for (int idx = tid; idx < g.Np * (HD / VEC); idx += 256) {
    const int i = idx / (HD / VEC), c = (idx % (HD / VEC)) * VEC;
    const TokInfo t = tok[i];
    const uint4 kv = tok_ld16<T>(a.k, a.pad_k, t.row, a.ld_qkv, hoff + c);
    const uint4 vv = tok_ld16<T>(a.v, a.pad_v, t.row, a.ld_qkv, hoff + c);
    *reinterpret_cast<uint4*>(Ks + i * HD + c) = kv;
    if constexpr (BF) {
      const bf16raw* e = reinterpret_cast<const bf16raw*>(&vv);
#pragma unroll
      for (int j = 0; j < VEC; ++j) reinterpret_cast<bf16raw*>(Vs)[(c + j) * VTS + i] = e[j];
    } else {
      *reinterpret_cast<uint4*>(Vs + i * HD + c) = vv;
    }
  }
  __syncthreads();

  const int grp = lane >> 4, ql = lane & 15;
  const int nqt = (g.N + 15) / 16;
  const int nkb = g.Np / 32;
  for (int qt = dfk_bid_y() * 4 + wave; qt < nqt; qt += 4 * qsplit) {
    const int q = qt * 16 + ql;
    const TokInfo tq = q < g.N ? tok[q] : TokInfo{-2, 0, -1};
    // Q fragment (B operand: lane holds Q[q][e-slots])
    const T* qp = tok_ptr<T>(a.q, a.pad_q, tq.row, a.ld_qkv, hoff);
    float m = -INFINITY, l = 0.f;
    f32x4 o[HD / 16];
#pragma unroll
    for (int i = 0; i < HD / 16; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};

    if constexpr (BF) {
      bf16x8 qf[HD / 32];
#pragma unroll
      for (int es = 0; es < HD / 32; ++es) {
        uint4 u = tok_ld16<T>(a.q, a.pad_q, tq.row, a.ld_qkv, hoff + es * 32 + grp * 8);
        qf[es] = *reinterpret_cast<bf16x8*>(&u);
      }
      for (int kb = 0; kb < nkb; ++kb) {
        f32x4 s[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s[h2] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int krow = kb * 32 + h2 * 16 + ql;
#pragma unroll
          for (int es = 0; es < HD / 32; ++es) {
            const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + krow * HD + es * 32 + grp * 8);
            s[h2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[es], s[h2], 0, 0, 0);
          }
        }
        // bias, mask, scale; block max
        float bm = -INFINITY;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = kb * 32 + h2 * 16 + grp * 4 + r;
            const TokInfo tk = tok[k];
            float v = s[h2][r] * a.scale;
            if (a.rpb) v += rpb[tq.pos - tk.pos + g.C0];
            if (g.use_mask && tq.lab != tk.lab) v -= 100.f;
            if (mrow && q < g.N && k < g.N) v += mrow[q * g.N + k];
            if (tk.row == -2) v = -INFINITY;
            s[h2][r] = v;
            bm = fmaxf(bm, v);
          }
        bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        const float mn = fmaxf(m, bm);
        const float alpha = __expf(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < HD / 16; ++i) o[i] *= alpha;
        float p[8];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) { p[h2 * 4 + r] = __expf(s[h2][r] - m); l += p[h2 * 4 + r]; }
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (__bf16)p[j];
        // O^T[e][q] += V^T[e][k] P^T[k][q]; k-slot j of group g <-> key kb*32 + (j>>2)*16 + 4g + (j&3)
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) {
          const bf16raw* vr = reinterpret_cast<const bf16raw*>(Vs) + (et * 16 + ql) * VTS + kb * 32 + grp * 4;
          const uint2 lo = *reinterpret_cast<const uint2*>(vr);
          const uint2 hi = *reinterpret_cast<const uint2*>(vr + 16);
          uint4 u = make_uint4(lo.x, lo.y, hi.x, hi.y);
          o[et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(*reinterpret_cast<bf16x8*>(&u), pf, o[et], 0, 0, 0);
        }
      }
    } else {
      float qf[HD / 4];
#pragma unroll
      for (int es = 0; es < HD / 4; ++es) qf[es] = qp ? qp[es * 4 + grp] : 0.f;
      for (int kb = 0; kb < nkb; ++kb) {
        f32x4 s[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          s[h2] = f32x4{0.f, 0.f, 0.f, 0.f};
          const int krow = kb * 32 + h2 * 16 + ql;
#pragma unroll
          for (int es = 0; es < HD / 4; ++es)
            s[h2] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ks[krow * HD + es * 4 + grp], qf[es], s[h2], 0, 0, 0);
        }
        float bm = -INFINITY;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int k = kb * 32 + h2 * 16 + grp * 4 + r;
            const TokInfo tk = tok[k];
            float v = s[h2][r] * a.scale;
            if (a.rpb) v += rpb[tq.pos - tk.pos + g.C0];
            if (g.use_mask && tq.lab != tk.lab) v -= 100.f;
            if (mrow && q < g.N && k < g.N) v += mrow[q * g.N + k];
            if (tk.row == -2) v = -INFINITY;
            s[h2][r] = v;
            bm = fmaxf(bm, v);
          }
        bm = fmaxf(bm, __shfl_xor(bm, 16, 64));
        bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
        const float mn = fmaxf(m, bm);
        const float alpha = __expf(m - mn);
        m = mn;
        l *= alpha;
#pragma unroll
        for (int i = 0; i < HD / 16; ++i) o[i] *= alpha;
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float p = __expf(s[h2][r] - m);
            l += p;
            const int k = kb * 32 + h2 * 16 + grp * 4 + r;  // k-slot grp of this 4-step
#pragma unroll
            for (int et = 0; et < HD / 16; ++et)
              o[et] = __builtin_amdgcn_mfma_f32_16x16x4f32(Vs[k * HD + et * 16 + ql], p, o[et], 0, 0, 0);
          }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.f / l;
    if (tq.row >= 0) {
      T* op = reinterpret_cast<T*>(a.out) + (long)tq.row * a.ld_out + hoff;
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) {
        const int e0 = et * 16 + grp * 4;
        if constexpr (BF) {
          uint2 u;
          bf16raw* pe = reinterpret_cast<bf16raw*>(&u);
#pragma unroll
          for (int r = 0; r < 4; ++r) pe[r] = f2bf(o[et][r] * inv);
          *reinterpret_cast<uint2*>(op + e0) = u;
        } else {
          *reinterpret_cast<float4*>(op + e0) =
              make_float4(o[et][0] * inv, o[et][1] * inv, o[et][2] * inv, o[et][3] * inv);
        }
      }
    }
    if (a.lse && grp == 0 && q < g.N) a.lse[((long)dfk_bid_x()) * g.Np + q] = m + __logf(l);
  }
}

// ------------------------------------------------------------ bf16 forward
// One workgroup = one (clip, window, head) (x qsplit), 4 waves; K and V of the window staged once in
// XOR-swizzled LDS tiles.  Each wave owns 32-query blocks: S^T = K Q^T with the query on the lane (row
// statistics are per-lane scalars, reduced over the 4 lane groups), base-2 online softmax with a lazy
// rescale (only when some query's running max grows by more than kRescale), O^T += V^T P^T with P^T taken
// straight from the accumulators and V^T read by ds_read_tr16, and the softmax denominator produced by
// the same MFMA chain (a ones tile in place of V^T) instead of per-element adds.
constexpr float kRescale = 8.f;   // log2 units: P stays <= 2^8 between rescales

template <int HD, bool RPB, bool MASK>
__global__ __launch_bounds__(256) void wattn_fwd_bf16_kernel(const dfk_wattn_args a, const Geo g, int qsplit) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lal = (g.L + 3) & ~3;
  char* p = smem;
  int& mixed = *reinterpret_cast<int*>(p); p += 16;             // window holds more than one shift region
  int* tpk = reinterpret_cast<int*>(p); p += 4 * g.Np;          // pos << 5 | label; label 31 = beyond N
  float* rpb2 = reinterpret_cast<float*>(p); p += 4 * Lal;      // rpb * log2(e)
  bf16raw* Ks = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)g.Np * HD;
  bf16raw* Vs = reinterpret_cast<bf16raw*>(p);

  const int tid = dfk_tid(), lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, ql = lane & 15, tq = ql >> 2, tp = ql & 3;
  int unit = dfk_bid_x();
  const int head = unit % a.heads;
  unit /= a.heads;
  const int win = unit % g.nW, b = unit / g.nW;
  const float* mrow = MASK ? a.mask + (((long)b * g.nW + win) % a.mask_nw) * g.N * g.N : nullptr;
  const int hoff = head * HD;
  if (tid == 0) mixed = 0;
  __syncthreads();
  int lab0 = -1;
  for (int i = tid; i < g.Np; i += dfk_bdim()) {
    const TokInfo t = token_info(a, g, b, win, i);
    tpk[i] = (t.pos << 5) | (t.row == -2 ? 31 : t.lab);
    if (t.row != -2) {
      if (lab0 < 0) lab0 = t.lab;
      else if (t.lab != lab0) mixed = 1;
    }
  }
  if (g.use_mask && lab0 >= 0 && lab0 != token_info(a, g, b, win, 0).lab) mixed = 1;
  if (RPB)
    for (int l = tid; l < g.L; l += dfk_bdim()) rpb2[l] = a.rpb[(long)l * a.heads + head] * kLog2e;
  __syncthreads();
  constexpr int CH = HD / 8;
  for (int idx = tid; idx < g.Np * CH; idx += dfk_bdim()) {
    const int i = idx / CH, c = (idx % CH) * 8;
    const int row = token_info_row(a, g, b, win, i);
    *reinterpret_cast<uint4*>(Ks + swz<HD>(i, c)) = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
    *reinterpret_cast<uint4*>(Vs + swz<HD>(i, c)) = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
  }
  __syncthreads();
  const bool use_mask = g.use_mask && mixed;

  const float scale2 = a.scale * kLog2e;
  const float mpen = -100.f * kLog2e;
  const int nkb = g.Np / 32, nqb = g.Np / 32;
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
  const int nw = dfk_bdim() >> 6;
  for (int qb = dfk_bid_y() * nw + wave; qb < nqb; qb += nw * qsplit) {
    // the lane's queries (one per 16-query half) and their Q^T B operands
    int qpk[2], qrow[2];
    bf16x8 qf[2][HD / 32];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int q = qb * 32 + qh * 16 + ql;
      qpk[qh] = tpk[q];
      qrow[qh] = q < g.N ? token_info_row(a, g, b, win, q) : -2;
#pragma unroll
      for (int es = 0; es < HD / 32; ++es)
        qf[qh][es] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.q, a.pad_q, qrow[qh], a.ld_qkv, hoff + es * 32 + grp * 8));
    }
    float m[2] = {-INFINITY, -INFINITY};
    f32x4 o[2][HD / 16], lsum[2];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      lsum[qh] = f32x4{0, 0, 0, 0};
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) o[qh][et] = f32x4{0, 0, 0, 0};
    }
    for (int kb = 0; kb < nkb; ++kb) {
      // key statistics of the lane's rows (keys kb*32 + h2*16 + 4grp + r) and the K A-operands
      int4 kp[2];
      bf16x8 ka[2][HD / 32];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        kp[h2] = *reinterpret_cast<const int4*>(tpk + kb * 32 + h2 * 16 + grp * 4);
#pragma unroll
        for (int es = 0; es < HD / 32; ++es)
          ka[h2][es] = *reinterpret_cast<const bf16x8*>(Ks + swz<HD>(kb * 32 + h2 * 16 + ql, es * 32 + grp * 8));
      }
      float x[2][2][4];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2) {
          f32x4 sacc = f32x4{0, 0, 0, 0};
#pragma unroll
          for (int es = 0; es < HD / 32; ++es)
            sacc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ka[h2][es], qf[qh][es], sacc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int kpk = kp[h2][r];
            float v = sacc[r] * scale2;
            if (RPB) v += rpb2[(qpk[qh] >> 5) - (kpk >> 5) + g.C0];
            if (use_mask) v += ((qpk[qh] ^ kpk) & 31) ? mpen : 0.f;
            if constexpr (MASK) {
              const int q = qb * 32 + qh * 16 + ql, k = kb * 32 + h2 * 16 + grp * 4 + r;
              if (q < g.N && k < g.N) v += mrow[q * g.N + k] * kLog2e;
            }
            x[qh][h2][r] = v;
          }
        }
      if (kb == nkb - 1) {   // keys beyond N (the only padded key block)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if ((kp[h2][r] & 31) == 31)
#pragma unroll
              for (int qh = 0; qh < 2; ++qh) x[qh][h2][r] = -INFINITY;
      }
      // running max (per query = per lane column, reduced over the 4 lane groups), lazy rescale
      bool grow = false;
      float mnew[2];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        float mx = x[qh][0][0];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) mx = fmaxf(mx, x[qh][h2][r]);
        mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
        mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
        mnew[qh] = mx > m[qh] + kRescale ? mx : m[qh];
        grow |= mnew[qh] != m[qh];
      }
      if (__builtin_amdgcn_ballot_w64(grow) != 0) {
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const float alpha = m[qh] == -INFINITY ? 0.f : __builtin_amdgcn_exp2f(m[qh] - mnew[qh]);
          m[qh] = mnew[qh];
          lsum[qh] *= alpha;
#pragma unroll
          for (int et = 0; et < HD / 16; ++et) o[qh][et] *= alpha;
        }
      }
      // P^T B operands: key slot j <-> (h2 = j>>2, row 4grp + (j&3))
      bf16x8 pf[2];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int r = 0; r < 4; ++r) pf[qh][h2 * 4 + r] = (__bf16)__builtin_amdgcn_exp2f(x[qh][h2][r] - m[qh]);
      // O^T[e][q] += V^T P^T (V^T by tr16 with the same key permutation); lsum += ones^T P^T
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) {
        const int c = et * 16 + tp * 4;
        const bf16x8 va = tr16x2(Vs + swz<HD>(kb * 32 + grp * 4 + tq, c), Vs + swz<HD>(kb * 32 + 16 + grp * 4 + tq, c));
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) o[qh][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(va, pf[qh], o[qh][et], 0, 0, 0);
      }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) lsum[qh] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, pf[qh], lsum[qh], 0, 0, 0);
    }
    // O = O^T / l: lane holds e = et*16 + 4grp + r of query ql
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int q = qb * 32 + qh * 16 + ql;
      const float l = lsum[qh][0];
      const float inv = 1.f / l;
      if (qrow[qh] >= 0) {
        bf16raw* op = reinterpret_cast<bf16raw*>(a.out) + (long)qrow[qh] * a.ld_out + hoff;
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) {
          uint2 u;
          u.x = (uint32_t)f2bf(o[qh][et][0] * inv) | ((uint32_t)f2bf(o[qh][et][1] * inv) << 16);
          u.y = (uint32_t)f2bf(o[qh][et][2] * inv) | ((uint32_t)f2bf(o[qh][et][3] * inv) << 16);
          *reinterpret_cast<uint2*>(op + et * 16 + grp * 4) = u;
        }
      }
      if (a.lse && grp == 0 && q < g.N) a.lse[((long)dfk_bid_x()) * g.Np + q] = (m[qh] + __log2f(l)) * 0.6931471805599453f;
    }
  }
}

// ------------------------------------------------------- bias tables (bf16 path)
// Per (shift class, head): the window's additive score bias in units of the raw product q.k,
//   (rpb[pos(q) - pos(k) + C0] + (label(q) != label(k) ? -100 : 0)) / scale,   -inf for keys >= N,
// as fp32, stored in the lane order of the MFMA accumulators it initialises (the C input of S), so
// the softmax loops read one 16-B vector per lane per tile and never gather, decode or compare:
//   fwd (key on the accumulator row, query on the lane): [c][h][Np/16][Np/32][64 lanes][8]
//       slot j = 4*h2 + r  <->  q = 16*qt + (lane&15),  k = 32*kb + 16*h2 + 4*(lane>>4) + r
//   bwd (query on the row, key on the lane):             [c][h][Np/32][Np/32][64 lanes][16]
//       slot j = 8*qh + 4*h2 + r  <->  q = 32*qb + 16*qh + 4*(lane>>4) + r,  k = 32*kb + 16*h2 + (lane&15)
// Shift class: one bit per shifted dim, set for the last window along it — the only window whose
// tokens straddle two regions of compute_mask (video_swin_transformer.py:319-333); interior windows
// are class 0 (no mask).  Labels and RPB positions are arithmetic (Q3: positions decode with the full
// window geometry; Q4: -100, not -inf).
struct TabGeo {
  int ncls;      // 8 when any shift > 0, else 1
  long per_ch;   // fwd (= bwd) entries per (class, head) = Np * Np
};

// table-kernel token record: RPB position << 3 | straddle bits (d, h, w: the token lies past the region
// split of the last window along that dim)
__device__ __forceinline__ int tab_token(const dfk_wattn_args& a, int i) {
  const int fd = i / (a.fh * a.fw), fh = (i / a.fw) % a.fh, fw = i % a.fw;
  const int pos = (fd * (2 * a.fh - 1) + fh) * (2 * a.fw - 1) + fw;
  const int td = i / (a.wh * a.ww), th = (i / a.ww) % a.wh, tw = i % a.ww;
  const int bits = (a.sd > 0 && td >= a.wd - a.sd ? 4 : 0) | (a.sh > 0 && th >= a.wh - a.sh ? 2 : 0) |
                   (a.sw > 0 && tw >= a.ww - a.sw ? 1 : 0);
  return pos << 3 | bits;
}

TabGeo tab_geo(const dfk_wattn_args& a, const Geo& g) {
  TabGeo t;
  t.ncls = g.use_mask ? 8 : 1;
  t.per_ch = (long)g.Np * g.Np;
  return t;
}

// table elements (fp32) of one layout
long tab_elems(const dfk_wattn_args& a, const Geo& g) {
  const TabGeo t = tab_geo(a, g);
  return (long)t.ncls * a.heads * t.per_ch;
}

// bf16 tables, fwd layout then bwd layout
long tab3_bytes(const dfk_wattn_args& a, const Geo& g) { return 2L * 2 * tab_elems(a, g); }
bf16raw* tab3_fwd(const dfk_wattn_args& a, const Geo& g) { return reinterpret_cast<bf16raw*>(a.tab); }

// the window's shift class (table index): one bit per shifted dim, set for the last window along it
__device__ __forceinline__ int win_class(const dfk_wattn_args& a, const Geo& g, int win) {
  if (!g.use_mask) return 0;
  const int wwi = win % g.nww, whi = (win / g.nww) % g.nwh, wdi = win / (g.nww * g.nwh);
  return (a.sd > 0 && wdi == g.nwd - 1 ? 4 : 0) | (a.sh > 0 && whi == g.nwh - 1 ? 2 : 0) |
         (a.sw > 0 && wwi == g.nww - 1 ? 1 : 0);
}

// Work order of the table kernels: units sorted by (shift class, clip, window, head) and dealt to the
// XCDs in contiguous chunks (blocks b and b+8 share an XCD).  The heads of one window run back to back on
// one XCD: head h's q / k / v columns are 2 HD bytes of a 6 C-byte token row, so one head alone uses part
// of every 128-B line it fetches, and its siblings take the rest from that XCD's L2 instead of fetching
// the line again from HBM.  A class's tables (heads x Np^2 bf16, ~1 MB at stage 1) stay L2-resident too.
struct WUnit {
  int b, win, head, cls, qpart;
  long lse_unit;   // (b*nW + win)*heads + head: the lse row, as the table-free kernels index it
};

__device__ __forceinline__ WUnit decode_unit(const dfk_wattn_args& a, const Geo& g, int qsplit) {
  const int total = dfk_gdim_x(), bid = dfk_bid_x();
  const int xcd = bid & 7, per = total >> 3, rr = total & 7;
  int u = (xcd < rr ? xcd * (per + 1) : rr * (per + 1) + (xcd - rr) * per) + (bid >> 3);
  WUnit w;
  w.qpart = u % qsplit;
  u /= qsplit;
  const int ncls = g.use_mask ? 8 : 1;
  int c = 0, nd = g.nwd, nh = g.nwh, nw = g.nww;
  for (; c < ncls; ++c) {
    nd = g.use_mask ? ((c & 4) ? (a.sd > 0) : g.nwd - (a.sd > 0)) : g.nwd;
    nh = g.use_mask ? ((c & 2) ? (a.sh > 0) : g.nwh - (a.sh > 0)) : g.nwh;
    nw = g.use_mask ? ((c & 1) ? (a.sw > 0) : g.nww - (a.sw > 0)) : g.nww;
    const int cnt = nd * nh * nw * a.B * a.heads;
    if (u < cnt) break;
    u -= cnt;
  }
  const int perw = nd * nh * nw;
  w.head = u % a.heads;
  u /= a.heads;
  w.b = u / perw;
  u %= perw;
  const int id = u / (nh * nw), ih = (u / nw) % nh, iw = u % nw;
  const int wdi = (c & 4) ? g.nwd - 1 : id, whi = (c & 2) ? g.nwh - 1 : ih, wwi = (c & 1) ? g.nww - 1 : iw;
  w.win = (wdi * g.nwh + whi) * g.nww + wwi;
  w.cls = c;
  w.lse_unit = ((long)w.b * g.nW + w.win) * a.heads + w.head;
  return w;
}

// Backward work groups (dRPB): one workgroup runs G windows of one (shift class, head) in turn and adds their dS^T
// into ONE slab of the dRPB scratch (the first window stores, the later ones read-modify-write the same tiles, which
// the same lanes wrote: a fixed order, no atomics), so the scratch and its reduction shrink G-fold.  Classes in the
// forward's order; inside a class, head innermost (consecutive workgroups gather the same qkv rows).
struct WGroup {
  int cls, head, t, n;   // class, head, group index in the class, windows in this group
  int nd, nh, nw;        // the class's window counts
  long slab;             // scratch slab: (groups of the earlier classes + t) * heads + head
};

__device__ __forceinline__ WGroup decode_group(const dfk_wattn_args& a, const Geo& g, int G) {
  const int total = dfk_gdim_x(), bid = dfk_bid_x();
  const int xcd = bid & 7, per = total >> 3, rr = total & 7;
  int u = (xcd < rr ? xcd * (per + 1) : rr * (per + 1) + (xcd - rr) * per) + (bid >> 3);
  const int ncls = g.use_mask ? 8 : 1;
  int c = 0, nd = g.nwd, nh = g.nwh, nw = g.nww;
  long gacc = 0;
  int cntw = 0;
  for (; c < ncls; ++c) {
    nd = g.use_mask ? ((c & 4) ? (a.sd > 0) : g.nwd - (a.sd > 0)) : g.nwd;
    nh = g.use_mask ? ((c & 2) ? (a.sh > 0) : g.nwh - (a.sh > 0)) : g.nwh;
    nw = g.use_mask ? ((c & 1) ? (a.sw > 0) : g.nww - (a.sw > 0)) : g.nww;
    cntw = nd * nh * nw * a.B;
    const int ngr = (cntw + G - 1) / G;
    if (u < ngr * a.heads) break;
    u -= ngr * a.heads;
    gacc += ngr;
  }
  WGroup r;
  r.cls = c;
  r.head = u % a.heads;
  r.t = u / a.heads;
  r.n = min(G, cntw - r.t * G);
  r.nd = nd; r.nh = nh; r.nw = nw;
  r.slab = (gacc + r.t) * a.heads + r.head;
  return r;
}

__device__ __forceinline__ WUnit group_window(const dfk_wattn_args& a, const Geo& g, const WGroup& gr, int G, int gi) {
  const int perw = gr.nd * gr.nh * gr.nw;
  int wl = gr.t * G + gi;
  WUnit w;
  w.qpart = 0;
  w.head = gr.head;
  w.cls = gr.cls;
  w.b = wl / perw;
  wl %= perw;
  const int id = wl / (gr.nh * gr.nw), ih = (wl / gr.nw) % gr.nh, iw = wl % gr.nw;
  const int c = gr.cls;
  const int wdi = (c & 4) ? g.nwd - 1 : id, whi = (c & 2) ? g.nwh - 1 : ih, wwi = (c & 1) ? g.nww - 1 : iw;
  w.win = (wdi * g.nwh + whi) * g.nww + wwi;
  w.lse_unit = ((long)w.b * g.nW + w.win) * a.heads + w.head;
  return w;
}

// wattn.hip is compiled with IEEE mode off and no-NaN semantics (build.py FILE_FLAGS), so fmaxf chains
// become v_max3_f32 without operand canonicalisation.
__device__ __forceinline__ float max3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// max over the 4 lane groups (lanes l, l^16, l^32, l^48) by the gfx950 row / half swaps
__device__ __forceinline__ float grp_max4(float v) {
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float m = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

// ------------------------------------------------- v3: bf16 bias tiles + 32x32x16 MFMA (forward)
// Score bias in log2 units, bf16, in the operand order of the MFMA that adds it:
//   bias'(q, k) = (rpb[pos(q) - pos(k) + C0] + (label(q) != label(k) ? -100 : 0)) * log2(e),
//   -1e4 for keys >= N (finite: the identity product below must never meet an infinity), 0 for queries >= N.
// The tile streams as 2 KB of bf16 (4 KB as fp32).  Forward and backward add it through the C input of the score
// MFMA (unpacked to fp32 on the VALU), so each layout is that accumulator's:
//   fwd layout (v4 / v5, S^T 32x32 accumulator: key on the row, query on the lane) [cls][head][qb][kb][c][64][8]:
//       lane l, element jj, j = 8 c + jj <-> q = 32 qb + (l & 31), k = 32 kb + (j & 3) + 8 (j >> 2) + 4 (l >> 5)
//   fwd16 layout (v6, four 16x16 S^T sub-tiles, dfk_wattn_fwd_policy version 6): same tile size and order,
//       lane l, element j of c <-> q = 32 qb + 16 c + (l & 15), k = 32 kb + 16 (j >> 2) + 4 (l >> 4) + (j & 3)
//   bwd layout (S 32x32 accumulator: query on the row, key on the lane) [cls][head][qb][kb][c][64 lanes][8]:
//       lane l, element jj, j = 8 c + jj <-> q = 32 qb + 8 (j >> 2) + 4 (l >> 5) + (j & 3), k = 32 kb + (l & 31)
//       (r5: through the C input with -L'; it was two identity-operand MFMAs, which the mel windows paid
//        for: mel1 backward 30 -> 25 us, the 392-token windows unchanged)
constexpr float kPadKey = -1.0e4f;

struct ClsMap { int c[8]; };   // the shift classes that occur (the grid's y covers only these)

__global__ __launch_bounds__(256) void wattn_tab3_kernel(const dfk_wattn_args a, const Geo g, bf16raw* __restrict__ tf,
                                                         bf16raw* __restrict__ tb, int fwd16, const ClsMap cm) {
  extern __shared__ int tsm[];
  int* tok = tsm;                                          // [Np]
  float* rp = reinterpret_cast<float*>(tsm + g.Np);        // [L]
  const int h = dfk_bid_y() % a.heads, cls = cm.c[dfk_bid_y() / a.heads], ch = cls * a.heads + h;
  const float pen = -100.f * kLog2e;
  for (int i = dfk_tid(); i < g.Np; i += dfk_bdim()) tok[i] = i < g.N ? tab_token(a, i) : 0;
  for (int l = dfk_tid(); l < g.L; l += dfk_bdim()) rp[l] = a.rpb ? a.rpb[(long)l * a.heads + h] * kLog2e : 0.f;
  __syncthreads();
  auto val = [&](int q, int k) -> float {
    if (k >= g.N) return kPadKey;
    if (q >= g.N) return 0.f;
    const int tq = tok[q], tk = tok[k];
    float v = rp[(tq >> 3) - (tk >> 3) + g.C0];
    if ((tq ^ tk) & cls & 7) v += pen;
    return v;
  };
  const int nkb = g.Np / 32;
  const long slots = (long)g.Np * g.Np / 8;   // 16-B slots per layout per (class, head)
  for (long t = (long)dfk_bid_x() * dfk_bdim() + dfk_tid(); t < 2 * slots; t += (long)dfk_gdim_x() * dfk_bdim()) {
    const bool bwd = t >= slots;
    const long u = bwd ? t - slots : t;
    const int lane = (int)(u & 63), c = (int)((u >> 6) & 1);
    const long blk = u >> 7;
    const int kb = (int)(blk % nkb), qb = (int)(blk / nkb);
    const int rr = lane & 31, hh = lane >> 5;
    uint4 w;
    uint32_t* pw = reinterpret_cast<uint32_t*>(&w);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      float v0, v1;
      if (!bwd && fwd16) {   // v6 (16x16x32 tiles): lane l, c = query half, j = 4 kh + r
        const int qq = qb * 32 + 16 * c + (lane & 15), kq = kb * 32 + 4 * (lane >> 4);
        v0 = val(qq, kq + 16 * (j >> 2) + (j & 3));
        v1 = val(qq, kq + 16 * ((j + 1) >> 2) + ((j + 1) & 3));
      } else if (!bwd) {
        const int j0 = 8 * c + j, j1 = j0 + 1;
        v0 = val(qb * 32 + rr, kb * 32 + (j0 & 3) + 8 * (j0 >> 2) + 4 * hh);
        v1 = val(qb * 32 + rr, kb * 32 + (j1 & 3) + 8 * (j1 >> 2) + 4 * hh);
      } else {
        const int j0 = 8 * c + j, j1 = j0 + 1;   // the C-input layout of the backward's S (key on the lane)
        v0 = val(qb * 32 + 8 * (j0 >> 2) + 4 * hh + (j0 & 3), kb * 32 + rr);
        v1 = val(qb * 32 + 8 * (j1 >> 2) + 4 * hh + (j1 & 3), kb * 32 + rr);
      }
      pw[j >> 1] = (uint32_t)f2bf(v0) | ((uint32_t)f2bf(v1) << 16);
    }
    *reinterpret_cast<uint4*>((bwd ? tb : tf) + ((long)ch * slots + u) * 8) = w;
  }
}

// identity operands of the bias product (B[slot][n] = slot == n - 16c), and the row-sum selector: a
// v_mfma_f32_16x16x32_bf16 A operand (lane l: row l & 15, k = 8 (l >> 4) + j) that is 1 iff row == (l >> 4) & 1,
// so that with a 32x32x16 B fragment X (query l & 31 on the lane) the 16x16 product's row 0 / row 1 hold the
// column sums of X for queries 0-15 / 16-31 — in lanes 0-15, registers 0 / 1 (4 accumulator registers, not 16)
__device__ __forceinline__ void bias_ident(int lane, bf16x8& i0, bf16x8& i1, bf16x8& sel) {
  const int r = lane & 31, hh = lane >> 5;
  const float sv = (lane & 15) == ((lane >> 4) & 1) ? 1.f : 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    i0[j] = (__bf16)(8 * hh + j == r ? 1.f : 0.f);
    i1[j] = (__bf16)(8 * hh + j + 16 == r ? 1.f : 0.f);
    sel[j] = (__bf16)sv;
  }
}

// the row sum of query r (= lane & 31) from the selector accumulator: lane r & 15, register r >> 4
__device__ __forceinline__ float selsum(const f32x4& l4, int lane) {
  const int r = lane & 31;
  const float v0 = __shfl(l4[0], r & 15, 64), v1 = __shfl(l4[1], r & 15, 64);
  return r < 16 ? v0 : v1;
}

// x rounded up (toward +inf) to the nearest bf16 value
__device__ __forceinline__ float bf16_ceil(float x) {
  uint32_t u = __float_as_uint(x);
  const uint32_t lo = u & 0xffffu;
  u &= 0xffff0000u;
  if (lo != 0u && !(u >> 31)) u += 0x10000u;   // positive with dropped bits: one bf16 ulp up
  return __uint_as_float(u);
}

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// Forward v3.  One workgroup = one (clip, window, head) (x qsplit), 4 waves; K and V of the window staged once
// in XOR-swizzled LDS tiles.  Per wave and 32-query block, per 32-key block:
//   D = K Q'^T + bias' - m        (Q' = Q * scale * log2e; -m enters as the C input of the first MFMA: a
//                                  16-register tile held per lane, rewritten only on a rescale)
//   P = 2^D                        (one v_exp per score, no subtract, no multiply)
//   O^T += V^T P^T, l = ones^T P^T (both on the MFMA; P^T is the accumulator tile converted in place)
// with a lazy rescale (m moves only when a block's max exceeds it by kRescale, or on the first block).
// Lane l holds query 32 qb + (l & 31) and keys (j & 3) + 8 (j >> 2) + 4 (l >> 5) of every tile.
template <int HD, bool TAB, bool DROP>
__global__ __launch_bounds__(256, (HD == 32 && !DROP) ? 3 : 2) void wattn_fwd3_kernel(const dfk_wattn_args a, const Geo g, int qsplit,
                                                         const bf16raw* __restrict__ tab) {
  constexpr int NKK = HD / 16, NOT = HD / 32, CH = HD / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* Ks = reinterpret_cast<bf16raw*>(smem);
  bf16raw* Vs = Ks + (size_t)g.Np * HD;
  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5, g16 = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const WUnit wu = decode_unit(a, g, qsplit);
  const int head = wu.head, win = wu.win, b = wu.b;
  const long unit = wu.lse_unit;
  const int hoff = head * HD;
  // K / V gather, KV_B chunks per thread in flight: every load of a batch is issued (clamped, branch-free
  // addresses) before the one wait that precedes its LDS writes — a load / wait / write chain per chunk
  // costs one HBM round trip each (7 K + 7 V per thread at Np 416)
  {
    constexpr int KV_B = 4;
    const int tot = g.Np * CH;
    for (int base = tid; base < tot; base += KV_B * dfk_bdim()) {
      uint4 kv[KV_B], vv[KV_B];
      int off[KV_B];
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        const int idx = min(base + u * (int)dfk_bdim(), tot - 1);
        const int i = idx / CH, c = (idx % CH) * 8;
        const int row = token_info_row(a, g, b, win, i);
        off[u] = swz<HD>(i, c);
        kv[u] = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
        vv[u] = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
      }
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        if (base + u * (int)dfk_bdim() < tot) {
          *reinterpret_cast<uint4*>(Ks + off[u]) = kv[u];
          *reinterpret_cast<uint4*>(Vs + off[u]) = vv[u];
        }
      }
    }
  }
  const int nkb = g.Np / 32, nqb = g.Np / 32;
  const bf16raw* tch = TAB ? tab + ((long)wu.cls * a.heads + head) * (long)g.Np * g.Np : nullptr;
  bf16x8 id0, id1, sel;
  bias_ident(lane, id0, id1, sel);
  const float qs = a.scale * kLog2e;
  const DropCtx dc = drop_ctx(a.drop);
  __syncthreads();

  const int nw = dfk_bdim() >> 6, qstep = nw * qsplit;
  int qrown;
  bf16x8 qfn[NKK];
  auto load_q = [&](int qb) {   // Q'^T B operands of query 32 qb + r: elements 8 hh + j of each 16-wide k-step
    const int q = qb * 32 + r;
    qrown = q < g.N ? token_info_row(a, g, b, win, q) : -2;
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk)
      qfn[kk] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.q, a.pad_q, qrown, a.ld_qkv, hoff + kk * 16 + hh * 8));
  };
  // per-lane LDS offsets of the K fragments and of the V^T tr16 reads: the tile swizzle depends on the row
  // only through (row >> 2) & 3 (hd 32) or row & 3, (row >> 2) & 1 (hd 64), which a key block's 32-row
  // step and the 16-row k-step leave unchanged, so one offset serves every block (+ kb 32 HD + 16 c HD)
  int koff[NKK], vlo[NOT], vhi[NOT];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) koff[kk] = swz<HD>(r, kk * 16 + hh * 8);
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int k0 = 4 * (g16 >> 1) + tq, col = ot * 32 + 16 * (g16 & 1) + 4 * tp;
    vlo[ot] = swz<HD>(k0, col);
    vhi[ot] = swz<HD>(k0 + 8, col);
  }
  // -m enters the scores as one more MFMA k-step, A[k][slot] = (slot == 0), B[slot][q] = -m (slot 0): m is
  // kept bf16-representable (rounded up), so the product is exact and the score tile needs no C input copy
  bf16x8 onesA;
#pragma unroll
  for (int j = 0; j < 8; ++j) onesA[j] = (__bf16)(hh == 0 && j == 0 ? 1.f : 0.f);
  // bias tiles through a buffer descriptor: the lane's 16 B in a VGPR offset, the (qb, kb) tile in an SGPR
  const uint64_t tp64 = reinterpret_cast<uint64_t>(tch);   // wave-uniform: keep the descriptor in SGPRs
  const uint64_t tpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp64 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tp64);   // no sign extension
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tpu), (short)0, TAB ? 0x7fffffff : 0, 0x00020000);
  load_q(min(wu.qpart * nw + wave, nqb - 1));
  for (int qb = wu.qpart * nw + wave; qb < nqb; qb += qstep) {
    const int qrow = qrown;
    bf16x8 qf[NKK];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[kk][j] = (__bf16)((float)qfn[kk][j] * qs);
    }
    load_q(min(qb + qstep, nqb - 1));
    auto load_bias = [&](bf16x8 (&bt)[2], int kb) {
      if constexpr (TAB) {
        const int so = __builtin_amdgcn_readfirstlane((qb * nkb + kb) * 2048);   // bytes: 1024 bf16 per (qb, kb)
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bt[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(trs, lane * 16, so + c * 1024, 0));
      }
    };
    f32x16 o[NOT];
    f32x4 l4 = f32x4{0.f, 0.f, 0.f, 0.f};
    float m = 0.f;
    bf16x8 mB;
#pragma unroll
    for (int j = 0; j < 8; ++j) mB[j] = (__bf16)0.f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int j = 0; j < 16; ++j) o[ot][j] = 0.f;
    bf16x8 bt[2];
    load_bias(bt, 0);
    auto block = [&](int kb) {
      const bf16raw* kbase = Ks + kb * 32 * HD;
      const bf16raw* vbase = Vs + kb * 32 * HD;
      // D = K Q'^T + bias' - m
      f32x16 d = mfma32(onesA, mB, f32x16{});
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) d = mfma32(*reinterpret_cast<const bf16x8*>(kbase + koff[kk]), qf[kk], d);
      if constexpr (TAB) {
        d = mfma32(bt[0], id0, d);
        d = mfma32(bt[1], id1, d);
        load_bias(bt, min(kb + 1, nkb - 1));   // next block's tile: in flight under this block's softmax and PV
      } else {
        if (kb == nkb - 1) {   // keys beyond N (no table: the only padded key block)
#pragma unroll
          for (int j = 0; j < 16; ++j)
            if (kb * 32 + (j & 3) + 8 * (j >> 2) + 4 * hh >= g.N) d[j] = -INFINITY;
        }
      }
      // lazy rescale: the block max relative to m (lanes l and l^32 hold the same query)
      float x0 = max3f(d[0], d[1], d[2]), x1 = max3f(d[3], d[4], d[5]), x2 = max3f(d[6], d[7], d[8]);
      float x3 = max3f(d[9], d[10], d[11]), x4 = max3f(d[12], d[13], d[14]);
      float bm = max3f(max3f(x0, x1, x2), max3f(x3, x4, d[15]), -INFINITY);
      const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(bm), __float_as_uint(bm), false, false);
      bm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
      const bool grow = kb == 0 || bm > kRescale;
      if (__builtin_amdgcn_ballot_w64(grow) != 0) {
        // m' = m + bm rounded up to a bf16 value: every exponent of this block stays <= 0
        const float mn = grow ? bf16_ceil(m + bm) : m;
        const float delta = mn - m;
        const float alpha = kb == 0 ? 0.f : __builtin_amdgcn_exp2f(-delta);
        m = mn;
        mB[0] = (__bf16)(hh == 0 ? -m : 0.f);
#pragma unroll
        for (int j = 0; j < 16; ++j) d[j] -= delta;
        // the row sums sit in lanes 0-15 (queries 0-15 in register 0, 16-31 in register 1): their factors
        const float a0 = __shfl(alpha, lane & 15, 64), a1 = __shfl(alpha, (lane & 15) + 16, 64);
        l4[0] *= a0;
        l4[1] *= a1;
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int j = 0; j < 16; ++j) o[ot][j] *= alpha;
      }
      // P = 2^D as the B operand of k-steps c = 0, 1 (registers 8c .. 8c+7)
      bf16x8 pf[2], pv[2];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[c][j] = (__bf16)__builtin_amdgcn_exp2f(d[8 * c + j]);
      if constexpr (DROP) {   // O accumulates the dropped probabilities, l the undropped ones
        const long qrow_id = unit * g.Np + qb * 32 + r;
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j)
            pv[c][j] = (__bf16)((float)pf[c][j] * drop_mul(dc, qrow_id, kb * 32 + 16 * c + 8 * (j >> 2) + 4 * hh + (j & 3)));
      } else {
        pv[0] = pf[0];
        pv[1] = pf[1];
      }
      // O^T += V^T P^T: A operand rows e = 32 ot + r, k-step c slots 8 hh + j <-> keys 16 c + 8 (j>>2) + 4 hh + (j&3)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const bf16x8 va = tr16x2(vbase + c * 16 * HD + vlo[ot], vbase + c * 16 * HD + vhi[ot]);
          o[ot] = mfma32(va, pv[c], o[ot]);
        }
        l4 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sel, pf[c], l4, 0, 0, 0);
      }
    };
    for (int kb = 0; kb < nkb; ++kb) block(kb);
    // O = O^T / l: lane holds e = 32 ot + (j & 3) + 8 (j >> 2) + 4 hh of query r
    const float l = selsum(l4, lane);
    const float inv = 1.f / l;
    if (qrow >= 0) {
      bf16raw* op = reinterpret_cast<bf16raw*>(a.out) + (long)qrow * a.ld_out + hoff;
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int jg = 0; jg < 4; ++jg) {
          uint2 u;
          u.x = (uint32_t)f2bf(o[ot][4 * jg] * inv) | ((uint32_t)f2bf(o[ot][4 * jg + 1] * inv) << 16);
          u.y = (uint32_t)f2bf(o[ot][4 * jg + 2] * inv) | ((uint32_t)f2bf(o[ot][4 * jg + 3] * inv) << 16);
          *reinterpret_cast<uint2*>(op + ot * 32 + 8 * jg + 4 * hh) = u;
        }
    }
    const int q = qb * 32 + r;
    if (a.lse && hh == 0 && q < g.N) a.lse[unit * g.Np + q] = (m + __log2f(l)) * 0.6931471805599453f;
  }
}

// Forward v4 (bias tables): v3's structure with the score bias entering as the C input of the first QK^T MFMA and
// the softmax denominator summed on the VALU — per 32x32 block the matrix pipe runs only the 4 algorithmic
// 32x32x16 products (v3: 8 MFMA-equivalents: the -m k-step, two identity-operand bias products and the selector
// row sums besides them, and the bias products sat on the chain QK^T -> bias -> max).  The bias tile arrives one
// block ahead (buffer loads, accumulator order: 2 x 16 B per lane) and is unpacked to fp32 minus m off the chain.
// QB query blocks per wave (2 for hd 32): each key block's K / V fragments are read from LDS once for both, and
// the two independent score -> softmax -> PV chains interleave (the kernel is latency-bound, not MFMA-bound:
// r4f ablations, profiles/attn/r4f_fwd4_ablations.txt).
// Lane l holds query 32 qb + (l & 31) and keys (j & 3) + 8 (j >> 2) + 4 (l >> 5) of every tile; lanes l and l ^ 32
// hold the two key halves of one query, so the per-lane partial sums meet in one permlane32 swap at the end.
template <int HD, bool DROP, int QB>
__global__ __launch_bounds__(256, (HD == 32 && !DROP) ? 3 : 2) void wattn_fwd4_kernel(const dfk_wattn_args a, const Geo g, int qsplit,
                                                         const bf16raw* __restrict__ tab) {
  constexpr int NKK = HD / 16, NOT = HD / 32, CH = HD / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* Ks = reinterpret_cast<bf16raw*>(smem);
  bf16raw* Vs = Ks + (size_t)g.Np * HD;
  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5, g16 = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const WUnit wu = decode_unit(a, g, qsplit);
  const int head = wu.head, win = wu.win, b = wu.b;
  const long unit = wu.lse_unit;
  const int hoff = head * HD;
  {   // K / V gather, KV_B chunks per thread in flight (as v3)
    constexpr int KV_B = 4;
    const int tot = g.Np * CH;
    for (int base = tid; base < tot; base += KV_B * dfk_bdim()) {
      uint4 kv[KV_B], vv[KV_B];
      int off[KV_B];
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        const int idx = min(base + u * (int)dfk_bdim(), tot - 1);
        const int i = idx / CH, c = (idx % CH) * 8;
        const int row = token_info_row(a, g, b, win, i);
        off[u] = swz<HD>(i, c);
#ifdef DFK_ABL_NOGATHER
        kv[u] = make_uint4(row, c, 0, 0); vv[u] = kv[u];
#else
        kv[u] = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
        vv[u] = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
#endif
      }
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        if (base + u * (int)dfk_bdim() < tot) {
          *reinterpret_cast<uint4*>(Ks + off[u]) = kv[u];
          *reinterpret_cast<uint4*>(Vs + off[u]) = vv[u];
        }
      }
    }
  }
  const int nkb = g.Np / 32, nqb = g.Np / 32, ngrp = (nqb + QB - 1) / QB;
  const bf16raw* tch = tab + ((long)wu.cls * a.heads + head) * (long)g.Np * g.Np;
  const float qs = a.scale * kLog2e;
  const DropCtx dc = drop_ctx(a.drop);
  __syncthreads();

  const int nw = dfk_bdim() >> 6, qstep = nw * qsplit;
  int qrown[QB];
  bf16x8 qfn[QB][NKK];
  // query group gi = query blocks QB gi .. QB gi + QB - 1 (clamped: a group past the last block recomputes it
  // and stores nothing)
  auto load_q = [&](int gi) {
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const int q = min(gi * QB + u, nqb - 1) * 32 + r;
      qrown[u] = q < g.N ? token_info_row(a, g, b, win, q) : -2;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
        qfn[u][kk] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.q, a.pad_q, qrown[u], a.ld_qkv, hoff + kk * 16 + hh * 8));
    }
  };
  int koff[NKK], vlo[NOT], vhi[NOT];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) koff[kk] = swz<HD>(r, kk * 16 + hh * 8);
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int k0 = 4 * (g16 >> 1) + tq, col = ot * 32 + 16 * (g16 & 1) + 4 * tp;
    vlo[ot] = swz<HD>(k0, col);
    vhi[ot] = swz<HD>(k0 + 8, col);
  }
  const uint64_t tp64 = reinterpret_cast<uint64_t>(tch);
  const uint64_t tpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp64 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tp64);
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tpu), (short)0, 0x7fffffff, 0x00020000);
  // QB == 1: the next group's Q is prefetched under this group's blocks; QB == 2 loads it at the group's start
  // (the 16 prefetch VGPRs would push the two-chain kernel past the 3-workgroup register budget)
  if constexpr (QB == 1) load_q(min(wu.qpart * nw + wave, ngrp - 1));
#ifdef DFK_ABL_NOCOMPUTE
  if (wave == -7)
#endif
  for (int gi = wu.qpart * nw + wave; gi < ngrp; gi += qstep) {
    int qbs[QB], qrow[QB];
    bf16x8 qf[QB][NKK];
    if constexpr (QB > 1) load_q(gi);
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      qbs[u] = min(gi * QB + u, nqb - 1);
      qrow[u] = gi * QB + u < nqb ? qrown[u] : -1;
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
        for (int j = 0; j < 8; ++j) qf[u][kk][j] = (__bf16)((float)qfn[u][kk][j] * qs);
    }
    if constexpr (QB == 1) load_q(min(gi + qstep, ngrp - 1));
    auto load_bias = [&](uint4 (&bt)[QB][2], int kb) {
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const int so = __builtin_amdgcn_readfirstlane((qbs[u] * nkb + kb) * 2048);   // bytes: 1024 bf16 per tile
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#ifdef DFK_ABL_NOBIAS
          bt[u][c] = make_uint4(so, c, 0, 0);
#else
          bt[u][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trs, lane * 16, so + c * 1024, 0));
#endif
        }
      }
    };
    f32x16 o[QB][NOT];
    float lsum[QB], m[QB];
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      lsum[u] = 0.f;
      m[u] = 0.f;
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int j = 0; j < 16; ++j) o[u][ot][j] = 0.f;
    }
    uint4 bt[QB][2];
    load_bias(bt, 0);
    for (int kb = 0; kb < nkb; ++kb) {
      const bf16raw* kbase = Ks + kb * 32 * HD;
      const bf16raw* vbase = Vs + kb * 32 * HD;
      bf16x8 kf[NKK];
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) kf[kk] = *reinterpret_cast<const bf16x8*>(kbase + koff[kk]);
      // C input: bias' - m (bf16 pairs unpacked by shift / mask), then D = K Q'^T + bias' - m
      f32x16 d[QB];
#pragma unroll
      for (int u = 0; u < QB; ++u)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t w[4] = {bt[u][c].x, bt[u][c].y, bt[u][c].z, bt[u][c].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            d[u][8 * c + 2 * i] = __uint_as_float(w[i] << 16) - m[u];
            d[u][8 * c + 2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u) - m[u];
          }
        }
      load_bias(bt, min(kb + 1, nkb - 1));   // next block's tiles: in flight under this block's softmax and PV
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk)
#pragma unroll
        for (int u = 0; u < QB; ++u) d[u] = mfma32(kf[kk], qf[u][kk], d[u]);
      bf16x8 va[2][NOT];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) va[c][ot] = tr16x2(vbase + c * 16 * HD + vlo[ot], vbase + c * 16 * HD + vhi[ot]);
      bf16x8 pv[QB][2];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        float x0 = max3f(d[u][0], d[u][1], d[u][2]), x1 = max3f(d[u][3], d[u][4], d[u][5]);
        float x2 = max3f(d[u][6], d[u][7], d[u][8]), x3 = max3f(d[u][9], d[u][10], d[u][11]);
        float x4 = max3f(d[u][12], d[u][13], d[u][14]);
        float bm = max3f(max3f(x0, x1, x2), max3f(x3, x4, d[u][15]), -INFINITY);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(bm), __float_as_uint(bm), false, false);
        bm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
        const bool grow = kb == 0 || bm > kRescale;
        if (__builtin_amdgcn_ballot_w64(grow) != 0) {
          const float mn = grow ? bf16_ceil(m[u] + bm) : m[u];
          const float delta = mn - m[u];
          const float alpha = kb == 0 ? 0.f : __builtin_amdgcn_exp2f(-delta);
          m[u] = mn;
#pragma unroll
          for (int j = 0; j < 16; ++j) d[u][j] -= delta;
          lsum[u] *= alpha;
#pragma unroll
          for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
            for (int j = 0; j < 16; ++j) o[u][ot][j] *= alpha;
        }
        // P = 2^D as the B operand of k-steps c = 0, 1 (registers 8c .. 8c+7); the denominator sums fp32 P
        float p[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) {
#ifdef DFK_ABL_NOEXP
          p[j] = d[u][j];
#else
          p[j] = __builtin_amdgcn_exp2f(d[u][j]);
#endif
        }
        const float s0 = (p[0] + p[1]) + (p[2] + p[3]), s1 = (p[4] + p[5]) + (p[6] + p[7]);
        const float s2 = (p[8] + p[9]) + (p[10] + p[11]), s3 = (p[12] + p[13]) + (p[14] + p[15]);
        lsum[u] += (s0 + s1) + (s2 + s3);
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float pj = p[8 * c + j];
            if constexpr (DROP)   // O accumulates the dropped probabilities, the denominator the undropped ones
              pj *= drop_mul(dc, unit * g.Np + qbs[u] * 32 + r, kb * 32 + 16 * c + 8 * (j >> 2) + 4 * hh + (j & 3));
            pv[u][c][j] = (__bf16)pj;
          }
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int u = 0; u < QB; ++u) o[u][ot] = mfma32(va[c][ot], pv[u][c], o[u][ot]);
    }
#pragma unroll
    for (int u = 0; u < QB; ++u) {
      const auto ls = __builtin_amdgcn_permlane32_swap(__float_as_uint(lsum[u]), __float_as_uint(lsum[u]), false, false);
      const float l = __uint_as_float(ls[0]) + __uint_as_float(ls[1]);
      const float inv = 1.f / l;
      if (qrow[u] >= 0) {
        bf16raw* op = reinterpret_cast<bf16raw*>(a.out) + (long)qrow[u] * a.ld_out + hoff;
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
          for (int jg = 0; jg < 4; ++jg) {
            uint2 w;
            w.x = (uint32_t)f2bf(o[u][ot][4 * jg] * inv) | ((uint32_t)f2bf(o[u][ot][4 * jg + 1] * inv) << 16);
            w.y = (uint32_t)f2bf(o[u][ot][4 * jg + 2] * inv) | ((uint32_t)f2bf(o[u][ot][4 * jg + 3] * inv) << 16);
            *reinterpret_cast<uint2*>(op + ot * 32 + 8 * jg + 4 * hh) = w;
          }
      }
      const int q = qbs[u] * 32 + r;
      if (a.lse && hh == 0 && q < g.N && gi * QB + u < nqb) a.lse[unit * g.Np + q] = (m[u] + __log2f(l)) * 0.6931471805599453f;
    }
  }
}

// Forward v5 (hd 32, bias tables, no dropout): v4 without the running maximum.  The scores are in log2 units
// (Q' = Q * scale * log2e, bias' = bias * log2e), and for every row a trained Swin layer produces they lie many
// binades inside fp32's exponent range, so P = 2^(S' + bias') is formed with NO max subtraction at all: no
// v_max3 reduction and permlane swap between the QK^T MFMAs and the v_exp (the old critical path), no rescale
// test, no -m in the C input — per 32x32 block and chain the VALU runs 16 bias unpacks, 16 v_exp, 15 adds and
// 8 packs (v4: +16 subtracts, ~9 max steps and the rescale ballot).  Exactness is checked, not assumed: a row is
// accepted when its denominator l = sum_k 2^(S'+bias') lies in [2^-80, 2^100] (no infinity / NaN reached the
// accumulators, and an element flushed to zero below 2^-126 weighs < 2^-37 of the row); any other row sends its
// whole query block through v4's max-subtracted loop (the SAFE instantiation of the same loop), so the output is
// the softmax the reference computes for every input.
// With no running max, partial (O, l) over disjoint key ranges simply add.  That balances the launch (BAL): with
// nqb query blocks = 2 * pairs + tail, waves 0-3 first run one full pair each (two chains sharing the K / V
// fragments, as v4), then the 2 remaining pairs are split into key halves and the tail block into key quarters
// over the 4 waves; the partials meet in LDS (the K / V tiles' space, free by then) and three waves finish the
// blocks.  Stage 1 (13 query blocks): every wave runs 13 pair steps + 7 pair steps + 3-4 single steps, against
// v4's 7 groups on 4 waves (waves 0-2 two groups, wave 3 one, block 12 recomputed as a clamped partner).
constexpr int kF5Slots = 13;   // per wave and lane: 8 float4 of pair partials, 4 of tail partials, 1 of l's

__device__ __forceinline__ bool f5_l_ok(float l) {   // bit test: NaN-proof under this file's no-NaN flags
#ifdef DFK5_ABL   // ablation builds (tools/exp_build.sh): never take the fallback
  return true;
#endif
  const uint32_t u = __float_as_uint(l);
  return u >= 0x17800000u && u <= 0x71800000u;          // 2^-80 <= l <= 2^100, positive, finite
}

template <bool BAL>
__global__ __launch_bounds__(256, 3) void wattn_fwd5_kernel(const dfk_wattn_args a, const Geo g, int qsplit,
                                                           const bf16raw* __restrict__ tab) {
  constexpr int HD = 32, CH = HD / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* Ks = reinterpret_cast<bf16raw*>(smem);
  bf16raw* Vs = Ks + (size_t)g.Np * HD;
  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5, g16 = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const WUnit wu = decode_unit(a, g, qsplit);
  const int head = wu.head, win = wu.win, b = wu.b;
  const long unit = wu.lse_unit;
  const int hoff = head * HD;
  auto gather = [&]() __attribute__((always_inline)) {   // K / V of the window -> swizzled LDS tiles, 4 chunks per thread in flight (as v4)
    constexpr int KV_B = 4;
    const int tot = g.Np * CH;
    for (int base = tid; base < tot; base += KV_B * dfk_bdim()) {
      uint4 kv[KV_B], vv[KV_B];
      int off[KV_B];
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        const int idx = min(base + u * (int)dfk_bdim(), tot - 1);
        const int i = idx / CH, c = (idx % CH) * 8;
        const int row = token_info_row(a, g, b, win, i);
        off[u] = swz<HD>(i, c);
        kv[u] = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
        vv[u] = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
      }
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        if (base + u * (int)dfk_bdim() < tot) {
          *reinterpret_cast<uint4*>(Ks + off[u]) = kv[u];
          *reinterpret_cast<uint4*>(Vs + off[u]) = vv[u];
        }
      }
    }
  };
  gather();
  const int nkb = g.Np / 32, nqb = nkb;
  const bf16raw* tch = tab + ((long)wu.cls * a.heads + head) * (long)g.Np * g.Np;
  const float qs = a.scale * kLog2e;
  int koff[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) koff[kk] = swz<HD>(r, kk * 16 + hh * 8);
  const int vk0 = 4 * (g16 >> 1) + tq, vcol = 16 * (g16 & 1) + 4 * tp;
  const int vlo = swz<HD>(vk0, vcol), vhi = swz<HD>(vk0 + 8, vcol);
  const uint64_t tp64 = reinterpret_cast<uint64_t>(tch);
  const uint64_t tpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp64 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tp64);
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tpu), (short)0, 0x7fffffff, 0x00020000);
  __syncthreads();

  // scaled Q fragment of query block qb (B operand: lane holds query 32 qb + r, k-slots 16 kk + 8 hh ..); its row
  auto load_q = [&](int qb, bf16x8 (&qf)[2]) __attribute__((always_inline)) -> int {
    const int q = qb * 32 + r;
    const int row = q < g.N ? token_info_row(a, g, b, win, q) : -2;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const bf16x8 raw = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.q, a.pad_q, row, a.ld_qkv, hoff + kk * 16 + hh * 8));
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[kk][j] = (__bf16)((float)raw[j] * qs);
    }
    return row;
  };

  // NC chains (query blocks qb[0..NC-1]) over key blocks [k0, k1): O^T, the lane's partial row sums and (SAFE
  // only) the running max accumulate into o / ls / m.  SAFE is v4's loop (k0 = 0 there).
  auto chains = [&](auto nc_t, auto safe_t, const int (&qb)[2], const bf16x8 (&qf)[2][2], int k0, int k1,
                    f32x16 (&o)[2], float (&ls)[2], float (&m)[2]) __attribute__((always_inline)) {
    constexpr int NC = decltype(nc_t)::value;
    constexpr bool SAFE = decltype(safe_t)::value;
    auto load_bias = [&](uint4 (&bt)[2][2], int kb) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        const int so = __builtin_amdgcn_readfirstlane((qb[u] * nkb + kb) * 2048);   // bytes: 1024 bf16 per tile
#pragma unroll
        for (int c = 0; c < 2; ++c) {
#ifdef DFK5_NOBIAS   // ablation builds only (tools/exp_build.sh)
          if constexpr (!SAFE) { bt[u][c] = make_uint4(so + c, kb, 0, 0); continue; }
#endif
          bt[u][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trs, lane * 16, so + c * 1024, 0));
        }
      }
    };
    uint4 bt[2][2];
    load_bias(bt, k0);
    for (int kb = k0; kb < k1; ++kb) {
      const bf16raw* kbase = Ks + kb * 32 * HD;
      const bf16raw* vbase = Vs + kb * 32 * HD;
      bf16x8 kf[2];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) kf[kk] = *reinterpret_cast<const bf16x8*>(kbase + koff[kk]);
#ifdef DFK5_NOKV
      if constexpr (!SAFE) for (int kk = 0; kk < 2; ++kk) for (int j = 0; j < 8; ++j) kf[kk][j] = (__bf16)(float)(kb + j);
#endif
      f32x16 d[2];
#pragma unroll
      for (int u = 0; u < NC; ++u)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t w[4] = {bt[u][c].x, bt[u][c].y, bt[u][c].z, bt[u][c].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            d[u][8 * c + 2 * i] = __uint_as_float(w[i] << 16);
            d[u][8 * c + 2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
            if constexpr (SAFE) {
              d[u][8 * c + 2 * i] -= m[u];
              d[u][8 * c + 2 * i + 1] -= m[u];
            }
          }
        }
      load_bias(bt, min(kb + 1, k1 - 1));   // next block's tiles: in flight under this block's softmax and PV
#ifdef DFK5_NOQK
      if constexpr (SAFE)
#endif
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int u = 0; u < NC; ++u) d[u] = mfma32(kf[kk], qf[u][kk], d[u]);
      bf16x8 va[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) va[c] = tr16x2(vbase + c * 16 * HD + vlo, vbase + c * 16 * HD + vhi);
#ifdef DFK5_NOKV
      if constexpr (!SAFE) for (int c = 0; c < 2; ++c) for (int j = 0; j < 8; ++j) va[c][j] = (__bf16)(float)(kb - j);
#endif
      bf16x8 pv[2][2];
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        if constexpr (SAFE) {
          float x0 = max3f(d[u][0], d[u][1], d[u][2]), x1 = max3f(d[u][3], d[u][4], d[u][5]);
          float x2 = max3f(d[u][6], d[u][7], d[u][8]), x3 = max3f(d[u][9], d[u][10], d[u][11]);
          float x4 = max3f(d[u][12], d[u][13], d[u][14]);
          float bm = max3f(max3f(x0, x1, x2), max3f(x3, x4, d[u][15]), -INFINITY);
          const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(bm), __float_as_uint(bm), false, false);
          bm = fmaxf(__uint_as_float(sw[0]), __uint_as_float(sw[1]));
          const bool grow = kb == k0 || bm > kRescale;
          if (__builtin_amdgcn_ballot_w64(grow) != 0) {
            const float mn = grow ? bf16_ceil(m[u] + bm) : m[u];
            const float delta = mn - m[u];
            const float alpha = kb == k0 ? 0.f : __builtin_amdgcn_exp2f(-delta);
            m[u] = mn;
#pragma unroll
            for (int j = 0; j < 16; ++j) d[u][j] -= delta;
            ls[u] *= alpha;
#pragma unroll
            for (int j = 0; j < 16; ++j) o[u][j] *= alpha;
          }
        }
        float p[16];
#pragma unroll
        for (int j = 0; j < 16; ++j) p[j] = __builtin_amdgcn_exp2f(d[u][j]);
#ifdef DFK5_NOEXP
        if constexpr (!SAFE) for (int j = 0; j < 16; ++j) p[j] = d[u][j];
#endif
        const float s0 = (p[0] + p[1]) + (p[2] + p[3]), s1 = (p[4] + p[5]) + (p[6] + p[7]);
        const float s2 = (p[8] + p[9]) + (p[10] + p[11]), s3 = (p[12] + p[13]) + (p[14] + p[15]);
        ls[u] += (s0 + s1) + (s2 + s3);
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[u][c][j] = (__bf16)p[8 * c + j];
      }
#ifdef DFK5_NOPV
      if constexpr (!SAFE) {
        for (int u = 0; u < NC; ++u) for (int j = 0; j < 8; ++j) o[u][j] += (float)pv[u][0][j] + (float)pv[u][1][j] + (float)va[0][j] + (float)va[1][j];
        continue;
      }
#endif
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int u = 0; u < NC; ++u) o[u] = mfma32(va[c], pv[u][c], o[u]);
    }
  };
  auto zero = [&](f32x16 (&o)[2], float (&ls)[2], float (&m)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      ls[u] = 0.f;
      m[u] = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) o[u][j] = 0.f;
    }
  };
  // O = O^T / l for query block qb (lane: query 32 qb + r, channels 8 jg + 4 hh + 0..3), lse; true: l rejected
  auto store = [&](int qb, int qrow, const f32x16& o, float ls, float m, bool real = true) __attribute__((always_inline)) -> bool {
    if (!real) return false;   // a clamped duplicate block: nothing stored
    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(ls), __float_as_uint(ls), false, false);
    const float l = __uint_as_float(sw[0]) + __uint_as_float(sw[1]);
    const float inv = 1.f / l;
    if (qrow >= 0) {
      bf16raw* op = reinterpret_cast<bf16raw*>(a.out) + (long)qrow * a.ld_out + hoff;
#pragma unroll
      for (int jg = 0; jg < 4; ++jg) {
        uint2 w;
        w.x = (uint32_t)f2bf(o[4 * jg] * inv) | ((uint32_t)f2bf(o[4 * jg + 1] * inv) << 16);
        w.y = (uint32_t)f2bf(o[4 * jg + 2] * inv) | ((uint32_t)f2bf(o[4 * jg + 3] * inv) << 16);
        *reinterpret_cast<uint2*>(op + 8 * jg + 4 * hh) = w;
      }
    }
    const int q = qb * 32 + r;
    if (a.lse && hh == 0 && q < g.N) a.lse[unit * g.Np + q] = (m + __log2f(l)) * 0.6931471805599453f;
    return !f5_l_ok(l);
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using FAST = std::false_type;
  using SAFE = std::true_type;
  // one query block through v4's max-subtracted loop (one chain: the retry must not raise the fast path's
  // register budget)
  auto safe_block = [&](int qb) __attribute__((always_inline)) {
    const int qbs[2] = {qb, qb};
    bf16x8 qf[2][2];
    const int row = load_q(qb, qf[0]);
    f32x16 o[2];
    float ls[2], m[2];
    zero(o, ls, m);
    chains(I1{}, SAFE{}, qbs, qf, 0, nkb, o, ls, m);
    store(qb, row, o[0], ls[0], m[0]);
  };
  // one pair (or a single block) over every key, fast; v4's loop again when a row is rejected
  auto full = [&](int qb0, int qb1) __attribute__((always_inline)) {
    const int qb[2] = {qb0, min(qb1, nqb - 1)};
    bf16x8 qf[2][2];
    int qrow[2];
    qrow[0] = load_q(qb[0], qf[0]);
    qrow[1] = load_q(qb[1], qf[1]);
    f32x16 o[2];
    float ls[2], m[2];
    zero(o, ls, m);
    chains(I2{}, FAST{}, qb, qf, 0, nkb, o, ls, m);
    bool bad = store(qb[0], qrow[0], o[0], ls[0], m[0]);
    bad |= store(qb[1], qrow[1], o[1], ls[1], m[1], qb1 < nqb);
    if (__builtin_amdgcn_ballot_w64(bad) != 0) {
      safe_block(qb[0]);
      if (qb1 < nqb) safe_block(qb1);
    }
  };
  const int nw = dfk_bdim() >> 6;
  if constexpr (!BAL) {
    const int ngrp = (nqb + 1) / 2, qstep = nw * qsplit;
    for (int gi = wu.qpart * nw + wave; gi < ngrp; gi += qstep) full(2 * gi, 2 * gi + 1);
    return;
  } else {
    // host guarantees: qsplit == 1, 4 waves, pairs % 4 in {0, 1, 2}, LDS >= 4 x kF5Slots KB
    // the fallback flag sits past the K / V tiles and the partial slots (dynamic LDS: a static __shared__
    // variable would make the 160 KB dynamic-size attribute fail for this kernel)
    int& f5_flag = *reinterpret_cast<int*>(smem + max(4 * g.Np * HD, 4 * kF5Slots * 1024));
    if (tid == 0) f5_flag = 0;   // read after two more barriers
    const int pairs = nqb / 2, tail = nqb & 1, R = pairs % 4, p1 = pairs - R;
    for (int p = wave; p < p1; p += 4) full(2 * p, 2 * p + 1);
    // phase 2: split pair(s) and the tail block, partial sums only
    f32x16 oa[2], ob[2];
    float la[2], lb[2], ma[2], mb[2];
    zero(oa, la, ma);
    zero(ob, lb, mb);
    const int pa = R == 2 ? p1 + (wave >> 1) : p1;   // this wave's split pair (R > 0)
    if (R > 0) {
      const int ka0 = R == 2 ? ((wave & 1) ? (nkb + 1) / 2 : 0) : (wave * nkb) / 4;
      const int ka1 = R == 2 ? ((wave & 1) ? nkb : (nkb + 1) / 2) : ((wave + 1) * nkb) / 4;
      const int qb[2] = {2 * pa, 2 * pa + 1};
      bf16x8 qf[2][2];
      load_q(qb[0], qf[0]);
      load_q(qb[1], qf[1]);
      chains(I2{}, FAST{}, qb, qf, ka0, ka1, oa, la, ma);
    }
    if (tail) {
      const int qb[2] = {nqb - 1, nqb - 1};
      bf16x8 qf[2][2];
      load_q(qb[0], qf[0]);
      chains(I1{}, FAST{}, qb, qf, (wave * nkb) / 4, ((wave + 1) * nkb) / 4, ob, lb, mb);
    }
    __syncthreads();   // every wave is done with K / V: their space takes the partials
    float4* ps = reinterpret_cast<float4*>(smem);
    auto slot = [&](int w, int s) __attribute__((always_inline)) -> float4* { return ps + (w * kF5Slots + s) * 64 + lane; };
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        *slot(wave, 4 * u + j4) = make_float4(oa[u][4 * j4], oa[u][4 * j4 + 1], oa[u][4 * j4 + 2], oa[u][4 * j4 + 3]);
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4)
      *slot(wave, 8 + j4) = make_float4(ob[0][4 * j4], ob[0][4 * j4 + 1], ob[0][4 * j4 + 2], ob[0][4 * j4 + 3]);
    *slot(wave, 12) = make_float4(la[0], la[1], lb[0], 0.f);
    __syncthreads();
    // finishers: R == 2: wave 0 (pair p1, halves of waves 0, 1), wave 2 (pair p1 + 1, waves 2, 3), wave 3 (tail);
    // R == 1: wave 0 (pair p1, quarters of all waves), wave 1 (tail); R == 0: wave 0 (tail)
    const bool fin_pair = R == 2 ? (wave == 0 || wave == 2) : (R == 1 && wave == 0);
    const bool fin_tail = tail && wave == (R == 2 ? 3 : (R == 1 ? 1 : 0));
    bool bad2 = false;
    if (fin_pair) {
      const int w0 = R == 2 ? wave : 0, w1 = R == 2 ? wave + 2 : 4;
      f32x16 o[2];
      float ls[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        ls[u] = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) o[u][j] = 0.f;
      }
      for (int w = w0; w < w1; ++w) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j4 = 0; j4 < 4; ++j4) {
            const float4 v = *slot(w, 4 * u + j4);
            o[u][4 * j4] += v.x; o[u][4 * j4 + 1] += v.y; o[u][4 * j4 + 2] += v.z; o[u][4 * j4 + 3] += v.w;
          }
        const float4 lv = *slot(w, 12);
        ls[0] += lv.x;
        ls[1] += lv.y;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int qb = 2 * pa + u, q = qb * 32 + r;
        const int row = q < g.N ? token_info_row(a, g, b, win, q) : -2;
        bad2 |= store(qb, row, o[u], ls[u], 0.f);
      }
    }
    if (fin_tail) {
      f32x16 o;
      float ls = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) o[j] = 0.f;
      for (int w = 0; w < 4; ++w) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const float4 v = *slot(w, 8 + j4);
          o[4 * j4] += v.x; o[4 * j4 + 1] += v.y; o[4 * j4 + 2] += v.z; o[4 * j4 + 3] += v.w;
        }
        ls += slot(w, 12)->z;
      }
      const int q = (nqb - 1) * 32 + r;
      const int row = q < g.N ? token_info_row(a, g, b, win, q) : -2;
      bad2 |= store(nqb - 1, row, o, ls, 0.f);
    }
    // a rejected split block (vanishingly rare): K / V again, and the block through the SAFE loop
    const bool wave_bad = __builtin_amdgcn_ballot_w64(bad2) != 0;   // every lane votes (not under lane == 0)
    if (lane == 0 && wave_bad) f5_flag = 1;
    __syncthreads();
    if (f5_flag) {
      gather();
      __syncthreads();
      if (__builtin_amdgcn_ballot_w64(bad2) != 0) {
        safe_block(fin_pair ? 2 * pa : nqb - 1);
        if (fin_pair) safe_block(2 * pa + 1);
      }
    }
  }
}

// sum over the 4 lane groups (lanes l, l^16, l^32, l^48)
__device__ __forceinline__ float grp_sum4(float v) {
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(r16[0]) + __uint_as_float(r16[1]);
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(r32[0]) + __uint_as_float(r32[1]);
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Forward v6 (hd 32, bias tables, no dropout; experiment, DFK_WATTN_V=6): v5 on v_mfma_f32_16x16x32_bf16.  With
// K = hd = 32 one 16x16x32 product is a whole 16x16 score sub-tile: the four sub-tiles of a 32x32 block are four
// independent MFMAs with no accumulate chain, and each sub-tile's v_exp can start as soon as its own product is
// done (v5's 32x32x16 tile waits on two dependent products before its first v_exp; r5e ablation: that wait is
// ~50 us of the stage-1 launch).  Lane l holds, per chain and query half qh, query 32 qb + 16 qh + (l & 15) and keys
// 16 kh + 4 (l >> 4) + r of each key half kh; the P^T operand of the PV product is the lane's own 8 scores
// (k-slots j <-> key 16 (j >> 2) + 4 (l >> 4) + (j & 3)), and V^T is read with the same slot order by ds_read_tr16.
// Row statistics are per (chain, half) and reduce over the 4 lane groups.  Bias tables in the fwd16 layout
// (wattn_tab3_kernel fwd16: [qh][64 lanes][kh][r]).
// ONES (A/B, non-BAL only): the softmax denominators by a third PV-shaped MFMA with an all-ones A operand (every
// output row = the column's sum of the bf16 P that also multiplies V) instead of 8 VALU adds per query half and
// the lane-group sum at the store: -16 VALU adds per 32x32 block for +2 MFMAs on the matrix pipe, which has slack
// W8 (A/B): up to 8 waves per workgroup (one query-block pair each) instead of 4 looping over the pairs
template <bool BAL, bool ONES = false, bool W8 = false>
__global__ __launch_bounds__(W8 ? 512 : 256, W8 ? 4 : 3) void wattn_fwd6_kernel(const dfk_wattn_args a, const Geo g, int qsplit,
                                                           const bf16raw* __restrict__ tab) {
  constexpr int HD = 32, CH = HD / 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* Ks = reinterpret_cast<bf16raw*>(smem);
  bf16raw* Vs = Ks + (size_t)g.Np * HD;
  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ql = lane & 15, g16 = lane >> 4, tq = ql >> 2, tp = ql & 3;
  const WUnit wu = decode_unit(a, g, qsplit);
  const int head = wu.head, win = wu.win, b = wu.b;
  const long unit = wu.lse_unit;
  const int hoff = head * HD;
  auto gather = [&]() __attribute__((always_inline)) {   // K / V of the window -> swizzled LDS tiles (as v5)
    constexpr int KV_B = 4;
    const int tot = g.Np * CH;
    for (int base = tid; base < tot; base += KV_B * dfk_bdim()) {
      uint4 kv[KV_B], vv[KV_B];
      int off[KV_B];
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        const int idx = min(base + u * (int)dfk_bdim(), tot - 1);
        const int i = idx / CH, c = (idx % CH) * 8;
        const int row = token_info_row(a, g, b, win, i);
        off[u] = swz<HD>(i, c);
        kv[u] = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
        vv[u] = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
      }
#pragma unroll
      for (int u = 0; u < KV_B; ++u) {
        if (base + u * (int)dfk_bdim() < tot) {
          *reinterpret_cast<uint4*>(Ks + off[u]) = kv[u];
          *reinterpret_cast<uint4*>(Vs + off[u]) = vv[u];
        }
      }
    }
  };
  gather();
  const int nkb = g.Np / 32, nqb = nkb;
  const bf16raw* tch = tab + ((long)wu.cls * a.heads + head) * (long)g.Np * g.Np;
  const float qs = a.scale * kLog2e;
  int koff[2], vlo[2], vhi[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    koff[h] = swz<HD>(16 * h + ql, 8 * g16);
    vlo[h] = swz<HD>(4 * g16 + tq, 16 * h + 4 * tp);
    vhi[h] = swz<HD>(16 + 4 * g16 + tq, 16 * h + 4 * tp);
  }
  const uint64_t tp64 = reinterpret_cast<uint64_t>(tch);
  const uint64_t tpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp64 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tp64);
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tpu), (short)0, 0x7fffffff, 0x00020000);
  __syncthreads();

  // scaled Q fragments of query block qb: half qh = B operand of the 16x16x32 products (query 32 qb + 16 qh + ql,
  // channels 8 g16 .. 8 g16 + 7)
  auto load_q = [&](int qb, bf16x8 (&qf)[2]) __attribute__((always_inline)) {
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const int q = qb * 32 + 16 * qh + ql;
      const int row = q < g.N ? token_info_row(a, g, b, win, q) : -2;
      const bf16x8 raw = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.q, a.pad_q, row, a.ld_qkv, hoff + 8 * g16));
#pragma unroll
      for (int j = 0; j < 8; ++j) qf[qh][j] = (__bf16)((float)raw[j] * qs);
    }
  };
  // element index in a chain's 16 registers: scores d[8 qh + 4 kh + r], output o[8 qh + 4 eh + r]
  auto chains = [&](auto nc_t, auto safe_t, const int (&qb)[2], const bf16x8 (&qf)[2][2], int k0, int k1,
                    f32x16 (&o)[2], float (&ls)[2][2], float (&m)[2][2]) __attribute__((always_inline)) {
    constexpr int NC = decltype(nc_t)::value;
    constexpr bool SAFE = decltype(safe_t)::value;
    auto load_bias = [&](uint4 (&bt)[2][2], int kb) __attribute__((always_inline)) {
#pragma unroll
      for (int u = 0; u < NC; ++u) {
        const int so = __builtin_amdgcn_readfirstlane((qb[u] * nkb + kb) * 2048);
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bt[u][c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trs, lane * 16, so + c * 1024, 0));
      }
    };
    uint4 bt[2][2];
    load_bias(bt, k0);
    f32x4 lac[2][2];   // ONES: the denominators as MFMA accumulators (all four registers hold the column's sum)
    bf16x8 ones;
    if constexpr (ONES) {
#pragma unroll
      for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;
#pragma unroll
      for (int u = 0; u < 2; ++u)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) lac[u][qh] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // one key block; KH: the block's second 16 keys are all beyond N (the window's last block when N mod 32 is in
    // (0, 16]: 392 = 12 x 32 + 8): their products, exponentials and P are skipped (P = 0 there anyway)
    auto block = [&](int kb, auto kh_t) __attribute__((always_inline)) {
      constexpr bool KH = decltype(kh_t)::value;
      const bf16raw* kbase = Ks + kb * 32 * HD;
      const bf16raw* vbase = Vs + kb * 32 * HD;
      bf16x8 kf[2];
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) kf[kh] = *reinterpret_cast<const bf16x8*>(kbase + koff[kh]);
      f32x4 d[2][4];
#pragma unroll
      for (int u = 0; u < NC; ++u)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint32_t w[4] = {bt[u][c].x, bt[u][c].y, bt[u][c].z, bt[u][c].w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            float lo = __uint_as_float(w[i] << 16), hi = __uint_as_float(w[i] & 0xffff0000u);
            if constexpr (SAFE) {
              lo -= m[u][c];
              hi -= m[u][c];
            }
            d[u][2 * c + (i >> 1)][2 * (i & 1)] = lo;
            d[u][2 * c + (i >> 1)][2 * (i & 1) + 1] = hi;
          }
        }
      load_bias(bt, min(kb + 1, k1 - 1));
#pragma unroll
      for (int u = 0; u < NC; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t)
          if (!KH || (t & 1) == 0) d[u][t] = mfma16(kf[t & 1], qf[u][t >> 1], d[u][t]);
      bf16x8 va[2];
#pragma unroll
      for (int eh = 0; eh < 2; ++eh) va[eh] = tr16x2(vbase + vlo[eh], vbase + vhi[eh]);
#pragma unroll
      for (int u = 0; u < NC; ++u) {
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          f32x4& d0 = d[u][2 * qh];
          f32x4& d1 = d[u][2 * qh + 1];
          if constexpr (SAFE) {
            float bm = max3f(max3f(d0[0], d0[1], d0[2]), max3f(d0[3], d1[0], d1[1]), max3f(d1[2], d1[3], -INFINITY));
            bm = grp_max4(bm);
            const bool grow = kb == k0 || bm > kRescale;
            if (__builtin_amdgcn_ballot_w64(grow) != 0) {
              const float mn = grow ? bf16_ceil(m[u][qh] + bm) : m[u][qh];
              const float delta = mn - m[u][qh];
              const float alpha = kb == k0 ? 0.f : __builtin_amdgcn_exp2f(-delta);
              m[u][qh] = mn;
#pragma unroll
              for (int j = 0; j < 4; ++j) {
                d0[j] -= delta;
                d1[j] -= delta;
              }
              ls[u][qh] *= alpha;
              if constexpr (ONES) lac[u][qh] = lac[u][qh] * alpha;
#pragma unroll
              for (int j = 0; j < 8; ++j) o[u][8 * qh + j] *= alpha;
            }
          }
          float p[8];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            p[j] = __builtin_amdgcn_exp2f(d0[j]);
            p[4 + j] = KH ? 0.f : __builtin_amdgcn_exp2f(d1[j]);
          }
          if constexpr (!ONES) {
            if constexpr (KH) ls[u][qh] += (p[0] + p[1]) + (p[2] + p[3]);
            else ls[u][qh] += ((p[0] + p[1]) + (p[2] + p[3])) + ((p[4] + p[5]) + (p[6] + p[7]));
          }
          bf16x8 pv;
#pragma unroll
          for (int j = 0; j < 8; ++j) pv[j] = (__bf16)p[j];
          if constexpr (ONES) lac[u][qh] = mfma16(ones, pv, lac[u][qh]);
#pragma unroll
          for (int eh = 0; eh < 2; ++eh) {
            f32x4 acc = {o[u][8 * qh + 4 * eh], o[u][8 * qh + 4 * eh + 1], o[u][8 * qh + 4 * eh + 2],
                         o[u][8 * qh + 4 * eh + 3]};
            acc = mfma16(va[eh], pv, acc);
#pragma unroll
            for (int j = 0; j < 4; ++j) o[u][8 * qh + 4 * eh + j] = acc[j];
          }
        }
      }
    };
    // the last block's second half is dead when N ends in its first half (SAFE keeps every block whole: its
    // running maximum must see the -1e4 bias of dead keys exactly as before)
    const bool tail_half = !SAFE && k1 == nkb && (nkb - 1) * 32 + 16 >= g.N;
    const int kfull = tail_half ? k1 - 1 : k1;
    for (int kb = k0; kb < kfull; ++kb) block(kb, std::false_type{});
    if (tail_half) block(k1 - 1, std::true_type{});
    if constexpr (ONES) {
#pragma unroll
      for (int u = 0; u < NC; ++u)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) ls[u][qh] += lac[u][qh][0];
    }
  };
  auto zero = [&](f32x16 (&o)[2], float (&ls)[2][2], float (&m)[2][2]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < 2; ++u) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) ls[u][qh] = m[u][qh] = 0.f;
#pragma unroll
      for (int j = 0; j < 16; ++j) o[u][j] = 0.f;
    }
  };
  // O = O^T / l for block qb (lane: queries 32 qb + 16 qh + ql, channels 16 eh + 4 g16 + 0..3), lse; true: rejected
  auto store = [&](int qb, const f32x16& o, const float (&ls)[2], const float (&m)[2], bool real = true,
                   bool reduced = false) __attribute__((always_inline)) -> bool {
    if (!real) return false;
    bool bad = false;
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      const float l = reduced ? ls[qh] : grp_sum4(ls[qh]);
      const float inv = 1.f / l;
      const int q = qb * 32 + 16 * qh + ql;
      const int row = q < g.N ? token_info_row(a, g, b, win, q) : -2;
      if (row >= 0) {
        bf16raw* op = reinterpret_cast<bf16raw*>(a.out) + (long)row * a.ld_out + hoff + 4 * g16;
#pragma unroll
        for (int eh = 0; eh < 2; ++eh) {
          uint2 w;
          w.x = (uint32_t)f2bf(o[8 * qh + 4 * eh] * inv) | ((uint32_t)f2bf(o[8 * qh + 4 * eh + 1] * inv) << 16);
          w.y = (uint32_t)f2bf(o[8 * qh + 4 * eh + 2] * inv) | ((uint32_t)f2bf(o[8 * qh + 4 * eh + 3] * inv) << 16);
          *reinterpret_cast<uint2*>(op + 16 * eh) = w;
        }
      }
      if (a.lse && g16 == 0 && q < g.N) a.lse[unit * g.Np + q] = (m[qh] + __log2f(l)) * 0.6931471805599453f;
      bad |= !f5_l_ok(l);
    }
    return bad;
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using FAST = std::false_type;
  using SAFE = std::true_type;
  auto safe_block = [&](int qb) __attribute__((always_inline)) {
    const int qbs[2] = {qb, qb};
    bf16x8 qf[2][2];
    load_q(qb, qf[0]);
    f32x16 o[2];
    float ls[2][2], m[2][2];
    zero(o, ls, m);
    chains(I1{}, SAFE{}, qbs, qf, 0, nkb, o, ls, m);
    store(qb, o[0], ls[0], m[0], true, ONES);
  };
  auto full = [&](int qb0, int qb1) __attribute__((always_inline)) {
    const int qb[2] = {qb0, min(qb1, nqb - 1)};
    bf16x8 qf[2][2];
    load_q(qb[0], qf[0]);
    f32x16 o[2];
    float ls[2][2], m[2][2];
    zero(o, ls, m);
    bool bad;
    if (qb1 < nqb) {
      load_q(qb[1], qf[1]);
      chains(I2{}, FAST{}, qb, qf, 0, nkb, o, ls, m);
      bad = store(qb[0], o[0], ls[0], m[0], true, ONES);
      bad |= store(qb[1], o[1], ls[1], m[1], true, ONES);
    } else {   // an odd block count's last block: one chain (it was computed twice, the copy discarded)
      chains(I1{}, FAST{}, qb, qf, 0, nkb, o, ls, m);
      bad = store(qb[0], o[0], ls[0], m[0], true, ONES);
    }
    if (__builtin_amdgcn_ballot_w64(bad) != 0) {
      safe_block(qb[0]);
      if (qb1 < nqb) safe_block(qb1);
    }
  };
  const int nw = dfk_bdim() >> 6;
  static_assert(!(BAL && ONES), "ONES: the simple schedule only");
  if constexpr (!BAL) {
    const int ngrp = (nqb + 1) / 2, qstep = nw * qsplit;
    for (int gi = wu.qpart * nw + wave; gi < ngrp; gi += qstep) full(2 * gi, 2 * gi + 1);
    return;
  } else {
    // v5's balanced schedule (host guarantees: qsplit == 1, 4 waves, pairs % 4 in {0, 1, 2}); the row sums are
    // reduced over the lane groups before they go to LDS, so the l's of a wave fit one float4 slot per lane
    int& f5_flag = *reinterpret_cast<int*>(smem + max(4 * g.Np * HD, 4 * kF5Slots * 1024));
    if (tid == 0) f5_flag = 0;
    const int pairs = nqb / 2, tail = nqb & 1, R = pairs % 4, p1 = pairs - R;
    for (int p = wave; p < p1; p += 4) full(2 * p, 2 * p + 1);
    f32x16 oa[2], ob[2];
    float la[2][2], lb[2][2], ma[2][2], mb[2][2];
    zero(oa, la, ma);
    zero(ob, lb, mb);
    const int pa = R == 2 ? p1 + (wave >> 1) : p1;
    if (R > 0) {
      const int ka0 = R == 2 ? ((wave & 1) ? (nkb + 1) / 2 : 0) : (wave * nkb) / 4;
      const int ka1 = R == 2 ? ((wave & 1) ? nkb : (nkb + 1) / 2) : ((wave + 1) * nkb) / 4;
      const int qb[2] = {2 * pa, 2 * pa + 1};
      bf16x8 qf[2][2];
      load_q(qb[0], qf[0]);
      load_q(qb[1], qf[1]);
      chains(I2{}, FAST{}, qb, qf, ka0, ka1, oa, la, ma);
    }
    if (tail) {
      const int qb[2] = {nqb - 1, nqb - 1};
      bf16x8 qf[2][2];
      load_q(qb[0], qf[0]);
      chains(I1{}, FAST{}, qb, qf, (wave * nkb) / 4, ((wave + 1) * nkb) / 4, ob, lb, mb);
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        la[u][qh] = grp_sum4(la[u][qh]);
        lb[u][qh] = grp_sum4(lb[u][qh]);
      }
    __syncthreads();   // every wave is done with K / V: their space takes the partials
    float4* ps = reinterpret_cast<float4*>(smem);
    auto slot = [&](int w, int s) __attribute__((always_inline)) -> float4* { return ps + (w * kF5Slots + s) * 64 + lane; };
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int j4 = 0; j4 < 4; ++j4)
        *slot(wave, 4 * u + j4) = make_float4(oa[u][4 * j4], oa[u][4 * j4 + 1], oa[u][4 * j4 + 2], oa[u][4 * j4 + 3]);
#pragma unroll
    for (int j4 = 0; j4 < 4; ++j4)
      *slot(wave, 8 + j4) = make_float4(ob[0][4 * j4], ob[0][4 * j4 + 1], ob[0][4 * j4 + 2], ob[0][4 * j4 + 3]);
    // slot 12: lanes of group 0 hold the pair's (chain, half) sums, group 1 the tail's (query = lane & 15)
    *slot(wave, 12) = g16 == 0 ? make_float4(la[0][0], la[0][1], la[1][0], la[1][1])
                               : make_float4(lb[0][0], lb[0][1], 0.f, 0.f);
    __syncthreads();
    const bool fin_pair = R == 2 ? (wave == 0 || wave == 2) : (R == 1 && wave == 0);
    const bool fin_tail = tail && wave == (R == 2 ? 3 : (R == 1 ? 1 : 0));
    bool bad2 = false;
    if (fin_pair) {
      const int w0 = R == 2 ? wave : 0, w1 = R == 2 ? wave + 2 : 4;
      f32x16 o[2];
      float ls[2][2], m0[2] = {0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        ls[u][0] = ls[u][1] = 0.f;
#pragma unroll
        for (int j = 0; j < 16; ++j) o[u][j] = 0.f;
      }
      for (int w = w0; w < w1; ++w) {
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int j4 = 0; j4 < 4; ++j4) {
            const float4 v = *slot(w, 4 * u + j4);
            o[u][4 * j4] += v.x; o[u][4 * j4 + 1] += v.y; o[u][4 * j4 + 2] += v.z; o[u][4 * j4 + 3] += v.w;
          }
        const float4 lv = ps[(w * kF5Slots + 12) * 64 + ql];
        ls[0][0] += lv.x; ls[0][1] += lv.y; ls[1][0] += lv.z; ls[1][1] += lv.w;
      }
#pragma unroll
      for (int u = 0; u < 2; ++u) bad2 |= store(2 * pa + u, o[u], ls[u], m0, true, true);
    }
    if (fin_tail) {
      f32x16 o;
      float ls[2] = {0.f, 0.f}, m0[2] = {0.f, 0.f};
#pragma unroll
      for (int j = 0; j < 16; ++j) o[j] = 0.f;
      for (int w = 0; w < 4; ++w) {
#pragma unroll
        for (int j4 = 0; j4 < 4; ++j4) {
          const float4 v = *slot(w, 8 + j4);
          o[4 * j4] += v.x; o[4 * j4 + 1] += v.y; o[4 * j4 + 2] += v.z; o[4 * j4 + 3] += v.w;
        }
        const float4 lv = ps[(w * kF5Slots + 12) * 64 + 16 + ql];
        ls[0] += lv.x;
        ls[1] += lv.y;
      }
      bad2 |= store(nqb - 1, o, ls, m0, true, true);
    }
    const bool wave_bad = __builtin_amdgcn_ballot_w64(bad2) != 0;   // every lane votes (not under lane == 0)
    if (lane == 0 && wave_bad) f5_flag = 1;
    __syncthreads();
    if (f5_flag) {   // a rejected split block (vanishingly rare): K / V again, the block through the SAFE loop
      gather();
      __syncthreads();
      if (__builtin_amdgcn_ballot_w64(bad2) != 0) {
        safe_block(fin_pair ? 2 * pa : nqb - 1);
        if (fin_pair) safe_block(2 * pa + 1);
      }
    }
  }
}

size_t fwd_lds_bf16(const dfk_wattn_args& a, const Geo& g) {
  return 16 + 4 * (size_t)g.Np + 4 * (size_t)((g.L + 3) & ~3) + 4 * (size_t)g.Np * a.hd;
}

Geo make_geo(const dfk_wattn_args& a) {
  Geo g;
  g.Dp = dfk_cdiv(a.D, a.wd) * a.wd;
  g.Hp = dfk_cdiv(a.H, a.wh) * a.wh;
  g.Wp = dfk_cdiv(a.W, a.ww) * a.ww;
  g.nwd = g.Dp / a.wd; g.nwh = g.Hp / a.wh; g.nww = g.Wp / a.ww;
  g.nW = g.nwd * g.nwh * g.nww;
  g.N = a.wd * a.wh * a.ww;
  g.Np = dfk_cdiv(g.N, 32) * 32;
  g.L = (2 * a.fd - 1) * (2 * a.fh - 1) * (2 * a.fw - 1);
  g.C0 = ((a.fd - 1) * (2 * a.fh - 1) + (a.fh - 1)) * (2 * a.fw - 1) + (a.fw - 1);
  g.use_mask = (a.sd > 0 || a.sh > 0 || a.sw > 0) ? 1 : 0;
  auto magic = [](int n) -> uint32_t { return n <= 1 ? 0u : (uint32_t)(0xFFFFFFFFull / (unsigned)n + 1); };
  g.m_hw = magic(a.wh * a.ww);
  g.m_w = magic(a.ww);
  return g;
}

bool args_ok(const dfk_wattn_args& a) {
  if (!a.q || !a.k || !a.v || !a.out) return false;
  if (a.hd != 32 && a.hd != 64) return false;
  if (a.mask && a.mask_nw <= 0) return false;
  if (a.wd <= 0 || a.wh <= 0 || a.ww <= 0 || a.fd <= 0 || a.fh <= 0 || a.fw <= 0) return false;
  if (a.wd * a.wh * a.ww > a.fd * a.fh * a.fw) return false;  // tokens decode inside the full window (Q3)
  if ((long)a.wd * a.wh * a.ww >= 65536) return false;        // fdiv16 token decode
  if (a.sd < 0 || a.sh < 0 || a.sw < 0 || a.sd >= a.wd || a.sh >= a.wh || a.sw >= a.ww) return false;
  const int vec = a.dtype == DFK_BF16 ? 8 : 4;
  if (a.ld_qkv % vec || a.ld_out % vec) return false;
  return true;
}

size_t fwd_lds(const dfk_wattn_args& a, const Geo& g) {
  const size_t es = a.dtype == DFK_BF16 ? 2 : 4;
  size_t v = a.dtype == DFK_BF16 ? (size_t)a.hd * (g.Np + 8) * es : (size_t)g.Np * a.hd * es;
  return sizeof(TokInfo) * g.Np + 4 * (size_t)((g.L + 3) & ~3) + (size_t)g.Np * a.hd * es + v;
}

}  // namespace

// dfk_wattn_fwd_policy (DFK_WATTN_V / DFK_WATTN_BALMIN set the start values for A/B runs)
// defaults: v6; the balanced schedule from 512 units for v5, off for v6 (measured slower there: r5h, stage 1
// 189.9 vs 178.5 us — the split phase's extra Q loads, barriers and spills cost more than the idle wave)
static int g_fwd_version = getenv("DFK_WATTN_V") ? atoi(getenv("DFK_WATTN_V")) : 6;
static long g_fwd_bal_min = getenv("DFK_WATTN_BALMIN") ? atol(getenv("DFK_WATTN_BALMIN")) : -1;   // -1: default

// the forward reads its bias tiles in the 16x16x32 layout (wattn_fwd6_kernel) — the same predicate as dfk_wattn_fwd
// v6 runs windows of at least 4 query blocks (Np >= 128: every Video Swin stage); the 49-token SwinV2 windows keep
// v4 — v6 gains nothing there (mel1: 14.5-15.7 vs 15.5 us) and v4's rounding keeps the SwinV2 logit_scale gradients
// where the goldens hold them (r5j: C1 mel layers.1.blocks.1 logit_scale norm 5.7 % with v4, 8.6 % with v6, against
// 1.1 % in the reference's own bf16 run — the same attention error, rms 2.8e-3 either way, tools/wattn_err.py, in a
// gradient that cancels to a few % of its terms)
static const int g_v6_min_qb = getenv("DFK_WATTN_V6MIN") ? atoi(getenv("DFK_WATTN_V6MIN")) : 4;   // A/B runs only
static const int g_v6_ones = getenv("DFK_WATTN_ONES") ? atoi(getenv("DFK_WATTN_ONES")) : 0;      // A/B runs only
static const int g_v6_w8 = getenv("DFK_WATTN_W8") ? atoi(getenv("DFK_WATTN_W8")) : 0;            // A/B runs only
static bool use_v6(const dfk_wattn_args& a, const Geo& g) {
  return g_fwd_version == 6 && a.hd == 32 && !a.drop.mode && g.Np / 32 >= g_v6_min_qb;
}
static bool fwd16_layout(const dfk_wattn_args& a, const Geo& g) { return use_v6(a, g); }

extern "C" int dfk_wattn_table(const dfk_wattn_args* ap, hipStream_t s) {
  if (!ap || !args_ok(*ap) || !ap->tab || ap->dtype != DFK_BF16 || ap->mask || !(ap->scale > 0.f)) return DFK_EINVAL;
  const dfk_wattn_args& a = *ap;
  const Geo g = make_geo(a);
  const TabGeo tg = tab_geo(a, g);
  bf16raw* t3 = tab3_fwd(a, g);
  // only the classes some window has (a class bit needs its dim shifted; the D-only shift of the Swin-T stage 4
  // uses 2 of the 8): the 192-channel stage-4 table took 125 us for 384 window-heads
  ClsMap cm{};
  int nc = 0;
  for (int c = 0; c < tg.ncls; ++c) {
    const long nd = !g.use_mask ? g.nwd : ((c & 4) ? (a.sd > 0) : g.nwd - (a.sd > 0));
    const long nh = !g.use_mask ? g.nwh : ((c & 2) ? (a.sh > 0) : g.nwh - (a.sh > 0));
    const long nw = !g.use_mask ? g.nww : ((c & 1) ? (a.sw > 0) : g.nww - (a.sw > 0));
    if (nd * nh * nw > 0) cm.c[nc++] = c;
  }
  if (nc == 0) return 0;
  // about eight 16-B slots per thread (the per-workgroup prologue — token labels, the head's RPB column —
  // amortised), unless that leaves fewer than 1024 workgroups (the small SwinV2 tables)
  const long slots2 = 2 * tg.per_ch / 8;
  long gx = std::min<long>(dfk_cdiv(slots2, 256 * 8), 64);
  if (gx * nc * a.heads < 1024) gx = std::min<long>(dfk_cdiv(slots2, 256), std::max<long>(gx, dfk_cdiv(1024, nc * a.heads)));
  hipLaunchKernelGGL(wattn_tab3_kernel, dim3((unsigned)gx, nc * a.heads),
                     dim3(256), 4 * (size_t)(g.Np + g.L), s, a, g, t3, t3 + tab_elems(a, g), fwd16_layout(a, g) ? 1 : 0,
                     cm);
  DFK_CHECK_LAUNCH();
  return 0;
}


extern "C" int dfk_wattn_fwd_policy(int32_t version, int64_t bal_min_units) {
  if (version >= 0) g_fwd_version = version;
  if (bal_min_units >= 0 || bal_min_units == -2) g_fwd_bal_min = bal_min_units >= 0 ? (long)bal_min_units : -1;
  return 0;
}

extern "C" int dfk_wattn_fwd(const dfk_wattn_args* ap, hipStream_t s) {
  if (!ap || !args_ok(*ap)) return DFK_EINVAL;
  const dfk_wattn_args& a = *ap;
  const Geo g = make_geo(a);
  if (a.drop.mode && !(a.dtype == DFK_BF16 && !a.mask && a.scale > 0.f)) return DFK_EINVAL;  // bf16 v3 path only
  if (a.dtype == DFK_BF16 && !a.mask && a.scale > 0.f && (a.tab || (!a.rpb && !g.use_mask))) {
    // v3: bias tiles from dfk_wattn_table (RPB and / or shift mask), or no bias at all
    const long units = (long)a.B * g.nW * a.heads;
    if (units <= 0) return 0;
    const bool tab = a.rpb || g.use_mask;
    const bf16raw* t3 = tab ? tab3_fwd(a, g) : nullptr;
    const size_t lds = 4 * (size_t)g.Np * a.hd;
    if (lds > 160 * 1024) return DFK_EINVAL;
    const int nqb = g.Np / 32;
    // query blocks per wave: 2 for the hd-32 table kernel (K / V fragment reads shared, two chains interleaved)
    static const int qgrp_env = getenv("DFK_WATTN_QB") ? atoi(getenv("DFK_WATTN_QB")) : 2;   // A/B runs only
    const int qgrp = tab && a.hd == 32 && !a.drop.mode && nqb >= 2 ? qgrp_env : 1;
    const int ngrp = dfk_cdiv(nqb, qgrp);
    const bool w8 = g_v6_w8 && tab && qgrp == 2 && use_v6(a, g);
    const int nw = std::min(w8 ? 8 : 4, ngrp);
    int qsplit = (int)std::max<long>(1, std::min<long>(dfk_cdiv(ngrp, nw), dfk_cdiv(1024, units)));
    // v5 (no running max; A/B: DFK_WATTN_V=4 keeps v4) and its balanced schedule (one workgroup per unit, the
    // remaining pairs and the tail split by keys over the 4 waves) from DFK_WATTN_BALMIN units (default 512)
    const bool v6 = tab && qgrp == 2 && use_v6(a, g);
    const bool v5 = tab && a.hd == 32 && !a.drop.mode && qgrp == 2 && g_fwd_version == 5;   // v4 otherwise
    const int pairs = nqb / 2;
    const long bal_min = g_fwd_bal_min >= 0 ? g_fwd_bal_min : (v5 ? 512 : LONG_MAX);
    const bool bal = (v5 || v6) && !w8 && nw == 4 && pairs % 4 != 3 && units >= bal_min;
    size_t lds_k = lds;
    if (bal) {
      qsplit = 1;
      lds_k = std::max(lds, (size_t)4 * kF5Slots * 64 * 16) + 16;   // + the fallback flag
    }
    dim3 grid((unsigned)(units * qsplit));
#define LAUNCH_K(KFN)                                                                                        \
  do {                                                                                                       \
    auto kfn = KFN;                                                                                          \
    static bool attr_set = false;                                                                            \
    if (!attr_set) {                                                                                         \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);   \
      attr_set = true;                                                                                       \
    }                                                                                                        \
    hipLaunchKernelGGL(kfn, grid, dim3(64 * nw), lds_k, s, a, g, qsplit, t3);                               \
  } while (0)
    // bias tables: v4 (bias through the QK^T C input, VALU row sums); no bias: v3's table-free form
    if (a.hd == 32) {
      if (tab) {
        if (a.drop.mode) LAUNCH_K((wattn_fwd4_kernel<32, true, 1>));
        else if (v6 && bal) LAUNCH_K((wattn_fwd6_kernel<true>));
        else if (v6 && g_v6_w8) LAUNCH_K((wattn_fwd6_kernel<false, false, true>));
        else if (v6 && g_v6_ones) LAUNCH_K((wattn_fwd6_kernel<false, true>));
        else if (v6) LAUNCH_K((wattn_fwd6_kernel<false>));
        else if (bal) LAUNCH_K((wattn_fwd5_kernel<true>));
        else if (v5) LAUNCH_K((wattn_fwd5_kernel<false>));
        else if (qgrp == 2) LAUNCH_K((wattn_fwd4_kernel<32, false, 2>));
        else LAUNCH_K((wattn_fwd4_kernel<32, false, 1>));
      } else {
        if (a.drop.mode) LAUNCH_K((wattn_fwd3_kernel<32, false, true>)); else LAUNCH_K((wattn_fwd3_kernel<32, false, false>));
      }
    } else {
      if (tab) {
        if (a.drop.mode) LAUNCH_K((wattn_fwd4_kernel<64, true, 1>)); else LAUNCH_K((wattn_fwd4_kernel<64, false, 1>));
      } else {
        if (a.drop.mode) LAUNCH_K((wattn_fwd3_kernel<64, false, true>)); else LAUNCH_K((wattn_fwd3_kernel<64, false, false>));
      }
    }
#undef LAUNCH_K
    DFK_CHECK_LAUNCH();
    return 0;
  }
  if (a.dtype == DFK_BF16) {
    const size_t lds = fwd_lds_bf16(a, g);
    if (lds > 160 * 1024) return DFK_EINVAL;
    const long units = (long)a.B * g.nW * a.heads;
    if (units <= 0) return 0;
    const int nqb = g.Np / 32;
    const int nw = std::min(4, nqb);   // small windows (SwinV2 7x7: two query blocks) get fewer waves
    const int qsplit = (int)std::max<long>(1, std::min<long>(dfk_cdiv(nqb, nw), dfk_cdiv(1024, units)));
    dim3 grid((unsigned)units, qsplit);
#define LAUNCH_F16(HD, RPB, MASK)                                                                          \
  do {                                                                                                     \
    auto kfn = wattn_fwd_bf16_kernel<HD, RPB, MASK>;                                                       \
    static bool attr_set = false;                                                                          \
    if (!attr_set) {                                                                                       \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr_set = true;                                                                                     \
    }                                                                                                      \
    hipLaunchKernelGGL(kfn, grid, dim3(64 * nw), lds, s, a, g, qsplit);                                    \
  } while (0)
#define PICK_F16(HD)                                                                            \
  do {                                                                                          \
    if (a.rpb) { if (a.mask) LAUNCH_F16(HD, true, true); else LAUNCH_F16(HD, true, false); }   \
    else { if (a.mask) LAUNCH_F16(HD, false, true); else LAUNCH_F16(HD, false, false); }       \
  } while (0)
    if (a.hd == 32) PICK_F16(32); else PICK_F16(64);
#undef PICK_F16
#undef LAUNCH_F16
    DFK_CHECK_LAUNCH();
    return 0;
  }
  const size_t lds = fwd_lds(a, g);
  if (lds > 160 * 1024) return DFK_EINVAL;
  const long units = (long)a.B * g.nW * a.heads;
  if (units <= 0) return 0;
  const int nqt = dfk_cdiv(g.N, 16);
  int qsplit = (int)std::max<long>(1, std::min<long>(dfk_cdiv(nqt, 4), dfk_cdiv(1024, units)));
  dim3 grid((unsigned)units, qsplit);
#define LAUNCH_F(T, HD)                                                                                 \
  do {                                                                                                  \
    auto kfn = wattn_fwd_kernel<T, HD>;                                                                 \
    static bool attr_set = false;  /* once per kernel: the 160 KiB LDS limit (never inside a capture) */ \
    if (!attr_set) {                                                                                    \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr_set = true;                                                                                  \
    }                                                                                                   \
    hipLaunchKernelGGL(kfn, grid, dim3(256), lds, s, a, g, qsplit);                                     \
  } while (0)
  if (a.hd == 32) LAUNCH_F(float, 32); else LAUNCH_F(float, 64);
#undef LAUNCH_F
  DFK_CHECK_LAUNCH();
  return 0;
}

// ---------------------------------------------------------------- backward
// One workgroup = one (clip, window, head).  Waves own 32-key blocks with the
// KEY on the MFMA lane: S = Q K^T and dP = dO V^T come out as [q rows][k lane]
// accumulators, which are directly the A operand of dV = P^T dO and
// dK = dS^T Q (X^T.B form), so dK/dV stay in registers for the whole sweep
// over queries.  dS crosses LDS once (per-wave scratch) for dQ = dS K, which
// all waves add into an fp32 LDS accumulator; dRPB is an LDS fp32 table
// flushed with one global atomic per entry.
namespace {

// this window-head's dRPB partial -> its workspace row (reduced by drpb_reduce_kernel);
// without a workspace, device-scope atomics on the shared [L,nH] table
__device__ __forceinline__ void flush_drpb(const dfk_wattn_bwd_args& ba, const Geo& g, const float* drpb, int head,
                                           int accum, int tid, int nthreads) {
  if (ba.ws) {
    float* w = ba.ws + (long)dfk_bid_x() * ((g.L + 3) & ~3);
    for (int l = tid; l < g.L; l += nthreads) w[l] = accum ? w[l] + drpb[l] : drpb[l];
  } else {
    for (int l = tid; l < g.L; l += nthreads)
      if (drpb[l] != 0.f) atomicAdd(ba.drpb + (long)l * ba.f.heads + head, drpb[l]);
  }
}

// drpb[l][h] += sum over window-heads u = h (mod heads) of ws[u][l]; 16 row phases per 64 entries
__global__ __launch_bounds__(1024) void drpb_reduce_kernel(const float* __restrict__ ws, long units, int heads, int L,
                                                           float* __restrict__ drpb) {
  __shared__ float part[16][64];
  const int Lal = (L + 3) & ~3;
  const int c = dfk_tid() & 63, ph = dfk_tid() >> 6, h = dfk_bid_y();
  const int l = dfk_bid_x() * 64 + c;
  float s = 0.f;
  if (l < L)
    for (long u = h + (long)heads * ph; u < units; u += (long)heads * 16) s += ws[u * Lal + l];
  part[ph][c] = s;
  __syncthreads();
  if (ph == 0 && l < L) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) t += part[i][c];
    drpb[(long)l * heads + h] += t;
  }
}

template <typename T, int HD>
__global__ __launch_bounds__(256) void wattn_bwd_kernel(const dfk_wattn_bwd_args ba, const Geo g, int q0, int Qn,
                                                        int accum_kv) {
  // queries [q0, q0+Qn) of every window are handled by this launch (Qn % 32 == 0);
  // larger windows in fp32 run as several launches with dK/dV accumulated (accum_kv).
  constexpr bool BF = sizeof(T) == 2;
  const dfk_wattn_args& a = ba.f;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lal = (g.L + 3) & ~3;
  char* p = smem;
  TokInfo* tok = reinterpret_cast<TokInfo*>(p); p += sizeof(TokInfo) * g.Np;
  float* rpb = reinterpret_cast<float*>(p); p += 4 * Lal;
  float* drpb = reinterpret_cast<float*>(p); p += 4 * Lal;
  float* lse = reinterpret_cast<float*>(p); p += 4 * Qn;
  float* delta = reinterpret_cast<float*>(p); p += 4 * Qn;
  float* dQacc = reinterpret_cast<float*>(p); p += 4 * (size_t)Qn * HD;
  T* Qs = reinterpret_cast<T*>(p); p += sizeof(T) * (size_t)Qn * HD;
  T* dOs = reinterpret_cast<T*>(p); p += sizeof(T) * (size_t)Qn * HD;
  T* Sd = reinterpret_cast<T*>(p);  // 4 waves x [32 q][32 k]

  const int tid = dfk_tid(), lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, ql = lane & 15;
  int unit = dfk_bid_x();
  const int head = unit % a.heads;
  unit /= a.heads;
  const int win = unit % g.nW, b = unit / g.nW;
  const float* mrow = a.mask ? a.mask + (((long)b * g.nW + win) % a.mask_nw) * g.N * g.N : nullptr;
  const int hoff = head * HD;
  constexpr int VEC = 16 / sizeof(T);

  for (int i = tid; i < g.Np; i += 256) tok[i] = token_info(a, g, b, win, i);
  for (int l = tid; l < g.L; l += 256) {
    rpb[l] = a.rpb ? a.rpb[(long)l * a.heads + head] : 0.f;
    drpb[l] = 0.f;
  }
  __syncthreads();
  // Q, dO rows -> LDS; lse; delta = rowsum(dO * O); zero dQ accumulator
  for (int idx = tid; idx < Qn * (HD / VEC); idx += 256) {
    const int li = idx / (HD / VEC), c = (idx % (HD / VEC)) * VEC;
    const TokInfo t = tok[q0 + li];
    *reinterpret_cast<uint4*>(Qs + li * HD + c) = ld16<T>(tok_ptr<T>(a.q, a.pad_q, t.row, a.ld_qkv, hoff + c));
    const T* dop = t.row >= 0 ? reinterpret_cast<const T*>(ba.dout) + (long)t.row * ba.ld_dout + hoff + c : nullptr;
    *reinterpret_cast<uint4*>(dOs + li * HD + c) = ld16<T>(dop);
  }
  for (int i = tid; i < Qn * HD; i += 256) dQacc[i] = 0.f;
  for (int li = tid; li < Qn; li += 256) {
    const int i = q0 + li;
    const TokInfo t = tok[i];
    float d = 0.f;
    if (t.row >= 0) {
      const T* op = reinterpret_cast<const T*>(a.out) + (long)t.row * a.ld_out + hoff;
      const T* dop = reinterpret_cast<const T*>(ba.dout) + (long)t.row * ba.ld_dout + hoff;
      for (int e = 0; e < HD; ++e) d += ldf<T>(op + e) * ldf<T>(dop + e);
    }
    delta[li] = d;
    lse[li] = (i < g.N) ? a.lse[(long)dfk_bid_x() * g.Np + i] : 0.f;
  }
  __syncthreads();

  T* Sw = Sd + wave * 32 * 32;
  const int nkb = g.Np / 32, nqb = Qn / 32;
  for (int kb = wave; kb < nkb; kb += 4) {
    // own keys: B fragments of K^T and V^T (key on lane) and K in natural-k B layout for dQ
    f32x4 dK[2][HD / 16], dV[2][HD / 16];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) { dK[h2][et] = f32x4{0, 0, 0, 0}; dV[h2][et] = f32x4{0, 0, 0, 0}; }
    TokInfo tk[2];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) tk[h2] = tok[kb * 32 + h2 * 16 + ql];

    if constexpr (BF) {
      bf16x8 kB[2][HD / 32], vB[2][HD / 32], kN[HD / 16];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const T* kp = tok_ptr<T>(a.k, a.pad_k, tk[h2].row, a.ld_qkv, hoff);
        const T* vp = tok_ptr<T>(a.v, a.pad_v, tk[h2].row, a.ld_qkv, hoff);
#pragma unroll
        for (int es = 0; es < HD / 32; ++es) {
          uint4 u = kp ? *reinterpret_cast<const uint4*>(kp + es * 32 + grp * 8) : make_uint4(0, 0, 0, 0);
          kB[h2][es] = *reinterpret_cast<bf16x8*>(&u);
          u = vp ? *reinterpret_cast<const uint4*>(vp + es * 32 + grp * 8) : make_uint4(0, 0, 0, 0);
          vB[h2][es] = *reinterpret_cast<bf16x8*>(&u);
        }
      }
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const TokInfo t = tok[kb * 32 + grp * 8 + j];
          const T* kp = tok_ptr<T>(a.k, a.pad_k, t.row, a.ld_qkv, hoff + et * 16 + ql);
          kN[et][j] = kp ? __builtin_bit_cast(__bf16, *reinterpret_cast<const bf16raw*>(kp)) : (__bf16)0.f;
        }
      }
      for (int qb = 0; qb < nqb; ++qb) {
        float pv[2][2][4], ds[2][2][4];  // [qh][h2][r]
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int qrow = qb * 32 + qh * 16 + ql;
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            f32x4 s = f32x4{0, 0, 0, 0}, dp = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int es = 0; es < HD / 32; ++es) {
              const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + qrow * HD + es * 32 + grp * 8);
              const bf16x8 da = *reinterpret_cast<const bf16x8*>(dOs + qrow * HD + es * 32 + grp * 8);
              s = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa, kB[h2][es], s, 0, 0, 0);
              dp = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da, vB[h2][es], dp, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int lq = qb * 32 + qh * 16 + grp * 4 + r;
              const int q = q0 + lq;
              const TokInfo tq = tok[q];
              float v = s[r] * a.scale;
              const int bidx = tq.pos - tk[h2].pos + g.C0;
              if (a.rpb) v += rpb[bidx];
              if (g.use_mask && tq.lab != tk[h2].lab) v -= 100.f;
              const int kk = kb * 32 + h2 * 16 + ql;
              if (mrow && q < g.N && kk < g.N) v += mrow[q * g.N + kk];
              float P = (tq.row == -2 || tk[h2].row == -2) ? 0.f : __expf(v - lse[lq]);
              const float dS = P * (dp[r] - delta[lq]);
              pv[qh][h2][r] = P;
              ds[qh][h2][r] = dS;
              if (a.rpb && dS != 0.f) atomicAdd(drpb + bidx, dS);
              Sw[(qh * 16 + grp * 4 + r) * 32 + h2 * 16 + ql] = f2bf(dS);
            }
          }
        }
        // dV[k][e] += sum_q P[q][k] dO[q][e] ; dK[k][e] += sum_q dS[q][k] Q[q][e]   (q-slot j <-> qh=j>>2, r=j&3)
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) {
          bf16x8 dob, qbv;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const int q = qb * 32 + (j >> 2) * 16 + grp * 4 + (j & 3);
            dob[j] = __builtin_bit_cast(__bf16, reinterpret_cast<const bf16raw*>(dOs)[q * HD + et * 16 + ql]);
            qbv[j] = __builtin_bit_cast(__bf16, reinterpret_cast<const bf16raw*>(Qs)[q * HD + et * 16 + ql]);
          }
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            bf16x8 pa, sa;
#pragma unroll
            for (int j = 0; j < 8; ++j) { pa[j] = (__bf16)pv[j >> 2][h2][j & 3]; sa[j] = (__bf16)ds[j >> 2][h2][j & 3]; }
            dV[h2][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa, dob, dV[h2][et], 0, 0, 0);
            dK[h2][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, qbv, dK[h2][et], 0, 0, 0);
          }
        }
        // dQ[q][e] += scale * sum_k dS[q][k] K[k][e]  (natural k order through the wave's scratch)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const bf16x8 sa = *reinterpret_cast<const bf16x8*>(Sw + (qh * 16 + ql) * 32 + grp * 8);
#pragma unroll
          for (int et = 0; et < HD / 16; ++et) {
            f32x4 acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa, kN[et], f32x4{0, 0, 0, 0}, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              atomicAdd(dQacc + (qb * 32 + qh * 16 + grp * 4 + r) * HD + et * 16 + ql, acc[r] * a.scale);
          }
        }
      }
    } else {
      float kB[2][HD / 4], vB[2][HD / 4], kN[HD / 16][8];
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2) {
        const T* kp = tok_ptr<T>(a.k, a.pad_k, tk[h2].row, a.ld_qkv, hoff);
        const T* vp = tok_ptr<T>(a.v, a.pad_v, tk[h2].row, a.ld_qkv, hoff);
#pragma unroll
        for (int es = 0; es < HD / 4; ++es) {
          kB[h2][es] = kp ? kp[es * 4 + grp] : 0.f;
          vB[h2][es] = vp ? vp[es * 4 + grp] : 0.f;
        }
      }
#pragma unroll
      for (int et = 0; et < HD / 16; ++et)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const TokInfo t = tok[kb * 32 + ks * 4 + grp];
          const T* kp = tok_ptr<T>(a.k, a.pad_k, t.row, a.ld_qkv, hoff + et * 16 + ql);
          kN[et][ks] = kp ? *kp : 0.f;
        }
      for (int qb = 0; qb < nqb; ++qb) {
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int qrow = qb * 32 + qh * 16 + ql;
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            f32x4 s = f32x4{0, 0, 0, 0}, dp = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int es = 0; es < HD / 4; ++es) {
              s = __builtin_amdgcn_mfma_f32_16x16x4f32(Qs[qrow * HD + es * 4 + grp], kB[h2][es], s, 0, 0, 0);
              dp = __builtin_amdgcn_mfma_f32_16x16x4f32(dOs[qrow * HD + es * 4 + grp], vB[h2][es], dp, 0, 0, 0);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int lq = qb * 32 + qh * 16 + grp * 4 + r;
              const int q = q0 + lq;
              const TokInfo tq = tok[q];
              float v = s[r] * a.scale;
              const int bidx = tq.pos - tk[h2].pos + g.C0;
              if (a.rpb) v += rpb[bidx];
              if (g.use_mask && tq.lab != tk[h2].lab) v -= 100.f;
              const int kk = kb * 32 + h2 * 16 + ql;
              if (mrow && q < g.N && kk < g.N) v += mrow[q * g.N + kk];
              const float P = (tq.row == -2 || tk[h2].row == -2) ? 0.f : __expf(v - lse[lq]);
              const float dS = P * (dp[r] - delta[lq]);
              if (a.rpb && dS != 0.f) atomicAdd(drpb + bidx, dS);
              Sw[(qh * 16 + grp * 4 + r) * 32 + h2 * 16 + ql] = dS;
              // dV/dK: A[i=k][slot grp <-> q] = P / dS ; B[slot][e] = dO / Q rows q
#pragma unroll
              for (int et = 0; et < HD / 16; ++et) {
                dV[h2][et] = __builtin_amdgcn_mfma_f32_16x16x4f32(P, dOs[lq * HD + et * 16 + ql], dV[h2][et], 0, 0, 0);
                dK[h2][et] = __builtin_amdgcn_mfma_f32_16x16x4f32(dS, Qs[lq * HD + et * 16 + ql], dK[h2][et], 0, 0, 0);
              }
            }
          }
        }
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int et = 0; et < HD / 16; ++et) {
            f32x4 acc = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
              acc = __builtin_amdgcn_mfma_f32_16x16x4f32(Sw[(qh * 16 + ql) * 32 + ks * 4 + grp], kN[et][ks], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r)
              atomicAdd(dQacc + (qb * 32 + qh * 16 + grp * 4 + r) * HD + et * 16 + ql, acc[r] * a.scale);
          }
      }
    }
    // write dK (scaled) and dV for the 32 owned keys: C layout col = e (lane), row = key 4g+r
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int k = kb * 32 + h2 * 16 + grp * 4 + r;
        const TokInfo t = tok[k];
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) {
          const int e = hoff + et * 16 + ql;
          const float vk = dK[h2][et][r] * a.scale, vv = dV[h2][et][r];
          if (t.row >= 0) {
            T* pk = reinterpret_cast<T*>(ba.dk) + (long)t.row * ba.ld_dqkv + e;
            T* pv = reinterpret_cast<T*>(ba.dv) + (long)t.row * ba.ld_dqkv + e;
            stf<T>(pk, accum_kv ? ldf<T>(pk) + vk : vk);
            stf<T>(pv, accum_kv ? ldf<T>(pv) + vv : vv);
          } else if (t.row == -1) {
            if (ba.dpad_k) atomicAdd(ba.dpad_k + e, vk);
            if (ba.dpad_v) atomicAdd(ba.dpad_v + e, vv);
          }
        }
      }
  }
  __syncthreads();
  for (int idx = tid; idx < Qn * HD; idx += 256) {
    const int li = idx / HD, e = idx % HD;
    const int i = q0 + li;
    if (i >= g.N) continue;
    const TokInfo t = tok[i];
    if (t.row >= 0) stf<T>(reinterpret_cast<T*>(ba.dq) + (long)t.row * ba.ld_dqkv + hoff + e, dQacc[idx]);
    else if (t.row == -1 && ba.dpad_q) atomicAdd(ba.dpad_q + hoff + e, dQacc[idx]);
  }
  if (a.rpb && ba.drpb) flush_drpb(ba, g, drpb, head, accum_kv, tid, 256);
}

// ------------------------------------------------------------ bf16 backward
// Same decomposition (key-owner waves, dK/dV in registers, dQ and dRPB in LDS
// fp32), re-laid for latency: up to 8 waves per window-head (2 waves / SIMD),
// per-query statistics (packed pos|label, lse, delta) fetched once per 32-query
// block as 16-B vectors, softmax in base 2 with no data-dependent branches,
// the dO / Q operands of dV = P^T dO and dK = dS^T Q read with ds_read_tr16
// from XOR-swizzled tiles, dS crossing the wave's scratch as dS^T (b64 stores,
// tr16 loads), and a bank-swizzled dQ accumulator.

template <int HD, bool RPB, bool MASK>
__global__ __launch_bounds__(HD == 32 ? 512 : 256) void wattn_bwd_bf16_kernel(const dfk_wattn_bwd_args ba, const Geo g,
                                                                              int q0, int Qn, int accum_kv,
                                                                              bf16raw* __restrict__ dsg) {
  // One workgroup = one (clip, window, head); wave w owns key blocks w, w + nwaves (dK, dV in registers).
  // All waves step through the query blocks together: per 32-query block each wave computes S, dP, P, dS
  // for its keys, accumulates dV += P^T dO and dK += dS^T Q, and its partial dQ = dS K; the partials are
  // summed through LDS (plain stores, one barrier pair per block) and the finished dQ rows stored.
  // dS^T also goes to global scratch (dsg) for the deterministic dRPB reduction.  No LDS atomics.
  const dfk_wattn_args& a = ba.f;
  constexpr int kDqStride = HD + 4;  // fp32 row stride of the per-wave dQ partials [32 queries][HD]
  const int nwaves = dfk_bdim() >> 6;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int Lal = (g.L + 3) & ~3;
  char* p = smem;
  int* trow = reinterpret_cast<int*>(p); p += 4 * g.Np;
  int* tpk = reinterpret_cast<int*>(p); p += 4 * g.Np;          // pos << 5 | region label
  float* rpb2 = reinterpret_cast<float*>(p); p += 4 * Lal;      // rpb * log2(e)
  float* lse2 = reinterpret_cast<float*>(p); p += 4 * Qn;       // lse * log2(e); +inf beyond N
  float* delta = reinterpret_cast<float*>(p); p += 4 * Qn;
  float* dQp = reinterpret_cast<float*>(p); p += 4 * (size_t)nwaves * 32 * kDqStride;  // per-wave dQ partials
  bf16raw* Qs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Qn * HD;
  bf16raw* dOs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Qn * HD;
  bf16raw* Sd = reinterpret_cast<bf16raw*>(p);

  const int tid = dfk_tid(), lane = tid & 63, wave = tid >> 6;
  const int grp = lane >> 4, ql = lane & 15, tq = ql >> 2, tp = ql & 3;
  int unit = dfk_bid_x();
  const int head = unit % a.heads;
  unit /= a.heads;
  const int win = unit % g.nW, b = unit / g.nW;
  const float* mrow = MASK ? a.mask + (((long)b * g.nW + win) % a.mask_nw) * g.N * g.N : nullptr;
  const int hoff = head * HD;
  const bf16raw* og = reinterpret_cast<const bf16raw*>(a.out);
  const bf16raw* dog = reinterpret_cast<const bf16raw*>(ba.dout);
  const bf16raw* qg = reinterpret_cast<const bf16raw*>(a.q);

  for (int i = tid; i < g.Np; i += dfk_bdim()) {
    const TokInfo t = token_info(a, g, b, win, i);
    trow[i] = t.row;
    tpk[i] = (t.pos << 5) | (t.lab & 31);
  }
  if (RPB)
    for (int l = tid; l < g.L; l += dfk_bdim()) rpb2[l] = a.rpb[(long)l * a.heads + head] * kLog2e;
  for (int li = tid; li < Qn; li += dfk_bdim()) {
    const int i = q0 + li;
    lse2[li] = i < g.N ? a.lse[(long)dfk_bid_x() * g.Np + i] * kLog2e : INFINITY;
  }
  __syncthreads();
  // Q, dO rows -> swizzled LDS tiles; delta = rowsum(O * dO) (CH lanes per row)
  constexpr int CH = HD / 8;
  for (int base = 0; base < Qn * CH; base += dfk_bdim()) {
    const int idx = base + tid;
    float d = 0.f;
    if (idx < Qn * CH) {
      const int li = idx / CH, c = (idx % CH) * 8;
      const int row = trow[q0 + li];
      const uint4 qv = tok_ld16<bf16raw>(a.q, a.pad_q, row, a.ld_qkv, hoff + c);
      const uint4 dv = tok_ld16<bf16raw>(ba.dout, nullptr, row, ba.ld_dout, hoff + c);
      const uint4 ov = tok_ld16<bf16raw>(a.out, nullptr, row, a.ld_out, hoff + c);
      d = dot8_bf16(ov, dv);
      *reinterpret_cast<uint4*>(Qs + swz<HD>(li, c)) = qv;
      *reinterpret_cast<uint4*>(dOs + swz<HD>(li, c)) = dv;
    }
#pragma unroll
    for (int o = 1; o < CH; o <<= 1) d += __shfl_xor(d, o, 64);
    if (idx < Qn * CH && (idx % CH) == 0) delta[idx / CH] = d;
  }

  __syncthreads();

  // ---- passes over the key blocks: in pass p, wave w owns key block p*nwaves + w
  const int nkb = g.Np / 32, nqb = Qn / 32;
  bf16raw* Sw = Sd + wave * 32 * kSdStride;
  float* myQ = dQp + wave * 32 * kDqStride;
  const float scale2 = a.scale * kLog2e;
  const float mpen = -100.f * kLog2e;
  bf16raw* dsu = RPB && dsg ? dsg + (long)dfk_bid_x() * g.Np * g.Np : nullptr;   // this window-head's dS^T [k][q]
  for (int pass = 0; pass * nwaves < nkb; ++pass) {
    const int kb = pass * nwaves + wave;
    const bool own = kb < nkb;
    const int kbc = own ? kb : 0;
    // K^T / V^T B operands (key on the lane), K natural-order B operand for dQ, key statistics
    int kpk[2];
    float kneg[2];
    bf16x8 kB[2][HD / 32], vB[2][HD / 32], kN[HD / 16];
    f32x4 dK[2][HD / 16], dV[2][HD / 16];
#pragma unroll
    for (int h2 = 0; h2 < 2; ++h2) {
      const int k = kbc * 32 + h2 * 16 + ql;
      const int row = trow[k];
      kpk[h2] = tpk[k];
      kneg[h2] = row == -2 ? -INFINITY : 0.f;
#pragma unroll
      for (int es = 0; es < HD / 32; ++es) {
        kB[h2][es] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + es * 32 + grp * 8));
        vB[h2][es] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + es * 32 + grp * 8));
      }
#pragma unroll
      for (int et = 0; et < HD / 16; ++et) { dK[h2][et] = f32x4{0, 0, 0, 0}; dV[h2][et] = f32x4{0, 0, 0, 0}; }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = trow[kbc * 32 + grp * 8 + j];
#pragma unroll
      for (int et = 0; et < HD / 16; ++et)
        kN[et][j] = __builtin_bit_cast(__bf16, tok_ld1<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + ql + et * 16));
    }

    for (int qb = 0; qb < nqb; ++qb) {
      const int qr0 = qb * 32;
      f32x4 dq[2][HD / 16];
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) dq[qh][et] = f32x4{0, 0, 0, 0};
      if (own) {
        // query-side operands and statistics of the block
        f32x4 L2[2], DL[2];
        int4 QP[2];
        bf16x8 qa[2][HD / 32], da[2][HD / 32];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int r0 = qr0 + qh * 16 + grp * 4;
          L2[qh] = *reinterpret_cast<const f32x4*>(lse2 + r0);
          DL[qh] = *reinterpret_cast<const f32x4*>(delta + r0);
          QP[qh] = *reinterpret_cast<const int4*>(tpk + q0 + r0);
#pragma unroll
          for (int es = 0; es < HD / 32; ++es) {
            const int off = swz<HD>(qr0 + qh * 16 + ql, es * 32 + grp * 8);
            qa[qh][es] = *reinterpret_cast<const bf16x8*>(Qs + off);
            da[qh][es] = *reinterpret_cast<const bf16x8*>(dOs + off);
          }
        }
        float bias[2][2][4];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              bias[qh][h2][r] = RPB ? rpb2[(QP[qh][r] >> 5) - (kpk[h2] >> 5) + g.C0] : 0.f;
        // S = Q K^T, dP = dO V^T : rows = queries, lanes = keys
        f32x4 s[2][2], dp[2][2];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            s[qh][h2] = f32x4{0, 0, 0, 0};
            dp[qh][h2] = f32x4{0, 0, 0, 0};
#pragma unroll
            for (int es = 0; es < HD / 32; ++es) {
              s[qh][h2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qa[qh][es], kB[h2][es], s[qh][h2], 0, 0, 0);
              dp[qh][h2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(da[qh][es], vB[h2][es], dp[qh][h2], 0, 0, 0);
            }
          }
        // P = 2^(s*scale*log2e + bias - lse2); dS = P (dP - delta); A operands of P^T / dS^T
        bf16x8 pa[2], sa[2];
#pragma unroll
        for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
          for (int qh = 0; qh < 2; ++qh) {
            float dsv[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              float x = s[qh][h2][r] * scale2 + (bias[qh][h2][r] + kneg[h2] - L2[qh][r]);
              if (g.use_mask) x += ((QP[qh][r] ^ kpk[h2]) & 31) ? mpen : 0.f;
              if constexpr (MASK) {
                const int q = q0 + qr0 + qh * 16 + grp * 4 + r, k = kb * 32 + h2 * 16 + ql;
                if (q < g.N && k < g.N) x += mrow[q * g.N + k] * kLog2e;
              }
              const float P = __builtin_amdgcn_exp2f(x);
              const float dS = P * (dp[qh][h2][r] - DL[qh][r]);
              pa[h2][qh * 4 + r] = (__bf16)P;
              sa[h2][qh * 4 + r] = (__bf16)dS;
              dsv[r] = dS;
            }
            uint2 w;
            w.x = (uint32_t)f2bf(dsv[0]) | ((uint32_t)f2bf(dsv[1]) << 16);
            w.y = (uint32_t)f2bf(dsv[2]) | ((uint32_t)f2bf(dsv[3]) << 16);
            // dS^T -> wave scratch [32 keys][32 queries]
            *reinterpret_cast<uint2*>(Sw + (h2 * 16 + ql) * kSdStride + qh * 16 + grp * 4) = w;
          }
        // dV[k][e] += P^T dO ; dK[k][e] += dS^T Q   (query slot j <-> row qr0 + (j>>2)*16 + 4grp + (j&3))
#pragma unroll
        for (int et = 0; et < HD / 16; ++et) {
          const int c = et * 16 + tp * 4;
          const int rlo = qr0 + grp * 4 + tq, rhi = rlo + 16;
          const bf16x8 dob = tr16x2(dOs + swz<HD>(rlo, c), dOs + swz<HD>(rhi, c));
          const bf16x8 qbv = tr16x2(Qs + swz<HD>(rlo, c), Qs + swz<HD>(rhi, c));
#pragma unroll
          for (int h2 = 0; h2 < 2; ++h2) {
            dV[h2][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pa[h2], dob, dV[h2][et], 0, 0, 0);
            dK[h2][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sa[h2], qbv, dK[h2][et], 0, 0, 0);
          }
        }
        asm volatile("" ::: "memory");
        // partial dQ[q][e] = dS K over this key block (dS rows via tr16 from the scratch, keys in natural order)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const bf16x8 sq = tr16x2(Sw + (grp * 8 + tq) * kSdStride + qh * 16 + tp * 4,
                                   Sw + (grp * 8 + 4 + tq) * kSdStride + qh * 16 + tp * 4);
#pragma unroll
          for (int et = 0; et < HD / 16; ++et)
            dq[qh][et] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(sq, kN[et], dq[qh][et], 0, 0, 0);
        }
        if (dsu) {  // scratch rows (32 keys x 64 B) -> global dS^T[k][q], 2 x 16 B per lane
          const int kr = lane >> 1, half = lane & 1;
          const uint4 v0 = *reinterpret_cast<const uint4*>(Sw + kr * kSdStride + half * 16);
          const uint4 v1 = *reinterpret_cast<const uint4*>(Sw + kr * kSdStride + half * 16 + 8);
          bf16raw* gp = dsu + (long)(kb * 32 + kr) * g.Np + q0 + qr0 + half * 16;
          *reinterpret_cast<uint4*>(gp) = v0;
          *reinterpret_cast<uint4*>(gp + 8) = v1;
        }
        asm volatile("" ::: "memory");
      }
      // ---- dQ block: partials -> LDS, sum over waves, store (pass 0) or add (later passes)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int et = 0; et < HD / 16; ++et)
#pragma unroll
          for (int r = 0; r < 4; ++r) myQ[(qh * 16 + grp * 4 + r) * kDqStride + et * 16 + ql] = dq[qh][et][r];
      __syncthreads();
      const int nw = min(nwaves, nkb - pass * nwaves);
      for (int t = tid; t < 32 * (HD / 8); t += dfk_bdim()) {
        const int lr = t / (HD / 8), c = (t % (HD / 8)) * 8;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int w = 0; w < nw; ++w) {
          const float* src = dQp + (w * 32 + lr) * kDqStride + c;
          const f32x4 x0 = *reinterpret_cast<const f32x4*>(src), x1 = *reinterpret_cast<const f32x4*>(src + 4);
#pragma unroll
          for (int j = 0; j < 4; ++j) { v[j] += x0[j]; v[4 + j] += x1[j]; }
        }
        const int i = q0 + qr0 + lr;
        const int row = i < g.N ? trow[i] : -2;
        if (row >= 0) {
          bf16raw* dst = reinterpret_cast<bf16raw*>(ba.dq) + (long)row * ba.ld_dqkv + hoff + c;
          uint4 u = pass > 0 ? *reinterpret_cast<const uint4*>(dst) : make_uint4(0, 0, 0, 0);
          bf16raw* pe = reinterpret_cast<bf16raw*>(&u);
#pragma unroll
          for (int j = 0; j < 8; ++j) pe[j] = f2bf((pass > 0 ? bf2f(pe[j]) : 0.f) + v[j] * a.scale);
          *reinterpret_cast<uint4*>(dst) = u;
        } else if (row == -1 && ba.dpad_q) {
#pragma unroll
          for (int j = 0; j < 8; ++j) atomicAdd(ba.dpad_q + hoff + c + j, v[j] * a.scale);
        }
      }
      __syncthreads();
    }
    // ---- dK (scaled), dV of the owned key block: C layout row = key 4grp+r, col = e
    if (own) {
#pragma unroll
      for (int h2 = 0; h2 < 2; ++h2)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = trow[kb * 32 + h2 * 16 + grp * 4 + r];
#pragma unroll
          for (int et = 0; et < HD / 16; ++et) {
            const int e = hoff + et * 16 + ql;
            const float vk = dK[h2][et][r] * a.scale, vv = dV[h2][et][r];
            if (row >= 0) {
              bf16raw* pk = reinterpret_cast<bf16raw*>(ba.dk) + (long)row * ba.ld_dqkv + e;
              bf16raw* pv = reinterpret_cast<bf16raw*>(ba.dv) + (long)row * ba.ld_dqkv + e;
              *pk = f2bf(accum_kv ? bf2f(*pk) + vk : vk);
              *pv = f2bf(accum_kv ? bf2f(*pv) + vv : vv);
            } else if (row == -1) {
              if (ba.dpad_k) atomicAdd(ba.dpad_k + e, vk);
              if (ba.dpad_v) atomicAdd(ba.dpad_v + e, vv);
            }
          }
        }
    }
  }
}

// ------------------------------------------------- v3 backward (bf16 bias tiles, 32x32x16 MFMA)
// One workgroup = one (clip, window, head); wave w owns key blocks w, w + nw, ... (dK^T, dV^T in registers) and
// sweeps every query block STAGGERED (wave w at step i takes block (i + w) mod nqb), so at each step the waves
// add their partial dQ = dS K into distinct blocks of the fp32 LDS accumulator, behind one barrier per step (a
// fixed add order: deterministic).  Per step (32 queries x 32 keys, queries on the MFMA row, keys on the lane):
//   S' = Q' K^T + bias' - L'   (Q' = Q scale log2e, staged so in LDS; bias' - L' enters as the C input: -lse log2e
//                               read from LDS plus the bwd-layout bias tile unpacked on the VALU)
//   dP' = dO V^T - delta        (-delta as the C input; delta = rowsum(dO O))
//   P = 2^S', dS = P dP'        (dropout: dS = P (dP Z/keep - delta), P Z/keep into dV)
//   dV^T += dO^T P, dK^T += Q'^T dS  (the score accumulators are the B operands: no lane movement)
//   dQ_part = dS K              (dS crosses the wave's LDS scratch once, as dS^T, read back transposed)
// dS^T also goes to the global scratch (dsg) for the deterministic dRPB reduction.
// COS (SwinV2 cosine attention, ba.dscore): the gradient of a per-head multiplier of the scores (logit_scale,
// swin_transformer2d.py:155-157), dscore[h] += sum_q sum_k dS ⊙ score — in fp32 from the fp32 P, dP and score the
// loop already holds, with the softmax-backward row constant taken exactly: per row, A' = sum_k P (dP - delta) r,
// D' = sum_k P (dP - delta), B = sum_k P r (r = the score before bias, sum_k P = 1), so sum_k dS r with the exact
// delta = sum_k P dP is A' - D' B whatever the bf16 forward output made of delta = dO . O.  The per-lane A' is one
// running sum; D' and B are reduced over the 32 key lanes (transposed halving) and added into per-row LDS sums by
// the wave that owns the row's block at that step (the staggered order: deterministic).
constexpr int kSdRow = 32;   // bf16 per row of the [32 keys][32 queries] dS^T scratch (64 B)

// element (k, q) of the dS^T scratch: 8-B column groups XOR-swizzled by k so that the packed stores (4 x 16 lanes,
// bank (a/4) mod 32) and the tr16 reads (2 x 32 lanes, mod 64) are conflict-free
__device__ __forceinline__ int sd_off(int k, int q) { return k * kSdRow + ((((q >> 2) ^ (k >> 1)) & 7) << 2) + (q & 3); }

// two packed bf16 pairs + two packed bf16 pairs, fp32 add, round to nearest even
__device__ __forceinline__ uint2 add_bf16x4(uint2 x, uint2 y) {
  typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
  auto add2 = [](uint32_t p, uint32_t q) {
    const float lo = __uint_as_float(p << 16) + __uint_as_float(q << 16);
    const float hi = __uint_as_float(p & 0xffff0000u) + __uint_as_float(q & 0xffff0000u);
    return __builtin_bit_cast(uint32_t, bf16x2v{(__bf16)lo, (__bf16)hi});   // v_cvt_pk_bf16_f32 (RNE)
  };
  return make_uint2(add2(x.x, y.x), add2(x.y, y.y));
}

// halving reduction of 16 per-lane values over the 32 lanes of a half-wave: lane l ends with the sum of register
// (l >> 1) & 15 over the 32 lanes (l = lane & 31)
__device__ __forceinline__ float halving_sum16(float (&v)[16], int lane) {
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int n = 8 >> st, m = 16 >> st;
    const bool lo = (lane & m) == 0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const float send = lo ? v[n + i] : v[i];
      const float keep = lo ? v[i] : v[n + i];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  return v[0] + __shfl_xor(v[0], 1, 64);
}

// the same, with the 16 values produced on the fly by f(j) (the first halving step consumes them in pairs j,
// j + 8: 8 live values instead of 16)
template <typename F>
__device__ __forceinline__ float halving_sum16_fn(F f, int lane) {
  float v[8];
  const bool lo16 = (lane & 16) == 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float a = f(i), b = f(8 + i);
    v[i] = (lo16 ? a : b) + __shfl_xor(lo16 ? b : a, 16, 64);
  }
#pragma unroll
  for (int st = 1; st < 4; ++st) {
    const int n = 8 >> st, m = 16 >> st;
    const bool lo = (lane & m) == 0;
#pragma unroll
    for (int i = 0; i < n; ++i) {
      const float send = lo ? v[n + i] : v[i];
      const float keep = lo ? v[i] : v[n + i];
      v[i] = keep + __shfl_xor(send, m, 64);
    }
  }
  return v[0] + __shfl_xor(v[0], 1, 64);
}

template <int HD, bool TAB, bool DROP, bool COS = false>
__global__ __launch_bounds__(COS ? 256 : 512) void wattn_bwd3_kernel(const dfk_wattn_bwd_args ba, const Geo g, int q0, int Qn,
                                                         int accum_kv, bf16raw* __restrict__ dsg,
                                                         const bf16raw* __restrict__ tabb, int G) {
  constexpr int NKK = HD / 16, NOT = HD / 32, CH = HD / 8;
  const dfk_wattn_args& a = ba.f;
  const int nw = dfk_bdim() >> 6;
  // queries [q0, q0 + Qn) of every window (Qn = Np unless the window's Q / dO / dQ do not fit the LDS: then
  // several launches, dK / dV accumulated in place by the later ones)
  const int Np = g.Np, nkb = Np / 32, nqb = Qn / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* p = smem;
  float* dQa = reinterpret_cast<float*>(p); p += 4 * (size_t)Qn * HD;   // [qb][ot][v][lane][4]
  bf16raw* Qs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Qn * HD;  // Q' = Q scale log2e
  bf16raw* dOs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Qn * HD;
  bf16raw* Sd = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)nw * 32 * kSdRow;
  int* trow = reinterpret_cast<int*>(p); p += 4 * Np;
  float* nl2 = reinterpret_cast<float*>(p); p += 4 * Qn;   // -lse log2e; -inf beyond N (P = 0)
  float* ndl = reinterpret_cast<float*>(p); p += 4 * Qn;   // -delta
  float* rowD = reinterpret_cast<float*>(p); p += COS ? 4 * Qn : 0;   // COS: D' and B per query row
  float* rowB = reinterpret_cast<float*>(p); p += COS ? 4 * Qn : 0;
  float* red = reinterpret_cast<float*>(p); p += COS ? 4 * 16 : 0;
  static_assert(!(COS && (DROP || !TAB)), "COS: bias-table path without dropout");

  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int r = lane & 31, hh = lane >> 5, g16 = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  const WGroup gr = decode_group(a, g, G);   // G windows of one (class, head), one dRPB scratch slab
  for (int gi = 0; gi < gr.n; ++gi) {
  float accA = 0.f;
  const WUnit wu = group_window(a, g, gr, G, gi);   // lse / dropout rows by lse_unit (the host runs G = 1 here)
  const int head = wu.head, win = wu.win, b = wu.b;
  const long unit = wu.lse_unit;
  const int hoff = head * HD;
  // bias tiles through a buffer descriptor (wave-uniform base in SGPRs): the lane's 16 B in the VGPR offset,
  // the (qb, kb) tile in the SGPR offset
  const uint64_t tp64 = TAB ? reinterpret_cast<uint64_t>(tabb + ((long)wu.cls * a.heads + head) * (long)Np * Np) : 0;
  const uint64_t tpu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(tp64 >> 32)) << 32) |
                       (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)tp64);   // no sign extension
  const __amdgpu_buffer_rsrc_t trs =
      __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tpu), (short)0, TAB ? 0x7fffffff : 0, 0x00020000);
  const float qs = a.scale * kLog2e;

  for (int i = tid; i < Np; i += dfk_bdim()) trow[i] = token_info_row(a, g, b, win, i);
  for (int i = tid; i < Qn; i += dfk_bdim())
    nl2[i] = q0 + i < g.N ? -a.lse[unit * Np + q0 + i] * kLog2e : -INFINITY;
  for (int i = tid * 4; i < Qn * HD; i += dfk_bdim() * 4) *reinterpret_cast<f32x4*>(dQa + i) = f32x4{0, 0, 0, 0};
  if constexpr (COS)
    for (int i = tid; i < Qn; i += dfk_bdim()) rowD[i] = rowB[i] = 0.f;
  __syncthreads();
  // Q / dO / O gather, QB row chunks per thread in flight (all loads of a batch issued before the wait that
  // precedes their use: one HBM round trip per batch, not per chunk)
  {
    constexpr int QB = 4;
    const int tot = Qn * CH;
    for (int base = 0; base < tot; base += QB * dfk_bdim()) {
      uint4 qv[QB], dv[QB], ov[QB];
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const int idx = min(base + u * (int)dfk_bdim() + tid, tot - 1);
        const int li = idx / CH, c = (idx % CH) * 8;
        const int row = trow[q0 + li];
        qv[u] = tok_ld16<bf16raw>(a.q, a.pad_q, row, a.ld_qkv, hoff + c);
        dv[u] = tok_ld16<bf16raw>(ba.dout, nullptr, row, ba.ld_dout, hoff + c);
        ov[u] = tok_ld16<bf16raw>(a.out, nullptr, row, a.ld_out, hoff + c);
      }
#pragma unroll
      for (int u = 0; u < QB; ++u) {
        const int idx = base + u * (int)dfk_bdim() + tid;   // CH | blockDim: a row's CH lanes agree on idx < tot
        float d = dot8_bf16(ov[u], dv[u]);
#pragma unroll
        for (int o = 1; o < CH; o <<= 1) d += __shfl_xor(d, o, 64);
        if (idx < tot) {
          const int li = idx / CH, c = (idx % CH) * 8;
          bf16x8 qb8 = __builtin_bit_cast(bf16x8, qv[u]);
#pragma unroll
          for (int j = 0; j < 8; ++j) qb8[j] = (__bf16)((float)qb8[j] * qs);   // the forward's Q' rounding, bit for bit
          *reinterpret_cast<bf16x8*>(Qs + swz<HD>(li, c)) = qb8;
          *reinterpret_cast<uint4*>(dOs + swz<HD>(li, c)) = dv[u];
          if ((idx % CH) == 0) ndl[li] = -d;
        }
      }
    }
  }
  __syncthreads();

  bf16raw* Sw = Sd + wave * 32 * kSdRow;
  const DropCtx dc = drop_ctx(a.drop);
  bf16raw* dsu = dsg ? dsg + gr.slab * Np * Np : nullptr;   // the group's dS^T slab [k][q]
  // per-lane LDS offsets (the tile swizzle sees a row only through bits a 32-row block step and a 16-row
  // k-step leave unchanged): Q' / dO row fragments (+ qr0 HD) and the transposed tr16 reads (+ qr0 HD + 16 c HD)
  int qoff[NKK], tlo[NOT], thi[NOT];
#pragma unroll
  for (int kk = 0; kk < NKK; ++kk) qoff[kk] = swz<HD>(r, kk * 16 + hh * 8);
#pragma unroll
  for (int ot = 0; ot < NOT; ++ot) {
    const int k0 = 4 * (g16 >> 1) + tq, col = ot * 32 + 16 * (g16 & 1) + 4 * tp;
    tlo[ot] = swz<HD>(k0, col);
    thi[ot] = swz<HD>(k0 + 8, col);
  }
  for (int pass = 0; pass * nw < nkb; ++pass) {
    const int kb = pass * nw + wave;
    if (kb >= nkb) {   // no key block this pass: keep the step barriers
      for (int i = 0; i < nqb; ++i) __syncthreads();
      continue;
    }
    // K^T / V^T B operands (key on the lane) and K as the B operand of dQ = dS K (e on the lane)
    const int krow = trow[kb * 32 + r];
    const float kneg = kb * 32 + r < g.N ? 0.f : -INFINITY;   // keys beyond N (the bias tiles also hold -1e4 there)
    bf16x8 kB[NKK], vB[NKK], kN[2][NOT];
#pragma unroll
    for (int kk = 0; kk < NKK; ++kk) {
      kB[kk] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.k, a.pad_k, krow, a.ld_qkv, hoff + kk * 16 + hh * 8));
      vB[kk] = __builtin_bit_cast(bf16x8, tok_ld16<bf16raw>(a.v, a.pad_v, krow, a.ld_qkv, hoff + kk * 16 + hh * 8));
    }
    {   // K as dQ's B operand (e on the lane): 16 NOT scattered 2-byte loads, all issued before any is used (one
        // after another, each behind its own vmcnt(0), they cost a memory round trip apiece)
      const bf16raw* kp[2][8][NOT];
      bool kok[2][8];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = trow[kb * 32 + 16 * s + 8 * hh + j];
#pragma unroll
          for (int ot = 0; ot < NOT; ++ot)
            kp[s][j][ot] = tok_src<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + ot * 32 + r, kok[s][j]);
        }
      bf16raw kv[2][8][NOT];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int ot = 0; ot < NOT; ++ot) kv[s][j][ot] = __builtin_nontemporal_load(kp[s][j][ot]);
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int ot = 0; ot < NOT; ++ot)
            kN[s][ot][j] = __builtin_bit_cast(__bf16, kok[s][j] ? kv[s][j][ot] : (bf16raw)0);
    }
    f32x16 dKt[NOT], dVt[NOT];
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int j = 0; j < 16; ++j) { dKt[ot][j] = 0.f; dVt[ot][j] = 0.f; }
    bf16x8 bt[2];
    auto load_bias = [&](int qb) {
      if constexpr (TAB) {
        const int so = __builtin_amdgcn_readfirstlane(((q0 / 32 + qb) * nkb + kb) * 2048);
#pragma unroll
        for (int c = 0; c < 2; ++c)
          bt[c] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(trs, lane * 16, so + c * 1024, 0));
      }
    };
    int qb = wave % nqb;
    load_bias(qb);
    for (int i = 0; i < nqb; ++i, qb = qb + 1 == nqb ? 0 : qb + 1) {
      const int qr0 = qb * 32;   // local row of the block in the chunk
      bf16raw* const gp = dsu ? dsu + (long)(kb * 32 + (lane >> 1)) * Np + q0 + qr0 + (lane & 1) * 16 : nullptr;
      // row constants as the C inputs: queries q0 + 8 v + 4 hh + (0..3) in registers 4v .. 4v+3
      f32x16 s, dp;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(nl2 + qr0 + 8 * v + 4 * hh);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(ndl + qr0 + 8 * v + 4 * hh);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          s[4 * v + t] = TAB ? l4[t] : l4[t] + kneg;   // the bias tiles hold -1e4 for keys beyond N
          dp[4 * v + t] = DROP ? 0.f : d4[t];
        }
      }
      if constexpr (TAB) {   // bias' (C-input layout: element 8c + j of the lane's key) added to -L'
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const uint4 w4 = __builtin_bit_cast(uint4, bt[c]);
          const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            s[8 * c + 2 * i] += __uint_as_float(w[i] << 16);
            s[8 * c + 2 * i + 1] += __uint_as_float(w[i] & 0xffff0000u);
          }
        }
        load_bias(qb + 1 == nqb ? 0 : qb + 1);
      }
      f32x16 cin;   // COS: the product alone is the score (rows beyond N: c = -inf, the product stays finite)
      if constexpr (COS) {
        cin = s;
#pragma unroll
        for (int j = 0; j < 16; ++j) s[j] = 0.f;
      }
#pragma unroll
      for (int kk = 0; kk < NKK; ++kk) {
        const int off = qr0 * HD + qoff[kk];
        const bf16x8 qa = *reinterpret_cast<const bf16x8*>(Qs + off);
        const bf16x8 da = *reinterpret_cast<const bf16x8*>(dOs + off);
        s = mfma32(qa, kB[kk], s);
        dp = mfma32(da, vB[kk], dp);
      }
      f32x16 raw;
      if constexpr (COS) {
        raw = s;
        s = s + cin;
      }

      // P = 2^S', dS = P dP'; B-operand fragments of k-steps c (registers 8c .. 8c+7)
      bf16x8 pa[2], sa[2];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float P = __builtin_amdgcn_exp2f(s[8 * c + j]);
          if constexpr (DROP) {
            const int q = qr0 + 8 * (2 * c + (j >> 2)) + 4 * hh + (j & 3);
            const float mk = drop_mul(dc, unit * Np + q0 + q, kb * 32 + r);
            pa[c][j] = (__bf16)(P * mk);
            sa[c][j] = (__bf16)(P * (dp[8 * c + j] * mk + ndl[q]));
          } else {
            pa[c][j] = (__bf16)P;
            sa[c][j] = (__bf16)(P * dp[8 * c + j]);
          }
        }
      float cosD = 0.f, cosB = 0.f;   // COS: this lane's row (register (r >> 1) & 15) sums over the block's keys
      if constexpr (COS) {   // the values produced as the halving consumes them (register pressure)
        cosD = halving_sum16_fn([&](int j) __attribute__((always_inline)) {
          const float ds = __builtin_amdgcn_exp2f(s[j]) * dp[j];
          accA += ds * raw[j];
          return ds;
        }, lane);
        cosB = halving_sum16_fn([&](int j) __attribute__((always_inline)) {
          return __builtin_amdgcn_exp2f(s[j]) * raw[j];
        }, lane);
      }
      // dS^T -> the wave's scratch: registers 4v .. 4v+3 (queries 8v + 4hh + 0..3) at [key r][8v + 4hh]
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const uint4 u = __builtin_bit_cast(uint4, sa[c]);
        *reinterpret_cast<uint2*>(Sw + sd_off(r, 16 * c + 4 * hh)) = make_uint2(u.x, u.y);
        *reinterpret_cast<uint2*>(Sw + sd_off(r, 16 * c + 8 + 4 * hh)) = make_uint2(u.z, u.w);
      }
      // dV^T += dO^T P, dK^T += Q'^T dS: A rows e = 32 ot + r, k-step c slots <-> queries 16 c + 8 (j>>2) + 4 hh + (j&3)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int rb = (qr0 + 16 * c) * HD;
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) {
          const bf16x8 doT = tr16x2(dOs + rb + tlo[ot], dOs + rb + thi[ot]);
          const bf16x8 qT = tr16x2(Qs + rb + tlo[ot], Qs + rb + thi[ot]);
          dVt[ot] = mfma32(doT, pa[c], dVt[ot]);
          dKt[ot] = mfma32(qT, sa[c], dKt[ot]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the wave's own scratch writes (LDS only)
      __builtin_amdgcn_wave_barrier();
      // partial dQ = dS K: A = dS (row q = r, k-step s slots 8 hh + j <-> keys 16 s + 8 hh + j) read transposed
      f32x16 dq[NOT];
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int j = 0; j < 16; ++j) dq[ot][j] = 0.f;
#pragma unroll
      for (int sk = 0; sk < 2; ++sk) {
        const int k0 = 16 * sk + 8 * (g16 >> 1) + tq, qc = 16 * (g16 & 1) + 4 * tp;
        const bf16x8 dsa = tr16x2(Sw + sd_off(k0, qc), Sw + sd_off(k0 + 4, qc));
#pragma unroll
        for (int ot = 0; ot < NOT; ++ot) dq[ot] = mfma32(dsa, kN[sk][ot], dq[ot]);
      }
      if (dsu) {   // scratch rows (32 keys x 64 B) -> global dS^T[k][q]: lane (key kr, half) un-swizzles 2 x 16 B
        const int kr = lane >> 1, half = lane & 1;
        const uint2 x0 = *reinterpret_cast<const uint2*>(Sw + sd_off(kr, half * 16));
        const uint2 x1 = *reinterpret_cast<const uint2*>(Sw + sd_off(kr, half * 16 + 4));
        const uint2 x2 = *reinterpret_cast<const uint2*>(Sw + sd_off(kr, half * 16 + 8));
        const uint2 x3 = *reinterpret_cast<const uint2*>(Sw + sd_off(kr, half * 16 + 12));
#ifdef DFK_DS_NT
        typedef unsigned int u32x4n __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(u32x4n{x0.x, x0.y, x1.x, x1.y}, reinterpret_cast<u32x4n*>(gp));
        __builtin_nontemporal_store(u32x4n{x2.x, x2.y, x3.x, x3.y}, reinterpret_cast<u32x4n*>(gp + 8));
#else
        *reinterpret_cast<uint4*>(gp) = make_uint4(x0.x, x0.y, x1.x, x1.y);
        *reinterpret_cast<uint4*>(gp + 8) = make_uint4(x2.x, x2.y, x3.x, x3.y);
#endif
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // scratch reads done before the next step's writes
      __builtin_amdgcn_wave_barrier();
      __syncthreads();   // every wave has finished the previous step's adds: block qb is this wave's alone
#pragma unroll
      for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          f32x4* ap = reinterpret_cast<f32x4*>(dQa + ((size_t)((qb * NOT + ot) * 4 + v) * 64 + lane) * 4);
          *ap = *ap + f32x4{dq[ot][4 * v], dq[ot][4 * v + 1], dq[ot][4 * v + 2], dq[ot][4 * v + 3]};
        }
      if constexpr (COS) {
        if ((r & 1) == 0) {   // register j = (r >> 1) & 15 <-> query 8 (j >> 2) + 4 hh + (j & 3) of the block
          const int j = (r >> 1) & 15, q = qr0 + 8 * (j >> 2) + 4 * hh + (j & 3);
          rowD[q] += cosD;
          rowB[q] += cosB;
        }
      }
    }
    // dK = scale sum dS q = (sum dS Q') ln 2, dV: lane holds key r, e = 32 ot + (j & 3) + 8 (j >> 2) + 4 hh
    const float kscale = 0.6931471805599453f;
#pragma unroll
    for (int ot = 0; ot < NOT; ++ot)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int e = hoff + ot * 32 + 8 * v + 4 * hh;
        if (krow >= 0) {
          bf16raw* pk = reinterpret_cast<bf16raw*>(ba.dk) + (long)krow * ba.ld_dqkv + e;
          bf16raw* pv = reinterpret_cast<bf16raw*>(ba.dv) + (long)krow * ba.ld_dqkv + e;
          float vk[4], vv[4];
#pragma unroll
          for (int t = 0; t < 4; ++t) { vk[t] = dKt[ot][4 * v + t] * kscale; vv[t] = dVt[ot][4 * v + t]; }
          if (accum_kv) {   // a later query chunk: add to the earlier chunks' partial sums
#pragma unroll
            for (int t = 0; t < 4; ++t) { vk[t] += bf2f(pk[t]); vv[t] += bf2f(pv[t]); }
          }
          uint2 uk, uv;
          uk.x = (uint32_t)f2bf(vk[0]) | ((uint32_t)f2bf(vk[1]) << 16);
          uk.y = (uint32_t)f2bf(vk[2]) | ((uint32_t)f2bf(vk[3]) << 16);
          uv.x = (uint32_t)f2bf(vv[0]) | ((uint32_t)f2bf(vv[1]) << 16);
          uv.y = (uint32_t)f2bf(vv[2]) | ((uint32_t)f2bf(vv[3]) << 16);
          *reinterpret_cast<uint2*>(pk) = uk;
          *reinterpret_cast<uint2*>(pv) = uv;
        } else if (krow == -1) {
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            if (ba.dpad_k) atomicAdd(ba.dpad_k + e + t, dKt[ot][4 * v + t] * kscale);
            if (ba.dpad_v) atomicAdd(ba.dpad_v + e + t, dVt[ot][4 * v + t]);
          }
        }
      }
  }
  __syncthreads();
  if constexpr (COS) {   // dscore[head] += ln2 (sum A' - sum_q D'_q B_q): the score is r' ln 2 (r' in log2 units)
    float t = accA;
    for (int i = tid; i < Qn; i += dfk_bdim()) t -= rowD[i] * rowB[i];
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) t += __shfl_xor(t, o, 64);
    if (lane == 0) red[wave] = t;
    __syncthreads();
    if (tid == 0) {
      float tot = 0.f;
      for (int w = 0; w < nw; ++w) tot += red[w];
      atomicAdd(ba.dscore + head, tot * 0.6931471805599453f);
    }
  }
  // dQ rows (scaled): (q, e) of block qb sits at [qb][ot][v][lane][t], q = 32 qb + 8 v + 4 h + t, lane = (e & 31) + 32 h
  for (int t8 = tid; t8 < Qn * (HD / 8); t8 += dfk_bdim()) {
    const int i = t8 / (HD / 8), c = (t8 % (HD / 8)) * 8;
    const int row = q0 + i < g.N ? trow[q0 + i] : -2;
    const int qb = i >> 5, qi = i & 31, v = qi >> 3, h2 = (qi >> 2) & 1, t = qi & 3, ot = c >> 5;
    const float* src = dQa + ((size_t)((qb * NOT + ot) * 4 + v) * 64 + (c & 31) + 32 * h2) * 4 + t;
    float vv[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) vv[j] = src[j * 4] * a.scale;
    if (row >= 0) {
      uint4 u;
      bf16raw* pe = reinterpret_cast<bf16raw*>(&u);
#pragma unroll
      for (int j = 0; j < 8; ++j) pe[j] = f2bf(vv[j]);
      *reinterpret_cast<uint4*>(reinterpret_cast<bf16raw*>(ba.dq) + (long)row * ba.ld_dqkv + hoff + c) = u;
    } else if (row == -1 && ba.dpad_q) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(ba.dpad_q + hoff + c + j, vv[j]);
    }
  }
  __syncthreads();   // the next window of the group reuses trow / dQa / the statistics
  }
}

// ------------------------------------------------- v4 backward: two passes, no barriers in the main loops
// One workgroup = G windows of one (shift class, head) in turn (decode_group); per window the prologue stages Q'
// (= Q scale log2e), dO, K and V of the whole window in LDS (one image each, XOR-swizzled), -lse log2e and -delta
// per query.  Then every wave takes work units on its own, with no barrier until the next window:
//   pass A, unit = key block kb (keys on the lane, as wattn_bwd3): for every query block S = Q' K^T + bias' - L',
//     dP = dO V^T - delta, P = 2^S, dS = P dP; dV^T += dO^T P, dK^T += Q'^T dS in registers; dS^T -> the dRPB slab.
//   pass B, unit = query block qb (queries on the lane, the v6 forward's 16x16x32 sub-tiles and bias layout): for
//     every key block S^T and dP^T the same way, dQ^T += K^T dS^T in registers (dS^T is the accumulator itself,
//     in the PV slot order of the forward: no LDS transpose).
// The score products run twice (S and dP in both passes: 14 instead of 10 MFMA-equivalents per block), in exchange
// for no dQ reduction across waves, no per-step barrier and no dS LDS round trip — wattn_bwd3's staggered loop
// spent most of each step waiting on those.  bf16 table path, hd 32, no dropout, windows of >= 4 query blocks (the
// v6 forward's bias layout).
constexpr int kB4Waves = 8;

// Which work units (pass-A key blocks 0..nb-1, pass-B query blocks nb..2nb-1) each wave of a bwd4 workgroup runs:
// byte w (w <= kB4Waves) = the first list position of wave w, the unit list from byte 16 on.  Round robin
// (u = wave, wave + 8, ...) gives a 392-token window's 26 units to the 8 waves as 4/4/3/.../3; the host plans a
// longest-processing-time assignment instead (a pass-A step runs 4 products, a pass-B step 3): makespan 12 against
// 14 such products per window.
struct B4Sched { uint32_t w[16]; };
__device__ __forceinline__ int b4_sched_byte(const B4Sched& sc, int i) { return (sc.w[i >> 2] >> (8 * (i & 3))) & 0xff; }

// Hand-counted buffer loads / stores for bwd4's pass A: the compiler's waitcnt placement put a vmcnt(0) at the top
// of every step of a loop that mixes loads and stores (each step then waited for its predecessor's scratch stores
// and read-modify-write loads to land), so the loop's memory operations are inline asm with explicit counts.  The
// compiler does not count them: its own waits can only grow more conservative, never wrong.
typedef int b4_v4i __attribute__((ext_vector_type(4)));
typedef unsigned int b4_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int b4_u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ b4_v4i b4_rsrc(const void* base, int bytes) {
  const uint64_t p = reinterpret_cast<uint64_t>(base);
  b4_v4i r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(uint32_t)p);
  r[1] = __builtin_amdgcn_readfirstlane((int)((uint32_t)(p >> 32) & 0xffffu));   // stride 0
  r[2] = __builtin_amdgcn_readfirstlane(bytes);
  r[3] = 0x00020000;
  return r;
}
__device__ __forceinline__ b4_u32x4 b4_ld128(b4_v4i rs, uint32_t voff, int soff) {
  b4_u32x4 d;
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(rs), "s"(soff));
  return d;
}
__device__ __forceinline__ b4_u32x2 b4_ld64(b4_v4i rs, uint32_t voff) {
  b4_u32x2 d;
  asm volatile("buffer_load_dwordx2 %0, %1, %2, 0 offen" : "=v"(d) : "v"(voff), "s"(rs));
  return d;
}
__device__ __forceinline__ void b4_st64(b4_v4i rs, uint32_t voff, b4_u32x2 x) {
  asm volatile("buffer_store_dwordx2 %0, %1, %2, 0 offen" : : "v"(x), "v"(voff), "s"(rs));
}

__global__ __launch_bounds__(512) void wattn_bwd4_kernel(const dfk_wattn_bwd_args ba, const Geo g,
                                                         bf16raw* __restrict__ dsg, const bf16raw* __restrict__ tabf,
                                                         const bf16raw* __restrict__ tabb, int G, const B4Sched sched) {
  constexpr int HD = 32, CH = HD / 8;
  const dfk_wattn_args& a = ba.f;
  const int Np = g.Np, nb = Np / 32;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* p = smem;
  bf16raw* Qs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Np * HD;
  bf16raw* dOs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Np * HD;
  bf16raw* Ks = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Np * HD;
  bf16raw* Vs = reinterpret_cast<bf16raw*>(p); p += 2 * (size_t)Np * HD;
  int* trow = reinterpret_cast<int*>(p); p += 4 * Np;
  float* nl2 = reinterpret_cast<float*>(p); p += 4 * Np;   // -lse log2e; -inf beyond N (P = 0)
  float* ndl = reinterpret_cast<float*>(p); p += 4 * Np;   // -delta

  const int tid = dfk_tid(), lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nw = dfk_bdim() >> 6;
  const int r = lane & 31, hh = lane >> 5, g16 = lane >> 4, ql = lane & 15, tq = ql >> 2, tp = lane & 3;
  const WGroup gr = decode_group(a, g, G);
  const int head = gr.head, hoff = head * HD;
  const float qs = a.scale * kLog2e;
  // bias tiles (bwd layout for pass A, the v6 forward layout for pass B) through buffer descriptors
  auto rsrc = [&](const bf16raw* base) __attribute__((always_inline)) {
    const uint64_t t64 = reinterpret_cast<uint64_t>(base + ((long)gr.cls * a.heads + head) * (long)Np * Np);
    const uint64_t tu = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(t64 >> 32)) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)t64);
    return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(tu), (short)0, 0x7fffffff, 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t trA = rsrc(tabb), trB = rsrc(tabf);
  // the group's dS^T slab [k][q] through buffer descriptors, so no branch surrounds its loads and stores (a
  // branch-guarded load got a vmcnt(0) right behind it): range 0 drops the stores / reads zeros
  bf16raw* const dsu = dsg ? dsg + gr.slab * Np * Np : nullptr;
  const int slab_bytes = __builtin_amdgcn_readfirstlane(dsu ? Np * Np * 2 : 0);
  const uint64_t s64 = reinterpret_cast<uint64_t>(dsu ? dsu : reinterpret_cast<bf16raw*>(ba.dq));
  const uint64_t su = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(s64 >> 32)) << 32) |
                      (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)s64);
  const b4_v4i sst = b4_rsrc(reinterpret_cast<void*>(su), slab_bytes);
  const b4_v4i tbA = b4_rsrc(tabb + ((long)gr.cls * a.heads + head) * (long)Np * Np, 0x7fffffff);

  // per-lane LDS offsets (swz<32> depends on row bits 2-3 only: valid at any 32-row block offset)
  int qoffA[2], tlo, thi, koffB[2], vlo[2], vhi[2];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) qoffA[kk] = swz<HD>(r, kk * 16 + hh * 8);
  {
    const int k0 = 4 * (g16 >> 1) + tq, col = 16 * (g16 & 1) + 4 * tp;
    tlo = swz<HD>(k0, col);
    thi = swz<HD>(k0 + 8, col);
  }
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    koffB[h] = swz<HD>(16 * h + ql, 8 * g16);
    vlo[h] = swz<HD>(4 * g16 + tq, 16 * h + 4 * tp);
    vhi[h] = swz<HD>(16 + 4 * g16 + tq, 16 * h + 4 * tp);
  }

  for (int gi = 0; gi < gr.n; ++gi) {
    const WUnit wu = group_window(a, g, gr, G, gi);
    // later windows of the group add into what the first one stored
    const b4_v4i sld = b4_rsrc(reinterpret_cast<void*>(su), gi > 0 ? slab_bytes : 0);
    const long unit = wu.lse_unit;
    for (int i = tid; i < Np; i += dfk_bdim()) {
      trow[i] = token_info_row(a, g, wu.b, wu.win, i);
      nl2[i] = i < g.N ? -a.lse[unit * Np + i] * kLog2e : -INFINITY;
    }
    __syncthreads();
    // Q' / dO / O / K / V gather (all of a batch's loads issued before the wait that precedes their use)
    {
      constexpr int QB = 2;
      const int tot = Np * CH;
      for (int base = 0; base < tot; base += QB * dfk_bdim()) {
        uint4 qv[QB], dv[QB], ov[QB], kv[QB], vv[QB];
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int idx = min(base + u * (int)dfk_bdim() + tid, tot - 1);
          const int li = idx / CH, c = (idx % CH) * 8;
          const int row = trow[li];
          qv[u] = tok_ld16<bf16raw>(a.q, a.pad_q, row, a.ld_qkv, hoff + c);
          dv[u] = tok_ld16<bf16raw>(ba.dout, nullptr, row, ba.ld_dout, hoff + c);
          ov[u] = tok_ld16<bf16raw>(a.out, nullptr, row, a.ld_out, hoff + c);
          kv[u] = tok_ld16<bf16raw>(a.k, a.pad_k, row, a.ld_qkv, hoff + c);
          vv[u] = tok_ld16<bf16raw>(a.v, a.pad_v, row, a.ld_qkv, hoff + c);
        }
#pragma unroll
        for (int u = 0; u < QB; ++u) {
          const int idx = base + u * (int)dfk_bdim() + tid;   // CH | blockDim: a row's CH lanes agree on idx < tot
          float d = dot8_bf16(ov[u], dv[u]);
#pragma unroll
          for (int o = 1; o < CH; o <<= 1) d += __shfl_xor(d, o, 64);
          if (idx < tot) {
            const int li = idx / CH, c = (idx % CH) * 8;
            bf16x8 qb8 = __builtin_bit_cast(bf16x8, qv[u]);
#pragma unroll
            for (int j = 0; j < 8; ++j) qb8[j] = (__bf16)((float)qb8[j] * qs);   // the forward's Q' rounding
            const int off = swz<HD>(li, c);
            *reinterpret_cast<bf16x8*>(Qs + off) = qb8;
            *reinterpret_cast<uint4*>(dOs + off) = dv[u];
            *reinterpret_cast<uint4*>(Ks + off) = kv[u];
            *reinterpret_cast<uint4*>(Vs + off) = vv[u];
            if ((idx % CH) == 0) ndl[li] = -d;
          }
        }
      }
    }
    __syncthreads();

    const int us0 = __builtin_amdgcn_readfirstlane(b4_sched_byte(sched, wave));
    const int us1 = __builtin_amdgcn_readfirstlane(b4_sched_byte(sched, wave + 1));
    for (int ui = us0; ui < us1; ++ui) {
      const int u = __builtin_amdgcn_readfirstlane(b4_sched_byte(sched, 16 + ui));
      if (u < nb) {
        // ---------------- pass A: key block kb, keys on the lane (C layout: row q = 8v + 4hh + t, col key r)
        const int kb = u;
        const int krow = trow[kb * 32 + r];
        bf16x8 kB[2], vB[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int off = kb * 32 * HD + qoffA[kk];
          kB[kk] = *reinterpret_cast<const bf16x8*>(Ks + off);
          vB[kk] = *reinterpret_cast<const bf16x8*>(Vs + off);
        }
        f32x16 dKt, dVt;
#pragma unroll
        for (int j = 0; j < 16; ++j) { dKt[j] = 0.f; dVt[j] = 0.f; }
        // per step i, in issue order: [wait bias(i)] bias(i+1) ... [wait old(i)] stores(i) old(i+1); so the bias of
        // step i has the 8 operations of step i-1's tail younger than it, and old(i) the 2 bias loads of step i
        b4_u32x4 bt0, bt1;
        auto load_bias = [&](int qb) __attribute__((always_inline)) {
          const int so = __builtin_amdgcn_readfirstlane((qb * nb + kb) * 2048);
          bt0 = b4_ld128(tbA, lane * 16, so);
          bt1 = b4_ld128(tbA, lane * 16 + 1024, so);
        };
        // slab tile (kb, qb): 2 KB at (kb nb + qb) 2048, [v][lane][4 queries] (drpb_from_ds_kernel tiled = 1)
        const uint32_t srow = (uint32_t)(kb * nb * 2048 + lane * 8);
        b4_u32x2 o0, o1, o2, o3;
        auto load_old = [&](int qb) __attribute__((always_inline)) {
          const uint32_t off = srow + 2048 * qb;
          o0 = b4_ld64(sld, off);
          o1 = b4_ld64(sld, off + 512);
          o2 = b4_ld64(sld, off + 1024);
          o3 = b4_ld64(sld, off + 1536);
        };
        // the next step's LDS operands (row constants, Q' / dO A fragments) are read during this step
        // (the row constants are read straight into the register order of the C input: no moves)
        f32x16 nlv, ndv;
        bf16x8 qa[2], da[2];
        auto load_rows = [&](int qb) __attribute__((always_inline)) {
          const float* pn = nl2 + qb * 32 + 4 * hh;
          const float* pd = ndl + qb * 32 + 4 * hh;
          const int qr0 = qb * 32;
          nlv.s0123 = *reinterpret_cast<const f32x4*>(pn);
          nlv.s4567 = *reinterpret_cast<const f32x4*>(pn + 8);
          nlv.s89ab = *reinterpret_cast<const f32x4*>(pn + 16);
          nlv.scdef = *reinterpret_cast<const f32x4*>(pn + 24);
          ndv.s0123 = *reinterpret_cast<const f32x4*>(pd);
          ndv.s4567 = *reinterpret_cast<const f32x4*>(pd + 8);
          ndv.s89ab = *reinterpret_cast<const f32x4*>(pd + 16);
          ndv.scdef = *reinterpret_cast<const f32x4*>(pd + 24);
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) {
            const int off = qr0 * HD + qoffA[kk];
            qa[kk] = *reinterpret_cast<const bf16x8*>(Qs + off);
            da[kk] = *reinterpret_cast<const bf16x8*>(dOs + off);
          }
        };
        // spread the waves' first query blocks; the offset is the round-robin wave of the unit, not the wave that runs
        // it, so the dK / dV summation order (and the result, bit for bit) does not depend on the unit plan
        int qb = __builtin_amdgcn_readfirstlane((kb + u % kB4Waves) % nb);
        load_old(qb);
        load_bias(qb);
        load_rows(qb);
        for (int i = 0; i < nb; ++i, qb = qb + 1 == nb ? 0 : qb + 1) {
          const int qr0 = qb * 32, qbn = qb + 1 == nb ? 0 : qb + 1;
          if (i == 0) asm volatile("s_waitcnt vmcnt(0)" : "+v"(bt0), "+v"(bt1));
          else asm volatile("s_waitcnt vmcnt(8)" : "+v"(bt0), "+v"(bt1));
          const bf16x8 bt[2] = {__builtin_bit_cast(bf16x8, bt0), __builtin_bit_cast(bf16x8, bt1)};
          // S = Q'K^T - L' (the row constants as the C input), then + bias'; dP = dO V^T - delta
          f32x16 s = mfma32(qa[0], kB[0], nlv), dp = mfma32(da[0], vB[0], ndv);
          s = mfma32(qa[1], kB[1], s);
          dp = mfma32(da[1], vB[1], dp);
          load_rows(qbn);
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const uint4 w4 = __builtin_bit_cast(uint4, bt[c]);
            const uint32_t w[4] = {w4.x, w4.y, w4.z, w4.w};
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
              s[8 * c + 2 * i2] += __uint_as_float(w[i2] << 16);
              s[8 * c + 2 * i2 + 1] += __uint_as_float(w[i2] & 0xffff0000u);
            }
          }
          load_bias(qbn);
          bf16x8 pa[2], sa[2];
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
              const float P = __builtin_amdgcn_exp2f(s[8 * c + j]);
              pa[c][j] = (__bf16)P;
              sa[c][j] = (__bf16)(P * dp[8 * c + j]);
            }
#pragma unroll
          for (int c = 0; c < 2; ++c) {
            const int rb = (qr0 + 16 * c) * HD;
            const bf16x8 doT = tr16x2(dOs + rb + tlo, dOs + rb + thi);
            const bf16x8 qT = tr16x2(Qs + rb + tlo, Qs + rb + thi);
            dVt = mfma32(doT, pa[c], dVt);
            dKt = mfma32(qT, sa[c], dKt);
          }
          {   // dS^T[k][q] (+ the slab's earlier sum): sa[c] elements 4 (v & 1) .. 4 (v & 1) + 3 are queries 8 v + 4 hh ..
            asm volatile("s_waitcnt vmcnt(2)" : "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
            const b4_u32x2 old[4] = {o0, o1, o2, o3};
            const uint32_t off = srow + 2048 * qb;
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const uint4 u4 = __builtin_bit_cast(uint4, sa[v >> 1]);
              const uint2 x = (v & 1) ? make_uint2(u4.z, u4.w) : make_uint2(u4.x, u4.y);
              const uint2 y = add_bf16x4(x, make_uint2(old[v].x, old[v].y));   // + 0 for the group's first window
              b4_st64(sst, off + 512 * v, b4_u32x2{y.x, y.y});
            }
            load_old(qbn);
          }
        }
        // the last step's prefetches land in these registers: drain them before the registers are reused
        asm volatile("s_waitcnt vmcnt(0)" : "+v"(bt0), "+v"(bt1), "+v"(o0), "+v"(o1), "+v"(o2), "+v"(o3));
        // dK = (sum dS Q') ln 2, dV: lane holds key r, e = 8 v + 4 hh + t
        const float kscale = 0.6931471805599453f;
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int e = hoff + 8 * v + 4 * hh;
          if (krow >= 0) {
            bf16raw* pk = reinterpret_cast<bf16raw*>(ba.dk) + (long)krow * ba.ld_dqkv + e;
            bf16raw* pv = reinterpret_cast<bf16raw*>(ba.dv) + (long)krow * ba.ld_dqkv + e;
            uint2 uk, uv;
            uk.x = (uint32_t)f2bf(dKt[4 * v] * kscale) | ((uint32_t)f2bf(dKt[4 * v + 1] * kscale) << 16);
            uk.y = (uint32_t)f2bf(dKt[4 * v + 2] * kscale) | ((uint32_t)f2bf(dKt[4 * v + 3] * kscale) << 16);
            uv.x = (uint32_t)f2bf(dVt[4 * v]) | ((uint32_t)f2bf(dVt[4 * v + 1]) << 16);
            uv.y = (uint32_t)f2bf(dVt[4 * v + 2]) | ((uint32_t)f2bf(dVt[4 * v + 3]) << 16);
            *reinterpret_cast<uint2*>(pk) = uk;
            *reinterpret_cast<uint2*>(pv) = uv;
          } else if (krow == -1) {
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              if (ba.dpad_k) atomicAdd(ba.dpad_k + e + t, dKt[4 * v + t] * kscale);
              if (ba.dpad_v) atomicAdd(ba.dpad_v + e + t, dVt[4 * v + t]);
            }
          }
        }
      } else {
        // ---------------- pass B: query block qb, queries on the lane (v6 forward layout: sub-tile t = 2 qh + kh,
        // lane (ql, g16) holds query 16 qh + ql, keys 16 kh + 4 g16 + 0..3)
        const int qb = __builtin_amdgcn_readfirstlane(u - nb);
        bf16x8 qf[2], df[2];
        float nlq[2];
        f32x4 ndq4[2];   // -delta splat: the dP^T products' C input (loop invariant, no per-step moves)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int q = qb * 32 + 16 * qh + ql;
          const int off = swz<HD>(q, 8 * g16);
          qf[qh] = *reinterpret_cast<const bf16x8*>(Qs + off);
          df[qh] = *reinterpret_cast<const bf16x8*>(dOs + off);
          nlq[qh] = nl2[q];
          const float nd = ndl[q];
          ndq4[qh] = f32x4{nd, nd, nd, nd};
        }
        f32x4 dq[2][2];
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int eh = 0; eh < 2; ++eh) dq[qh][eh] = f32x4{0.f, 0.f, 0.f, 0.f};
        uint4 bt[2];
        auto load_bias = [&](int kb) __attribute__((always_inline)) {
          const int so = __builtin_amdgcn_readfirstlane((qb * nb + kb) * 2048);
#pragma unroll
          for (int c = 0; c < 2; ++c)
            bt[c] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(trB, lane * 16, so + c * 1024, 0));
        };
        bf16x8 kf[2], vf[2], ka[2];   // the next key block's fragments are read during this step
        auto load_kv = [&](int kb) __attribute__((always_inline)) {
          const bf16raw* kbase = Ks + kb * 32 * HD;
          const bf16raw* vbase = Vs + kb * 32 * HD;
#pragma unroll
          for (int kh = 0; kh < 2; ++kh) {
            kf[kh] = *reinterpret_cast<const bf16x8*>(kbase + koffB[kh]);
            vf[kh] = *reinterpret_cast<const bf16x8*>(vbase + koffB[kh]);
          }
#pragma unroll
          for (int eh = 0; eh < 2; ++eh) ka[eh] = tr16x2(kbase + vlo[eh], kbase + vhi[eh]);
        };
        int kb = __builtin_amdgcn_readfirstlane((qb + u % kB4Waves) % nb);   // as pass A: independent of the plan
        load_bias(kb);
        load_kv(kb);
        for (int i = 0; i < nb; ++i, kb = kb + 1 == nb ? 0 : kb + 1) {
          const int kbn = kb + 1 == nb ? 0 : kb + 1;
          f32x4 d[4], e[4];
#pragma unroll
          for (int c = 0; c < 2; ++c) {   // c = qh: element j of word i <-> key 16 (j >> 2) + 4 g16 + (j & 3)
            const uint32_t w[4] = {bt[c].x, bt[c].y, bt[c].z, bt[c].w};
#pragma unroll
            for (int i2 = 0; i2 < 4; ++i2) {
              d[2 * c + (i2 >> 1)][2 * (i2 & 1)] = __uint_as_float(w[i2] << 16) + nlq[c];
              d[2 * c + (i2 >> 1)][2 * (i2 & 1) + 1] = __uint_as_float(w[i2] & 0xffff0000u) + nlq[c];
            }
            e[2 * c] = e[2 * c + 1] = ndq4[c];
          }
          load_bias(kbn);
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            d[t] = mfma16(kf[t & 1], qf[t >> 1], d[t]);
            e[t] = mfma16(vf[t & 1], df[t >> 1], e[t]);
          }
          const bf16x8 kac[2] = {ka[0], ka[1]};
          load_kv(kbn);
#pragma unroll
          for (int qh = 0; qh < 2; ++qh) {
            bf16x8 ds8;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              ds8[j] = (__bf16)(__builtin_amdgcn_exp2f(d[2 * qh][j]) * e[2 * qh][j]);
              ds8[4 + j] = (__bf16)(__builtin_amdgcn_exp2f(d[2 * qh + 1][j]) * e[2 * qh + 1][j]);
            }
#pragma unroll
            for (int eh = 0; eh < 2; ++eh) dq[qh][eh] = mfma16(kac[eh], ds8, dq[qh][eh]);
          }
        }
        // dQ = scale sum dS K: lane (ql, g16) of (qh, eh) holds query 16 qh + ql, e = 16 eh + 4 g16 + 0..3
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const int q = qb * 32 + 16 * qh + ql;
          const int row = q < g.N ? trow[q] : -2;
#pragma unroll
          for (int eh = 0; eh < 2; ++eh) {
            const int e = hoff + 16 * eh + 4 * g16;
            if (row >= 0) {
              uint2 w;
              w.x = (uint32_t)f2bf(dq[qh][eh][0] * a.scale) | ((uint32_t)f2bf(dq[qh][eh][1] * a.scale) << 16);
              w.y = (uint32_t)f2bf(dq[qh][eh][2] * a.scale) | ((uint32_t)f2bf(dq[qh][eh][3] * a.scale) << 16);
              *reinterpret_cast<uint2*>(reinterpret_cast<bf16raw*>(ba.dq) + (long)row * ba.ld_dqkv + e) = w;
            } else if (row == -1 && ba.dpad_q) {
#pragma unroll
              for (int t = 0; t < 4; ++t) atomicAdd(ba.dpad_q + e + t, dq[qh][eh][t] * a.scale);
            }
          }
        }
      }
    }
    __syncthreads();   // the next window of the group restages the LDS images
  }
}

size_t bwd4_lds(const Geo& g) { return (size_t)g.Np * (8 * 32 + 12); }

// the two-pass kernel's geometry (bf16 bias tables of the v6 forward layout, hd 32, no dropout); it alone groups
// windows into shared dRPB slabs (wattn_bwd3's read-modify-write of the slab, behind a branch, stalled each step)
extern int g_bwd_version;
bool bwd4_geometry(const dfk_wattn_args& a, const Geo& g) {
  return g_bwd_version == 4 && a.dtype == DFK_BF16 && !a.mask && a.scale > 0.f && a.tab && a.hd == 32 &&
         !a.drop.mode && fwd16_layout(a, g) && bwd4_lds(g) <= 160 * 1024 && 2 * (g.Np / 32) <= 48;   // B4Sched
}

size_t bwd3_lds(const dfk_wattn_args& a, const Geo& g, int Qn, int nw, bool cos = false) {
  return 8 * (size_t)Qn * a.hd + 2 * (size_t)nw * 32 * kSdRow + 4 * (size_t)g.Np + 8 * (size_t)Qn +
         (cos ? 8 * (size_t)Qn + 64 : 0);
}

// dRPB from the dS^T scratch: drpb[pos(q) - pos(k) + C0] += sum over windows of dS[q][k].
// Block (chunk, head, split): 8 consecutive (k, q) elements per thread summed over the split's windows,
// scattered into an LDS table (once per element per block), table -> one workspace row.
// tiled = 0: a slab is dS^T [k][q] (wattn_bwd3); 1: 32 x 32 tiles (kb nb + qb) of 2 KB in the register order of
// wattn_bwd4's dK/dV pass, [v][lane][t] with key 32 kb + (lane & 31), query 32 qb + 8 v + 4 (lane >> 5) + t (each
// store instruction of that pass writes 512 contiguous bytes)
__global__ __launch_bounds__(256) void drpb_from_ds_kernel(const bf16raw* __restrict__ ds, long units, int heads,
                                                           int Np, int N, int fh, int fw, int C0, int L, int wps,
                                                           float* __restrict__ rows, int tiled) {
  extern __shared__ float tab[];
  const int chunk = dfk_bid_x(), h = dfk_bid_y(), split = dfk_bid_z();
  const int Lal = (L + 3) & ~3;
  for (int l = dfk_tid(); l < L; l += dfk_bdim()) tab[l] = 0.f;
  __syncthreads();
  const long e0 = ((long)chunk * dfk_bdim() + dfk_tid()) * 8;
  const long NN = (long)Np * Np;
  if (e0 < NN) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const long nwin = units / heads;
    const long w0 = (long)split * wps, w1 = min(nwin, w0 + wps);
    const bf16raw* src = ds + (w0 * heads + h) * NN + e0;
    const long wstride = (long)heads * NN;
    long w = w0;
#ifndef DFK_DRPB_IF
#define DFK_DRPB_IF 8
#endif
    constexpr int IF = DFK_DRPB_IF;   // independent 16-B loads in flight per thread
    for (; w + IF <= w1; w += IF, src += IF * wstride) {
      uint4 v[IF];
#pragma unroll
      for (int u = 0; u < IF; ++u) {
#ifndef DFK_DRPB_TEMPORAL   // streamed once: non-temporal (r5z: stage-1 backward with dRPB 934 -> 892 us, stage 3 250 -> 207)
        typedef unsigned int u32x4n __attribute__((ext_vector_type(4)));
        v[u] = __builtin_bit_cast(uint4, __builtin_nontemporal_load(reinterpret_cast<const u32x4n*>(src + u * wstride)));
#else
        v[u] = *reinterpret_cast<const uint4*>(src + u * wstride);
#endif
      }
#pragma unroll
      for (int u = 0; u < IF; ++u) {
        const bf16raw* pe = reinterpret_cast<const bf16raw*>(&v[u]);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(pe[j]);
      }
    }
    for (; w < w1; ++w, src += wstride) {
      const uint4 v = *reinterpret_cast<const uint4*>(src);
      const bf16raw* pe = reinterpret_cast<const bf16raw*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(pe[j]);
    }
    auto pos = [&](int i) { return ((i / (fh * fw)) * (2 * fh - 1) + (i / fw) % fh) * (2 * fw - 1) + i % fw; };
    if (!tiled) {
      const int k = (int)(e0 / Np), qb = (int)(e0 % Np);
      if (k < N) {
        const int pk = pos(k);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          if (qb + j < N) atomicAdd(tab + pos(qb + j) - pk + C0, acc[j]);
      }
    } else {
      const int nb = Np / 32, tile = (int)(e0 >> 10), w = (int)(e0 & 1023);
      const int kb = tile / nb, qb = tile % nb, v = w >> 8, l0 = (w & 255) >> 2;
#pragma unroll
      for (int hl = 0; hl < 2; ++hl) {
        const int ln = l0 + hl, k = kb * 32 + (ln & 31), q0 = qb * 32 + 8 * v + 4 * (ln >> 5);
        if (k < N) {
          const int pk = pos(k);
#pragma unroll
          for (int t = 0; t < 4; ++t)
            if (q0 + t < N) atomicAdd(tab + pos(q0 + t) - pk + C0, acc[4 * hl + t]);
        }
      }
    }
  }
  __syncthreads();
  float* row = rows + ((long)(split * dfk_gdim_x() + chunk) * heads + h) * Lal;
  for (int l = dfk_tid(); l < L; l += dfk_bdim()) row[l] = tab[l];
}

struct DsPlan {
  long ds_elems;   // bf16 dS^T scratch elements
  int nchunks, nsplit, wps;
  long rows;       // workspace rows of L floats
};

// windows per backward work group (wattn_bwd3_kernel, decode_group): enough groups left for ~3 rounds of one
// workgroup per CU (768), at most 8 (DFK_DRPB_G: A/B runs only)
int g_bwd_group = getenv("DFK_DRPB_G") ? atoi(getenv("DFK_DRPB_G")) : 0;   // dfk_wattn_bwd_policy
int g_bwd_version = getenv("DFK_WATTN_BWD") ? atoi(getenv("DFK_WATTN_BWD")) : 4;
// bwd4's unit assignment (B4Sched): the smallest makespan over the waves for unit costs cA (a pass-A key block) and
// cB (a pass-B query block) — units of one pass are interchangeable, so a plan is a count (a_w, b_w) per wave, found by
// a DP per candidate makespan (DFK_B4_SCHED=0: round robin; DFK_B4_COST="cA,cB", default 4,3 products per step)
B4Sched b4_sched(int nb) {
  static const int mode = getenv("DFK_B4_SCHED") ? atoi(getenv("DFK_B4_SCHED")) : 1;   // A/B runs only
  static int cA = 4, cB = 3;
  static const bool parsed = [] {
    if (const char* e = getenv("DFK_B4_COST")) {
      int x = 0, y = 0;
      if (sscanf(e, "%d,%d", &x, &y) == 2 && x > 0 && y > 0) { cA = x; cB = y; }
    }
    return true;
  }();
  (void)parsed;
  constexpr int W = kB4Waves;
  int na[W] = {}, nbw[W] = {};
  if (mode == 0) {
    for (int u = 0; u < 2 * nb; ++u) (u < nb ? na : nbw)[u % W] += 1;
  } else {
    // smallest T such that W waves hold nb A units and nb B units with cA a_w + cB b_w <= T
    for (int T = ((nb * (cA + cB)) + W - 1) / W;; ++T) {
      int cap[W + 1][64];   // cap[w][a] = max B units the first w waves hold with a A units among them (-1: none)
      for (int w = 0; w <= W; ++w)
        for (int a = 0; a <= nb; ++a) cap[w][a] = -1;
      cap[0][0] = 0;
      for (int w = 0; w < W; ++w)
        for (int a = 0; a <= nb; ++a) {
          if (cap[w][a] < 0) continue;
          for (int x = 0; a + x <= nb && cA * x <= T; ++x)
            cap[w + 1][a + x] = std::max(cap[w + 1][a + x], cap[w][a] + (T - cA * x) / cB);
        }
      if (cap[W][nb] < nb) continue;
      // walk back: choose a_w per wave (any choice that keeps the rest feasible), b_w greedily
      int a = nb, b = nb;
      for (int w = W - 1; w >= 0; --w) {
        for (int x = 0; x <= a && cA * x <= T; ++x) {
          const int prev = cap[w][a - x];
          if (prev < 0) continue;
          const int take = std::min(b, (T - cA * x) / cB);
          if (prev >= b - take) { na[w] = x; nbw[w] = take; a -= x; b -= take; break; }
        }
      }
      break;
    }
  }
  B4Sched sc{};
  uint8_t* by = reinterpret_cast<uint8_t*>(sc.w);
  int pos = 0, ua = 0, ub = nb;
  for (int w = 0; w < W; ++w) {
    by[w] = (uint8_t)pos;
    for (int i = 0; i < na[w]; ++i) by[16 + pos++] = (uint8_t)ua++;
    for (int i = 0; i < nbw[w]; ++i) by[16 + pos++] = (uint8_t)ub++;
  }
  by[W] = (uint8_t)pos;
  return sc;
}

int bwd3_group(const dfk_wattn_args& a, const Geo& g) {
  if (g_bwd_group > 0) return g_bwd_group;
  // Step-level sweep (round 6, full training step, same box): G=8 280.0 clips/s, G=6 275.2, G=12 274.2,
  // G=16 268.8, G=32 233.8, old auto rule (units/768, 4/2/1 per stage) 271.4. Fewer, longer
  // workgroups overlap better with the branch streams than the isolated kernel time suggests.
  static const long minwg = getenv("DFK_DRPB_GMINWG") ? atol(getenv("DFK_DRPB_GMINWG")) : 64;   // A/B runs only
  static const long gmax = getenv("DFK_DRPB_GMAX") ? atol(getenv("DFK_DRPB_GMAX")) : 8;         // A/B runs only
  const long units = (long)a.B * g.nW * a.heads;
  return (int)std::max<long>(1, std::min<long>(gmax, units / std::max<long>(1, minwg)));
}

// dS^T slabs per head (window groups over the shift classes, as decode_group counts them)
long bwd3_slab_windows(const dfk_wattn_args& a, const Geo& g, int G) {
  const int ncls = g.use_mask ? 8 : 1;
  long tot = 0;
  for (int c = 0; c < ncls; ++c) {
    const long nd = g.use_mask ? ((c & 4) ? (a.sd > 0) : g.nwd - (a.sd > 0)) : g.nwd;
    const long nh = g.use_mask ? ((c & 2) ? (a.sh > 0) : g.nwh - (a.sh > 0)) : g.nwh;
    const long nw = g.use_mask ? ((c & 1) ? (a.sw > 0) : g.nww - (a.sw > 0)) : g.nww;
    tot += dfk_cdiv(nd * nh * nw * a.B, (long)G);
  }
  return tot;
}

DsPlan ds_plan(const dfk_wattn_args& a, const Geo& g, long nwin) {
  DsPlan pl;
  const long units = nwin * a.heads;   // slabs (a window group's summed dS^T, or one window's)
  pl.ds_elems = units * g.Np * g.Np;
  pl.nchunks = (int)dfk_cdiv((long)g.Np * g.Np, 256 * 8);
  // about 1.5k workgroups over the chip, each summing wps windows (fewer, longer sums: fewer partial rows)
  const long want = std::max<long>(1, std::min<long>(nwin, 1536 / std::max(1, pl.nchunks * a.heads)));
  pl.wps = (int)dfk_cdiv(nwin, want);
  pl.nsplit = (int)dfk_cdiv(nwin, pl.wps);
  pl.rows = (long)pl.nsplit * pl.nchunks * a.heads;
  return pl;
}

size_t bwd_lds_bf16(const dfk_wattn_args& a, const Geo& g, int Qn, int nwaves) {
  const size_t Lal = (g.L + 3) & ~3;
  return 8 * (size_t)g.Np + 4 * Lal + 8 * (size_t)Qn + (size_t)nwaves * 32 * (a.hd + 4) * 4 + 4 * (size_t)Qn * a.hd +
         (size_t)nwaves * 32 * kSdStride * 2;
}

// LDS bytes for a query chunk of Qn rows
size_t bwd_lds(const dfk_wattn_args& a, const Geo& g, int Qn) {
  const size_t es = a.dtype == DFK_BF16 ? 2 : 4;
  const size_t Lal = (g.L + 3) & ~3;
  return sizeof(TokInfo) * g.Np + 8 * Lal + 8 * (size_t)Qn + 4 * (size_t)Qn * a.hd + 2 * es * (size_t)Qn * a.hd +
         es * 4 * 32 * 32;
}

void reduce_drpb(const dfk_wattn_bwd_args& ba, const Geo& g, long units, hipStream_t s) {
  if (!ba.f.rpb || !ba.drpb || !ba.ws) return;
  hipLaunchKernelGGL(drpb_reduce_kernel, dim3(dfk_cdiv(g.L, 64), ba.f.heads), dim3(1024), 0, s, ba.ws, units,
                     ba.f.heads, g.L, ba.drpb);
}

}  // namespace

extern "C" int dfk_wattn_bwd(const dfk_wattn_bwd_args* bp, hipStream_t s) {
  if (!bp || !args_ok(bp->f) || !bp->f.lse || !bp->dout || !bp->dq || !bp->dk || !bp->dv) return DFK_EINVAL;
  const dfk_wattn_args& a = bp->f;
  const int vec = a.dtype == DFK_BF16 ? 8 : 4;
  if (bp->ld_dqkv % vec || bp->ld_dout % vec) return DFK_EINVAL;
  const Geo g = make_geo(a);
  if (a.dtype == DFK_BF16 && !a.mask && a.scale > 0.f && (a.tab || (!a.rpb && !g.use_mask))) {
    // v3 (the forward's bias tiles, bwd layout)
    const long units = (long)a.B * g.nW * a.heads;
    if (units <= 0) return 0;
    const bool tab = a.rpb || g.use_mask;
    const bf16raw* tb = tab ? tab3_fwd(a, g) + tab_elems(a, g) : nullptr;
    const int nkb = g.Np / 32;
    int nw = dfk_cdiv(nkb, dfk_cdiv(nkb, 8));   // passes of at most 8 waves, balanced
    const bool cos = bp->dscore != nullptr;
    if (cos && (!tab || a.drop.mode)) return DFK_EINVAL;   // dscore: the bias-table path without dropout only
    if (cos) nw = std::min(nw, 4);   // its instantiation is bounded to 256 threads (the row sums' registers)
    int Qn = g.Np;                               // largest query chunk whose Q / dO / dQ fit the LDS ...
    while (Qn > 32 && bwd3_lds(a, g, Qn, nw, cos) > 160 * 1024) Qn -= 32;
    const int nch = dfk_cdiv(g.Np, Qn);          // ... then balanced chunks
    Qn = 32 * dfk_cdiv(g.Np / 32, nch);
    nw = std::min(nw, g.Np / 32 - (nch - 1) * (Qn / 32));   // the staggered sweep needs a distinct block per wave
    const size_t lds = bwd3_lds(a, g, Qn, nw, cos);
    if (lds > 160 * 1024) return DFK_EINVAL;
    const bool want_drpb = a.rpb && bp->drpb;
    if (want_drpb && !bp->ws) return DFK_EINVAL;
    bf16raw* dsg = want_drpb ? reinterpret_cast<bf16raw*>(bp->ws) : nullptr;
    const bool v4 = tab && bwd4_geometry(a, g);
    if (v4 && cos) return DFK_EINVAL;   // dscore: the single-pass kernel (SwinV2's 49-token windows) only
    const int G = v4 ? bwd3_group(a, g) : 1;
    const long slabw = bwd3_slab_windows(a, g, G);
    if (v4) {   // the two-pass kernel (the v6 windows)
      static bool attr4 = false;
      if (!attr4) {
        (void)hipFuncSetAttribute((const void*)wattn_bwd4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr4 = true;
      }
      hipLaunchKernelGGL(wattn_bwd4_kernel, dim3((unsigned)(slabw * a.heads)), dim3(64 * kB4Waves), bwd4_lds(g), s,
                         *bp, g, dsg, tab3_fwd(a, g), tb, G, b4_sched(g.Np / 32));
    }
#define LAUNCH_B3(HD, TB, DR, CS)                                                                          \
  do {                                                                                                     \
    auto kfn = wattn_bwd3_kernel<HD, TB, DR, CS>;                                                            \
    static bool attr_set = false;                                                                          \
    if (!attr_set) {                                                                                       \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr_set = true;                                                                                     \
    }                                                                                                      \
    for (int q0 = 0; q0 < g.Np; q0 += Qn)                                                                  \
      hipLaunchKernelGGL(kfn, dim3((unsigned)(slabw * a.heads)), dim3(64 * nw), lds, s, *bp, g, q0,        \
                         std::min(Qn, g.Np - q0), q0 > 0 ? 1 : 0, dsg, tb, G);                             \
  } while (0)
#define PICK_B3(HD)                                                                            \
  do {                                                                                         \
    if (cos) LAUNCH_B3(HD, true, false, true);                                                 \
    else if (tab) { if (a.drop.mode) LAUNCH_B3(HD, true, true, false); else LAUNCH_B3(HD, true, false, false); } \
    else { if (a.drop.mode) LAUNCH_B3(HD, false, true, false); else LAUNCH_B3(HD, false, false, false); }        \
  } while (0)
    if (!v4) {
      if (a.hd == 32) PICK_B3(32); else PICK_B3(64);
    }
#undef PICK_B3
#undef LAUNCH_B3
    if (want_drpb) {
      const DsPlan pl = ds_plan(a, g, slabw);
      float* rows = reinterpret_cast<float*>(reinterpret_cast<char*>(bp->ws) + ((pl.ds_elems * 2 + 15) & ~15L));
      hipLaunchKernelGGL(drpb_from_ds_kernel, dim3(pl.nchunks, a.heads, pl.nsplit), dim3(256),
                         ((g.L + 3) & ~3) * 4, s, dsg, slabw * a.heads, a.heads, g.Np, g.N, a.fh, a.fw, g.C0, g.L,
                         pl.wps, rows, v4 ? 1 : 0);
      hipLaunchKernelGGL(drpb_reduce_kernel, dim3(dfk_cdiv(g.L, 64), a.heads), dim3(1024), 0, s, rows, pl.rows,
                         a.heads, g.L, bp->drpb);
    }
    DFK_CHECK_LAUNCH();
    return 0;
  }
  if (bp->dscore) return DFK_EINVAL;   // the score-multiplier gradient: v3 (bias tables, bf16) only
  if (a.dtype == DFK_BF16) {
    const int nwaves = std::min(a.hd == 32 ? kBwdWaves : kBwdWaves / 2, g.Np / 32);  // hd 64: 4 waves, 512 VGPRs
    int Qn = g.Np;
    while (Qn > 32 && bwd_lds_bf16(a, g, Qn, nwaves) > 160 * 1024) Qn -= 32;
    const size_t lds = bwd_lds_bf16(a, g, Qn, nwaves);
    if (lds > 160 * 1024) return DFK_EINVAL;
    const long units = (long)a.B * g.nW * a.heads;
    if (units <= 0) return 0;
#define LAUNCH_B16(HD, RPB, MASK)                                                                          \
  do {                                                                                                     \
    auto kfn = wattn_bwd_bf16_kernel<HD, RPB, MASK>;                                                       \
    static bool attr_set = false;                                                                          \
    if (!attr_set) {                                                                                       \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr_set = true;                                                                                     \
    }                                                                                                      \
    for (int q0 = 0; q0 < g.Np; q0 += Qn)                                                                  \
      hipLaunchKernelGGL(kfn, dim3((unsigned)units), dim3(64 * nwaves), lds, s, *bp, g, q0,                \
                         std::min(Qn, g.Np - q0), q0 > 0 ? 1 : 0, dsg);                                    \
  } while (0)
#define PICK_B16(HD)                                                 \
  do {                                                               \
    if (a.rpb) { if (a.mask) LAUNCH_B16(HD, true, true); else LAUNCH_B16(HD, true, false); } \
    else { if (a.mask) LAUNCH_B16(HD, false, true); else LAUNCH_B16(HD, false, false); }     \
  } while (0)
    const bool want_drpb = a.rpb && bp->drpb;
    if (want_drpb && !bp->ws) return DFK_EINVAL;  // dRPB needs the dfk_wattn_bwd_workspace scratch
    const DsPlan pl = ds_plan(a, g, units / a.heads);
    bf16raw* dsg = want_drpb ? reinterpret_cast<bf16raw*>(bp->ws) : nullptr;
    if (a.drop.mode) return DFK_EINVAL;   // attention dropout: v3 kernels only (as the forward)
    if (a.hd == 32) PICK_B16(32); else PICK_B16(64);
#undef PICK_B16
#undef LAUNCH_B16
    if (want_drpb) {
      float* rows = reinterpret_cast<float*>(reinterpret_cast<char*>(bp->ws) + ((pl.ds_elems * 2 + 15) & ~15L));
      hipLaunchKernelGGL(drpb_from_ds_kernel, dim3(pl.nchunks, a.heads, pl.nsplit), dim3(256),
                         ((g.L + 3) & ~3) * 4, s, dsg, units, a.heads, g.Np, g.N, a.fh, a.fw, g.C0, g.L, pl.wps,
                         rows, 0);
      hipLaunchKernelGGL(drpb_reduce_kernel, dim3(dfk_cdiv(g.L, 64), a.heads), dim3(1024), 0, s, rows, pl.rows,
                         a.heads, g.L, bp->drpb);
    }
    DFK_CHECK_LAUNCH();
    return 0;
  }
  // fp32 (parity mode): largest query chunk (multiple of 32) that fits the 160 KiB LDS
  if (a.drop.mode) return DFK_EINVAL;
  int Qn = g.Np;
  while (Qn > 32 && bwd_lds(a, g, Qn) > 160 * 1024) Qn -= 32;
  const size_t lds = bwd_lds(a, g, Qn);
  if (lds > 160 * 1024) return DFK_EINVAL;
  const long units = (long)a.B * g.nW * a.heads;
  if (units <= 0) return 0;
  dim3 grid((unsigned)units);
#define LAUNCH_B(T, HD)                                                                                 \
  do {                                                                                                  \
    auto kfn = wattn_bwd_kernel<T, HD>;                                                                 \
    static bool attr_set = false;  /* once per kernel: the 160 KiB LDS limit (never inside a capture) */ \
    if (!attr_set) {                                                                                    \
      (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024); \
      attr_set = true;                                                                                  \
    }                                                                                                   \
    for (int q0 = 0; q0 < g.Np; q0 += Qn)                                                               \
      hipLaunchKernelGGL(kfn, grid, dim3(256), lds, s, *bp, g, q0, std::min(Qn, g.Np - q0), q0 > 0 ? 1 : 0); \
  } while (0)
  if (a.hd == 32) LAUNCH_B(float, 32); else LAUNCH_B(float, 64);
#undef LAUNCH_B
  reduce_drpb(*bp, g, units, s);
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int64_t dfk_wattn_table_workspace(const dfk_wattn_args* f) {
  if (!f || !args_ok(*f)) return -1;
  if (f->dtype != DFK_BF16 || f->mask) return 0;
  const Geo g = make_geo(*f);
  if (!f->rpb && !g.use_mask) return 0;   // no bias at all (wav2vec2): the kernels mask the padded keys themselves
  return tab3_bytes(*f, g);   // bf16 fwd + bwd layouts
}

extern "C" int64_t dfk_wattn_bwd_workspace(const dfk_wattn_args* f) {
  if (!f || !args_ok(*f)) return -1;
  if (!f->rpb) return 0;
  const Geo g = make_geo(*f);
  const int64_t Lal = (g.L + 3) & ~3;
  if (f->dtype == DFK_BF16) {  // dS^T scratch (bf16) + per-block dRPB rows
    const bool v4 = bwd4_geometry(*f, g);   // dfk_wattn_bwd's two-pass path: grouped slabs
    const DsPlan pl = ds_plan(*f, g, v4 ? bwd3_slab_windows(*f, g, bwd3_group(*f, g)) : (long)f->B * g.nW);
    return ((pl.ds_elems * 2 + 15) & ~15L) + pl.rows * Lal * 4;
  }
  return (int64_t)f->B * g.nW * f->heads * Lal * 4;  // fp32: one dRPB row per window-head
}

extern "C" int dfk_wattn_bwd_policy(int32_t group, int32_t version) {
  if (group < 0 || group > 64 || (version != -1 && version != 3 && version != 4)) return DFK_EINVAL;
  g_bwd_group = group;
  if (version > 0) g_bwd_version = version;
  return 0;
}
