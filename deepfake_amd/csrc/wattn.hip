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
};

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

template <typename T> struct LdsLayout;

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

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int unit = blockIdx.x;
  const int head = unit % a.heads;
  unit /= a.heads;
  const int win = unit % g.nW, b = unit / g.nW;

  for (int i = tid; i < g.Np; i += 256) tok[i] = token_info(a, g, b, win, i);
  if (a.rpb)
    for (int l = tid; l < g.L; l += 256) rpb[l] = a.rpb[(long)l * a.heads + head];
  __syncthreads();
  // K, V of the window -> LDS
  const int hoff = head * HD;
  for (int idx = tid; idx < g.Np * (HD / VEC); idx += 256) {
    const int i = idx / (HD / VEC), c = (idx % (HD / VEC)) * VEC;
    const TokInfo t = tok[i];
    const uint4 kv = ld16<T>(tok_ptr<T>(a.k, a.pad_k, t.row, a.ld_qkv, hoff + c));
    const uint4 vv = ld16<T>(tok_ptr<T>(a.v, a.pad_v, t.row, a.ld_qkv, hoff + c));
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
  for (int qt = blockIdx.y * 4 + wave; qt < nqt; qt += 4 * qsplit) {
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
        uint4 u = qp ? *reinterpret_cast<const uint4*>(qp + es * 32 + grp * 8) : make_uint4(0, 0, 0, 0);
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
    if (a.lse && grp == 0 && q < g.N) a.lse[((long)blockIdx.x) * g.Np + q] = m + __logf(l);
  }
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
  return g;
}

bool args_ok(const dfk_wattn_args& a) {
  if (!a.q || !a.k || !a.v || !a.out) return false;
  if (a.hd != 32 && a.hd != 64) return false;
  if (a.wd <= 0 || a.wh <= 0 || a.ww <= 0 || a.wd > a.fd || a.wh > a.fh || a.ww > a.fw) return false;
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

extern "C" int dfk_wattn_fwd(const dfk_wattn_args* ap, hipStream_t s) {
  if (!ap || !args_ok(*ap)) return DFK_EINVAL;
  const dfk_wattn_args& a = *ap;
  const Geo g = make_geo(a);
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
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds); \
    hipLaunchKernelGGL(kfn, grid, dim3(256), lds, s, a, g, qsplit);                                     \
  } while (0)
  if (a.dtype == DFK_BF16) {
    if (a.hd == 32) LAUNCH_F(bf16raw, 32); else LAUNCH_F(bf16raw, 64);
  } else {
    if (a.hd == 32) LAUNCH_F(float, 32); else LAUNCH_F(float, 64);
  }
#undef LAUNCH_F
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_wattn_bwd(const dfk_wattn_bwd_args* ap, hipStream_t s) {
  (void)ap; (void)s;
  return DFK_EINVAL;  // TODO(round1): backward kernel
}
