// Fused PatchEmbed3D (video_swin_transformer.py:420-460): pad + Conv3d(3 -> C, kernel = stride = 2x4x4)
// + LayerNorm(C), bf16 compute, in ONE pass over the clip:
//
//   forward : the fp32 clip is read once (coalesced 16-B loads into an LDS slab per token row), the
//             K = 96 patch projection runs on MFMA against the weight held in LDS, bias + LayerNorm are
//             applied in registers and the normalised bf16 tokens are written once (+ 8 B of LN
//             statistics per token).  Algorithmic bytes per clip at C2: 19.27 MB read + 9.63 MB written
//             (+0.4 MB stats); the three-pass path (im2col -> GEMM -> LN) moved ~2.3x that.
//   backward: per token row the conv output is recomputed from the clip (no patch matrix is ever
//             stored), the LayerNorm backward gives dconv in registers, and dW = dconv^T . patches,
//             db, dgamma, dbeta accumulate in registers across the token rows of a persistent
//             workgroup — one fp32 atomic per weight per workgroup at the end.  The clip needs no
//             gradient (it is data).
//
// Geometry fixed by the Swin-T/B video stem: Cin = 3, patch (2, 4, 4) -> K = 96 (three 32-deep MFMA
// k-chunks), C = NB * 16 output channels (96 Swin-T, 128 Swin-B).  Token row = the Wo tokens of one
// (clip, d, h): its 3 x 2 x 4 = 24 input rows of Wo*4 floats are staged once; zero beyond T/H/W (= F.pad).
#include <algorithm>

#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int PK = 96, PKS = PK + 8;   // patch length, LDS row stride of the weight (bf16)
constexpr int SROWS = 24;              // staged input rows per token row (cin * pd * ph)
constexpr int NT = 256, MAXT = 64;     // 4 waves x 16 tokens: token rows of up to 64 tokens

struct PeGeo {
  int Do, Ho, Wo, Ws;                  // Ws: slab row stride (floats)
  int xbytes;                          // bytes of the clip batch (buffer-descriptor range)
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// register-staged slab: each thread's share of the token row's 24 input rows (float4 chunks), so the next
// row's loads are in flight while the current row computes (persistent forward)
constexpr int SLAB_REGS = 6;   // ceil(24 rows * 64 chunks / 256 threads)

__device__ __forceinline__ void slab_load(const dfk_patch_embed_args& a, const PeGeo& g, long r,
                                          float4 (&v)[SLAB_REGS]) {
  const int h = (int)(r % g.Ho);
  const long r2 = r / g.Ho;
  const int d = (int)(r2 % g.Do);
  const long b = r2 / g.Do;
  const int q4 = g.Wo;
  // branch-free (W % 4 == 0, pe_geo): buffer loads through a descriptor of the whole clip batch; a chunk
  // past T / H (F.pad) or past the row's 24 x Wo chunks gets an out-of-range offset and reads as zero, so
  // all SLAB_REGS loads are in flight together (a branch around a load makes hipcc wait for it there)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), (short)0, g.xbytes,
                                                                      0x00020000);
#pragma unroll
  for (int j = 0; j < SLAB_REGS; ++j) {
    const int i = threadIdx.x + j * NT;
    const int sr = i / q4, x0 = (i - sr * q4) * 4;
    const int c = sr / 8, kd = (sr / 4) % 2, kh = sr % 4;
    const int t = d * 2 + kd, y = h * 4 + kh;
    const bool ok = i < SROWS * q4 && t < a.T && y < a.H;
    const long e = b * a.sb + c * a.sc + (long)t * a.st + (long)y * a.sh + x0;
    const uint32_t off = ok ? (uint32_t)(e * 4) : 0xfffffff0u;
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
    v[j] = make_float4(__uint_as_float(u[0]), __uint_as_float(u[1]), __uint_as_float(u[2]), __uint_as_float(u[3]));
  }
}

__device__ __forceinline__ void slab_store(const PeGeo& g, const float4 (&v)[SLAB_REGS], float* slab) {
  const int q4 = g.Wo;
#pragma unroll
  for (int j = 0; j < SLAB_REGS; ++j) {
    const int i = threadIdx.x + j * NT;
    if (i < SROWS * q4) {
      const int sr = i / q4, x0 = (i - sr * q4) * 4;
      *reinterpret_cast<float4*>(slab + sr * g.Ws + x0) = v[j];
    }
  }
}

__device__ __forceinline__ void stage_slab(const dfk_patch_embed_args& a, const PeGeo& g, long r, float* slab) {
  const int h = (int)(r % g.Ho);
  const long r2 = r / g.Ho;
  const int d = (int)(r2 % g.Do);
  const long b = r2 / g.Do;
  const int q4 = g.Wo;                  // 16-B chunks per staged row (Wo tokens x 4 columns)
  const float* x = reinterpret_cast<const float*>(a.x);
  for (int i = threadIdx.x; i < SROWS * q4; i += NT) {
    const int sr = i / q4, x0 = (i - sr * q4) * 4;
    const int c = sr / 8, kd = (sr / 4) % 2, kh = sr % 4;
    const int t = d * 2 + kd, y = h * 4 + kh;
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
    *reinterpret_cast<float4*>(slab + sr * g.Ws + x0) = v;
  }
}

// patch columns k0..k0+7 of token w (k = ((c*2 + kd)*4 + kh)*4 + kw): two staged rows x 4 columns
__device__ __forceinline__ bf16x8 patch_frag(const float* slab, int Ws, int w, int k0) {
  const int sr = k0 >> 2;
  const float4 lo = *reinterpret_cast<const float4*>(slab + sr * Ws + w * 4);
  const float4 hi = *reinterpret_cast<const float4*>(slab + (sr + 1) * Ws + w * 4);
  bf16x8 f;
  f[0] = (__bf16)lo.x; f[1] = (__bf16)lo.y; f[2] = (__bf16)lo.z; f[3] = (__bf16)lo.w;
  f[4] = (__bf16)hi.x; f[5] = (__bf16)hi.y; f[6] = (__bf16)hi.z; f[7] = (__bf16)hi.w;
  return f;
}

template <int NB>
__device__ __forceinline__ void load_weight(const dfk_patch_embed_args& a, bf16raw* w_lds) {
  const bf16raw* W = reinterpret_cast<const bf16raw*>(a.w);
  for (int idx = threadIdx.x; idx < NB * 16 * (PK / 8); idx += NT) {
    const int j = idx / (PK / 8), kc = (idx % (PK / 8)) * 8;
    *reinterpret_cast<uint4*>(w_lds + j * PKS + kc) = *reinterpret_cast<const uint4*>(W + (long)j * PK + kc);
  }
}

// conv output of this lane's token / channels: acc[nb][r] = channel nb*16 + 4*(lane>>4) + r of token w
template <int NB>
__device__ __forceinline__ void conv_tokens(const float* slab, int Ws, const bf16raw* w_lds, int w, f32x4 (&acc)[NB]) {
  const int lane = threadIdx.x & 63, mrow = lane & 15, kq = (lane >> 4) * 8;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < PK / 32; ++kc) {
    const bf16x8 af = patch_frag(slab, Ws, w, kc * 32 + kq);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const bf16x8 wf = *reinterpret_cast<const bf16x8*>(w_lds + (nb * 16 + mrow) * PKS + kc * 32 + kq);
      acc[nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, af, acc[nb], 0, 0, 0);
    }
  }
}

// sum over the four lane groups (lanes l, l^16, l^32, l^48 hold the other channels of the same token)
__device__ __forceinline__ float group_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}

// bias / LN gamma / LN beta of this lane's channels nb*16 + 4*(lane>>4) + r, loaded once per workgroup
// (per-row global loads would make every row wait for the next row's clip prefetch: vmcnt is in order)
template <int NB>
struct PeParams {
  float b[NB][4], g[NB][4], t[NB][4];
};

template <int NB>
__device__ __forceinline__ PeParams<NB> load_params(const dfk_patch_embed_args& a) {
  PeParams<NB> P;
  const int nq = ((threadIdx.x & 63) >> 4) * 4;
  const bf16raw* bias = reinterpret_cast<const bf16raw*>(a.b);
  const bf16raw* gam = reinterpret_cast<const bf16raw*>(a.ln_w);
  const bf16raw* bet = reinterpret_cast<const bf16raw*>(a.ln_b);
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      P.b[nb][r] = bf2f(bias[nb * 16 + nq + r]);
      P.g[nb][r] = bf2f(gam[nb * 16 + nq + r]);
      P.t[nb][r] = bf2f(bet[nb * 16 + nq + r]);
    }
  return P;
}

template <int NB>
__device__ __forceinline__ void pe_fwd_row(const dfk_patch_embed_args& a, const PeGeo& g, long row, const float* slab,
                                           const bf16raw* w_lds, bf16raw* stg_all, const PeParams<NB>& P) {
  constexpr int C = NB * 16, SS = C + 8;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mrow = lane & 15, nq = (lane >> 4) * 4;
  const int w = wave * 16 + mrow;                  // token within the row
  if (wave * 16 >= g.Wo) return;                   // idle wave: no barrier inside this function
  f32x4 acc[NB];
  conv_tokens<NB>(slab, g.Ws, w_lds, w < g.Wo ? w : 0, acc);
  float s = 0.f;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc[nb][r] += P.b[nb][r];
      s += acc[nb][r];
    }
  const float mean = group_sum(s) * (1.f / C);
  float q = 0.f;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float dlt = acc[nb][r] - mean;
      q += dlt * dlt;
    }
  const float rstd = rsqrtf(group_sum(q) * (1.f / C) + a.eps);
  const long tok0 = row * g.Wo;                    // first token of this row
  bf16raw* stg = stg_all + wave * 16 * SS;
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int n = nb * 16 + nq;
    float v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = (acc[nb][r] - mean) * rstd * P.g[nb][r] + P.t[nb][r];
    uint2 o;
    o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
    o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
    *reinterpret_cast<uint2*>(stg + mrow * SS + n) = o;
  }
  if (lane < 16 && w < g.Wo) {
    a.mean[tok0 + w] = mean;
    a.rstd[tok0 + w] = rstd;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  bf16raw* out = reinterpret_cast<bf16raw*>(a.out);
  constexpr int CPR = C / 8;                        // 16-B chunks per token
  for (int c = lane; c < 16 * CPR; c += 64) {
    const int r = c / CPR, ch = (c % CPR) * 8;
    if (wave * 16 + r < g.Wo)
      *reinterpret_cast<uint4*>(out + (tok0 + wave * 16 + r) * C + ch) = *reinterpret_cast<const uint4*>(stg + r * SS + ch);
  }
}

template <int NB, int DEPTH>
__global__ __launch_bounds__(NT) void pe_fwd_kernel(const dfk_patch_embed_args a, const PeGeo g, long nrows) {
  constexpr int C = NB * 16, SS = C + 8;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* w_lds = reinterpret_cast<bf16raw*>(smem);
  bf16raw* stg_all = w_lds + C * PKS;
  float* slab = reinterpret_cast<float*>(stg_all + 4 * 16 * SS);
  load_weight<NB>(a, w_lds);
  const PeParams<NB> P = load_params<NB>(a);
  // persistent over token rows: the clip rows of the next DEPTH token rows (r + G, r + 2G) stream into
  // registers while row r computes
  const long G = gridDim.x;
  float4 b0[SLAB_REGS], b1[SLAB_REGS];
  long r = blockIdx.x;
  if (r < nrows) slab_load(a, g, r, b0);
  if (DEPTH == 2 && r + G < nrows) slab_load(a, g, r + G, b1);
  auto step = [&](float4 (&cur)[SLAB_REGS]) {
    __syncthreads();                               // the previous row's slab reads are done
    slab_store(g, cur, slab);
    __syncthreads();
    if (r + DEPTH * G < nrows) slab_load(a, g, r + DEPTH * G, cur);
    pe_fwd_row<NB>(a, g, r, slab, w_lds, stg_all, P);
    r += G;
  };
  while (r < nrows) {
    step(b0);
    if (DEPTH == 1 || r >= nrows) continue;
    step(b1);
  }
}

// Backward, persistent over token rows.  LDS: weight, slab, dconv^T [C][MAXT] and patches^T [96][MAXT]
// (bf16, the operands of dW = dconv^T . patches over the row's tokens), the bias / LN gamma (fp32).
// Software-pipelined like the forward: two register sets hold the clip rows (slab) and the dy / LN-statistics
// rows of the next two token rows, the loop handles two rows per iteration, and a set is reloaded as soon as
// its row has consumed it — the loop issues no global store, so the loads' waits stay counted (partial
// vmcnt).  (The synchronous form — stage the slab, barrier, then load dy, mean, rstd, bias and gamma — paid
// three exposed memory round trips per row: 472 us per C2 launch.)
template <int NB>
__global__ __launch_bounds__(NT) void pe_bwd_kernel(const dfk_patch_embed_args a, const PeGeo g, long nrows,
                                                    const bf16raw* __restrict__ dy) {
  constexpr int C = NB * 16, TS = MAXT + 8;        // transposed tiles' row stride (bf16)
  constexpr int NTILE = NB * (PK / 16), TPW = NTILE / 4;   // dW 16x16 tiles, per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  bf16raw* w_lds = reinterpret_cast<bf16raw*>(smem);
  bf16raw* dcT = w_lds + C * PKS;                  // [C][TS]
  bf16raw* paT = dcT + C * TS;                     // [96][TS]
  float* slab = reinterpret_cast<float*>(paT + PK * TS);
  float* cb = slab + SROWS * g.Ws;                 // [C] conv bias, [C] LN gamma
  float* cg = cb + C;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mrow = lane & 15, nq = (lane >> 4) * 4, kq = (lane >> 4) * 8;
  load_weight<NB>(a, w_lds);
  {
    const bf16raw* gam = reinterpret_cast<const bf16raw*>(a.ln_w);
    const bf16raw* bias = reinterpret_cast<const bf16raw*>(a.b);
    for (int n = tid; n < C; n += NT) { cb[n] = bf2f(bias[n]); cg[n] = bf2f(gam[n]); }
  }
  float dgam[NB][4], dbet[NB][4], dbia[NB][4];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) dgam[nb][r] = dbet[nb][r] = dbia[nb][r] = 0.f;
  f32x4 dw[TPW];
#pragma unroll
  for (int i = 0; i < TPW; ++i) dw[i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int w = wave * 16 + mrow;
  const bool wok = w < g.Wo;
  const int wc = wok ? w : 0;
  // this lane's dy channels and the token's LN statistics for token row `row` (rows past the end: clamped;
  // their values are never used)
  struct RowOps { uint2 d[NB]; float mean, rstd; };
  auto load_ops = [&](long row, RowOps& o) {
    const long tok = (row < nrows ? row : nrows - 1) * g.Wo + wc;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) o.d[nb] = *reinterpret_cast<const uint2*>(dy + tok * C + nb * 16 + nq);
    o.mean = a.mean[tok];
    o.rstd = a.rstd[tok];
  };
  auto compute = [&](const RowOps& o) {
    // patches^T [k][token] (zero for tokens past Wo)
    for (int i = tid; i < PK * MAXT; i += NT) {
      const int k = i / MAXT, m = i % MAXT;
      float v = 0.f;
      if (m < g.Wo) v = slab[(k >> 2) * g.Ws + m * 4 + (k & 3)];
      paT[k * TS + m] = f2bf(v);
    }
    f32x4 acc[NB];
    conv_tokens<NB>(slab, g.Ws, w_lds, wc, acc);
    const float mean = wok ? o.mean : 0.f, rstd = wok ? o.rstd : 0.f;
    float xh[NB][4], gg[NB][4], dyv[NB][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = nb * 16 + nq;
      const uint2 u = wok ? o.d[nb] : make_uint2(0, 0);
      dyv[nb][0] = __uint_as_float(u.x << 16); dyv[nb][1] = __uint_as_float(u.x & 0xffff0000u);
      dyv[nb][2] = __uint_as_float(u.y << 16); dyv[nb][3] = __uint_as_float(u.y & 0xffff0000u);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        xh[nb][r] = (acc[nb][r] + cb[n + r] - mean) * rstd;
        gg[nb][r] = dyv[nb][r] * cg[n + r];
        s1 += gg[nb][r];
        s2 += gg[nb][r] * xh[nb][r];
      }
    }
    const float c1 = group_sum(s1) * (1.f / C), c2 = group_sum(s2) * (1.f / C);
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float dc = wok ? rstd * (gg[nb][r] - c1 - xh[nb][r] * c2) : 0.f;
        dgam[nb][r] += dyv[nb][r] * xh[nb][r];
        dbet[nb][r] += dyv[nb][r];
        dbia[nb][r] += dc;
        dcT[(nb * 16 + nq + r) * TS + w] = f2bf(dc);    // w < 64 always (4 waves x 16)
      }
    __syncthreads();
    // dW[n][k] += sum over the row's tokens of dconv[token][n] * patch[token][k]
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = wave + 4 * i, nt = t % NB, kt = t / NB;
#pragma unroll
      for (int mc = 0; mc < MAXT / 32; ++mc) {
        const bf16x8 af = *reinterpret_cast<const bf16x8*>(dcT + (nt * 16 + mrow) * TS + mc * 32 + kq);
        const bf16x8 bf = *reinterpret_cast<const bf16x8*>(paT + (kt * 16 + mrow) * TS + mc * 32 + kq);
        dw[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bf, dw[i], 0, 0, 0);
      }
    }
  };
  const long G = gridDim.x;
  long row = blockIdx.x;
  float4 s0[SLAB_REGS], s1[SLAB_REGS];
  RowOps o0, o1;
  slab_load(a, g, row, s0);                        // rows past the end read zeros (out-of-range offsets)
  load_ops(row, o0);
  slab_load(a, g, row + G, s1);
  load_ops(row + G, o1);
  // one row per half-iteration: store its slab, reload that register set for the row two ahead, compute
  auto half = [&](float4 (&sr)[SLAB_REGS], RowOps& o) {
    __syncthreads();                               // the previous row's LDS reads are done
    slab_store(g, sr, slab);
    __syncthreads();
    slab_load(a, g, row + 2 * G, sr);
    compute(o);
    load_ops(row + 2 * G, o);
    row += G;
  };
  while (row < nrows) {
    half(s0, o0);
    if (row >= nrows) break;
    half(s1, o1);
  }
  // ---- one atomic per weight (and per LN / bias channel) per workgroup
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int t = wave + 4 * i, nt = t % NB, kt = t / NB;
#pragma unroll
    for (int r = 0; r < 4; ++r) atomicAdd(a.dw + (long)(nt * 16 + nq + r) * PK + kt * 16 + mrow, dw[i][r]);
  }
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float x1 = dgam[nb][r], x2 = dbet[nb][r], x3 = dbia[nb][r];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {              // sum over the 16 tokens of the lane group
        x1 += __shfl_xor(x1, o, 64);
        x2 += __shfl_xor(x2, o, 64);
        x3 += __shfl_xor(x3, o, 64);
      }
      if (mrow == 0) {
        const int n = nb * 16 + nq + r;
        atomicAdd(a.dln_w + n, x1);
        atomicAdd(a.dln_b + n, x2);
        atomicAdd(a.db + n, x3);
      }
    }
}

bool pe_geo(const dfk_patch_embed_args& a, PeGeo& g) {
  if (!a.x || !a.w || !a.b || !a.ln_w || !a.ln_b || a.B <= 0) return false;
  if (a.C != 96 && a.C != 128) return false;
  if (a.sw != 1 || a.sb % 4 || a.sc % 4 || a.st % 4 || a.sh % 4 || (reinterpret_cast<uintptr_t>(a.x) & 15)) return false;
  g.Do = (a.T + 1) / 2;
  g.Ho = (a.H + 3) / 4;
  g.Wo = (a.W + 3) / 4;
  g.Ws = g.Wo * 4 + 4;
  // extent of the clip batch (the largest element offset + 1), for the loads' bounds check
  const long last = (long)(a.B - 1) * a.sb + 2L * a.sc + (long)(a.T - 1) * a.st + (long)(a.H - 1) * a.sh + a.W;
  if (last * 4 >= 0x7fffffffL) return false;
  g.xbytes = (int)(last * 4);
  return g.Wo <= MAXT && a.W % 4 == 0;
}

size_t pe_lds_fwd(int C, const PeGeo& g) { return (size_t)C * PKS * 2 + 4 * 16 * (C + 8) * 2 + (size_t)SROWS * g.Ws * 4; }
size_t pe_lds_bwd(int C, const PeGeo& g) {
  return (size_t)C * PKS * 2 + (size_t)(C + PK) * (MAXT + 8) * 2 + (size_t)SROWS * g.Ws * 4 + (size_t)C * 8;
}

}  // namespace

extern "C" int dfk_patch_embed_fwd(const dfk_patch_embed_args* ap, hipStream_t s) {
  if (!ap) return DFK_EINVAL;
  const dfk_patch_embed_args& a = *ap;
  PeGeo g;
  if (!pe_geo(a, g) || !a.out || !a.mean || !a.rstd || (reinterpret_cast<uintptr_t>(a.out) & 15)) return DFK_EINVAL;
  const long rows = (long)a.B * g.Do * g.Ho;
  const size_t lds = pe_lds_fwd(a.C, g);
  if (lds > 80 * 1024) return DFK_EINVAL;   // two workgroups per CU
  static bool attr_set = false;   // C = 128 (Swin-B) needs a little over 64 KB; once per process, never in a capture
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)pe_fwd_kernel<6, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)pe_fwd_kernel<6, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)pe_fwd_kernel<8, 1>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    (void)hipFuncSetAttribute((const void*)pe_fwd_kernel<8, 2>, hipFuncAttributeMaxDynamicSharedMemorySize, 80 * 1024);
    attr_set = true;
  }
  // persistent: two workgroups per CU (tuning knobs DFK_PE_PERCU / DFK_PE_DEPTH for tools/pe_bench.py)
  static const int env_cu = getenv("DFK_PE_PERCU") ? atoi(getenv("DFK_PE_PERCU")) : 2;
  static const int depth = getenv("DFK_PE_DEPTH") ? atoi(getenv("DFK_PE_DEPTH")) : 2;
  const unsigned grid = (unsigned)std::min<long>(rows, 256L * std::max(1, env_cu));
  if (a.C == 96) {
    if (depth == 1) hipLaunchKernelGGL((pe_fwd_kernel<6, 1>), dim3(grid), dim3(NT), lds, s, a, g, rows);
    else hipLaunchKernelGGL((pe_fwd_kernel<6, 2>), dim3(grid), dim3(NT), lds, s, a, g, rows);
  } else {
    if (depth == 1) hipLaunchKernelGGL((pe_fwd_kernel<8, 1>), dim3(grid), dim3(NT), lds, s, a, g, rows);
    else hipLaunchKernelGGL((pe_fwd_kernel<8, 2>), dim3(grid), dim3(NT), lds, s, a, g, rows);
  }
  DFK_CHECK_LAUNCH();
  return 0;
}

extern "C" int dfk_patch_embed_bwd(const dfk_patch_embed_args* ap, const void* dy, hipStream_t s) {
  if (!ap || !dy) return DFK_EINVAL;
  const dfk_patch_embed_args& a = *ap;
  PeGeo g;
  if (!pe_geo(a, g) || !a.mean || !a.rstd || !a.dw || !a.db || !a.dln_w || !a.dln_b) return DFK_EINVAL;
  if (reinterpret_cast<uintptr_t>(dy) & 7) return DFK_EINVAL;
  const long rows = (long)a.B * g.Do * g.Ho;
  const size_t lds = pe_lds_bwd(a.C, g);
  if (lds > 160 * 1024) return DFK_EINVAL;
  static bool attr_set = false;   // once per process (never inside a capture: the first call is eager)
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)pe_bwd_kernel<6>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)pe_bwd_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr_set = true;
  }
  // one workgroup per CU (the kernel's VGPR + AGPR budget leaves one wave per SIMD), persistent over rows
  const unsigned grid = (unsigned)std::min<long>(rows, 256);
  if (a.C == 96)
    hipLaunchKernelGGL(pe_bwd_kernel<6>, dim3(grid), dim3(NT), lds, s, a, g, rows, (const bf16raw*)dy);
  else
    hipLaunchKernelGGL(pe_bwd_kernel<8>, dim3(grid), dim3(NT), lds, s, a, g, rows, (const bf16raw*)dy);
  DFK_CHECK_LAUNCH();
  return 0;
}
