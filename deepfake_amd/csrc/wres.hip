// Weight-resident streaming GEMM for the HBM-bound Linears of the Swin stages 1-2 (and the mel
// branch's stage 1): C[M, N] = A[M, K] . W^T with a small weight (N*K <= WRES_LIMIT elements per
// column slice) and a huge token count M (50k-400k rows).  dfk_gemm routes such launches here.
//
// Why a separate kernel: with K = 96..384 the tiled GEMM's k-loop is 2-6 steps long, so every
// output tile pays a full prologue (two dependent global->LDS->MFMA round trips) and only one tile
// per workgroup is ever in flight: the stage-1 qkv Linear (401k x 96 -> 288) ran at 1.5 TB/s of the
// 8 TB/s HBM roofline.  Here a persistent workgroup loads its W column slice into LDS ONCE and then
// streams 128-row tiles of A: each wave owns 16 rows, loads its A fragments straight from HBM into
// registers (16-B loads in MFMA fragment order, no LDS round trip), prefetches the next tile's
// fragments while it computes the current one, and stores its outputs without LDS staging.
//
// Operand order is swapped (D = W . A^T) so that every lane ends up with FOUR CONSECUTIVE OUTPUT
// CHANNELS of one token: v_mfma_f32_16x16x32_bf16 leaves D[n = 4*(l>>4) + r][m = l&15] in lane l,
// so bias / residual / aux / C are 8-byte vector accesses along a token row.
//
//   W operand: B view rows = output channels j; b_kmajor = 0: W[j][k] (nn.Linear weight, forward),
//              b_kmajor = 1: W[k][j] (the dX GEMM dy . W reads the weight transposed)
//   A operand: a_kmajor = 0 only (token rows, k contiguous), bf16.
#include <algorithm>

#include "common.h"

namespace {

// cache policy of the output stores (buffer-store aux bits; 2 = non-temporal: the outputs stream past the L2 —
// stage-1 fc1 93 vs 124 us, fc2 dX 93 vs 127 us once the loop keeps its loads in flight, r4z2)
#ifndef DFK_WRES_NT
#define DFK_WRES_NT 2
#endif

constexpr int WRES_LIMIT = 49152;      // W slice elements (96 KiB bf16) -> one 8-wave workgroup per CU
constexpr int NT = 512;                // 8 waves x 16 token rows = 128-row tiles

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int KC, int NBW, int NSPLIT>
constexpr int wres_lds() { return (NBW * 16 * NSPLIT * (KC * 32 + 8) + 8 * 16 * (NBW * 16 + 8)) * 2 + NBW * 16 * NSPLIT * 4; }

// Workgroups per CU: two (4 waves per SIMD, <= 128 VGPRs) where the W slice, the staging tiles and the bias fit
// twice in the LDS (K <= 128 at 6 column blocks) — the launches are latency-bound, so twice the waves in flight
// is twice the bytes in flight — otherwise one (2 waves per SIMD, <= 256 VGPRs).
#ifndef DFK_WRES_R9
#define DFK_WRES_R9 4   // register rings for the 9-block-wide variants up to this KC
#endif
#ifndef DFK_WRES_TWO
#define DFK_WRES_TWO 0
#endif
template <int KC, int NBW, int NSPLIT>
constexpr bool wres_two_per_cu() { return DFK_WRES_TWO && NBW == 6 && KC <= 4; }

// ACT: 0 plain, 1 GELU (pre-activation -> aux), 2 times gelu'(aux); RES: residual add.  Template parameters so
// the epilogue has no data-dependent branches around its loads (a branch around a load makes the compiler wait
// vmcnt(0) there, and vmcnt also counts the previous tile's stores) and loads nothing it does not use
template <int KC, int NBW, int NSPLIT, int ACT, bool RES>
__global__ __launch_bounds__(512, (wres_two_per_cu<KC, NBW, NSPLIT>() ? 4 : 2))
void wres_kernel(const dfk_gemm_args g, int nslices, int ntiles) {
  // slice of BN = NSPLIT*NBW*16 output channels; the 8 waves form (8/NSPLIT) row groups x NSPLIT column
  // groups, each wave computing 16 tokens x NBW*16 channels (few accumulators -> several waves per SIMD)
  constexpr int K = KC * 32, BN = NBW * 16 * NSPLIT, WS = K + 8;   // LDS row stride (elements), padded 16 B
  constexpr int ROWS_T = 16 * (8 / NSPLIT);
  constexpr int SS = NBW * 16 + 8;                                 // output staging row stride
  __shared__ __attribute__((aligned(16))) bf16raw w_lds[BN * WS + 8 * 16 * SS];
  __shared__ __attribute__((aligned(16))) float b_lds[BN];   // the slice's bias (0 without one), fp32
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  bf16raw* stg = w_lds + BN * WS + wave * 16 * SS;
  const int rg = wave / NSPLIT, cg = wave % NSPLIT;
  // block -> (column slice, first tile).  When the grid is a multiple of 8 x nslices, the nslices slices of one
  // row tile are blocks b, b + 8, b + 16, ... — one XCD (blocks are dealt to the 8 XCDs round robin) — so the
  // A rows they all read come from that XCD's L2 after the first; otherwise slice-major as before
#ifndef DFK_WRES_XCD
#define DFK_WRES_XCD 1
#endif
  const bool xcd_map = DFK_WRES_XCD && nslices > 1 && gridDim.x % (8 * nslices) == 0;
  const int bj = blockIdx.x >> 3;
  const int slice = xcd_map ? bj % nslices : blockIdx.x % nslices;
  const int t_first = xcd_map ? (bj / nslices) * 8 + (blockIdx.x & 7) : blockIdx.x / nslices;
  const int n0 = slice * BN;
  const int stride = gridDim.x / nslices;
  const bf16raw* W = reinterpret_cast<const bf16raw*>(g.b.ptr);

  // ---- W slice -> LDS [BN][K] (rows past N zero-filled)
  if (!g.b_kmajor) {            // W[j][k]: rows of K contiguous elements, 16-B copies
    for (int idx = tid; idx < BN * (K / 8); idx += NT) {
      const int j = idx / (K / 8), kc = (idx % (K / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + j < g.N) v = *reinterpret_cast<const uint4*>(W + (long)(n0 + j) * g.b.ld + kc);
      *reinterpret_cast<uint4*>(w_lds + j * WS + kc) = v;
    }
  } else {                      // W[k][j]: 8 output channels of one k per 16-B load, transposed into LDS
    for (int idx = tid; idx < K * (BN / 8); idx += NT) {
      const int k = idx / (BN / 8), jc = (idx % (BN / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (n0 + jc < g.N) v = *reinterpret_cast<const uint4*>(W + (long)k * g.b.ld + n0 + jc);
      const bf16raw* e = reinterpret_cast<const bf16raw*>(&v);
#pragma unroll
      for (int i = 0; i < 8; ++i) w_lds[(jc + i) * WS + k] = e[i];
    }
  }
  const bf16raw* bias = reinterpret_cast<const bf16raw*>(g.bias);
  for (int j = tid; j < BN; j += NT) b_lds[j] = bias && n0 + j < g.N ? bf2f(bias[n0 + j]) : 0.f;
  __syncthreads();

  const bf16raw* A = reinterpret_cast<const bf16raw*>(g.a.ptr);
  const bf16raw* res = reinterpret_cast<const bf16raw*>(g.residual);
  bf16raw* aux = reinterpret_cast<bf16raw*>(g.aux);
  bf16raw* C = reinterpret_cast<bf16raw*>(g.c);
  const int mrow = lane & 15, kq = (lane >> 4) * 8, nq = (lane >> 4) * 4;
  const DropCtx dc = drop_ctx(g.drop);   // dropout / DropPath of the output (mode 0: none)
  const bf16raw* wbase = w_lds + (cg * NBW * 16 + mrow) * WS + kq;
  const int c0 = n0 + cg * NBW * 16;                    // first channel of this wave's columns
  // buffer descriptors of the outputs: exactly the M rows (bounds-checked stores)
  auto rsrc_of = [&](void* p, long ld) {
    const long bytes = (long)g.M * ld * 2;
    return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)(bytes < 0x7fffffffL ? bytes : 0x7fffffffL), 0x00020000);
  };
  const __amdgpu_buffer_rsrc_t rC = rsrc_of(C, g.ldc);
  const __amdgpu_buffer_rsrc_t rAux = rsrc_of(aux ? (void*)aux : (void*)C, aux ? g.ldaux : g.ldc);

  // this wave's fragment row of tile t: token m = t*ROWS_T + rg*16 + (lane&15)
  auto load_a = [&](int t, uint4 (&fr)[KC]) {
    const long m = (long)t * ROWS_T + rg * 16 + mrow;
    const bool ok = m < g.M;
    // rows past M read row 0 and are NOT zeroed: output row m depends on A row m alone and the stores drop rows
    // >= M.  (Zeroing them made the compiler place the mask — and an s_waitcnt vmcnt(0) on this very prefetch,
    // and every store before it — at the end of the previous tile, so no load or store was ever in flight
    // across a tile boundary.)
    const bf16raw* p = A + (ok ? m : 0) * g.a.ld + kq;
#pragma unroll
    for (int kc = 0; kc < KC; ++kc) fr[kc] = *reinterpret_cast<const uint4*>(p + kc * 32);
  };

  constexpr int NAX = ACT == 2 ? NBW : 1, NRR = RES ? NBW : 1;
  // the tile's per-token epilogue operands (residual, gelu input rows; the bias is in LDS)
  auto load_epi = [&](int t, uint2 (&rr)[NRR], uint2 (&ax)[NAX]) {
    const long m = (long)t * ROWS_T + rg * 16 + mrow;
    const long mc = m < g.M ? m : g.M - 1;               // clamped row (the store mask drops the tail)
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) {
      const int n = min(c0 + nb * 16 + nq, g.N - 4);
      if constexpr (RES) rr[nb] = *reinterpret_cast<const uint2*>(res + mc * g.ldr + n);
      if constexpr (ACT == 2) ax[nb] = *reinterpret_cast<const uint2*>(aux + mc * g.ldaux + n);
    }
  };

  auto process = [&](int t, const uint4 (&a_cur)[KC], const uint2 (&rr)[NRR], const uint2 (&ax)[NAX]) {
    const long m = (long)t * ROWS_T + rg * 16 + mrow;

    f32x4 acc[NBW];
#pragma unroll
    for (int nb = 0; nb < NBW; ++nb) acc[nb] = f32x4{0.f, 0.f, 0.f, 0.f};
    // W fragments stream from LDS through a 4-deep register ring (each is used by exactly one MFMA):
    // the read for step i+RING-1 is issued before MFMA i, and a scheduling barrier keeps the compiler
    // from hoisting all KC*NBW reads to the top (that spilled the accumulators)
    constexpr int T = KC * NBW, RING = 4;
    auto wfrag = [&](int i) {
      return *reinterpret_cast<const bf16x8*>(wbase + (i % NBW) * 16 * WS + (i / NBW) * 32);
    };
    bf16x8 wr[RING];
#pragma unroll
    for (int i = 0; i < RING - 1 && i < T; ++i) wr[i] = wfrag(i);
#pragma unroll
    for (int i = 0; i < T; ++i) {
      if (i + RING - 1 < T) wr[(i + RING - 1) % RING] = wfrag(i + RING - 1);
      acc[i % NBW] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wr[i % RING], __builtin_bit_cast(bf16x8, a_cur[i / NBW]),
                                                              acc[i % NBW], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    }

    // ---- epilogue: lane holds channels n0 + (cg*NBW + nb)*16 + nq .. +3 of token m.  Outputs go through
    // a per-wave LDS tile so that global stores are whole 16-B chunks of token rows (8-B stores scattered
    // over 16 rows per instruction ran the write-heavy launches at 2.2-2.8 TB/s)
    auto bias4 = [&](int nb, float (&v)[4]) {
      const f32x4 b = *reinterpret_cast<const f32x4*>(b_lds + cg * NBW * 16 + nb * 16 + nq);
      v[0] = acc[nb][0] + b[0]; v[1] = acc[nb][1] + b[1]; v[2] = acc[nb][2] + b[2]; v[3] = acc[nb][3] + b[3];
    };
    const long mt0 = (long)t * ROWS_T + rg * 16;          // first token of this wave's tile
    // LDS-only wave syncs: a release fence would also wait vmcnt(0), i.e. for the next tile's A prefetch
    auto lds_sync = [] {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    };
    // staged [16][NBW*16] tile -> dst rows by buffer stores: rows past M fall outside the descriptor's range
    // and columns past N get an out-of-range offset, so the hardware drops them and no branch surrounds a
    // store (a branch around a store makes hipcc wait vmcnt(0) — for the A prefetch too — after it)
    auto flush = [&](__amdgpu_buffer_rsrc_t rs, long ld) {
      lds_sync();
      constexpr int CPR = NBW * 2;                          // 16-B chunks per row
#pragma unroll
      for (int c = lane; c < 16 * CPR; c += 64) {
        const int r = c / CPR, ch = (c % CPR) * 8;
        const u32x4 u = *reinterpret_cast<const u32x4*>(stg + r * SS + ch);
        const long e = (mt0 + r) * ld + c0 + ch;            // element offset
        const uint32_t off = (c0 + ch < g.N && e < 0x7fffffffL) ? (uint32_t)(e * 2) : 0xfffffff0u;
        __builtin_amdgcn_raw_buffer_store_b128(u, rs, off, 0, DFK_WRES_NT);
      }
      lds_sync();                                         // reads done before the tile is rewritten
    };
    auto put = [&](int nb, const float (&v)[4], bf16raw* dst, long ld) {
      uint2 o;
      o.x = (uint32_t)f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16);
      o.y = (uint32_t)f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16);
      *reinterpret_cast<uint2*>(stg + mrow * SS + nb * 16 + nq) = o;   // (dfk_wres_try guarantees staging)
    };
    if constexpr (ACT == 1) {       // the pre-activation (GELU backward input) first
      if (aux) {
#pragma unroll
        for (int nb = 0; nb < NBW; ++nb) {
          float v[4];
          bias4(nb, v);
          put(nb, v, aux, g.ldaux);
        }
        flush(rAux, g.ldaux);
      }
    }
    {
      const float gmul = dc.mode == 2 ? drop_mul(dc, m, 0) : 1.f;   // DropPath: one draw per token group
#pragma unroll
      for (int nb = 0; nb < NBW; ++nb) {
        const int n = c0 + nb * 16 + nq;
        float v[4];
        bias4(nb, v);
        if constexpr (ACT == 1) {
#pragma unroll
          for (int e = 0; e < 4; e += 2) {
            const f32x2 r = gelu_bf2(f32x2{v[e], v[e + 1]});
            v[e] = r.x;
            v[e + 1] = r.y;
          }
        } else if constexpr (ACT == 2) {
          const uint2 a = ax[nb];
          const f32x2 d0 = dgelu_bf2(f32x2{__uint_as_float(a.x << 16), __uint_as_float(a.x & 0xffff0000u)});
          const f32x2 d1 = dgelu_bf2(f32x2{__uint_as_float(a.y << 16), __uint_as_float(a.y & 0xffff0000u)});
          v[0] *= d0.x; v[1] *= d0.y; v[2] *= d1.x; v[3] *= d1.y;
        }
        if (dc.mode == 2) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= gmul;
        } else if (dc.mode == 1) {
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] *= drop_mul(dc, m, n + e);
        }
        if constexpr (RES) {
          const uint2 r = rr[nb];
          v[0] += __uint_as_float(r.x << 16); v[1] += __uint_as_float(r.x & 0xffff0000u);
          v[2] += __uint_as_float(r.y << 16); v[3] += __uint_as_float(r.y & 0xffff0000u);
        }
        put(nb, v, C, g.ldc);
      }
      flush(rC, g.ldc);
    }
  };

  // Software pipeline.  RING2 (the narrow-K variants with registers to spare): two register sets of A fragments
  // and epilogue operands, the loop unrolled by two tiles; tile tt + 2 stride is requested into the set tile tt
  // has just consumed, so each load has a whole tile in flight and no register is ever copied (a copy of a
  // loaded register waits for the load — an earlier form copied the freshly issued prefetch and waited vmcnt(0),
  // i.e. for it and every store, once per tile).  Otherwise one set: the next tile's A is requested before this
  // tile computes (copied first), its epilogue operands at its start.  A tile index past the end computes on
  // clamped loads and its stores fall outside the output descriptor (rows >= M): no branch surrounds a load or
  // a store.
  constexpr bool RING2 = (NBW == 6 ? KC <= 8 : KC <= DFK_WRES_R9) && !wres_two_per_cu<KC, NBW, NSPLIT>();
  int t = t_first;
  if constexpr (RING2) {
    uint4 a0[KC], a1[KC];
    uint2 r0[NRR], r1[NRR], x0[NAX], x1[NAX];
    load_a(min(t, ntiles - 1), a0);
    load_epi(t, r0, x0);
    load_a(min(t + stride, ntiles - 1), a1);
    load_epi(t + stride, r1, x1);
    for (; t < ntiles; t += 2 * stride) {
      process(t, a0, r0, x0);
      load_a(min(t + 2 * stride, ntiles - 1), a0);
      load_epi(t + 2 * stride, r0, x0);
      __builtin_amdgcn_sched_barrier(0);
      process(t + stride, a1, r1, x1);
      load_a(min(t + 3 * stride, ntiles - 1), a1);
      load_epi(t + 3 * stride, r1, x1);
      __builtin_amdgcn_sched_barrier(0);
    }
  } else {
    uint4 a0[KC];
    load_a(min(t, ntiles - 1), a0);
    for (; t < ntiles; t += stride) {
      uint4 cur[KC];
#pragma unroll
      for (int kc = 0; kc < KC; ++kc) cur[kc] = a0[kc];
      uint2 rr[NRR], ax[NAX];
      load_epi(t, rr, ax);
      load_a(min(t + stride, ntiles - 1), a0);
      process(t, cur, rr, ax);
    }
  }
}

template <int KC, int NBW, int NSPLIT>
void launch_wres(const dfk_gemm_args& g, int nslices, hipStream_t s) {
  static_assert(NT == 512, "8-wave workgroups");
  // persistent grid: as many 8-wave workgroups per CU as the W slice's LDS allows (1 or 2), a multiple
  // of the slice count so every workgroup keeps one slice for its whole life
  constexpr int per_cu = wres_two_per_cu<KC, NBW, NSPLIT>() ? 2 : 1;
  const int ntiles = dfk_cdiv(g.M, 16 * (8 / NSPLIT));
  const int per = std::max(1, std::min(ntiles, 256 * per_cu / nslices));
  const dim3 grid(per * nslices);
#define WRES_L(ACT, RES) hipLaunchKernelGGL((wres_kernel<KC, NBW, NSPLIT, ACT, RES>), grid, dim3(NT), 0, s, g, nslices, ntiles)
  const bool res = g.residual != nullptr;
  if (g.act == 1) { if (res) WRES_L(1, true); else WRES_L(1, false); }
  else if (g.act == 2) { if (res) WRES_L(2, true); else WRES_L(2, false); }
  else { if (res) WRES_L(0, true); else WRES_L(0, false); }
#undef WRES_L
}

bool al8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7) == 0; }

}  // namespace

// 1 = launched, 0 = not applicable (caller runs the tiled GEMM), < 0 = launch error
int dfk_wres_try(const dfk_gemm_args& g, hipStream_t s) {
  static const bool off = getenv("DFK_WRES") && atoi(getenv("DFK_WRES")) == 0;
  if (off) return 0;
  if (g.dtype != DFK_BF16 || g.a_kmajor || g.c_f32 || g.atomic || g.splitk != 1 || g.rowsum) return 0;
  if (g.nz0 != 1 || g.nz1 != 1 || g.a.conv_cg > 0 || g.b.conv_cg > 0 || g.beta != 0.f) return 0;
  if (g.M < 16384 || g.K % 32 || g.K > 384 || g.N % 4) return 0;
  if ((g.act == 2 && !g.aux) || g.act == 3 || (g.alpha != 0.f && g.alpha != 1.f)) return 0;
  if (g.a.ld % 8 || ((uintptr_t)g.a.ptr & 15) || g.b.ld % 8 || ((uintptr_t)g.b.ptr & 15)) return 0;
  if (g.ldc % 4 || !al8(g.c) || (g.bias && !al8(g.bias)) || (g.residual && (g.ldr % 4 || !al8(g.residual))) ||
      (g.aux && (g.ldaux % 4 || !al8(g.aux))))
    return 0;
  if (g.b_kmajor && g.N % 8) return 0;
  // outputs leave through the per-wave LDS staging tile as whole 16-B chunks of token rows
  if (g.ldc % 8 || ((uintptr_t)g.c & 15) || g.N % 8 || (g.aux && (g.ldaux % 8 || ((uintptr_t)g.aux & 15)))) return 0;
  const int KC = g.K / 32;
  // widest slice (fewest A re-reads) that fits WRES_LIMIT, then the least padding among equal counts
  int best = 0, best_sl = 1 << 30, best_waste = 1 << 30;
  for (int bn : {288, 192, 96}) {
    if (bn * g.K > WRES_LIMIT) continue;
    const int sl = dfk_cdiv(g.N, bn), waste = sl * bn - g.N;
    if (sl < best_sl || (sl == best_sl && waste < best_waste)) { best = bn; best_sl = sl; best_waste = waste; }
  }
  if (!best || best_sl > 8) return 0;
  // slice = NSPLIT column groups of NBW*16 channels: 96 (6x1), 192 (6x2), 288 (9x2)
#define WRES_CASE(kc, nbw, ns) \
  if (KC == kc && best == nbw * 16 * ns) { launch_wres<kc, nbw, ns>(g, best_sl, s); DFK_CHECK_LAUNCH(); return 1; }
  WRES_CASE(3, 9, 2) WRES_CASE(4, 9, 2)
  WRES_CASE(3, 6, 2) WRES_CASE(4, 6, 2) WRES_CASE(6, 6, 2) WRES_CASE(8, 6, 2)
  WRES_CASE(3, 6, 1) WRES_CASE(4, 6, 1) WRES_CASE(6, 6, 1) WRES_CASE(8, 6, 1) WRES_CASE(9, 6, 1) WRES_CASE(12, 6, 1)
#undef WRES_CASE
  return 0;
}
