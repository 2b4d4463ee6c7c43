// Token-streaming weight-gradient GEMM for the HBM-bound Linears of the Swin stages 1-2 (and the mel branch's
// stage 1): dW[R, C] += dy^T x over T = 16k-401k tokens, with a small output (R x C <= 384 x 384 per slice),
// plus the bias gradient db[R] += colsum(dy) from the same pass.  dfk_gemm routes such launches here (the
// weight gradients of video_swin_transformer.py:134,136 and src/utils.py:249-251, i.e. the dW of qkv / proj /
// fc1 / fc2 / PatchMerging.reduction).
//
// Why a separate kernel: the tiled GEMM covers dW with 128 x 128 output tiles and a caller-planned split of the
// token reduction, so every output tile re-reads its operand columns (x was read once per 128 rows of dW: three
// times for the stage-1 qkv) and every split pays a prologue.  Here a workgroup owns a whole output SLICE in
// registers (each wave a 48x96 / 96x48 / 64x64 block of fp32 accumulators) and streams a contiguous token range
// of dy and x through LDS exactly once; the partial slice is added to dW with fp32 atomics at the end.
//
// Data movement: per 64-token chunk, dy[t0:t0+64, r0:r0+NS] and x[t0:t0+64, c0:c0+KS] go HBM -> LDS by
// buffer_load ... lds (16 B per lane, 1 KB per wave-instruction, no VGPR staging), two LDS stages.  The MFMA
// operands contract over TOKENS, so both are read token-transposed with ds_read_b64_tr_b16.  Conflict-freedom of
// those reads (2 groups of 32 lanes, each 8 token rows x 32 B): (1) token rows are stored permuted within each
// 32-token k-step (bits 2 and 3 of the token index swapped), so a lane group's 8 rows are 8 CONSECUTIVE image
// rows; (2) within a row, 32-B column pairs are XOR-swizzled by the row (on the source address) so that 8
// consecutive rows land on 8 distinct 8-dword bank windows whatever the row pitch mod 256 B.
//
// Slice assignment: workgroup (partition p, slice s) with p on XCD p mod 8: the slices of one token range run on
// one XCD, so their re-reads of dy / x columns hit that XCD's L2.
#include <algorithm>

#include "common.h"

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short short4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) short4v lds_short4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int TS = 64;   // tokens per chunk (two 32-token MFMA k-steps)

// image row of token t within its 32-token k-step: bits 2 and 3 swapped (an involution)
__host__ __device__ constexpr int tok_row(int t) { return (t & ~12) | ((t & 4) << 1) | ((t & 8) >> 1); }

// 32-B column-pair XOR of image row r for a row pitch of W bf16: u = pitch in 8-dword bank windows mod 8
template <int W>
__device__ __forceinline__ int pair_xor(int r) {
  constexpr int u = (W / 16) % 8;
  if constexpr (u == 0) return r & 7;
  else if constexpr (u == 4) return (r >> 1) & 3;
  else if constexpr (u == 2 || u == 6) return (r >> 2) & 1;
  else return 0;
}
template <int W>
constexpr bool pair_xor_ok() {   // the XOR stays inside the row's column pairs
  constexpr int u = (W / 16) % 8, pairs = W / 16;
  return W % 16 == 0 && (u % 2 == 1 || (u == 0 && pairs % 8 == 0) || (u == 4 && pairs % 4 == 0) ||
                         ((u == 2 || u == 6) && pairs % 2 == 0));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory");
}

// one operand's chunk: image [TS][W] bf16, NI 1-KB wave-instructions spread round-robin over the NW waves
template <int W, int NW>
struct ChunkDma {
  static constexpr int NI = TS * W * 2 / 1024;          // = W / 8
  static constexpr int PER = (NI + NW - 1) / NW;        // instructions of the busiest wave
  static constexpr int MIN = NI / NW;                   // ... of the least busy one
  __device__ static __forceinline__ void issue(__amdgpu_buffer_rsrc_t rs, long ld, int col0, long t0, long tend,
                                               bf16raw* img, int wave, int lane) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = i * NW + wave;                      // wave-uniform
      if (NI % NW == 0 || j < NI) {
        const int s = j * 64 + lane;                    // 16-B slot of the image
        const int r = s / (W / 8), c = s % (W / 8);
        const long t = t0 + tok_row(r);                 // tok_row is its own inverse
        const int col = col0 + 16 * ((c >> 1) ^ pair_xor<W>(r)) + 8 * (c & 1);
        const uint32_t off = t < tend ? (uint32_t)((t * ld + col) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(img + j * 512), 16, off, 0, 0, 0);
      }
    }
  }
};

// 16 channels (block m of the image's 16-column blocks) x 8 tokens of k-step ks, token-transposed:
// lane l receives channel 16m + (l&15), tokens 8(l>>4) .. +7 of the k-step (the MFMA A / B operand layout)
template <int W>
__device__ __forceinline__ bf16x8 frag_t(const bf16raw* img, int ks, int m, int rowoff, int lx, int p4) {
  const bf16raw* a0 = img + ks * 32 * W + rowoff + 16 * (m ^ lx) + p4;
  const short4v lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0));
  const short4v hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_short4*)(a0 + 8 * W));
  short8 u = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8, u);
}

// NBR x NBC 16x16 output blocks per wave, WR x WC waves: slice NS x KS = (16 WR NBR) x (16 WC NBC)
template <int NBR, int NBC, int WR, int WC, bool RS>
__global__ __launch_bounds__(WR * WC * 64) void wgrad_kernel(const dfk_gemm_args g, int nsl_c, int nsl, long tpw) {
  constexpr int NW = WR * WC, NS = 16 * WR * NBR, KS = 16 * WC * NBC;
  static_assert(pair_xor_ok<NS>() && pair_xor_ok<KS>(), "slice widths without a conflict-free swizzle");
  using DA = ChunkDma<NS, NW>;
  using DB = ChunkDma<KS, NW>;
  constexpr int STAGE = TS * NS + TS * KS;
  __shared__ __attribute__((aligned(16))) bf16raw smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / WC, wc = wave % WC;

  // workgroup -> (token partition p, slice): the slices of partition p share its XCD (bid mod 8)
  const int bid = blockIdx.x, xcd = bid & 7, jx = bid >> 3;
  const int p = xcd + 8 * (jx / nsl), slice = jx % nsl;
  const int r0 = (slice / nsl_c) * NS, c0 = (slice % nsl_c) * KS;
  const long t0 = (long)p * tpw, tend = t0 + tpw < (long)g.K ? t0 + tpw : (long)g.K;
  const int nch = tend > t0 ? (int)((tend - t0 + TS - 1) / TS) : 0;

  const bf16raw* A = reinterpret_cast<const bf16raw*>(g.a.ptr);   // dy [T][R] (a_kmajor view)
  const bf16raw* B = reinterpret_cast<const bf16raw*>(g.b.ptr);   // x  [T][C] (b_kmajor view)
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16raw*>(A), (short)0, (int)(((long)g.K - 1) * g.a.ld * 2 + (long)g.M * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<bf16raw*>(B), (short)0, (int)(((long)g.K - 1) * g.b.ld * 2 + (long)g.N * 2), 0x00020000);

  auto issue = [&](int ch, bf16raw* st) {
    const long tc = t0 + (long)ch * TS;
    DA::issue(ra, g.a.ld, r0, tc, tend, st, wave, lane);
    DB::issue(rb, g.b.ld, c0, tc, tend, st + TS * NS, wave, lane);
  };

  // lane constants of the transposed fragment reads: image row 16(g>>1) + 4(g&1) + q (+8 for tokens 4..7)
  const int li = lane & 15, q = li >> 2, gq = lane >> 4;
  const int rl = 16 * (gq >> 1) + 4 * (gq & 1) + q;
  const int p4 = 4 * (li & 3);
  const int lxa = pair_xor<NS>(rl), lxb = pair_xor<KS>(rl);
  const int roa = rl * NS, rob = rl * KS;

  f32x4 acc[NBR][NBC];
#pragma unroll
  for (int i = 0; i < NBR; ++i)
#pragma unroll
    for (int j = 0; j < NBC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accr[NBR];
#pragma unroll
  for (int i = 0; i < NBR; ++i) accr[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_rs = RS && wc == 0 && c0 == 0;   // the bias gradient once per output row
  bf16x8 ones;
#pragma unroll
  for (int j = 0; j < 8; ++j) ones[j] = (__bf16)1.0f;

  if (nch > 0) issue(0, smem);
  for (int ch = 0; ch < nch; ++ch) {
    wait_vm<0>();                                          // this wave's DMAs of chunk ch have landed
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");     // and its reads of chunk ch-1 are done
    __builtin_amdgcn_s_barrier();                          // ... for every wave
    asm volatile("" ::: "memory");
    if (ch + 1 < nch) issue(ch + 1, smem + ((ch + 1) & 1) * STAGE);
    const bf16raw* ia = smem + (ch & 1) * STAGE;
    const bf16raw* ib = ia + TS * NS;
#pragma unroll
    for (int ks = 0; ks < TS / 32; ++ks) {
      bf16x8 fa[NBR], fb[NBC];
#pragma unroll
      for (int i = 0; i < NBR; ++i) fa[i] = frag_t<NS>(ia, ks, wr * NBR + i, roa, lxa, p4);
#pragma unroll
      for (int j = 0; j < NBC; ++j) fb[j] = frag_t<KS>(ib, ks, wc * NBC + j, rob, lxb, p4);
#pragma unroll
      for (int i = 0; i < NBR; ++i)
#pragma unroll
        for (int j = 0; j < NBC; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], fb[j], acc[i][j], 0, 0, 0);
      if (RS && do_rs) {
#pragma unroll
        for (int i = 0; i < NBR; ++i) accr[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[i], ones, accr[i], 0, 0, 0);
      }
    }
  }
  if (nch == 0) return;
  // partial slice -> dW (fp32 atomics): lane l holds rows 4(l>>4) + r, column l&15 of each 16x16 block
  float* C = reinterpret_cast<float*>(g.c);
#pragma unroll
  for (int i = 0; i < NBR; ++i)
#pragma unroll
    for (int j = 0; j < NBC; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = r0 + (wr * NBR + i) * 16 + 4 * gq + r, col = c0 + (wc * NBC + j) * 16 + li;
        atomicAdd(C + (long)row * g.ldc + col, acc[i][j][r]);
      }
  if (RS && do_rs && li == 0) {
#pragma unroll
    for (int i = 0; i < NBR; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) atomicAdd(g.rowsum + r0 + (wr * NBR + i) * 16 + 4 * gq + r, accr[i][r]);
  }
}

struct WgShape { int nbr, nbc, wr, wc; };
// the instantiated wave grids (C2 / C4 Swin-T / Swin-B / SwinV2-B stage-1-2 dW shapes, PatchMerging reductions)
constexpr WgShape kShapes[] = {
    {3, 6, 6, 1}, {3, 6, 8, 1}, {3, 6, 2, 1}, {6, 3, 1, 8}, {3, 6, 4, 2},
    {6, 3, 2, 4}, {4, 4, 3, 2}, {4, 4, 4, 2}, {4, 4, 2, 4}, {4, 4, 2, 2},
};

template <int NBR, int NBC, int WR, int WC>
void launch_wg(const dfk_gemm_args& g, hipStream_t s) {
  constexpr int NS = 16 * WR * NBR, KS = 16 * WC * NBC;
  const int nsl_r = g.M / NS, nsl_c = g.N / KS, nsl = nsl_r * nsl_c;
  constexpr long lds = 2L * TS * (NS + KS) * 2;
  const int per_cu = std::max(1, (int)std::min<long>(160 * 1024 / lds, 16 / (WR * WC)));
  // token partitions: a multiple of 8 (one XCD each), about one resident workgroup per slot, >= 4 chunks each
  const long want = std::max<long>(1, (long)256 * per_cu / nsl);
  long P = std::max<long>(8, (want + 4) / 8 * 8);
  P = std::min<long>(P, std::max<long>(8, ((long)g.K / (4 * TS)) / 8 * 8));
  long tpw = dfk_cdiv((long)g.K, P);
  tpw = dfk_cdiv(tpw, (long)TS) * TS;
  const dim3 grid((unsigned)(P * nsl));
  if (g.rowsum) hipLaunchKernelGGL((wgrad_kernel<NBR, NBC, WR, WC, true>), grid, dim3(WR * WC * 64), 0, s, g, nsl_c, nsl, tpw);
  else hipLaunchKernelGGL((wgrad_kernel<NBR, NBC, WR, WC, false>), grid, dim3(WR * WC * 64), 0, s, g, nsl_c, nsl, tpw);
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

// 1 = launched, 0 = not applicable (the caller runs the tiled GEMM), < 0 = launch error
int dfk_wgrad_try(const dfk_gemm_args& g, hipStream_t s) {
  // opt-in (DFK_WGRAD=1): faster than the tiled split-K dW in isolation on the stage-1/2 shapes, slower inside
  // the replayed step (its one-per-CU persistent workgroups with 100-123 KB of LDS wait for CUs the other branch
  // streams hold; profiles/gemm/r4o_wgrad_instep.txt)
  const char* env = getenv("DFK_WGRAD");   // read per call: tests switch it inside one process
  if (!env || atoi(env) == 0) return 0;
  if (g.dtype != DFK_BF16 || !g.a_kmajor || !g.b_kmajor || !g.c_f32) return 0;
  if (!(g.atomic || g.beta == 1.f)) return 0;   // C += product only (atomics)
  if (g.nz0 != 1 || g.nz1 != 1 || g.a.conv_cg > 0 || g.b.conv_cg > 0) return 0;
  if (g.bias || g.residual || g.act || g.drop.mode || (g.alpha != 0.f && g.alpha != 1.f)) return 0;
  if (g.K < 16384 || g.M <= 0 || g.N <= 0) return 0;
  if (g.a.ld % 8 || g.b.ld % 8 || !al16(g.a.ptr) || !al16(g.b.ptr)) return 0;
  if (((long)g.K - 1) * g.a.ld * 2 + (long)g.M * 2 >= 0x7fffffffL ||
      ((long)g.K - 1) * g.b.ld * 2 + (long)g.N * 2 >= 0x7fffffffL)
    return 0;
  // fewest HBM bytes: dy is read once per column slice, x once per row slice
  int best = -1;
  long best_cost = 0;
  for (int i = 0; i < (int)(sizeof(kShapes) / sizeof(kShapes[0])); ++i) {
    const WgShape& w = kShapes[i];
    const int NS = 16 * w.wr * w.nbr, KS = 16 * w.wc * w.nbc;
    if (g.M % NS || g.N % KS) continue;
    const long cost = (long)g.M * (g.N / KS) + (long)g.N * (g.M / NS);
    if (best < 0 || cost < best_cost) { best = i; best_cost = cost; }
  }
  if (best < 0) return 0;
  const WgShape& w = kShapes[best];
#define WG_CASE(a, b, c, d) \
  if (w.nbr == a && w.nbc == b && w.wr == c && w.wc == d) { launch_wg<a, b, c, d>(g, s); DFK_CHECK_LAUNCH(); return 1; }
  WG_CASE(3, 6, 6, 1) WG_CASE(3, 6, 8, 1) WG_CASE(3, 6, 2, 1) WG_CASE(6, 3, 1, 8) WG_CASE(3, 6, 4, 2)
  WG_CASE(6, 3, 2, 4) WG_CASE(4, 4, 3, 2) WG_CASE(4, 4, 4, 2) WG_CASE(4, 4, 2, 4) WG_CASE(4, 4, 2, 2)
#undef WG_CASE
  return 0;
}
