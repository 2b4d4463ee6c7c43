// Host-side checks of libdfk under AddressSanitizer (CPU only; no kernel is launched).  Exercises the C ABI's
// host code: workspace planners (GEMM split-K, attention table / backward scratch, LayerNorm slab, wav2vec2
// conv0, mel), argument validation on malformed inputs (null pointers, bad strides / shapes, unsupported head
// dims), which must return DFK_EINVAL before touching the device.  Built and run by tools/asan/run.sh.
#include <cstdio>
#include <cstring>

#include "../../include/dfk.h"

static int fails = 0;
#define EXPECT(c)                                                      \
  do {                                                                 \
    if (!(c)) { std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c); ++fails; } \
  } while (0)

int main() {
  // GEMM workspace: a small-M grid asks for split-K slabs, a large one for none
  dfk_gemm_args g;
  std::memset(&g, 0, sizeof(g));
  g.M = 1592; g.N = 3072; g.K = 768; g.dtype = DFK_BF16; g.nz0 = g.nz1 = 1; g.splitk = 1;
  g.a.ld = 768; g.b.ld = 768; g.ldc = 3072;
  const int64_t ws_small = dfk_gemm_workspace(&g);
  EXPECT(ws_small >= 0);
  g.M = 401408; g.N = 288; g.K = 96;
  EXPECT(dfk_gemm_workspace(&g) == 0);
  EXPECT(dfk_gemm_workspace(nullptr) < 0);
  // dfk_gemm rejects missing operands and contradictory epilogues before any launch
  EXPECT(dfk_gemm(&g, nullptr) != 0);                       // null A / B / C
  g.a.ptr = g.b.ptr = reinterpret_cast<void*>(0x1000); g.c = reinterpret_cast<void*>(0x2000);
  g.act = 2;                                                // dGELU without aux
  EXPECT(dfk_gemm(&g, nullptr) != 0);
  g.act = 7;
  EXPECT(dfk_gemm(&g, nullptr) != 0);
  g.act = 0; g.atomic = 1; g.c_f32 = 0;                     // atomics need an fp32 C
  EXPECT(dfk_gemm(&g, nullptr) != 0);
  // attention planners and validation
  dfk_wattn_args a;
  std::memset(&a, 0, sizeof(a));
  a.B = 8; a.D = 16; a.H = 56; a.W = 56; a.wd = 8; a.wh = 7; a.ww = 7; a.fd = 8; a.fh = 7; a.fw = 7;
  a.sd = 4; a.sh = 3; a.sw = 3; a.heads = 3; a.hd = 32; a.scale = 0.1767767f; a.dtype = DFK_BF16;
  a.ld_qkv = 288; a.ld_out = 96;
  a.q = a.k = a.v = reinterpret_cast<void*>(0x1000); a.out = reinterpret_cast<void*>(0x2000);
  EXPECT(dfk_wattn_table_workspace(&a) > 0);
  EXPECT(dfk_wattn_bwd_workspace(&a) == 0);                 // no RPB: no dRPB scratch
  a.rpb = reinterpret_cast<const float*>(0x3000);
  EXPECT(dfk_wattn_bwd_workspace(&a) > 0);
  a.rpb = nullptr;
  a.hd = 48;                                                // unsupported head dim
  EXPECT(dfk_wattn_fwd(&a, nullptr) != 0);
  a.hd = 32; a.sd = 8;                                      // shift >= window
  EXPECT(dfk_wattn_fwd(&a, nullptr) != 0);
  EXPECT(dfk_wattn_fwd(nullptr, nullptr) != 0);
  // other planners
  EXPECT(dfk_layernorm_bwd_workspace(401408, 96) > 0);
  EXPECT(dfk_layernorm_bwd_workspace(6272, 768) > 0);
  EXPECT(dfk_layernorm_bwd_workspace(0, 96) == 0);
  EXPECT(dfk_w2v_conv0_fwd_workspace(8, 64000) > 0);
  EXPECT(dfk_w2v_conv0_bwd_workspace(8, 64000) > 0);
  EXPECT(dfk_w2v_conv0_fwd_workspace(8, 5) == 0);
  EXPECT(dfk_mel_workspace(8, 88200, 2048, 512, 128) > 0);
  // validation of the other entry points
  EXPECT(dfk_layernorm_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, 10, 96, 1e-5f, DFK_BF16, nullptr,
                           nullptr, nullptr) != 0);
  EXPECT(dfk_sgd_step(nullptr, nullptr, nullptr, nullptr, 10, nullptr, 0.1f, 0.9f, 0.f, 0, nullptr, nullptr) != 0);
  EXPECT(dfk_cpb_bias_fwd(nullptr, nullptr, nullptr, nullptr, nullptr, 169, 512, 64, nullptr) != 0);
  std::printf("host_check: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
