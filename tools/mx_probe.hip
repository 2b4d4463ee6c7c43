// Hardware probe of the gfx950 block-scaled MFMA (v_mfma_scale_f32_16x16x128_f8f6f4 / 32x32x64) operand
// and scale lane maps, and of the e4m3 conversion instruction.  Structured experiments (one-hot lanes, coded
// byte values, one doubled scale at a time); tools/mx_probe.py decodes the maps from the raw outputs.
//   hipcc -O2 --offload-arch=gfx950 tools/mx_probe.hip -o tools/mx_probe && ./tools/mx_probe out.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef float v16f __attribute__((ext_vector_type(16)));

// one experiment per workgroup: A/B [exp][64 lanes][32 bytes], scales [exp][64], D [exp][64][16]
// C comes from memory (zeros) so the accumulator registers are distinct from the A/B operands
__global__ void mma16(const uint8_t* A, const uint8_t* B, const uint32_t* sa, const uint32_t* sb, const float* C0,
                      float* D) {
  const int l = threadIdx.x, e = blockIdx.x;
  v8i a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = *reinterpret_cast<const int*>(A + (e * 64 + l) * 32 + 4 * i);
    b[i] = *reinterpret_cast<const int*>(B + (e * 64 + l) * 32 + 4 * i);
  }
  v4f c;
  for (int i = 0; i < 4; ++i) c[i] = C0[(e * 64 + l) * 16 + i];
  // a loop-carried accumulator (the GEMM form: dst tied to srcC); two passes -> 2x the product
#pragma unroll 1
  for (int it = 0; it < 2; ++it)
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, (int)sa[e * 64 + l], 0, (int)sb[e * 64 + l]);
  for (int i = 0; i < 4; ++i) D[(e * 64 + l) * 16 + i] = 0.5f * c[i];
}

__global__ void mma32(const uint8_t* A, const uint8_t* B, const uint32_t* sa, const uint32_t* sb, const float* C0,
                      float* D) {
  const int l = threadIdx.x, e = blockIdx.x;
  v8i a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = *reinterpret_cast<const int*>(A + (e * 64 + l) * 32 + 4 * i);
    b[i] = *reinterpret_cast<const int*>(B + (e * 64 + l) * 32 + 4 * i);
  }
  v16f c;
  for (int i = 0; i < 16; ++i) c[i] = C0[(e * 64 + l) * 16 + i];
#pragma unroll 1
  for (int it = 0; it < 2; ++it)
    c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 0, 0, 0, (int)sa[e * 64 + l], 0, (int)sb[e * 64 + l]);
  for (int i = 0; i < 16; ++i) D[(e * 64 + l) * 16 + i] = 0.5f * c[i];
}

// two floats -> two e4m3 bytes (low half of the result word)
__global__ void cvt(const float* x, uint8_t* y, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 >= n) return;
  const int r = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
  y[2 * i] = (uint8_t)(r & 0xff);
  y[2 * i + 1] = (uint8_t)((r >> 8) & 0xff);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static const uint8_t ONE = 0x38;   // e4m3 1.0

int main(int argc, char** argv) {
  const char* path = argc > 1 ? argv[1] : "mx_probe.bin";
  FILE* f = fopen(path, "wb");
  if (!f) return 1;
  srand(1234);
  // experiments (the same list for both shapes):
  //   [0, 64)    A lane L all ones, B all ones                      -> A lane -> rows
  //   [64, 128)  B lane L all ones, A all ones                      -> B lane -> cols
  //   [128, 256) A, B all ones, A lane L scale 120 / 134            -> scale values below / above 1
  //   [256, 320) A, B all ones, A lane L scale 128 (2x)             -> A scale lane map
  //   [320, 384) A, B all ones, B lane L scale 128                  -> B scale lane map
  //   [384, 386) random small integers, random A scales / random B scales -> end-to-end check
  const int NE = 386;
  std::vector<uint8_t> A(NE * 2048, 0), B(NE * 2048, 0);
  std::vector<uint32_t> sa(NE * 64, 127), sb(NE * 64, 127);
  for (int L = 0; L < 64; ++L) {
    for (int j = 0; j < 32; ++j) A[L * 2048 + L * 32 + j] = ONE;
    for (int i = 0; i < 2048; ++i) B[L * 2048 + i] = ONE;
    for (int j = 0; j < 32; ++j) B[(64 + L) * 2048 + L * 32 + j] = ONE;
    for (int i = 0; i < 2048; ++i) A[(64 + L) * 2048 + i] = ONE;
  }
  for (int t = 0; t < 128; ++t) {   // A, B ones; one A lane scaled 2^-7 ([128,192)) or 2^7 ([192,256))
    const int e = 128 + t, L = t % 64;
    for (int i = 0; i < 2048; ++i) { A[e * 2048 + i] = ONE; B[e * 2048 + i] = ONE; }
    sa[e * 64 + L] = t < 64 ? 120 : 134;
  }
  for (int L = 0; L < 64; ++L) {
    for (int i = 0; i < 2048; ++i) { A[(256 + L) * 2048 + i] = ONE; B[(256 + L) * 2048 + i] = ONE; }
    sa[(256 + L) * 64 + L] = 128;
    for (int i = 0; i < 2048; ++i) { A[(320 + L) * 2048 + i] = ONE; B[(320 + L) * 2048 + i] = ONE; }
    sb[(320 + L) * 64 + L] = 128;
  }
  static const uint8_t pos[5] = {0x00, 0x38, 0x40, 0x44, 0x48};
  for (int e = 384; e < 386; ++e)
    for (int i = 0; i < 2048; ++i) {
      int va = rand() % 9 - 4, vb = rand() % 9 - 4;
      A[e * 2048 + i] = pos[abs(va)] | (va < 0 ? 0x80 : 0);
      B[e * 2048 + i] = pos[abs(vb)] | (vb < 0 ? 0x80 : 0);
    }
  for (int l = 0; l < 64; ++l) sa[384 * 64 + l] = 120 + rand() % 15;   // A scales only
  for (int l = 0; l < 64; ++l) sb[385 * 64 + l] = 120 + rand() % 15;   // B scales only

  uint8_t *dA, *dB;
  uint32_t *dsa, *dsb;
  float *dC, *dD;
  CK(hipMalloc(&dA, A.size())); CK(hipMalloc(&dB, B.size()));
  CK(hipMalloc(&dsa, sa.size() * 4)); CK(hipMalloc(&dsb, sb.size() * 4));
  CK(hipMalloc(&dC, NE * 64 * 16 * 4)); CK(hipMalloc(&dD, NE * 64 * 16 * 4));
  CK(hipMemcpy(dA, A.data(), A.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dB, B.data(), B.size(), hipMemcpyHostToDevice));
  CK(hipMemcpy(dsa, sa.data(), sa.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dsb, sb.data(), sb.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemset(dC, 0, NE * 64 * 16 * 4));
  fwrite(A.data(), 1, A.size(), f); fwrite(B.data(), 1, B.size(), f);
  fwrite(sa.data(), 4, sa.size(), f); fwrite(sb.data(), 4, sb.size(), f);
  std::vector<float> D(NE * 64 * 16);
  for (int shape = 0; shape < 2; ++shape) {
    CK(hipMemset(dD, 0, NE * 64 * 16 * 4));
    if (shape == 0) hipLaunchKernelGGL(mma16, dim3(NE), dim3(64), 0, 0, dA, dB, dsa, dsb, dC, dD);
    else hipLaunchKernelGGL(mma32, dim3(NE), dim3(64), 0, 0, dA, dB, dsa, dsb, dC, dD);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(D.data(), dD, D.size() * 4, hipMemcpyDeviceToHost));
    fwrite(D.data(), 4, D.size(), f);
  }
  // conversion sweep
  const int n = 1 << 16;
  std::vector<float> x(n);
  for (int i = 0; i < n; ++i) {
    const uint32_t r = (uint32_t)rand() * 2654435761u ^ (uint32_t)rand();
    const int e = (int)(r % 40) - 14;
    const float m = 1.0f + (float)((r >> 8) & 0xffff) / 65536.0f;
    x[i] = ldexpf(m, e) * ((r >> 30) & 1 ? -1.f : 1.f);
  }
  float* dx;
  uint8_t* dy;
  CK(hipMalloc(&dx, n * 4)); CK(hipMalloc(&dy, n));
  CK(hipMemcpy(dx, x.data(), n * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(cvt, dim3(n / 512), dim3(256), 0, 0, dx, dy, n);
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> y(n);
  CK(hipMemcpy(y.data(), dy, n, hipMemcpyDeviceToHost));
  fwrite(x.data(), 4, n, f);
  fwrite(y.data(), 1, n, f);
  fclose(f);
  printf("mx_probe: wrote %s\n", path);
  return 0;
}
