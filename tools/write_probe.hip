// Write-heavy HBM probe: the stage-1 GELU Linear's traffic (read X [M, 96] bf16, write two [M, 384] bf16
// outputs) under different store patterns, to find what bounds wres_kernel's write-heavy launches.
//   hipcc --offload-arch=gfx950 -O3 -o write_probe tools/write_probe.hip && ./write_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr long M = 401408;
constexpr int K = 96, N = 384;

// v0: grid-stride, one 16-B output chunk per thread per output, rows contiguous (ideal pattern)
__global__ void v_flat(const uint4* __restrict__ x, uint4* __restrict__ o1, uint4* __restrict__ o2, long chunks) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < chunks; i += (long)gridDim.x * blockDim.x) {
    const long row = i / (N / 8);
    uint4 v = x[row * (K / 8) + (i % (K / 8))];
    v.x += (uint32_t)i;
    o1[i] = v;
    v.y += 1;
    o2[i] = v;
  }
}

// v1: wres-like: persistent grid of 256 x 512 threads (or blocks_per_cu x 256), 2 column slices of 192 channels,
// wave = 16 rows x 96 channels, staged through LDS and stored as 16-B chunks (CPR = 12 per row)
template <int NT>
__global__ __launch_bounds__(NT) void v_wres(const uint4* __restrict__ x, uint16_t* __restrict__ o1,
                                             uint16_t* __restrict__ o2, int nslices, int ntiles, int nt_store) {
  constexpr int NSPLIT = 2, ROWS_T = 16 * (NT / 64 / NSPLIT);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, rg = wave / NSPLIT, cg = wave % NSPLIT;
  const int slice = blockIdx.x % nslices, stride = gridDim.x / nslices;
  const int c0 = slice * 192 + cg * 96;
  __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(o1, 0, 0x7fffffff, 0x00020000);
  __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(o2, 0, 0x7fffffff, 0x00020000);
  for (int t = blockIdx.x / nslices; t < ntiles; t += stride) {
    const long mt0 = (long)t * ROWS_T + rg * 16;
    const uint4 a = x[(mt0 + (lane & 15)) * (K / 8) + (lane >> 4)];
#pragma unroll
    for (int c = lane; c < 16 * 12; c += 64) {
      const int r = c / 12, ch = (c % 12) * 8;
      const long e = (mt0 + r) * N + c0 + ch;
      uint4 v = a;
      v.x += (uint32_t)e;
      if (nt_store) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r1, (uint32_t)(e * 2), 0, 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r2, (uint32_t)(e * 2), 0, 2);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r1, (uint32_t)(e * 2), 0, 0);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r2, (uint32_t)(e * 2), 0, 0);
      }
    }
  }
}

// v2: as v1 but each wave writes whole rows (16 rows x 384 channels: one slice, 8 waves x 16 rows per tile)
template <int NT>
__global__ __launch_bounds__(NT) void v_rows(const uint4* __restrict__ x, uint16_t* __restrict__ o1,
                                             uint16_t* __restrict__ o2, int ntiles) {
  constexpr int ROWS_T = 16 * (NT / 64);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __amdgpu_buffer_rsrc_t r1 = __builtin_amdgcn_make_buffer_rsrc(o1, 0, 0x7fffffff, 0x00020000);
  __amdgpu_buffer_rsrc_t r2 = __builtin_amdgcn_make_buffer_rsrc(o2, 0, 0x7fffffff, 0x00020000);
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const long mt0 = (long)t * ROWS_T + wave * 16;
    const uint4 a = x[(mt0 + (lane & 15)) * (K / 8) + (lane >> 4)];
#pragma unroll
    for (int c = lane; c < 16 * 48; c += 64) {
      const long e = mt0 * N + c * 8;
      uint4 v = a;
      v.x += (uint32_t)e;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r1, (uint32_t)(e * 2), 0, 0);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r2, (uint32_t)(e * 2), 0, 0);
    }
  }
}

template <typename F>
float timeit(F f) {
  hipEvent_t s, e;
  (void)hipEventCreate(&s); (void)hipEventCreate(&e);
  f();
  hipDeviceSynchronize();
  hipEventRecord(s);
  for (int i = 0; i < 20; ++i) f();
  hipEventRecord(e);
  hipEventSynchronize(e);
  float ms;
  hipEventElapsedTime(&ms, s, e);
  return ms / 20;
}

int main() {
  uint4 *x, *o1, *o2;
  CK(hipMalloc(&x, M * K * 2));
  CK(hipMalloc(&o1, M * N * 2));
  CK(hipMalloc(&o2, M * N * 2));
  CK(hipMemset(x, 0, M * K * 2));
  const double bytes = M * K * 2.0 + 2.0 * M * N * 2;
  auto rep = [&](const char* name, float ms) { printf("%-44s %8.1f us  %5.2f TB/s\n", name, ms * 1e3, bytes / ms / 1e9); };
  const long chunks = M * N / 8;
  rep("flat grid-stride (4096 x 256)", timeit([&] { hipLaunchKernelGGL(v_flat, dim3(4096), dim3(256), 0, 0, x, o1, o2, chunks); }));
  rep("flat one chunk per thread", timeit([&] { hipLaunchKernelGGL(v_flat, dim3(chunks / 256), dim3(256), 0, 0, x, o1, o2, chunks); }));
  const int nt512 = (int)(M / 64);
  for (int per : {1, 2, 4}) {
    char nm[96];
    snprintf(nm, sizeof nm, "wres-like 512 thr, %d WG/CU", per);
    rep(nm, timeit([&] { hipLaunchKernelGGL(v_wres<512>, dim3(256 * per * 2 / 2), dim3(512), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, 2, nt512, 0); }));
  }
  rep("wres-like 512 thr, 1 WG/CU, nt stores", timeit([&] { hipLaunchKernelGGL(v_wres<512>, dim3(256), dim3(512), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, 2, nt512, 1); }));
  rep("wres-like 256 thr, 2 WG/CU", timeit([&] { hipLaunchKernelGGL(v_wres<256>, dim3(512), dim3(256), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, 2, (int)(M / 32), 0); }));
  rep("whole rows 512 thr, 1 WG/CU", timeit([&] { hipLaunchKernelGGL(v_rows<512>, dim3(256), dim3(512), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, (int)(M / 128)); }));
  rep("whole rows 512 thr, 2 WG/CU", timeit([&] { hipLaunchKernelGGL(v_rows<512>, dim3(512), dim3(512), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, (int)(M / 128)); }));
  rep("whole rows 512 thr, non-persistent", timeit([&] { hipLaunchKernelGGL(v_rows<512>, dim3(M / 128), dim3(512), 0, 0, x, (uint16_t*)o1, (uint16_t*)o2, (int)(M / 128)); }));
  CK(hipDeviceSynchronize());
  return 0;
}
