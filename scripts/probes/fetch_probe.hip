// Dev probe: calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 against KNOWN byte counts, per access
// form, so the HBM-traffic figures in profiles/*/SUMMARY.md can be corrected per kernel instead of by one 2x
// factor (MI355X_MICROARCH.md calibrates the 2x only for 16-B/lane streaming reads).  Each kernel reads (or
// writes) exactly BYTES of a buffer far larger than the 256 MB Infinity Cache, once, then the host prints the
// bytes each kernel moved; the counters come from separate `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
// runs (scripts/fetch_calib.sh).  Build: hipcc -O3 --offload-arch=gfx950 fetch_probe.hip -o fetch_probe
//   rd4 / rd8 / rd16      coalesced streaming reads of 4 / 8 / 16 B per lane (consecutive lanes, consecutive bytes)
//   rd16_rows192          16 B per lane from rows 192 B apart (channels-last fp32 rows of 48 channels: the narrow
//                         BigVGAN tail / upsampler access form); every byte of every row is read once overall
//   rd4_col               4 B per lane, 16 lanes of consecutive columns per row, 4 rows per instruction (the MFMA
//                         C-fragment layout of the wide-conv epilogue's residual / accumulate loads)
//   lds16                 global_load_lds_dwordx4 (LDS-DMA) streaming, 16 B per lane
//   wr4 / wr16            coalesced streaming writes of 4 / 16 B per lane
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr size_t BYTES = size_t(1) << 30;  // 1 GiB per kernel

__global__ __launch_bounds__(256) void rd4(const float* __restrict__ p, float* out) {
  const size_t n = BYTES / 4;
  float s = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i];
  if (s == 1.2345f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void rd8(const float2* __restrict__ p, float* out) {
  const size_t n = BYTES / 8;
  float s = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += p[i].x + p[i].y;
  if (s == 1.2345f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void rd16(const float4* __restrict__ p, float* out) {
  const size_t n = BYTES / 16;
  float s = 0.f;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float4 v = p[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 1.2345f) out[threadIdx.x] = s;
}
// rows of 192 B (12 float4); lane l of a wave reads piece k of row (wave row base + l): over k = 0..11 every byte
__global__ __launch_bounds__(256) void rd16_rows192(const float4* __restrict__ p, float* out) {
  const size_t rows = BYTES / 192;
  float s = 0.f;
  for (size_t r = blockIdx.x * 256ull + threadIdx.x; r < rows; r += (size_t)gridDim.x * 256)
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const float4 v = p[r * 12 + k];
      s += v.x + v.y + v.z + v.w;
    }
  if (s == 1.2345f) out[threadIdx.x] = s;
}
// a 64 x 96-column fp32 tile per wave as the 16x16 MFMA C layout: lane (l & 15) = column, (l >> 4) * 4 + r = row
__global__ __launch_bounds__(256) void rd4_col(const float* __restrict__ p, float* out) {
  constexpr int N = 768;  // row length in floats (the C = 768 stage-0 layer)
  const size_t rows = BYTES / (N * 4);
  const int lane = threadIdx.x & 63;
  const size_t nt = (rows / 64) * (N / 96);
  float s = 0.f;
  for (size_t t = blockIdx.x * 4ull + (threadIdx.x >> 6); t < nt; t += (size_t)gridDim.x * 4) {
    const size_t r0 = (t / (N / 96)) * 64, c0 = (t % (N / 96)) * 96;
#pragma unroll 4
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int j = 0; j < 6; ++j)
          s += p[(r0 + i * 16 + (lane >> 4) * 4 + r) * N + c0 + j * 16 + (lane & 15)];
  }
  if (s == 1.2345f) out[threadIdx.x] = s;
}
__global__ __launch_bounds__(256) void lds16(const float4* __restrict__ p, float* out) {
  __shared__ float4 buf[4][64];
  const size_t n = BYTES / 16;
  const int w = threadIdx.x >> 6;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)(p + i),
                                     (__attribute__((address_space(3))) void*)(&buf[w][0]), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  const float4 v = buf[w][threadIdx.x & 63];
  if (v.x == 1.2345f) out[threadIdx.x] = v.y;
}
__global__ __launch_bounds__(256) void wr4(float* __restrict__ p) {
  const size_t n = BYTES / 4;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = 1.f;
}
__global__ __launch_bounds__(256) void wr16(float4* __restrict__ p) {
  const size_t n = BYTES / 16;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    p[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

int main() {
  float *a = nullptr, *out = nullptr;
  if (hipMalloc(&a, BYTES) != hipSuccess || hipMalloc(&out, 4096) != hipSuccess) return 1;
  hipMemset(a, 0, BYTES);
  hipDeviceSynchronize();
  const dim3 g(4096), b(256);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](const char* name, auto launch, size_t bytes = BYTES) {
    hipEventRecord(e0, 0);
    launch();
    hipEventRecord(e1, 0);
    hipEventSynchronize(e1);
    float ms = 0.f;
    hipEventElapsedTime(&ms, e0, e1);
    std::printf("%-14s bytes %zu  %.3f ms  %.1f GB/s\n", name, bytes, ms, bytes / (ms * 1e-3) / 1e9);
  };
  run("rd4", [&] { hipLaunchKernelGGL(rd4, g, b, 0, 0, a, out); });
  run("rd8", [&] { hipLaunchKernelGGL(rd8, g, b, 0, 0, (const float2*)a, out); });
  run("rd16", [&] { hipLaunchKernelGGL(rd16, g, b, 0, 0, (const float4*)a, out); });
  run("rd16_rows192", [&] { hipLaunchKernelGGL(rd16_rows192, g, b, 0, 0, (const float4*)a, out); });
  run("rd4_col", [&] { hipLaunchKernelGGL(rd4_col, g, b, 0, 0, a, out); }, BYTES / (768 * 4) / 64 * 64 * 768 * 4);
  run("lds16", [&] { hipLaunchKernelGGL(lds16, g, b, 0, 0, (const float4*)a, out); });
  run("wr4", [&] { hipLaunchKernelGGL(wr4, g, b, 0, 0, a); });
  run("wr16", [&] { hipLaunchKernelGGL(wr16, g, b, 0, 0, (float4*)a); });
  const hipError_t e = hipDeviceSynchronize();
  std::printf("status %s\n", hipGetErrorString(e));
  hipFree(a);
  hipFree(out);
  return e == hipSuccess ? 0 : 2;
}
