// Dev probe: hardware v_cos_f32 (revolutions) with and without a v_fract_f32 argument reduction, against a
// float64 cos, over the SnakeBeta argument range (|x e^alpha / pi| up to 64).  Build: hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

__global__ void k(const float* z, float* a, float* b, int n) {
  int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  a[i] = __builtin_amdgcn_cosf(__builtin_amdgcn_fractf(z[i]));
  b[i] = __builtin_amdgcn_cosf(z[i]);
}

int main() {
  const int n = 1 << 22;
  std::vector<float> z(n), a(n), b(n);
  unsigned s = 12345;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    const float u = (s >> 8) * (1.0f / 16777216.0f);
    const float mag = (i % 4 == 0) ? 4096.f : (i % 4 == 1 ? 256.f : (i % 4 == 2 ? 64.f : 1.f));
    z[i] = (2.f * u - 1.f) * mag;
  }
  float *dz, *da, *db;
  hipMalloc(&dz, n * 4); hipMalloc(&da, n * 4); hipMalloc(&db, n * 4);
  hipMemcpy(dz, z.data(), n * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dz, da, db, n);
  hipMemcpy(a.data(), da, n * 4, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), db, n * 4, hipMemcpyDeviceToHost);
  double ea[4] = {0}, eb[4] = {0}, dab = 0;
  for (int i = 0; i < n; ++i) {
    const double zr = z[i] - std::floor((double)z[i]);
    const double ref = std::cos(2.0 * M_PI * zr);
    ea[i % 4] = std::max(ea[i % 4], std::fabs(a[i] - ref));
    eb[i % 4] = std::max(eb[i % 4], std::fabs(b[i] - ref));
    dab = std::max(dab, (double)std::fabs(a[i] - b[i]));
  }
  const char* nm[4] = {"|z|<4096", "|z|<256", "|z|<64", "|z|<1"};
  for (int r = 0; r < 4; ++r) printf("%-8s max|err| fract+cos %.3e   cos alone %.3e\n", nm[r], ea[r], eb[r]);
  printf("max |fract+cos - cos| %.3e\n", dab);
  return 0;
}
