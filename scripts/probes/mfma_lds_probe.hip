// Dev probe: 16x16x32 f16 MFMA loop of the wide-conv wave tile (64 x 96 per wave, 24 MFMAs per 32-deep slice, 8
// waves per CU) with its fragments read from LDS in different ways, to separate the MFMA rate from the cost of the
// fragment reads and of a per-step barrier.  Build: hipcc -O3 --offload-arch=gfx950 mfma_lds_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

typedef __attribute__((address_space(3))) void lds_void_t;
typedef __attribute__((address_space(1))) void gbl_void_t;

// V >= 3: + three 1-KB LDS-DMA instructions per wave per step into the weight slot two steps ahead, counted vmcnt
// wait (V = 3: source 64 KB, L2-resident; V = 4: a 256 MB stream)
template <int V>
__global__ __launch_bounds__(512, 1) void probe(float* out, int steps, const char* src, long src_bytes) {
  constexpr int TM = 4, TN = 6;
  __shared__ __attribute__((aligned(1024))) char smem[155648];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < 155648 / 4; i += 512) reinterpret_cast<float*>(smem)[i] = (float)(i % 7) * 1e-3f;
  __syncthreads();
  const int wm = wave >> 1, wn = wave & 1;
  const int arow0 = wm * 64 + (lane & 15), nrow0 = wn * 96 + (lane & 15);
  auto rdA = [&](int tap, int sub, int i) -> f16x8 {
    const int arow = arow0 + tap;
    return *reinterpret_cast<const f16x8*>(smem + arow * 128 + (((4 * sub + (lane >> 4)) ^ (arow & 7)) << 4) +
                                           i * 16 * 128);
  };
  auto rdB = [&](int sl, int sub, int j) -> f16x8 {
    return *reinterpret_cast<const f16x8*>(smem + 81920 + sl * 24576 + nrow0 * 128 +
                                           (((4 * sub + (lane >> 4)) ^ (lane & 7)) << 4) + j * 16 * 128);
  };
  f32x4 acc[TM][TN];
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  f16x8 aA[TM], aB[TM], bA[TN], bB[TN];
  for (int i = 0; i < TM; ++i) aA[i] = aB[i] = rdA(0, 0, i);
  for (int j = 0; j < TN; ++j) bA[j] = bB[j] = rdB(0, 0, j);
  for (int g = 0; g < steps; ++g) {
    const int tap = g % 11, sl = g % 3;
    // slice 0
    __builtin_amdgcn_s_setprio(1);
    for (int i = 0; i < TM; ++i) {
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aA[i], bA[j], acc[i][j], 0, 0, 0);
      if (V >= 1 && i == 0) {
        for (int j = 0; j < TN; ++j) bB[j] = rdB(sl, 1, j);
        for (int ii = 0; ii < TM; ++ii) aB[ii] = rdA(tap, 1, ii);
      }
    }
    if (V >= 1) {
      __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, TN + TM, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, (TM - 1) * TN, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    if (V >= 5) {
      // + the conv's window stream: every 11th step five 1-KB DMA instructions per wave from the 256 MB buffer
      // into the other window buffer (here: the upper 40 KB of the A region), waited on with the weights
      if (tap == 10) __builtin_amdgcn_s_waitcnt((8) | (7 << 4));
      else __builtin_amdgcn_s_waitcnt((3) | (7 << 4));
      __builtin_amdgcn_s_barrier();
      if (tap == 0) {
        const long wb = ((long)blockIdx.x * 40960 * 31 + (long)g * 40960) % (src_bytes - 40960);
        for (int j = 0; j < 5; ++j)
          __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + wb + (wave + 8 * j) * 1024 + lane * 16),
                                           (lds_void_t*)(smem + 40960 + (wave + 8 * j) * 1024), 16, 0, 0);
      }
      const long base = ((long)g * 24576) % 65536;
      for (int j = 0; j < 3; ++j)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + base + (wave + 8 * j) * 1024 + lane * 16),
                                         (lds_void_t*)(smem + 81920 + sl * 24576 + (wave + 8 * j) * 1024), 16, 0, 0);
    } else if (V >= 3) {
      __builtin_amdgcn_s_waitcnt((3) | (7 << 4));  // vmcnt(3) lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
      const long base = (V == 3 ? ((long)g * 24576) % 65536 : ((long)blockIdx.x * 24576 * 97 + (long)g * 24576) % (src_bytes - 24576));
      for (int j = 0; j < 3; ++j)
        __builtin_amdgcn_global_load_lds((gbl_void_t*)(src + base + (wave + 8 * j) * 1024 + lane * 16),
                                         (lds_void_t*)(smem + 81920 + sl * 24576 + (wave + 8 * j) * 1024), 16, 0, 0);
    } else if (V >= 2) {
      __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (3 << 14) | (15));  // lgkmcnt(0)
      __builtin_amdgcn_s_barrier();
    }
    // slice 1
    __builtin_amdgcn_s_setprio(1);
    for (int i = 0; i < TM; ++i) {
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aB[i], bB[j], acc[i][j], 0, 0, 0);
      if (V >= 1 && i == 0) {
        for (int j = 0; j < TN; ++j) bA[j] = rdB((sl + 1) % 3, 0, j);
        for (int ii = 0; ii < TM; ++ii) aA[ii] = rdA(tap + 1, 0, ii);
      }
    }
    if (V >= 1) {
      __builtin_amdgcn_sched_group_barrier(0x8, TN, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, TN + TM, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, (TM - 1) * TN, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  }
  float s = 0.f;
  for (int i = 0; i < TM; ++i)
    for (int j = 0; j < TN; ++j) s += acc[i][j][0] + acc[i][j][3];
  out[blockIdx.x * 512 + tid] = s;
}

template <int V>
void run(float* out, int grid, int steps, const char* name, const char* src, long nb) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(512), 0, 0, out, steps, src, nb);
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(probe<V>, dim3(grid), dim3(512), 0, 0, out, steps, src, nb);
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  const double flops = 2.0 * 256 * 192 * 64 * (double)steps * grid;
  printf("%-44s %8.3f ms  %7.1f TF/s\n", name, ms, flops / ms / 1e9);
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 512 * 4 * 4);
  const int steps = 660;
  const long nb = 256l << 20;
  char* src;
  (void)hipMalloc(&src, nb);
  (void)hipMemset(src, 0, nb);
  for (int rep = 0; rep < 2; ++rep) {
    run<0>(out, 256, steps, "V0 MFMA only (fragments in registers)", src, nb);
    run<1>(out, 256, steps, "V1 + fragment reads one slice ahead", src, nb);
    run<2>(out, 256, steps, "V2 + lgkmcnt(0) + barrier per step", src, nb);
    run<3>(out, 256, steps, "V3 + 24 KB DMA per step (L2-resident)", src, nb);
    run<4>(out, 256, steps, "V4 + 24 KB DMA per step (streamed)", src, nb);
    run<5>(out, 256, steps, "V5 V3 + 40 KB streamed window per 11 steps", src, nb);
  }
  return 0;
}
