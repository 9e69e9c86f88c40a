// Store-pattern microbenchmark for the rollout's per-step slab writes.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/wbench.hip -o tools/wbench
// Each wave owns `tpw` trajectories of `d` floats; per step it writes its
// tpw*d*4-byte piece of slab t (slab = W*tpw*d*4 bytes), optionally reading the
// same-shaped piece of an input slab first (read+write, like dw -> x).
// Lane mapping: P = 64/tpw lanes per trajectory, M = ceil(d/P) dwords per lane.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

template <int P, int M, bool RW>
__global__ __launch_bounds__(64) void k_pattern(const float* __restrict__ in, float* __restrict__ out,
                                                int d, int N, long slab) {
  const int lane = threadIdx.x, p = lane % P, g = lane / P;
  const long traj = (long)blockIdx.x * (64 / P) + g;
  float acc[M];
#pragma unroll
  for (int m = 0; m < M; ++m) acc[m] = (float)(lane + m);
  for (int t = 0; t < N; ++t) {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const int j = p * M + m;
      if (j < d) {
        const long o = t * slab + traj * d + j;
        if (RW) acc[m] = acc[m] * 0.5f + in[o];
        out[o] = acc[m];
      }
    }
  }
}

// contiguous control: the same bytes per wave-step written as plain dwords by
// all 64 lanes (no per-trajectory structure), per-step slab identical.
template <bool RW>
__global__ __launch_bounds__(64) void k_flat(const float* __restrict__ in, float* __restrict__ out,
                                             int per_wave, int N, long slab) {
  float a = threadIdx.x;
  for (int t = 0; t < N; ++t)
    for (int i = threadIdx.x; i < per_wave; i += 64) {
      const long o = t * slab + (long)blockIdx.x * per_wave + i;
      if (RW) a = a * 0.5f + in[o];
      out[o] = a;
    }
}

template <class F>
float time_it(F launch, int reps) {
  hipEvent_t s, e;
  CK(hipEventCreate(&s)); CK(hipEventCreate(&e));
  for (int i = 0; i < 3; ++i) launch();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(s));
  for (int i = 0; i < reps; ++i) launch();
  CK(hipEventRecord(e));
  CK(hipEventSynchronize(e));
  float ms; CK(hipEventElapsedTime(&ms, s, e));
  return ms / reps;
}

int main(int argc, char** argv) {
  const int d = 20, N = 200;
  std::vector<long> Bs = {4096, 16384};
  for (long B : Bs) {
    const long slab = B * d;
    float *in, *out;
    CK(hipMalloc(&in, slab * N * 4)); CK(hipMalloc(&out, slab * N * 4));
    CK(hipMemset(in, 0, slab * N * 4));
    const double bytes_w = (double)slab * N * 4;
    auto report = [&](const char* name, bool rw, float ms) {
      const double by = bytes_w * (rw ? 2 : 1);
      printf("{\"B\": %ld, \"pattern\": \"%s\", \"rw\": %d, \"us\": %.2f, \"GBps\": %.0f}\n", B, name,
             (int)rw, ms * 1e3, by / ms / 1e6);
    };
#define RUNP(P, M, RW, NAME)                                                               \
    report(NAME, RW, time_it([&] { hipLaunchKernelGGL((k_pattern<P, M, RW>),              \
        dim3(B / (64 / P)), dim3(64), 0, 0, in, out, d, N, slab); }, 50));
    RUNP(16, 2, false, "P16_M2");
    RUNP(8, 3, false, "P8_M3");
    RUNP(4, 5, false, "P4_M5");
    RUNP(32, 1, false, "P32_M1");
    RUNP(16, 2, true, "P16_M2");
    RUNP(8, 3, true, "P8_M3");
    RUNP(4, 5, true, "P4_M5");
#define RUNF(TPW, RW, NAME)                                                                \
    report(NAME, RW, time_it([&] { hipLaunchKernelGGL((k_flat<RW>), dim3(B / TPW), dim3(64), \
        0, 0, in, out, TPW * d, N, slab); }, 50));
    RUNF(4, false, "flat_320B");
    RUNF(16, false, "flat_1280B");
    RUNF(4, true, "flat_320B");
    RUNF(16, true, "flat_1280B");
    CK(hipFree(in)); CK(hipFree(out));
  }
  return 0;
}
