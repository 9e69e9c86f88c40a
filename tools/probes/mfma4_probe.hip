// Layout probe for v_mfma_f32_4x4x1_16b_f32 on gfx950: A[lane] = 1000 + lane,
// B[lane] = lane, C = 0; prints, for every lane and accumulator slot, which
// (A lane, B lane) pair(s) the product came from (a single product per slot).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float v4f __attribute__((ext_vector_type(4)));
__global__ void k(float* out, int mode) {
  const int l = threadIdx.x;
  float a = mode == 0 ? (l == 5 ? 1.f : 0.f) : 1.f;      // mode 0: only A lane 5 nonzero
  float b = mode == 0 ? 1.f : (l == 9 ? 1.f : 0.f);      // mode 1: only B lane 9 nonzero
  v4f c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
  for (int i = 0; i < 4; ++i) out[l * 4 + i] = c[i];
}
int main() {
  float* d; hipMalloc(&d, 256 * 4);
  float h[256];
  for (int mode = 0; mode < 2; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, mode);
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    printf("mode %d (%s lane %d set): nonzero outputs (lane, slot):", mode, mode ? "B" : "A", mode ? 9 : 5);
    for (int i = 0; i < 256; ++i) if (h[i] != 0) printf(" (%d,%d)", i / 4, i % 4);
    printf("\n");
  }
  return 0;
}
