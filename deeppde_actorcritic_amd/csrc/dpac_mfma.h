// dpac_mfma.h — the 16x16x4 MFMA tile in f32 and f64 (gfx950), shared by the
// fused NN rollout and the row-parallel MLP kernels.
#pragma once

#include <hip/hip_runtime.h>

namespace dpac {

// A[row l&15][k l>>4], B[k l>>4][col l&15]; the accumulator's element i of
// lane l is C[row(l, i)][l&15].
template <typename T>
struct Mfma;
template <>
struct Mfma<float> {
  using acc_t = __attribute__((ext_vector_type(4))) float;
  __device__ __forceinline__ static acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static int row(int lane, int i) { return (lane >> 4) * 4 + i; }
};
template <>
struct Mfma<double> {
  using acc_t = __attribute__((ext_vector_type(4))) double;
  __device__ __forceinline__ static acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ __forceinline__ static int row(int lane, int i) { return (lane >> 4) + 4 * i; }  // f64 C map
};

}  // namespace dpac
