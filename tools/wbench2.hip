// Rollout memory-shape microbenchmark: per-step narrow loads/stores (step-major
// [N][B][d] slabs, the current k_rollout) against chunked wide transfers
// (trajectory-major [B][N][d] rows, 16 steps staged in LDS, dwordx4 by all 64
// lanes), both around the same dependent per-step chain (packed update, 4-level
// DPP sum, two sqrt).  Timing only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/wbench2.hip -o tools/wbench2
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int D = 20, P = 16, M = 2, G = 64 / P;

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL,
                                                                0xF, 0xF, true));
}
__device__ __forceinline__ float gsum(float v) {
  v += dpp<0xB1>(v);
  v += dpp<0x4E>(v);
  v += dpp<0x141>(v);
  v += dpp<0x140>(v);
  return v;
}
__device__ __forceinline__ void chain(float (&x)[M], const float (&w)[M], float& r) {
  const float dt = fmaxf((1.0f - r) * (1.0f - r) * 0.3f, 1e-4f);
  const float sq = __builtin_amdgcn_sqrtf(dt);
  float q = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    x[m] = x[m] * (1.0f - 0.1f * dt) + sq * w[m] * 0.05f;
    q = fmaf(x[m], x[m], q);
  }
  const float rn = __builtin_amdgcn_sqrtf(gsum(q));
  const bool in = rn < 1.0f;
#pragma unroll
  for (int m = 0; m < M; ++m) x[m] = in ? x[m] : x[m] * 0.5f;
  r = in ? rn : r * 0.5f;
}

// ---- A: per-step narrow access, step-major slabs, KB-deep register prefetch ----
template <int KB>
__global__ __launch_bounds__(64) void k_step(const float* __restrict__ dw, float* __restrict__ x,
                                             int B, int N) {
  const int lane = threadIdx.x, p = lane % P, g = lane / P;
  const long b = (long)blockIdx.x * G + g;
  const bool act = p * M < D;
  const long stride = (long)B * D;
  float xs[M] = {0.01f * p, 0.02f}, r = 0.1f;
  float ring[KB][M];
#pragma unroll
  for (int k = 0; k < KB; ++k)
#pragma unroll
    for (int m = 0; m < M; ++m) ring[k][m] = act ? dw[k * stride + b * D + p * M + m] : 0.f;
  for (int t0 = 0; t0 < N; t0 += KB) {
#pragma unroll
    for (int k = 0; k < KB; ++k) {
      const int t = t0 + k;
      float w[M];
#pragma unroll
      for (int m = 0; m < M; ++m) w[m] = ring[k][m];
      const int tn = min(t + KB, N - 1);
#pragma unroll
      for (int m = 0; m < M; ++m) ring[k][m] = act ? dw[tn * stride + b * D + p * M + m] : 0.f;
      chain(xs, w, r);
      if (act) {
#pragma unroll
        for (int m = 0; m < M; ++m) x[(t + 1) * stride + b * D + p * M + m] = xs[m];
      }
    }
  }
}

// ---- B: chunked wide access, trajectory-major rows, S steps staged in LDS ----
template <int S>
__global__ __launch_bounds__(64) void k_chunk(const float* __restrict__ dw, float* __restrict__ x,
                                              int B, int N) {
  constexpr int ROWF = S * D;             // floats per trajectory per chunk
  constexpr int PIECES = G * ROWF / 4;    // float4 pieces per wave-chunk
  constexpr int NI = (PIECES + 63) / 64;  // wide instructions per chunk
  __shared__ float4 lds_w[2][G * ROWF / 4];
  __shared__ float4 lds_x[G * ROWF / 4];
  const int lane = threadIdx.x, p = lane % P, g = lane / P;
  const long b0 = (long)blockIdx.x * G;
  const bool act = p * M < D;
  float xs[M] = {0.01f * p, 0.02f}, r = 0.1f;
  float4 pre[NI];
  auto gload = [&](int t0, float4 (&dst)[NI]) {
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = lane + 64 * k;
      const int gg = i / (ROWF / 4), w = i % (ROWF / 4);
      const long off = (b0 + gg) * (long)N * D + (long)t0 * D + w * 4;
      dst[k] = i < PIECES ? *(const float4*)(dw + off) : float4{};
    }
  };
  auto lput = [&](int buf, const float4 (&src)[NI]) {
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = lane + 64 * k;
      if (i < PIECES) lds_w[buf][i] = src[k];
    }
  };
  gload(0, pre);
  lput(0, pre);
  int buf = 0;
  for (int t0 = 0; t0 < N; t0 += S) {
    if (t0 + S < N) gload(t0 + S, pre);
    const float* wrow = (const float*)lds_w[buf] + g * ROWF;
    float* xrow = (float*)lds_x + g * ROWF;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      float w[M];
#pragma unroll
      for (int m = 0; m < M; ++m) w[m] = act ? wrow[s * D + p * M + m] : 0.f;
      chain(xs, w, r);
      if (act) {
#pragma unroll
        for (int m = 0; m < M; ++m) xrow[s * D + p * M + m] = xs[m];
      }
    }
#pragma unroll
    for (int k = 0; k < NI; ++k) {
      const int i = lane + 64 * k;
      const int gg = i / (ROWF / 4), w = i % (ROWF / 4);
      const long off = (b0 + gg) * (long)(N + 1) * D + (long)(t0 + 1) * D + w * 4;
      if (i < PIECES) *(float4*)(x + off) = lds_x[i];
    }
    if (t0 + S < N) lput(buf ^ 1, pre);
    buf ^= 1;
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

int main() {
  const int N = 208;  // multiple of 16 for the chunked variant
  for (int B : {4096, 16384}) {
    float *dw, *x;
    const size_t nb = (size_t)B * (N + 1) * D * 4;
    CK(hipMalloc(&dw, nb)); CK(hipMalloc(&x, nb));
    CK(hipMemset(dw, 0, nb)); CK(hipMemset(x, 0, nb));
    const double by = 2.0 * B * N * D * 4;
    auto rep = [&](const char* name, float ms) {
      printf("{\"B\": %d, \"N\": %d, \"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.0f}\n", B, N, name,
             ms * 1e3, by / ms / 1e6);
    };
    rep("step_kb8", time_it([&] { hipLaunchKernelGGL(k_step<8>, dim3(B / G), dim3(64), 0, 0, dw, x, B, N); }, 50));
    rep("step_kb16", time_it([&] { hipLaunchKernelGGL(k_step<16>, dim3(B / G), dim3(64), 0, 0, dw, x, B, N); }, 50));
    rep("chunk8", time_it([&] { hipLaunchKernelGGL(k_chunk<8>, dim3(B / G), dim3(64), 0, 0, dw, x, B, N); }, 50));
    rep("chunk16", time_it([&] { hipLaunchKernelGGL(k_chunk<16>, dim3(B / G), dim3(64), 0, 0, dw, x, B, N); }, 50));
    CK(hipFree(dw)); CK(hipFree(x));
  }
  return 0;
}
