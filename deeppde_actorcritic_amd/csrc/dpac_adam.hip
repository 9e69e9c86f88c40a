// dpac_adam.hip — one optimizer step of TF-form Adam over a list of parameter
// tensors in one launch (the reference's tf.keras Adam, solver.py:16-21, whose
// ResourceApplyAdam update is):
//   m   += (g - m)(1 - b1)
//   v   += (g*g - v)(1 - b2)
//   var -= (m*alpha) / (sqrt(v) + eps),   alpha = lr*sqrt(1 - b2^t)/(1 - b1^t)
// Every operation rounds on its own (the library builds with -ffp-contract=off),
// in the order above, so the result is bitwise that of the same update written
// as separate elementwise tensor ops.  Each workgroup row (blockIdx.y) owns one
// tensor; blocks stride over its elements.  Elementwise and HBM-bound: 16 bytes
// read + 12 written per fp32 element.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dpac.h"

namespace dpac {

namespace {

constexpr int kAdamMax = 32;  // tensors per launch (kernel-argument struct stays < 2 KiB)
constexpr int kAdamThreads = 256;

template <typename T>
struct AdamArgs {
  int64_t numel[kAdamMax];
  T* var[kAdamMax];
  const T* grad[kAdamMax];
  T* m[kAdamMax];
  T* v[kAdamMax];
  T alpha, omb1, omb2, eps;
};

template <typename T>
__global__ __launch_bounds__(kAdamThreads) void k_adam(const AdamArgs<T> a) {
  const int i = blockIdx.y;
  const int64_t n = a.numel[i];
  T* __restrict__ var = a.var[i];
  const T* __restrict__ g = a.grad[i];
  T* __restrict__ m = a.m[i];
  T* __restrict__ v = a.v[i];
  for (int64_t e = (int64_t)blockIdx.x * kAdamThreads + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * kAdamThreads) {
    const T ge = g[e];
    T me = m[e];
    T ve = v[e];
    me = me + (ge - me) * a.omb1;
    ve = ve + (ge * ge - ve) * a.omb2;
    const T den = sqrt(ve) + a.eps;
    var[e] = var[e] - (me * a.alpha) / den;
    m[e] = me;
    v[e] = ve;
  }
}

template <typename T>
int launch(int n, const int64_t* numel, void* const* var, const void* const* grad, void* const* m,
           void* const* v, double alpha, double b1, double b2, double eps, hipStream_t s) {
  for (int base = 0; base < n; base += kAdamMax) {
    const int cnt = std::min(kAdamMax, n - base);
    AdamArgs<T> a{};
    int64_t mx = 1;
    for (int j = 0; j < cnt; ++j) {
      a.numel[j] = numel[base + j];
      a.var[j] = (T*)var[base + j];
      a.grad[j] = (const T*)grad[base + j];
      a.m[j] = (T*)m[base + j];
      a.v[j] = (T*)v[base + j];
      mx = std::max(mx, a.numel[j]);
    }
    a.alpha = (T)alpha;
    a.omb1 = (T)(1.0 - b1);
    a.omb2 = (T)(1.0 - b2);
    a.eps = (T)eps;
    const unsigned gx = (unsigned)std::min<int64_t>((mx + kAdamThreads - 1) / kAdamThreads, 64);
    hipLaunchKernelGGL(k_adam<T>, dim3(gx, (unsigned)cnt), dim3(kAdamThreads), 0, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

}  // namespace

int adam_launch(int dtype, int n, const int64_t* numel, void* const* var, const void* const* grad,
                void* const* m, void* const* v, double alpha, double b1, double b2, double eps,
                hipStream_t s) {
  return dtype == DPAC_F64 ? launch<double>(n, numel, var, grad, m, v, alpha, b1, b2, eps, s)
                           : launch<float>(n, numel, var, grad, m, v, alpha, b1, b2, eps, s);
}

}  // namespace dpac
