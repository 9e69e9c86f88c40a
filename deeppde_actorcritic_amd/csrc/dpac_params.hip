// dpac_params.hip — kernels on the parameters of the MLPs rather than on
// trajectories: the derived tensors every MLP kernel reads (dpac_mlp_prepare) and
// the optimizer step (dpac_adam_apply); and the critic loss's gradient at V's output
// (dpac_critic_loss_grad), the one elementwise step between the critic's kernels.
//
// Adam: one optimizer step of TF-form Adam over a list of parameter tensors in
// one launch (the reference's tf.keras Adam, solver.py:16-21, whose
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
#include "dpac_device.h"

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
    a.omb1 = T(1) - (T)b1;  // in T, as ResourceApplyAdam forms (T(1) - beta1())
    a.omb2 = T(1) - (T)b2;
    a.eps = (T)eps;
    const unsigned gx = (unsigned)std::min<int64_t>((mx + kAdamThreads - 1) / kAdamThreads, 64);
    hipLaunchKernelGGL(k_adam<T>, dim3(gx, (unsigned)cnt), dim3(kAdamThreads), 0, s, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

// dpac_mlp_prepare: s_i = gamma_scale * gamma_i for every BN layer (concatenated)
// (and the split-fp16 images x3_i / tx3_i of km_i / tkm_i's operands, float only)
// and, optionally, for every dense layer (each segment concatenated over i):
//   wt_i  = (W_i ⊙ s_{i+1})^T         [w_{i+1}][w_i]
//   km_i  = W_i^T, k-major padded      [w_{i+1}][K16(w_i)]      (forward image)
//   tkm_i = W_i ⊙ s_{i+1}, padded      [w_i][K16(w_{i+1})]      (backward image)
// the operands the MLP kernels read.  Element-parallel over the concatenation;
// each output is one multiply (the same rounding as forming gamma_scale*gamma
// and W*s as tensor ops) or a copy.
template <typename T>
struct PrepArgs {
  int L;
  int width[DPAC_MLP_MAX_HIDDEN + 2];
  const T* gamma[DPAC_MLP_MAX_HIDDEN + 2];
  const T* W[DPAC_MLP_MAX_HIDDEN + 1];
  int64_t soff[DPAC_MLP_MAX_HIDDEN + 3];  // offsets of s_i in `scales`
  int64_t woff[DPAC_MLP_MAX_HIDDEN + 2];  // offsets of wt_i in `wt`
  int64_t koff[DPAC_MLP_MAX_HIDDEN + 2];  // offsets of km_i in `km`
  int64_t toff[DPAC_MLP_MAX_HIDDEN + 2];  // offsets of tkm_i in `tkm`
  int64_t xoff[DPAC_MLP_MAX_HIDDEN + 2];  // offsets (halves) of x3_i in `x3`
  int64_t yoff[DPAC_MLP_MAX_HIDDEN + 2];  // offsets (halves) of tx3_i in `tx3`
  T gscale;
  T *scales, *wt, *km, *tkm;
  _Float16 *x3, *tx3;                     // split-fp16 images (float only)
  uint32_t* status;                       // the range guard (dpac.h dpac_mlp.status), or null
};

__device__ __forceinline__ int k16(int k) { return (k + 15) / 16 * 16; }

// part 0 (hi) or 1 (lo) of operand value v in a split-fp16 image (dpac.h dpac_mlp.weight_x3):
// hi = fp16(v), lo = fp16((v - hi) * 2^12), as dpac_mlp_x3.h splits activations.
__device__ __forceinline__ _Float16 x3_part(float v, int part) {
  const _Float16 hi = (_Float16)v;
  return part == 0 ? hi : (_Float16)((v - (float)hi) * 4096.f);
}

template <typename T>
__global__ __launch_bounds__(kAdamThreads) void k_mlp_prepare(const PrepArgs<T> a) {
  const int64_t ns = a.soff[a.L + 2];
  const int64_t nw = a.wt ? a.woff[a.L + 1] : 0;
  const int64_t nk = a.km ? a.koff[a.L + 1] : 0;
  const int64_t nt = a.tkm ? a.toff[a.L + 1] : 0;
  const int64_t nx = a.x3 ? a.xoff[a.L + 1] : 0;
  const int64_t ny = a.tx3 ? a.yoff[a.L + 1] : 0;
  const int64_t n4 = ns + nw + nk + nt;
  bool bad = false;  // a split-fp16 image value outside the split range
  for (int64_t e = (int64_t)blockIdx.x * kAdamThreads + threadIdx.x; e < n4 + nx + ny;
       e += (int64_t)gridDim.x * kAdamThreads) {
    if (e >= n4) {  // split-fp16 images, fragment-major: [tile][chunk][hi|lo][lane][8] halves per layer
      const bool fwd = e < n4 + nx;
      const int64_t f = fwd ? e - n4 : e - n4 - nx;
      const int64_t* off = fwd ? a.xoff : a.yoff;
      int i = 0;
      while (f >= off[i + 1]) ++i;
      const int64_t r = f - off[i];
      const int K = fwd ? a.width[i] : a.width[i + 1], nch = (K + 31) / 32;
      const int cols = fwd ? a.width[i + 1] : a.width[i];
      const int64_t tc = r / 1024;                       // (tile, chunk)
      const int t = (int)(tc / nch), c = (int)(tc % nch);
      const int part = (int)(r / 512) & 1, lane = (int)(r / 8) & 63, el = (int)(r & 7);
      const int n = 16 * t + (lane & 15), k = 32 * c + 8 * (lane >> 4) + el;
      float v = 0.f;
      if (k < K && n < cols)  // forward: W_i[k][n]; backward: W_i[n][k] * s_{i+1}[k] (as tkm_i)
        v = fwd ? (float)a.W[i][(int64_t)k * a.width[i + 1] + n]
                : (float)(a.W[i][(int64_t)n * K + k] * (a.gscale * a.gamma[i + 1][k]));
      (fwd ? a.x3 : a.tx3)[f] = x3_part(v, part);
      bad |= x3_bad(v);
      continue;
    }
    if (e < ns) {
      int i = 0;
      while (e >= a.soff[i + 1]) ++i;
      a.scales[e] = a.gscale * a.gamma[i][e - a.soff[i]];
    } else if (e < ns + nw) {
      const int64_t f = e - ns;
      int i = 0;
      while (f >= a.woff[i + 1]) ++i;
      const int64_t r = f - a.woff[i];
      const int K = a.width[i];               // wt_i is [w_{i+1}][w_i]
      const int64_t j = r / K, k = r % K;     // wt_i[j][k] = W_i[k][j] * s_{i+1}[j]
      const T sj = a.gscale * a.gamma[i + 1][j];
      a.wt[f] = a.W[i][k * a.width[i + 1] + j] * sj;
    } else if (e < ns + nw + nk) {
      const int64_t f = e - ns - nw;
      int i = 0;
      while (f >= a.koff[i + 1]) ++i;
      const int64_t r = f - a.koff[i];
      const int K = a.width[i], KP = k16(K);  // km_i[n][k] = W_i[k][n]
      const int64_t n = r / KP, k = r % KP;
      a.km[f] = k < K ? a.W[i][k * a.width[i + 1] + n] : T(0);
    } else {
      const int64_t f = e - ns - nw - nk;
      int i = 0;
      while (f >= a.toff[i + 1]) ++i;
      const int64_t r = f - a.toff[i];
      const int K = a.width[i + 1], KP = k16(K);  // tkm_i[n][k] = W_i[n][k] * s_{i+1}[k]
      const int64_t n = r / KP, k = r % KP;
      a.tkm[f] = k < K ? a.W[i][n * K + k] * (a.gscale * a.gamma[i + 1][k]) : T(0);
    }
  }
  if (bad) x3_flag(a.status);
}

template <typename T>
int prepare(const dpac_mlp& net, double gscale, void* scales, void* wt, void* km, void* tkm,
            void* x3, void* tx3, hipStream_t s) {
  PrepArgs<T> a{};
  a.L = net.n_hidden;
  int64_t so = 0, wo = 0, ko = 0, to = 0, xo = 0, yo = 0;
  for (int i = 0; i <= a.L + 1; ++i) {
    a.width[i] = net.width[i];
    a.gamma[i] = (const T*)net.bn_scale[i];
    a.soff[i] = so;
    so += net.width[i];
  }
  a.soff[a.L + 2] = so;
  auto pad16 = [](int k) { return (int64_t)((k + 15) / 16 * 16); };
  for (int i = 0; i <= a.L; ++i) {
    a.W[i] = (const T*)net.weight[i];
    a.woff[i] = wo;
    a.koff[i] = ko;
    a.toff[i] = to;
    a.xoff[i] = xo;
    a.yoff[i] = yo;
    wo += (int64_t)net.width[i] * net.width[i + 1];
    ko += (int64_t)net.width[i + 1] * pad16(net.width[i]);
    to += (int64_t)net.width[i] * pad16(net.width[i + 1]);
    xo += (int64_t)((net.width[i + 1] + 15) / 16) * 1024 * ((net.width[i] + 31) / 32);
    yo += (int64_t)((net.width[i] + 15) / 16) * 1024 * ((net.width[i + 1] + 31) / 32);
  }
  a.woff[a.L + 1] = wo;
  a.koff[a.L + 1] = ko;
  a.toff[a.L + 1] = to;
  a.xoff[a.L + 1] = xo;
  a.yoff[a.L + 1] = yo;
  a.x3 = (_Float16*)x3;
  a.tx3 = (_Float16*)tx3;
  a.status = (x3 || tx3) ? net.status : nullptr;
  a.gscale = (T)gscale;
  a.scales = (T*)scales;
  a.wt = (T*)wt;
  a.km = (T*)km;
  a.tkm = (T*)tkm;
  const int64_t total = so + (wt ? wo : 0) + (km ? ko : 0) + (tkm ? to : 0) + (x3 ? xo : 0) + (tx3 ? yo : 0);
  const unsigned g = (unsigned)std::min<int64_t>((total + kAdamThreads - 1) / kAdamThreads, 1024);
  hipLaunchKernelGGL(k_mlp_prepare<T>, dim3(g), dim3(kAdamThreads), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace

// dpac_critic_loss_grad: the gradient of loss_critic (solver.py:73-78) at V's outputs, from
// V at [x_0; x_N; x_bdry] (3B), the TD target y, the discount disc_N and Z_tf(x_bdry)
// (solver.py:189-190):
//   delta = (V0 - y) - VN * disc,  delta_b = Vb - zb,
//   h'(z) = 2 z if |z| < clip else (2 clip) sign(z),   g = h'(delta) * scale,  g_b = h'(delta_b) * scale,
//   g_out = [g; (-g) * disc; g_b],  neg_g = -g   (dL/dy, what the TD backward reads)
// each operation rounded as the same tensor expressions round them (-ffp-contract=off).
template <typename T>
__global__ __launch_bounds__(256) void k_critic_loss_grad(int64_t B, const T* __restrict__ V, const T* __restrict__ y,
                                                          const T* __restrict__ disc, const T* __restrict__ zb,
                                                          T scale, T clip, T* __restrict__ g_out,
                                                          T* __restrict__ neg_g) {
  const int64_t b = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  auto hgrad = [&](T z) {
    const T sg = z > T(0) ? T(1) : (z < T(0) ? T(-1) : z);  // sign(z); NaN stays NaN as in torch.where
    return fabs(z) < clip ? T(2) * z : (T(2) * clip) * sg;
  };
  const T dc = disc[b];
  const T delta = (V[b] - y[b]) - V[B + b] * dc;
  const T delta_b = V[2 * B + b] - zb[b];
  const T g = hgrad(delta) * scale;
  g_out[b] = g;
  g_out[B + b] = (-g) * dc;
  g_out[2 * B + b] = hgrad(delta_b) * scale;
  neg_g[b] = -g;
}

int critic_loss_launch(int dtype, int64_t B, const void* V, const void* y, const void* disc, const void* zb,
                       double scale, double clip, void* g_out, void* neg_g, hipStream_t s) {
  const dim3 grid((unsigned)((B + 255) / 256));
  if (dtype == DPAC_F64)
    hipLaunchKernelGGL(k_critic_loss_grad<double>, grid, dim3(256), 0, s, B, (const double*)V, (const double*)y,
                       (const double*)disc, (const double*)zb, scale, clip, (double*)g_out, (double*)neg_g);
  else
    hipLaunchKernelGGL(k_critic_loss_grad<float>, grid, dim3(256), 0, s, B, (const float*)V, (const float*)y,
                       (const float*)disc, (const float*)zb, (float)scale, (float)clip, (float*)g_out,
                       (float*)neg_g);
  return (int)hipGetLastError();
}

int mlp_prepare_launch(int dtype, const dpac_mlp& net, double gamma_scale, void* scales, void* wt,
                       void* km, void* tkm, void* x3, void* tx3, hipStream_t s) {
  return dtype == DPAC_F64 ? prepare<double>(net, gamma_scale, scales, wt, km, tkm, nullptr, nullptr, s)
                           : prepare<float>(net, gamma_scale, scales, wt, km, tkm, x3, tx3, s);
}

int adam_launch(int dtype, int n, const int64_t* numel, void* const* var, const void* const* grad,
                void* const* m, void* const* v, double alpha, double b1, double b2, double eps,
                hipStream_t s) {
  return dtype == DPAC_F64 ? launch<double>(n, numel, var, grad, m, v, alpha, b1, b2, eps, s)
                           : launch<float>(n, numel, var, grad, m, v, alpha, b1, b2, eps, s);
}

}  // namespace dpac
