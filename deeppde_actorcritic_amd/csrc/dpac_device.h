// dpac_device.h — device building blocks shared by every libdpac kernel:
//   * lane-group reductions (a trajectory is owned by P consecutive lanes of a
//     64-wide wavefront; sums over its d components use DPP / ds_swizzle),
//   * the Brownian-increment stream (rocRAND Philox4x32-10 + Box–Muller),
//   * the four equation families as device functors (coefficients, analytic
//     solutions and the vector-Jacobian products needed by the rollout backward).
//
// Reference: equation.py:5-311 (Equation, LQR, VDP, ekn, LQR_var).
#pragma once

#include <hip/hip_runtime.h>
#include <rocrand/rocrand_kernel.h>
#include <stdint.h>

#include "dpac.h"

namespace dpac {

// ---------------------------------------------------------------------------
// Lane-group reductions.  Group g of a wave = lanes [g*P, g*P+P); every lane of
// the group ends with the same (bitwise) sum because each butterfly level adds
// two operands in commutative order.
// ---------------------------------------------------------------------------
template <int MASK>
__device__ __forceinline__ int shfl_xor_i32(int v) {
  static_assert(MASK > 0 && MASK < 32, "group reductions stay within 32 lanes");
  if constexpr (MASK == 1) {
    return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, true);  // quad_perm(1,0,3,2)
  } else if constexpr (MASK == 2) {
    return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, true);  // quad_perm(2,3,0,1)
  } else {
    return __builtin_amdgcn_ds_swizzle(v, (MASK << 10) | 0x1F);  // bit-mode xor
  }
}

template <int MASK>
__device__ __forceinline__ float shfl_xor(float v) {
  return __builtin_bit_cast(float, shfl_xor_i32<MASK>(__builtin_bit_cast(int, v)));
}
template <int MASK>
__device__ __forceinline__ double shfl_xor(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = shfl_xor_i32<MASK>(static_cast<int>(b));
  const int hi = shfl_xor_i32<MASK>(static_cast<int>(b >> 32));
  return __builtin_bit_cast(
      double, (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}

template <int P>
struct Lanes {
  static_assert(P == 1 || P == 2 || P == 4 || P == 8 || P == 16, "bad group size");
  template <typename T>
  __device__ __forceinline__ static T sum(T v) {
    if constexpr (P >= 2) v = v + shfl_xor<1>(v);
    if constexpr (P >= 4) v = v + shfl_xor<2>(v);
    if constexpr (P >= 8) v = v + shfl_xor<4>(v);
    if constexpr (P >= 16) v = v + shfl_xor<8>(v);
    return v;
  }
};

// Lanes per trajectory for a componentwise equation of dimension D: keep ~4-5
// components per lane so the per-trajectory scalar work (norms, step size,
// flags) is shared by few lanes while B = 4096 still fills 256 CUs.
__host__ __device__ constexpr int lanes_for_dim(int D) {
  return (D % 4 == 0 && D >= 16) ? 4 : ((D % 2 == 0 && D >= 8) ? 2 : 1);
}

// ---------------------------------------------------------------------------
// Brownian increments: rocRAND Philox4x32-10, subsequence = global trajectory
// index, counter block = (tag << 48) | index.  The d components of step t are
// cut into R = lanes_for_dim(d) chunks of C = d / R components; chunk r uses
// BPC = ceil(C / PB) consecutive counter blocks, PB numbers per block (4 float
// normals, 2 double normals, or 4 bounded values).  So a lane that owns one
// chunk draws its own increments with no cross-lane traffic, and the stream is
// a fixed function of (seed, global trajectory, t, j) for every GPU count.
// Normal: rocRAND's Box–Muller (float: box_muller_hw below; double:
// normal_distribution_double2).  Bounded:
// k = floor(6·u32 / 2^32) ∈ {0..5}, value floor((k-1)/4)·√3 (equation.py:31-32).
// ---------------------------------------------------------------------------
enum : uint64_t { kTagDw = 0, kTagDir = 1, kTagRadius = 2, kTagBdry = 3 };

__device__ __forceinline__ uint4 philox_block(uint64_t seed, uint64_t subseq,
                                              uint64_t block) {
  rocrand_state_philox4x32_10 st;
  rocrand_init(seed, subseq, block * 4ull, &st);
  return rocrand4(&st);  // the 4 words of counter `block`; the engine copy dies here
}

template <typename T>
struct Rng;
// rocRAND's float Box–Muller mapping (rocrand_normal.h box_muller: u in (0,1],
// angle in (0, 2pi]) evaluated with the hardware v_log_f32 / v_sqrt_f32 /
// v_sin/cos_f32 instead of the correctly-rounded expansions: ~1 ulp, ~4x fewer
// instructions per normal.
__device__ __forceinline__ void box_muller_hw(unsigned int x, unsigned int y, float& a, float& b) {
  const float u = ROCRAND_2POW32_INV + (x * ROCRAND_2POW32_INV);
  const float v = ROCRAND_2POW32_INV_2PI + (y * ROCRAND_2POW32_INV_2PI);
  const float s = __builtin_amdgcn_sqrtf(-2.0f * __logf(u));
  float sn, cs;
  __sincosf(v, &sn, &cs);
  a = sn * s;
  b = cs * s;
}

template <>
struct Rng<float> {
  static constexpr int kNormalPerBlock = 4;
  __device__ static void normals(uint4 v, float (&o)[4]) {
    box_muller_hw(v.x, v.y, o[0], o[1]);
    box_muller_hw(v.z, v.w, o[2], o[3]);
  }
};
template <>
struct Rng<double> {
  static constexpr int kNormalPerBlock = 2;
  __device__ static void normals(uint4 v, double (&o)[2]) {
    const double2 n = rocrand_device::detail::normal_distribution_double2(v);
    o[0] = n.x; o[1] = n.y;
  }
};

template <typename T>
__device__ __forceinline__ T bounded_value(unsigned int w) {
  const unsigned int k = static_cast<unsigned int>((static_cast<unsigned long long>(w) * 6ull) >> 32);
  const T s3 = static_cast<T>(1.7320508075688772);  // np.sqrt(3.0)
  return k == 0u ? -s3 : (k == 5u ? s3 : static_cast<T>(0));
}

template <typename T>
__host__ __device__ constexpr int dw_per_block(int sample_type) {
  return sample_type == DPAC_SAMPLE_BOUNDED ? 4 : (sizeof(T) == 4 ? 4 : 2);
}

// Increments of chunk `r` (C components starting at r*C) of step t.
template <typename T, int D, int C>
__device__ __forceinline__ void draw_chunk(uint64_t seed, uint64_t traj, int t, int r,
                                           int sample_type, T (&out)[C]) {
  constexpr int R = D / C;
  if (sample_type == DPAC_SAMPLE_BOUNDED) {
    constexpr int BPC = (C + 3) / 4;
    const uint64_t base = (uint64_t)t * (R * BPC) + (uint64_t)r * BPC;
#pragma unroll
    for (int blk = 0; blk < BPC; ++blk) {
      const uint4 v = philox_block(seed, traj, (kTagDw << 48) | (base + blk));
      const unsigned int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (blk * 4 + e < C) out[blk * 4 + e] = bounded_value<T>(w[e]);
    }
  } else {
    constexpr int PB = Rng<T>::kNormalPerBlock;
    constexpr int BPC = (C + PB - 1) / PB;
    const uint64_t base = (uint64_t)t * (R * BPC) + (uint64_t)r * BPC;
#pragma unroll
    for (int blk = 0; blk < BPC; ++blk) {
      T n[PB];
      Rng<T>::normals(philox_block(seed, traj, (kTagDw << 48) | (base + blk)), n);
#pragma unroll
      for (int e = 0; e < PB; ++e)
        if (blk * PB + e < C) out[blk * PB + e] = n[e];
    }
  }
}

// ---------------------------------------------------------------------------
// Equation functors.  A lane owns M = D/P consecutive state components
// (j = p*M + m) and MC control components.  Methods see only the owned slice;
// anything needing the whole vector receives the group-reduced |x|^2 (`S`) or
// reduces through Lanes<P>.  All constants are computed on the host in double,
// in the reference's evaluation order, then rounded to T.
// ---------------------------------------------------------------------------
struct HostConsts {  // double-precision constants shared by all equations
  double gamma, R, sigma_up, dt0, sqrt_dt0, dt_min, den, c_layer, R2;
};

// LQR — equation.py:144-176
template <typename T, int D, int P>
struct EqLQR {
  static constexpr int M = D / P, MC = M, kP = P;
  static constexpr bool kNeedsNorm = false;
  T p, q, beta, kappa, two_kd, kR2, sqrt2, two_k, k, two_p, two_q;
  static EqLQR make(const dpac_eqn_params& e) {
    EqLQR r;
    r.p = (T)e.p; r.q = (T)e.q; r.beta = (T)e.beta; r.k = (T)e.k;
    r.kappa = (T)(-e.beta * e.k / e.q);     // u_true: -beta*k/q*x (:164)
    r.two_kd = (T)(2.0 * e.k * e.dim);      // w: ... - 2*k*dim (:155)
    r.kR2 = (T)(e.k * (e.R * e.R));         // Z = k*R^2 (:158)
    r.sqrt2 = (T)1.4142135623730951;        // np.sqrt(2.0) (:170)
    r.two_k = (T)(2.0 * e.k);               // V_grad = 2*k*x (:167)
    r.two_p = (T)(2.0 * e.p); r.two_q = (T)(2.0 * e.q);
    return r;
  }
  __device__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = kappa * x[m];
  }
  __device__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = beta * u[m];
  }
  __device__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  __device__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T a = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) a += p * (x[m] * x[m]) + q * (u[m] * u[m]);
    return a;
  }
  __device__ T w_finish(T s) const { return s - two_kd; }
  __device__ T V_true(const T (&x)[M], T S) const { return S * k; }
  __device__ T Z(const T (&x)[M], T S) const { return kR2; }
  __device__ void V_grad(const T (&x)[M], T S, T (&g)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = two_k * x[m];
  }
  // VJPs: accumulate a·∂drift/∂(x,u), a·∂sigma/∂(x,u), gw·∂w/∂(x,u)
  __device__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T S, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) gu[m] += beta * a[m];
  }
  __device__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {}
  __device__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M],
                        T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gx[m] += gw * (two_p * x[m]);
      gu[m] += gw * (two_q * u[m]);
    }
  }
};

// LQR_var — equation.py:278-311 (state- and control-dependent diagonal sigma)
template <typename T, int D, int P>
struct EqLQRVar {
  static constexpr int M = D / P, MC = M, kP = P;
  static constexpr bool kNeedsNorm = false;
  T q, beta, eps, k, c1, c2, gk, two_kd, kR2, sqrt2, bpe, qk, e2, two_k, two_q, two_gk,
      sqrt2_eps, two_c1q;
  static EqLQRVar make(const dpac_eqn_params& e) {
    EqLQRVar r;
    r.q = (T)e.q; r.beta = (T)e.beta; r.eps = (T)e.epsilon; r.k = (T)e.k;
    const double bpe = e.beta + 2.0 * e.epsilon;
    r.c1 = (T)(e.k * e.k * (bpe * bpe));             // k**2*(beta+2eps)**2 (:289)
    r.c2 = (T)(2.0 * e.k * (e.epsilon * e.epsilon));  // 2*k*eps**2 (:289)
    r.gk = (T)(e.gamma * e.k);                        // gamma*k (:290)
    r.two_kd = (T)(2.0 * e.k * e.dim);
    r.kR2 = (T)(e.k * (e.R * e.R));
    r.sqrt2 = (T)1.4142135623730951;
    r.bpe = (T)bpe;                                   // u_true numerator (:299)
    r.qk = (T)(e.q / e.k);
    r.e2 = (T)(2.0 * (e.epsilon * e.epsilon));
    r.two_k = (T)(2.0 * e.k); r.two_q = (T)(2.0 * e.q); r.two_gk = (T)(2.0 * e.gamma * e.k);
    r.sqrt2_eps = (T)(1.4142135623730951 * e.epsilon);
    r.two_c1q = (T)(2.0 * (e.k * e.k * (bpe * bpe)) * e.q);
    return r;
  }
  __device__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = (-bpe * x[m]) / (qk + e2 * (x[m] * x[m]));
  }
  __device__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = beta * u[m];
  }
  __device__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2 * (1 + (eps * x[m]) * u[m]);
  }
  __device__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T a = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const T x2 = x[m] * x[m];
      a += (c1 * x2) / (q + c2 * x2) + (gk * x2 + q * (u[m] * u[m]));
    }
    return a;
  }
  __device__ T w_finish(T s) const { return s - two_kd; }
  __device__ T V_true(const T (&x)[M], T S) const { return S * k; }
  __device__ T Z(const T (&x)[M], T S) const { return kR2; }
  __device__ void V_grad(const T (&x)[M], T S, T (&g)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = two_k * x[m];
  }
  __device__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T S, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) gu[m] += beta * a[m];
  }
  __device__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gx[m] += a[m] * (sqrt2_eps * u[m]);
      gu[m] += a[m] * (sqrt2_eps * x[m]);
    }
  }
  __device__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M],
                        T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const T den = q + c2 * (x[m] * x[m]);
      gx[m] += gw * (two_c1q * x[m] / (den * den) + two_gk * x[m]);
      gu[m] += gw * (two_q * u[m]);
    }
  }
};

// ekn (configs say "EKN") — diffusive Eikonal, equation.py:240-276
template <typename T, int D, int P>
struct EqEKN {
  static constexpr int M = D / P, MC = M, kP = P;
  static constexpr bool kNeedsNorm = true;
  T a2, a3, K, two_a2, three_a3, sqrt2;
  static EqEKN make(const dpac_eqn_params& e) {
    EqEKN r;
    r.a2 = (T)e.a2; r.a3 = (T)e.a3;
    r.K = (T)(3.0 * (e.dim + 1) * e.a3 / 2.0 / e.a2 / e.dim);  // (:272) numerator chain
    r.two_a2 = (T)(2.0 * e.a2); r.three_a3 = (T)(3.0 * e.a3);
    r.sqrt2 = (T)1.4142135623730951;
    return r;
  }
  __device__ static T norm(T S) { return sqrt(S); }
  __device__ void u_true(const T (&x)[M], T S, T (&u)[MC]) const {
    const T r = norm(S);
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = x[m] / r;
  }
  __device__ void drift(const T (&x)[M], const T (&u)[MC], T S, T (&f)[M]) const {
    const T c = K / (two_a2 - three_a3 * norm(S));
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = c * u[m];
  }
  __device__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  __device__ T w_part(const T (&x)[M], const T (&u)[MC]) const { return 0; }
  __device__ T w_finish(T) const { return 1; }  // 0*sum(x) + 1 (:250)
  __device__ T V_true(const T (&x)[M], T S) const {
    const T r = norm(S);
    return a3 * (r * r * r) - a2 * (r * r);
  }
  __device__ T Z(const T (&x)[M], T S) const { return V_true(x, S); }
  __device__ void V_grad(const T (&x)[M], T S, T (&g)[M]) const {
    const T c = three_a3 * norm(S) - two_a2;
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = c * x[m];
  }
  __device__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T S, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
    const T r = norm(S);
    const T den = two_a2 - three_a3 * r;
    const T c = K / den;
    T au = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gu[m] += c * a[m];
      au += a[m] * u[m];
    }
    au = Lanes<P>::sum(au);
    // d c / d r = K*3a3/den^2 ; d r / d x = x / r
    const T f = au * (K * three_a3 / (den * den)) / r;
#pragma unroll
    for (int m = 0; m < M; ++m) gx[m] += f * x[m];
  }
  __device__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {}
  __device__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M],
                        T (&gu)[MC]) const {}
};

// VDP — stochastic Van der Pol oscillator, equation.py:179-238.  x = (x1, x2),
// c = d/2; px/nx are the cyclic shifts inside each half (:192-195).  The
// coupling between halves keeps the whole state in one lane (P = 1).
template <typename T, int D, int P>
struct EqVDP {
  static_assert(P == 1 && D % 2 == 0, "VDP keeps a trajectory in one lane");
  static constexpr int M = D, C = D / 2, MC = D / 2, kP = 1;
  static constexpr bool kNeedsNorm = false;
  T a, eps, q, gamma, geps, ga, two_ad, sqrt2, two_a, inv2q, two_ga, two_q;
  static EqVDP make(const dpac_eqn_params& e) {
    EqVDP r;
    r.a = (T)e.a; r.eps = (T)e.epsilon; r.q = (T)e.q; r.gamma = (T)e.gamma;
    r.geps = (T)(-e.gamma * e.epsilon);  // -gamma*epsl (:198)
    r.ga = (T)(e.gamma * e.a);           // gamma*a (:199)
    r.two_ad = (T)(2.0 * e.a * e.dim);   // 2*a*dim (:199)
    r.sqrt2 = (T)1.4142135623730951;
    r.two_a = (T)(2.0 * e.a);
    r.inv2q = (T)(1.0 / (2.0 * e.q));
    r.two_ga = (T)(2.0 * e.gamma * e.a);
    r.two_q = (T)(2.0 * e.q);
    return r;
  }
  __device__ static constexpr int nxt(int i) { return (i + 1) % C; }
  __device__ static constexpr int prv(int i) { return (i + C - 1) % C; }
  // dv = 2a*v - eps*(px + nx) on one half (:196-197, :217, :227)
  __device__ void Lop(const T* v, T* o) const {
#pragma unroll
    for (int i = 0; i < C; ++i) o[i] = two_a * v[i] - eps * (v[nxt(i)] + v[prv(i)]);
  }
  __device__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
    T dv2[C];
    Lop(x + C, dv2);
#pragma unroll
    for (int i = 0; i < C; ++i) u[i] = -dv2[i] / 2 / q;  // (:217)
  }
  __device__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      f[i] = x2;
      f[C + i] = (1 - x1 * x1) * x2 - x1 + u[i];  // (:235)
    }
  }
  __device__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  __device__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T dv1[C], dv2[C];
    Lop(x, dv1);
    Lop(x + C, dv2);
    T acc = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      const T px1 = x[nxt(i)], px2 = x[C + nxt(i)];
      const T temp = geps * (x1 * px1 + x2 * px2) + (dv2[i] * dv2[i]) / 4 / q - x2 * dv1[i] -
                     ((1 - x1 * x1) * x2 - x1) * dv2[i];
      acc += temp + q * (u[i] * u[i]) + ga * (x1 * x1 + x2 * x2);
    }
    return acc;
  }
  __device__ T w_finish(T s) const { return s - two_ad; }
  __device__ T V_true(const T (&x)[M], T S) const {  // (:210)
    T cross = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) cross += x[i] * x[nxt(i)] + x[C + i] * x[C + nxt(i)];
    return a * S - eps * cross;
  }
  __device__ T Z(const T (&x)[M], T S) const { return V_true(x, S); }
  __device__ void V_grad(const T (&x)[M], T S, T (&g)[M]) const {  // (:227)
    Lop(x, g);
    Lop(x + C, g + C);
  }
  __device__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T S, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i], a1 = a[i], a2v = a[C + i];
      gx[i] += a2v * (-2 * x1 * x2 - 1);
      gx[C + i] += a1 + a2v * (1 - x1 * x1);
      gu[i] += a2v;
    }
  }
  __device__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {}
  // gradient of w (derivation in DESIGN.md §4.3): with L v = 2a v - eps(px v + nx v),
  // g = (1 - x1^2) x2 - x1:
  //   dw/dx1 = -gamma*eps*(px1+nx1) + 2 x1 x2 dv2 + 2 gamma a x1
  //   dw/dx2 = -gamma*eps*(px2+nx2) + L(dv2)/(2q) - dv1 - (1 - x1^2) dv2 - L(g) + 2 gamma a x2
  __device__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M],
                        T (&gu)[MC]) const {
    T dv1[C], dv2[C], g[C], Ldv2[C], Lg[C];
    Lop(x, dv1);
    Lop(x + C, dv2);
#pragma unroll
    for (int i = 0; i < C; ++i) g[i] = (1 - x[i] * x[i]) * x[C + i] - x[i];
    Lop(dv2, Ldv2);
    Lop(g, Lg);
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      const T s1 = x[nxt(i)] + x[prv(i)], s2 = x[C + nxt(i)] + x[C + prv(i)];
      const T d1 = geps * s1 + 2 * x1 * x2 * dv2[i] + two_ga * x1;
      const T d2 = geps * s2 + Ldv2[i] * inv2q - dv1[i] - (1 - x1 * x1) * dv2[i] - Lg[i] +
                   two_ga * x2;
      gx[i] += gw * d1;
      gx[C + i] += gw * d2;
      gu[i] += gw * (two_q * u[i]);
    }
  }
};

}  // namespace dpac
