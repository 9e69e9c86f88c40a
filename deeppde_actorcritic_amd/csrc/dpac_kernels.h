// dpac_kernels.h — kernel templates of libdpac and the per-equation launcher.
//
// Mapping (all kernels): 64-thread workgroups = one wavefront; a trajectory is
// owned by P = E::kP consecutive lanes, each holding M = d/P state components in
// registers.  The time loop runs inside the kernel, so a trajectory's state
// never leaves registers between steps; what goes to HBM is exactly what the
// reference materialises (x_smp, dt, coef: equation.py:63-70, 97-104).
// Per-step inputs (dw, and for the TD pass x/u/G/dt/coef) are prefetched
// 2*KB steps ahead through a register ring (pipelined()).
#pragma once

#include <cmath>
#include <type_traits>

#include "dpac_device.h"

namespace dpac {

enum Op : int {
  OP_ROLLOUT = 0,
  OP_FLAG_INIT,
  OP_STEP_FWD,
  OP_STEP_BWD,
  OP_TD_FWD,
  OP_TD_BWD,
  OP_EVAL,
};

// Everything any op may need; unused fields are ignored.
struct OpArgs {
  int op;
  dpac_eqn_params eq;
  int scheme, dtype, td_type, cost_order, sample_type, what;
  int64_t B, traj_offset;
  int N;
  double T;
  uint64_t seed;
  const void *x0, *dw, *x, *u, *dt_in, *coef_in, *G, *disc_in, *y_in;
  const int32_t* flag_in;
  const void *g_x_out, *g_disc_out, *g_y_out;
  void *x_out, *dt, *coef, *u_out, *y, *disc, *disc_out, *y_out;
  int32_t* flag_out;
  void *g_x, *g_u, *g_disc, *g_G, *out;
  hipStream_t stream;
};

inline HostConsts host_consts(const OpArgs& a) {
  HostConsts h;
  const double d = a.eq.dim;
  h.gamma = a.eq.gamma;
  h.R = a.eq.R;
  h.sigma_up = a.eq.sigma_up;
  h.dt0 = a.T / a.N;                                          // delta_t = T / N (:48, :75)
  h.sqrt_dt0 = std::sqrt(h.dt0);                              // np.sqrt(delta_t) (:49)
  h.dt_min = h.dt0 * 1e-4;                                    // delta_t*1e-4 (:86)
  h.den = 3 * a.eq.dim * (a.eq.sigma_up * a.eq.sigma_up);     // 3*dim*sigma_Up**2 (:85)
  h.c_layer = a.eq.sigma_up * std::sqrt(3 * d * h.dt0);       // sigma_Up*sqrt(3*dim*dt) (:80, :94)
  h.R2 = a.eq.R * a.eq.R;                                     // R**2 (:122)
  return h;
}

template <typename T>
struct DevConsts {
  T gamma, R, dt0, sqrt_dt0, dt_min, den, c_layer, R2, neg_gamma;
  static DevConsts make(const HostConsts& h) {
    DevConsts c;
    c.gamma = (T)h.gamma; c.R = (T)h.R; c.dt0 = (T)h.dt0; c.sqrt_dt0 = (T)h.sqrt_dt0;
    c.dt_min = (T)h.dt_min; c.den = (T)h.den; c.c_layer = (T)h.c_layer; c.R2 = (T)h.R2;
    c.neg_gamma = (T)(-h.gamma);
    return c;
  }
};

// ---------------------------------------------------------------------------
// Software-pipelined time loop: frames for steps [t, t+KB) are loaded while
// the previous KB steps compute.  Frame arrays are indexed only by unrolled
// constants, so they live in VGPRs.
// ---------------------------------------------------------------------------
template <int KB, class F, class LoadF, class BodyF>
__device__ __forceinline__ void pipelined(int N, LoadF&& load, BodyF&& body) {
  F A[KB], Bq[KB];
#pragma unroll
  for (int k = 0; k < KB; ++k)
    if (k < N) load(k, A[k]);
  for (int t0 = 0; t0 < N; t0 += 2 * KB) {
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (t0 + KB + k < N) load(t0 + KB + k, Bq[k]);
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (t0 + k < N) body(t0 + k, A[k]);
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (t0 + 2 * KB + k < N) load(t0 + 2 * KB + k, A[k]);
#pragma unroll
    for (int k = 0; k < KB; ++k)
      if (t0 + KB + k < N) body(t0 + KB + k, Bq[k]);
  }
}

// Lane coordinates: trajectory index b (clamped into range for the idle
// groups of the last wave, which compute on a duplicate but never store) and
// component slice p.
template <int P>
struct LaneCoord {
  int p;
  int64_t b;
  bool live;
  __device__ LaneCoord(int64_t B) {
    const int lane = threadIdx.x;
    p = lane % P;
    b = (int64_t)blockIdx.x * (64 / P) + lane / P;
    live = b < B;
    if (!live) b = B - 1;
  }
};

template <typename T>
__device__ __forceinline__ int sgn(T v) {
  return (v > T(0)) - (v < T(0));
}

// floor(v/2) for v in {-2..2} (the reference's tf.math.floor(temp/2))
__device__ __forceinline__ int floor_half(int v) { return v >= 0 ? v / 2 : -((-v + 1) / 2); }

// Adaptive flag of a point at radius r: 2 inner, 1 boundary layer, 0 outside
// (equation.py:80-82 and :94-95 before the sign(flag) factor).
template <typename T>
__device__ __forceinline__ int adaptive_flag(T r, const DevConsts<T>& c) {
  const int tmp = sgn((c.R - r) - c.c_layer) + sgn(c.R - r);
  return 1 + floor_half(tmp);
}

// Step size of the adaptive scheme (equation.py:85-86): (2f-f^2)(R-r)^2/den +
// (f^2-2f+1)dt0 is exactly (R-r)^2/den for f == 1 and dt0 for f in {0, 2}.
template <typename T>
__device__ __forceinline__ T adaptive_dt_raw(int flag, T r, const DevConsts<T>& c) {
  return flag == 1 ? ((c.R - r) * (c.R - r)) / c.den : c.dt0;
}

// One transition of the scheme for the owned slice.  In: x, u, dw, flag, S = |x|^2.
// Out: dx, coef, new flag, St = |x + dx|^2, dt and sqrt(dt).
template <typename T, class E, int SCHEME>
struct Transition {
  static constexpr int M = E::M, MC = E::MC, P = E::kP;
  T dx[M];
  T dt, sq, St;
  int coef, flag_new;
  __device__ __forceinline__ void run(const E& eq, const DevConsts<T>& c, const T (&x)[M],
                                      const T (&u)[MC], const T (&dw)[M], int flag, T S) {
    if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
      const T r = sqrt(S);
      const T raw = adaptive_dt_raw(flag, r, c);
      dt = raw >= c.dt_min ? raw : c.dt_min;  // tf.maximum(dt_i, delta_t*1e-4)
      sq = sqrt(dt);
    } else {
      dt = c.dt0;
      sq = c.sqrt_dt0;
    }
    T f[M], s[M];
    eq.drift(x, u, S, f);
    eq.sigma(x, u, s);
    T acc = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      dx[m] = f[m] * dt + (s[m] * dw[m]) * sq;  // drift*dt + diffusion*sqrt(dt) (:58, :91)
      const T xt = x[m] + dx[m];
      acc += xt * xt;
    }
    St = Lanes<P>::sum(acc);
    if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
      const int nf = flag > 0 ? adaptive_flag(sqrt(St), c) : 0;  // * sign(flag) (:95)
      coef = (flag > 0 && nf > 0) ? 1 : 0;                          // sign(flag)*sign(new_flag) (:96)
      flag_new = nf;
    } else {
      const int exit_ = (St - c.R2) >= T(0) ? 1 : 0;  // ceil((sign(b(x))+1)/2) (:60-61)
      coef = flag * (1 - exit_);                      // (:62)
      flag_new = coef;                                 // flag *= 1 - Exit (:69)
    }
  }
};

template <typename T, int ORDER>
__device__ __forceinline__ T cost_increment(T w, T coef, T dt, T disc) {
  if constexpr (ORDER == DPAC_COST_ACTOR)
    return ((coef * w) * dt) * disc;  // coef*w*dt*discount (solver.py:218)
  else
    return (w * disc) * (coef * dt);  // (w*discount)*(coef*dt) (solver.py:170-174)
}

template <typename T>
__device__ __forceinline__ T disc_factor(T dt, T coef, const DevConsts<T>& c) {
  return exp((c.neg_gamma * dt) * coef);  // exp(-gamma*dt*coef) (solver.py:187, :219)
}

// ---------------------------------------------------------------------------
// Fused rollout with the analytic control u_true (reference `cheat` path).
// ---------------------------------------------------------------------------
template <typename T>
struct RolloutArgs {
  int64_t B, traj_offset;
  int N, sample_type;
  uint64_t seed;
  const T* x0;
  const T* dw;
  T *x, *dt, *coef, *u, *y, *disc;
};

template <typename T, int M>
struct DwFrame {
  T dw[M];
};

template <typename T, class E, int D, int SCHEME, bool PHILOX, bool COST, int ORDER, int KB>
__global__ __launch_bounds__(64) void k_rollout(const E eq, const DevConsts<T> c,
                                                 const RolloutArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(a.B);
  const int64_t B = a.B;
  const int64_t row = lc.b * D + lc.p * M;
  T x[M];
#pragma unroll
  for (int m = 0; m < M; ++m) x[m] = a.x0[row + m];
  if (lc.live) {
#pragma unroll
    for (int m = 0; m < M; ++m) a.x[row + m] = x[m];
  }
  T acc = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) acc += x[m] * x[m];
  T S = Lanes<P>::sum(acc);
  int flag = SCHEME == DPAC_SCHEME_ADAPTIVE ? adaptive_flag(sqrt(S), c) : 1;
  T disc = 1, y = 0;
  const uint64_t gtraj = (uint64_t)(a.traj_offset + lc.b);

  auto load = [&](int t, DwFrame<T, M>& fr) {
    if constexpr (PHILOX) {
      if constexpr (P == 1) {
        constexpr int R = lanes_for_dim(D), C = D / R;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          T tmp[C];
          draw_chunk<T, D, C>(a.seed, gtraj, t, r, a.sample_type, tmp);
#pragma unroll
          for (int i = 0; i < C; ++i) fr.dw[r * C + i] = tmp[i];
        }
      } else {
        static_assert(lanes_for_dim(D) == P, "RNG chunking follows the lane split");
        draw_chunk<T, D, M>(a.seed, gtraj, t, lc.p, a.sample_type, fr.dw);
      }
    } else {
      const T* src = a.dw + ((int64_t)t * B) * D + row;
#pragma unroll
      for (int m = 0; m < M; ++m) fr.dw[m] = src[m];
    }
  };
  auto body = [&](int t, DwFrame<T, M>& fr) {
    T u[MC];
    eq.u_true(x, S, u);
    Transition<T, E, SCHEME> tr;
    tr.run(eq, c, x, u, fr.dw, flag, S);
    const T cf = (T)tr.coef;
    if constexpr (COST) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
      y += cost_increment<T, ORDER>(w, cf, tr.dt, disc);
      disc = disc * disc_factor(tr.dt, cf, c);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = x[m] + tr.dx[m] * cf;  // x + delta_x*coef (:67, :103)
    if (tr.coef) S = tr.St;
    flag = tr.flag_new;
    if (lc.live) {
      T* xo = a.x + ((int64_t)(t + 1) * B) * D + row;
#pragma unroll
      for (int m = 0; m < M; ++m) xo[m] = x[m];
      if (a.u) {
        T* uo = a.u + ((int64_t)t * B + lc.b) * (MC * P) + lc.p * MC;
#pragma unroll
        for (int m = 0; m < MC; ++m) uo[m] = u[m];
      }
      const int64_t o = (int64_t)t * B + lc.b;
      if constexpr (P == 1) {
        a.dt[o] = tr.dt;
        a.coef[o] = cf;
      } else {
        if (lc.p == 0) a.dt[o] = tr.dt;
        if (lc.p == 1) a.coef[o] = cf;
      }
    }
  };
  pipelined<KB, DwFrame<T, M>>(a.N, load, body);
  if constexpr (COST) {
    if (lc.live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}

// ---------------------------------------------------------------------------
// Flag initialisation (adaptive: equation.py:78-82; naive: np.ones, :52)
// ---------------------------------------------------------------------------
template <typename T, class E, int D, int SCHEME>
__global__ __launch_bounds__(64) void k_flag_init(const E eq, const DevConsts<T> c,
                                                   int64_t B, const T* x0, int32_t* flag) {
  constexpr int P = E::kP, M = E::M;
  const LaneCoord<P> lc(B);
  const int64_t row = lc.b * D + lc.p * M;
  T acc = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) acc += x0[row + m] * x0[row + m];
  const T S = Lanes<P>::sum(acc);
  if (lc.live && lc.p == 0)
    flag[lc.b] = SCHEME == DPAC_SCHEME_ADAPTIVE ? adaptive_flag(sqrt(S), c) : 1;
}

// ---------------------------------------------------------------------------
// One transition with an external control (NN actor), fused cost/discount.
// ---------------------------------------------------------------------------
template <typename T>
struct StepArgs {
  int64_t B;
  const T *x, *u, *dw, *disc_in, *y_in;
  const int32_t* flag_in;
  T *x_out, *disc_out, *y_out, *dt, *coef;
  int32_t* flag_out;
  // backward
  const T *g_x_out, *g_disc_out, *g_y_out;
  T *g_x, *g_u, *g_disc;
};

template <typename T, class E, int D, int SCHEME, int ORDER>
__global__ __launch_bounds__(64) void k_step_fwd(const E eq, const DevConsts<T> c,
                                                  const StepArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(a.B);
  const int64_t row = lc.b * D + lc.p * M;
  const int64_t urow = lc.b * (MC * P) + lc.p * MC;
  T x[M], u[MC], dw[M];
  T acc = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    x[m] = a.x[row + m];
    dw[m] = a.dw[row + m];
    acc += x[m] * x[m];
  }
#pragma unroll
  for (int m = 0; m < MC; ++m) u[m] = a.u[urow + m];
  const T S = Lanes<P>::sum(acc);
  const int flag = a.flag_in[lc.b];
  const T disc = a.disc_in ? a.disc_in[lc.b] : T(1);
  Transition<T, E, SCHEME> tr;
  tr.run(eq, c, x, u, dw, flag, S);
  const T cf = (T)tr.coef;
  const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
  if (!lc.live) return;  // after the last cross-lane op
#pragma unroll
  for (int m = 0; m < M; ++m) a.x_out[row + m] = x[m] + tr.dx[m] * cf;
  if (lc.p == 0) {
    const T yin = a.y_in ? a.y_in[lc.b] : T(0);
    if (a.y_out) a.y_out[lc.b] = yin + cost_increment<T, ORDER>(w, cf, tr.dt, disc);
    if (a.disc_out) a.disc_out[lc.b] = disc * disc_factor(tr.dt, cf, c);
    if (a.dt) a.dt[lc.b] = tr.dt;
    if (a.coef) a.coef[lc.b] = cf;
    a.flag_out[lc.b] = tr.flag_new;
  }
}

// VJP of k_step_fwd.  Derivation: with lam = dL/dx', E = exp(-g dt c),
//   dL/ddisc = g_disc'*E + g_y'*c*w*dt
//   dL/ddt   = g_disc'*disc*E*(-g*c) + g_y'*c*w*disc + c*Σ_j lam_j*(f_j + s_j dw_j/(2 sqrt(dt)))
//   dL/du    = c*dt*lam·∂f/∂u + c*sqrt(dt)*(lam⊙dw)·∂s/∂u + g_y'*c*dt*disc*∂w/∂u
//   dL/dx    = lam + (same three terms w.r.t. x) + dL/ddt * ∂dt/∂x
//   ∂dt/∂x   = -2(R-r)x/(r*den) if flag == 1 and dt_raw >= 1e-4 dt0 (TF max tie rule), else 0
template <typename T, class E, int D, int SCHEME, int ORDER>
__global__ __launch_bounds__(64) void k_step_bwd(const E eq, const DevConsts<T> c,
                                                  const StepArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(a.B);
  const int64_t row = lc.b * D + lc.p * M;
  const int64_t urow = lc.b * (MC * P) + lc.p * MC;
  T x[M], u[MC], dw[M], lam[M];
  T acc = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    x[m] = a.x[row + m];
    dw[m] = a.dw[row + m];
    lam[m] = a.g_x_out[row + m];
    acc += x[m] * x[m];
  }
#pragma unroll
  for (int m = 0; m < MC; ++m) u[m] = a.u[urow + m];
  const T S = Lanes<P>::sum(acc);
  const int flag = a.flag_in[lc.b];
  const T disc = a.disc_in ? a.disc_in[lc.b] : T(1);
  const T gD1 = a.g_disc_out ? a.g_disc_out[lc.b] : T(0);
  const T gy1 = a.g_y_out ? a.g_y_out[lc.b] : T(0);

  Transition<T, E, SCHEME> tr;
  tr.run(eq, c, x, u, dw, flag, S);
  const T cf = (T)tr.coef;
  const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
  const T Ef = disc_factor(tr.dt, cf, c);

  T f[M], s[M];
  eq.drift(x, u, S, f);
  eq.sigma(x, u, s);
  T gx[M], gu[MC], a_f[M], a_s[M];
  T part = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    gx[m] = lam[m];
    a_f[m] = lam[m] * cf * tr.dt;
    a_s[m] = lam[m] * cf * tr.sq * dw[m];
    part += lam[m] * (f[m] + s[m] * dw[m] / (2 * tr.sq));
  }
#pragma unroll
  for (int m = 0; m < MC; ++m) gu[m] = 0;
  eq.drift_vjp(x, u, S, a_f, gx, gu);
  eq.sigma_vjp(x, u, a_s, gx, gu);
  const T gw = gy1 * cf * tr.dt * disc;
  eq.w_vjp(x, u, gw, gx, gu);
  const T g_disc = gD1 * Ef + gy1 * cf * w * tr.dt;
  if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
    const T g_dt = gD1 * disc * Ef * (c.neg_gamma * cf) + gy1 * cf * w * disc +
                   cf * Lanes<P>::sum(part);
    const T r = sqrt(S);
    const T raw = adaptive_dt_raw(flag, r, c);
    if (flag == 1 && raw >= c.dt_min) {
      const T k = g_dt * (-2 * (c.R - r) / c.den) / r;
#pragma unroll
      for (int m = 0; m < M; ++m) gx[m] += k * x[m];
    }
  }
  if (!lc.live) return;
#pragma unroll
  for (int m = 0; m < M; ++m) a.g_x[row + m] = gx[m];
#pragma unroll
  for (int m = 0; m < MC; ++m) a.g_u[urow + m] = gu[m];
  if (a.g_disc && lc.p == 0) a.g_disc[lc.b] = g_disc;
}

// ---------------------------------------------------------------------------
// TD target assembly over a finished trajectory (solver.py:166-190) and its
// backward with respect to G.
// ---------------------------------------------------------------------------
template <typename T>
struct TdArgs {
  int64_t B, traj_offset;
  int N, sample_type;
  uint64_t seed;
  const T *x, *u, *dw, *dt, *coef, *G, *g_y;
  T *y, *disc, *g_G;
};

template <typename T, int M, int MC, bool HAS_G>
struct TdFrame {
  T x[M], u[MC], dw[M], G[HAS_G ? M : 1];
  T dt, coef;
};

template <typename T, class E, int D, bool TD1, bool PHILOX, int ORDER, bool BWD>
__device__ __forceinline__ void td_common(const E& eq, const DevConsts<T>& c,
                                          const TdArgs<T>& a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  constexpr bool HAS_G = TD1 && !BWD;
  constexpr int KB = sizeof(T) == 4 ? 4 : 2;
  using F = TdFrame<T, M, MC, HAS_G>;
  const LaneCoord<P> lc(a.B);
  const int64_t B = a.B;
  const int64_t row = lc.b * D + lc.p * M;
  const int64_t urow = lc.b * (MC * P) + lc.p * MC;
  const uint64_t gtraj = (uint64_t)(a.traj_offset + lc.b);
  T disc = 1, y = 0;
  const T gy = BWD ? a.g_y[lc.b] : T(0);

  auto load = [&](int t, F& fr) {
    const int64_t so = (int64_t)t * B;
#pragma unroll
    for (int m = 0; m < M; ++m) fr.x[m] = a.x[so * D + row + m];
#pragma unroll
    for (int m = 0; m < MC; ++m) fr.u[m] = a.u[so * (MC * P) + urow + m];
    if constexpr (TD1 || BWD) {
      if constexpr (PHILOX) {
        if constexpr (P == 1) {
          constexpr int R = lanes_for_dim(D), C = D / R;
#pragma unroll
          for (int r = 0; r < R; ++r) {
            T tmp[C];
            draw_chunk<T, D, C>(a.seed, gtraj, t, r, a.sample_type, tmp);
#pragma unroll
            for (int i = 0; i < C; ++i) fr.dw[r * C + i] = tmp[i];
          }
        } else {
          draw_chunk<T, D, M>(a.seed, gtraj, t, lc.p, a.sample_type, fr.dw);
        }
      } else {
#pragma unroll
        for (int m = 0; m < M; ++m) fr.dw[m] = a.dw[so * D + row + m];
      }
    }
    if constexpr (HAS_G) {
#pragma unroll
      for (int m = 0; m < M; ++m) fr.G[m] = a.G[so * D + row + m];
    }
    fr.dt = a.dt[so + lc.b];
    fr.coef = a.coef[so + lc.b];
  };
  auto body = [&](int t, F& fr) {
    if constexpr (!BWD) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(fr.x, fr.u)));
      y += cost_increment<T, ORDER>(w, fr.coef, fr.dt, disc);
    }
    if constexpr (TD1 || BWD) {
      T s[M];
      eq.sigma(fr.x, fr.u, s);
      if constexpr (BWD) {
        // d y / d G_j = -disc*coef*sqrt(dt)*diff_j ; g_G = g_y * that
        const T k = -gy * (disc * (fr.coef * sqrt(fr.dt)));
        if (lc.live) {
          T* go = a.g_G + (int64_t)t * B * D + row;
#pragma unroll
          for (int m = 0; m < M; ++m) go[m] = k * (s[m] * fr.dw[m]);
        }
      } else {
        T acc = 0;
#pragma unroll
        for (int m = 0; m < M; ++m) acc += (s[m] * fr.dw[m]) * fr.G[m];
        const T dot = Lanes<P>::sum(acc);
        y -= (dot * disc) * (fr.coef * sqrt(fr.dt));  // solver.py:180-184
      }
    }
    disc = disc * disc_factor(fr.dt, fr.coef, c);
  };
  pipelined<KB, F>(a.N, load, body);
  if constexpr (!BWD) {
    if (lc.live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}

template <typename T, class E, int D, bool TD1, bool PHILOX, int ORDER>
__global__ __launch_bounds__(64) void k_td_fwd(const E eq, const DevConsts<T> c,
                                                const TdArgs<T> a) {
  td_common<T, E, D, TD1, PHILOX, ORDER, false>(eq, c, a);
}

template <typename T, class E, int D, bool PHILOX>
__global__ __launch_bounds__(64) void k_td_bwd(const E eq, const DevConsts<T> c,
                                                const TdArgs<T> a) {
  td_common<T, E, D, true, PHILOX, DPAC_COST_CRITIC, true>(eq, c, a);
}

// ---------------------------------------------------------------------------
// Row-wise evaluation of one Equation method (parity tests, metrics).  One row
// per lane group as in every other kernel.
// ---------------------------------------------------------------------------
template <typename T, class E, int D>
__global__ __launch_bounds__(64) void k_eval(const E eq, const DevConsts<T> c, int64_t B,
                                              int what, const T* x, const T* u, T* out) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(B);
  const int64_t row = lc.b * D + lc.p * M;
  const int64_t urow = lc.b * (MC * P) + lc.p * MC;
  T xv[M], uv[MC];
  T acc = 0;
#pragma unroll
  for (int m = 0; m < M; ++m) {
    xv[m] = x[row + m];
    acc += xv[m] * xv[m];
  }
  const bool has_u = u != nullptr;
#pragma unroll
  for (int m = 0; m < MC; ++m) uv[m] = has_u ? u[urow + m] : T(0);
  const T S = Lanes<P>::sum(acc);
  T v[M];
  T scalar = 0;
  bool vec = false, ctl = false;
  switch (what) {
    case DPAC_EVAL_DRIFT: eq.drift(xv, uv, S, v); vec = true; break;
    case DPAC_EVAL_SIGMA: eq.sigma(xv, uv, v); vec = true; break;
    case DPAC_EVAL_W: scalar = eq.w_finish(Lanes<P>::sum(eq.w_part(xv, uv))); break;
    case DPAC_EVAL_Z: scalar = eq.Z(xv, S); break;
    case DPAC_EVAL_V_TRUE: scalar = eq.V_true(xv, S); break;
    case DPAC_EVAL_U_TRUE: {
      T uu[MC];
      eq.u_true(xv, S, uu);
      if (lc.live) {
#pragma unroll
        for (int m = 0; m < MC; ++m) out[urow + m] = uu[m];
      }
      ctl = true;
      break;
    }
    case DPAC_EVAL_V_GRAD: eq.V_grad(xv, S, v); vec = true; break;
    case DPAC_EVAL_B: scalar = S - c.R2; break;
    default: break;
  }
  if (!lc.live || ctl) return;
  if (vec) {
#pragma unroll
    for (int m = 0; m < M; ++m) out[row + m] = v[m];
  } else if (lc.p == 0) {
    out[lc.b] = scalar;
  }
}

// ---------------------------------------------------------------------------
// Launcher for one (T, equation functor, D).
// ---------------------------------------------------------------------------
inline dim3 grid_for(int64_t B, int P) {
  const int64_t per = 64 / P;
  return dim3((unsigned)((B + per - 1) / per));
}

template <typename T, class E, int D>
int run_op(const OpArgs& a) {
  const E eq = E::make(a.eq);
  const DevConsts<T> c = DevConsts<T>::make(host_consts(a));
  constexpr int P = E::kP;
  const dim3 grid = grid_for(a.B, P), block(64);
  hipStream_t s = a.stream;
  const bool adaptive = a.scheme == DPAC_SCHEME_ADAPTIVE;
  const bool actor = a.cost_order == DPAC_COST_ACTOR;
  switch (a.op) {
    case OP_ROLLOUT: {
      RolloutArgs<T> r;
      r.B = a.B; r.traj_offset = a.traj_offset; r.N = a.N; r.sample_type = a.sample_type;
      r.seed = a.seed;
      r.x0 = (const T*)a.x0; r.dw = (const T*)a.dw;
      r.x = (T*)a.x_out; r.dt = (T*)a.dt; r.coef = (T*)a.coef; r.u = (T*)a.u_out;
      r.y = (T*)a.y; r.disc = (T*)a.disc;
      const bool philox = a.dw == nullptr, cost = a.y != nullptr;
      constexpr int KB = sizeof(T) == 4 ? 8 : 4;
#define DPAC_ROLL(SCH, PH, CO, ORD) \
  hipLaunchKernelGGL((k_rollout<T, E, D, SCH, PH, CO, ORD, KB>), grid, block, 0, s, eq, c, r)
#define DPAC_ROLL_SCH(SCH)                                          \
  if (philox) {                                                     \
    if (!cost) DPAC_ROLL(SCH, true, false, 0);                      \
    else if (actor) DPAC_ROLL(SCH, true, true, DPAC_COST_ACTOR);    \
    else DPAC_ROLL(SCH, true, true, DPAC_COST_CRITIC);              \
  } else {                                                          \
    if (!cost) DPAC_ROLL(SCH, false, false, 0);                     \
    else if (actor) DPAC_ROLL(SCH, false, true, DPAC_COST_ACTOR);   \
    else DPAC_ROLL(SCH, false, true, DPAC_COST_CRITIC);             \
  }
      if (adaptive) { DPAC_ROLL_SCH(DPAC_SCHEME_ADAPTIVE) } else { DPAC_ROLL_SCH(DPAC_SCHEME_NAIVE) }
#undef DPAC_ROLL_SCH
#undef DPAC_ROLL
      break;
    }
    case OP_FLAG_INIT:
      if (adaptive)
        hipLaunchKernelGGL((k_flag_init<T, E, D, DPAC_SCHEME_ADAPTIVE>), grid, block, 0, s, eq, c,
                           a.B, (const T*)a.x0, a.flag_out);
      else
        hipLaunchKernelGGL((k_flag_init<T, E, D, DPAC_SCHEME_NAIVE>), grid, block, 0, s, eq, c,
                           a.B, (const T*)a.x0, a.flag_out);
      break;
    case OP_STEP_FWD:
    case OP_STEP_BWD: {
      StepArgs<T> st;
      st.B = a.B;
      st.x = (const T*)a.x; st.u = (const T*)a.u; st.dw = (const T*)a.dw;
      st.disc_in = (const T*)a.disc_in; st.y_in = (const T*)a.y_in; st.flag_in = a.flag_in;
      st.x_out = (T*)a.x_out; st.disc_out = (T*)a.disc_out; st.y_out = (T*)a.y_out;
      st.dt = (T*)a.dt; st.coef = (T*)a.coef; st.flag_out = a.flag_out;
      st.g_x_out = (const T*)a.g_x_out; st.g_disc_out = (const T*)a.g_disc_out;
      st.g_y_out = (const T*)a.g_y_out;
      st.g_x = (T*)a.g_x; st.g_u = (T*)a.g_u; st.g_disc = (T*)a.g_disc;
#define DPAC_STEP(K, SCH, ORD) hipLaunchKernelGGL((K<T, E, D, SCH, ORD>), grid, block, 0, s, eq, c, st)
#define DPAC_STEP_K(K)                                                   \
  if (adaptive) {                                                        \
    if (actor) DPAC_STEP(K, DPAC_SCHEME_ADAPTIVE, DPAC_COST_ACTOR);      \
    else DPAC_STEP(K, DPAC_SCHEME_ADAPTIVE, DPAC_COST_CRITIC);           \
  } else {                                                               \
    if (actor) DPAC_STEP(K, DPAC_SCHEME_NAIVE, DPAC_COST_ACTOR);         \
    else DPAC_STEP(K, DPAC_SCHEME_NAIVE, DPAC_COST_CRITIC);              \
  }
      if (a.op == OP_STEP_FWD) { DPAC_STEP_K(k_step_fwd) } else { DPAC_STEP_K(k_step_bwd) }
#undef DPAC_STEP_K
#undef DPAC_STEP
      break;
    }
    case OP_TD_FWD:
    case OP_TD_BWD: {
      TdArgs<T> td;
      td.B = a.B; td.traj_offset = a.traj_offset; td.N = a.N; td.sample_type = a.sample_type;
      td.seed = a.seed;
      td.x = (const T*)a.x; td.u = (const T*)a.u; td.dw = (const T*)a.dw;
      td.dt = (const T*)a.dt_in; td.coef = (const T*)a.coef_in; td.G = (const T*)a.G;
      td.g_y = (const T*)a.g_y_out;
      td.y = (T*)a.y; td.disc = (T*)a.disc; td.g_G = (T*)a.g_G;
      const bool philox = a.dw == nullptr;
      if (a.op == OP_TD_BWD) {
        if (philox) hipLaunchKernelGGL((k_td_bwd<T, E, D, true>), grid, block, 0, s, eq, c, td);
        else hipLaunchKernelGGL((k_td_bwd<T, E, D, false>), grid, block, 0, s, eq, c, td);
      } else {
        const bool td1 = a.td_type == DPAC_TD1;
#define DPAC_TD(TD1, PH, ORD) hipLaunchKernelGGL((k_td_fwd<T, E, D, TD1, PH, ORD>), grid, block, 0, s, eq, c, td)
        if (td1) {
          if (philox) { if (actor) DPAC_TD(true, true, DPAC_COST_ACTOR); else DPAC_TD(true, true, DPAC_COST_CRITIC); }
          else { if (actor) DPAC_TD(true, false, DPAC_COST_ACTOR); else DPAC_TD(true, false, DPAC_COST_CRITIC); }
        } else {
          if (actor) DPAC_TD(false, false, DPAC_COST_ACTOR); else DPAC_TD(false, false, DPAC_COST_CRITIC);
        }
#undef DPAC_TD
      }
      break;
    }
    case OP_EVAL:
      hipLaunchKernelGGL((k_eval<T, E, D>), grid, block, 0, s, eq, c, a.B, a.what,
                         (const T*)a.x, (const T*)a.u, (T*)a.out);
      break;
    default:
      return DPAC_EINVAL;
  }
  return (int)hipGetLastError();
}

// Dispatch over the compiled dimensions of one equation family for one dtype.
// EQ<T, D> is the functor with its lane split already chosen.
template <template <typename, int> class EQ, int... Ds>
struct DimList {
  template <typename T, int D0, int... Rest>
  static int go(const OpArgs& a) {
    if (a.eq.dim == D0) return run_op<T, EQ<T, D0>, D0>(a);
    if constexpr (sizeof...(Rest) > 0) return go<T, Rest...>(a);
    return DPAC_EUNSUP;
  }
  template <typename T>
  static int dispatch(const OpArgs& a) {
    return go<T, Ds...>(a);
  }
  static bool has(int d) { return ((d == Ds) || ...); }
};

}  // namespace dpac
