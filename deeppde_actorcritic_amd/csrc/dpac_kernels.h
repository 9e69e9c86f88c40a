// dpac_kernels.h — kernel templates of libdpac and the per-equation launcher.
//
// Mapping: a trajectory is owned by P = E::kP consecutive lanes of a 64-wide
// wavefront, each lane holding M = d/P state components in registers.
//  * k_rollout: one wavefront per workgroup, the whole time loop in-kernel, so a
//    trajectory's state never leaves registers between steps; HBM traffic is
//    exactly what the reference materialises (x_smp, dt, coef: equation.py:63-70,
//    97-104).  Per-step increments are prefetched 2*KB steps ahead (pipelined()).
//  * k_td: the TD sums have no state dependence, only the discount product is
//    sequential; 4 wavefronts per workgroup split the horizon into 4 chunks and
//    combine (local sum, local discount) pairs in LDS.
//  * k_step_fwd / k_step_bwd / k_flag_init / k_eval: one row per lane group.
// Floating-point contraction is off (-ffp-contract=off); the fused multiply-adds
// are written out, so every kernel variant rounds identically.
#pragma once

#include <cmath>
#include <type_traits>
#include <utility>

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
  OP_ROLLOUT_NN,
  OP_ROLLOUT_NN_BWD,
};

// Bytes per 16-row tile of the sign-bit mask (FwdEpiM): 13 16-column tiles per hidden layer
// (the fast path's 193..208-wide layers), 64 bytes each.
inline int nn_mask_tile_bytes(int n_hidden) { return 13 * 64 * n_hidden; }

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
  dpac_mlp mlp;                  // OP_ROLLOUT_NN: the actor MLP
  void *save_z, *save_disc;      // OP_ROLLOUT_NN: optional backward saves
  int32_t* save_flag;
  uint8_t* save_mask;            // OP_ROLLOUT_NN: optional sign-bit mask (fast path only)
  int32_t* mask_written;         // OP_ROLLOUT_NN: host flag, 1 if the mask was written
  const uint8_t* mask_in;        // OP_ROLLOUT_NN_BWD: the forward's mask, or null
  const void* mlp_wt[DPAC_MLP_MAX_HIDDEN + 1];  // OP_ROLLOUT_NN_BWD: (W_i diag s_{i+1})^T
  hipStream_t stream;
};

inline HostConsts host_consts(const OpArgs& a) {
  HostConsts h;
  const double d = a.eq.dim;
  h.gamma = a.eq.gamma;
  h.R = a.eq.R;
  h.sigma_up = a.eq.sigma_up;
  h.dt0 = a.T / a.N;                                       // delta_t = T / N (:48, :75)
  h.sqrt_dt0 = std::sqrt(h.dt0);                           // np.sqrt(delta_t) (:49)
  h.dt_min = h.dt0 * 1e-4;                                 // delta_t*1e-4 (:86)
  h.den = 3 * a.eq.dim * (a.eq.sigma_up * a.eq.sigma_up);  // 3*dim*sigma_Up**2 (:85)
  h.c_layer = a.eq.sigma_up * std::sqrt(3 * d * h.dt0);    // sigma_Up*sqrt(3*dim*dt) (:80, :94)
  h.R2 = a.eq.R * a.eq.R;                                  // R**2 (:122)
  return h;
}

template <typename T>
struct DevConsts {
  T gamma, R, dt0, sqrt_dt0, dt_min, inv_den, two_inv_den, c_layer, R2, neg_gamma;
  static DevConsts make(const HostConsts& h) {
    DevConsts c;
    c.gamma = (T)h.gamma; c.R = (T)h.R; c.dt0 = (T)h.dt0; c.sqrt_dt0 = (T)h.sqrt_dt0;
    c.dt_min = (T)h.dt_min; c.inv_den = (T)(1.0 / h.den); c.two_inv_den = (T)(2.0 / h.den);
    c.c_layer = (T)h.c_layer; c.R2 = (T)h.R2; c.neg_gamma = (T)(-h.gamma);
    return c;
  }
};

// Prefetch depth (steps per half ring) of the time loops.  The ring of 2*KB
// frames gets a fixed VGPR budget, so wide per-lane frames (VDP keeps the whole
// state in one lane) get a shallow ring instead of spilling: KB = 8 (f32) /
// 4 (f64) for the canonical d = 20 rollout frame of 2 values.
#ifndef DPAC_RING_VGPRS
#define DPAC_RING_VGPRS 32
#endif
#ifndef DPAC_ROLLOUT_KB_CAP
#define DPAC_ROLLOUT_KB_CAP 8
#endif
// Cache-policy immediates of k_rollout's streamed dw loads and x stores (0 = default,
// 2 = nt).  Measured with 5 rotating buffer sets (HBM, not Infinity-Cache resident):
// nt x stores 39.8 -> 38.0 us at B = 4096, 146 -> 131 us at 16384; nt dw loads no gain.
#ifndef DPAC_ROLLOUT_DW_AUX
#define DPAC_ROLLOUT_DW_AUX 0
#endif
#ifndef DPAC_ROLLOUT_X_AUX
#define DPAC_ROLLOUT_X_AUX 2
#endif
// KB = 0 (a frame larger than half the budget): no ring, each step loads its
// own frame right before computing.
constexpr int ring_kb(int frame_bytes, int budget_vgprs, int cap) {
  const int kb = budget_vgprs * 4 / (2 * frame_bytes);
  return kb > cap ? cap : kb;
}
// k_rollout's ring: its dt/coef flush writes F = min(P, 2*KB) steps at compile-time
// phases of the 2*KB-step period, so F must divide 2*KB and be a power of two (P is).
// Round KB down to the nearest value that keeps that: a multiple of P/2 when 2*KB >= P
// (F = P), else a power of two (F = 2*KB).  E.g. P = 8, M = 3: 5 -> 4; P = 4, M = 5: 3 -> 2.
constexpr int rollout_kb(int kb, int P) {
  if (kb < 1) kb = 1;
  if (2 * kb >= P) return kb - kb % (P / 2 > 0 ? P / 2 : 1);
  int p2 = 1;
  while (p2 * 2 <= kb) p2 *= 2;
  return p2;
}
// Timing-only ablations (never in a shipped build): 1 = skip the per-step
// stores of x/dt/coef, 2 = synthesize dw instead of loading it, 3 = skip the
// dt/coef stores, 4 = skip the x stores.
#ifndef DPAC_ABLATE
#define DPAC_ABLATE 0
#endif


// sqrt: the hardware v_sqrt_f32 for float (1 ulp), correctly rounded for double.
__device__ __forceinline__ float dsqrt(float v) { return __builtin_amdgcn_sqrtf(v); }
__device__ __forceinline__ double dsqrt(double v) { return sqrt(v); }

// ---------------------------------------------------------------------------
// Software-pipelined time loop over [t_begin, t_end): frames for KB steps are
// loaded while the previous KB steps compute.  Frame arrays are indexed only by
// unrolled constants, so they live in VGPRs.  body(t, frame, phase) receives
// phase = (t - t_begin) mod 2*KB as a compile-time constant wherever the
// unrolled position fixes it, and Phase<-1> in the scalar tail loop.
// ---------------------------------------------------------------------------
template <int V>
using Phase = std::integral_constant<int, V>;

// body(t + K, fr[K], Phase<BASE + K>) for K in the sequence; with CHECK,
// bodies with t + K >= t_end are skipped.
template <int BASE, bool CHECK, class F, class BodyF, int... K>
__device__ __forceinline__ void run_bodies(BodyF& body, int t, F* fr, int t_end,
                                           std::integer_sequence<int, K...>) {
  if constexpr (CHECK)
    ((t + K < t_end ? body(t + K, fr[K], Phase<BASE + K>{}) : void()), ...);
  else
    (body(t + K, fr[K], Phase<BASE + K>{}), ...);
}

template <int KB, class F, class LoadF, class BodyF>
__device__ __forceinline__ void pipelined(int t_begin, int t_end, LoadF&& load, BodyF&& body) {
  if (t_end <= t_begin) return;
  if constexpr (KB == 0) {
    for (int t = t_begin; t < t_end; ++t) {
      F f;
      load(t, f);
      body(t, f, Phase<-1>{});
    }
  } else {
    const int last = t_end - 1;
    F A[KB], Bq[KB];
    // Loads are never predicated: a load past the end re-reads the last step (in
    // bounds, unused).  A predicated load would force its wait at the branch join
    // and serialise the prefetch.
#pragma unroll
    for (int k = 0; k < KB; ++k) load(min(t_begin + k, last), A[k]);
    int t0 = t_begin;
    for (; t0 + 2 * KB <= t_end; t0 += 2 * KB) {
#pragma unroll
      for (int k = 0; k < KB; ++k) load(t0 + KB + k, Bq[k]);
      run_bodies<0, false>(body, t0, A, t_end, std::make_integer_sequence<int, KB>{});
#pragma unroll
      for (int k = 0; k < KB; ++k) load(min(t0 + 2 * KB + k, last), A[k]);
      run_bodies<KB, false>(body, t0 + KB, Bq, t_end, std::make_integer_sequence<int, KB>{});
    }
    // remainder (< 2*KB steps): A holds steps [t0, t0+KB)
    run_bodies<0, true>(body, t0, A, t_end, std::make_integer_sequence<int, KB>{});
    for (int t = t0 + KB; t < t_end; ++t) {
      F f;
      load(t, f);
      body(t, f, Phase<-1>{});
    }
  }
}

// |v|^2 of the owned slice (fma chain; every kernel uses this one form so all
// variants round identically).
template <typename T, int M>
__device__ __forceinline__ T sumsq(const T (&v)[M]) {
  T q = v[0] * v[0];
#pragma unroll
  for (int m = 1; m < M; ++m) q = fma(v[m], v[m], q);
  return q;
}

// XCD-aware block order (cdna_hip_programming.md §5.5 T1): the dispatcher deals
// blocks round-robin over the 8 XCDs, so blocks b and b+1 — whose per-step rows
// share cache lines (4 trajectories x 80 B = 2.5 lines) — would be written back
// from two different L2s as partial lines.  Remap so that each XCD owns one
// contiguous run of trajectory blocks (bijective for any grid size).
__device__ __forceinline__ int64_t xcd_block(int64_t b, int64_t nb) {
  const int64_t q = nb / 8, r = nb % 8, x = b % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + b / 8;
}

// Lane coordinates: trajectory b and lane slot p within its group.  Lane groups
// past the end of the batch compute on a duplicate of the last trajectory and
// store the same values it does (identical bits), so no store needs a guard.
template <int P>
struct LaneCoord {
  int p;
  int64_t b;
  bool live;
  __device__ __forceinline__ LaneCoord(int64_t B, int lane, int64_t group0) {
    p = lane % P;
    b = group0 + lane / P;
    live = b < B;
    if (!live) b = B - 1;
  }
};

// Adaptive-scheme state of a trajectory as two lane masks: alive = flag > 0,
// layer = flag == 1 (equation.py:80-82: flag 2 inner, 1 boundary layer, 0 out).
struct Flags {
  bool alive, layer;
  __device__ __forceinline__ int encode() const { return alive ? (layer ? 1 : 2) : 0; }
  __device__ __forceinline__ static Flags decode(int f) { return Flags{f > 0, f == 1}; }
};

// Region of a point at radius r: 1 + floor((sign(R-r-c) + sign(R-r))/2) is
// 2 if R-r-c > 0, 1 if R-r > 0, else 0 (equation.py:80-82, :94-95).
template <typename T>
__device__ __forceinline__ Flags region(T r, const DevConsts<T>& c) {
  const T b = c.R - r;
  const bool inball = b > T(0);
  const bool inner = b - c.c_layer > T(0);
  return Flags{inball, inball && !inner};
}

// (2f-f^2)(R-r)^2/den + (f^2-2f+1)dt0 (equation.py:85) is (R-r)^2/den for f == 1
// and dt0 for f in {0, 2}; the division is a multiply by 1/den.
template <typename T>
__device__ __forceinline__ T adaptive_dt_raw(bool layer, T r, const DevConsts<T>& c) {
  const T b = c.R - r;
  return layer ? (b * b) * c.inv_den : c.dt0;
}

// One transition of the scheme for the owned slice.  In: x, u, dw (masked),
// flags and r = |x|.  Out: xt = x + dx, coef, next flags, St = |xt|^2, rt = |xt|
// (adaptive or norm-dependent equations), dt and sqrt(dt).
template <typename T, class E, int SCHEME>
struct Transition {
  static constexpr int M = E::M, MC = E::MC, P = E::kP;
  static constexpr bool kRadius = SCHEME == DPAC_SCHEME_ADAPTIVE || E::kNeedsNorm;
  T xt[M], dx[M];
  T dt, sq, St, rt;
  bool coef;
  Flags next;
  __device__ __forceinline__ void run(const E& eq, const DevConsts<T>& c, const T (&x)[M],
                                      const T (&u)[MC], const T (&dw)[M], Flags fl, T r) {
    if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
      // tf.maximum(dt_i, delta_t*1e-4) (:86): dt0 always exceeds the floor, so
      // only the boundary-layer branch is clamped (same bits, one instruction less)
      const T b = c.R - r;
      dt = fl.layer ? fmax((b * b) * c.inv_den, c.dt_min) : c.dt0;
      sq = dsqrt(dt);
    } else {
      dt = c.dt0;
      sq = c.sqrt_dt0;
    }
    T f[M], s[M];
    eq.drift(x, u, r, f);
    eq.sigma(x, u, s);
#pragma unroll
    for (int m = 0; m < M; ++m) {
      dx[m] = fma(f[m], dt, (s[m] * dw[m]) * sq);  // drift*dt + diffusion*sqrt(dt) (:58, :91)
      xt[m] = x[m] + dx[m];
    }
    St = Lanes<P>::sum(sumsq(xt));
    rt = kRadius ? dsqrt(St) : T(0);
    if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
      const Flags nf = region(rt, c);
      coef = fl.alive && nf.alive;                 // sign(flag)*sign(new_flag) (:96)
      next = Flags{coef, coef && nf.layer};        // new_flag*sign(flag) (:95)
    } else {
      const bool out = St - c.R2 >= T(0);         // ceil((sign(b(x))+1)/2) == 1 (:60-61)
      coef = fl.alive && !out;                    // flag*(1-Exit) (:62)
      next = Flags{coef, false};                  // flag *= 1 - Exit (:69)
    }
  }
};

template <typename T>
__device__ __forceinline__ T cost_increment(int order, T w, T coef, T dt, T disc) {
  return order == DPAC_COST_ACTOR ? ((coef * w) * dt) * disc   // coef*w*dt*discount (solver.py:218)
                                  : (w * disc) * (coef * dt);  // (w*discount)*(coef*dt) (:170-174)
}

template <typename T>
__device__ __forceinline__ T disc_factor(T dt, T coef, const DevConsts<T>& c) {
  return exp((c.neg_gamma * dt) * coef);  // exp(-gamma*dt*coef) (solver.py:187, :219)
}

// The increments of this lane's components at step t (in-kernel Philox).
template <typename T, class E, int D>
__device__ __forceinline__ void draw_owned(uint64_t seed, uint64_t gtraj, int t, int p,
                                           int sample_type, T (&out)[E::M]) {
  if constexpr (E::kP == 1) {
    draw_all<T, D>(seed, gtraj, t, sample_type, out);
  } else {
    static_assert(lanes_for_dim(D) == E::kP && comps_per_lane(D) == E::M,
                  "RNG slots follow the lane split");
    draw_slot<T, D>(seed, gtraj, t, p, sample_type, out);
  }
}

// ---------------------------------------------------------------------------
// Fused rollout with the analytic control u_true (reference `cheat` path).
// ---------------------------------------------------------------------------
template <typename T>
struct RolloutArgs {
  int64_t B, traj_offset;
  int N, sample_type, cost_order;
  uint64_t seed;
  const T* x0;
  const T* dw;
  T *x, *dt, *coef, *u, *y, *disc;
};

template <typename T, int M>
struct DwFrame {
  T dw[M];
};

// Optional outputs of k_rollout (template bits, so the time loop never tests them).
enum : int { kOutCost = 1, kOutU = 2 };

template <typename T, class E, int D, int SCHEME, bool PHILOX, int OUT, int KB>
__global__ __launch_bounds__(64) void k_rollout(const E eq, const DevConsts<T> c,
                                                 const RolloutArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  constexpr bool COST = (OUT & kOutCost) != 0, WANT_U = (OUT & kOutU) != 0;
  // dt / coef rows are trajectory-major [B][N] (the reference's dt[B,N]): lane
  // group keeps its last F steps in a lane shift register (lane p: step t - p,
  // dt with the sign of coef) and writes the F values of its row at once every
  // F steps (F divides the pipeline period 2*KB, so each unrolled body knows at
  // compile time whether it flushes).
  constexpr int F = P < 2 * KB ? P : 2 * KB;
  static_assert(KB >= 1 && (2 * KB) % F == 0 && (F & (F - 1)) == 0,
                "the dt/coef flush needs F | 2*KB and F a power of two (rollout_kb)");
  using TR = Transition<T, E, SCHEME>;
  const LaneCoord<P> lc(a.B, threadIdx.x, xcd_block(blockIdx.x, gridDim.x) * (64 / P));
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  const BufSlab<T, D, P> sx(own, lc.b, lc.live);           // x0, dw[t], x[t] rows
  const BufSlab<T, E::CDIM, P> su(ownu, lc.b, lc.live);    // u[t] rows
  // whole-array descriptors (host: every array < 2 GiB); the step goes in soffset
  const uint32_t slab = (uint32_t)(a.B * D * sizeof(T));
  const uint32_t slab_u = (uint32_t)(a.B * E::CDIM * sizeof(T));
  const uint32_t row_bytes = (uint32_t)(a.N * sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(a.x, slab * (uint32_t)(a.N + 1));
  const __amdgpu_buffer_rsrc_t rs_dw = make_rsrc(a.dw, PHILOX ? 0u : slab * (uint32_t)a.N);
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(a.u, WANT_U ? slab_u * (uint32_t)a.N : 0u);
  const __amdgpu_buffer_rsrc_t rs_dt = make_rsrc(a.dt, (uint32_t)a.B * row_bytes);
  const __amdgpu_buffer_rsrc_t rs_cf = make_rsrc(a.coef, (uint32_t)a.B * row_bytes);
  T keep = 0;  // coef_t ? dt_t : -dt_t (dt > 0 always) of step t_last - p
  auto flush = [&](int t_last, int count) {  // steps (t_last - count, t_last] of the row
    const uint32_t off = (lc.live && lc.p < count)
                             ? (uint32_t)((lc.b * a.N + t_last - lc.p) * (int64_t)sizeof(T)) : kOOB;
    buf_store_scalar<T>(rs_dt, off, fabs(keep));
    buf_store_scalar<T>(rs_cf, off, keep > T(0) ? T(1) : T(0));
  };

  T x[M];
  sx.load(make_rsrc(a.x0, slab), x);
  sx.store(rs_x, x);
  T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  Flags fl = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c) : Flags{true, false};
  T disc = 1, y = 0;
  const uint64_t gtraj = (uint64_t)(a.traj_offset + lc.b);

  // in-kernel Philox, paired layout (dpac_device.h): the even step of a pair draws both steps'
  // increments; the odd step takes the half kept here (loads come in step order: pipelined())
  constexpr bool kPairable = PHILOX && E::kP > 1 && 2 * M <= 4;
  const bool paired = kPairable && dw_steps_per_block<T>(M, a.sample_type) == 2;
  T pend[M];
#pragma unroll
  for (int m = 0; m < M; ++m) pend[m] = T(0);
  auto load = [&](int t, DwFrame<T, M>& fr) {
    if constexpr (PHILOX) {
      if constexpr (kPairable) {
        if (paired) {
          if ((t & 1) == 0) {
            T v[2 * M];
            draw_slot_pair<T, D>(a.seed, gtraj, t >> 1, lc.p, a.sample_type, v);
#pragma unroll
            for (int m = 0; m < M; ++m) {
              fr.dw[m] = v[m];
              pend[m] = v[M + m];
            }
          } else {
#pragma unroll
            for (int m = 0; m < M; ++m) fr.dw[m] = pend[m];
          }
          return;
        }
      }
      draw_owned<T, E, D>(a.seed, gtraj, t, lc.p, a.sample_type, fr.dw);
    } else if constexpr (DPAC_ABLATE == 2 || DPAC_ABLATE == 5) {
#pragma unroll
      for (int m = 0; m < M; ++m) fr.dw[m] = T(((t * 7 + m + lc.p) & 3) - 1.5) * T(0.5);
    } else {
      sx.template load<DPAC_ROLLOUT_DW_AUX>(rs_dw, fr.dw, (uint32_t)t * slab);  // zero past d: no mask
    }
  };
  auto body = [&](int t, DwFrame<T, M>& fr, auto phase) {
    T dwv[M];
#pragma unroll
    for (int m = 0; m < M; ++m) dwv[m] = fr.dw[m];
    if constexpr (PHILOX) own.mask(dwv);
    T u[MC];
    eq.u_true(x, r, u);
    TR tr;
    tr.run(eq, c, x, u, dwv, fl, r);
    const T cf = tr.coef ? T(1) : T(0);
    if constexpr (COST) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
      y += cost_increment(a.cost_order, w, cf, tr.dt, disc);
      disc = disc * disc_factor(tr.dt, cf, c);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = tr.coef ? tr.xt[m] : x[m];  // x + delta_x*coef (:67, :103)
    if constexpr (TR::kRadius) r = tr.coef ? tr.rt : r;
    fl = tr.next;
    if constexpr (DPAC_ABLATE == 1 || DPAC_ABLATE == 5) {
      if (t + 1 == a.N) sx.store(rs_x, x, (uint32_t)(t + 1) * slab);
      return;
    }
    if constexpr (DPAC_ABLATE != 4) sx.template store<DPAC_ROLLOUT_X_AUX>(rs_x, x, (uint32_t)(t + 1) * slab);
    if constexpr (WANT_U) su.store(rs_u, u, (uint32_t)t * slab_u);
    if constexpr (DPAC_ABLATE != 3) {
      constexpr int PH = decltype(phase)::value;
      keep = group_shift_in<P>(keep, tr.coef ? tr.dt : -tr.dt, lc.p == 0);
      if constexpr (PH >= 0) {
        if constexpr (PH % F == F - 1) flush(t, F);
      } else if ((t & (F - 1)) == F - 1) {
        flush(t, F);
      }
    }
  };
  pipelined<KB, DwFrame<T, M>>(0, a.N, load, body);
  if constexpr (DPAC_ABLATE != 3 && DPAC_ABLATE != 1 && DPAC_ABLATE != 5) {
    const int rem = a.N & (F - 1);
    if (rem) flush(a.N - 1, rem);
  }
  if constexpr (COST) {
    if (lc.live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}

// ---------------------------------------------------------------------------
// k_rollout with the increments staged through LDS by a loader wavefront.
//
// Why: gfx950 counts a wave's vector loads and stores in ONE in-order vmcnt, so in
// k_rollout the wait for step t's dw also waits for every x / dt / coef store issued
// before that load.  With HBM-cold data (measured, 5 rotating sets, B = 4096): loads
// alone 24.9 us, stores alone 26.8 us, both 38.5 us — the coupling, not bandwidth,
// costs the difference (profiles/r02_rollout_cold_ablations.txt).
// Here a workgroup is CW = 4 compute wavefronts (16 trajectories at P = 16) plus one
// LOADER wavefront that copies the workgroup's dw rows of each step (one contiguous
// row block in the step-major layout) into an RS-step LDS ring with global_load_lds,
// CH steps ahead of use; the compute wavefronts read dw from LDS and only store.  The
// loader's vmcnt holds only its DMA; the compute waves' holds only stores, which no
// one waits for.  Hand-off through LDS counters: `ready` (steps landed, loader) and
// `done[w]` (steps consumed, per compute wave), polled with s_sleep; the loader stays
// at most RS steps ahead.  Arithmetic per step is k_rollout's (bitwise the same).
// ---------------------------------------------------------------------------
#ifndef DPAC_ST_CHUNKS
#define DPAC_ST_CHUNKS 4  // hand-off chunks in the LDS ring
#endif
#ifndef DPAC_ST_TIGHT
#define DPAC_ST_TIGHT 0  // timing knob: 16-byte-aligned slots for every plan
#endif
#ifndef DPAC_ST_TIGHT_CHUNKS
#define DPAC_ST_TIGHT_CHUNKS 3  // hand-off chunks of a ring of 16-byte-aligned slots
#endif
#ifndef DPAC_ST_PD
#define DPAC_ST_PD 1  // compute waves: steps of dw read from the ring ahead of use
#endif
constexpr int kStCW = 4;   // compute wavefronts per workgroup
constexpr int kStCH = 16;  // steps per hand-off chunk
constexpr int kStPD = DPAC_ST_PD;
static_assert(kStPD >= 1 && kStPD <= kStCH, "prefetch distance within a chunk");
template <typename T, int D, int P>
struct StagedPlan {
  static constexpr int TPW = kStCW * (64 / P);                                   // trajectories per workgroup
  static constexpr int SLOT = TPW * D * (int)sizeof(T);                          // bytes of one step's rows
  static constexpr int PIECES = (SLOT + 1023) / 1024;                            // 1 KB DMA instructions per step
  // ring depth (steps): the loader publishes a chunk once the next one is issued, so it
  // needs >= 2 chunks; 4 keep it far enough ahead that the compute waves never wait
  // (measured at B = 4096, cold: 4 chunks 29.3 us, 2 chunks 41.6, k_rollout 38.3).  Slots
  // are 1 KB-aligned when 4 chunks of them fit in 128 KB; otherwise (float64 at d = 20:
  // 2560-byte slots) 3 chunks of 16-byte-aligned slots (121 KB) — every DMA piece still
  // starts inside its slot and the lane-0 filler write (at k*1024 < SLOT) never reaches
  // the pad.  Plans that fit neither way run k_rollout.
  static constexpr int kLdsCap = 128 * 1024;
  static constexpr int SLOT_1K = (SLOT + 16 + 1023) / 1024 * 1024;
  static constexpr int SLOT_16 = (SLOT + 16 + 15) / 16 * 16;
  static constexpr bool kWide = !DPAC_ST_TIGHT && DPAC_ST_CHUNKS * kStCH * SLOT_1K <= kLdsCap;
  static constexpr int CHUNKS = kWide ? DPAC_ST_CHUNKS : DPAC_ST_TIGHT_CHUNKS;
  static constexpr int SLOT_LDS = kWide ? SLOT_1K : SLOT_16;  // + a zero pad no DMA writes
  static constexpr int PADOFF = SLOT_LDS - 16;                 // where empty lanes read 0
  static constexpr int RS = CHUNKS * kStCH;
  static_assert(P < 4 || (SLOT % 16 == 0 && (PIECES - 1) * 1024 + 16 <= SLOT), "DMA pieces stay inside the slot");
  static constexpr bool kOk = P >= 4 && RS * SLOT_LDS <= kLdsCap && kStCH * PIECES <= 62;
};

template <class Fn, int... S>
__device__ __forceinline__ void unroll_phases(Fn& fn, std::integer_sequence<int, S...>) {
  (fn(Phase<S>{}), ...);
}

__device__ __forceinline__ int lds_load_relaxed(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_store_relaxed(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// GEN > 0 (round 6): the in-kernel Philox rollout on the same ring.  GEN
// generator wavefronts (one per SIMD) take the loader's place and draw the workgroup's increments
// into the ring, one counter block per lane and pass (the paired stream layout of dpac_device.h:
// a block is one lane slot's two components at two steps), so all 64 lanes of a generator do
// useful Philox and Box-Muller work, beside the compute wavefronts' latency-bound time loop,
// instead of each compute lane drawing its own (6 of 16 lanes idle at d = 20).  Values and
// arithmetic are k_rollout's Philox path's: bitwise its results.
template <int GEN>
constexpr int st_waves() { return kStCW + (GEN > 0 ? GEN : 1); }
#ifndef DPAC_ST_GEN
#define DPAC_ST_GEN 12  // generator wavefronts of the Philox variant (three per SIMD; round 6: 2 / 4 / 8 / 12 measured)
#endif
constexpr int kStGen = DPAC_ST_GEN;

template <typename T, class E, int D, int SCHEME, int OUT, int KB, int GEN = 0>
__global__ __launch_bounds__(64 * st_waves<GEN>()) void k_rollout_staged(const E eq, const DevConsts<T> c,
                                                                          const RolloutArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  using PL = StagedPlan<T, D, P>;
  constexpr int TPW = PL::TPW, RS = PL::RS, PIECES = PL::PIECES, SLOT_LDS = PL::SLOT_LDS;
  constexpr bool COST = (OUT & kOutCost) != 0, WANT_U = (OUT & kOutU) != 0;
  constexpr int F = P < kStCH ? P : kStCH;
  constexpr int NREADY = GEN > 0 ? GEN : 1;  // producers: the loader, or the generators
  static_assert(kStCH % F == 0 && (F & (F - 1)) == 0, "flush phase fixed per unrolled body");
  static_assert(GEN == 0 || (2 * M <= 4 && kStCH % 2 == 0), "generators draw the paired layout");
  using TR = Transition<T, E, SCHEME>;
  __shared__ __attribute__((aligned(16))) unsigned char s_ring[RS * SLOT_LDS];
  __shared__ int s_ready[NREADY], s_done[kStCW];
  const int wave = __builtin_amdgcn_readfirstlane((int)threadIdx.x / 64), lane = (int)threadIdx.x % 64;
  const int64_t row0 = xcd_block(blockIdx.x, gridDim.x) * TPW;
  const int N = a.N;
  if (threadIdx.x == 0) {
#pragma unroll
    for (int w = 0; w < NREADY; ++w) s_ready[w] = 0;
#pragma unroll
    for (int w = 0; w < kStCW; ++w) s_done[w] = 0;
  }
  if (threadIdx.x < RS * 4)  // the zero pads (lanes that own no component read them)
    reinterpret_cast<uint32_t*>(s_ring + (threadIdx.x / 4) * SLOT_LDS + PL::PADOFF)[threadIdx.x % 4] = 0u;
  __syncthreads();

  if constexpr (GEN > 0) {
    if (wave >= kStCW) {  // ---- generator g: its share of each chunk's counter blocks -> the ring ----
      const int g = wave - kStCW;
      const int64_t rows_live = (a.B - row0) < TPW ? (a.B - row0) : TPW;
      constexpr int PLS = (D + M - 1) / M;                // lane slots that own components
      constexpr int NBLK = (kStCH / 2) * TPW * PLS;       // blocks per chunk (d = 20: 8 x 16 x 10)
      constexpr int PASSES = (NBLK + 64 * GEN - 1) / (64 * GEN);
      constexpr int SLOT_T = SLOT_LDS / (int)sizeof(T);
      T* const ringw = reinterpret_cast<T*>(s_ring);
      for (int c0 = 0; c0 < N; c0 += kStCH) {
        const int need = c0 + kStCH - RS;  // the chunk's slots were last read at steps < need
        if (need > 0) {
          for (;;) {
            int mn = lds_load_relaxed(&s_done[0]);
#pragma unroll
            for (int w = 1; w < kStCW; ++w) mn = min(mn, lds_load_relaxed(&s_done[w]));
            if (mn >= need) break;
            __builtin_amdgcn_s_sleep(2);
          }
        }
        asm volatile("" ::: "memory");
#pragma unroll 1
        for (int k = 0; k < PASSES; ++k) {
          const int e = (k * GEN + g) * 64 + lane;
          const int u = e / (TPW * PLS), rem = e - u * (TPW * PLS);
          const int i = rem / PLS, p = rem - i * PLS;
          const int t0 = c0 + 2 * u;
          if (e < NBLK && t0 < N && i < rows_live) {
            T v[4];
            dw_block_values<T>(a.seed, (uint64_t)(a.traj_offset + row0 + i), (uint64_t)(t0 >> 1) * P + p,
                               a.sample_type, v);
            T* d0 = ringw + (t0 % RS) * SLOT_T + i * D + p * M;
            T* d1 = ringw + ((t0 + 1) % RS) * SLOT_T + i * D + p * M;
#pragma unroll
            for (int m = 0; m < M; ++m) {
              if (p * M + m < D) {
                d0[m] = v[m];
                if (t0 + 1 < N) d1[m] = v[M + m];
              }
            }
          }
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) lds_store_relaxed(&s_ready[g], c0 + kStCH < N ? c0 + kStCH : N);
      }
      return;
    }
  } else if (wave == kStCW) {  // ---- loader: dw rows of steps t -> ring slot t % RS ----
    const int64_t rows_live = (a.B - row0) < TPW ? (a.B - row0) : TPW;
    const uint32_t bytes = (uint32_t)(rows_live * D * (int64_t)sizeof(T));
    const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)s_ring;
    const char* base = (const char*)(a.dw + row0 * D);
    const int64_t step_bytes = a.B * D * (int64_t)sizeof(T);
    for (int c0 = 0; c0 < N; c0 += kStCH) {
      // the slots of this chunk were last read at steps c0 + s - RS: wait for every consumer
      const int need = c0 + kStCH - RS;
      if (need > 0) {
        for (;;) {
          int mn = lds_load_relaxed(&s_done[0]);
#pragma unroll
          for (int w = 1; w < kStCW; ++w) mn = min(mn, lds_load_relaxed(&s_done[w]));
          if (mn >= need) break;
          __builtin_amdgcn_s_sleep(2);
        }
      }
      asm volatile("" ::: "memory");
#pragma unroll
      for (int s = 0; s < kStCH; ++s) {
        const int t = c0 + s < N ? c0 + s : N - 1;  // past the end: re-copy the last step (unused)
        const char* src = base + t * step_bytes;
        const uint32_t slot = lds0 + (uint32_t)((t % RS) * SLOT_LDS);
#pragma unroll
        for (int k = 0; k < PIECES; ++k) {
          const uint32_t off = (uint32_t)((k * 64 + lane) * 16);
          const char* gp = src + (off < bytes ? off : 0u);  // lane 0 past the rows re-reads row 0
          const uint32_t m0 = __builtin_amdgcn_readfirstlane(slot + (uint32_t)(k * 1024));
          // lanes past the rows write nothing (the zero pad stays zero); lane 0 always issues,
          // so every instruction counts in vmcnt (it lands at k*1024, never on the pad)
          if (off < bytes || lane == 0) {
            int keep;
            asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                         : "=&s"(keep) : "v"(gp), "s"(m0) : "memory");
          }
        }
      }
      // the previous chunk has landed once only this chunk's copies are outstanding
      if (c0 > 0) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kStCH * PIECES) : "memory");
        if (lane == 0) lds_store_relaxed(&s_ready[0], c0);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) lds_store_relaxed(&s_ready[0], N);
    return;
  }

  // ---- compute wavefronts: k_rollout's time loop with dw from the ring ----
  const LaneCoord<P> lc(a.B, lane, row0 + wave * (64 / P));
  const int gl = wave * (64 / P) + lane / P;  // trajectory within the workgroup
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  const BufSlab<T, D, P> sx(own, lc.b, lc.live);
  const BufSlab<T, E::CDIM, P> su(ownu, lc.b, lc.live);
  const uint32_t slab = (uint32_t)(a.B * D * sizeof(T));
  const uint32_t slab_u = (uint32_t)(a.B * E::CDIM * sizeof(T));
  const uint32_t row_bytes = (uint32_t)(N * sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(a.x, slab * (uint32_t)(N + 1));
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(a.u, WANT_U ? slab_u * (uint32_t)N : 0u);
  const __amdgpu_buffer_rsrc_t rs_dt = make_rsrc(a.dt, (uint32_t)a.B * row_bytes);
  const __amdgpu_buffer_rsrc_t rs_cf = make_rsrc(a.coef, (uint32_t)a.B * row_bytes);
  const T* ring = reinterpret_cast<const T*>(s_ring);
  const int lds_e = gl * D + lc.p * M;  // element offset of this lane's components in a slot
  // full-or-empty lanes: one vector LDS read per step, empty lanes aimed at the zero pad
  constexpr bool kVecRead = Own<D, P>::kFull && (M * sizeof(T) == 8 || M * sizeof(T) == 16);
  const uint32_t lane_off = own.active() ? (uint32_t)(lds_e * (int)sizeof(T)) : (uint32_t)PL::PADOFF;
  T keep = 0;
  auto flush = [&](int t_last, int count) {
    const uint32_t off = (lc.live && lc.p < count)
                             ? (uint32_t)((lc.b * N + t_last - lc.p) * (int64_t)sizeof(T)) : kOOB;
    buf_store_scalar<T>(rs_dt, off, fabs(keep));
    buf_store_scalar<T>(rs_cf, off, keep > T(0) ? T(1) : T(0));
  };
  T x[M];
  sx.load(make_rsrc(a.x0, slab), x);
  sx.store(rs_x, x);
  T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  Flags fl = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c) : Flags{true, false};
  T disc = 1, y = 0;
  // slot_bytes: (t % RS) * SLOT_LDS, formed once per chunk plus a compile-time step offset
  auto read_dw_at = [&](int t, uint32_t slot_bytes, T (&dwv)[M]) {  // components past d read 0
    if constexpr (kVecRead) {
      typedef T vec __attribute__((ext_vector_type(M)));
      const vec v = *reinterpret_cast<const vec*>(s_ring + slot_bytes + lane_off);
#pragma unroll
      for (int m = 0; m < M; ++m) dwv[m] = v[m];
    } else {
      const T* slot = ring + (t % RS) * (SLOT_LDS / (int)sizeof(T)) + lds_e;
#pragma unroll
      for (int m = 0; m < M; ++m) dwv[m] = own.valid(m) ? slot[m] : T(0);
    }
  };
  auto read_dw = [&](int t, T (&dwv)[M]) { read_dw_at(t, (uint32_t)((t % RS) * SLOT_LDS), dwv); };
  auto body = [&](int t, const T (&dwv)[M], auto phase) {
    T u[MC];
    eq.u_true(x, r, u);
    TR tr;
    tr.run(eq, c, x, u, dwv, fl, r);
    const T cf = tr.coef ? T(1) : T(0);
    if constexpr (COST) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
      y += cost_increment(a.cost_order, w, cf, tr.dt, disc);
      disc = disc * disc_factor(tr.dt, cf, c);
    }
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = tr.coef ? tr.xt[m] : x[m];
    if constexpr (TR::kRadius) r = tr.coef ? tr.rt : r;
    fl = tr.next;
    sx.template store<DPAC_ROLLOUT_X_AUX>(rs_x, x, (uint32_t)(t + 1) * slab);
    if constexpr (WANT_U) su.store(rs_u, u, (uint32_t)t * slab_u);
    constexpr int PH = decltype(phase)::value;
    keep = group_shift_in<P>(keep, tr.coef ? tr.dt : -tr.dt, lc.p == 0);
    if constexpr (PH >= 0) {
      if constexpr (PH % F == F - 1) flush(t, F);
    } else if ((t & (F - 1)) == F - 1) {
      flush(t, F);
    }
  };
  for (int c0 = 0; c0 < N; c0 += kStCH) {
    const int want = c0 + kStCH < N ? c0 + kStCH : N;
    for (;;) {  // every producer has published the chunk
      int mn = lds_load_relaxed(&s_ready[0]);
#pragma unroll
      for (int w = 1; w < NREADY; ++w) mn = min(mn, lds_load_relaxed(&s_ready[w]));
      if (mn >= want) break;
      __builtin_amdgcn_s_sleep(1);
    }
    asm volatile("" ::: "memory");
    if (c0 + kStCH <= N) {
      // RS is a multiple of kStCH: the chunk's slots are contiguous from cb
      const uint32_t cb = (uint32_t)__builtin_amdgcn_readfirstlane((c0 % RS) * SLOT_LDS);
      constexpr int PD = kStPD;  // steps of dw in registers ahead of use
      T nxt[PD][M];
#pragma unroll
      for (int q = 0; q < PD; ++q) read_dw_at(c0 + q, cb + (uint32_t)(q * SLOT_LDS), nxt[q]);
      auto one = [&](auto sidx) {
        constexpr int S = decltype(sidx)::value;
        T cur[M];
#pragma unroll
        for (int m = 0; m < M; ++m) cur[m] = nxt[S % PD][m];
        if constexpr (S + PD < kStCH) read_dw_at(c0 + S + PD, cb + (uint32_t)((S + PD) * SLOT_LDS), nxt[S % PD]);
        if constexpr (PD > 1) __builtin_amdgcn_sched_barrier(0);  // issue the read here, PD steps ahead
        body(c0 + S, cur, Phase<S>{});
      };
      unroll_phases(one, std::make_integer_sequence<int, kStCH>{});
    } else {
      for (int t = c0; t < N; ++t) {
        T cur[M];
        read_dw(t, cur);
        body(t, cur, Phase<-1>{});
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_store_relaxed(&s_done[wave], want);
  }
  const int rem = N & (F - 1);
  if (rem) flush(N - 1, rem);
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
__global__ __launch_bounds__(64) void k_flag_init(const E eq, const DevConsts<T> c, int64_t B,
                                                   const T* x0, int32_t* flag) {
  constexpr int P = E::kP, M = E::M;
  const LaneCoord<P> lc(B, threadIdx.x, xcd_block(blockIdx.x, gridDim.x) * (64 / P));
  const Own<D, P> own(lc.p);
  T xv[M];
  own.load_masked(x0 + lc.b * D, xv);
  const T r = dsqrt(Lanes<P>::sum(sumsq(xv)));
  if (lc.p == 0) flag[lc.b] = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c).encode() : 1;
}

// ---------------------------------------------------------------------------
// One transition with an external control (NN actor), fused cost/discount.
// ---------------------------------------------------------------------------
template <typename T>
struct StepArgs {
  int64_t B;
  int cost_order;
  const T *x, *u, *dw, *disc_in, *y_in;
  const int32_t* flag_in;
  T *x_out, *disc_out, *y_out, *dt, *coef;
  int32_t* flag_out;
  // backward
  const T *g_x_out, *g_disc_out, *g_y_out;
  T *g_x, *g_u, *g_disc;
};

template <typename T, class E, int D, int SCHEME>
__global__ __launch_bounds__(64) void k_step_fwd(const E eq, const DevConsts<T> c,
                                                  const StepArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  using TR = Transition<T, E, SCHEME>;
  const LaneCoord<P> lc(a.B, threadIdx.x, xcd_block(blockIdx.x, gridDim.x) * (64 / P));
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  T x[M], u[MC], dw[M];
  own.load_masked(a.x + lc.b * D, x);
  own.load_masked(a.dw + lc.b * D, dw);
  ownu.load_masked(a.u + lc.b * E::CDIM, u);
  const T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  const Flags fl = Flags::decode(a.flag_in[lc.b]);
  const T disc = a.disc_in ? a.disc_in[lc.b] : T(1);
  TR tr;
  tr.run(eq, c, x, u, dw, fl, r);
  const T cf = tr.coef ? T(1) : T(0);
  const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
  T xn[M];
#pragma unroll
  for (int m = 0; m < M; ++m) xn[m] = tr.coef ? tr.xt[m] : x[m];
  own.store(a.x_out + lc.b * D, xn);
  if (lc.p == 0) {
    const T yin = a.y_in ? a.y_in[lc.b] : T(0);
    if (a.y_out) a.y_out[lc.b] = yin + cost_increment(a.cost_order, w, cf, tr.dt, disc);
    if (a.disc_out) a.disc_out[lc.b] = disc * disc_factor(tr.dt, cf, c);
    if (a.dt) a.dt[lc.b] = tr.dt;
    if (a.coef) a.coef[lc.b] = cf;
    a.flag_out[lc.b] = SCHEME == DPAC_SCHEME_ADAPTIVE ? tr.next.encode() : (tr.coef ? 1 : 0);
  }
}

// VJP of k_step_fwd.  Derivation: with lam = dL/dx', E = exp(-g dt c),
//   dL/ddisc = g_disc'*E + g_y'*c*w*dt
//   dL/ddt   = g_disc'*disc*E*(-g*c) + g_y'*c*w*disc + c*Σ_j lam_j*(f_j + s_j dw_j/(2 sqrt(dt)))
//   dL/du    = c*dt*lam·∂f/∂u + c*sqrt(dt)*(lam⊙dw)·∂s/∂u + g_y'*c*dt*disc*∂w/∂u
//   dL/dx    = lam + (same three terms w.r.t. x) + dL/ddt * ∂dt/∂x
//   ∂dt/∂x   = -2(R-r)x/(r*den) if flag == 1 and dt_raw >= 1e-4 dt0 (TF max tie rule), else 0
// The VJP of one transition for the owned slice (shared by k_step_bwd and the
// fused reverse rollout).  lam = dL/dx', gD1 = dL/ddisc', gy1 = dL/dy'.
template <typename T, class E, int SCHEME>
__device__ __forceinline__ void step_vjp(const E& eq, const DevConsts<T>& c, const T (&x)[E::M],
                                         const T (&u)[E::MC], const T (&dw)[E::M], Flags fl,
                                         T disc, const T (&lam)[E::M], T gD1, T gy1,
                                         T (&gx)[E::M], T (&gu)[E::MC], T& g_disc) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  using TR = Transition<T, E, SCHEME>;
  const T r = dsqrt(Lanes<P>::sum(sumsq(x)));
  TR tr;
  tr.run(eq, c, x, u, dw, fl, r);
  const T cf = tr.coef ? T(1) : T(0);
  const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
  const T Ef = disc_factor(tr.dt, cf, c);

  T f[M], s[M];
  eq.drift(x, u, r, f);
  eq.sigma(x, u, s);
  T a_f[M], a_s[M];
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
  eq.drift_vjp(x, u, r, a_f, gx, gu);
  eq.sigma_vjp(x, u, a_s, gx, gu);
  const T gw = gy1 * cf * tr.dt * disc;
  eq.w_vjp(x, u, gw, gx, gu);
  g_disc = gD1 * Ef + gy1 * cf * w * tr.dt;
  if constexpr (SCHEME == DPAC_SCHEME_ADAPTIVE) {
    const T g_dt = gD1 * disc * Ef * (c.neg_gamma * cf) + gy1 * cf * w * disc + cf * Lanes<P>::sum(part);
    const T raw = adaptive_dt_raw(fl.layer, r, c);
    if (fl.layer && raw >= c.dt_min) {
      const T k = g_dt * (-(c.R - r) * c.two_inv_den) / r;
#pragma unroll
      for (int m = 0; m < M; ++m) gx[m] += k * x[m];
    }
  }
}

template <typename T, class E, int D, int SCHEME>
__global__ __launch_bounds__(64) void k_step_bwd(const E eq, const DevConsts<T> c,
                                                  const StepArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(a.B, threadIdx.x, xcd_block(blockIdx.x, gridDim.x) * (64 / P));
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  T x[M], u[MC], dw[M], lam[M];
  own.load_masked(a.x + lc.b * D, x);
  own.load_masked(a.dw + lc.b * D, dw);
  own.load_masked(a.g_x_out + lc.b * D, lam);
  ownu.load_masked(a.u + lc.b * E::CDIM, u);
  const Flags fl = Flags::decode(a.flag_in[lc.b]);
  const T disc = a.disc_in ? a.disc_in[lc.b] : T(1);
  const T gD1 = a.g_disc_out ? a.g_disc_out[lc.b] : T(0);
  const T gy1 = a.g_y_out ? a.g_y_out[lc.b] : T(0);
  T gx[M], gu[MC], g_disc;
  step_vjp<T, E, SCHEME>(eq, c, x, u, dw, fl, disc, lam, gD1, gy1, gx, gu, g_disc);
  own.store(a.g_x + lc.b * D, gx);
  ownu.store(a.g_u + lc.b * E::CDIM, gu);
  if (a.g_disc && lc.p == 0) a.g_disc[lc.b] = g_disc;
}

// ---------------------------------------------------------------------------
// TD target assembly over a finished trajectory (solver.py:166-190) and its
// backward with respect to G.  Workgroup = 4 wavefronts over the same 64/P
// trajectories; wavefront w owns steps [w*Nc, (w+1)*Nc).  Each computes its
// chunk with a local discount starting at 1, then the (sum, product) pairs are
// combined in chunk order through LDS: y = Σ_w D_w L_w, D_{w+1} = D_w E_w.
// ---------------------------------------------------------------------------
constexpr int kTdChunks = 4;

template <typename T>
struct TdArgs {
  int64_t B, traj_offset;
  int N, sample_type, cost_order;
  uint64_t seed;
  const T *x, *u, *dw, *dt, *coef, *G, *g_y;
  T *y, *disc, *g_G;
  const T* gd;  // GDOT forward: [N][B] diffusion dots from dpac_mlp_rows_fwd_td1
  T* g_gd;      // GDOT backward: [N][B] d y / d gdot
};

template <typename T, int M, int MC, bool HAS_DW, bool HAS_G>
struct TdFrame {
  T x[M], u[MC], dw[HAS_DW ? M : 1], G[HAS_G ? M : 1];
  T dt, coef, gd;
};

// GDOT: the TD1 diffusion dot of each trajectory-step comes
// precomputed from the G network's epilogue (dpac_mlp_rows_fwd_td1, bitwise the dot
// below), so the forward reads one scalar instead of G and dw, and the backward writes
// the scalar d y / d gdot instead of d y / d G (the G network's backward forms the
// latter in its prologue, dpac_mlp_rows_bwd_td1) and reads neither x, u nor dw.
template <typename T, class E, int D, bool TD1, bool PHILOX, bool BWD, bool GDOT = false>
__global__ __launch_bounds__(256) void k_td(const E eq, const DevConsts<T> c, const TdArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC, GPW = 64 / P;
  constexpr bool USE_DW = (TD1 || BWD) && !GDOT;
  constexpr bool HAS_G = TD1 && !BWD && !GDOT;
  using F = TdFrame<T, M, MC, USE_DW && !PHILOX, HAS_G>;
  constexpr int KB = ring_kb((int)sizeof(F), 3 * DPAC_RING_VGPRS, sizeof(T) == 4 ? 4 : 2);
  __shared__ T s_sum[kTdChunks][GPW];
  __shared__ T s_prod[kTdChunks][GPW];

  // wave index is wave-uniform: say so, or the chunk loops become divergent branches
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / 64), lane = threadIdx.x % 64;
  const LaneCoord<P> lc(a.B, lane, xcd_block(blockIdx.x, gridDim.x) * GPW);
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  const BufSlab<T, D, P> sx(own, lc.b, lc.live);         // x[t], dw[t], G[t], g_G[t] rows
  const BufSlab<T, E::CDIM, P> su(ownu, lc.b, lc.live);  // u[t] rows
  const int g = lane / P;
  const int64_t B = a.B, stride = a.B * D, stride_u = a.B * E::CDIM;
  const uint32_t slab = (uint32_t)(stride * sizeof(T)), slab_u = (uint32_t)(stride_u * sizeof(T));
  const uint64_t gtraj = (uint64_t)(a.traj_offset + lc.b);
  const int nc = (a.N + kTdChunks - 1) / kTdChunks;
  const int t_begin = min(a.N, wave * nc), t_end = min(a.N, (wave + 1) * nc);

  // whole-array descriptors (host: every array < 2 GiB); the step goes in soffset
  const uint32_t row_bytes = (uint32_t)(a.N * sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(a.x, slab * (uint32_t)a.N);
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(a.u, slab_u * (uint32_t)a.N);
  const __amdgpu_buffer_rsrc_t rs_dw = make_rsrc(a.dw, (USE_DW && !PHILOX) ? slab * (uint32_t)a.N : 0u);
  const __amdgpu_buffer_rsrc_t rs_G = make_rsrc(a.G, HAS_G ? slab * (uint32_t)a.N : 0u);
  const __amdgpu_buffer_rsrc_t rs_gG = make_rsrc(a.g_G, (BWD && !GDOT) ? slab * (uint32_t)a.N : 0u);
  const uint32_t gd_bytes = (uint32_t)(B * a.N * (int64_t)sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_gd = make_rsrc(GDOT ? (BWD ? (const T*)a.g_gd : a.gd) : nullptr,
                                                 GDOT ? gd_bytes : 0u);
  const uint32_t off_gd = (uint32_t)(lc.b * (int64_t)sizeof(T));  // gdot rows are [N][B]
  const __amdgpu_buffer_rsrc_t rs_dt = make_rsrc(a.dt, (uint32_t)a.B * row_bytes);
  const __amdgpu_buffer_rsrc_t rs_cf = make_rsrc(a.coef, (uint32_t)a.B * row_bytes);
  const uint32_t off_row = (uint32_t)(lc.b * row_bytes);  // dt / coef rows are [B][N]
  auto load_scalar = [&](__amdgpu_buffer_rsrc_t r, int t) {
    uint32_t w[sizeof(T) / 4];
    buf_load_dwords<sizeof(T) / 4>(r, off_row, w, (uint32_t)t * (uint32_t)sizeof(T));
    T v;
    __builtin_memcpy(&v, &w[0], sizeof(T));
    return v;
  };
  auto load = [&](int t, F& fr) {
    if constexpr (!(GDOT && BWD)) {
      sx.load(rs_x, fr.x, (uint32_t)t * slab);
      su.load(rs_u, fr.u, (uint32_t)t * slab_u);
    }
    if constexpr (USE_DW && !PHILOX) sx.load(rs_dw, fr.dw, (uint32_t)t * slab);
    if constexpr (HAS_G) sx.load(rs_G, fr.G, (uint32_t)t * slab);
    if constexpr (GDOT && !BWD) {
      uint32_t w[sizeof(T) / 4];
      buf_load_dwords<sizeof(T) / 4>(rs_gd, off_gd, w, (uint32_t)t * (uint32_t)(B * sizeof(T)));
      __builtin_memcpy(&fr.gd, &w[0], sizeof(T));
    }
    fr.dt = load_scalar(rs_dt, t);
    fr.coef = load_scalar(rs_cf, t);
  };
  auto increments = [&](int t, F& fr, T (&dwv)[M]) {
    if constexpr (PHILOX) {
      draw_owned<T, E, D>(a.seed, gtraj, t, lc.p, a.sample_type, dwv);
      own.mask(dwv);
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) dwv[m] = fr.dw[m];
    }
  };

  T disc = 1;
  if constexpr (!BWD) {
    T y = 0;
    auto body = [&](int t, F& fr, auto) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(fr.x, fr.u)));
      y += cost_increment(a.cost_order, w, fr.coef, fr.dt, disc);
      if constexpr (GDOT) {
        y -= (fr.gd * disc) * (fr.coef * dsqrt(fr.dt));  // solver.py:180-184, dot precomputed
      } else if constexpr (TD1) {
        T s[M], dwv[M];
        eq.sigma(fr.x, fr.u, s);
        increments(t, fr, dwv);
        T acc = (s[0] * dwv[0]) * fr.G[0];
#pragma unroll
        for (int m = 1; m < M; ++m) acc = fma(s[m] * dwv[m], fr.G[m], acc);
        const T dot = Lanes<P>::sum(acc);
        y -= (dot * disc) * (fr.coef * dsqrt(fr.dt));  // solver.py:180-184
      }
      disc = disc * disc_factor(fr.dt, fr.coef, c);
    };
    pipelined<KB, F>(t_begin, t_end, load, body);
    if (lc.p == 0) {
      s_sum[wave][g] = y;
      s_prod[wave][g] = disc;
    }
    __syncthreads();
    if (wave == 0 && lc.p == 0 && lc.live) {
      T Dw = 1, tot = 0;
#pragma unroll
      for (int w = 0; w < kTdChunks; ++w) {
        tot += Dw * s_sum[w][g];
        Dw *= s_prod[w][g];
      }
      a.y[lc.b] = tot;
      a.disc[lc.b] = Dw;
    }
  } else {
    // pass A: the chunk's discount product from (dt, coef) only
    for (int t = t_begin; t < t_end; ++t) {
      const int64_t so = lc.b * a.N + t;
      disc = disc * disc_factor(a.dt[so], a.coef[so], c);
    }
    if (lc.p == 0) s_prod[wave][g] = disc;
    __syncthreads();
    T Dw = 1;
    for (int w = 0; w < wave; ++w) Dw *= s_prod[w][g];
    disc = Dw;
    const T gy = a.g_y[lc.b];
    auto body = [&](int t, F& fr, auto) {
      // d y / d G_j = -disc_t*coef_t*sqrt(dt_t)*diff_j
      const T k = -gy * (disc * (fr.coef * dsqrt(fr.dt)));
      if constexpr (GDOT) {
        const uint32_t off = (lc.live && lc.p == 0) ? off_gd : kOOB;
        buf_store_scalar<T>(rs_gd, off, k, (uint32_t)t * (uint32_t)(B * sizeof(T)));
      } else {
        T s[M], dwv[M], out[M];
        eq.sigma(fr.x, fr.u, s);
        increments(t, fr, dwv);
#pragma unroll
        for (int m = 0; m < M; ++m) out[m] = k * (s[m] * dwv[m]);
        sx.store(rs_gG, out, (uint32_t)t * slab);
      }
      disc = disc * disc_factor(fr.dt, fr.coef, c);
    };
    pipelined<KB, F>(t_begin, t_end, load, body);
  }
}

// ---------------------------------------------------------------------------
// Row-wise evaluation of one Equation method (parity tests, metrics).
// ---------------------------------------------------------------------------
template <typename T, class E, int D>
__global__ __launch_bounds__(64) void k_eval(const E eq, const DevConsts<T> c, int64_t B,
                                              int what, const T* x, const T* u, T* out) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  const LaneCoord<P> lc(B, threadIdx.x, xcd_block(blockIdx.x, gridDim.x) * (64 / P));
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  T xv[M], uv[MC];
  own.load_masked(x + lc.b * D, xv);
  if (u) {
    ownu.load_masked(u + lc.b * E::CDIM, uv);
  } else {
#pragma unroll
    for (int m = 0; m < MC; ++m) uv[m] = 0;
  }
  const T S = Lanes<P>::sum(sumsq(xv));
  const T r = dsqrt(S);
  T v[M];
  T scalar = 0;
  bool vec = false, ctl = false;
  switch (what) {
    case DPAC_EVAL_DRIFT: eq.drift(xv, uv, r, v); vec = true; break;
    case DPAC_EVAL_SIGMA: eq.sigma(xv, uv, v); vec = true; break;
    case DPAC_EVAL_W: scalar = eq.w_finish(Lanes<P>::sum(eq.w_part(xv, uv))); break;
    case DPAC_EVAL_Z: scalar = eq.Z(xv, S, r); break;
    case DPAC_EVAL_V_TRUE: scalar = eq.V_true(xv, S, r); break;
    case DPAC_EVAL_U_TRUE: {
      T uu[MC];
      eq.u_true(xv, r, uu);
      ownu.store(out + lc.b * E::CDIM, uu);
      ctl = true;
      break;
    }
    case DPAC_EVAL_V_GRAD: eq.V_grad(xv, S, r, v); vec = true; break;
    case DPAC_EVAL_B: scalar = S - c.R2; break;
    default: break;
  }
  if (ctl) return;
  if (vec) {
    own.store(out + lc.b * D, v);
  } else if (lc.p == 0) {
    out[lc.b] = scalar;
  }
}

#include "dpac_rollout_nn.h"
#include "dpac_rollout_nn_bwd.h"
#include "dpac_rollout_nn4.h"
#include "dpac_rollout_nn_x3.h"

// ---------------------------------------------------------------------------
// Launcher for one (T, equation functor, D).
// ---------------------------------------------------------------------------
// The kernel-side view of a dpac_mlp (column offsets of each layer's saved z).
template <typename T>
NnMlp<T> nn_mlp(const dpac_mlp& h) {
  NnMlp<T> m{};
  m.L = h.n_hidden;
  m.ekn = h.ekn_head;
  int z = 0;
  for (int i = 0; i <= m.L + 1; ++i) {
    m.width[i] = h.width[i];
    m.scale[i] = (const T*)h.bn_scale[i];
    m.shift[i] = (const T*)h.bn_shift[i];
    m.zoff[i] = i == 0 ? 0 : z;
    if (i > 0) z += m.width[i];
  }
  m.ztot = z;
  for (int i = 0; i <= m.L; ++i) {
    m.weight[i] = (const T*)h.weight[i];
    m.wkm[i] = (const T*)h.weight_km[i];
  }
  m.bias = (const T*)h.bias;
  m.status = h.status;
  return m;
}

// Row tile of the fused NN rollout for float: 4 (4x4x1 MFMA blocks) or 16
// (16x16x4 tiles; float64 always uses these); by default 4 for B <= 1024.
// DPAC_NN_TILE=4 / 16 forces one (tests compare the two).
// BPTT kernel: 2 = k_rollout_nn_bwd2 (stager + writer wavefronts, default), 1 = k_rollout_nn_bwd.
inline int bptt_kernel() {
  const char* e = getenv("DPAC_BPTT");  // read per launch: tests switch it in-process
  return (e && e[0] == '1') ? 1 : 2;
}

// Dynamic LDS of k_rollout_nn_bwd2: at least what it needs; DPAC_BPTT_LDS=max claims the
// whole LDS so no other kernel's workgroup shares a BPTT CU (timing experiments).
inline uint32_t bptt_lds(uint32_t need, uint32_t cap) {
  const char* e = getenv("DPAC_BPTT_LDS");  // read per launch
  if (!e) return need;
  const uint32_t v = (e[0] == 'm') ? cap : (uint32_t)atoi(e);
  return v > need ? (v < cap ? v : cap) : need;
}

// Analytic rollout with dw staged through LDS (k_rollout_staged, default) or read directly
// (k_rollout): DPAC_ROLLOUT_STAGED=0 forces the latter (tests compare the two bit for bit).
inline bool rollout_staged() {
  const char* e = getenv("DPAC_ROLLOUT_STAGED");  // read per launch
  return !(e && e[0] == '0');
}

inline int nn_tile_rows() {
  const char* e = getenv("DPAC_NN_TILE");  // read per launch: tests switch it in-process
  const int v = e ? atoi(e) : 0;
  return (v == 4 || v == 16) ? v : 0;     // 0: by batch size
}

// Trajectories per workgroup of the split-fp16 NN kernels (k_rollout_nn_x3, k_rollout_nn_bwd_x3):
// 16 (one MFMA row tile) or 8 (half a tile, twice the workgroups).  DPAC_NX_ROWS=8 / 16 forces one.
inline int nx_rows(int64_t B) {
  const char* e = getenv("DPAC_NX_ROWS");  // read per launch: tests switch it in-process
  const int v = e ? atoi(e) : 0;
  if (v == 8 || v == 16) return v;
  (void)B;
  return 16;
}

inline dim3 grid_for(int64_t B, int P) {
  const int64_t per = 64 / P;
  return dim3((unsigned)((B + per - 1) / per));
}

template <typename T, class E, int D>
int run_op(const OpArgs& a) {
  constexpr bool kFastOk = std::is_same<T, float>::value;  // the NN fast path is float-only
  const E eq = E::make(a.eq);
  const DevConsts<T> c = DevConsts<T>::make(host_consts(a));
  constexpr int P = E::kP;
  const dim3 grid = grid_for(a.B, P), block(64);
  hipStream_t s = a.stream;
  const bool adaptive = a.scheme == DPAC_SCHEME_ADAPTIVE;
  switch (a.op) {
    case OP_ROLLOUT: {
      RolloutArgs<T> r;
      r.B = a.B; r.traj_offset = a.traj_offset; r.N = a.N; r.sample_type = a.sample_type;
      r.cost_order = a.cost_order; r.seed = a.seed;
      r.x0 = (const T*)a.x0; r.dw = (const T*)a.dw;
      r.x = (T*)a.x_out; r.dt = (T*)a.dt; r.coef = (T*)a.coef; r.u = (T*)a.u_out;
      r.y = (T*)a.y; r.disc = (T*)a.disc;
      const bool philox = a.dw == nullptr, cost = a.y != nullptr;
      constexpr int KB = rollout_kb(ring_kb((int)sizeof(DwFrame<T, E::M>), DPAC_RING_VGPRS, DPAC_ROLLOUT_KB_CAP), E::kP);
      const int out = (cost ? kOutCost : 0) | (a.u_out ? kOutU : 0);
      using SP = StagedPlan<T, D, E::kP>;
      // the Philox variant on the ring (generator wavefronts): float, the paired stream layout
      constexpr bool kGenOk = SP::kOk && std::is_same<T, float>::value && 2 * E::M <= 4;
      if constexpr (kGenOk) {
        if (philox && rollout_staged() && dw_steps_per_block<T>(E::M, a.sample_type) == 2) {
          const dim3 sgrid((unsigned)((a.B + SP::TPW - 1) / SP::TPW)), sblock(64 * st_waves<kStGen>());
#define DPAC_ROLL_GEN(SCH, OUT) \
  hipLaunchKernelGGL((k_rollout_staged<T, E, D, SCH, OUT, KB, kStGen>), sgrid, sblock, 0, s, eq, c, r)
#define DPAC_ROLL_GEN_SCH(SCH)                                 \
  switch (out) {                                               \
    case 0: DPAC_ROLL_GEN(SCH, 0); break;                      \
    case kOutCost: DPAC_ROLL_GEN(SCH, kOutCost); break;        \
    case kOutU: DPAC_ROLL_GEN(SCH, kOutU); break;              \
    default: DPAC_ROLL_GEN(SCH, kOutCost | kOutU); break;      \
  }
          if (adaptive) { DPAC_ROLL_GEN_SCH(DPAC_SCHEME_ADAPTIVE) } else { DPAC_ROLL_GEN_SCH(DPAC_SCHEME_NAIVE) }
#undef DPAC_ROLL_GEN_SCH
#undef DPAC_ROLL_GEN
          break;
        }
      }
      if constexpr (SP::kOk) {
        if (!philox && rollout_staged()) {  // dw through the loader wave's LDS ring
          const dim3 sgrid((unsigned)((a.B + SP::TPW - 1) / SP::TPW)), sblock(64 * (kStCW + 1));
#define DPAC_ROLL_ST(SCH, OUT) \
  hipLaunchKernelGGL((k_rollout_staged<T, E, D, SCH, OUT, KB>), sgrid, sblock, 0, s, eq, c, r)
#define DPAC_ROLL_ST_SCH(SCH)                                  \
  switch (out) {                                               \
    case 0: DPAC_ROLL_ST(SCH, 0); break;                       \
    case kOutCost: DPAC_ROLL_ST(SCH, kOutCost); break;         \
    case kOutU: DPAC_ROLL_ST(SCH, kOutU); break;               \
    default: DPAC_ROLL_ST(SCH, kOutCost | kOutU); break;       \
  }
          if (adaptive) { DPAC_ROLL_ST_SCH(DPAC_SCHEME_ADAPTIVE) } else { DPAC_ROLL_ST_SCH(DPAC_SCHEME_NAIVE) }
#undef DPAC_ROLL_ST_SCH
#undef DPAC_ROLL_ST
          break;
        }
      }
#define DPAC_ROLL(SCH, PH, OUT) \
  hipLaunchKernelGGL((k_rollout<T, E, D, SCH, PH, OUT, KB>), grid, block, 0, s, eq, c, r)
#define DPAC_ROLL_PH(SCH, PH)                              \
  switch (out) {                                           \
    case 0: DPAC_ROLL(SCH, PH, 0); break;                  \
    case kOutCost: DPAC_ROLL(SCH, PH, kOutCost); break;    \
    case kOutU: DPAC_ROLL(SCH, PH, kOutU); break;          \
    default: DPAC_ROLL(SCH, PH, kOutCost | kOutU); break;  \
  }
#define DPAC_ROLL_SCH(SCH) \
  if (philox) { DPAC_ROLL_PH(SCH, true) } else { DPAC_ROLL_PH(SCH, false) }
      if (adaptive) { DPAC_ROLL_SCH(DPAC_SCHEME_ADAPTIVE) } else { DPAC_ROLL_SCH(DPAC_SCHEME_NAIVE) }
#undef DPAC_ROLL_SCH
#undef DPAC_ROLL_PH
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
      st.B = a.B; st.cost_order = a.cost_order;
      st.x = (const T*)a.x; st.u = (const T*)a.u; st.dw = (const T*)a.dw;
      st.disc_in = (const T*)a.disc_in; st.y_in = (const T*)a.y_in; st.flag_in = a.flag_in;
      st.x_out = (T*)a.x_out; st.disc_out = (T*)a.disc_out; st.y_out = (T*)a.y_out;
      st.dt = (T*)a.dt; st.coef = (T*)a.coef; st.flag_out = a.flag_out;
      st.g_x_out = (const T*)a.g_x_out; st.g_disc_out = (const T*)a.g_disc_out;
      st.g_y_out = (const T*)a.g_y_out;
      st.g_x = (T*)a.g_x; st.g_u = (T*)a.g_u; st.g_disc = (T*)a.g_disc;
      if (a.op == OP_STEP_FWD) {
        if (adaptive) hipLaunchKernelGGL((k_step_fwd<T, E, D, DPAC_SCHEME_ADAPTIVE>), grid, block, 0, s, eq, c, st);
        else hipLaunchKernelGGL((k_step_fwd<T, E, D, DPAC_SCHEME_NAIVE>), grid, block, 0, s, eq, c, st);
      } else {
        if (adaptive) hipLaunchKernelGGL((k_step_bwd<T, E, D, DPAC_SCHEME_ADAPTIVE>), grid, block, 0, s, eq, c, st);
        else hipLaunchKernelGGL((k_step_bwd<T, E, D, DPAC_SCHEME_NAIVE>), grid, block, 0, s, eq, c, st);
      }
      break;
    }
    case OP_TD_FWD:
    case OP_TD_BWD: {
      TdArgs<T> td;
      td.B = a.B; td.traj_offset = a.traj_offset; td.N = a.N; td.sample_type = a.sample_type;
      td.cost_order = a.cost_order; td.seed = a.seed;
      td.x = (const T*)a.x; td.u = (const T*)a.u; td.dw = (const T*)a.dw;
      td.dt = (const T*)a.dt_in; td.coef = (const T*)a.coef_in; td.G = (const T*)a.G;
      td.g_y = (const T*)a.g_y_out;
      td.y = (T*)a.y; td.disc = (T*)a.disc; td.g_G = (T*)a.g_G;
      td.gd = (const T*)a.G; td.g_gd = (T*)a.g_G;
      const bool philox = a.dw == nullptr;
      const dim3 tblock(64 * kTdChunks);
#define DPAC_TD(TD1, PH, BW) hipLaunchKernelGGL((k_td<T, E, D, TD1, PH, BW>), grid, tblock, 0, s, eq, c, td)
      if (a.td_type == DPAC_TD1_GDOT) {
        if (a.op == OP_TD_BWD)
          hipLaunchKernelGGL((k_td<T, E, D, true, false, true, true>), grid, tblock, 0, s, eq, c, td);
        else
          hipLaunchKernelGGL((k_td<T, E, D, true, false, false, true>), grid, tblock, 0, s, eq, c, td);
      } else if (a.op == OP_TD_BWD) {
        if (philox) DPAC_TD(true, true, true); else DPAC_TD(true, false, true);
      } else if (a.td_type == DPAC_TD1) {
        if (philox) DPAC_TD(true, true, false); else DPAC_TD(true, false, false);
      } else {
        DPAC_TD(false, false, false);
      }
#undef DPAC_TD
      break;
    }
    case OP_EVAL:
      hipLaunchKernelGGL((k_eval<T, E, D>), grid, block, 0, s, eq, c, a.B, a.what,
                         (const T*)a.x, (const T*)a.u, (T*)a.out);
      break;
    case OP_ROLLOUT_NN_BWD: {
      NnMlp<T> m = nn_mlp<T>(a.mlp);
      NnBackArgs<T> r{};
      r.B = a.B; r.N = a.N;
      r.x = (const T*)a.x; r.u = (const T*)a.u; r.dw = (const T*)a.dw;
      r.disc_t = (const T*)a.save_disc; r.z = (const T*)a.save_z; r.flag = a.save_flag;
      r.g_xN = (const T*)a.g_x_out; r.g_disc = (const T*)a.g_disc_out; r.g_y = (const T*)a.g_y_out;
      r.G = (T*)a.g_G; r.g_x0 = (T*)a.g_x;
      int go = 0;
      for (int i = 0; i <= m.L + 1; ++i) {
        r.goff[i] = go;
        go += m.width[i];
      }
      r.gtot = go;
      for (int i = 0; i <= m.L; ++i) {
        r.wt[i] = (const T*)a.mlp_wt[i];
        r.wtkm[i] = (const T*)a.mlp.weight_km[i];  // k-major images of wt (dpac.h)
      }
      // the fast path serves k_rollout_nn_bwd2 (the generic k_rollout_nn_bwd ignores it)
      r.fast = nn_fast_host<T>(m.L, m.width, (const void* const*)r.wtkm, m.width[m.L + 1], m.width[0]);
      r.mask = r.fast ? a.mask_in : nullptr;
      r.mb = nn_mask_tile_bytes(m.L);
      const dim3 ngrid((unsigned)((a.B + kNnRows - 1) / kNnRows)), nblock(kNnThreads);
      const int gphase = m.status ? a.mlp.guard_phase : DPAC_GUARD_INLINE;  // dpac.h guard_phase
      if constexpr (kFastOk) {  // split-fp16 chain (dpac_rollout_nn_x3.h): needs the forward's mask
        // (guarded by a status word: only with the f32 fast path's operands for the fallback)
        if (r.mask && bptt_kernel() == 2 && (!m.status || r.fast) &&
            nn_x3_host(m.L, m.width, (const void* const*)a.mlp.weight_t_x3, m.width[m.L + 1], m.width[0])) {
          for (int i = 0; i <= m.L; ++i) r.wtx3[i] = (const _Float16*)a.mlp.weight_t_x3[i];
          r.tr = nx_rows(a.B);
          auto kfn = adaptive ? k_rollout_nn_bwd_x3<E, D, DPAC_SCHEME_ADAPTIVE>
                              : k_rollout_nn_bwd_x3<E, D, DPAC_SCHEME_NAIVE>;
          if (gphase != DPAC_GUARD_FALLBACK_ONLY) {
            if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)NxLds::total))
              return (int)e;
            hipLaunchKernelGGL(kfn, dim3((unsigned)((a.B + r.tr - 1) / r.tr)), nblock, NxLds::total, s, eq, c, m, r);
          }
          if (m.status && gphase != DPAC_GUARD_SPLIT_ONLY) {
            // the f32 BPTT, run only once the x3 kernel fell back (dpac.h dpac_mlp.status)
            int wsum = 0;
            for (int i = 0; i <= m.L + 1; ++i) wsum += m.width[i];
            const BwdPlan<T, D, E::CDIM> pl(wsum, m.ztot, true, r.mb);
            const uint32_t lds = bptt_lds(pl.total, BwdPlan<T, D, E::CDIM>::kMaxDyn);
            NnBackArgs<T> f = r;
            f.guard = m.status;
            auto ffn = adaptive ? k_rollout_nn_bwd2<T, E, D, DPAC_SCHEME_ADAPTIVE, false, true, true>
                                : k_rollout_nn_bwd2<T, E, D, DPAC_SCHEME_NAIVE, false, true, true>;
            if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(ffn),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
              return (int)e;
            hipLaunchKernelGGL(ffn, ngrid, dim3(kNnBwdThreads), lds, s, eq, c, m, f);
          }
          break;
        }
      }
      if (gphase == DPAC_GUARD_FALLBACK_ONLY) break;  // phase 1 did the whole work
      if (bptt_kernel() == 2) {
        int wsum = 0;
        for (int i = 0; i <= m.L + 1; ++i) wsum += m.width[i];
        const BwdPlan<T, D, E::CDIM> pl(wsum, m.ztot, true, r.mask ? r.mb : 0);
        const uint32_t lds = bptt_lds(pl.total, BwdPlan<T, D, E::CDIM>::kMaxDyn);
        const dim3 nb2(kNnBwdThreads);
#define DPAC_BWD2(SCH, ZS)                                                                          \
  {                                                                                                 \
    auto kfn = r.fast ? k_rollout_nn_bwd2<T, E, D, SCH, ZS, kFastOk> : k_rollout_nn_bwd2<T, E, D, SCH, ZS, false>; \
    if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),                      \
                                           hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))     \
      return (int)e;                                                                                \
    hipLaunchKernelGGL(kfn, ngrid, nb2, lds, s, eq, c, m, r);                                       \
  }
        if constexpr (kFastOk) {
          if (r.mask) {  // the sign-bit mask instead of z (fast path)
            auto kfn = adaptive ? k_rollout_nn_bwd2<T, E, D, DPAC_SCHEME_ADAPTIVE, false, true, true>
                                : k_rollout_nn_bwd2<T, E, D, DPAC_SCHEME_NAIVE, false, true, true>;
            if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                                   hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
              return (int)e;
            hipLaunchKernelGGL(kfn, ngrid, nb2, lds, s, eq, c, m, r);
            break;
          }
        }
        if (adaptive) {
          if (pl.zst) DPAC_BWD2(DPAC_SCHEME_ADAPTIVE, true) else DPAC_BWD2(DPAC_SCHEME_ADAPTIVE, false)
        } else {
          if (pl.zst) DPAC_BWD2(DPAC_SCHEME_NAIVE, true) else DPAC_BWD2(DPAC_SCHEME_NAIVE, false)
        }
#undef DPAC_BWD2
        break;
      }
      if (adaptive) hipLaunchKernelGGL((k_rollout_nn_bwd<T, E, D, DPAC_SCHEME_ADAPTIVE>), ngrid, nblock, 0, s, eq, c, m, r);
      else hipLaunchKernelGGL((k_rollout_nn_bwd<T, E, D, DPAC_SCHEME_NAIVE>), ngrid, nblock, 0, s, eq, c, m, r);
      break;
    }
    case OP_ROLLOUT_NN: {
      NnMlp<T> m{};
      m.L = a.mlp.n_hidden;
      m.ekn = a.mlp.ekn_head;
      int z = 0;
      for (int i = 0; i <= m.L + 1; ++i) {
        m.width[i] = a.mlp.width[i];
        m.scale[i] = (const T*)a.mlp.bn_scale[i];
        m.shift[i] = (const T*)a.mlp.bn_shift[i];
        m.zoff[i] = i == 0 ? 0 : z;
        if (i > 0) z += m.width[i];
      }
      m.ztot = z;
      for (int i = 0; i <= m.L; ++i) {
        m.weight[i] = (const T*)a.mlp.weight[i];
        m.wkm[i] = (const T*)a.mlp.weight_km[i];
      }
      m.bias = (const T*)a.mlp.bias;
      m.status = a.mlp.status;
      m.fast = nn_fast_host<T>(m.L, m.width, (const void* const*)m.wkm, m.width[0], m.width[m.L + 1]);
      NnRolloutArgs<T> r{};
      r.B = a.B; r.N = a.N; r.cost_order = a.cost_order;
      r.x0 = (const T*)a.x0; r.dw = (const T*)a.dw;
      r.x = (T*)a.x_out; r.dt = (T*)a.dt; r.coef = (T*)a.coef; r.u = (T*)a.u_out;
      r.y = (T*)a.y; r.disc = (T*)a.disc;
      r.save_z = (T*)a.save_z; r.save_disc = (T*)a.save_disc; r.save_flag = a.save_flag;
      r.save_mask = nullptr;
      r.mb = nn_mask_tile_bytes(m.L);
      const bool cost = a.y != nullptr;
      const int gphase = m.status ? a.mlp.guard_phase : DPAC_GUARD_INLINE;  // dpac.h guard_phase
      if constexpr (std::is_same<T, float>::value) {
        // 4-row MFMA blocks (dpac_rollout_nn4.h) where the 16-row tiles would leave
        // most CUs idle: 4x4x1 costs 4x the cycles per flop of 16x16x4, and measured
        // 11.4 vs 15.4 us per step at B <= 1024, 15.8 vs 15.4 at 2048, 31 vs 15.4 at 4096
        const int tile = nn_tile_rows();
        if (tile == 4 || (tile == 0 && a.B <= 1024)) {
          if (gphase == DPAC_GUARD_FALLBACK_ONLY) break;  // no split-fp16 launch here: nothing to redo
          const int rg = a.B <= 1024 ? 1 : 2;
          const dim3 g4((unsigned)((a.B + 4 * rg - 1) / (4 * rg))), b4(kN4Threads);
#define DPAC_ROLL_NN4(SCH, CO, RG) \
  hipLaunchKernelGGL((k_rollout_nn4<T, E, D, SCH, CO, RG>), g4, b4, 0, s, eq, c, m, r)
#define DPAC_ROLL_NN4_RG(SCH, CO) \
  if (rg == 1) { DPAC_ROLL_NN4(SCH, CO, 1); } else { DPAC_ROLL_NN4(SCH, CO, 2); }
          if (adaptive) {
            if (cost) { DPAC_ROLL_NN4_RG(DPAC_SCHEME_ADAPTIVE, true) } else { DPAC_ROLL_NN4_RG(DPAC_SCHEME_ADAPTIVE, false) }
          } else {
            if (cost) { DPAC_ROLL_NN4_RG(DPAC_SCHEME_NAIVE, true) } else { DPAC_ROLL_NN4_RG(DPAC_SCHEME_NAIVE, false) }
          }
#undef DPAC_ROLL_NN4_RG
#undef DPAC_ROLL_NN4
          break;
        }
      }
      const dim3 ngrid((unsigned)((a.B + kNnRows - 1) / kNnRows)), nblock(kNnThreads);
      bool x3 = false;
      if constexpr (kFastOk)  // guarded by a status word: only with the f32 fast path's operands for the fallback
        x3 = (!m.status || m.fast) &&
             nn_x3_host(m.L, m.width, (const void* const*)a.mlp.weight_x3, m.width[0], m.width[m.L + 1]);
      if ((m.fast || x3) && a.save_mask && a.save_z) {  // the 16-row fast paths write the sign bits
        r.save_mask = a.save_mask;
        if (a.mask_written) *a.mask_written = 1;
      }
      if constexpr (kFastOk) {  // split-fp16 MLP (dpac_rollout_nn_x3.h)
        if (x3) {
          for (int i = 0; i <= m.L; ++i) m.wx3[i] = (const _Float16*)a.mlp.weight_x3[i];
          const bool save = r.save_z != nullptr, mask = r.save_mask != nullptr;
          r.tr = nx_rows(a.B);
          const dim3 xgrid((unsigned)((a.B + r.tr - 1) / r.tr));
          hipError_t e = hipSuccess;
#define DPAC_NX_LAUNCH(SCH, CO, SV, MK)                                                                    \
  {                                                                                                       \
    auto kfn = k_rollout_nn_x3<E, D, SCH, CO, SV, MK>;                                                    \
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, \
                            (int)NxLds::total);                                                           \
    if (e == hipSuccess) hipLaunchKernelGGL(kfn, xgrid, nblock, NxLds::total, s, eq, c, m, r);            \
  }
#define DPAC_NX_SV(SCH, CO)                                    \
  if (mask) DPAC_NX_LAUNCH(SCH, CO, true, true)                \
  else if (save) DPAC_NX_LAUNCH(SCH, CO, true, false)          \
  else DPAC_NX_LAUNCH(SCH, CO, false, false)
          if (gphase != DPAC_GUARD_FALLBACK_ONLY) {
            if (adaptive) {
              if (cost) { DPAC_NX_SV(DPAC_SCHEME_ADAPTIVE, true) } else { DPAC_NX_SV(DPAC_SCHEME_ADAPTIVE, false) }
            } else {
              if (cost) { DPAC_NX_SV(DPAC_SCHEME_NAIVE, true) } else { DPAC_NX_SV(DPAC_SCHEME_NAIVE, false) }
            }
          }
#undef DPAC_NX_SV
#undef DPAC_NX_LAUNCH
          if (e != hipSuccess) return (int)e;
          if (!m.status || gphase == DPAC_GUARD_SPLIT_ONLY) break;
          r.guard = m.status;  // then the f32 kernel below, run only once the x3 kernel fell back
        }
      }
      if (gphase == DPAC_GUARD_FALLBACK_ONLY && !r.guard) break;  // phase 1 did the whole work
#define DPAC_ROLL_NN(SCH, CO)                                                                                   \
  do {                                                                                                          \
    if (m.fast && r.save_mask)                                                                                  \
      hipLaunchKernelGGL((k_rollout_nn<T, E, D, SCH, CO, 1, kFastOk, kFastOk>), ngrid, nblock, 0, s, eq, c, m, r); \
    else if (m.fast) hipLaunchKernelGGL((k_rollout_nn<T, E, D, SCH, CO, 1, kFastOk>), ngrid, nblock, 0, s, eq, c, m, r); \
    else hipLaunchKernelGGL((k_rollout_nn<T, E, D, SCH, CO, 1, false>), ngrid, nblock, 0, s, eq, c, m, r);      \
  } while (0)
      if (adaptive) {
        if (cost) DPAC_ROLL_NN(DPAC_SCHEME_ADAPTIVE, true); else DPAC_ROLL_NN(DPAC_SCHEME_ADAPTIVE, false);
      } else {
        if (cost) DPAC_ROLL_NN(DPAC_SCHEME_NAIVE, true); else DPAC_ROLL_NN(DPAC_SCHEME_NAIVE, false);
      }
#undef DPAC_ROLL_NN
      break;
    }
    default:
      return DPAC_EINVAL;
  }
  return (int)hipGetLastError();
}

// Kernel instantiations register themselves per (equation family, dim, dtype): each
// equation TU is compiled once per dtype and state dimension (Makefile), so the heavy
// template instantiations build in parallel, and dpac_abi.hip finds them in a table.
// EQ<T, D> is the functor with its lane split already chosen.
using DispatchFn = int (*)(const OpArgs&);
void register_dispatch(int eqn, int dim, int f64, DispatchFn fn);
DispatchFn find_dispatch(int eqn, int dim, int f64);
constexpr int kMaxRegDim = 64;  // the dispatch table's dimension range (dpac_abi.hip)

template <template <typename, int> class EQ, typename T, int... Ds>
struct Registrar {
  static_assert(((Ds >= 1 && Ds <= kMaxRegDim) && ...),
                "DPAC_DIMS holds a dimension outside the dispatch table (1..kMaxRegDim)");
  explicit Registrar(int eqn) {
    (register_dispatch(eqn, Ds, std::is_same<T, double>::value ? 1 : 0, &run_op<T, EQ<T, Ds>, Ds>), ...);
  }
};

}  // namespace dpac
