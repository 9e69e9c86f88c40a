// dpac_abi.hip — the extern "C" surface of libdpac (include/dpac.h): argument
// validation, thread-local error reporting, dispatch to the per-equation
// kernel instantiations, and the on-device Brownian sampler.
#include <cstdarg>
#include <cstdio>
#include <string>

#include "dpac_kernels.h"

namespace dpac {
// The instantiation table the equation TUs fill at load time (Registrar, dpac_kernels.h):
// [equation id][dim][f64] (dim up to kMaxRegDim, dpac_kernels.h, checked at build time by
// Registrar).  Zero-initialised before any constructor runs.
static DispatchFn g_dispatch[4][kMaxRegDim + 1][2];
void register_dispatch(int eqn, int dim, int f64, DispatchFn fn) {
  if (eqn >= 0 && eqn < 4 && dim >= 1 && dim <= kMaxRegDim && (f64 == 0 || f64 == 1)) g_dispatch[eqn][dim][f64] = fn;
}
DispatchFn find_dispatch(int eqn, int dim, int f64) {
  if (eqn < 0 || eqn >= 4 || dim < 1 || dim > kMaxRegDim || (f64 != 0 && f64 != 1)) return nullptr;
  return g_dispatch[eqn][dim][f64];
}
int64_t mlp_param_grads_ws_bytes(int dtype, int64_t rows, const dpac_mlp& net);
int mlp_param_grads_launch(int dtype, int64_t rows, const dpac_mlp& net, double gamma_scale,
                           const void* x, int64_t ldx, const void* z, const void* G, void* ws,
                           void* out, hipStream_t s);
int mlp_rows_fwd_launch(int dtype, int64_t rows, const dpac_mlp& net, const void* x, int64_t ldx,
                        void* out, void* save_z, const TdRows* td, uint8_t* mask, int32_t* written,
                        hipStream_t s);
int mlp_rows_bwd_launch(int dtype, int64_t rows, const dpac_mlp& net, const void* const* wt,
                        const void* save_z, const uint8_t* mask, const void* g_out, void* G, void* g_x,
                        const TdRows* td, hipStream_t s);
int64_t mlp_rows_mask_bytes(int dtype, int64_t rows, const dpac_mlp& net);
int mlp_prepare_launch(int dtype, const dpac_mlp& net, double gamma_scale, void* scales, void* wt,
                       void* wkm, void* wtkm, void* wx3, void* wtx3, hipStream_t s);
int critic_loss_launch(int dtype, int64_t B, const void* V, const void* y, const void* disc, const void* zb,
                       double scale, double clip, void* g_out, void* neg_g, hipStream_t s);
int adam_launch(int dtype, int n, const int64_t* numel, void* const* var, const void* const* grad,
                void* const* m, void* const* v, double alpha, double b1, double b2, double eps,
                hipStream_t s);

namespace {
thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

int ok() {
  g_err.clear();
  return DPAC_OK;
}

int check_eq(const dpac_eqn_params* eq) {
  if (!eq) return fail(DPAC_EINVAL, "eqn params pointer is NULL");
  if (eq->reserved != 0) return fail(DPAC_EINVAL, "eqn params: reserved must be 0");
  if (eq->dim < 1) return fail(DPAC_EINVAL, "dim must be >= 1 (got %d)", eq->dim);
  switch (eq->eqn) {
    case DPAC_EQN_LQR:
    case DPAC_EQN_EKN:
    case DPAC_EQN_LQR_VAR:
      if (eq->control_dim != eq->dim)
        return fail(DPAC_EINVAL, "control_dim (%d) must equal dim (%d) for this equation",
                    eq->control_dim, eq->dim);
      break;
    case DPAC_EQN_VDP:
      if (eq->dim != 2 * eq->control_dim)
        return fail(DPAC_EINVAL, "VDP needs dim == 2*control_dim (dim %d, control_dim %d)",
                    eq->dim, eq->control_dim);
      break;
    default:
      return fail(DPAC_EINVAL, "unknown equation id %d", eq->eqn);
  }
  if (!(eq->R > 0)) return fail(DPAC_EINVAL, "R must be > 0");
  const bool has = find_dispatch(eq->eqn, eq->dim, 0) && find_dispatch(eq->eqn, eq->dim, 1);
  if (!has)
    return fail(DPAC_EUNSUP, "equation %d has no kernel instantiation for dim %d", eq->eqn,
                eq->dim);
  return DPAC_OK;
}

int check_common(const dpac_eqn_params* eq, int32_t dtype, int64_t B) {
  if (int e = check_eq(eq)) return e;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (B < 1) return fail(DPAC_EINVAL, "num_sample must be >= 1 (got %lld)", (long long)B);
  if (B > (int64_t)1 << 31) return fail(DPAC_EINVAL, "num_sample too large");
  return DPAC_OK;
}

int check_time(int32_t scheme, int32_t N, double T) {
  if (scheme != DPAC_SCHEME_NAIVE && scheme != DPAC_SCHEME_ADAPTIVE)
    return fail(DPAC_EINVAL, "bad scheme %d", scheme);
  if (N < 1) return fail(DPAC_EINVAL, "num_steps must be >= 1 (got %d)", N);
  if (!(T > 0)) return fail(DPAC_EINVAL, "total_time must be > 0");
  return DPAC_OK;
}

int check_sample_type(int32_t st) {
  if (st != DPAC_SAMPLE_NORMAL && st != DPAC_SAMPLE_BOUNDED && st != DPAC_SAMPLE_ZERO_X0)
    return fail(DPAC_EINVAL, "bad sample_type %d", st);
  return DPAC_OK;
}

// dpac_mlp.guard_phase: one of DPAC_GUARD_*, and a split phase only with a status word
int check_guard_phase(const dpac_mlp* net) {
  if (net->guard_phase < DPAC_GUARD_INLINE || net->guard_phase > DPAC_GUARD_FALLBACK_ONLY)
    return fail(DPAC_EINVAL, "guard_phase must be 0, 1 or 2 (got %d)", net->guard_phase);
  if (net->guard_phase != DPAC_GUARD_INLINE && !net->status)
    return fail(DPAC_EINVAL, "guard_phase %d needs a status word", net->guard_phase);
  return DPAC_OK;
}

int check_mlp(const dpac_eqn_params* eq, const dpac_mlp* actor) {
  if (!actor) return fail(DPAC_EINVAL, "actor MLP pointer is NULL");
  const int L = actor->n_hidden;
  if (L < 1 || L > DPAC_MLP_MAX_HIDDEN)
    return fail(DPAC_EINVAL, "actor: n_hidden must be in [1, %d] (got %d)", DPAC_MLP_MAX_HIDDEN, L);
  if (actor->ekn_head != 0 && actor->ekn_head != 1)
    return fail(DPAC_EINVAL, "actor: ekn_head must be 0 or 1");
  if (actor->ekn_head && eq->eqn != DPAC_EQN_EKN)
    return fail(DPAC_EINVAL, "actor: the Eikonal head applies to the EKN equation only");
  for (int i = 0; i <= L + 1; ++i) {
    if (actor->width[i] < 1 || actor->width[i] > DPAC_MLP_MAX_WIDTH)
      return fail(DPAC_EINVAL, "actor: width[%d] = %d outside [1, %d]", i, actor->width[i],
                  DPAC_MLP_MAX_WIDTH);
    if (!actor->bn_scale[i] || !actor->bn_shift[i])
      return fail(DPAC_EINVAL, "actor: bn_scale/bn_shift[%d] is NULL", i);
    if (i <= L && !actor->weight[i]) return fail(DPAC_EINVAL, "actor: weight[%d] is NULL", i);
  }
  if (!actor->bias) return fail(DPAC_EINVAL, "actor: bias is NULL");
  if (actor->width[0] != eq->dim)
    return fail(DPAC_EINVAL, "actor: width[0] (%d) must equal dim (%d)", actor->width[0], eq->dim);
  if (actor->width[L + 1] != eq->control_dim + actor->ekn_head)
    return fail(DPAC_EINVAL, "actor: output width %d must be control_dim%s (%d)",
                actor->width[L + 1], actor->ekn_head ? " + 1" : "",
                eq->control_dim + actor->ekn_head);
  return check_guard_phase(actor);
}

// A dpac_mlp for the row-parallel kernels (no equation attached).
int check_net(const dpac_mlp* net) {
  if (!net) return fail(DPAC_EINVAL, "MLP pointer is NULL");
  const int L = net->n_hidden;
  if (L < 1 || L > DPAC_MLP_MAX_HIDDEN)
    return fail(DPAC_EINVAL, "n_hidden must be in [1, %d] (got %d)", DPAC_MLP_MAX_HIDDEN, L);
  for (int i = 0; i <= L + 1; ++i) {
    if (net->width[i] < 1 || net->width[i] > DPAC_MLP_MAX_WIDTH)
      return fail(DPAC_EINVAL, "width[%d] = %d outside [1, %d]", i, net->width[i],
                  DPAC_MLP_MAX_WIDTH);
    if (!net->bn_scale[i] || !net->bn_shift[i])
      return fail(DPAC_EINVAL, "bn_scale/bn_shift[%d] is NULL", i);
  }
  if (!net->bias) return fail(DPAC_EINVAL, "bias is NULL");
  return check_guard_phase(net);
}

#define DPAC_REQUIRE(ptr) \
  if (!(ptr)) return fail(DPAC_EINVAL, "%s: required pointer '%s' is NULL", __func__, #ptr)

OpArgs blank(const dpac_eqn_params* eq, int op) {
  OpArgs a{};
  a.op = op;
  a.eq = *eq;
  return a;
}

int launch(const OpArgs& a) {
  int r = DPAC_EUNSUP;
  const bool f64 = a.dtype == DPAC_F64;
  // Kernels address each [N+1][B][d] / [N][B][c] / [B][N] array through one
  // 32-bit buffer descriptor whose offsets >= 2^31 mean "out of range".
  const int64_t esz = f64 ? 8 : 4;
  const int64_t width = a.eq.dim > a.eq.control_dim ? a.eq.dim : a.eq.control_dim;
  // B <= 2^31 and width <= 2^31 are checked before, so row_bytes cannot overflow; the step
  // count is compared by division (B * width * (N + 1) * esz overflows int64 for huge N:
  // found by the host UBSan run, tests/abi_sanitize.c)
  if (width > (1 << 16)) return fail(DPAC_EINVAL, "dim %d / control_dim %d too large", a.eq.dim, a.eq.control_dim);
  const int64_t limit = (int64_t)1 << 31, row_bytes = a.B * width * esz;
  if (row_bytes >= limit || ((int64_t)a.N + 1) > (limit - 1) / row_bytes)
    return fail(DPAC_EINVAL, "batch too large for one launch: every [N+1][B][d] array must stay "
                "below 2 GiB (B=%lld, N=%d, d=%d); split the batch over launches with "
                "traj_offset", (long long)a.B, a.N, a.eq.dim);
  const DispatchFn fn = find_dispatch(a.eq.eqn, a.eq.dim, f64 ? 1 : 0);
  r = fn ? fn(a) : DPAC_EUNSUP;
  if (r == DPAC_EUNSUP) return fail(r, "no kernel for equation %d dim %d", a.eq.eqn, a.eq.dim);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

// ---------------------------------------------------------------------------
// Sampler kernels (equation.py:13-44), stream layout in dpac_device.h.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void k_sample_dw(int64_t B, int64_t b0, int nb, int N, int D, int sample_type,
                                                   uint64_t seed, int64_t traj_offset, T* dw, bool pairs8) {
  // thread (unit u, trajectory b0 + bl, lane slot p, block): the stream layout of draw_slot(); a
  // unit is a step pair in the paired layout (S = 2), else one step.  x runs over this launch's
  // (bl, p, block) in 32-bit arithmetic, y over the units with a stride (round 6: the index
  // divisions formed once per thread, not per block: they cost more than its Philox rounds)
  const int P = lanes_for_dim(D), M = comps_per_lane(D);
  const int PB = dw_per_block<T>(sample_type);
  const int S = dw_steps_per_block<T>(M, sample_type);
  const int BPU = S == 2 ? 1 : (M + PB - 1) / PB;  // counter blocks per (unit, lane slot)
  const int units = S == 2 ? (N + 1) / 2 : N;
  const int PL = (D + M - 1) / M;                  // lane slots that own components (d = 20: 10 of 16)
  const uint32_t per_b = (uint32_t)(PL * BPU);
  const uint32_t idx = blockIdx.x * 256u + threadIdx.x;
  if (idx >= (uint32_t)nb * per_b) return;
  const uint32_t bl = idx / per_b, rem = idx - bl * per_b;
  const int p = (int)rem / BPU, blk = (int)rem - p * BPU;
  const int64_t b = b0 + bl;
  const uint64_t traj = (uint64_t)(traj_offset + b);
  // the values' places, fixed per thread: step offset within the unit and component (-1: none)
  int toff[4], jj[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int iv = blk * PB + e;  // the value's place in the lane slot's unit
    const int m = S == 2 ? iv % M : iv;
    const bool ok = e < PB && (S == 2 ? iv < 2 * M : m < M) && p * M + m < D;
    toff[e] = S == 2 ? iv / M : 0;
    jj[e] = ok ? p * M + m : -1;
  }
  T* const dwb = dw + b * D;
  const int64_t step = B * D;
  // two components per lane slot and step, d even, four values a block (f32 d = 20): each step's
  // pair is one 8-byte store
  if constexpr (sizeof(T) == 4) {
    if (pairs8 && S == 2 && M == 2 && PB == 4 && (D & 1) == 0) {  // pairs8: dw 8-byte aligned
      if (jj[0] < 0) return;
      for (int u = blockIdx.y; u < units; u += gridDim.y) {
        T vals[4];
        dw_block_values<T>(seed, traj, (uint64_t)u * P + p, sample_type, vals);
        const int t = 2 * u;
        *reinterpret_cast<float2*>(dwb + (int64_t)t * step + jj[0]) = make_float2(vals[0], vals[1]);
        if (t + 1 < N)
          *reinterpret_cast<float2*>(dwb + (int64_t)(t + 1) * step + jj[0]) = make_float2(vals[2], vals[3]);
      }
      return;
    }
  }
  for (int u = blockIdx.y; u < units; u += gridDim.y) {  // a few units per thread (grid y ~ 16)
    T vals[4];
    dw_block_values<T>(seed, traj, ((uint64_t)u * P + p) * BPU + blk, sample_type, vals);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int t = (S == 2 ? 2 * u : u) + toff[e];
      if (jj[e] >= 0 && t < N) dwb[(int64_t)t * step + jj[e]] = vals[e];
    }
  }
}

// A Gaussian direction (tag) of trajectory traj: component j is element j % PB of counter block
// (tag << 48) | (j / PB).  dir_sumsq: sum_j g_j^2 in component order; dir_write: out[j] =
// (scale * g_j) / nrm.  Each computes the ceil(D / PB) blocks once (round 6; rounds 1-5 drew a
// whole block per component, twice).
template <typename T>
__device__ T dir_sumsq(uint64_t seed, uint64_t traj, uint64_t tag, int D) {
  constexpr int PB = Rng<T>::kNormalPerBlock;
  T ss = 0;
  for (int c = 0; c * PB < D; ++c) {
    T n[PB];
    Rng<T>::normals(philox_block(seed, traj, (tag << 48) | (uint64_t)c), n);
#pragma unroll
    for (int e = 0; e < PB; ++e)
      if (c * PB + e < D) ss += n[e] * n[e];
  }
  return ss;
}
template <typename T>
__device__ void dir_write(uint64_t seed, uint64_t traj, uint64_t tag, int D, T scale, T nrm, T* out) {
  constexpr int PB = Rng<T>::kNormalPerBlock;
  for (int c = 0; c * PB < D; ++c) {
    T n[PB];
    Rng<T>::normals(philox_block(seed, traj, (tag << 48) | (uint64_t)c), n);
#pragma unroll
    for (int e = 0; e < PB; ++e)
      if (c * PB + e < D) out[c * PB + e] = (scale * n[e]) / nrm;
  }
}

template <typename T>
__global__ __launch_bounds__(256) void k_sample_points(int64_t B, int D, double R,
                                                       int sample_type, uint64_t seed,
                                                       int64_t traj_offset, T* x0, T* x_bdry) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint64_t traj = (uint64_t)(traj_offset + b);
  const T Rt = (T)R;
  if (x0) {
    if (sample_type == DPAC_SAMPLE_ZERO_X0) {
      for (int j = 0; j < D; ++j) x0[b * D + j] = (T)0.01;  // np.zeros + 0.01 (:39)
    } else {
      // r = (R*U)^(1/d) * R^((d-1)/d), U uniform (0,1]  (:14-15)
      const uint4 v = philox_block(seed, traj, kTagRadius << 48);
      T U;
      if constexpr (sizeof(T) == 4) U = rocrand_device::detail::uniform_distribution(v.x);
      else U = rocrand_device::detail::uniform_distribution_double(v.x, v.y);
      const T r = pow(Rt * U, (T)1 / (T)D) * pow(Rt, (T)(D - 1) / (T)D);
      dir_write<T>(seed, traj, kTagDir, D, r, sqrt(dir_sumsq<T>(seed, traj, kTagDir, D)), x0 + b * D);
    }
  }
  if (x_bdry)  // R * g / |g|  (:20-22)
    dir_write<T>(seed, traj, kTagBdry, D, Rt, sqrt(dir_sumsq<T>(seed, traj, kTagBdry, D)), x_bdry + b * D);
}

// One group of G = pow2 >= ceil(D / PB) lanes per (trajectory, point): lane c draws block c of
// the direction, lane 0 folds the squares in component order through shuffles (the same sum, bit
// for bit, as dir_sumsq), and every lane writes its block's components (round 6: the one-thread-
// per-trajectory kernel ran 16 workgroups at B = 4096, 10 us for 0.6 MB).  Point 0 is x0, 1 x_bdry.
template <typename T>
__global__ __launch_bounds__(256) void k_sample_points_grouped(int64_t B, int D, int G, double R,
                                                               int sample_type, uint64_t seed,
                                                               int64_t traj_offset, T* x0, T* x_bdry) {
  constexpr int PB = Rng<T>::kNormalPerBlock;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int c = (int)(idx & (G - 1));
  const int64_t task = idx / G;
  const int64_t b = task >> 1;
  const int kind = (int)(task & 1);
  T* const out = kind == 0 ? x0 : x_bdry;
  if (b >= B || out == nullptr) return;  // whole groups: G divides 64 and the grid
  const T Rt = (T)R;
  if (kind == 0 && sample_type == DPAC_SAMPLE_ZERO_X0) {
    for (int j = c; j < D; j += G) x0[b * D + j] = (T)0.01;  // np.zeros + 0.01 (:39)
    return;
  }
  const uint64_t traj = (uint64_t)(traj_offset + b);
  const uint64_t tag = kind == 0 ? kTagDir : kTagBdry;
  const int nblk = (D + PB - 1) / PB;
  T n[PB];
  if (c < nblk) {
    Rng<T>::normals(philox_block(seed, traj, (tag << 48) | (uint64_t)c), n);
  } else {
#pragma unroll
    for (int e = 0; e < PB; ++e) n[e] = 0;
  }
  T ss = 0;
  for (int k = 0; k < nblk; ++k) {
#pragma unroll
    for (int e = 0; e < PB; ++e) {
      const T v = __shfl(n[e], k, G);
      if (k * PB + e < D) ss += v * v;
    }
  }
  const T nrm = sqrt(__shfl(ss, 0, G));
  T scale = Rt;
  if (kind == 0) {  // r = (R*U)^(1/d) * R^((d-1)/d), U uniform (0,1]  (:14-15)
    const uint4 v = philox_block(seed, traj, kTagRadius << 48);
    T U;
    if constexpr (sizeof(T) == 4) U = rocrand_device::detail::uniform_distribution(v.x);
    else U = rocrand_device::detail::uniform_distribution_double(v.x, v.y);
    scale = pow(Rt * U, (T)1 / (T)D) * pow(Rt, (T)(D - 1) / (T)D);
  }
  if (c < nblk) {
#pragma unroll
    for (int e = 0; e < PB; ++e)
      if (c * PB + e < D) out[b * D + c * PB + e] = (scale * n[e]) / nrm;
  }
}

template <typename T>
int sample_impl(const dpac_eqn_params* eq, int32_t sample_type, int64_t B, int32_t N,
                uint64_t seed, int64_t off, void* x0, void* dw, void* x_bdry, hipStream_t s) {
  const int D = eq->dim;
  if (dw) {
    const int M = comps_per_lane(D);
    const int st = sample_type == DPAC_SAMPLE_ZERO_X0 ? DPAC_SAMPLE_NORMAL : sample_type;
    const int PB = dw_per_block<T>(st), S = dw_steps_per_block<T>(M, st);
    const int per_b = ((D + M - 1) / M) * (S == 2 ? 1 : (M + PB - 1) / PB);
    const int units = S == 2 ? (N + 1) / 2 : N;
    const int64_t chunk = (int64_t)1 << 24;  // trajectories per launch: 32-bit thread indices
    for (int64_t b0 = 0; b0 < B; b0 += chunk) {
      const int nb = (int)std::min<int64_t>(chunk, B - b0);
      // y: a few units per thread, more when x alone would not fill the chip
      const int64_t gx = ((int64_t)nb * per_b + 255) / 256;
      const int gy = (int)std::min<int64_t>(units, std::max<int64_t>(16, (4096 + gx - 1) / gx));
      const dim3 g((unsigned)gx, (unsigned)gy);
      const bool pairs8 = (reinterpret_cast<uintptr_t>(dw) & 7) == 0;  // a caller's odd-float view: scalar stores
      hipLaunchKernelGGL(k_sample_dw<T>, g, dim3(256), 0, s, B, b0, nb, N, D, st, seed, off, (T*)dw, pairs8);
      if (hipError_t e = hipGetLastError()) return (int)e;
    }
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  if (x0 || x_bdry) {
    const int nblk = (D + Rng<T>::kNormalPerBlock - 1) / Rng<T>::kNormalPerBlock;
    int G = 1;
    while (G < nblk) G *= 2;
    const char* serial = getenv("DPAC_SAMPLE_POINTS_SERIAL");  // read per call: tests compare the two
    if (G <= 64 && !(serial && serial[0] == '1')) {
      const int64_t threads = 2 * B * G;
      hipLaunchKernelGGL(k_sample_points_grouped<T>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s,
                         B, D, G, eq->R, sample_type, seed, off, (T*)x0, (T*)x_bdry);
    } else {  // more than 64 blocks of a direction: one thread per trajectory
      hipLaunchKernelGGL(k_sample_points<T>, dim3((unsigned)((B + 255) / 256)), dim3(256), 0, s, B,
                         D, eq->R, sample_type, seed, off, (T*)x0, (T*)x_bdry);
    }
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  return 0;
}

}  // namespace
}  // namespace dpac

using namespace dpac;

extern "C" {

int32_t dpac_abi_version(void) { return DPAC_ABI_VERSION; }

const char* dpac_last_error(void) { return g_err.c_str(); }

int32_t dpac_supported(const dpac_eqn_params* eq) { return check_eq(eq) == DPAC_OK ? 1 : 0; }

int dpac_sample(const dpac_eqn_params* eq, int32_t sample_type, int32_t dtype, int64_t num_sample,
                int32_t num_steps, uint64_t seed, int64_t traj_offset, void* x0, void* dw,
                void* x_bdry, void* stream) {
  if (!eq) return fail(DPAC_EINVAL, "eqn params pointer is NULL");
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (eq->dim < 1) return fail(DPAC_EINVAL, "dim must be >= 1");
  if (num_sample < 1) return fail(DPAC_EINVAL, "num_sample must be >= 1");
  if (dw && num_steps < 1) return fail(DPAC_EINVAL, "num_steps must be >= 1");
  if (int e = check_sample_type(sample_type)) return e;
  if (traj_offset < 0) return fail(DPAC_EINVAL, "traj_offset must be >= 0");
  hipStream_t s = (hipStream_t)stream;
  const int r = dtype == DPAC_F64
                    ? sample_impl<double>(eq, sample_type, num_sample, num_steps, seed,
                                          traj_offset, x0, dw, x_bdry, s)
                    : sample_impl<float>(eq, sample_type, num_sample, num_steps, seed,
                                         traj_offset, x0, dw, x_bdry, s);
  if (r) return fail(r, "sampler launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_rollout_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype, int64_t num_sample,
                     int32_t num_steps, double total_time, const void* x0, const void* dw,
                     uint64_t seed, int64_t traj_offset, int32_t sample_type, void* x, void* dt,
                     void* coef, void* u, int32_t cost_order, void* y, void* disc, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  DPAC_REQUIRE(x0);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(dt);
  DPAC_REQUIRE(coef);
  if ((y == nullptr) != (disc == nullptr))
    return fail(DPAC_EINVAL, "y and disc must both be given or both be NULL");
  if (cost_order != DPAC_COST_CRITIC && cost_order != DPAC_COST_ACTOR)
    return fail(DPAC_EINVAL, "bad cost_order %d", cost_order);
  if (!dw) {
    if (int e = check_sample_type(sample_type)) return e;
    if (traj_offset < 0) return fail(DPAC_EINVAL, "traj_offset must be >= 0");
  }
  OpArgs a = blank(eq, OP_ROLLOUT);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.x0 = x0; a.dw = dw; a.seed = seed; a.traj_offset = traj_offset;
  a.sample_type = sample_type == DPAC_SAMPLE_ZERO_X0 ? DPAC_SAMPLE_NORMAL : sample_type;
  a.x_out = x; a.dt = dt; a.coef = coef; a.u_out = u; a.cost_order = cost_order; a.y = y;
  a.disc = disc; a.stream = (hipStream_t)stream;
  return launch(a);
}

int32_t dpac_rollout_nn_mask_tile_bytes(const dpac_mlp* actor) {
  if (!actor || actor->n_hidden < 1 || actor->n_hidden > DPAC_MLP_MAX_HIDDEN) return 0;
  return nn_mask_tile_bytes(actor->n_hidden);
}

int64_t dpac_rollout_nn_mask_bytes(const dpac_mlp* actor, int32_t dtype, int64_t num_sample,
                                   int32_t num_steps) {
  if (!actor || actor->n_hidden < 1 || actor->n_hidden > DPAC_MLP_MAX_HIDDEN || num_sample < 1 ||
      num_steps < 1 || (dtype != DPAC_F32 && dtype != DPAC_F64))
    return fail(DPAC_EINVAL, "dpac_rollout_nn_mask_bytes: bad arguments"), -1;
  ok();
  // the same selection as run_op's OP_ROLLOUT_NN: float, 16-row tiles, the fast path
  if (dtype != DPAC_F32) return 0;
  const int tile = nn_tile_rows();
  if (tile == 4 || (tile == 0 && num_sample <= 1024)) return 0;
  const int L = actor->n_hidden;
  if (!nn_fast_host<float>(L, actor->width, actor->weight_km, actor->width[0], actor->width[L + 1]) &&
      !nn_x3_host(L, actor->width, actor->weight_x3, actor->width[0], actor->width[L + 1]))
    return 0;
  return (int64_t)num_steps * ((num_sample + 15) / 16) * nn_mask_tile_bytes(L);
}

int dpac_rollout_nn_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                        int64_t num_sample, int32_t num_steps, double total_time,
                        const dpac_mlp* actor, const void* x0, const void* dw, void* x,
                        void* dt, void* coef, void* u, int32_t cost_order, void* y,
                        void* disc, void* save_z, int32_t* save_flag, void* save_disc,
                        void* stream) {
  return dpac_rollout_nn_fwd_masked(eq, scheme, dtype, num_sample, num_steps, total_time, actor, x0, dw, x,
                                    dt, coef, u, cost_order, y, disc, save_z, save_flag, save_disc, nullptr,
                                    nullptr, stream);
}

int dpac_rollout_nn_fwd_masked(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                               int64_t num_sample, int32_t num_steps, double total_time,
                               const dpac_mlp* actor, const void* x0, const void* dw, void* x,
                               void* dt, void* coef, void* u, int32_t cost_order, void* y,
                               void* disc, void* save_z, int32_t* save_flag, void* save_disc,
                               uint8_t* save_mask, int32_t* mask_written, void* stream) {
  if (mask_written) *mask_written = 0;
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  if (int e = check_mlp(eq, actor)) return e;
  DPAC_REQUIRE(x0);
  DPAC_REQUIRE(dw);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(dt);
  DPAC_REQUIRE(coef);
  if ((y == nullptr) != (disc == nullptr))
    return fail(DPAC_EINVAL, "y and disc must both be given or both be NULL");
  if (cost_order != DPAC_COST_CRITIC && cost_order != DPAC_COST_ACTOR)
    return fail(DPAC_EINVAL, "bad cost_order %d", cost_order);
  const int nsave = (save_z != nullptr) + (save_flag != nullptr) + (save_disc != nullptr);
  if (nsave != 0 && nsave != 3)
    return fail(DPAC_EINVAL, "save_z, save_flag and save_disc must all be given or all be NULL");
  OpArgs a = blank(eq, OP_ROLLOUT_NN);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.x0 = x0; a.dw = dw; a.mlp = *actor;
  a.x_out = x; a.dt = dt; a.coef = coef; a.u_out = u; a.cost_order = cost_order; a.y = y;
  a.disc = disc; a.save_z = save_z; a.save_flag = save_flag; a.save_disc = save_disc;
  if (save_mask && nsave != 3) return fail(DPAC_EINVAL, "save_mask needs the other backward saves");
  a.save_mask = save_mask; a.mask_written = mask_written;
  a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_rollout_nn_bwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                        int64_t num_sample, int32_t num_steps, double total_time,
                        const dpac_mlp* actor, const void* const* weight_t,
                        const void* const* weight_t_km, const void* x,
                        const void* u, const void* dw, const void* save_z,
                        const int32_t* save_flag, const void* save_disc, const void* g_xN,
                        const void* g_disc, const void* g_y, void* G, void* g_x0,
                        void* stream) {
  return dpac_rollout_nn_bwd_masked(eq, scheme, dtype, num_sample, num_steps, total_time, actor, weight_t,
                                    weight_t_km, x, u, dw, save_z, save_flag, save_disc, nullptr, g_xN,
                                    g_disc, g_y, G, g_x0, stream);
}

int dpac_rollout_nn_bwd_masked(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                               int64_t num_sample, int32_t num_steps, double total_time,
                               const dpac_mlp* actor, const void* const* weight_t,
                               const void* const* weight_t_km, const void* x,
                               const void* u, const void* dw, const void* save_z,
                               const int32_t* save_flag, const void* save_disc,
                               const uint8_t* save_mask, const void* g_xN,
                               const void* g_disc, const void* g_y, void* G, void* g_x0,
                               void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  if (int e = check_mlp(eq, actor)) return e;
  DPAC_REQUIRE(weight_t);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(u);
  DPAC_REQUIRE(dw);
  DPAC_REQUIRE(save_z);
  DPAC_REQUIRE(save_flag);
  DPAC_REQUIRE(save_disc);
  DPAC_REQUIRE(G);
  for (int i = 0; i <= actor->n_hidden; ++i)
    if (!weight_t[i]) return fail(DPAC_EINVAL, "weight_t[%d] is NULL", i);
  OpArgs a = blank(eq, OP_ROLLOUT_NN_BWD);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.mlp = *actor;
  for (int i = 0; i <= actor->n_hidden; ++i) {
    a.mlp_wt[i] = weight_t[i];
    a.mlp.weight_km[i] = weight_t_km ? weight_t_km[i] : nullptr;  // the backward's images
  }
  a.x = x; a.u = u; a.dw = dw; a.save_z = const_cast<void*>(save_z);
  a.save_flag = const_cast<int32_t*>(save_flag); a.save_disc = const_cast<void*>(save_disc);
  a.g_x_out = g_xN; a.g_disc_out = g_disc; a.g_y_out = g_y; a.g_G = G; a.g_x = g_x0;
  a.mask_in = save_mask;
  a.stream = (hipStream_t)stream;
  return launch(a);
}

int64_t dpac_mlp_rows_mask_bytes(const dpac_mlp* net, int32_t dtype, int64_t rows) {
  if (check_net(net)) return -1;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype), -1;
  if (rows < 1) return fail(DPAC_EINVAL, "rows must be >= 1"), -1;
  ok();
  return mlp_rows_mask_bytes(dtype, rows, *net);
}

int dpac_mlp_rows_fwd(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* x,
                      int64_t ldx, void* out, void* save_z, void* stream) {
  return dpac_mlp_rows_fwd_masked(dtype, rows, net, x, ldx, out, save_z, nullptr, nullptr, stream);
}

int dpac_mlp_rows_fwd_masked(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* x,
                             int64_t ldx, void* out, void* save_z, uint8_t* save_mask,
                             int32_t* mask_written, void* stream) {
  if (mask_written) *mask_written = 0;
  if (int e = check_net(net)) return e;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (rows < 1) return fail(DPAC_EINVAL, "rows must be >= 1 (got %lld)", (long long)rows);
  if (ldx < net->width[0]) return fail(DPAC_EINVAL, "ldx (%lld) < width[0] (%d)", (long long)ldx,
                                       net->width[0]);
  for (int i = 0; i <= net->n_hidden; ++i)
    if (!net->weight[i]) return fail(DPAC_EINVAL, "weight[%d] is NULL", i);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(out);
  if (save_mask && !save_z) return fail(DPAC_EINVAL, "save_mask needs save_z");
  const int r = mlp_rows_fwd_launch(dtype, rows, *net, x, ldx, out, save_z, nullptr, save_mask, mask_written,
                                    (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_mlp_rows_bwd(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* const* weight_t,
                      const void* const* weight_t_km, const void* save_z, const void* g_out, void* G,
                      void* g_x, void* stream) {
  return dpac_mlp_rows_bwd_masked(dtype, rows, net, weight_t, weight_t_km, save_z, nullptr, g_out, G, g_x,
                                  stream);
}

int dpac_mlp_rows_bwd_masked(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* const* weight_t,
                             const void* const* weight_t_km, const void* save_z, const uint8_t* save_mask,
                             const void* g_out, void* G, void* g_x, void* stream) {
  if (int e = check_net(net)) return e;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (rows < 1) return fail(DPAC_EINVAL, "rows must be >= 1 (got %lld)", (long long)rows);
  DPAC_REQUIRE(weight_t);
  DPAC_REQUIRE(save_z);
  DPAC_REQUIRE(g_out);
  DPAC_REQUIRE(G);
  for (int i = 0; i <= net->n_hidden; ++i)
    if (!weight_t[i]) return fail(DPAC_EINVAL, "weight_t[%d] is NULL", i);
  dpac_mlp bnet = *net;  // the struct's weight_km (forward images) never reach the backward
  for (int i = 0; i <= net->n_hidden; ++i) bnet.weight_km[i] = weight_t_km ? weight_t_km[i] : nullptr;
  const int r = mlp_rows_bwd_launch(dtype, rows, bnet, weight_t, save_z, save_mask, g_out, G, g_x, nullptr,
                                    (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

// The equation's elementwise sigma as (sa, sb) and k_td's lane split, for the fused
// TD1 entry points (TdRows, dpac_device.h; used by dpac_mlp_rows.h).  Both come from the
// equation functors themselves (E::sigma_form, eqn_lanes), over an explicit allow-list of
// equation ids, so a new equation cannot reach the fused path with another's sigma.
static int td_rows_setup(const dpac_eqn_params* eq, int32_t dtype, int64_t rows, const dpac_mlp* net,
                         dpac::TdRows& td) {
  if (int e = check_common(eq, dtype, rows)) return e;
  if (int e = check_net(net)) return e;
  if (net->ekn_head) return fail(DPAC_EINVAL, "the fused TD1 G network takes no Eikonal head");
  const int d = eq->dim;
  if (net->width[net->n_hidden + 1] != d)
    return fail(DPAC_EINVAL, "the network's output width (%d) must equal dim (%d)",
                net->width[net->n_hidden + 1], d);
  if (net->width[0] != d)
    return fail(DPAC_EINVAL, "the network's input width (%d) must equal dim (%d)", net->width[0], d);
  switch (eq->eqn) {  // the functor's template arguments do not enter sigma_form
    case DPAC_EQN_LQR: dpac::EqLQR<double, 1, 1>::sigma_form(*eq, td.sa, td.sb); break;
    case DPAC_EQN_LQR_VAR: dpac::EqLQRVar<double, 1, 1>::sigma_form(*eq, td.sa, td.sb); break;
    case DPAC_EQN_EKN: dpac::EqEKN<double, 1, 1>::sigma_form(*eq, td.sa, td.sb); break;
    case DPAC_EQN_VDP: dpac::EqVDP<double, 2, 1>::sigma_form(*eq, td.sa, td.sb); break;
    default: return fail(DPAC_EUNSUP, "no fused TD1 path for equation %d", eq->eqn);
  }
  td.p = eqn_lanes(eq->eqn, d);  // E::kP of the equation's k_td
  td.ldu = eq->control_dim;
  return 0;
}

int dpac_mlp_rows_fwd_td1(const dpac_eqn_params* eq, int32_t dtype, int64_t rows, const dpac_mlp* net,
                          const void* x, int64_t ldx, const void* u, const void* dw, void* gdot,
                          void* save_z, void* stream) {
  return dpac_mlp_rows_fwd_td1_masked(eq, dtype, rows, net, x, ldx, u, dw, gdot, save_z, nullptr, nullptr,
                                      stream);
}

int dpac_mlp_rows_fwd_td1_masked(const dpac_eqn_params* eq, int32_t dtype, int64_t rows, const dpac_mlp* net,
                                 const void* x, int64_t ldx, const void* u, const void* dw, void* gdot,
                                 void* save_z, uint8_t* save_mask, int32_t* mask_written, void* stream) {
  if (mask_written) *mask_written = 0;
  dpac::TdRows td{};
  if (int e = td_rows_setup(eq, dtype, rows, net, td)) return e;
  if (ldx < eq->dim) return fail(DPAC_EINVAL, "ldx (%lld) < dim (%d)", (long long)ldx, eq->dim);
  for (int i = 0; i <= net->n_hidden; ++i)
    if (!net->weight[i]) return fail(DPAC_EINVAL, "weight[%d] is NULL", i);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(dw);
  DPAC_REQUIRE(gdot);
  if (td.sb != 0.0) DPAC_REQUIRE(u);
  if (save_mask && !save_z) return fail(DPAC_EINVAL, "save_mask needs save_z");
  td.x = x; td.ldx = ldx; td.u = u; td.dw = dw; td.gdot = gdot;
  const int r = mlp_rows_fwd_launch(dtype, rows, *net, x, ldx, nullptr, save_z, &td, save_mask, mask_written,
                                    (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_mlp_rows_bwd_td1(const dpac_eqn_params* eq, int32_t dtype, int64_t rows, const dpac_mlp* net,
                          const void* const* weight_t, const void* const* weight_t_km,
                          const void* save_z, const void* x, int64_t ldx, const void* u,
                          const void* dw, const void* g_gdot, void* G, void* g_x, void* stream) {
  return dpac_mlp_rows_bwd_td1_masked(eq, dtype, rows, net, weight_t, weight_t_km, save_z, nullptr, x, ldx, u,
                                      dw, g_gdot, G, g_x, stream);
}

int dpac_mlp_rows_bwd_td1_masked(const dpac_eqn_params* eq, int32_t dtype, int64_t rows, const dpac_mlp* net,
                                 const void* const* weight_t, const void* const* weight_t_km,
                                 const void* save_z, const uint8_t* save_mask, const void* x, int64_t ldx,
                                 const void* u, const void* dw, const void* g_gdot, void* G, void* g_x,
                                 void* stream) {
  dpac::TdRows td{};
  if (int e = td_rows_setup(eq, dtype, rows, net, td)) return e;
  if (ldx < eq->dim) return fail(DPAC_EINVAL, "ldx (%lld) < dim (%d)", (long long)ldx, eq->dim);
  DPAC_REQUIRE(weight_t);
  DPAC_REQUIRE(save_z);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(dw);
  DPAC_REQUIRE(g_gdot);
  DPAC_REQUIRE(G);
  if (td.sb != 0.0) DPAC_REQUIRE(u);
  for (int i = 0; i <= net->n_hidden; ++i)
    if (!weight_t[i]) return fail(DPAC_EINVAL, "weight_t[%d] is NULL", i);
  dpac_mlp bnet = *net;
  for (int i = 0; i <= net->n_hidden; ++i) bnet.weight_km[i] = weight_t_km ? weight_t_km[i] : nullptr;
  td.x = x; td.ldx = ldx; td.u = u; td.dw = dw; td.g_gdot = g_gdot;
  const int r = mlp_rows_bwd_launch(dtype, rows, bnet, weight_t, save_z, save_mask, nullptr, G, g_x, &td,
                                    (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int64_t dpac_mlp_param_grads_workspace(int32_t dtype, int64_t rows, const dpac_mlp* net) {
  if (check_net(net)) return -1;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype), -1;
  if (rows < 1) return fail(DPAC_EINVAL, "rows must be >= 1"), -1;
  ok();
  return mlp_param_grads_ws_bytes(dtype, rows, *net);
}

int dpac_mlp_param_grads(int32_t dtype, int64_t rows, const dpac_mlp* net, double gamma_scale,
                         const void* x, int64_t ldx, const void* save_z, const void* G,
                         void* workspace, int64_t workspace_bytes, void* grads, void* stream) {
  if (int e = check_net(net)) return e;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (rows < 1) return fail(DPAC_EINVAL, "rows must be >= 1 (got %lld)", (long long)rows);
  if (ldx < net->width[0]) return fail(DPAC_EINVAL, "ldx (%lld) < width[0] (%d)", (long long)ldx,
                                       net->width[0]);
  {
    int gtot = 0;
    for (int i = 0; i <= net->n_hidden + 1; ++i) gtot += net->width[i];
    if (ldx > gtot)
      return fail(DPAC_EINVAL, "ldx (%lld) must not exceed the G row width (%d)", (long long)ldx,
                  gtot);
  }
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(save_z);
  DPAC_REQUIRE(G);
  DPAC_REQUIRE(workspace);
  DPAC_REQUIRE(grads);
  const int64_t need = mlp_param_grads_ws_bytes(dtype, rows, *net);
  if (workspace_bytes < need)
    return fail(DPAC_EINVAL, "workspace too small: %lld bytes, need %lld",
                (long long)workspace_bytes, (long long)need);
  const int r = mlp_param_grads_launch(dtype, rows, *net, gamma_scale, x, ldx, save_z, G,
                                       workspace, grads, (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_flag_init(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype, int64_t num_sample,
                   int32_t num_steps, double total_time, const void* x0, int32_t* flag,
                   void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  DPAC_REQUIRE(x0);
  DPAC_REQUIRE(flag);
  OpArgs a = blank(eq, OP_FLAG_INIT);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.x0 = x0; a.flag_out = flag; a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_step_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype, int64_t num_sample,
                  int32_t num_steps, double total_time, const void* x, const void* u,
                  const void* dw_t, const int32_t* flag_in, const void* disc_in, const void* y_in,
                  int32_t cost_order, void* x_out, int32_t* flag_out, void* disc_out, void* y_out,
                  void* dt, void* coef, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(u);
  DPAC_REQUIRE(dw_t);
  DPAC_REQUIRE(flag_in);
  DPAC_REQUIRE(x_out);
  DPAC_REQUIRE(flag_out);
  if (x_out == x) return fail(DPAC_EINVAL, "x_out must not alias x");
  if (cost_order != DPAC_COST_CRITIC && cost_order != DPAC_COST_ACTOR)
    return fail(DPAC_EINVAL, "bad cost_order %d", cost_order);
  OpArgs a = blank(eq, OP_STEP_FWD);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.x = x; a.u = u; a.dw = dw_t; a.flag_in = flag_in; a.disc_in = disc_in; a.y_in = y_in;
  a.cost_order = cost_order; a.x_out = x_out; a.flag_out = flag_out; a.disc_out = disc_out;
  a.y_out = y_out; a.dt = dt; a.coef = coef; a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_step_bwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype, int64_t num_sample,
                  int32_t num_steps, double total_time, const void* x, const void* u,
                  const void* dw_t, const int32_t* flag_in, const void* disc_in,
                  int32_t cost_order, const void* g_x_out, const void* g_disc_out,
                  const void* g_y_out, void* g_x, void* g_u, void* g_disc, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (int e = check_time(scheme, num_steps, total_time)) return e;
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(u);
  DPAC_REQUIRE(dw_t);
  DPAC_REQUIRE(flag_in);
  DPAC_REQUIRE(g_x_out);
  DPAC_REQUIRE(g_x);
  DPAC_REQUIRE(g_u);
  if (cost_order != DPAC_COST_CRITIC && cost_order != DPAC_COST_ACTOR)
    return fail(DPAC_EINVAL, "bad cost_order %d", cost_order);
  OpArgs a = blank(eq, OP_STEP_BWD);
  a.scheme = scheme; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = total_time;
  a.x = x; a.u = u; a.dw = dw_t; a.flag_in = flag_in; a.disc_in = disc_in;
  a.cost_order = cost_order; a.g_x_out = g_x_out; a.g_disc_out = g_disc_out;
  a.g_y_out = g_y_out; a.g_x = g_x; a.g_u = g_u; a.g_disc = g_disc;
  a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_td_assemble_fwd(const dpac_eqn_params* eq, int32_t td_type, int32_t cost_order,
                         int32_t dtype, int64_t num_sample, int32_t num_steps, const void* x,
                         const void* u, const void* dw, uint64_t seed, int64_t traj_offset,
                         int32_t sample_type, const void* dt, const void* coef, const void* G,
                         void* y, void* disc, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (num_steps < 1) return fail(DPAC_EINVAL, "num_steps must be >= 1");
  if (td_type != DPAC_TD1 && td_type != DPAC_TD2 && td_type != DPAC_TD1_GDOT)
    return fail(DPAC_EINVAL, "bad td_type %d", td_type);
  if (cost_order != DPAC_COST_CRITIC && cost_order != DPAC_COST_ACTOR)
    return fail(DPAC_EINVAL, "bad cost_order %d", cost_order);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(u);
  DPAC_REQUIRE(dt);
  DPAC_REQUIRE(coef);
  DPAC_REQUIRE(y);
  DPAC_REQUIRE(disc);
  if (td_type == DPAC_TD1) {
    DPAC_REQUIRE(G);
    if (!dw) {
      if (int e = check_sample_type(sample_type)) return e;
    }
  }
  if (td_type == DPAC_TD1_GDOT) DPAC_REQUIRE(G);  // gdot [N][B]; dw is not read
  OpArgs a = blank(eq, OP_TD_FWD);
  a.td_type = td_type; a.cost_order = cost_order; a.dtype = dtype; a.B = num_sample;
  a.N = num_steps; a.T = 1.0; a.x = x; a.u = u; a.dw = dw; a.seed = seed;
  a.traj_offset = traj_offset;
  a.sample_type = sample_type == DPAC_SAMPLE_ZERO_X0 ? DPAC_SAMPLE_NORMAL : sample_type;
  a.dt_in = dt; a.coef_in = coef; a.G = G; a.y = y; a.disc = disc;
  a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_td_assemble_bwd(const dpac_eqn_params* eq, int32_t dtype, int64_t num_sample,
                         int32_t num_steps, const void* x, const void* u, const void* dw,
                         uint64_t seed, int64_t traj_offset, int32_t sample_type, const void* dt,
                         const void* coef, const void* g_y, void* g_G, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (num_steps < 1) return fail(DPAC_EINVAL, "num_steps must be >= 1");
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(u);
  DPAC_REQUIRE(dt);
  DPAC_REQUIRE(coef);
  DPAC_REQUIRE(g_y);
  DPAC_REQUIRE(g_G);
  if (!dw) {
    if (int e = check_sample_type(sample_type)) return e;
  }
  OpArgs a = blank(eq, OP_TD_BWD);
  a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = 1.0; a.x = x; a.u = u; a.dw = dw;
  a.seed = seed; a.traj_offset = traj_offset;
  a.sample_type = sample_type == DPAC_SAMPLE_ZERO_X0 ? DPAC_SAMPLE_NORMAL : sample_type;
  a.dt_in = dt; a.coef_in = coef; a.g_y_out = g_y; a.g_G = g_G; a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_td_assemble_bwd_gdot(const dpac_eqn_params* eq, int32_t dtype, int64_t num_sample,
                              int32_t num_steps, const void* dt, const void* coef, const void* g_y,
                              void* g_gdot, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (num_steps < 1) return fail(DPAC_EINVAL, "num_steps must be >= 1");
  DPAC_REQUIRE(dt);
  DPAC_REQUIRE(coef);
  DPAC_REQUIRE(g_y);
  DPAC_REQUIRE(g_gdot);
  OpArgs a = blank(eq, OP_TD_BWD);
  a.td_type = DPAC_TD1_GDOT; a.dtype = dtype; a.B = num_sample; a.N = num_steps; a.T = 1.0;
  a.dt_in = dt; a.coef_in = coef; a.g_y_out = g_y; a.g_G = g_gdot; a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_actor_cost_fwd(const dpac_eqn_params* eq, int32_t dtype, int64_t num_sample,
                        int32_t num_steps, const void* x, const void* u, const void* dt,
                        const void* coef, void* y, void* disc, void* stream) {
  return dpac_td_assemble_fwd(eq, DPAC_TD2, DPAC_COST_ACTOR, dtype, num_sample, num_steps, x, u,
                              nullptr, 0, 0, DPAC_SAMPLE_NORMAL, dt, coef, nullptr, y, disc, stream);
}

int dpac_equation_eval(const dpac_eqn_params* eq, int32_t what, int32_t dtype, int64_t num_sample,
                       const void* x, const void* u, void* out, void* stream) {
  if (int e = check_common(eq, dtype, num_sample)) return e;
  if (what < DPAC_EVAL_DRIFT || what > DPAC_EVAL_B) return fail(DPAC_EINVAL, "bad eval id %d", what);
  DPAC_REQUIRE(x);
  DPAC_REQUIRE(out);
  if ((what == DPAC_EVAL_DRIFT || what == DPAC_EVAL_SIGMA || what == DPAC_EVAL_W) && !u)
    return fail(DPAC_EINVAL, "eval %d needs u", what);
  OpArgs a = blank(eq, OP_EVAL);
  a.what = what; a.dtype = dtype; a.B = num_sample; a.N = 1; a.T = 1.0; a.x = x; a.u = u;
  a.out = out; a.stream = (hipStream_t)stream;
  return launch(a);
}

int dpac_mlp_prepare(int32_t dtype, const dpac_mlp* net, double gamma_scale, void* scales,
                     void* weight_t, void* weight_km, void* weight_t_km, void* weight_x3,
                     void* weight_t_x3, void* stream) {
  if (int e = check_net(net)) return e;
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  DPAC_REQUIRE(scales);
  if ((weight_x3 || weight_t_x3) && dtype != DPAC_F32)
    return fail(DPAC_EINVAL, "split-fp16 images (weight_x3 / weight_t_x3) are float-only");
  if (weight_t || weight_km || weight_t_km || weight_x3 || weight_t_x3)
    for (int i = 0; i <= net->n_hidden; ++i)
      if (!net->weight[i]) return fail(DPAC_EINVAL, "weight[%d] is NULL", i);
  const int r = mlp_prepare_launch(dtype, *net, gamma_scale, scales, weight_t, weight_km,
                                   weight_t_km, weight_x3, weight_t_x3, (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_adam_apply(int32_t dtype, int32_t n_tensors, const int64_t* numel, void* const* var,
                    const void* const* grad, void* const* m, void* const* v, double alpha,
                    double beta_1, double beta_2, double epsilon, void* stream) {
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (n_tensors < 0) return fail(DPAC_EINVAL, "n_tensors must be >= 0 (got %d)", n_tensors);
  if (n_tensors == 0) return ok();
  DPAC_REQUIRE(numel);
  DPAC_REQUIRE(var);
  DPAC_REQUIRE(grad);
  DPAC_REQUIRE(m);
  DPAC_REQUIRE(v);
  for (int i = 0; i < n_tensors; ++i) {
    if (numel[i] < 1) return fail(DPAC_EINVAL, "tensor %d: numel must be >= 1", i);
    if (!var[i] || !grad[i] || !m[i] || !v[i])
      return fail(DPAC_EINVAL, "tensor %d: a pointer is NULL", i);
  }
  const int r = adam_launch(dtype, n_tensors, numel, var, grad, m, v, alpha, beta_1, beta_2,
                            epsilon, (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

int dpac_critic_loss_grad(int32_t dtype, int64_t num_sample, const void* V, const void* y, const void* disc,
                          const void* z_bdry, double scale, double delta_clip, void* g_out, void* neg_g,
                          void* stream) {
  if (dtype != DPAC_F32 && dtype != DPAC_F64) return fail(DPAC_EINVAL, "bad dtype %d", dtype);
  if (num_sample < 1) return fail(DPAC_EINVAL, "num_sample must be >= 1 (got %lld)", (long long)num_sample);
  if (!(delta_clip > 0)) return fail(DPAC_EINVAL, "delta_clip must be > 0");
  DPAC_REQUIRE(V);
  DPAC_REQUIRE(y);
  DPAC_REQUIRE(disc);
  DPAC_REQUIRE(z_bdry);
  DPAC_REQUIRE(g_out);
  DPAC_REQUIRE(neg_g);
  const int r = critic_loss_launch(dtype, num_sample, V, y, disc, z_bdry, scale, delta_clip, g_out, neg_g,
                                   (hipStream_t)stream);
  if (r != 0) return fail(r, "kernel launch failed: %s", hipGetErrorString((hipError_t)r));
  return ok();
}

}  // extern "C"
