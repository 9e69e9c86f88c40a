/*
 * dpac.h — C ABI of libdpac, the MI355X (gfx950) hot path of the actor-critic
 * HJB solver: batched Euler–Maruyama rollout of the boundary-stopped controlled
 * SDE, running-cost / discount accumulation, VR-LSTD (TD1) / LSTD (TD2) target
 * assembly, the per-step transition used for back-propagation through the
 * rollout, and the on-device Brownian sampler.
 *
 * The reference (MoZhou1995/DeepPDE_ActorCritic) has no FFI: its "plugin" surface
 * is the Python `Equation` class in equation.py and the `CriticModel` /
 * `ActorModel` classes in solver.py, with TensorFlow ops underneath.  Every entry
 * point below replaces one of those Python/TF code paths; the replaced lines are
 * cited on each declaration.  The Python package `deeppde_actorcritic_amd` binds
 * this header with ctypes.
 *
 * Conventions
 *  - Plain C: no C++ types, no torch types, no exceptions across the ABI.
 *  - The caller owns every buffer.  All data pointers are DEVICE pointers
 *    (hipMalloc / torch tensors on the GPU) unless the name says otherwise.
 *  - Every launch is stream-ordered on `stream` (a hipStream_t; NULL = the legacy
 *    default stream).  Nothing synchronises the host.
 *  - `dtype` is DPAC_F32 or DPAC_F64 and applies to every floating buffer of the
 *    call.  Flags are int32.
 *  - Return value: 0 on success, DPAC_EINVAL for a bad argument, DPAC_EUNSUP for
 *    an unsupported (equation, dim) combination, otherwise the hipError_t of the
 *    failed launch.  dpac_last_error() returns a thread-local message.
 *
 * HBM layouts (B = num_sample, d = dim, c = control_dim, N = num_steps).  State,
 * noise and control are step-major (one [B][d] slab per step, read/written as a
 * unit by every step of the time loop); the per-step scalars dt and coef are
 * trajectory-major, exactly the reference's dt[B,N] / coef[B,N]
 * (equation.py:70,99):
 *    x0, x_bdry  [B][d]            x     [N+1][B][d]      dw  [N][B][d]
 *    u           [N][B][c]         dt    [B][N]           coef [B][N]
 *    G           [N][B][d]         flag  [B] (int32)      y, disc [B]
 * The single-step entry points (dpac_step_fwd/bwd) take and return one step's
 * [B] vectors.  The reference keeps x_smp as [B][d][N+1] and dw as [B][d][N]
 * (equation.py:19,50,68); the Python shims transpose only at the parity boundary.
 * Limit: B·(N+1)·max(d,c)·sizeof(T) must stay below 2 GiB (each array is
 * addressed through one 32-bit buffer descriptor); else DPAC_EINVAL.  Larger
 * batches are split over launches; traj_offset keeps the in-kernel noise of
 * every trajectory the same under any split.
 */
#ifndef DPAC_H_
#define DPAC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: dpac_rollout_nn_bwd / dpac_mlp_rows_bwd take weight_t_km (round 2); adds
 * dpac_rollout_nn_mask_bytes.  3: dpac_mlp gains weight_x3 / weight_t_x3 (split-fp16
 * images) and dpac_mlp_prepare writes them.  4: the split-fp16 images are fragment-major
 * (below) and the float fused rollout / BPTT (dpac_rollout_nn_fwd[_masked],
 * dpac_rollout_nn_bwd_masked) read them too.  5: adds dpac_critic_loss_grad.  6: dpac_mlp gains
 * `status` (the split-fp16 range guard, below).  7: adds the row kernels' sign-bit mask
 * (dpac_mlp_rows_mask_bytes, dpac_mlp_rows_{fwd,bwd}[_td1]_masked).  8: dpac_mlp gains
 * `guard_phase` (the range guard's fallback launched apart from its split-fp16 launch, below).
 * Bindings must refuse a library of another version. */
#define DPAC_ABI_VERSION 8

/* status codes besides hipError_t values */
#define DPAC_OK 0
#define DPAC_EINVAL (-1)
#define DPAC_EUNSUP (-2)

/* dtypes */
#define DPAC_F32 0
#define DPAC_F64 1

/* equations — reference classes equation.py:144 (LQR), :179 (VDP), :240 (ekn), :278 (LQR_var) */
#define DPAC_EQN_LQR 0
#define DPAC_EQN_VDP 1
#define DPAC_EQN_EKN 2
#define DPAC_EQN_LQR_VAR 3

/* time-stepping schemes — equation.py:46 (naive), :73 (adaptive) */
#define DPAC_SCHEME_NAIVE 0
#define DPAC_SCHEME_ADAPTIVE 1

/* TD targets — solver.py:177 ("TD1" = VR-LSTD with the G control variate; "TD2" = LSTD) */
#define DPAC_TD1 1
#define DPAC_TD2 2
#define DPAC_TD1_GDOT 3 /* TD1 with the diffusion dot precomputed (dpac_mlp_rows_fwd_td1) */

/* cost-accumulation order: the critic (solver.py:170-174) and the actor
 * (solver.py:218) multiply the same four factors in different orders */
#define DPAC_COST_CRITIC 0
#define DPAC_COST_ACTOR 1

/* Brownian increments — equation.py:13 (normal), :25 (bounded 3-point), :38 (sample0) */
#define DPAC_SAMPLE_NORMAL 0
#define DPAC_SAMPLE_BOUNDED 1
#define DPAC_SAMPLE_ZERO_X0 2 /* sample0: x0 = 0.01 in every component, dw normal */

/* quantities for dpac_equation_eval (device versions of the Equation methods) */
#define DPAC_EVAL_DRIFT 0     /* out [B][d]  equation.py:136 drift(x,u) */
#define DPAC_EVAL_SIGMA 1     /* out [B][d]  diagonal of sigma(x,u), equation.py:132 */
#define DPAC_EVAL_W 2         /* out [B]     w_tf(x,u), equation.py:108 */
#define DPAC_EVAL_Z 3         /* out [B]     Z_tf(x), equation.py:112 */
#define DPAC_EVAL_V_TRUE 4    /* out [B]     V_true(x), equation.py:124 */
#define DPAC_EVAL_U_TRUE 5    /* out [B][c]  u_true(x), equation.py:128 */
#define DPAC_EVAL_V_GRAD 6    /* out [B][d]  V_grad_true(x), e.g. equation.py:166 */
#define DPAC_EVAL_B 7         /* out [B]     b_tf(x) = |x|^2 - R^2, equation.py:120 */

/*
 * Equation coefficients, filled by the host from eqn_config (equation.py:7-11 and
 * each subclass __init__).  Derived constants are computed by the host exactly as
 * the reference does: LQR k (equation.py:151), LQR_var k = (sqrt(5)-1)/2
 * (equation.py:282), sigma_up = sqrt(2) (equation.py:152,186,247,286).
 */
typedef struct dpac_eqn_params {
  int32_t eqn;         /* DPAC_EQN_* */
  int32_t dim;         /* d */
  int32_t control_dim; /* c (VDP: d/2, otherwise d) */
  int32_t reserved;    /* must be 0 */
  double gamma;        /* discount */
  double R;            /* domain radius */
  double sigma_up;     /* upper bound of sigma used by the adaptive scheme */
  double p, q, beta, k; /* LQR (p,q,beta,k); LQR_var (q,beta,k); VDP (q) */
  double a, epsilon;    /* VDP (a, epsilon); LQR_var (epsilon) */
  double a2, a3;        /* EKN */
} dpac_eqn_params;

/* ---- introspection ------------------------------------------------------ */
int32_t dpac_abi_version(void);
const char* dpac_last_error(void);
/* 1 if (eqn, dim, control_dim) has a compiled kernel instantiation */
int32_t dpac_supported(const dpac_eqn_params* eq);

/* ---- sampler (on-device, rocRAND Philox4x32-10) -------------------------
 * Replaces Equation.sample_normal / sample_bounded / sample0
 * (equation.py:13-23, 25-36, 38-44).  Trajectory b of this call is global
 * trajectory traj_offset + b: the stream is keyed by (seed, global trajectory,
 * step, component), so a batch sharded over ranks draws exactly the numbers the
 * unsharded batch would.  Any of x0 / dw / x_bdry may be NULL to skip it. */
int dpac_sample(const dpac_eqn_params* eq, int32_t sample_type, int32_t dtype,
                int64_t num_sample, int32_t num_steps, uint64_t seed,
                int64_t traj_offset, void* x0, void* dw, void* x_bdry,
                void* stream);

/* ---- fused rollout with the analytic control (the reference's `cheat` path)
 * Replaces Equation.propagate_naive / propagate_adaptive with cheat=True
 * (equation.py:46-71 / 73-106, control from u_true at :54-55 / :87-88).
 * dw == NULL draws the increments in-kernel from the same Philox stream as
 * dpac_sample(seed, traj_offset, sample_type).  u may be NULL (controls not kept).
 * If cost != NULL the same launch also accumulates the running cost in the order
 * cost_order and writes y[B] (Σ_t coef·w·dt·disc) and disc[B] (disc_N):
 * the reference's ActorModel loop (solver.py:213-219) / the drift part of
 * CriticModel (solver.py:166-175,187) under cheat_control. */
int dpac_rollout_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                     int64_t num_sample, int32_t num_steps, double total_time,
                     const void* x0, const void* dw, uint64_t seed,
                     int64_t traj_offset, int32_t sample_type, void* x,
                     void* dt, void* coef, void* u, int32_t cost_order,
                     void* y, void* disc, void* stream);

/* ---- one transition with an externally supplied control ----------------
 * One iteration of the propagate loop body with u_t = NN_control(x_t) computed
 * by the caller (equation.py:57-69 naive / :84-105 adaptive), fused with the
 * actor's running-cost and discount update (solver.py:218-219, order
 * DPAC_COST_ACTOR) or the critic's (solver.py:170-174,187, DPAC_COST_CRITIC).
 * flag_in / flag_out are the scheme's per-trajectory flags (naive: 1 = alive,
 * 0 = exited; adaptive: 2 inner, 1 boundary layer, 0 stopped); flag_out may alias
 * flag_in.  y_in/y_out and disc_in/disc_out may alias.  Any of dt, coef may be
 * NULL. */
int dpac_flag_init(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                   int64_t num_sample, int32_t num_steps, double total_time,
                   const void* x0, int32_t* flag, void* stream);

int dpac_step_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                  int64_t num_sample, int32_t num_steps, double total_time,
                  const void* x, const void* u, const void* dw_t,
                  const int32_t* flag_in, const void* disc_in,
                  const void* y_in, int32_t cost_order, void* x_out,
                  int32_t* flag_out, void* disc_out, void* y_out, void* dt,
                  void* coef, void* stream);

/* Vector-Jacobian product of dpac_step_fwd for back-propagation through the
 * rollout (what tf.GradientTape does for solver.py:95 through equation.py:84-105
 * and solver.py:213-219).  Inputs are the SAME x, u, dw_t, flag_in, disc_in
 * given to the forward call and the gradients of its outputs (g_x_out [B][d],
 * g_disc_out [B], g_y_out [B]; g_disc_out / g_y_out may be NULL = zero).  Writes
 * g_x [B][d], g_u [B][c], g_disc [B] (g_disc may be NULL).  The gradient of
 * y_in is g_y_out (identity) and is not written.  Flags, coef and exit tests
 * carry zero gradient, as TF's sign/floor/ceil do; the adaptive step size is
 * differentiated through max(dt, 1e-4·Δt) with TF's tie rule. */
int dpac_step_bwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                  int64_t num_sample, int32_t num_steps, double total_time,
                  const void* x, const void* u, const void* dw_t,
                  const int32_t* flag_in, const void* disc_in,
                  int32_t cost_order, const void* g_x_out,
                  const void* g_disc_out, const void* g_y_out, void* g_x,
                  void* g_u, void* g_disc, void* stream);

/* ---- TD target assembly ---------------------------------------------------
 * The critic's per-step loop over a finished trajectory (solver.py:166-187):
 *   y = Σ_t (w(x_t,u_t)·disc_t)·(coef_t·dt_t)
 *       − [TD1] Σ_t (Σ_j (σ(x_t,u_t)dw_t)_j·G_j(x_t) · disc_t)·(coef_t·√dt_t)
 *   disc_{t+1} = disc_t·exp(−γ·dt_t·coef_t),  disc_0 = 1
 * Writes y[B] and disc[B] (= disc_N, the factor of V(x_N) in delta, solver.py:189).
 * G may be NULL for TD2.  With td_type = DPAC_TD2 and cost_order = DPAC_COST_ACTOR
 * this is the actor's pathwise cost without the terminal value
 * (solver.py:213-219): dpac_actor_cost_fwd is that alias.
 * dw may be NULL → regenerated from the Philox stream (seed, traj_offset,
 * sample_type) exactly as dpac_sample / dpac_rollout_fwd drew it.
 * td_type = DPAC_TD1_GDOT: TD1 with G holding gdot [N][B], the per-step dots
 * Σ_j (σ(x_t,u_t)dw_t)_j·G_j(x_t) written by dpac_mlp_rows_fwd_td1; dw is not read.
 * y and disc are bitwise those of DPAC_TD1 on the same G. */
int dpac_td_assemble_fwd(const dpac_eqn_params* eq, int32_t td_type,
                         int32_t cost_order, int32_t dtype, int64_t num_sample,
                         int32_t num_steps, const void* x, const void* u,
                         const void* dw, uint64_t seed, int64_t traj_offset,
                         int32_t sample_type, const void* dt, const void* coef,
                         const void* G, void* y, void* disc, void* stream);

/* d y / d G for TD1: g_G[t][b][j] = −g_y[b]·disc_t·coef_t·√dt_t·(σ(x_t,u_t)dw_t)_j
 * (the tape gradient of solver.py:177-184 with respect to NN_value_grad's output). */
int dpac_td_assemble_bwd(const dpac_eqn_params* eq, int32_t dtype,
                         int64_t num_sample, int32_t num_steps, const void* x,
                         const void* u, const void* dw, uint64_t seed,
                         int64_t traj_offset, int32_t sample_type,
                         const void* dt, const void* coef, const void* g_y,
                         void* g_G, void* stream);

/* d y / d gdot for DPAC_TD1_GDOT: g_gdot[t][b] = −g_y[b]·disc_t·coef_t·√dt_t (reads
 * only dt, coef and g_y); dpac_mlp_rows_bwd_td1 turns it into d y / d G. */
int dpac_td_assemble_bwd_gdot(const dpac_eqn_params* eq, int32_t dtype,
                              int64_t num_sample, int32_t num_steps, const void* dt,
                              const void* coef, const void* g_y, void* g_gdot,
                              void* stream);

/* ActorModel pathwise cost without the terminal term (solver.py:213-219). */
int dpac_actor_cost_fwd(const dpac_eqn_params* eq, int32_t dtype,
                        int64_t num_sample, int32_t num_steps, const void* x,
                        const void* u, const void* dt, const void* coef,
                        void* y, void* disc, void* stream);

/* ---- rollout with the actor MLP as control, fused (one launch) ----------
 * equation.py:46-106 with u_t = NN_control(x_t) (solver.py:260-278) evaluated
 * inside the time loop on MFMA tiles.  The MLP is bn_0 -> (dense -> bn -> y+relu(y))
 * x n_hidden -> dense(+bias) -> bn_last [-> Eikonal head], with the weights of
 * `dpac_mlp` in the call's dtype:
 *   width[0] = dim, width[1..n_hidden] = hidden widths, width[n_hidden+1] = out
 *     (control_dim, or control_dim + 1 with ekn_head, solver.py:255-274);
 *   bn_scale[i] = gamma_i / sqrt(1 + 1e-6), bn_shift[i] = beta_i, [width[i]],
 *     i = 0..n_hidden+1 (BatchNormalization in inference form, solver.py:239-245);
 *   weight[i] = [width[i]][width[i+1]] row-major (x @ W), i = 0..n_hidden;
 *   bias = [out];
 *   weight_km[i] (optional, float only; NULL = not used): the k-major image of
 *     weight[i], [cols][K16] with K = width[i], cols = width[i+1], K16 =
 *     roundup(K, 16) and zeros for k >= K, read by the FORWARD entry points
 *     (dpac_rollout_nn_fwd, dpac_mlp_rows_fwd).  The backward entry points ignore
 *     it and take the images of weight_t in their own `weight_t_km` argument, so
 *     one struct serves both directions.  dpac_mlp_prepare writes both kinds.
 *     The wide layers then load 4 k per lane and instruction.
 *   weight_x3[i] / weight_t_x3[i] (optional, float only; NULL = not used): split-fp16
 *     images of weight[i] (forward entry points) and of weight_t[i] (backward entry
 *     points).  With every slot of a direction set, the float row kernels
 *     (dpac_mlp_rows_fwd[_td1] / dpac_mlp_rows_bwd[_td1]) and, for the actor-shape
 *     networks (d, out <= 32, hidden layers 193..208 wide), the fused rollout and its
 *     BPTT run the products on v_mfma_f32_16x16x32_f16 as hi*hi + hi*lo + lo*hi of the
 *     operands' splits a = hi + lo * 2^-12 (hi = fp16(a), lo = fp16((a - hi) * 2^12)),
 *     accumulated in f32: f32-accurate products at 5.3x fewer MFMA cycles (DESIGN.md
 *     §4.3).  Image layout (fragment-major: one 64-lane 16-byte load reads 1 KB of
 *     contiguous memory), with cols / K = width[i+1] / width[i] (forward) and
 *     width[i] / width[i+1] (backward): [ceil(cols / 16)][ceil(K / 32)][2][64][8] halves,
 *     element [t][c][p][l][e] = part p (0 hi, 1 lo) of the operand at column
 *     n = 16 t + (l % 16), k = 32 c + 8 (l / 16) + e, zero where n >= cols or k >= K.
 *     Operand range: an operand is split exactly only while |a| < 2^15 (hi and the 2^12-scaled
 *     lo both finite fp16 numbers); see `status`.
 *   status (optional, float split-fp16 only; NULL = unguarded): a device word, the range
 *     guard of the split-fp16 products.  Every split-fp16 kernel checks each operand it splits
 *     (activations, the backward chain's scaled gradients, the parameter gradients' A rows) and
 *     dpac_mlp_prepare checks the weight images it writes; an operand with !(|a| < 2^15) (so
 *     also inf / NaN) sets bit 0 (DPAC_X3_FELL_BACK).  Each split-fp16 launch is followed on
 *     the same stream by the exact-f32 kernel of the same operation, which runs only when the
 *     word is set (it then rewrites every output; a split-fp16 kernel that finds the word set
 *     at its start does no work), so no split-fp16 entry point returns a value the f32 kernels
 *     would not.  The word is sticky: once set, every later guarded launch with it runs on
 *     f32.  The caller clears it (zero) only while no guarded launch that uses it is in flight.
 *     The f32 fallback needs the f32 operands of the direction: weight and weight_km (forward
 *     entry points), weight_t and weight_t_km (backward entry points); without them the
 *     split-fp16 kernels are not used when a status word is given.
 *   guard_phase (with a status word; 0 when no status is given): which launches of a guarded
 *     call are made.  DPAC_GUARD_INLINE (0): the split-fp16 launch and then its guarded f32
 *     fallback, as above.  DPAC_GUARD_SPLIT_ONLY (1): the split-fp16 launch (and the launches
 *     that follow it unconditionally, e.g. the parameter gradients' reduce) but not the fallback.
 *     DPAC_GUARD_FALLBACK_ONLY (2): only the guarded fallback of the same call (and, for the
 *     parameter gradients, a guarded reduce after it): no-ops while the word is clear, and with
 *     the word set they rewrite every output from the call's inputs.  A caller may therefore
 *     make a chain of phase-1 calls and their phase-2 calls later, in the same order on one
 *     stream, as long as the inputs of every call stay unchanged until its phase-2 call (a
 *     split-fp16 launch that finds the word set does no work, so every phase-2 call after it
 *     recomputes the chain).  Calls whose launches do not use the split-fp16 kernels make their
 *     whole work in phase 1 and nothing in phase 2.
 * 1 <= n_hidden <= DPAC_MLP_MAX_HIDDEN, every width <= DPAC_MLP_MAX_WIDTH.
 * Outputs as dpac_rollout_fwd, with u [N][B][c] the control actually applied.
 * y/disc (optional, both or neither): the pathwise cost in `cost_order`.
 * Backward saves (optional, all or none): save_z [N][B][Σ_{i>=1} width[i]] the
 * pre-BN output of every dense layer (layer i at column offset
 * Σ_{1<=k<i} width[k]), save_flag [N][B] and save_disc [N][B] the flag and the
 * discount entering step t. */
#define DPAC_MLP_MAX_HIDDEN 4
#define DPAC_MLP_MAX_WIDTH 256
typedef struct dpac_mlp {
  int32_t n_hidden;
  int32_t ekn_head;
  int32_t width[DPAC_MLP_MAX_HIDDEN + 2];
  const void* bn_scale[DPAC_MLP_MAX_HIDDEN + 2];
  const void* bn_shift[DPAC_MLP_MAX_HIDDEN + 2];
  const void* weight[DPAC_MLP_MAX_HIDDEN + 1];
  const void* bias;
  const void* weight_km[DPAC_MLP_MAX_HIDDEN + 1];
  const void* weight_x3[DPAC_MLP_MAX_HIDDEN + 1];
  const void* weight_t_x3[DPAC_MLP_MAX_HIDDEN + 1];
  uint32_t* status; /* the split-fp16 range guard (above); NULL = unguarded */
  int32_t guard_phase; /* DPAC_GUARD_* (above); 0 = the split-fp16 launch and its fallback */
} dpac_mlp;
#define DPAC_X3_FELL_BACK 1u /* status bit: an operand left the split-fp16 range */
#define DPAC_GUARD_INLINE 0
#define DPAC_GUARD_SPLIT_ONLY 1
#define DPAC_GUARD_FALLBACK_ONLY 2

int dpac_rollout_nn_fwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                        int64_t num_sample, int32_t num_steps, double total_time,
                        const dpac_mlp* actor, const void* x0, const void* dw, void* x,
                        void* dt, void* coef, void* u, int32_t cost_order, void* y,
                        void* disc, void* save_z, int32_t* save_flag, void* save_disc,
                        void* stream);

/* The actor's BPTT through a dpac_rollout_nn_fwd rollout (what GradientTape does
 * for solver.py:92-97), as one launch.  Inputs: the forward's x, u, dw and its
 * saves; `weight_t[i]` = (weight[i] * bn_scale[i+1])^T, [width[i+1]][width[i]]
 * row-major, i = 0..n_hidden; weight_t_km (optional, float only, NULL = not used)
 * their k-major images, [width[i]][roundup(width[i+1], 16)] (dpac_mlp_prepare's
 * weight_t_km output); the upstream gradients g_xN [B][d] (dL/dx_N),
 * g_disc [B] (dL/d disc_N) and g_y [B] (dL/dy, the actor-order cost), each
 * optional (NULL = 0).  Output G [N][B][Σ_i width[i]]: block i (column offset
 * Σ_{k<i} width[k]) is dL/d(output of BN_i) at step t — for i = 0 the gradient
 * entering a_0 = BN_0(x_t); for i = n_hidden+1 the network output before the
 * Eikonal head.  The parameter gradients follow from G, the saved z and x by
 * products over the N*B rows.  g_x0 [B][d] (optional): dL/dx_0. */
int dpac_rollout_nn_bwd(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                        int64_t num_sample, int32_t num_steps, double total_time,
                        const dpac_mlp* actor, const void* const* weight_t,
                        const void* const* weight_t_km, const void* x,
                        const void* u, const void* dw, const void* save_z,
                        const int32_t* save_flag, const void* save_disc, const void* g_xN,
                        const void* g_disc, const void* g_y, void* G, void* g_x0, void* stream);

/* The same forward / BPTT pair with a sign-bit mask: the BPTT needs of the saved pre-BN
 * outputs z only whether each hidden BN output was positive (the activation factor
 * 1 + [y > 0]); dpac_rollout_nn_fwd_masked records those bits as the forward computes
 * them, save_mask [N][ceil(B / 16)][dpac_rollout_nn_mask_tile_bytes(actor)] bytes (per
 * 16-row tile: row r of hidden layer l, column c at bit r % 4 of byte
 * 13*64 l + 64 (c / 16) + 16 (r / 4) + c % 16, the MFMA accumulator's lane layout), and
 * dpac_rollout_nn_bwd_masked reads them instead of z (z is still needed by the parameter
 * gradients and the Eikonal head).  The mask is written only on the float 16-row fast path
 * (hidden layers 193..208 wide, d and out <= 32, k-major images, batches > 1024 or
 * DPAC_NN_TILE=16): *mask_written (host) reports whether it was; pass it to the backward only
 * then.  Results are bitwise those of the unmasked pair. */
int32_t dpac_rollout_nn_mask_tile_bytes(const dpac_mlp* actor);
/* The save_mask bytes dpac_rollout_nn_fwd_masked writes for this call
 * (N * ceil(B / 16) * dpac_rollout_nn_mask_tile_bytes), or 0 where it writes none (float64,
 * 4-row tiles at B <= 1024, no fast path): allocate the mask only when this is > 0.
 * -1 on a bad argument. */
int64_t dpac_rollout_nn_mask_bytes(const dpac_mlp* actor, int32_t dtype, int64_t num_sample,
                                   int32_t num_steps);
int dpac_rollout_nn_fwd_masked(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                               int64_t num_sample, int32_t num_steps, double total_time,
                               const dpac_mlp* actor, const void* x0, const void* dw, void* x,
                               void* dt, void* coef, void* u, int32_t cost_order, void* y,
                               void* disc, void* save_z, int32_t* save_flag, void* save_disc,
                               uint8_t* save_mask, int32_t* mask_written, void* stream);
int dpac_rollout_nn_bwd_masked(const dpac_eqn_params* eq, int32_t scheme, int32_t dtype,
                               int64_t num_sample, int32_t num_steps, double total_time,
                               const dpac_mlp* actor, const void* const* weight_t,
                               const void* const* weight_t_km, const void* x,
                               const void* u, const void* dw, const void* save_z,
                               const int32_t* save_flag, const void* save_disc,
                               const uint8_t* save_mask, const void* g_xN,
                               const void* g_disc, const void* g_y, void* G, void* g_x0,
                               void* stream);

/* ---- a dpac_mlp over independent rows (the critic's networks) -------------
 * Forward: out [rows][width[n_hidden+1]] = the network (bn_0 -> (dense -> bn ->
 * y+relu(y)) x n_hidden -> dense(+bias) -> bn_last, solver.py:260-271) applied to
 * every row of x (row stride ldx), on MFMA tiles.  ekn_head is ignored: `out` is
 * the network output before the Eikonal head (solver.py:272-274).  save_z
 * (optional) [rows][Σ_{i>=1} width[i]]: the pre-BN output of every dense layer,
 * as dpac_rollout_nn_fwd saves it.  Replaces DeepNN.call (solver.py:260-278) for
 * NN_value / NN_value_grad on the TD loop's states (solver.py:161-190).
 * Backward: given g_out [rows][width[n_hidden+1]] (dL/d out) and the forward's
 * save_z, writes G [rows][Σ_i width[i]], block i = dL/d(output of BN_i) — the
 * input of dpac_mlp_param_grads — and optionally g_x [rows][width[0]] = dL/dx.
 * weight_t[i] = (weight[i] * bn_scale[i+1])^T, [width[i+1]][width[i]] row-major;
 * weight_t_km (optional, float only) their k-major images, as for dpac_rollout_nn_bwd. */
int dpac_mlp_rows_fwd(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* x,
                      int64_t ldx, void* out, void* save_z, void* stream);
int dpac_mlp_rows_bwd(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* const* weight_t,
                      const void* const* weight_t_km, const void* save_z, const void* g_out, void* G,
                      void* g_x, void* stream);

/* ---- the G network with the TD1 dot fused ---------
 * solver.py:179-184 evaluates G = NN_value_grad(x_t) and immediately dots it with
 * σ(x_t,u_t)dw_t.  dpac_mlp_rows_fwd_td1 runs the network (width[0] = width[L+1]
 * = d) over the rollout rows x [rows][ldx] (rows = N·B, step-major, as x[:N]) and
 * writes only gdot[r] = Σ_j (σ(x_r,u_r)dw_r)_j·G_j(x_r) — G itself never reaches
 * HBM — plus the optional backward saves.  u [rows][control_dim] is read only for
 * LQR_var (state-dependent σ, equation.py:302); dw [rows][d].  gdot is bitwise the
 * dot dpac_td_assemble_fwd(DPAC_TD1) forms from the same G.
 * dpac_mlp_rows_bwd_td1 is dpac_mlp_rows_bwd with dL/d out = g_gdot[r]·(σ dw)_r,
 * formed in its prologue (bitwise dpac_td_assemble_bwd's d y / d G times the same
 * upstream gradient). */
int dpac_mlp_rows_fwd_td1(const dpac_eqn_params* eq, int32_t dtype, int64_t rows,
                          const dpac_mlp* net, const void* x, int64_t ldx, const void* u,
                          const void* dw, void* gdot, void* save_z, void* stream);
int dpac_mlp_rows_bwd_td1(const dpac_eqn_params* eq, int32_t dtype, int64_t rows,
                          const dpac_mlp* net, const void* const* weight_t,
                          const void* const* weight_t_km, const void* save_z, const void* x,
                          int64_t ldx, const void* u, const void* dw, const void* g_gdot,
                          void* G, void* g_x, void* stream);

/* The row kernels with a sign-bit mask (round 5, ABI 7).  The backward chain needs of the
 * forward's saved z only whether each hidden BN output was positive (the activation factor
 * 1 + [y > 0], solver.py:269); the split-fp16 forward records those bits as it computes them,
 * save_mask = dpac_mlp_rows_mask_bytes bytes of 32-bit words: per hidden layer h = 1..n_hidden
 * and 64-row block b (nblk = ceil(rows / 64) of them), 512 words; word
 * ((h - 1) nblk + b) * 512 + 64 w + 16 q + r (w < 8, q < 4, r < 16) holds at bit 4 (2 t + j) + e
 * (t, e < 4; j < 2) whether BN_h's output of row 64 b + 16 t + r, feature 16 (w + 8 j) + 4 q + e,
 * is > 0 (0 past width[h] and past the last row) — the split-fp16 kernels' accumulator layout,
 * so each lane writes and reads one word per layer.  The masked backward reads them instead of z (z is
 * still required: the parameter gradients and the exact-f32 fallback read it).  The mask is
 * written only by the float split-fp16 forward (every weight_x3 given) and only with save_z:
 * *mask_written (host, optional) reports whether it was; pass it to the backward only then.
 * Results are bitwise those of the unmasked entry points (tests/test_gpu_mlp.py).
 * dpac_mlp_rows_mask_bytes: the bytes for `rows` rows, 0 where no mask is written (float64,
 * no split-fp16 images), -1 on a bad argument. */
int64_t dpac_mlp_rows_mask_bytes(const dpac_mlp* net, int32_t dtype, int64_t rows);
int dpac_mlp_rows_fwd_masked(int32_t dtype, int64_t rows, const dpac_mlp* net, const void* x,
                             int64_t ldx, void* out, void* save_z, uint8_t* save_mask,
                             int32_t* mask_written, void* stream);
int dpac_mlp_rows_bwd_masked(int32_t dtype, int64_t rows, const dpac_mlp* net,
                             const void* const* weight_t, const void* const* weight_t_km,
                             const void* save_z, const uint8_t* save_mask, const void* g_out,
                             void* G, void* g_x, void* stream);
int dpac_mlp_rows_fwd_td1_masked(const dpac_eqn_params* eq, int32_t dtype, int64_t rows,
                                 const dpac_mlp* net, const void* x, int64_t ldx, const void* u,
                                 const void* dw, void* gdot, void* save_z, uint8_t* save_mask,
                                 int32_t* mask_written, void* stream);
int dpac_mlp_rows_bwd_td1_masked(const dpac_eqn_params* eq, int32_t dtype, int64_t rows,
                                 const dpac_mlp* net, const void* const* weight_t,
                                 const void* const* weight_t_km, const void* save_z,
                                 const uint8_t* save_mask, const void* x, int64_t ldx,
                                 const void* u, const void* dw, const void* g_gdot, void* G,
                                 void* g_x, void* stream);

/* ---- parameter gradients of a dpac_mlp over independent rows -------------
 * What GradientTape returns for DeepNN's trainable variables (solver.py:88,95
 * through solver.py:260-271), given the backward chain's G [rows][Σ_i width[i]]
 * (as written by dpac_rollout_nn_bwd or dpac_mlp_rows_bwd) and the forward's
 * save_z [rows][Σ_{i>=1} width[i]]; x [rows] with row stride ldx is the network
 * input (ldx <= Σ_i width[i]).  With s_i = bn_scale[i], a_0 = bn_shift[0] + x*s_0 and
 * a_i = y_i + relu(y_i), y_i = bn_shift[i] + z_i*s_i:
 *   dW_i = Σ_r a_i^T (G_{i+1} ⊙ s_{i+1}),  dbeta_i = Σ_r G_i,
 *   dgamma_i = gamma_scale · Σ_r G_i ⊙ zin_i  (zin_0 = x, zin_{L+1} = z_{L+1} + bias),
 *   dbias = s_{L+1} ⊙ dbeta_{L+1};
 * gamma_scale = 1/sqrt(1 + 1e-6) (d bn_scale / d gamma).  grads is one flat
 * buffer in DeepNN's variable order: gamma_0..gamma_{L+1}, beta_0..beta_{L+1},
 * W_0..W_L (row-major), bias.  The sums over rows run chunk-wise into
 * `workspace` (size from dpac_mlp_param_grads_workspace, -1 on a bad argument)
 * and are combined in a fixed order: deterministic.  weight[] of `net` is not
 * read (may be NULL).  The reference has no such entry point: this replaces the
 * TF-internal gradient ops of the Dense / BatchNormalization layers. */
int64_t dpac_mlp_param_grads_workspace(int32_t dtype, int64_t rows, const dpac_mlp* net);
int dpac_mlp_param_grads(int32_t dtype, int64_t rows, const dpac_mlp* net, double gamma_scale,
                         const void* x, int64_t ldx, const void* save_z, const void* G,
                         void* workspace, int64_t workspace_bytes, void* grads, void* stream);

/* ---- derived MLP operands --------------------------------------------
 * The tensors the MLP kernels read, formed from a DeepNN's raw variables in one
 * launch: with net->bn_scale[i] pointing at the raw BN gamma_i (NOT the scale)
 * and net->weight[i] at W_i, writes scales = [s_0 | s_1 | ... | s_{L+1}],
 * s_i = gamma_scale * gamma_i (the inference BatchNormalization scale of
 * solver.py:246-258, gamma_scale = 1/sqrt(1 + 1e-6)), and, if weight_t is not
 * NULL, weight_t = [wt_0 | ... | wt_L], wt_i = (W_i ⊙ s_{i+1})^T [width[i+1]][width[i]]
 * row-major (the weight_t operand of dpac_mlp_rows_bwd / dpac_rollout_nn_bwd).
 * Optional k-major images (see dpac_mlp.weight_km), concatenated over i:
 * weight_km = [W_i^T padded: [width[i+1]][roundup(width[i], 16)]] (forward) and
 * weight_t_km = [(W_i ⊙ s_{i+1}) padded: [width[i]][roundup(width[i+1], 16)]]
 * (backward).  Optional split-fp16 images (float only; see dpac_mlp.weight_x3), each
 * concatenated over i in dpac_mlp.weight_x3's layout: weight_x3 = [W_i: ceil(width[i+1]/16)
 * x ceil(width[i]/32) x 1024 halves] and weight_t_x3 = [(W_i ⊙ s_{i+1})^T: ceil(width[i]/16)
 * x ceil(width[i+1]/32) x 1024 halves].
 * bn_shift, bias, net->weight_km and the x3 slots of net are not read.  With net->status set, a
 * split-fp16 image value outside the split range (|v| >= 2^15, inf, NaN) sets DPAC_X3_FELL_BACK
 * in it. */
int dpac_mlp_prepare(int32_t dtype, const dpac_mlp* net, double gamma_scale, void* scales,
                     void* weight_t, void* weight_km, void* weight_t_km, void* weight_x3,
                     void* weight_t_x3, void* stream);

/* ---- optimizer step --------------------------------------------------
 * One step of TF-form Adam (the reference's tf.keras Adam, solver.py:16-21;
 * ResourceApplyAdam) over n_tensors parameter tensors of `dtype`, one launch:
 *   m += (g - m)(1 - beta_1);  v += (g*g - v)(1 - beta_2);
 *   var -= (m*alpha) / (sqrt(v) + epsilon),
 * with alpha = lr*sqrt(1 - beta_2^t)/(1 - beta_1^t) formed by the caller.  Each
 * operation rounds separately, in this order.  Arrays hold n_tensors device
 * pointers / element counts; var, m, v are updated in place. */
int dpac_adam_apply(int32_t dtype, int32_t n_tensors, const int64_t* numel, void* const* var,
                    const void* const* grad, void* const* m, void* const* v, double alpha,
                    double beta_1, double beta_2, double epsilon, void* stream);

/* ---- the critic loss's gradient at V's outputs (one launch) -------------
 * loss_critic (solver.py:73-78) differentiated at V = NN_value([x_0; x_N; x_bdry]) (3B):
 * delta = V0 − y − VN·disc, delta_b = Vb − z_bdry (solver.py:189-190), h'(z) = 2z for
 * |z| < delta_clip else 2·delta_clip·sign(z); g = h'(delta)·scale, g_b = h'(delta_b)·scale;
 * writes g_out = [g; −g·disc; g_b] (3B) and neg_g = −g (B, dL/dy for the TD backward).
 * Rounds as the same tensor expressions do. */
int dpac_critic_loss_grad(int32_t dtype, int64_t num_sample, const void* V, const void* y,
                          const void* disc, const void* z_bdry, double scale, double delta_clip,
                          void* g_out, void* neg_g, void* stream);

/* ---- device equation coefficients (for parity tests and metrics) -------
 * Evaluates one Equation method row-wise on x [B][d] (and u [B][c] where the
 * method takes a control): drift/sigma/w/Z/V_true/u_true/V_grad_true/b_tf
 * (equation.py:108-311).  `what` is DPAC_EVAL_*. */
int dpac_equation_eval(const dpac_eqn_params* eq, int32_t what, int32_t dtype,
                       int64_t num_sample, const void* x, const void* u,
                       void* out, void* stream);

#ifdef __cplusplus
} /* extern "C" */
#endif

#endif /* DPAC_H_ */
