/*
 * abi_sanitize.c — host-side AddressSanitizer / UndefinedBehaviorSanitizer run of
 * libdpac's C-ABI validation layer (csrc/dpac_abi.hip), built by `make sanitize`
 * against a host-instrumented libdpac (device code unchanged).  Every entry point of
 * include/dpac.h is called with malformed arguments (NULL structs and buffers, bad
 * enums, zero / negative / overflowing sizes, inconsistent optional outputs); each
 * call must return DPAC_EINVAL or DPAC_EUNSUP with a message, before any device work.
 * Runs on a machine without a GPU (no call reaches a launch).  Exit 0 = all checks
 * passed and the sanitizers reported nothing (they abort the process otherwise).
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "dpac.h"

static int fails = 0, checks = 0;

static void expect_err(int rc, const char* what) {
  ++checks;
  const char* msg = dpac_last_error();
  if (!(rc == DPAC_EINVAL || rc == DPAC_EUNSUP) || !msg || !msg[0]) {
    printf("FAIL %-48s rc=%d msg='%s'\n", what, rc, msg ? msg : "(null)");
    ++fails;
  } else {
    printf("ok   %-48s rc=%d %s\n", what, rc, msg);
  }
}

static dpac_eqn_params lqr(int dim) {
  dpac_eqn_params e;
  memset(&e, 0, sizeof e);
  e.eqn = DPAC_EQN_LQR;
  e.dim = dim;
  e.control_dim = dim;
  e.gamma = 1.0;
  e.R = 1.0;
  e.sigma_up = 1.4142135623730951;
  e.p = e.q = e.beta = 1.0;
  e.k = 0.6180339887;
  return e;
}

int main(void) {
  /* fake device pointers: never dereferenced, every call below fails validation first */
  static char buf[64];
  void* P = buf;
  dpac_eqn_params e = lqr(20), bad;
  if (dpac_abi_version() != DPAC_ABI_VERSION) {
    printf("FAIL abi version\n");
    return 1;
  }
  if (dpac_supported(NULL) != 0) ++fails;

  /* equation parameters */
  expect_err(dpac_rollout_fwd(NULL, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: NULL eqn");
  bad = e; bad.reserved = 7;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: reserved != 0");
  bad = e; bad.eqn = 99;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: unknown equation");
  bad = e; bad.dim = 7; bad.control_dim = 7;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: dim without kernels");
  bad = e; bad.dim = INT32_MAX; bad.control_dim = INT32_MAX;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: dim INT32_MAX");
  bad = e; bad.control_dim = 3;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: control_dim mismatch");
  bad = e; bad.R = -1.0;
  expect_err(dpac_rollout_fwd(&bad, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: R < 0");
  /* sizes, enums, buffers */
  expect_err(dpac_rollout_fwd(&e, 5, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL, DPAC_COST_CRITIC, NULL,
                              NULL, NULL), "rollout: bad scheme");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, 9, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: bad dtype");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 0, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: B = 0");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, -5, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: B < 0");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, INT64_MAX, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: B = INT64_MAX");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F64, 1 << 30, INT32_MAX, 0.2, P, P, 1, 0, 0, P, P, P,
                              NULL, DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: B*N*d bytes overflow");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 0, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: N = 0");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, -0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: T < 0");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, 0.2, NULL, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: x0 NULL");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, P, NULL, NULL), "rollout: y without disc");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, 0.2, P, P, 1, 0, 0, P, P, P, NULL, 7, P, P,
                              NULL), "rollout: bad cost_order");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, 0.2, P, NULL, 1, -3, 0, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: traj_offset < 0");
  expect_err(dpac_rollout_fwd(&e, DPAC_SCHEME_NAIVE, DPAC_F32, 16, 10, 0.2, P, NULL, 1, 0, 12, P, P, P, NULL,
                              DPAC_COST_CRITIC, NULL, NULL, NULL), "rollout: bad sample_type");

  expect_err(dpac_sample(NULL, DPAC_SAMPLE_NORMAL, DPAC_F32, 16, 10, 1, 0, P, P, P, NULL), "sample: NULL eqn");
  expect_err(dpac_sample(&e, DPAC_SAMPLE_NORMAL, 3, 16, 10, 1, 0, P, P, P, NULL), "sample: bad dtype");
  expect_err(dpac_sample(&e, DPAC_SAMPLE_NORMAL, DPAC_F32, 0, 10, 1, 0, P, P, P, NULL), "sample: B = 0");
  expect_err(dpac_sample(&e, DPAC_SAMPLE_NORMAL, DPAC_F32, 16, 0, 1, 0, P, P, P, NULL), "sample: N = 0 with dw");
  expect_err(dpac_sample(&e, DPAC_SAMPLE_NORMAL, DPAC_F32, 16, 10, 1, -1, P, P, P, NULL), "sample: offset < 0");
  expect_err(dpac_sample(&e, 42, DPAC_F32, 16, 10, 1, 0, P, P, P, NULL), "sample: bad sample_type");

  expect_err(dpac_flag_init(&e, 9, DPAC_F32, 16, 10, 0.2, P, (int32_t*)P, NULL), "flag_init: bad scheme");
  expect_err(dpac_flag_init(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, NULL, (int32_t*)P, NULL),
             "flag_init: x0 NULL");
  expect_err(dpac_step_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, NULL, P, (int32_t*)P, P, P,
                           DPAC_COST_ACTOR, P, (int32_t*)P, P, P, NULL, NULL, NULL), "step_fwd: u NULL");
  expect_err(dpac_step_bwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, P, P, P, (int32_t*)P, P,
                           DPAC_COST_ACTOR, NULL, NULL, NULL, P, P, NULL, NULL), "step_bwd: g_x_out NULL");
  expect_err(dpac_td_assemble_fwd(&e, 3, DPAC_COST_CRITIC, DPAC_F32, 16, 10, P, P, P, 1, 0, 0, P, P, P, P, P,
                                  NULL), "td_fwd: bad td_type");
  expect_err(dpac_td_assemble_fwd(&e, DPAC_TD1, DPAC_COST_CRITIC, DPAC_F32, 16, 10, P, P, P, 1, 0, 0, P, P, NULL,
                                  P, P, NULL), "td_fwd: TD1 without G");
  expect_err(dpac_td_assemble_bwd(&e, DPAC_F32, 16, 10, P, P, P, 1, 0, 0, P, P, P, NULL, NULL),
             "td_bwd: g_G NULL");
  expect_err(dpac_actor_cost_fwd(&e, DPAC_F32, -1, 10, P, P, P, P, P, P, NULL), "actor_cost: B < 0");
  expect_err(dpac_equation_eval(&e, 99, DPAC_F32, 16, P, P, P, NULL), "eval: bad quantity");
  expect_err(dpac_equation_eval(&e, DPAC_EVAL_DRIFT, DPAC_F32, 16, P, NULL, P, NULL), "eval: drift without u");

  /* MLP entry points */
  dpac_mlp m;
  memset(&m, 0, sizeof m);
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, NULL, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: NULL mlp");
  m.n_hidden = 9;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: n_hidden 9");
  m.n_hidden = 2;
  m.width[0] = 20; m.width[1] = 300; m.width[2] = 64; m.width[3] = 20;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: width 300");
  m.width[1] = 64;
  for (int i = 0; i < 4; ++i) m.bn_scale[i] = m.bn_shift[i] = P;
  for (int i = 0; i < 3; ++i) m.weight[i] = P;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: bias NULL");
  m.bias = P;
  m.ekn_head = 1;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: ekn head on LQR");
  m.ekn_head = 0;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, P, NULL, NULL, NULL), "rollout_nn: partial saves");
  m.width[0] = 19;
  expect_err(dpac_rollout_nn_fwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, P, P, P, P, P, P,
                                 DPAC_COST_ACTOR, NULL, NULL, NULL, NULL, NULL, NULL), "rollout_nn: width[0] != dim");
  m.width[0] = 20;
  const void* wt3[3] = {P, NULL, P};
  expect_err(dpac_rollout_nn_bwd(&e, DPAC_SCHEME_ADAPTIVE, DPAC_F32, 16, 10, 0.2, &m, wt3, NULL, P, P, P, P,
                                 (int32_t*)P, P, NULL, NULL, P, P, NULL, NULL), "rollout_nn_bwd: weight_t[1] NULL");
  expect_err(dpac_mlp_rows_fwd(DPAC_F32, 0, &m, P, 20, P, NULL, NULL), "rows_fwd: rows = 0");
  expect_err(dpac_mlp_rows_fwd(DPAC_F32, 16, &m, P, 5, P, NULL, NULL), "rows_fwd: ldx < width[0]");
  expect_err(dpac_mlp_rows_bwd(7, 16, &m, wt3, NULL, P, P, P, NULL, NULL), "rows_bwd: bad dtype");
  expect_err(dpac_mlp_rows_bwd(DPAC_F32, 16, &m, wt3, NULL, P, P, P, NULL, NULL), "rows_bwd: weight_t[1] NULL");
  ++checks;
  if (dpac_mlp_param_grads_workspace(DPAC_F32, -1, &m) != -1) {
    printf("FAIL param_grads_workspace: rows < 0 must give -1\n");
    ++fails;
  }
  expect_err(dpac_mlp_param_grads(DPAC_F32, 16, &m, 1.0, P, 20, P, P, P, 0, P, NULL), "param_grads: workspace 0 B");
  expect_err(dpac_mlp_param_grads(DPAC_F32, 16, NULL, 1.0, P, 20, P, P, P, 1 << 20, P, NULL), "param_grads: NULL mlp");
  expect_err(dpac_mlp_prepare(DPAC_F32, NULL, 1.0, P, P, NULL, NULL, NULL, NULL, NULL), "prepare: NULL mlp");
  int64_t numel[2] = {10, -4};
  void* vars[2] = {P, P};
  const void* grads[2] = {P, P};
  expect_err(dpac_adam_apply(DPAC_F32, 2, numel, vars, grads, vars, vars, 1e-3, 0.9, 0.999, 1e-8, NULL),
             "adam: negative numel");
  expect_err(dpac_adam_apply(DPAC_F32, -1, numel, vars, grads, vars, vars, 1e-3, 0.9, 0.999, 1e-8, NULL),
             "adam: n_tensors < 0");
  expect_err(dpac_adam_apply(DPAC_F32, 2, NULL, vars, grads, vars, vars, 1e-3, 0.9, 0.999, 1e-8, NULL),
             "adam: numel NULL");

  printf("%d checks, %d failed\n", checks, fails);
  return fails ? 1 : 0;
}
