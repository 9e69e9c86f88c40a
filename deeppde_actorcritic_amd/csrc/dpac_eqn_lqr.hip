// Kernel instantiations for the LQR equation family (equation.py, class LQR),
// compiled once per dtype: -DDPAC_TU_DOUBLE=0 (float) / 1 (double).
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqLQRFor = EqLQR<T, D, eqn_lanes(DPAC_EQN_LQR, D)>;
using lqrDims = DimList<EqLQRFor, DPAC_DIMS>;
#if DPAC_TU_DOUBLE
int dispatch_lqr_f64(const OpArgs& a) { return lqrDims::dispatch<double>(a); }
#else
int dispatch_lqr_f32(const OpArgs& a) { return lqrDims::dispatch<float>(a); }
bool has_dim_lqr(int d) { return lqrDims::has(d); }
#endif
}  // namespace dpac

#if DPAC_NN_TRACE && !DPAC_TU_DOUBLE
// Timing builds only: copy the NN kernels' clock table (dpac_rollout_nn.h) to the host.
extern "C" int dpac_debug_trace(void* host, int64_t bytes) {
  const int64_t n = bytes < (int64_t)sizeof(dpac::g_nn_trace) ? bytes : (int64_t)sizeof(dpac::g_nn_trace);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(dpac::g_nn_trace), (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif
