// Kernel instantiations for the LQR equation family (equation.py, class LQR) for one
// dtype (-DDPAC_TU_DOUBLE=0 float / 1 double) and the state dimensions in DPAC_DIMS
// (the Makefile builds one object per dimension); they register with dpac_abi.hip's table.
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqLQRFor = EqLQR<T, D, eqn_lanes(DPAC_EQN_LQR, D)>;
namespace {
const Registrar<EqLQRFor, std::conditional_t<DPAC_TU_DOUBLE, double, float>, DPAC_DIMS> reg(DPAC_EQN_LQR);
}  // namespace
}  // namespace dpac

#if DPAC_NN_TRACE && DPAC_TU_TRACE
// Timing builds only (tools/build_variant.sh): copy the NN kernels' clock table
// (dpac_rollout_nn.h) of this translation unit to the host.
extern "C" int dpac_debug_trace(void* host, int64_t bytes) {
  const int64_t n = bytes < (int64_t)sizeof(dpac::g_nn_trace) ? bytes : (int64_t)sizeof(dpac::g_nn_trace);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(dpac::g_nn_trace), (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif
