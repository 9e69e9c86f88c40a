// Kernel instantiations for the LQR_var equation family (equation.py, class LQR_var) for one
// dtype (-DDPAC_TU_DOUBLE=0 float / 1 double) and the state dimensions in DPAC_DIMS
// (the Makefile builds one object per dimension); they register with dpac_abi.hip's table.
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqLQRVarFor = EqLQRVar<T, D, eqn_lanes(DPAC_EQN_LQR_VAR, D)>;
namespace {
const Registrar<EqLQRVarFor, std::conditional_t<DPAC_TU_DOUBLE, double, float>, DPAC_DIMS> reg(DPAC_EQN_LQR_VAR);
}  // namespace
}  // namespace dpac
