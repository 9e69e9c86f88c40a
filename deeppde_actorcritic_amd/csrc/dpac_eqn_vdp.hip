// Kernel instantiations for the VDP equation family (equation.py, class VDP) for one
// dtype (-DDPAC_TU_DOUBLE=0 float / 1 double) and the state dimensions in DPAC_DIMS_EVEN
// (the Makefile builds one object per dimension); they register with dpac_abi.hip's table.
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqVDPFor = EqVDP<T, D, eqn_lanes(DPAC_EQN_VDP, D)>;
namespace {
const Registrar<EqVDPFor, std::conditional_t<DPAC_TU_DOUBLE, double, float>, DPAC_DIMS_EVEN> reg(DPAC_EQN_VDP);
}  // namespace
}  // namespace dpac
