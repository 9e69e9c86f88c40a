// Kernel instantiations for the LQR_var equation family (equation.py, class LQR_var),
// compiled once per dtype: -DDPAC_TU_DOUBLE=0 (float) / 1 (double).
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqLQRVarFor = EqLQRVar<T, D, eqn_lanes(DPAC_EQN_LQR_VAR, D)>;
using lqrvarDims = DimList<EqLQRVarFor, DPAC_DIMS>;
#if DPAC_TU_DOUBLE
int dispatch_lqrvar_f64(const OpArgs& a) { return lqrvarDims::dispatch<double>(a); }
#else
int dispatch_lqrvar_f32(const OpArgs& a) { return lqrvarDims::dispatch<float>(a); }
bool has_dim_lqrvar(int d) { return lqrvarDims::has(d); }
#endif
}  // namespace dpac
