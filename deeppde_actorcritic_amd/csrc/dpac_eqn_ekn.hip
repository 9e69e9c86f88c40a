// Kernel instantiations for the ekn equation family (equation.py, class ekn),
// compiled once per dtype: -DDPAC_TU_DOUBLE=0 (float) / 1 (double).
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqEKNFor = EqEKN<T, D, eqn_lanes(DPAC_EQN_EKN, D)>;
using eknDims = DimList<EqEKNFor, DPAC_DIMS>;
#if DPAC_TU_DOUBLE
int dispatch_ekn_f64(const OpArgs& a) { return eknDims::dispatch<double>(a); }
#else
int dispatch_ekn_f32(const OpArgs& a) { return eknDims::dispatch<float>(a); }
bool has_dim_ekn(int d) { return eknDims::has(d); }
#endif
}  // namespace dpac
