// Kernel instantiations for the VDP equation family (equation.py, class VDP),
// compiled once per dtype: -DDPAC_TU_DOUBLE=0 (float) / 1 (double).
#include "dpac_kernels.h"

namespace dpac {
template <typename T, int D>
using EqVDPFor = EqVDP<T, D, eqn_lanes(DPAC_EQN_VDP, D)>;
using vdpDims = DimList<EqVDPFor, DPAC_DIMS_EVEN>;
#if DPAC_TU_DOUBLE
int dispatch_vdp_f64(const OpArgs& a) { return vdpDims::dispatch<double>(a); }
#else
int dispatch_vdp_f32(const OpArgs& a) { return vdpDims::dispatch<float>(a); }
bool has_dim_vdp(int d) { return vdpDims::has(d); }
#endif
}  // namespace dpac
