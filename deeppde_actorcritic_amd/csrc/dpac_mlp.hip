// dpac_mlp.hip — host side of the equation-independent MLP kernels (parameter
// gradients over independent rows, dpac_mlp_grad.h), compiled once for both
// dtypes.  Argument checking and error strings live in dpac_abi.hip.
#include <algorithm>

#include <cstdlib>

#include "dpac_mlp_grad.h"
#include "dpac_mlp_grad_x3.h"
#include "dpac_mlp_rows.h"
#include "dpac_mlp_x3.h"

namespace dpac {

namespace {

template <typename T>
PgArgs<T> pg_args(const dpac_mlp& net, int64_t rows, const void* x, int64_t ldx, const void* z,
                  const void* G) {
  PgArgs<T> a{};
  const int L = net.n_hidden;
  a.rows = rows;
  a.L = L;
  int zt = 0, gt = 0, sw = 0;
  for (int i = 0; i <= L + 1; ++i) {
    a.width[i] = net.width[i];
    a.scale[i] = (const T*)net.bn_scale[i];
    a.shift[i] = (const T*)net.bn_shift[i];
    a.zoff[i] = i == 0 ? 0 : zt;
    if (i > 0) zt += net.width[i];
    a.goff[i] = gt;
    gt += net.width[i];
    sw += net.width[i];
  }
  a.bias = (const T*)net.bias;
  a.x = (const T*)x;
  a.z = (const T*)z;
  a.G = (const T*)G;
  a.ldx = (int)ldx;
  a.ztot = zt;
  a.gtot = gt;
  int64_t o = 0;
  for (int i = 0; i <= L + 1; ++i) { a.off_gamma[i] = o; o += net.width[i]; }
  for (int i = 0; i <= L + 1; ++i) { a.off_beta[i] = o; o += net.width[i]; }
  for (int i = 0; i <= L; ++i) { a.off_W[i] = o; o += (int64_t)net.width[i] * net.width[i + 1]; }
  a.ptot = o;
  (void)sw;
  return a;
}

#ifndef DPAC_PG_CHUNKS
#define DPAC_PG_CHUNKS 256  // 2 workgroups per CU on the wide layers (measured 819 -> 681 us at 204800 rows)
#endif
#ifndef DPAC_PG_MIN_ROWS
#define DPAC_PG_MIN_ROWS 256  // rows per chunk at least: small row counts (the critic's V over 3B rows)
#endif                        // would otherwise write and re-read ~256 near-empty partials
// DPAC_PG_MIN_ROWS in the environment overrides the floor (timing comparisons; read per call, so
// a process must keep one value between sizing its workspace and launching)
inline int64_t pg_min_rows() {
  const char* e = getenv("DPAC_PG_MIN_ROWS");
  const long long v = e ? atoll(e) : 0;
  return v >= 16 ? (int64_t)v : (int64_t)DPAC_PG_MIN_ROWS;
}

template <typename T>
int64_t pg_chunk_rows(int64_t rows, int64_t max_ld) {
  // DPAC_PG_CHUNKS chunks of at least DPAC_PG_MIN_ROWS rows: the wide layers' two column
  // groups give 2 workgroups per CU, the narrow ones one, and a partial buffer the reduce
  // reads in ~25 us.  A chunk's rows are addressed through 32-bit buffer descriptors: keep
  // them below 2 GiB.
  constexpr int SR = PgCfg<T>::SR;
  int64_t per = (rows + DPAC_PG_CHUNKS - 1) / DPAC_PG_CHUNKS;
  per = std::max<int64_t>(per, pg_min_rows());
  const int64_t cap = (((int64_t)1 << 31) - 1) / (max_ld * (int64_t)sizeof(T)) / SR * SR;
  per = (per + SR - 1) / SR * SR;
  return std::max<int64_t>(std::min(per, cap), SR);
}

template <typename T>
int64_t max_ld(const PgArgs<T>& a) {
  return std::max<int64_t>(std::max(a.ldx, a.ztot), a.gtot);
}

template <typename T>
int64_t ws_bytes(int64_t rows, const dpac_mlp& net) {
  const PgArgs<T> a = pg_args<T>(net, rows, nullptr, net.width[0], nullptr, nullptr);
  const int64_t per = pg_chunk_rows<T>(rows, max_ld(a));
  const int64_t nch = (rows + per - 1) / per;
  return nch * a.ptot * (int64_t)sizeof(T);
}

#ifndef DPAC_PG_FORK
#define DPAC_PG_FORK 0  // narrow layers' launches on a forked stream beside the wide ones
#endif
// The fork: a per-device auxiliary stream and two events, created on first use (outside
// any capture: dpac_mlp_param_grads_workspace, which every caller runs first, creates
// them).  Inside a stream capture the event record / wait pair becomes graph edges, so
// the narrow layers are a parallel branch of the captured graph.
struct PgFork {
  hipStream_t aux = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
};
PgFork* pg_fork() {
  static PgFork f[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  PgFork& r = f[dev];
  if (!r.aux) {
    if (hipStreamCreateWithFlags(&r.aux, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&r.fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&r.join, hipEventDisableTiming) != hipSuccess) {
      r.aux = nullptr;
      return nullptr;
    }
  }
  return &r;
}

// one layer of the f32 / f64 kernel (k_param_grads): the wave grid and the tile counts are
// template bins (wide layers: 1 x 4 waves, 2 column tiles each (f64: 1), row tiles
// 1/2/4/8/13/16; layers of <= 32 outputs: 4 x 1 waves over the row tiles)
template <typename T>
int launch_f32_layer(const PgArgs<T>& a, int l, int64_t nch, hipStream_t s) {
  const int K = a.width[l], H = a.width[l + 1];
  const int nti = (K + 15) / 16;
  if (H <= 32) {
    const int ntj = (H + 15) / 16, nt4 = (nti + 3) / 4;
    const dim3 grid((unsigned)nch, 1u);
#define DPAC_PGN(NI, NJ) hipLaunchKernelGGL((k_param_grads<T, NI, NJ, 4>), grid, dim3(kPgThreads), 0, s, a, l)
#define DPAC_PGN_J(NI) if (ntj == 1) DPAC_PGN(NI, 1); else DPAC_PGN(NI, 2);
    if (nt4 <= 1) { DPAC_PGN_J(1) }
    else if (nt4 <= 2) { DPAC_PGN_J(2) }
    else if (nt4 <= 3) { DPAC_PGN_J(3) }
    else { DPAC_PGN_J(4) }
#undef DPAC_PGN_J
#undef DPAC_PGN
  } else {
    constexpr int NJ = sizeof(T) == 4 ? 2 : 1;
    constexpr int CW = 16 * NJ * 4;
    const dim3 grid((unsigned)nch, (unsigned)((H + CW - 1) / CW));
#define DPAC_PG(NI) hipLaunchKernelGGL((k_param_grads<T, NI, NJ, 1>), grid, dim3(kPgThreads), 0, s, a, l)
    if (nti <= 1) DPAC_PG(1);
    else if (nti <= 2) DPAC_PG(2);
    else if (nti <= 4) DPAC_PG(4);
    else if (nti <= 8) DPAC_PG(8);
    else if (nti <= 13) DPAC_PG(13);
    else DPAC_PG(16);
#undef DPAC_PG
  }
  return (int)hipGetLastError();
}

// Whether a float network's parameter gradients run on split-fp16 MFMA (dpac_mlp_grad_x3.h):
// the caller gave the split-fp16 weight images (it asked for split-fp16 products), every
// width fits the staging map, and DPAC_PG_X3=0 does not force the f32 kernel (tests).
inline bool pg_x3(const dpac_mlp& net) {
  const char* e = getenv("DPAC_PG_X3");  // read per launch
  if (e && e[0] == '0') return false;
  for (int i = 0; i <= net.n_hidden; ++i)
    if (!net.weight_x3[i]) return false;
  for (int i = 0; i <= net.n_hidden + 1; ++i)
    if (net.width[i] > DPAC_MLP_MAX_WIDTH) return false;
  return true;
}

// one split-fp16 launch (dynamic LDS: the plan's size)
template <int NTI, int NTJ, int WI, bool L0, int NW = kPgxWaves>
int pgx_launch(const PgArgs<float>& a, int l, dim3 grid, hipStream_t s) {
  using PL = PgxPlan<NTI, NTJ, WI, L0, NW>;
  auto k = k_param_grads_x3<NTI, NTJ, WI, L0, NW>;
  if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, PL::kSmem))
    return (int)e;
  hipLaunchKernelGGL(k, grid, dim3(PL::kThreads), PL::kSmem, s, a, l);
  return (int)hipGetLastError();
}


// The merged-group kernel (k_param_grads_x3w: one 256-column group, A read once per chunk) for
// the wide hidden layers and for the input layer into a wide layer: rows of A, z_{l+1} (and G_0
// for the input layer) move by 16-byte LDS-DMA, so every row start must be 16-byte aligned.
// Outputs of <= 32 columns keep the 8-wavefront kernel (the merged-group one measured 78.5 vs
// 75 us on the lqr_d20 output layer).  DPAC_PGX_W=0 selects the two-group kernels.
inline bool pgx_w_ok(const PgArgs<float>& a, int l) {
  const char* e = getenv("DPAC_PGX_W");  // read per launch
  if (e && e[0] == '0') return false;
  const int K = a.width[l], H = a.width[l + 1];
  const bool out = H <= kPgwCW && H % 4 == 0 && a.ztot % 4 == 0 && a.zoff[l + 1] % 4 == 0 &&
                   (reinterpret_cast<uintptr_t>(a.z) & 15) == 0;
  if (l == 0)  // BN_0's sums read G_0 rows too
    return K <= 32 && H > 32 && K % 4 == 0 && a.ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(a.x) & 15) == 0 &&
           a.gtot % 4 == 0 && a.goff[0] % 4 == 0 && (reinterpret_cast<uintptr_t>(a.G) & 15) == 0 && out;
  return K > 32 && H > 32 && K <= 208 && K % 4 == 0 && a.zoff[l] % 4 == 0 && out;
}

// Layer l >= 1 on the merged-group kernel's 13-tile bin: a wide hidden layer (pgx_w_ok), or the
// output layer of <= 32 columns (one launch with the wide layers before it; its 16 waves then
// hold 2 column tiles, the others idle) — both with 129..208 inputs.
inline bool pgw13_ok(const PgArgs<float>& a, int l) {
  const int K = a.width[l], H = a.width[l + 1];
  if (K <= 128 || K > 208 || K % 4 != 0 || a.zoff[l] % 4 != 0) return false;
  if (pgx_w_ok(a, l)) return true;
  // the output layer joins only with DPAC_PG_MERGE_OUT=1: on the merged-group kernel it is slower
  // than on its own 8-wavefront kernel (round 5: all layers 467 vs 447 us at 204 800 rows)
  const char* e = getenv("DPAC_PG_MERGE_OUT");
  return l == a.L && H <= 32 && H % 4 == 0 && a.ztot % 4 == 0 && a.zoff[l + 1] % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(a.z) & 15) == 0 && e && e[0] == '1';
}

static_assert(PgwPlan<13>::kSmem + kPgwRawG0c <= 160 * 1024, "a merged launch from the input layer fits the LDS");

// DPAC_PG_MERGE=0: every layer its own launch (timing comparisons; bitwise the same results)
inline bool pg_merge() {
  const char* e = getenv("DPAC_PG_MERGE");  // read per launch
  return !(e && e[0] == '0');
}
// DPAC_PG_MERGE_IN=1: the input layer in the merged launch too (k_param_grads_x3w MODE 2).  Off
// by default: the run-time input-layer state makes that instantiation spill 54 VGPRs (round 5).
inline bool pg_merge_in() {
  const char* e = getenv("DPAC_PG_MERGE_IN");  // read per launch
  return pg_merge() && e && e[0] == '1';
}

template <int NTI, bool L0 = false, int MODE = 0>
int pgw_launch(const PgArgs<float>& a, int l, int64_t nch, hipStream_t s, int extra_lds = 0) {
  using PL = PgwPlan<NTI, L0>;
  auto k = k_param_grads_x3w<NTI, L0, MODE>;
  const int lds = PL::kSmem + extra_lds;  // + the merged input layer's compact G_0 slots
  if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, lds))
    return (int)e;
  hipLaunchKernelGGL(k, dim3((unsigned)nch), dim3(kPgwThreads), lds, s, a, l);
  return (int)hipGetLastError();
}

#ifndef DPAC_PGW_DEFAULT_D
#define DPAC_PGW_DEFAULT_D 0  // k_param_grads_x3d by default (DPAC_PGW_KERNEL overrides)
#endif
// DPAC_PGW_KERNEL=w: the 16-wavefront merged-group kernel (k_param_grads_x3w, rounds 4-5); d: its
// double-buffered 8-wavefront form (k_param_grads_x3d, round 6), bitwise the same results.
inline bool pg_double() {
  const char* e = getenv("DPAC_PGW_KERNEL");  // read per launch
  return e ? e[0] == 'd' : DPAC_PGW_DEFAULT_D;
}

template <int NTI, bool L0 = false, int MODE = 0>
int pgd_launch(const PgArgs<float>& a, int l, int64_t nch, hipStream_t s) {
  using PL = PgdPlan<NTI, L0>;
  auto k = k_param_grads_x3d<NTI, L0, MODE>;
  if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, PL::kSmem))
    return (int)e;
  hipLaunchKernelGGL(k, dim3((unsigned)nch), dim3(kPgdThreads), PL::kSmem, s, a, l);
  return (int)hipGetLastError();
}

// one layer of the split-fp16 kernel: the wide hidden layers and the input layer one 256-column
// group of 16 waves (pgx_w_ok), other wide outputs 1 x 8 waves (one column tile each,
// 128-column groups), outputs of <= 32 columns 8 x 1 waves over the row tiles
int launch_x3_layer(const PgArgs<float>& a, int l, int64_t nch, hipStream_t s) {
  const int K = a.width[l], H = a.width[l + 1];
  const int nti = (K + 15) / 16;
  if (pgx_w_ok(a, l) && pg_double()) {
    if (l == 0) return nti <= 1 ? pgd_launch<1, true>(a, l, nch, s) : pgd_launch<2, true>(a, l, nch, s);
    if (nti <= 4) return pgd_launch<4>(a, l, nch, s);
    if (nti <= 8) return pgd_launch<8>(a, l, nch, s);
    return pgd_launch<13>(a, l, nch, s);
  }
  if (pgx_w_ok(a, l)) {
    if (l == 0) return nti <= 1 ? pgw_launch<1, true>(a, l, nch, s) : pgw_launch<2, true>(a, l, nch, s);
    if (nti <= 4) return pgw_launch<4>(a, l, nch, s);
    if (nti <= 8) return pgw_launch<8>(a, l, nch, s);
    return pgw_launch<13>(a, l, nch, s);  // K <= 208 (13 tiles: 128 VGPRs without spills in the loop)
  }
  if (H <= 32) {
    const int ntj = (H + 15) / 16, nt8 = (nti + 7) / 8;
    const dim3 grid((unsigned)nch, 1u);
    if (nt8 <= 1) return ntj == 1 ? pgx_launch<1, 1, 8, false>(a, l, grid, s) : pgx_launch<1, 2, 8, false>(a, l, grid, s);
    return ntj == 1 ? pgx_launch<2, 1, 8, false>(a, l, grid, s) : pgx_launch<2, 2, 8, false>(a, l, grid, s);
  }
  if (l == 0) {  // the input layer (d <= 32: launch() sends the others to the f32 kernel)
    const dim3 grid((unsigned)nch, (unsigned)((H + 127) / 128));
    return nti <= 1 ? pgx_launch<1, 1, 1, true>(a, l, grid, s) : pgx_launch<2, 1, 1, true>(a, l, grid, s);
  }
  const dim3 grid((unsigned)nch, (unsigned)((H + 127) / 128));
  if (nti <= 1) return pgx_launch<1, 1, 1, false>(a, l, grid, s);
  if (nti <= 2) return pgx_launch<2, 1, 1, false>(a, l, grid, s);
  if (nti <= 4) return pgx_launch<4, 1, 1, false>(a, l, grid, s);
  if (nti <= 8) return pgx_launch<8, 1, 1, false>(a, l, grid, s);
  return pgx_launch<13, 1, 1, false>(a, l, grid, s);
}

// The configuration launch_x3_layer gives layer l off the merged-group kernels (pgx_w_ok false)
// and its column groups, as a k_param_grads_x3_seg segment
inline int x3_layer_cfg(const PgArgs<float>& a, int l, int& ngrp) {
  const int K = a.width[l], H = a.width[l + 1];
  const int nti = (K + 15) / 16;
  if (H <= 32) {
    const int ntj = (H + 15) / 16, nt8 = (nti + 7) / 8;
    ngrp = 1;
    if (nt8 <= 1) return ntj == 1 ? kPgxN11 : kPgxN12;
    return ntj == 1 ? kPgxN21 : kPgxN22;
  }
  ngrp = (H + 127) / 128;
  if (l == 0) return nti <= 1 ? kPgxIn1 : kPgxIn2;
  if (nti <= 1) return kPgxW1;
  if (nti <= 2) return kPgxW2;
  if (nti <= 4) return kPgxW4;
  if (nti <= 8) return kPgxW8;
  return kPgxW13;
}

#ifndef DPAC_PG_SEG_MAX_BLOCKS
#define DPAC_PG_SEG_MAX_BLOCKS 1024  // every layer in one launch up to this many workgroups in all
#endif
// Round 6: when every layer runs on the 8-wavefront split-fp16 kernel and their grids together
// stay small (the critic's V network over 3 B rows: 168 workgroups), one k_param_grads_x3_seg
// launch runs them side by side (measured per layer, the four launches were latency-bound:
// 17-28 us each on 24-48 workgroups).  DPAC_PG_SEG=0 keeps one launch per layer (tests compare
// the two bit for bit).
inline bool pg_seg_build(const PgArgs<float>& a, int64_t nch, PgxSegs& sg, int& smem) {
  const char* e = getenv("DPAC_PG_SEG");  // read per launch
  if (e && e[0] == '0') return false;
  if (a.L + 1 > (int)(sizeof(sg.s) / sizeof(sg.s[0]))) return false;
  sg.n = 0;
  smem = 0;
  int64_t b0 = 0;
  for (int l = 0; l <= a.L; ++l) {
    const int K = a.width[l], H = a.width[l + 1];
    const bool x3ok = l == 0 ? (K <= 32 && H > 32) : (H <= 32 || K <= 208);
    if (!x3ok || pgx_w_ok(a, l)) return false;
    int ngrp = 1;
    const int cfg = x3_layer_cfg(a, l, ngrp);
    if (!pgx_seg_cfg_ok(cfg)) return false;
    sg.s[sg.n++] = PgxSeg{l, cfg, ngrp, b0};
    b0 += nch * ngrp;
    smem = std::max(smem, pgx_cfg_smem(cfg));
  }
  return b0 <= DPAC_PG_SEG_MAX_BLOCKS;
}

constexpr int64_t kFallbackBlocksPg = 256;  // the guarded f32 parameter-gradient fallback's grid

template <typename T>
int launch(int64_t rows, const dpac_mlp& net, double gamma_scale, const void* x, int64_t ldx,
           const void* z, const void* G, void* ws, void* out, hipStream_t s0) {
  PgArgs<T> a = pg_args<T>(net, rows, x, ldx, z, G);
  a.rows_per_chunk = pg_chunk_rows<T>(rows, max_ld(a));
  if constexpr (std::is_same<T, float>::value) {
    if (pg_x3(net)) {
      // 32-row sub-chunks: chunks of a multiple of 32 rows, never more chunks than the
      // workspace (sized for the f32 kernel's 16-row rounding) holds
      a.rows_per_chunk = std::max<int64_t>((a.rows_per_chunk + kPgxSR - 1) / kPgxSR * kPgxSR, kPgxSR);
      const int64_t cap = (((int64_t)1 << 31) - 1) / (max_ld(a) * 4) / kPgxSR * kPgxSR;
      if (a.rows_per_chunk <= cap) {
        a.part = (float*)ws;
        a.status = net.status;
        const int64_t nch = (rows + a.rows_per_chunk - 1) / a.rows_per_chunk;
        const bool fb_only = net.guard_phase == DPAC_GUARD_FALLBACK_ONLY;
        PgxSegs sg;
        int seg_smem = 0;
        const bool seg = !fb_only && pg_seg_build(a, nch, sg, seg_smem);
        if (seg) {
          auto k = k_param_grads_x3_seg;
          if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k),
                                                 hipFuncAttributeMaxDynamicSharedMemorySize, seg_smem))
            return (int)e;
          const int64_t nb = sg.s[sg.n - 1].b0 + nch * sg.s[sg.n - 1].ngrp;
          hipLaunchKernelGGL(k, dim3((unsigned)nb), dim3(64 * kPgxWaves), seg_smem, s0, a, sg);
          if (hipError_t e = hipGetLastError()) return (int)e;
        }
        for (int l = 0; l <= a.L && !fb_only && !seg; ++l) {
          // a run of adjacent layers of the merged-group kernel's 13-tile bin (the wide hidden
          // layers, and the output layer after them): one launch (k_param_grads_x3w, lsel < 0)
          // (and the input layer before them, run by the same kernel at run time)
          const bool in = l == 0 && pg_merge_in() && pgx_w_ok(a, 0);
          int nl = in ? 1 : 0;
          while (pg_merge() && (l >= 1 || in) && l + nl <= a.L && pgw13_ok(a, l + nl)) ++nl;
          if (nl >= 2) {
            const int64_t g = (nch + 7) / 8 * 8 * nl;
            if (int e = in ? pgw_launch<13, false, 2>(a, -(l + 8 * nl), g, s0, kPgwRawG0c)
                           : (pg_double() ? pgd_launch<13, false, 1>(a, -(l + 8 * nl), g, s0)
                                          : pgw_launch<13, false, 1>(a, -(l + 8 * nl), g, s0)))
              return e;
            l += nl - 1;
            continue;
          }
          // layers the split kernel does not cover (a wide layer with more than 13 input
          // tiles; an input layer wider than 32 or into a layer of <= 32) take the f32
          // kernel on the same chunks and partial layout
          const int K = a.width[l], H = a.width[l + 1];
          const bool x3ok = l == 0 ? (K <= 32 && H > 32) : (H <= 32 || K <= 208);
          int e = 0;
          if (x3ok) e = launch_x3_layer(a, l, nch, s0);
          else e = launch_f32_layer<float>(a, l, nch, s0);
          if (e) return e;
        }
        if (net.status && net.guard_phase != DPAC_GUARD_SPLIT_ONLY) {
          // the f32 kernel over every layer, run only once an x3 kernel fell back
          PgArgs<float> f = a;
          f.status = nullptr;
          f.guard = net.status;
          int hmax = 0;
          for (int l = 0; l <= a.L; ++l) hmax = std::max(hmax, a.width[l + 1]);
          const int ngrp = (hmax + 127) / 128;  // 128-column groups of <16, 2, 1>
          hipLaunchKernelGGL((k_param_grads<float, 16, 2, 1>),
                             dim3((unsigned)std::min<int64_t>(nch * ngrp * (a.L + 1), kFallbackBlocksPg)),
                             dim3(kPgThreads), 0, s0, f, -ngrp);
          if (hipError_t e = hipGetLastError()) return (int)e;
        }
        const int64_t n = a.ptot + a.width[a.L + 1];
        PgArgs<float> r = a;  // phase 2: the reduce too runs only once an x3 kernel fell back
        r.guard = fb_only ? net.status : nullptr;
        hipLaunchKernelGGL(k_param_grads_reduce<float>, dim3((unsigned)((n + kRedCols - 1) / kRedCols)), dim3(256), 0, s0,
                           r, (int)nch, (float)gamma_scale, (float*)out);
        return (int)hipGetLastError();
      }
      a.rows_per_chunk = pg_chunk_rows<T>(rows, max_ld(a));
    }
  }
  if (net.guard_phase == DPAC_GUARD_FALLBACK_ONLY) return 0;  // phase 1 did the whole work
  a.part = (T*)ws;
  const int64_t nch = (rows + a.rows_per_chunk - 1) / a.rows_per_chunk;
  // narrow layers (K or H <= 32: grids of 256-512 small workgroups) on the forked
  // stream; every layer writes its own partial columns, so the branches share nothing
  PgFork* fk = DPAC_PG_FORK ? pg_fork() : nullptr;
  bool forked = false;
  for (int l = 0; l <= a.L; ++l) {  // one launch per layer
    const int K = a.width[l], H = a.width[l + 1];
    hipStream_t s = s0;
    if (fk && (K <= 32 || H <= 32)) {
      if (!forked) {
        if (hipError_t e = hipEventRecord(fk->fork, s0)) return (int)e;
        if (hipError_t e = hipStreamWaitEvent(fk->aux, fk->fork, 0)) return (int)e;
        forked = true;
      }
      s = fk->aux;
    }
    if (int e = launch_f32_layer<T>(a, l, nch, s)) return e;
    if (hipError_t e = hipGetLastError()) return (int)e;
  }
  if (forked) {
    if (hipError_t e = hipEventRecord(fk->join, fk->aux)) return (int)e;
    if (hipError_t e = hipStreamWaitEvent(s0, fk->join, 0)) return (int)e;
  }
  const int64_t n = a.ptot + a.width[a.L + 1];
  hipLaunchKernelGGL(k_param_grads_reduce<T>, dim3((unsigned)((n + kRedCols - 1) / kRedCols)), dim3(256), 0, s0,
                     a, (int)nch, (T)gamma_scale, (T*)out);
  return (int)hipGetLastError();
}

template <typename T>
MrArgs<T> mr_args(const dpac_mlp& net, int64_t rows) {
  MrArgs<T> a{};
  a.rows = rows;
  a.L = net.n_hidden;
  int zt = 0, gt = 0;
  for (int i = 0; i <= a.L + 1; ++i) {
    a.width[i] = net.width[i];
    a.scale[i] = (const T*)net.bn_scale[i];
    a.shift[i] = (const T*)net.bn_shift[i];
    a.zoff[i] = i == 0 ? 0 : zt;
    if (i > 0) zt += net.width[i];
    a.goff[i] = gt;
    gt += net.width[i];
  }
  for (int i = 0; i <= a.L; ++i) {
    a.weight[i] = (const T*)net.weight[i];
    a.wkm[i] = (const T*)net.weight_km[i];
  }
  a.bias = (const T*)net.bias;
  a.ztot = zt;
  a.gtot = gt;
  return a;
}

template <typename T>
void set_td(MrArgs<T>& a, const TdRows* td) {
  if (!td) return;
  a.td_x = (const T*)td->x;
  a.td_ldx = td->ldx;
  a.td_u = (const T*)td->u;
  a.td_ldu = td->ldu;
  a.td_dw = (const T*)td->dw;
  a.td_p = td->p;
  a.td_sa = (T)td->sa;
  a.td_sb = (T)td->sb;
}

// The split-fp16 row kernels (dpac_mlp_x3.h) when every image of the direction is given.
inline bool x3_all(const dpac_mlp& net, const void* const* img) {
  for (int i = 0; i <= net.n_hidden; ++i)
    if (!img[i]) return false;
  return true;
}

X3Args x3_args(const dpac_mlp& net, int64_t rows, const void* const* img, const TdRows* td) {
  X3Args a{};
  const MrArgs<float> m = mr_args<float>(net, rows);
  a.rows = rows;
  a.L = m.L;
  for (int i = 0; i <= a.L + 1; ++i) {
    a.width[i] = m.width[i];
    a.scale[i] = m.scale[i];
    a.shift[i] = m.shift[i];
    a.zoff[i] = m.zoff[i];
    a.goff[i] = m.goff[i];
  }
  for (int i = 0; i <= a.L; ++i) a.wx3[i] = (const _Float16*)img[i];
  a.bias = m.bias;
  a.ztot = m.ztot;
  a.gtot = m.gtot;
  a.nblk = (rows + 63) / 64;  // the sign-bit mask's 64-row blocks
  if (td) {
    a.td_x = (const float*)td->x;
    a.td_ldx = td->ldx;
    a.td_u = (const float*)td->u;
    a.td_ldu = td->ldu;
    a.td_dw = (const float*)td->dw;
    a.td_p = td->p;
    a.td_sa = (float)td->sa;
    a.td_sb = (float)td->sb;
  }
  return a;
}

// one workgroup per `rows_per` rows (the forward's kX3Rows, the backward's kX3RowsB), `lds` bytes
template <class K>
int x3_launch(K kfn, const X3Args& a, hipStream_t s, int rows_per = kX3Rows, uint32_t lds = kX3LdsBytes) {
  if (hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kfn),
                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds))
    return (int)e;
  hipLaunchKernelGGL(kfn, dim3((unsigned)((a.rows + rows_per - 1) / rows_per)), dim3(kX3Threads), lds, s, a);
  return (int)hipGetLastError();
}

// Grid of a guarded f32 fallback launch (dpac.h dpac_mlp.status): a grid-stride pass over
// every row tile; when the word is clear each workgroup exits after one load.
constexpr int64_t kFallbackBlocks = 256;  // one workgroup per CU (round 4: 512)

template <typename T>
int rows_fwd(int64_t rows, const dpac_mlp& net, const void* x, int64_t ldx, void* out,
             void* save_z, const TdRows* td, uint8_t* mask, int32_t* written, hipStream_t s) {
  if (written) *written = 0;
  MrArgs<T> a = mr_args<T>(net, rows);
  set_td(a, td);
  if (td) a.gdot = (T*)td->gdot;
  a.x = (const T*)x;
  a.ldx = ldx;
  a.out = (T*)out;
  a.z = (T*)save_z;
  constexpr int ROWS = MrCfg<T>::RT * 16;
  const int64_t nblk = (rows + ROWS - 1) / ROWS;
  if constexpr (std::is_same<T, float>::value) {
    // split-fp16 products when the images are given (and, guarded, the f32 operands too)
    if (x3_all(net, net.weight_x3) && (!net.status || x3_all(net, net.weight))) {
      X3Args xa = x3_args(net, rows, net.weight_x3, td);
      if (td) xa.gdot = (float*)td->gdot;
      xa.x = (const float*)x;
      xa.ldx = ldx;
      xa.out = (float*)out;
      xa.z = (float*)save_z;
      xa.status = net.status;
      xa.mask = (save_z && kX3RT == 4) ? reinterpret_cast<uint32_t*>(mask) : nullptr;  // 64-row blocks
      if (net.guard_phase != DPAC_GUARD_FALLBACK_ONLY)
        if (int e = x3_launch(k_mlp_rows_fwd_x3, xa, s)) return e;
      if (written && xa.mask) *written = 1;
      if (!net.status || net.guard_phase == DPAC_GUARD_SPLIT_ONLY) return 0;
      a.guard = net.status;  // the f32 kernel recomputes everything once the x3 kernel fell back
      hipLaunchKernelGGL(k_mlp_rows_fwd<T>, dim3((unsigned)std::min(nblk, kFallbackBlocks)), dim3(kMrThreads), 0,
                         s, a);
      return (int)hipGetLastError();
    }
  }
  if (net.guard_phase == DPAC_GUARD_FALLBACK_ONLY) return 0;  // phase 1 did the whole work
  hipLaunchKernelGGL(k_mlp_rows_fwd<T>, dim3((unsigned)nblk), dim3(kMrThreads), 0, s, a);
  return (int)hipGetLastError();
}

template <typename T>
int rows_bwd(int64_t rows, const dpac_mlp& net, const void* const* wt, const void* save_z,
             const uint8_t* mask, const void* g_out, void* G, void* g_x, const TdRows* td, hipStream_t s) {
  if constexpr (std::is_same<T, float>::value) {
    if (x3_all(net, net.weight_t_x3) && (!net.status || x3_all(net, wt))) {
      X3Args a = x3_args(net, rows, net.weight_t_x3, td);
      if (td) a.g_gdot = (const float*)td->g_gdot;
      a.z = (float*)save_z;
      a.g_out = (const float*)g_out;
      a.G = (float*)G;
      a.g_x = (float*)g_x;
      a.status = net.status;
      a.mask = reinterpret_cast<uint32_t*>(const_cast<uint8_t*>(mask));
      if (net.guard_phase != DPAC_GUARD_FALLBACK_ONLY)
        if (int e = mask ? x3_launch(k_mlp_rows_bwd_x3<true>, a, s, kX3RowsB, kX3LdsBytesB)
                         : x3_launch(k_mlp_rows_bwd_x3<false>, a, s, kX3RowsB, kX3LdsBytesB))
          return e;
      if (!net.status || net.guard_phase == DPAC_GUARD_SPLIT_ONLY) return 0;
      MrArgs<T> f = mr_args<T>(net, rows);  // the f32 kernel, run only once the x3 kernel fell back
      set_td(f, td);
      if (td) f.g_gdot = (const T*)td->g_gdot;
      for (int i = 0; i <= f.L; ++i) f.wt[i] = (const T*)wt[i];
      f.z = (T*)save_z;
      f.g_out = (const T*)g_out;
      f.G = (T*)G;
      f.g_x = (T*)g_x;
      f.guard = net.status;
      constexpr int ROWS = MrCfg<T>::RT * 16;
      hipLaunchKernelGGL(k_mlp_rows_bwd<T>, dim3((unsigned)std::min((rows + ROWS - 1) / ROWS, kFallbackBlocks)),
                         dim3(kMrThreads), 0, s, f);
      return (int)hipGetLastError();
    }
  }
  if (net.guard_phase == DPAC_GUARD_FALLBACK_ONLY) return 0;  // phase 1 did the whole work
  MrArgs<T> a = mr_args<T>(net, rows);
  set_td(a, td);
  if (td) a.g_gdot = (const T*)td->g_gdot;
  for (int i = 0; i <= a.L; ++i) a.wt[i] = (const T*)wt[i];
  a.z = (T*)save_z;
  a.g_out = (const T*)g_out;
  a.G = (T*)G;
  a.g_x = (T*)g_x;
  constexpr int ROWS = MrCfg<T>::RT * 16;
  hipLaunchKernelGGL(k_mlp_rows_bwd<T>, dim3((unsigned)((rows + ROWS - 1) / ROWS)),
                     dim3(kMrThreads), 0, s, a);
  return (int)hipGetLastError();
}

}  // namespace

int mlp_rows_fwd_launch(int dtype, int64_t rows, const dpac_mlp& net, const void* x, int64_t ldx,
                        void* out, void* save_z, const TdRows* td, uint8_t* mask, int32_t* written,
                        hipStream_t s) {
  return dtype == DPAC_F64 ? rows_fwd<double>(rows, net, x, ldx, out, save_z, td, nullptr, written, s)
                           : rows_fwd<float>(rows, net, x, ldx, out, save_z, td, mask, written, s);
}

int mlp_rows_bwd_launch(int dtype, int64_t rows, const dpac_mlp& net, const void* const* wt,
                        const void* save_z, const uint8_t* mask, const void* g_out, void* G, void* g_x,
                        const TdRows* td, hipStream_t s) {
  return dtype == DPAC_F64 ? rows_bwd<double>(rows, net, wt, save_z, nullptr, g_out, G, g_x, td, s)
                           : rows_bwd<float>(rows, net, wt, save_z, mask, g_out, G, g_x, td, s);
}

int64_t mlp_rows_mask_bytes(int dtype, int64_t rows, const dpac_mlp& net) {
  // only the split-fp16 forward writes it, over 64-row workgroups (dpac_mlp_x3.h X3Args::mask)
  if (dtype != DPAC_F32 || !x3_all(net, net.weight_x3) || kX3RT != 4) return 0;
  return (int64_t)net.n_hidden * ((rows + 63) / 64) * kX3MaskWords * 4;
}

int64_t mlp_param_grads_ws_bytes(int dtype, int64_t rows, const dpac_mlp& net) {
  if (DPAC_PG_FORK) (void)pg_fork();
  return dtype == DPAC_F64 ? ws_bytes<double>(rows, net) : ws_bytes<float>(rows, net);
}

int mlp_param_grads_launch(int dtype, int64_t rows, const dpac_mlp& net, double gamma_scale,
                           const void* x, int64_t ldx, const void* z, const void* G, void* ws,
                           void* out, hipStream_t s) {
  return dtype == DPAC_F64 ? launch<double>(rows, net, gamma_scale, x, ldx, z, G, ws, out, s)
                           : launch<float>(rows, net, gamma_scale, x, ldx, z, G, ws, out, s);
}

}  // namespace dpac

#if DPAC_X3_TRACE
// Timing builds only: copy the x3 row kernels' clock table (dpac_mlp_x3.h) to the host.
extern "C" int dpac_debug_x3_trace(void* host, int64_t bytes) {
  const int64_t n = bytes < (int64_t)sizeof(dpac::g_x3_trace) ? bytes : (int64_t)sizeof(dpac::g_x3_trace);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(dpac::g_x3_trace), (size_t)n, 0, hipMemcpyDeviceToHost);
}
#endif
