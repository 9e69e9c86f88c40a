// dpac_mlp_rows.h — a DeepNN (solver.py:227-278) over R independent rows, on
// MFMA: the forward with the backward saves, and the backward's input-gradient
// chain.  Used for the critic's V and G networks (solver.py:161-190), which the
// reference evaluates per step inside the TD loop (solver.py:166-184) — here the
// G network runs once over all N*B rows of the finished rollout.
//
// Workgroup = 4 wavefronts over RT*16 consecutive rows.  Every dense layer is an
// [RT*16 x K] x [K x H] product: the waves split the 16-column tiles, each wave
// keeps RT x NT accumulator tiles, B fragments (the weights, L2-resident) stream
// through an 8-deep register ring shared by the RT row tiles, A fragments come
// from the LDS image of the layer input.  Activations never leave LDS between
// layers; the epilogues apply BN / y + relu(y) (forward) or the activation
// factor (backward) and write the saves / G rows.
#pragma once

#include "dpac_device.h"

namespace dpac {

constexpr int kMrThreads = 256;
constexpr int kMrWaves = 4;
#ifndef DPAC_MR_LD_PAD
#define DPAC_MR_LD_PAD 8  // row stride 264 = 8 mod 64 dwords: conflict-free ds_read_b128 A reads on gfx950 (+4 left 2-way conflicts)
#endif
constexpr int kMrLd = DPAC_MLP_MAX_WIDTH + DPAC_MR_LD_PAD;  // LDS row stride: 16 rows x 4 k hit 64 banks
constexpr int kMrPrefetch = 8;
#ifndef DPAC_MR_ROT
#define DPAC_MR_ROT 0  // rotate the waves' column-tile sets per workgroup (timing knob)
#endif
#ifndef DPAC_MR_PIN
#define DPAC_MR_PIN 0  // sched_barrier after each k group of the k-major layers (timing knob)
#endif

template <typename T>
struct MrCfg;
#ifndef DPAC_MR_RT_F32
#define DPAC_MR_RT_F32 1
#endif
template <>
struct MrCfg<float> {
  static constexpr int RT = DPAC_MR_RT_F32;  // 16 rows per workgroup: occupancy beats B reuse (measured)
};
template <>
struct MrCfg<double> {
  static constexpr int RT = 2;
};

template <typename T>
struct MrArgs {
  int64_t rows;
  int L;
  int width[DPAC_MLP_MAX_HIDDEN + 2];
  const T* scale[DPAC_MLP_MAX_HIDDEN + 2];
  const T* shift[DPAC_MLP_MAX_HIDDEN + 2];
  const T* weight[DPAC_MLP_MAX_HIDDEN + 1];  // forward: W_i [w_i][w_{i+1}]
  const T* wt[DPAC_MLP_MAX_HIDDEN + 1];      // backward: (W_i diag s_{i+1})^T [w_{i+1}][w_i]
  const T* wkm[DPAC_MLP_MAX_HIDDEN + 1];     // k-major images of weight (fwd) / wt (bwd), optional
  const T* bias;
  int zoff[DPAC_MLP_MAX_HIDDEN + 2], goff[DPAC_MLP_MAX_HIDDEN + 2];
  int ztot, gtot;
  const T* x;      // [rows][ldx]
  int64_t ldx;
  T* out;          // [rows][w_{L+1}]
  T* z;            // saves [rows][ztot] (forward: optional output; backward: input)
  const T* g_out;  // backward: dL/d out [rows][w_{L+1}]
  T* G;            // backward: [rows][gtot]
  T* g_x;          // backward, optional: dL/dx [rows][w_0]
  // TD1 fused with the output layer (dpac_mlp_rows_fwd_td1 /
  // _bwd_td1): the output G (width d) meets (sigma(x,u) dw) of its own row, with
  // sigma_j = sa (sb == 0) or sa * (1 + (sb * x_j) * u_j) — every equation's
  // elementwise sigma (dpac_device.h).  Components are owned as k_td owns them (lane
  // p of a td_p-lane group: j = p*M + m) and summed with the same DPP tree, so the
  // dot is bitwise k_td's.
  const T* td_x;     // [rows][td_ldx] raw state rows
  const T* td_u;     // [rows][td_ldu] (read only when sb != 0)
  const T* td_dw;    // [rows][d]
  int64_t td_ldx;
  int td_ldu, td_p;
  T td_sa, td_sb;
  T* gdot;           // forward: [rows] sum_j (sigma_j dw_j) G_j; `out` is not written
  const T* g_gdot;   // backward: [rows]; dL/d out_j = g_gdot * (sigma_j dw_j)
  // the f32 fallback of a split-fp16 launch (dpac.h dpac_mlp.status): run only once the
  // word is set, over all row tiles with a grid-stride loop (a small grid); null = always run
  const uint32_t* guard;
};

// The TD1 operands (x, u, dw) of one row block [row0, row0 + live) through buffer descriptors
// sized to exactly those rows (round 6): a row past the block reads 0, never memory past the
// arrays (round 5's fault: a dead 16-row block read its first row's sigma dw through plain
// pointers, up to 48 rows past the end of dw).
template <typename T>
struct TdSrc {
  __amdgpu_buffer_rsrc_t x, u, dw;
  int64_t row0;
  int live, ldx, ldu, d;
  T sa, sb;
};

template <typename T>
__device__ __forceinline__ TdSrc<T> td_src(const MrArgs<T>& a, int64_t row0, int live, int d) {
  return TdSrc<T>{rows_rsrc(a.td_x, row0, live, a.td_ldx), rows_rsrc(a.td_u, row0, live, a.td_ldu),
                  rows_rsrc(a.td_dw, row0, live, d), row0, live, (int)a.td_ldx, (int)a.td_ldu, d, a.td_sa,
                  a.td_sb};
}

// (sigma(x,u) dw)_j of row r (0 past d, and 0 for a row outside the block).
template <typename T>
__device__ __forceinline__ T td_sdw(const TdSrc<T>& t, int64_t r, int j) {
  if (j >= t.d) return T(0);
  DPAC_CHECK_ROW(r - t.row0, t.live);
  const uint32_t o = (uint32_t)(r - t.row0);
  T s = t.sa;
  if (t.sb != T(0))
    s = t.sa * (1 + (t.sb * buf_load_elem<T>(t.x, (o * (uint32_t)t.ldx + (uint32_t)j) * (uint32_t)sizeof(T))) *
                        buf_load_elem<T>(t.u, (o * (uint32_t)t.ldu + (uint32_t)j) * (uint32_t)sizeof(T)));
  return s * buf_load_elem<T>(t.dw, (o * (uint32_t)t.d + (uint32_t)j) * (uint32_t)sizeof(T));
}

template <int P, typename T>
__device__ __forceinline__ T td_group_sum(T v) {
  return Lanes<P>::sum(v);
}

// gdot for the ROWS rows of this workgroup from the LDS image G [ROWS][kMrLd]: 16
// lanes per row, the first td_p of them own the components (k_td's split).
// With one row per 16 lanes (ROWS == 16) and at most kTdPre components per lane, the
// lane's (sigma dw) values are loaded at kernel start (td_prefetch), so the dot phase
// after the last layer reads only LDS.
constexpr int kTdPre = 4;
template <typename T, int ROWS>
__device__ __forceinline__ bool td_prefetch(const MrArgs<T>& a, int64_t row0, int rows_live, int d, int tid,
                                            T (&pre)[kTdPre]) {
  const int P = a.td_p, M = (d + P - 1) / P;
  if (!a.gdot || ROWS != kMrThreads / 16 || M > kTdPre) return false;
  const int l16 = tid % 16, rr = tid / 16;
  const TdSrc<T> src = td_src(a, row0, rows_live, d);
  const int64_t r = row0 + rr;  // past the block: reads 0 (unused: td_dot_rows stores live rows only)
#pragma unroll
  for (int m = 0; m < kTdPre; ++m)
    pre[m] = (l16 < P && m < M && rr < rows_live) ? td_sdw(src, r, l16 * M + m) : T(0);
  return true;
}

// rows_live <= 0 (a 16-row block of the split-fp16 forward's last workgroup past the last row):
// nothing to do.  Round 5: such a block used to read its first row's sigma dw anyway, past the
// end of dw (and of x, u for LQR_var) — an out-of-bounds read that faults only when the rows end
// near the end of mapped memory (seen once, tests/test_gpu_td_fused.py, LQR d = 4).
template <typename T, int ROWS>
__device__ __forceinline__ void td_dot_rows(const MrArgs<T>& a, const T* G, int64_t row0, int rows_live,
                                            int d, int tid, bool have_pre, const T (&pre)[kTdPre]) {
  if (rows_live <= 0) return;  // uniform over the call's threads
  const int l16 = tid % 16, P = a.td_p, M = (d + P - 1) / P;
  const TdSrc<T> src = td_src(a, row0, rows_live, d);
  for (int rr = tid / 16; rr < ROWS; rr += kMrThreads / 16) {
    const int64_t r = row0 + (rr < rows_live ? rr : 0);
    T acc = T(0);
    if (l16 < P) {
      if (have_pre) {
#pragma unroll
        for (int m = 0; m < kTdPre; ++m) {
          const int j = l16 * M + m;
          const T g = (m < M && j < d) ? G[rr * kMrLd + j] : T(0);
          if (m < M) acc = m == 0 ? pre[m] * g : fma(pre[m], g, acc);
        }
      } else {
        for (int m = 0; m < M; ++m) {
          const int j = l16 * M + m;
          const T g = j < d ? G[rr * kMrLd + j] : T(0);
          const T sdw = td_sdw(src, r, j);
          acc = m == 0 ? sdw * g : fma(sdw, g, acc);
        }
      }
    }
    switch (P) {
      case 2: acc = td_group_sum<2>(acc); break;
      case 4: acc = td_group_sum<4>(acc); break;
      case 8: acc = td_group_sum<8>(acc); break;
      case 16: acc = td_group_sum<16>(acc); break;
      default: break;
    }
    if (l16 == 0 && rr < rows_live) a.gdot[r] = acc;
  }
}

// acc[RT][NT] = in[RT*16 x K] @ W[K x Nout] for this wave's NT column tiles
// (wave, wave + 4, ...), then epi.template finish<NT>(acc).  `in` is an LDS
// [RT*16][kMrLd] image whose columns past K hold finite values (the B rows past
// K read 0 through the descriptor, so they add nothing).
template <typename T, int NT, int RT, class EPI>
__device__ __forceinline__ void mr_layer_nt(const T* in, int K, int Nout, const T* W, int wave,
                                            int lane, EPI& epi) {
  using MF = Mfma<T>;
  const int col_l = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (uint32_t)(K * Nout * (int)sizeof(T)));
  uint32_t voff[NT];
  typename MF::acc_t acc[RT][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kMrWaves * j) * 16 + col_l;
    voff[j] = col < Nout ? (uint32_t)((kq * Nout + col) * (int)sizeof(T)) : kOOB;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt][j] = typename MF::acc_t{0, 0, 0, 0};
  }
  const uint32_t kstep_bytes = (uint32_t)(4 * Nout * (int)sizeof(T));
  const int nks = (K + 3) / 4;
  const T* arow = in + col_l * kMrLd + kq;
  auto loadB = [&](int ks, int j) {
    uint32_t w[sizeof(T) / 4];
    buf_load_dwords<sizeof(T) / 4>(rW, voff[j] + (uint32_t)ks * kstep_bytes, w);
    T v;
    __builtin_memcpy(&v, &w[0], sizeof(T));
    return v;
  };
  auto loadA = [&](int ks, int rt) { return arow[rt * 16 * kMrLd + 4 * (ks < nks ? ks : nks - 1)]; };
  T bq[kMrPrefetch][NT], av[kMrPrefetch][RT];
#pragma unroll
  for (int q = 0; q < kMrPrefetch; ++q) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) av[q][rt] = loadA(q, rt);
#pragma unroll
    for (int j = 0; j < NT; ++j) bq[q][j] = loadB(q, j);
  }
  for (int ks0 = 0; ks0 < nks; ks0 += kMrPrefetch) {
    T an[kMrPrefetch][RT];
#pragma unroll
    for (int q = 0; q < kMrPrefetch; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) an[q][rt] = loadA(ks0 + kMrPrefetch + q, rt);
#pragma unroll
    for (int q = 0; q < kMrPrefetch; ++q) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) acc[rt][j] = MF::mma(av[q][rt], bq[q][j], acc[rt][j]);
        bq[q][j] = loadB(ks0 + q + kMrPrefetch, j);
      }
    }
#pragma unroll
    for (int q = 0; q < kMrPrefetch; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) av[q][rt] = an[q][rt];
  }
  epi.template finish<NT>(acc, wave, lane);
}

// The same product from a k-major weight image (float; dpac_mlp.weight_km): one
// dwordx4 per lane and tile brings 4 consecutive k of one column and one
// ds_read_b128 per row tile the matching A values; the k of MFMA e of group s in
// lane quad kq is 16s + 4kq + e (as mfma_rows16_km in dpac_rollout_nn.h).
template <int NT, int RT, class EPI>
__device__ __forceinline__ void mr_layer_nt_km(const float* in, int K, int Nout, const float* Wkm,
                                               int wave, int lane, EPI& epi) {
  using MF = Mfma<float>;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int col_l = lane & 15, kq = lane >> 4;
  const int K16 = (K + 15) / 16 * 16, ng = K16 / 16;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
  uint32_t voff[NT];
  MF::acc_t acc[RT][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kMrWaves * j) * 16 + col_l;
    voff[j] = col < Nout ? (uint32_t)((col * K16 + 4 * kq) * 4) : kOOB;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) acc[rt][j] = MF::acc_t{0, 0, 0, 0};
  }
  const float* arow = in + col_l * kMrLd + 4 * kq;  // 16-byte aligned: kMrLd % 4 == 0
  auto loadB = [&](int s, int j) {
    uint32_t w[4];
    buf_load_dwords<4>(rW, s < ng ? voff[j] + (uint32_t)(s * 64) : kOOB, w);
    f4 v;
    __builtin_memcpy(&v, &w[0], 16);
    return v;
  };
  auto loadA = [&](int s, int rt) {
    return *reinterpret_cast<const f4*>(arow + rt * 16 * kMrLd + 16 * (s < ng ? s : ng - 1));
  };
  constexpr int PG = 2;  // groups (8 k-steps) of B in flight per tile
  f4 bq[PG][NT], av[PG][RT];
#pragma unroll
  for (int q = 0; q < PG; ++q) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) av[q][rt] = loadA(q, rt);
#pragma unroll
    for (int j = 0; j < NT; ++j) bq[q][j] = loadB(q, j);
  }
  for (int s0 = 0; s0 < ng; s0 += PG) {
    f4 an[PG][RT];
#pragma unroll
    for (int q = 0; q < PG; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) an[q][rt] = loadA(s0 + PG + q, rt);
#pragma unroll
    for (int q = 0; q < PG; ++q) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int rt = 0; rt < RT; ++rt) acc[rt][j] = MF::mma(av[q][rt][e], bq[q][j][e], acc[rt][j]);
        bq[q][j] = loadB(s0 + q + PG, j);
      }
#if DPAC_MR_PIN
      __builtin_amdgcn_sched_barrier(0);  // keep the B ring PG groups ahead (dpac_rollout_nn.h)
#endif
    }
#pragma unroll
    for (int q = 0; q < PG; ++q)
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) av[q][rt] = an[q][rt];
  }
  epi.template finish<NT>(acc, wave, lane);
}

template <typename T, int RT, class EPI>
__device__ __forceinline__ void mr_layer(const T* in, int K, int Nout, const T* W, const T* Wkm,
                                         int wave, int lane, EPI& epi) {
  const int ntiles = (Nout + 15) / 16;
  const int mine = ntiles > wave ? (ntiles - wave + kMrWaves - 1) / kMrWaves : 0;
  static_assert(DPAC_MLP_MAX_WIDTH / 16 / kMrWaves == 4, "dispatch below covers 1..4 tiles");
  if constexpr (sizeof(T) == 4) {
    if (Wkm) {  // block-uniform
      switch (mine) {
        case 1: mr_layer_nt_km<1, RT>(in, K, Nout, Wkm, wave, lane, epi); break;
        case 2: mr_layer_nt_km<2, RT>(in, K, Nout, Wkm, wave, lane, epi); break;
        case 3: mr_layer_nt_km<3, RT>(in, K, Nout, Wkm, wave, lane, epi); break;
        case 4: mr_layer_nt_km<4, RT>(in, K, Nout, Wkm, wave, lane, epi); break;
        default: break;
      }
      return;
    }
  }
  switch (mine) {
    case 1: mr_layer_nt<T, 1, RT>(in, K, Nout, W, wave, lane, epi); break;
    case 2: mr_layer_nt<T, 2, RT>(in, K, Nout, W, wave, lane, epi); break;
    case 3: mr_layer_nt<T, 3, RT>(in, K, Nout, W, wave, lane, epi); break;
    case 4: mr_layer_nt<T, 4, RT>(in, K, Nout, W, wave, lane, epi); break;
    default: break;
  }
}

// Forward epilogue of dense layer l (output width Nout): z -> save -> BN(z (+ b))
// -> [y + relu(y)] into the next LDS image, or (output layer) to `out`.
template <typename T, int RT>
struct MrFwdEpi {
  const T *scale, *shift, *bias;  // BN_{l+1}; bias only for the output layer
  bool hidden;
  int Nout, rows_live;
  T* lds;           // next layer's input image
  T* save;          // z of row 0 of the workgroup at this layer's column offset, or null
  int64_t save_ld;
  T* out;           // output layer: out row 0 of the workgroup
  int64_t out_ld;
  template <int NT>
  __device__ __forceinline__ void finish(typename Mfma<T>::acc_t (&acc)[RT][NT], int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = (wave + kMrWaves * j) * 16 + (lane & 15);
      const bool valid = col < Nout;
      const T s = valid ? scale[col] : T(0), sh = valid ? shift[col] : T(0);
      const T bb = (valid && bias) ? bias[col] : T(0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rt * 16 + Mfma<T>::row(lane, i);
          const T zv = acc[rt][j][i];
          const bool st = valid && row < rows_live;
          if (save && st) save[row * save_ld + col] = zv;
          T yv = bias ? zv + bb : zv;   // addmm(b, y, W) (solver.py:270)
          yv = sh + yv * s;              // addcmul(beta, y, gamma/sqrt(1+eps))
          if (hidden) {
            yv = yv + fmax(yv, T(0));    // y + relu(y) (solver.py:269)
            lds[row * kMrLd + col] = valid ? yv : T(0);
          } else if (!out) {             // TD1 fused: G stays in LDS
            lds[row * kMrLd + col] = valid ? yv : T(0);
          } else if (st) {
            out[row * out_ld + col] = yv;
          }
        }
      }
    }
  }
};

// Backward epilogue of the input-gradient product g = G_{l+1} @ (W_l diag s_{l+1})^T
// (output width Nout = w_l): for l >= 1 times the activation factor 1 + [y_l > 0]
// (y_l = BN_l(z_l), z_l from the saves), then G_l to global and to LDS.
template <typename T, int RT>
struct MrBwdEpi {
  const T *scale, *shift;  // BN_l, or null for l == 0
  const T* z;              // z_l of row 0 of the workgroup (l >= 1)
  int64_t z_ld;
  int Nout, rows_live;
  T* lds;
  T* g;                    // G_l of row 0 of the workgroup
  int64_t g_ld;
  template <int NT>
  __device__ __forceinline__ void finish(typename Mfma<T>::acc_t (&acc)[RT][NT], int wave, int lane) {
    T zz[NT][RT][4];
    if (scale) {  // all the z loads first, then the stores
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = (wave + kMrWaves * j) * 16 + (lane & 15);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = rt * 16 + Mfma<T>::row(lane, i);
            zz[j][rt][i] = (col < Nout && row < rows_live) ? z[row * z_ld + col] : T(0);
          }
      }
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int col = (wave + kMrWaves * j) * 16 + (lane & 15);
      const bool valid = col < Nout;
      const T s = (scale && valid) ? scale[col] : T(0), sh = (scale && valid) ? shift[col] : T(0);
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = rt * 16 + Mfma<T>::row(lane, i);
          T v = acc[rt][j][i];
          if (scale) {
            const T yv = sh + zz[j][rt][i] * s;     // the forward's BN_l output
            v = v * (yv > T(0) ? T(2) : T(1));      // d(y + relu(y))/dy
          }
          if (valid && row < rows_live) g[row * g_ld + col] = v;
          lds[row * kMrLd + col] = valid ? v : T(0);
        }
      }
    }
  }
};

// The wave's column-tile set.  13 tiles over 4 waves leave one wave with 4; with
// DPAC_MR_ROT the heavy set rotates over the workgroups that share a CU (the
// dispatcher deals blocks round-robin over the 8 XCDs, so blocks b, b+8, ... share
// an XCD).  Each tile is still computed by one wave in one k order: bitwise the same.
__device__ __forceinline__ int mr_wave(int tid) {
  int w = tid / 64;
  if constexpr (DPAC_MR_ROT == 1) w = (w + (int)(blockIdx.x >> 3)) & (kMrWaves - 1);
  if constexpr (DPAC_MR_ROT == 2) w = (w + (int)blockIdx.x) & (kMrWaves - 1);
  return __builtin_amdgcn_readfirstlane(w);
}

template <typename T>
__global__ __launch_bounds__(kMrThreads) void k_mlp_rows_fwd(const MrArgs<T> a) {
  constexpr int RT = MrCfg<T>::RT, ROWS = RT * 16;
  __shared__ T s_img[2][ROWS * kMrLd];
  if (a.guard && !x3_status_set(a.guard)) return;  // a fallback launch: only once the x3 kernel fell back
  const int tid = threadIdx.x;
  const int wave = mr_wave(tid), lane = tid % 64;
  const int64_t nblk = (a.rows + ROWS - 1) / ROWS;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // one pass unless a fallback launch
    if (blk != (int64_t)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    const int64_t row0 = blk * ROWS;
    const int rows_live = (int)((a.rows - row0) < ROWS ? (a.rows - row0) : ROWS);
    const int d = a.width[0];
    // a_0 = BN_0(x) into image 0 (solver.py:265); everything else zero
    const __amdgpu_buffer_rsrc_t rx = rows_rsrc(a.x, row0, rows_live, a.ldx);
    for (int e = tid; e < ROWS * kMrLd; e += kMrThreads) {
      const int r = e / kMrLd, k = e % kMrLd;
      T v = T(0);
      if (k < d && r < rows_live) {
        DPAC_CHECK_ROW(r, rows_live);
        v = a.shift[0][k] + buf_load_elem<T>(rx, (uint32_t)(r * a.ldx + k) * (uint32_t)sizeof(T)) * a.scale[0][k];
      }
      s_img[0][e] = v;
      s_img[1][e] = T(0);
    }
    T td_pre[kTdPre];
    const bool have_pre = td_prefetch<T, ROWS>(a, row0, rows_live, a.width[a.L + 1], tid, td_pre);
    __syncthreads();
    int pq = 0;
    for (int l = 0; l <= a.L; ++l) {
      const int Nout = a.width[l + 1];
      MrFwdEpi<T, RT> epi{a.scale[l + 1], a.shift[l + 1], l == a.L ? a.bias : nullptr, l < a.L,
                          Nout, rows_live, s_img[pq ^ 1],
                          a.z ? a.z + row0 * a.ztot + a.zoff[l + 1] : nullptr, a.ztot,
                          a.gdot ? nullptr : a.out + row0 * Nout, Nout};
      mr_layer<T, RT>(s_img[pq], a.width[l], Nout, a.weight[l], a.wkm[l], wave, lane, epi);
      __syncthreads();
      pq ^= 1;
    }
    if (a.gdot) td_dot_rows<T, ROWS>(a, s_img[pq], row0, rows_live, a.width[a.L + 1], tid, have_pre, td_pre);
  }
}

template <typename T>
__global__ __launch_bounds__(kMrThreads) void k_mlp_rows_bwd(const MrArgs<T> a) {
  constexpr int RT = MrCfg<T>::RT, ROWS = RT * 16;
  __shared__ T s_img[2][ROWS * kMrLd];
  if (a.guard && !x3_status_set(a.guard)) return;  // a fallback launch: only once the x3 kernel fell back
  const int tid = threadIdx.x;
  const int wave = mr_wave(tid), lane = tid % 64;
  const int L = a.L, hout = a.width[L + 1];
  const int64_t nblk = (a.rows + ROWS - 1) / ROWS;
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {  // one pass unless a fallback launch
    if (blk != (int64_t)blockIdx.x) __syncthreads();  // the previous tile's LDS reads are done
    const int64_t row0 = blk * ROWS;
    const int rows_live = (int)((a.rows - row0) < ROWS ? (a.rows - row0) : ROWS);
    // G_{L+1} = dL/d out: into image 0 and to G
    const TdSrc<T> src = td_src(a, row0, rows_live, hout);
    const __amdgpu_buffer_rsrc_t rgd = rows_rsrc(a.g_gdot, row0, rows_live, 1);
    const __amdgpu_buffer_rsrc_t rgo = rows_rsrc(a.g_out, row0, rows_live, hout);
    for (int e = tid; e < ROWS * kMrLd; e += kMrThreads) {
      const int r = e / kMrLd, k = e % kMrLd;
      T v = T(0);
      if (k < hout && r < rows_live) {
        DPAC_CHECK_ROW(r, rows_live);
        v = a.g_gdot ? buf_load_elem<T>(rgd, (uint32_t)r * (uint32_t)sizeof(T)) * td_sdw(src, row0 + r, k)
                     : buf_load_elem<T>(rgo, (uint32_t)(r * hout + k) * (uint32_t)sizeof(T));  // td_assemble_bwd's product
        a.G[(row0 + r) * a.gtot + a.goff[L + 1] + k] = v;
      }
      s_img[0][e] = v;
      s_img[1][e] = T(0);
    }
    __syncthreads();
    int pq = 0;
    for (int l = L; l >= 0; --l) {
      MrBwdEpi<T, RT> epi{l >= 1 ? a.scale[l] : nullptr, l >= 1 ? a.shift[l] : nullptr,
                          a.z + row0 * a.ztot + a.zoff[l], a.ztot, a.width[l], rows_live,
                          s_img[pq ^ 1], a.G + row0 * a.gtot + a.goff[l], a.gtot};
      mr_layer<T, RT>(s_img[pq], a.width[l + 1], a.width[l], a.wt[l], a.wkm[l], wave, lane, epi);
      __syncthreads();
      pq ^= 1;
    }
    if (a.g_x) {  // dL/dx = G_0 * s_0 (a_0 = beta_0 + x * s_0)
      const int d = a.width[0];
      for (int e = tid; e < rows_live * d; e += kMrThreads) {
        const int r = e / d, k = e % d;
        a.g_x[(row0 + r) * d + k] = s_img[pq][r * kMrLd + k] * a.scale[0][k];
      }
    }
  }
}

}  // namespace dpac
