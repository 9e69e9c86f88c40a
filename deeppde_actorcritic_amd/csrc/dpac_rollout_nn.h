// dpac_rollout_nn.h — the rollout with the actor MLP as control, fused into one
// launch: equation.py:46-106 with NN_control
// (solver.py:260-278) evaluated inside the time loop.
//
// One workgroup (256 threads, 4 wavefronts) owns kNnRows = 16 trajectories for
// all N steps.  Per step:
//   1. the step lanes write a0 = BN_0(x_t) into LDS (solver.py:265);
//   2. every hidden layer is a [16 x K] x [K x H] product on 16x16x4 MFMA tiles
//      (f32 or f64 in, same-precision accumulate), the 4 wavefronts splitting
//      the 16-column tiles; BN and y + relu(y) run in the epilogue
//      (solver.py:266-269) and write the next layer's input to LDS;
//   3. the output layer adds the bias and BN_last (solver.py:270-271) -> u_t;
//   4. the step lanes (P per trajectory, the k_rollout layout) apply the Eikonal
//      head if any (solver.py:272-274) and one transition of the scheme.
// Activations never leave LDS; the weights (<= 0.35 MB at 3 x 200) are read
// through buffer descriptors from L2, with out-of-range offsets returning the
// zero padding of partial tiles.  Optionally the pre-BN layer outputs, the
// flags and the discount of every step are saved for the backward pass.
#pragma once
// Included by dpac_kernels.h inside namespace dpac.

constexpr int kNnRows = 16;      // trajectories per workgroup = one MFMA row tile
constexpr int kNnThreads = 256;  // 4 wavefronts
constexpr int kNnWaves = kNnThreads / 64;
constexpr int kNnLd = DPAC_MLP_MAX_WIDTH + 4;  // LDS row stride (elements)
constexpr int kNnMaxTilesPerWave = (DPAC_MLP_MAX_WIDTH / 16 + kNnWaves - 1) / kNnWaves;
constexpr int kNnPrefetch = 8;  // k-steps of B in flight per tile
#ifndef DPAC_NN_ABLATE
#define DPAC_NN_ABLATE 0  // timing-only builds: 1 = constant weights, 2 = skip the MLP
#endif
// The ring reads A up to k < 4 * roundup(ceil(K/4), kNnPrefetch) <= 256 for K <= 256.
static_assert(DPAC_MLP_MAX_WIDTH <= 256 && kNnLd >= 256, "A reads stay inside an LDS row");

// 16x16x4 MFMA for one precision.  A[row l&15][k l>>4], B[k l>>4][col l&15];
// the accumulator's element i of lane l is C[row(l, i)][l&15].
template <typename T>
struct Mfma;
template <>
struct Mfma<float> {
  using acc_t = __attribute__((ext_vector_type(4))) float;
  __device__ static acc_t mma(float a, float b, acc_t c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  __device__ static int row(int lane, int i) { return (lane >> 4) * 4 + i; }
};
template <>
struct Mfma<double> {
  using acc_t = __attribute__((ext_vector_type(4))) double;
  __device__ static acc_t mma(double a, double b, acc_t c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  __device__ static int row(int lane, int i) { return (lane >> 4) + 4 * i; }  // f64 C map
};

// The MLP as the kernel sees it (from dpac_mlp, include/dpac.h).
template <typename T>
struct NnMlp {
  int L, ekn;
  int width[DPAC_MLP_MAX_HIDDEN + 2];
  int zoff[DPAC_MLP_MAX_HIDDEN + 2];  // column offset of layer i's z in a save row
  int ztot;
  const T* scale[DPAC_MLP_MAX_HIDDEN + 2];
  const T* shift[DPAC_MLP_MAX_HIDDEN + 2];
  const T* weight[DPAC_MLP_MAX_HIDDEN + 1];
  const T* bias;
};

template <typename T>
struct NnRolloutArgs {
  int64_t B;
  int N, cost_order;
  const T *x0, *dw;
  T *x, *dt, *coef, *u, *y, *disc, *save_z, *save_disc;
  int32_t* save_flag;
};

// One dense layer for the workgroup's 16 rows: out = act(BN(in @ W (+ b))).
// in/out are [16][kNnLd] LDS images; columns >= Nout of the last tile are
// written as 0 so the next layer's K padding reads zeros.  NT = this wave's
// 16-column tiles (wave, wave + 4, ...): a template constant, so the K loop is
// straight-line MFMA code with no per-tile predicate.
template <typename T, int NT>
__device__ __forceinline__ void nn_layer_tiles(const T* in, T* out, int K, int Nout, const T* W,
                                               const T* scale, const T* shift, const T* bias,
                                               bool hidden, int wave, int lane, T* save_row0,
                                               int64_t save_stride, int rows_live) {
  using MF = Mfma<T>;
  const int col_l = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (uint32_t)(K * Nout * (int)sizeof(T)));
  uint32_t voff[NT];
  typename MF::acc_t acc[NT];
  T s[NT], sh[NT], bb[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    const bool valid = col < Nout;
    voff[j] = valid ? (uint32_t)((kq * Nout + col) * (int)sizeof(T)) : kOOB;
    acc[j] = typename MF::acc_t{0, 0, 0, 0};
    s[j] = valid ? scale[col] : T(0);  // epilogue constants, loaded before the K loop
    sh[j] = valid ? shift[col] : T(0);
    bb[j] = (valid && bias) ? bias[col] : T(0);
  }
  const uint32_t kstep_bytes = (uint32_t)(4 * Nout * (int)sizeof(T));
  const int nks = (K + 3) / 4;
  const T* arow = in + col_l * kNnLd + kq;  // A[row = lane&15][k = 4ks + lane>>4]
  // B comes from L2 (~0.5-1k cycles): a kNnPrefetch-deep ring of k-steps keeps that
  // many loads per tile in flight.  Rows k >= K fall outside the descriptor and
  // read 0, so the ring needs no predicate; A past K is LDS zero padding.
  auto loadB = [&](int ks, int j) {
#if DPAC_NN_ABLATE == 1
    return T(1e-3) * T(j + 1) + T(ks & 1);  // timing only: no weight traffic
#endif
    uint32_t w[sizeof(T) / 4];
    buf_load_dwords<sizeof(T) / 4>(rW, voff[j] + (uint32_t)ks * kstep_bytes, w);
    T v;
    __builtin_memcpy(&v, &w[0], sizeof(T));
    return v;
  };
  // A (LDS) is read one ring iteration ahead too; k-steps past the last are
  // clamped to it (their B is 0, so the product adds nothing).
  auto loadA = [&](int ks) { return arow[4 * (ks < nks ? ks : nks - 1)]; };
  T bq[kNnPrefetch][NT], av[kNnPrefetch];
#pragma unroll
  for (int q = 0; q < kNnPrefetch; ++q) {
    av[q] = loadA(q);
#pragma unroll
    for (int j = 0; j < NT; ++j) bq[q][j] = loadB(q, j);
  }
  for (int ks0 = 0; ks0 < nks; ks0 += kNnPrefetch) {
    T an[kNnPrefetch];
#pragma unroll
    for (int q = 0; q < kNnPrefetch; ++q) an[q] = loadA(ks0 + kNnPrefetch + q);
#pragma unroll
    for (int q = 0; q < kNnPrefetch; ++q) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        acc[j] = MF::mma(av[q], bq[q][j], acc[j]);
        bq[q][j] = loadB(ks0 + q + kNnPrefetch, j);
      }
    }
#pragma unroll
    for (int q = 0; q < kNnPrefetch; ++q) av[q] = an[q];
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    const bool valid = col < Nout;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = MF::row(lane, i);
      const T z = acc[j][i];
      if (save_row0 && valid && row < rows_live) save_row0[row * save_stride + col] = z;
      T yv = bias ? z + bb[j] : z;            // addmm(b, y, W) (solver.py:270)
      yv = sh[j] + yv * s[j];                 // addcmul(beta, y, gamma/sqrt(1+eps))
      if (hidden) yv = yv + fmax(yv, T(0));   // y + relu(y) (solver.py:269)
      out[row * kNnLd + col] = valid ? yv : T(0);
    }
  }
}

template <typename T>
__device__ __forceinline__ void nn_layer(const T* in, T* out, int K, int Nout, const T* W,
                                         const T* scale, const T* shift, const T* bias,
                                         bool hidden, int wave, int lane, T* save_row0,
                                         int64_t save_stride, int rows_live) {
  const int ntiles = (Nout + 15) / 16;
  const int mine = ntiles > wave ? (ntiles - wave + kNnWaves - 1) / kNnWaves : 0;  // wave-uniform
  static_assert(kNnMaxTilesPerWave == 4, "dispatch below covers 1..4 tiles");
  switch (mine) {
    case 1: nn_layer_tiles<T, 1>(in, out, K, Nout, W, scale, shift, bias, hidden, wave, lane, save_row0, save_stride, rows_live); break;
    case 2: nn_layer_tiles<T, 2>(in, out, K, Nout, W, scale, shift, bias, hidden, wave, lane, save_row0, save_stride, rows_live); break;
    case 3: nn_layer_tiles<T, 3>(in, out, K, Nout, W, scale, shift, bias, hidden, wave, lane, save_row0, save_stride, rows_live); break;
    case 4: nn_layer_tiles<T, 4>(in, out, K, Nout, W, scale, shift, bias, hidden, wave, lane, save_row0, save_stride, rows_live); break;
    default: break;
  }
}

template <typename T, class E, int D, int SCHEME, bool COST, int KB>
__global__ __launch_bounds__(kNnThreads) void k_rollout_nn(const E eq, const DevConsts<T> c,
                                                          const NnMlp<T> mlp,
                                                          const NnRolloutArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  using TR = Transition<T, E, SCHEME>;
  __shared__ T s_x0[kNnRows * kNnLd];   // BN_0(x_t)
  __shared__ T s_pq[2][kNnRows * kNnLd];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int64_t row0 = (int64_t)blockIdx.x * kNnRows;
  const int rows_live = (int)((a.B - row0) < kNnRows ? (a.B - row0) : kNnRows);
  // step lanes: trajectory g = tid / P of the workgroup, slot p
  const bool stepper = tid < kNnRows * P;
  const int g = stepper ? tid / P : 0;
  const LaneCoord<P> lc(a.B, stepper ? tid % P : 0, row0 + g);
  const bool live = stepper && lc.live;
  const Own<D, P> own(lc.p);
  const Own<E::CDIM, P> ownu(lc.p);
  const BufSlab<T, D, P> sx(own, lc.b, live);
  const BufSlab<T, E::CDIM, P> su(ownu, lc.b, live);
  const uint32_t slab = (uint32_t)(a.B * D * sizeof(T));
  const uint32_t slab_u = (uint32_t)(a.B * E::CDIM * sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(a.x, slab * (uint32_t)(a.N + 1));
  const __amdgpu_buffer_rsrc_t rs_dw = make_rsrc(a.dw, slab * (uint32_t)a.N);
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(a.u, a.u ? slab_u * (uint32_t)a.N : 0u);
  const int L = mlp.L, c_out = mlp.width[L + 1];

  // zero padding: A columns past K (up to a prefetch ring beyond) read zeros
  for (int i = tid; i < kNnRows * kNnLd; i += kNnThreads) {
    s_x0[i] = T(0);
    s_pq[0][i] = T(0);
    s_pq[1][i] = T(0);
  }
  // BN_0 coefficients of the owned components
  T s0[M], b0[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int j = own.j(m);
    s0[m] = own.valid(m) ? mlp.scale[0][j] : T(0);
    b0[m] = own.valid(m) ? mlp.shift[0][j] : T(0);
  }
  auto write_a0 = [&](const T (&xv)[M]) {  // addcmul(beta0, x, gamma0/sqrt(1+eps)), solver.py:265
    if (stepper) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (own.valid(m)) s_x0[g * kNnLd + own.j(m)] = b0[m] + xv[m] * s0[m];
    }
  };

  T x[M];
  sx.load(make_rsrc(a.x0, slab), x);
  sx.store(rs_x, x);
  T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  Flags fl = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c) : Flags{true, false};
  T disc = 1, y = 0;
  __syncthreads();  // padding zeroed before the first a0 write
  write_a0(x);

  auto load = [&](int t, DwFrame<T, M>& fr) { sx.load(rs_dw, fr.dw, (uint32_t)t * slab); };
  auto body = [&](int t, DwFrame<T, M>& fr, auto) {
    __syncthreads();  // a0 of step t is in s_x0; the previous step's reads are done
    // ---- actor MLP on MFMA (all four wavefronts) ----
    const T* in = s_x0;
    int pq = 0;
    for (int l = 0; l <= (DPAC_NN_ABLATE == 2 ? -1 : L); ++l) {  // ablation 2: no MLP (timing)
      T* out = s_pq[pq];
      T* save = a.save_z ? a.save_z + ((int64_t)t * a.B + row0) * mlp.ztot + mlp.zoff[l + 1] : nullptr;
      nn_layer<T>(in, out, mlp.width[l], mlp.width[l + 1], mlp.weight[l], mlp.scale[l + 1],
                  mlp.shift[l + 1], l == L ? mlp.bias : nullptr, l < L, wave, lane, save, mlp.ztot,
                  rows_live);
      __syncthreads();
      in = out;
      pq ^= 1;
    }
    if (!stepper) return;
    // ---- u_t and the transition (step lanes) ----
    const T* yo = in + g * kNnLd;
    T u[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) u[m] = ownu.valid(m) ? yo[ownu.j(m)] : T(0);
    if (mlp.ekn) {  // y[:, :d] / (1e-15 + relu(y[:, d]) + |y[:, :d]|) (solver.py:272-274)
      const T nrm = dsqrt(Lanes<P>::sum(sumsq(u)));
      const T den = (T(1e-15) + fmax(yo[c_out - 1], T(0))) + nrm;
#pragma unroll
      for (int m = 0; m < MC; ++m) u[m] = u[m] / den;
    }
    if (a.save_flag && lc.p == 0 && live) {
      a.save_flag[(int64_t)t * a.B + lc.b] = fl.encode();
      a.save_disc[(int64_t)t * a.B + lc.b] = disc;
    }
    T dwv[M];
#pragma unroll
    for (int m = 0; m < M; ++m) dwv[m] = fr.dw[m];
    TR tr;
    tr.run(eq, c, x, u, dwv, fl, r);
    const T cf = tr.coef ? T(1) : T(0);
    if constexpr (COST) {
      const T w = eq.w_finish(Lanes<P>::sum(eq.w_part(x, u)));
      y += cost_increment(a.cost_order, w, cf, tr.dt, disc);
    }
    disc = disc * disc_factor(tr.dt, cf, c);  // also feeds save_disc
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = tr.coef ? tr.xt[m] : x[m];
    if constexpr (TR::kRadius) r = tr.coef ? tr.rt : r;
    fl = tr.next;
    sx.store(rs_x, x, (uint32_t)(t + 1) * slab);
    if (a.u) su.store(rs_u, u, (uint32_t)t * slab_u);
    if (lc.p == 0 && live) {
      a.dt[lc.b * a.N + t] = tr.dt;
      a.coef[lc.b * a.N + t] = cf;
    }
    write_a0(x);
  };
  pipelined<KB, DwFrame<T, M>>(0, a.N, load, body);
  if constexpr (COST) {
    if (live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}
