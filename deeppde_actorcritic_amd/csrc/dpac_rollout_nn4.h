// dpac_rollout_nn4.h — the fused NN-control rollout (dpac_rollout_nn.h) with
// 4-row MFMA blocks, for float: v_mfma_f32_4x4x1_16b_f32 computes a [4 x 1] x
// [1 x 64] product per instruction (16 blocks of 4x4, every block fed the same 4
// rows), so a workgroup can own as few as 4 trajectories and a batch of 2048
// spreads over every CU of the chip (the 16-row tiles of k_rollout_nn leave half
// of them idle at that size, and the per-step latency, not the MFMA rate, sets
// the time).  Same arithmetic per element as the 16x16x4 path; only the order
// of the K sums differs (split over the 8 wavefronts, combined in wave order).
//
// Workgroup = 8 wavefronts over ROWS = 4*RG trajectories.  Per dense layer
// [ROWS x K] x [K x H]:
//   * wavefront w takes the K slice [w*KW, (w+1)*KW) for ALL output columns;
//     per k it loads one B row segment (lane l: W[k][4l..4l+3], one 16-byte
//     load; the four columns go to four interleaved 64-column MFMA chunks) and
//     issues RG x 4 MFMAs; narrow layers (H <= 64, or H not a multiple of 4)
//     load W[k][64c + l] per 64-column chunk c instead;
//   * the 8 partial [ROWS x H] products meet in LDS, and all 512 threads run
//     the epilogue (sum in wave order, saves, BN, activation) on 4 columns each.
// Layer-to-layer and step-to-step state stays in LDS, as in k_rollout_nn.
#pragma once
// Included by dpac_kernels.h inside namespace dpac, after dpac_rollout_nn.h.

constexpr int kN4Waves = 8;
constexpr int kN4Threads = 64 * kN4Waves;
constexpr int kN4Ld = DPAC_MLP_MAX_WIDTH + 8;  // image row stride (>= 256 + PF)
constexpr int kN4Pw = DPAC_MLP_MAX_WIDTH;      // partial row stride
constexpr int kN4Prefetch = 8;                 // k-steps of B in flight per wavefront
typedef float n4v4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ n4v4 mfma4(float a, float b, n4v4 c) {
  return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// This wavefront's K slice of out[ROWS x H] = in[ROWS x K] @ W[K x H] into its
// partial rows part[wave][ROWS][kN4Pw] (columns >= H hold zeros).  VEC: lane l
// owns columns 4l..4l+3 (chunk e = column 4l+e); else lane l owns 64c + l.
template <int RG, int NC, bool VEC>
__device__ __forceinline__ void n4_layer_impl(const float* in, int K, int H, const float* W,
                                              int wave, int lane, float* part) {
  constexpr int ROWS = 4 * RG;
  constexpr int NB = VEC ? 4 : NC;               // B values (MFMA chunks) per k
  constexpr int SETS = RG * NB >= 4 ? 1 : 2;     // independent accumulator sets
  const int KW = (K + kN4Waves - 1) / kN4Waves;
  const int k0 = wave * KW;
  const int k1 = min(K, k0 + KW);
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (uint32_t)(K * H * 4));
  uint32_t boff[VEC ? 1 : NC];
  if constexpr (VEC) {
    boff[0] = 4 * lane < H ? (uint32_t)((k0 * H + 4 * lane) * 4) : kOOB;
  } else {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      boff[c] = 64 * c + lane < H ? (uint32_t)((k0 * H + 64 * c + lane) * 4) : kOOB;
  }
  const uint32_t kstride = (uint32_t)(H * 4);
  // rows past K read 0 through the descriptor; kOOB + q*kstride stays out of range
  auto loadB = [&](int q, float (&b)[NB]) {
    if constexpr (VEC) {
      uint32_t w[4];
      buf_load_dwords<4>(rW, boff[0] + (uint32_t)q * kstride, w);
      __builtin_memcpy(&b[0], &w[0], 16);
    } else {
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        uint32_t w[1];
        buf_load_dwords<1>(rW, boff[c] + (uint32_t)q * kstride, w);
        __builtin_memcpy(&b[c], &w[0], 4);
      }
    }
  };
  n4v4 acc[SETS][RG][NB];
#pragma unroll
  for (int s = 0; s < SETS; ++s)
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int e = 0; e < NB; ++e) acc[s][g][e] = n4v4{0, 0, 0, 0};
  const float* arow = in + (lane & 3) * kN4Ld;  // every 4x4 block takes rows 0..3
  float bq[kN4Prefetch][NB];
#pragma unroll
  for (int q = 0; q < kN4Prefetch; ++q) loadB(q, bq[q]);
  for (int q0 = 0; q0 < KW; q0 += kN4Prefetch) {
    float av[kN4Prefetch][RG];
#pragma unroll
    for (int q = 0; q < kN4Prefetch; ++q) {
      const int k = k0 + q0 + q;
#pragma unroll
      for (int g = 0; g < RG; ++g) av[q][g] = k < k1 ? arow[g * 4 * kN4Ld + k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kN4Prefetch; ++q) {
#pragma unroll
      for (int g = 0; g < RG; ++g)
#pragma unroll
        for (int e = 0; e < NB; ++e)
          acc[q % SETS][g][e] = mfma4(av[q][g], bq[q][e], acc[q % SETS][g][e]);
      loadB(q0 + q + kN4Prefetch, bq[q]);
    }
  }
  float* prow = part + wave * ROWS * kN4Pw;
#pragma unroll
  for (int g = 0; g < RG; ++g) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float v[NB];
#pragma unroll
      for (int e = 0; e < NB; ++e) {
        v[e] = acc[0][g][e][i];
        if constexpr (SETS == 2) v[e] += acc[1][g][e][i];
      }
      float* pr = prow + (4 * g + i) * kN4Pw;
      if constexpr (VEC) {
        *reinterpret_cast<n4v4*>(pr + 4 * lane) = n4v4{v[0], v[1], v[2], v[3]};
      } else {
#pragma unroll
        for (int c = 0; c < NC; ++c) pr[64 * c + lane] = v[c];
      }
    }
  }
}

template <int RG>
__device__ __forceinline__ void n4_layer(const float* in, int K, int H, const float* W, int wave,
                                         int lane, float* part) {
  if (H % 4 == 0 && H > 64) {
    n4_layer_impl<RG, 4, true>(in, K, H, W, wave, lane, part);
  } else {
    switch ((H + 63) / 64) {
      case 1: n4_layer_impl<RG, 1, false>(in, K, H, W, wave, lane, part); break;
      case 2: n4_layer_impl<RG, 2, false>(in, K, H, W, wave, lane, part); break;
      case 3: n4_layer_impl<RG, 3, false>(in, K, H, W, wave, lane, part); break;
      default: n4_layer_impl<RG, 4, false>(in, K, H, W, wave, lane, part); break;
    }
  }
}

// Sum the 8 partials of (row r, columns 4q..4q+3) in wave order and hand them
// to epi(r, c0, z[4]); every thread of the workgroup takes one (r, q) at a time.
template <int RG, class EPI>
__device__ __forceinline__ void n4_epilogue(const float* part, int H, int tid, EPI&& epi) {
  constexpr int ROWS = 4 * RG;
  const int nq = (H + 3) / 4;
  for (int e = tid; e < ROWS * 64; e += kN4Threads) {
    const int r = e / 64, q = e % 64;
    if (q >= nq) continue;
    n4v4 z = *reinterpret_cast<const n4v4*>(part + r * kN4Pw + 4 * q);
#pragma unroll
    for (int w = 1; w < kN4Waves; ++w)
      z += *reinterpret_cast<const n4v4*>(part + (w * ROWS + r) * kN4Pw + 4 * q);
    float zz[4] = {z[0], z[1], z[2], z[3]};
    epi(r, 4 * q, zz);
  }
}

template <typename T, class E, int D, int SCHEME, bool COST, int RG>
__global__ __launch_bounds__(kN4Threads) void k_rollout_nn4(const E eq, const DevConsts<T> c,
                                                           const NnMlp<T> mlp,
                                                           const NnRolloutArgs<T> a) {
  static_assert(std::is_same<T, float>::value, "4x4x1 MFMA path is float only");
  constexpr int P = E::kP, M = E::M, MC = E::MC, ROWS = 4 * RG;
  static_assert(ROWS * P <= kN4Threads, "step lanes fit the workgroup");
  using TR = Transition<T, E, SCHEME>;
  __shared__ __attribute__((aligned(16))) float s_x0[ROWS * kN4Ld];      // BN_0(x_t)
  __shared__ __attribute__((aligned(16))) float s_img[2][ROWS * kN4Ld];  // layer outputs
  __shared__ __attribute__((aligned(16))) float s_part[kN4Waves * ROWS * kN4Pw];
  __shared__ __attribute__((aligned(16))) float s_bn[DPAC_MLP_MAX_HIDDEN + 1][3][DPAC_MLP_MAX_WIDTH];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int64_t row0 = (int64_t)blockIdx.x * ROWS;
  const int rows_live = (int)((a.B - row0) < ROWS ? (a.B - row0) : ROWS);
  const bool stepper = tid < ROWS * P;
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
  // BN scale / shift of every dense layer's output (and the output bias) in LDS
  for (int l = 0; l <= L; ++l)
    for (int col = tid; col < mlp.width[l + 1]; col += kN4Threads) {
      s_bn[l][0][col] = mlp.scale[l + 1][col];
      s_bn[l][1][col] = mlp.shift[l + 1][col];
      s_bn[l][2][col] = l == L ? mlp.bias[col] : 0.f;
    }

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
        if (own.valid(m)) s_x0[g * kN4Ld + own.j(m)] = b0[m] + xv[m] * s0[m];
    }
  };

  T x[M];
  sx.load(make_rsrc(a.x0, slab), x);
  sx.store(rs_x, x);
  T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  Flags fl = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c) : Flags{true, false};
  T disc = 1, y = 0;
  write_a0(x);

  auto load = [&](int t, DwFrame<T, M>& fr) { sx.load(rs_dw, fr.dw, (uint32_t)t * slab); };
  auto body = [&](int t, DwFrame<T, M>& fr, auto) {
    __syncthreads();  // a0 of step t is in s_x0; the previous step's reads are done
    // ---- actor MLP (all eight wavefronts) ----
    const float* in = s_x0;
    int pq = 0;
    for (int l = 0; l <= L; ++l) {
      const int H = mlp.width[l + 1];
      n4_layer<RG>(in, mlp.width[l], H, mlp.weight[l], wave, lane, s_part);
      __syncthreads();
      float* out = s_img[pq];
      const float* sc = s_bn[l][0];
      const float* sh = s_bn[l][1];
      const float* bi = s_bn[l][2];
      const bool hidden = l < L;
      T* save = a.save_z ? a.save_z + ((int64_t)t * a.B + row0) * mlp.ztot + mlp.zoff[l + 1] : nullptr;
      n4_epilogue<RG>(s_part, H, tid, [&](int rr, int c0, const float (&z)[4]) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = c0 + j;
          if (col < H) {
            if (save && rr < rows_live) save[rr * mlp.ztot + col] = z[j];
            T yv = hidden ? z[j] : z[j] + bi[col];         // addmm(b, y, W) (solver.py:270)
            yv = sh[col] + yv * sc[col];                   // addcmul(beta, y, gamma/sqrt(1+eps))
            if (hidden) yv = yv + fmax(yv, T(0));          // y + relu(y) (solver.py:269)
            out[rr * kN4Ld + col] = yv;
          }
        }
      });
      __syncthreads();
      in = out;
      pq ^= 1;
    }
    if (!stepper) return;
    // ---- u_t and the transition (step lanes) ----
    const T* yo = in + g * kN4Ld;
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
  pipelined<1, DwFrame<T, M>>(0, a.N, load, body);
  if constexpr (COST) {
    if (live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}
