// dpac_rollout_nn.h — the rollout with the actor MLP as control, fused into one
// launch: equation.py:46-106 with NN_control
// (solver.py:260-278) evaluated inside the time loop.
//
// One workgroup (kNnWaves = 8 wavefronts) owns kNnRows = 16 trajectories for
// all N steps.  Per step:
//   1. the step lanes write a0 = BN_0(x_t) into LDS (solver.py:265);
//   2. every hidden layer is a [16 x K] x [K x H] product on 16x16x4 MFMA tiles
//      (f32 or f64 in, same-precision accumulate), the wavefronts splitting
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

#ifndef DPAC_NN_WAVES
#define DPAC_NN_WAVES 8  // 2 wavefronts per SIMD: measured 18.2 -> 15.4 us per step at lqr_d20
#endif
constexpr int kNnRows = 16;  // trajectories per workgroup = one MFMA row tile
constexpr int kNnWaves = DPAC_NN_WAVES;
constexpr int kNnThreads = 64 * kNnWaves;
#ifndef DPAC_NN_LD_PAD
#define DPAC_NN_LD_PAD 4  // LDS row stride = max width + pad (elements)
#endif
constexpr int kNnLd = DPAC_MLP_MAX_WIDTH + DPAC_NN_LD_PAD;  // LDS row stride (elements)
constexpr int kNnMaxTilesPerWave = (DPAC_MLP_MAX_WIDTH / 16 + kNnWaves - 1) / kNnWaves;
#ifndef DPAC_NN_PREFETCH
#define DPAC_NN_PREFETCH 4  // measured 14.9 -> 14.7 us per step (12, 16: slower)
#endif
constexpr int kNnPrefetch = DPAC_NN_PREFETCH;
#ifndef DPAC_NN_KM_PG
#define DPAC_NN_KM_PG 2  // k-major path: groups of 4 k-steps of B in flight per tile
#endif  // k-steps of B in flight per tile
#ifndef DPAC_NN_ABLATE
#define DPAC_NN_ABLATE 0  // timing-only builds: 1 = constant weights, 2 = skip the MLP
#endif
#ifndef DPAC_BWD_ABLATE
#define DPAC_BWD_ABLATE 0  // timing-only BPTT builds (bits): 1 = no z loads, 2 = no G stores,
                           // 4 = no step-lane loads, 8 = skip the MLP chain
#endif
// Timing-only builds (-DDPAC_NN_TRACE=1): lane 0 of every wavefront of workgroup 0
// records the shader clock at fixed points of the first 64 steps into a per-TU device
// table, read back by dpac_debug_trace (tools/probe_trace.py).
#ifndef DPAC_NN_TRACE
#define DPAC_NN_TRACE 0
#endif
#if DPAC_NN_TRACE
static __device__ uint32_t g_nn_trace[64 * 16 * 16];  // [step][wave][point]
#define NN_MARK(t, pt)                                                                   \
  do {                                                                                   \
    if (blockIdx.x == 0 && lane == 0 && (t) < 64)                                        \
      g_nn_trace[((t) * 16 + wave) * 16 + (pt)] = (uint32_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define NN_MARK(t, pt) \
  do {               \
  } while (0)
#endif
// The ring reads A up to k < 4 * roundup(ceil(K/4), kNnPrefetch) <= 256 for K <= 256.
static_assert(DPAC_MLP_MAX_WIDTH <= 256 && kNnLd >= 256, "A reads stay inside an LDS row");

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
  const T* wkm[DPAC_MLP_MAX_HIDDEN + 1];  // k-major images of weight (optional, float)
  const T* bias;
  int fast;  // the actor-shape fast path applies (nn_fast_host)
  const _Float16* wx3[DPAC_MLP_MAX_HIDDEN + 1];  // split-fp16 images of weight (k_rollout_nn_x3)
  uint32_t* status;  // the split-fp16 range guard (dpac.h dpac_mlp.status), or null
};

template <typename T>
struct NnRolloutArgs {
  int64_t B;
  int N, cost_order;
  const T *x0, *dw;
  T *x, *dt, *coef, *u, *y, *disc, *save_z, *save_disc;
  int32_t* save_flag;
  uint8_t* save_mask;   // optional (fast path only): the hidden activations' sign bits,
                        // [N][ceil(B/16)][mb] bytes (FwdEpiM's layout per 16-row tile)
  int mb;               // mask bytes per 16-row tile
  const uint32_t* guard;  // the f32 fallback of a split-fp16 launch: run only once this word
                          // is set (dpac.h dpac_mlp.status); null = always run
  int tr;               // k_rollout_nn_x3: trajectories per workgroup (16, or 8: half a row tile)
};

// out[16 x Nout] = in[16 x K] @ W[K x Nout] for the workgroup's 16 rows, this
// wave's NT 16-column tiles (wave, wave + 4, ...), followed by a per-element
// epilogue.  `in` is a [16][kNnLd] LDS image whose columns >= K are zero; W is
// row-major in global memory (L2-resident).  NT is a template constant, so the
// K loop is straight-line MFMA code with no per-tile predicate.
//   EPI::Col load(col, valid)                       per-column constants (before the K loop)
//   void store(i, row, col, valid, acc, const Col&) one output element (i: accumulator slot)
// The same product from a k-major weight image (float): Wkm[n][k] = W[k][n] for
// k < K, 0 for K <= k < K16 = roundup(K, 16), row stride K16 (dpac_mlp_prepare
// writes them).  One dwordx4 per lane and tile brings 4 consecutive k of one
// column, one ds_read_b128 the matching 4 A values, so a group of 4 MFMAs costs 2
// memory instructions instead of 8: the k of MFMA e of group s in lane quad kq is
// 16s + 4kq + e (a permutation of the K sum; every k once).  Columns K..K16-1 of
// the A image are zero or finite leftovers, times a zero B.  Measured 14.7 ->
// 13.3 us per step (B = 2048) and 58 -> 52 (B = 16384) at lqr_d20's actor shape.
template <int NT, class EPI>
__device__ __forceinline__ void mfma_rows16_km(const float* in, int K, int Nout, const float* Wkm,
                                               int wave, int lane, EPI& epi) {
  using MF = Mfma<float>;
  typedef float f4 __attribute__((ext_vector_type(4)));
  const int col_l = lane & 15, kq = lane >> 4;
  const int K16 = (K + 15) / 16 * 16, ng = K16 / 16;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
  uint32_t voff[NT];
  MF::acc_t acc[NT];
  typename EPI::Col cc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    const bool valid = col < Nout;
    voff[j] = valid ? (uint32_t)((col * K16 + 4 * kq) * 4) : kOOB;
    acc[j] = MF::acc_t{0, 0, 0, 0};
    cc[j] = epi.load(col, valid);  // issued before the K loop: its latency hides there
  }
  const float* arow = in + col_l * kNnLd + 4 * kq;  // 16-byte aligned: kNnLd % 4 == 0
  // groups past the last read 0 (kOOB); A reads are clamped to the last group
  auto loadB = [&](int s, int j) {
    uint32_t w[4];
    buf_load_dwords<4>(rW, s < ng ? voff[j] + (uint32_t)(s * 64) : kOOB, w);
    f4 v;
    __builtin_memcpy(&v, &w[0], 16);
    return v;
  };
  auto loadA = [&](int s) { return *reinterpret_cast<const f4*>(arow + 16 * (s < ng ? s : ng - 1)); };
  constexpr int PG = DPAC_NN_KM_PG;  // groups (4 k-steps each) of B in flight per tile
  f4 bq[PG][NT], av[PG];
#pragma unroll
  for (int q = 0; q < PG; ++q) {
    av[q] = loadA(q);
#pragma unroll
    for (int j = 0; j < NT; ++j) bq[q][j] = loadB(q, j);
  }
  for (int s0 = 0; s0 < ng; s0 += PG) {
    f4 an[PG];
#pragma unroll
    for (int q = 0; q < PG; ++q) an[q] = loadA(s0 + PG + q);
#pragma unroll
    for (int q = 0; q < PG; ++q) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[j] = MF::mma(av[q][e], bq[q][j][e], acc[j]);
        bq[q][j] = loadB(s0 + q + PG, j);
      }
    }
#pragma unroll
    for (int q = 0; q < PG; ++q) av[q] = an[q];
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int i = 0; i < 4; ++i) epi.store(i, MF::row(lane, i), col, col < Nout, acc[j][i], cc[j]);
  }
}

#ifndef DPAC_NN_KMS
#define DPAC_NN_KMS 1  // 1: static-K (fully unrolled) k-major layers for the specialised K16
#endif
#ifndef DPAC_NN_SAVE_NT
#define DPAC_NN_SAVE_NT 0
#endif
#ifndef DPAC_NN_PIN
#define DPAC_NN_PIN 1  // sched_barrier after each k group of the static-K layers
#endif
#ifndef DPAC_NN_KMS_PG
#define DPAC_NN_KMS_PG 2  // groups of B in flight per tile in the static-K layer (3, 4 measured slower)
#endif

// mfma_rows16_km with the group count NG = K16 / 16 a template constant: the K loop is
// straight-line code, so the A operand of every group is read from LDS up front (NG
// ds_read_b128, one wait), the B ring issues exactly the groups that exist (no
// past-the-end loads) and every wait is a counted vmcnt.  Same products, same order.
template <int NT, int NG, class EPI>
__device__ __forceinline__ void mfma_rows16_kms(const float* in, int Nout, const float* Wkm, int wave,
                                                int lane, EPI& epi) {
  using MF = Mfma<float>;
  typedef float f4 __attribute__((ext_vector_type(4)));
  constexpr int K16 = 16 * NG;
  constexpr int PG = DPAC_NN_KMS_PG < NG ? DPAC_NN_KMS_PG : NG;
  const int col_l = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
  uint32_t voff[NT];
  MF::acc_t acc[NT];
  typename EPI::Col cc[NT];
  auto loadB = [&](int s, int j) {
#if DPAC_NN_ABLATE == 1
    return f4{1e-3f * (j + 1), 1e-3f * s, 0.5f, -0.25f};  // timing only: no weight traffic
#endif
    uint32_t w[4];
    buf_load_dwords<4>(rW, voff[j] + (uint32_t)(s * 64), w);
    f4 v;
    __builtin_memcpy(&v, &w[0], 16);
    return v;
  };
  f4 b[PG][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    voff[j] = col < Nout ? (uint32_t)((col * K16 + 4 * kq) * 4) : kOOB;
    acc[j] = MF::acc_t{0, 0, 0, 0};
  }
#pragma unroll
  for (int q = 0; q < PG; ++q)
#pragma unroll
    for (int j = 0; j < NT; ++j) b[q][j] = loadB(q, j);
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    cc[j] = epi.load(col, col < Nout);
  }
  const float* arow = in + col_l * kNnLd + 4 * kq;  // 16-byte aligned: kNnLd % 4 == 0
  constexpr int AG = 4;  // A groups read ahead from LDS
  f4 a[AG];
#pragma unroll
  for (int s = 0; s < AG && s < NG; ++s) a[s] = *reinterpret_cast<const f4*>(arow + 16 * s);
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const f4 as = a[s % AG];
    if (s + AG < NG) a[s % AG] = *reinterpret_cast<const f4*>(arow + 16 * (s + AG));
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[j] = MF::mma(as[e], b[s % PG][j][e], acc[j]);
      if (s + PG < NG) b[s % PG][j] = loadB(s + PG, j);
    }
#if DPAC_NN_PIN
    __builtin_amdgcn_sched_barrier(0);  // keep the B ring's loads PG groups ahead (see kms_pre)
#endif
  }
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int i = 0; i < 4; ++i) epi.store(i, MF::row(lane, i), col, col < Nout, acc[j][i], cc[j]);
  }
}

template <typename T, int NT, class EPI>
__device__ __forceinline__ void mfma_rows16(const T* in, int K, int Nout, const T* W, const T* Wkm,
                                            int wave, int lane, EPI& epi) {
  if constexpr (sizeof(T) == 4) {
    if (Wkm) {  // block-uniform
#if DPAC_NN_KMS
      // the actor shapes' K16 (d = 20 -> 32; hidden 200 -> 208) as straight-line layers
      const int ng = (K + 15) / 16;
      if (ng == 2) { mfma_rows16_kms<NT, 2>(in, Nout, Wkm, wave, lane, epi); return; }
      if (ng == 13) { mfma_rows16_kms<NT, 13>(in, Nout, Wkm, wave, lane, epi); return; }
#endif
      mfma_rows16_km<NT>(in, K, Nout, Wkm, wave, lane, epi);
      return;
    }
  }
  using MF = Mfma<T>;
  const int col_l = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (uint32_t)(K * Nout * (int)sizeof(T)));
  uint32_t voff[NT];
  typename MF::acc_t acc[NT];
  typename EPI::Col cc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    const bool valid = col < Nout;
    voff[j] = valid ? (uint32_t)((kq * Nout + col) * (int)sizeof(T)) : kOOB;
    acc[j] = typename MF::acc_t{0, 0, 0, 0};
    cc[j] = epi.load(col, valid);  // issued before the K loop: its latency hides there
  }
  const uint32_t kstep_bytes = (uint32_t)(4 * Nout * (int)sizeof(T));
  const int nks = (K + 3) / 4;
  const T* arow = in + col_l * kNnLd + kq;  // A[row = lane&15][k = 4ks + lane>>4]
  // B comes from L2 (~0.5-1k cycles): a kNnPrefetch-deep ring of k-steps keeps that
  // many loads per tile in flight.  Rows k >= K fall outside the descriptor and
  // read 0, so the ring needs no predicate.  A is read one ring iteration ahead;
  // k-steps past the last are clamped to it (their B is 0, the product adds nothing).
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
#pragma unroll
    for (int i = 0; i < 4; ++i) epi.store(i, MF::row(lane, i), col, col < Nout, acc[j][i], cc[j]);
  }
}

#ifndef DPAC_NN_SPLITK
#define DPAC_NN_SPLITK 1  // narrow layers (Nout <= 32) split K over all wavefronts
#endif

// A narrow layer (Nout <= 32, i.e. NT <= 2 column tiles) as a split-K product: a
// column split would leave all but NT wavefronts idle through a K/4-long
// dependent MFMA chain (50 x 40 cycles at K = 200).  Wavefront w multiplies the
// K slice [32w, 32w + 32) for every column tile (8 k-steps: K <= 256; rows past
// K read 0 through the descriptor, A columns past K are the zero padding), its
// partial [16 x 32] goes to LDS (`part`, which the layer's output image may
// serve as: nothing reads it during this layer), and each of the 512 threads
// sums one output element over the wavefronts in wave order and runs the
// epilogue on it.
template <typename T, int NT, class EPI>
__device__ __forceinline__ void mfma_rows16_splitk(const T* in, int K, int Nout, const T* W,
                                                   const T* Wkm, int wave, int lane, EPI& epi,
                                                   T* part) {
  static_assert(kNnWaves == 8 && NT <= 2, "16 rows x 32 columns = one element per thread");
  using MF = Mfma<T>;
  constexpr int KS = 8;
  const int col_l = lane & 15, kq = lane >> 4;
  // this thread's output element and its epilogue constants (latency hidden below)
  const int tid = wave * 64 + lane, erow = tid >> 5, ecol = tid & 31;
  const bool evalid = ecol < Nout;
  const typename EPI::ColE ce = epi.loadE(erow, ecol, evalid);
  typename MF::acc_t acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = typename MF::acc_t{0, 0, 0, 0};
  bool done = false;
  if constexpr (sizeof(T) == 4) {
    if (Wkm) {  // block-uniform: the slice as 2 groups of 16 k from the k-major image
      typedef float f4 __attribute__((ext_vector_type(4)));
      const int K16 = (K + 15) / 16 * 16;
      const __amdgpu_buffer_rsrc_t rK = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
      f4 bk[2][NT], ak[2];
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int kb = wave * 32 + 16 * g;  // group base; groups at or past K16 read 0
        ak[g] = kb < K16 ? *reinterpret_cast<const f4*>(in + col_l * kNnLd + kb + 4 * kq)
                         : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int j = 0; j < NT; ++j) {
          const int col = j * 16 + col_l;
          const uint32_t off = (col < Nout && kb < K16) ? (uint32_t)((col * K16 + kb + 4 * kq) * 4) : kOOB;
          uint32_t w[4];
          buf_load_dwords<4>(rK, off, w);
          __builtin_memcpy(&bk[g][j], &w[0], 16);
        }
      }
#pragma unroll
      for (int g = 0; g < 2; ++g)
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[j] = MF::mma(ak[g][e], bk[g][j][e], acc[j]);
      done = true;
    }
  }
  if (!done) {
    const __amdgpu_buffer_rsrc_t rW = make_rsrc(W, (uint32_t)(K * Nout * (int)sizeof(T)));
    T b[KS][NT], av[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int k = (wave * KS + ks) * 4 + kq;
      av[ks] = k < K ? in[col_l * kNnLd + k] : T(0);  // the image past K may hold a wider layer's data
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int col = j * 16 + col_l;
        const uint32_t off = col < Nout ? (uint32_t)((k * Nout + col) * (int)sizeof(T)) : kOOB;
        uint32_t w[sizeof(T) / 4];
        buf_load_dwords<sizeof(T) / 4>(rW, off, w);
        __builtin_memcpy(&b[ks][j], &w[0], sizeof(T));
      }
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j] = MF::mma(av[ks], b[ks][j], acc[j]);
  }
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) part[(wave * 16 + MF::row(lane, i)) * 32 + j * 16 + col_l] = acc[j][i];
  __syncthreads();
  T v = part[erow * 32 + ecol];
#pragma unroll
  for (int w = 1; w < kNnWaves; ++w) v += part[(w * 16 + erow) * 32 + ecol];
  __syncthreads();  // every partial read before the epilogue overwrites `part`
  if (ecol < NT * 16) epi.storeE(erow, ecol, evalid, v, ce);
}

// Whether mfma_layer runs the layer as the split-K product (two internal barriers).
__device__ __forceinline__ bool nn_splitk_layer(int K, int Nout) {
  return DPAC_NN_SPLITK && kNnWaves == 8 && Nout <= 32 && K > 32;
}

// Run mfma_rows16 with this wave's (wave-uniform) tile count.
template <typename T, class EPI>
__device__ __forceinline__ void mfma_layer(const T* in, int K, int Nout, const T* W, const T* Wkm,
                                           int wave, int lane, EPI& epi) {
#if DPAC_NN_SPLITK
  if constexpr (kNnWaves == 8) {
    static_assert(8 * 16 * 32 <= kNnRows * kNnLd, "partials fit the output image");
    if (Nout <= 32 && K > 32) {  // block-uniform
      if (Nout <= 16) mfma_rows16_splitk<T, 1>(in, K, Nout, W, Wkm, wave, lane, epi, epi.out);
      else mfma_rows16_splitk<T, 2>(in, K, Nout, W, Wkm, wave, lane, epi, epi.out);
      return;
    }
  }
#endif
  const int ntiles = (Nout + 15) / 16;
  const int mine = ntiles > wave ? (ntiles - wave + kNnWaves - 1) / kNnWaves : 0;
  static_assert(kNnMaxTilesPerWave <= 4, "dispatch below covers 1..4 tiles");
  switch (mine) {
    case 1: mfma_rows16<T, 1>(in, K, Nout, W, Wkm, wave, lane, epi); break;
    case 2: mfma_rows16<T, 2>(in, K, Nout, W, Wkm, wave, lane, epi); break;
    case 3: mfma_rows16<T, 3>(in, K, Nout, W, Wkm, wave, lane, epi); break;
    case 4: mfma_rows16<T, 4>(in, K, Nout, W, Wkm, wave, lane, epi); break;
    default: break;
  }
}

// ---------------------------------------------------------------------------
// Actor-shape fast path (float, k-major weight images): the BASELINE actors are
// d -> 200 -> 200 -> 200 -> c with d, c <= 32.  The clock trace of one step
// (profiles/r02_nn_phase_trace_base.json, B = 2048) shows the two narrow layers —
// 0.4 us of MFMA work each — taking 1.5-1.8 us of wall time, and every layer
// starting with an L2 round trip for its first weights.  So:
//  * the narrow layers' B fragments stay in VGPRs for the whole launch: the
//    narrow-K layer (K16 <= 32, e.g. 20 -> 200) as NG groups of this wave's NT <= 2
//    tiles, the narrow-output split-K layer (e.g. 200 -> 20) as this wave's two
//    16-k groups of its K slice — 16 VGPRs each;
//  * a wide layer's first PG groups of weights are loaded before the barrier that
//    precedes it (weights do not depend on the activations), into 16 VGPRs.
// The products are the same, in the same order, as mfma_layer's: bitwise equal.
// ---------------------------------------------------------------------------
typedef float nnf4 __attribute__((ext_vector_type(4)));

struct NarrowIn {   // B of a K16 <= 32 layer: [group s][tile j], tiles j >= mine read 0
  nnf4 b[2][2];
};
struct NarrowOut {  // B of the split-K layer: [group g of the wave's K slice][tile j]
  nnf4 b[2][2];
};
struct WidePre {    // the first DPAC_NN_KMS_PG groups of a wide layer's B
  nnf4 b[DPAC_NN_KMS_PG][2];
};

__device__ __forceinline__ nnf4 nn_load_f4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  uint32_t w[4];
  buf_load_dwords<4>(r, off, w);
  nnf4 v;
  __builtin_memcpy(&v, &w[0], 16);
  return v;
}

// this wave's tile count of an Nout-wide column split
__device__ __forceinline__ int nn_mine(int Nout, int wave) {
  const int ntiles = (Nout + 15) / 16;
  return ntiles > wave ? (ntiles - wave + kNnWaves - 1) / kNnWaves : 0;
}

__device__ __forceinline__ void load_narrow_in(NarrowIn& r, const float* Wkm, int K, int Nout, int wave,
                                               int lane) {
  const int col_l = lane & 15, kq = lane >> 4;
  const int K16 = (K + 15) / 16 * 16;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int s = 0; s < 2; ++s)
      r.b[s][j] = nn_load_f4(rW, (col < Nout && 16 * s < K16) ? (uint32_t)((col * K16 + 4 * kq + 16 * s) * 4) : kOOB);
  }
}

__device__ __forceinline__ void load_narrow_out(NarrowOut& r, const float* Wkm, int K, int Nout, int wave,
                                                int lane) {
  const int col_l = lane & 15, kq = lane >> 4;
  const int K16 = (K + 15) / 16 * 16;
  const __amdgpu_buffer_rsrc_t rK = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int kb = wave * 32 + 16 * g;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = j * 16 + col_l;
      r.b[g][j] = nn_load_f4(rK, (col < Nout && kb < K16) ? (uint32_t)((col * K16 + kb + 4 * kq) * 4) : kOOB);
    }
  }
}

// the first PG groups of the wide layer (K, Nout) this wave will multiply
__device__ __forceinline__ void load_wide_pre(WidePre& r, const float* Wkm, int K, int Nout, int wave, int lane) {
  const int col_l = lane & 15, kq = lane >> 4;
  const int K16 = (K + 15) / 16 * 16;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int q = 0; q < DPAC_NN_KMS_PG; ++q)
      r.b[q][j] = nn_load_f4(rW, col < Nout ? (uint32_t)((col * K16 + 4 * kq + 16 * q) * 4) : kOOB);
  }
}

// mfma_rows16_kms<NT, NG> for NG <= 2 with B from registers (no weight loads)
struct NoMark {
  __device__ __forceinline__ void operator()(int) const {}
};

template <int NT, int NG, class EPI, class MK = NoMark>
__device__ __forceinline__ void mfma_rows16_res(const float* in, int Nout, const NarrowIn& r, int wave, int lane,
                                                EPI& epi, MK mk = MK{}) {
  using MF = Mfma<float>;
  const int col_l = lane & 15, kq = lane >> 4;
  MF::acc_t acc[NT];
  typename EPI::Col cc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    acc[j] = MF::acc_t{0, 0, 0, 0};
    cc[j] = epi.load(col, col < Nout);
  }
  const float* arow = in + col_l * kNnLd + 4 * kq;
  nnf4 a[NG];
#pragma unroll
  for (int s = 0; s < NG; ++s) a[s] = *reinterpret_cast<const nnf4*>(arow + 16 * s);
#if DPAC_NN_TRACE
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  mk(10);  // A in registers
#endif
#pragma unroll
  for (int s = 0; s < NG; ++s)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[j] = MF::mma(a[s][e], r.b[s][j][e], acc[j]);
#if DPAC_NN_TRACE
  asm volatile("" ::"v"(acc[NT - 1][3]));
  mk(11);  // products done
#endif
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int i = 0; i < 4; ++i) epi.store(i, MF::row(lane, i), col, col < Nout, acc[j][i], cc[j]);
  }
}

#ifndef DPAC_NN_PRE_EARLY
#define DPAC_NN_PRE_EARLY 1  // 0: the next layer's prefetch after the epilogue (timing knob)
#endif
struct NoNext {
  __device__ __forceinline__ void operator()() const {}
};

// mfma_rows16_kms<NT, NG> with its first PG groups of B already in registers; nx() runs
// between the products and the epilogue (the next layer's weight prefetch: issued there,
// its loads are not queued behind this epilogue's z / mask stores in vmcnt order)
template <int NT, int NG, class EPI, class NX = NoNext>
__device__ __forceinline__ void mfma_rows16_kms_pre(const float* in, int Nout, const float* Wkm, const WidePre& pre,
                                                    int wave, int lane, EPI& epi, NX nx = NX{}) {
  using MF = Mfma<float>;
  constexpr int K16 = 16 * NG;
  constexpr int PG = DPAC_NN_KMS_PG < NG ? DPAC_NN_KMS_PG : NG;
  static_assert(PG == DPAC_NN_KMS_PG, "the prefetch holds PG groups");
  const int col_l = lane & 15, kq = lane >> 4;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wkm, (uint32_t)(Nout * K16 * 4));
  uint32_t voff[NT];
  MF::acc_t acc[NT];
  typename EPI::Col cc[NT];
  nnf4 b[PG][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
    voff[j] = col < Nout ? (uint32_t)((col * K16 + 4 * kq) * 4) : kOOB;
    acc[j] = MF::acc_t{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < PG; ++q) b[q][j] = pre.b[q][j];
    cc[j] = epi.load(col, col < Nout);
  }
  // A from LDS through a ring of AG groups (not all NG up front: 36 fewer VGPRs, which
  // the 10-wavefront BPTT workgroup, capped at 168, needs for the resident narrow layers)
  constexpr int AG = 4;
  const float* arow = in + col_l * kNnLd + 4 * kq;
  nnf4 a[AG];
#pragma unroll
  for (int s = 0; s < AG && s < NG; ++s) a[s] = *reinterpret_cast<const nnf4*>(arow + 16 * s);
#pragma unroll
  for (int s = 0; s < NG; ++s) {
    const nnf4 as = a[s % AG];
    if (s + AG < NG) a[s % AG] = *reinterpret_cast<const nnf4*>(arow + 16 * (s + AG));
#pragma unroll
    for (int j = 0; j < NT; ++j) {
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[j] = MF::mma(as[e], b[s % PG][j][e], acc[j]);
      if (s + PG < NG) b[s % PG][j] = nn_load_f4(rW, voff[j] + (uint32_t)((s + PG) * 64));
    }
    // pin the ring: without this the scheduler sinks each load next to its first use
    // (one load in flight, the L2 latency exposed every 4 MFMAs)
    __builtin_amdgcn_sched_barrier(0);
  }
#if DPAC_NN_PRE_EARLY
  nx();
#endif
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int col = (wave + kNnWaves * j) * 16 + col_l;
#pragma unroll
    for (int i = 0; i < 4; ++i) epi.store(i, MF::row(lane, i), col, col < Nout, acc[j][i], cc[j]);
  }
#if !DPAC_NN_PRE_EARLY
  nx();
#endif
}

// mfma_rows16_splitk's k-major branch with the wave's slice of B in registers
template <int NT, class EPI>
__device__ __forceinline__ void mfma_rows16_splitk_res(const float* in, int K, int Nout, const NarrowOut& r,
                                                       int wave, int lane, EPI& epi, float* part) {
  using MF = Mfma<float>;
  const int col_l = lane & 15, kq = lane >> 4;
  const int tid = wave * 64 + lane, erow = tid >> 5, ecol = tid & 31;
  const bool evalid = ecol < Nout;
  const typename EPI::ColE ce = epi.loadE(erow, ecol, evalid);
  const int K16 = (K + 15) / 16 * 16;
  MF::acc_t acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = MF::acc_t{0, 0, 0, 0};
  nnf4 ak[2];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
    const int kb = wave * 32 + 16 * g;
    ak[g] = kb < K16 ? *reinterpret_cast<const nnf4*>(in + col_l * kNnLd + kb + 4 * kq) : nnf4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) acc[j] = MF::mma(ak[g][e], r.b[g][j][e], acc[j]);
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) part[(wave * 16 + MF::row(lane, i)) * 32 + j * 16 + col_l] = acc[j][i];
  __syncthreads();
  float v = part[erow * 32 + ecol];
#pragma unroll
  for (int w = 1; w < kNnWaves; ++w) v += part[(w * 16 + erow) * 32 + ecol];
  __syncthreads();
  if (ecol < NT * 16) epi.storeE(erow, ecol, evalid, v, ce);
}

// Whether a network takes the fast path (host side, per launch): float k-major images, a
// narrow first product (K16 <= 32), hidden layers of 13 column tiles (193..208 wide), a
// split-K last product.  `kin` / `kout`: the widths entering the first / leaving the last
// product in the kernel's layer order (forward: width[0] / width[L+1]; BPTT: reversed).
// DPAC_NN_FAST=0 forces the generic path (tests compare the two bit for bit).
template <typename T>
inline bool nn_fast_host(int L, const int* width, const void* const* km, int kin, int kout) {
  if (!std::is_same<T, float>::value || L < 1 || kin > 32 || kout > 32 || kNnWaves != 8 || !DPAC_NN_SPLITK)
    return false;
  const char* e = getenv("DPAC_NN_FAST");  // read per launch
  if (e && e[0] == '0') return false;
  for (int i = 1; i <= L; ++i)
    if ((width[i] + 15) / 16 != 13) return false;
  for (int i = 0; i <= L; ++i)
    if (!km[i]) return false;
  return true;
}

// the narrow-K product with resident B: this wave's tile count, NG in {1, 2}
template <class EPI, class MK = NoMark>
__device__ __forceinline__ void nn_layer_narrow_in(const float* in, int K, int Nout, const NarrowIn& r, int wave,
                                                   int lane, EPI& epi, MK mk = MK{}) {
  const int mine = nn_mine(Nout, wave);
  if (K <= 16) {
    if (mine == 1) mfma_rows16_res<1, 1>(in, Nout, r, wave, lane, epi, mk);
    else if (mine == 2) mfma_rows16_res<2, 1>(in, Nout, r, wave, lane, epi, mk);
  } else {
    if (mine == 1) mfma_rows16_res<1, 2>(in, Nout, r, wave, lane, epi, mk);
    else if (mine == 2) mfma_rows16_res<2, 2>(in, Nout, r, wave, lane, epi, mk);
  }
}

template <class EPI, class NX = NoNext>
__device__ __forceinline__ void nn_layer_wide(const float* in, int Nout, const float* Wkm, const WidePre& pre,
                                              int wave, int lane, EPI& epi, NX nx = NX{}) {
  const int mine = nn_mine(Nout, wave);
  if (mine == 1) mfma_rows16_kms_pre<1, 13>(in, Nout, Wkm, pre, wave, lane, epi, nx);
  else if (mine == 2) mfma_rows16_kms_pre<2, 13>(in, Nout, Wkm, pre, wave, lane, epi, nx);
}

template <class EPI>
__device__ __forceinline__ void nn_layer_narrow_out(const float* in, int K, int Nout, const NarrowOut& r, int wave,
                                                    int lane, EPI& epi) {
  if (Nout <= 16) mfma_rows16_splitk_res<1>(in, K, Nout, r, wave, lane, epi, epi.out);
  else mfma_rows16_splitk_res<2>(in, K, Nout, r, wave, lane, epi, epi.out);
}

// Forward epilogue of a dense layer: z -> (save z) -> BN(z (+ b)) -> [y + relu(y)]
// into the next layer's LDS input.  Padding columns are written as 0.
template <typename T>
struct FwdEpi {
  struct Col {
    T s, sh, bb;
  };
  const T *scale, *shift, *bias;
  bool hidden;
  T* out;          // LDS [16][kNnLd]
  T* save;         // global row block of this layer's z, or null
  int64_t save_stride;
  int rows_live;
  __device__ __forceinline__ Col load(int col, bool valid) const {
    return Col{valid ? scale[col] : T(0), valid ? shift[col] : T(0),
               (valid && bias) ? bias[col] : T(0)};
  }
  // one element (split-K epilogue): the same constants and arithmetic
  using ColE = Col;
  __device__ __forceinline__ ColE loadE(int, int col, bool valid) const { return load(col, valid); }
  __device__ __forceinline__ void storeE(int row, int col, bool valid, T z, const ColE& k) const {
    store(0, row, col, valid, z, k);
  }
  __device__ __forceinline__ void store(int, int row, int col, bool valid, T z, const Col& k) const {
#if DPAC_NN_SAVE_NT  // timing knob: non-temporal z saves
    if (save && valid && row < rows_live) __builtin_nontemporal_store(z, save + row * save_stride + col);
#else
    if (save && valid && row < rows_live) save[row * save_stride + col] = z;
#endif
    T yv = bias ? z + k.bb : z;          // addmm(b, y, W) (solver.py:270)
    yv = k.sh + yv * k.s;                // addcmul(beta, y, gamma/sqrt(1+eps))
    if (hidden) yv = yv + fmax(yv, T(0));  // y + relu(y) (solver.py:269)
    out[row * kNnLd + col] = valid ? yv : T(0);
  }
};

// FwdEpi that also records the sign of every hidden BN output (the only thing the BPTT
// needs of z: the activation factor 1 + [y > 0]) in the accumulator's own layout: per
// 16-row tile, hidden layer l, column c, row r: bit r % 4 of byte [13 l + c / 16][16 (r / 4)
// + c % 16] (a 16x16 accumulator keeps a lane's four slots in one row quad and column, so
// the byte is the lane's).  Each lane ORs its four slots' comparisons into one byte; a
// 64-byte coalesced store per column tile, no cross-lane step.
template <typename T>
struct FwdEpiM : FwdEpi<T> {
  uint8_t* mask;  // this step's mask tile of the workgroup's rows at this layer's offset
  uint32_t nib;   // the four slots' bits of the current column tile
  __device__ __forceinline__ void store(int i, int row, int col, bool valid, T z, const typename FwdEpi<T>::Col& k) {
    if (this->save && valid && row < this->rows_live) this->save[row * this->save_stride + col] = z;
    T yv = this->bias ? z + k.bb : z;
    yv = k.sh + yv * k.s;
    // the forward's own comparison, so the BPTT's activation factor is bitwise the z-based one
    nib = (i == 0 ? 0u : nib) | ((valid && yv > T(0)) ? 1u << i : 0u);
    yv = yv + fmax(yv, T(0));  // hidden layers only
    this->out[row * kNnLd + col] = valid ? yv : T(0);
    // dead rows' bits are written too and never read
    if (i == 3) mask[(col >> 4) * 64 + 16 * (row >> 2) + (col & 15)] = (uint8_t)nib;
  }
};

// Backward epilogue of a dense layer's input-gradient product g = G_{l+1} @ (W_l diag s_{l+1})^T:
// for l >= 1 multiply by the activation factor 1 + [y_l > 0] of the forward step
// (y_l = BN_l(z_l), z_l saved by the forward), then store the gradient entering
// BN_l's output to global (the parameter gradients use it) and to LDS (the next
// product's A).  l == 0 (no factor): the gradient entering a_0 = BN_0(x).
template <typename T>
struct BwdEpi {
  struct Col {
    T s, sh, z[4];
  };
  const T *scale, *shift;  // BN_l, or null for l == 0
  const T* z;              // z_l of row 0 of the workgroup at this step
  int64_t z_stride;
  int rows_live, lane;
  T* out;                  // LDS [16][kNnLd]
  T* g;                    // G_l of row 0 of the workgroup at this step
  int64_t g_stride;
  __device__ __forceinline__ Col load(int col, bool valid) const {
    Col k{};
    if (scale) {
      k.s = valid ? scale[col] : T(0);
      k.sh = valid ? shift[col] : T(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = Mfma<T>::row(lane, i);
#if DPAC_BWD_ABLATE & 1
        k.z[i] = T(row - col);
#else
        k.z[i] = (valid && row < rows_live) ? z[row * z_stride + col] : T(0);
#endif
      }
    }
    return k;
  }
  struct ColE {
    T s, sh, z;
  };
  __device__ __forceinline__ ColE loadE(int row, int col, bool valid) const {
    ColE k{};
    if (scale) {
      k.s = valid ? scale[col] : T(0);
      k.sh = valid ? shift[col] : T(0);
      k.z = (valid && row < rows_live) ? z[row * z_stride + col] : T(0);
    }
    return k;
  }
  __device__ __forceinline__ void storeE(int row, int col, bool valid, T acc, const ColE& k) const {
    T v = acc;
    if (scale) {
      const T yv = k.sh + k.z * k.s;
      v = acc * (yv > T(0) ? T(2) : T(1));
    }
#if !(DPAC_BWD_ABLATE & 2)
    if (valid && row < rows_live) g[row * g_stride + col] = v;
#endif
    out[row * kNnLd + col] = valid ? v : T(0);
  }
  __device__ __forceinline__ void store(int i, int row, int col, bool valid, T acc, const Col& k) const {
    T v = acc;
    if (scale) {
      const T yv = k.sh + k.z[i] * k.s;  // the forward's BN_l output, same expression
      v = acc * (yv > T(0) ? T(2) : T(1));  // d(y + relu(y))/dy
    }
#if !(DPAC_BWD_ABLATE & 2)
    if (valid && row < rows_live) g[row * g_stride + col] = v;
#endif
    out[row * kNnLd + col] = valid ? v : T(0);
  }
};

template <typename T>
struct NnBackArgs {
  int64_t B;
  int N;
  const T *x, *u, *dw, *disc_t, *z;
  const int32_t* flag;
  const T *g_xN, *g_disc, *g_y;
  T *G, *g_x0;
  const T* wt[DPAC_MLP_MAX_HIDDEN + 1];  // (W_i diag s_{i+1})^T, [width[i+1]][width[i]]
  const T* wtkm[DPAC_MLP_MAX_HIDDEN + 1];  // their k-major images (optional, float)
  int goff[DPAC_MLP_MAX_HIDDEN + 2];     // column offset of G_i in a G row
  int gtot;
  int fast;  // the actor-shape fast path applies to the transposed chain (nn_fast_host)
  const uint8_t* mask;  // optional (fast path): the forward's sign bits, [N][ceil(B/16)][mb]
  int mb;
  const _Float16* wtx3[DPAC_MLP_MAX_HIDDEN + 1];  // split-fp16 images of wt (k_rollout_nn_bwd_x3)
  const uint32_t* guard;  // as NnRolloutArgs::guard
  int tr;                 // as NnRolloutArgs::tr (k_rollout_nn_bwd_x3)
};

// The actor's BPTT through a fused NN rollout, as one launch: the reverse time
// loop of step_vjp (the adjoint of the transition and the running cost) and the
// MLP's input-gradient chain on MFMA, writing the gradient entering every BN
// output of every step (G) for the parameter gradients.  Same workgroup layout
// as k_rollout_nn.
template <typename T, class E, int D, int SCHEME>
__global__ __launch_bounds__(kNnThreads) void k_rollout_nn_bwd(const E eq, const DevConsts<T> c,
                                                              const NnMlp<T> mlp,
                                                              const NnBackArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC, CD = E::CDIM;
  __shared__ T s_pq[2][kNnRows * kNnLd];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int64_t row0 = (int64_t)blockIdx.x * kNnRows;
  const int rows_live = (int)((a.B - row0) < kNnRows ? (a.B - row0) : kNnRows);
  const bool stepper = tid < kNnRows * P;
  const int g = stepper ? tid / P : 0;
  const LaneCoord<P> lc(a.B, stepper ? tid % P : 0, row0 + g);
  const bool live = stepper && lc.live;
  const Own<D, P> own(lc.p);
  const Own<CD, P> ownu(lc.p);
  const int L = mlp.L;
  for (int i = tid; i < kNnRows * kNnLd; i += kNnThreads) {
    s_pq[0][i] = T(0);
    s_pq[1][i] = T(0);
  }
  T s0[M], lam[M], gxd[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    s0[m] = own.valid(m) ? mlp.scale[0][own.j(m)] : T(0);
    lam[m] = T(0);
    gxd[m] = T(0);
  }
  if (a.g_xN) own.load_masked(a.g_xN + lc.b * D, lam);
  T gD = a.g_disc ? a.g_disc[lc.b] : T(0);
  const T gy = a.g_y ? a.g_y[lc.b] : T(0);
  const T* sL = mlp.scale[L + 1];
  const T* shL = mlp.shift[L + 1];
  __syncthreads();
  for (int t = a.N - 1; t >= 0; --t) {
    const int64_t rowt = (int64_t)t * a.B;
    if (stepper) {
      T x[M], u[MC], dwv[M], gu[MC], gdn;
#if DPAC_BWD_ABLATE & 4
#pragma unroll
      for (int m = 0; m < M; ++m) x[m] = dwv[m] = T(0.01) * T(m + t);
#pragma unroll
      for (int m = 0; m < MC; ++m) u[m] = T(0.02) * T(m - t);
      const Flags fl = Flags::decode(2 - (t & 1));
      const T dsc = T(1);
#else
      own.load_masked(a.x + (rowt + lc.b) * D, x);
      own.load_masked(a.dw + (rowt + lc.b) * D, dwv);
      ownu.load_masked(a.u + (rowt + lc.b) * CD, u);
      const Flags fl = Flags::decode(a.flag[rowt + lc.b]);
      const T dsc = a.disc_t[rowt + lc.b];
#endif
      step_vjp<T, E, SCHEME>(eq, c, x, u, dwv, fl, dsc, lam, gD, gy, gxd, gu, gdn);
      gD = gdn;
      // gradient at the network output, through the Eikonal head (solver.py:272-274)
      T* grow = a.G + (rowt + lc.b) * a.gtot + a.goff[L + 1];
      T* lrow = s_pq[0] + g * kNnLd;
      if (mlp.ekn) {
        const T* zr = a.z + (rowt + lc.b) * mlp.ztot + mlp.zoff[L + 1];
        T o[MC];
#pragma unroll
        for (int m = 0; m < MC; ++m) {
          const int j = ownu.j(m);
          o[m] = ownu.valid(m) ? shL[j] + (zr[j] + mlp.bias[j]) * sL[j] : T(0);
        }
        const T oc = shL[CD] + (zr[CD] + mlp.bias[CD]) * sL[CD];
        const T nrm = dsqrt(Lanes<P>::sum(sumsq(o)));
        const T den = (T(1e-15) + fmax(oc, T(0))) + nrm;
        T dot = 0;
#pragma unroll
        for (int m = 0; m < MC; ++m) dot += gu[m] * o[m];
        const T k = Lanes<P>::sum(dot) / (den * den);
#pragma unroll
        for (int m = 0; m < MC; ++m) gu[m] = gu[m] / den - (k / nrm) * o[m];
        if (lc.p == 0) {
          const T goc = oc > T(0) ? -k : T(0);
          lrow[CD] = goc;
          if (live) grow[CD] = goc;
        }
      }
#pragma unroll
      for (int m = 0; m < MC; ++m) {
        if (ownu.valid(m)) {
          lrow[ownu.j(m)] = gu[m];
          if (live) grow[ownu.j(m)] = gu[m];
        }
      }
    }
    __syncthreads();
    // ---- input-gradient chain through the MLP (all four wavefronts) ----
    const T* in = s_pq[0];
    int pq = 1;
    for (int l = L; l >= ((DPAC_BWD_ABLATE & 8) ? L + 1 : 0); --l) {
      T* out = s_pq[pq];
      BwdEpi<T> epi{l >= 1 ? mlp.scale[l] : nullptr, l >= 1 ? mlp.shift[l] : nullptr,
                    a.z + (rowt + row0) * mlp.ztot + mlp.zoff[l], mlp.ztot, rows_live, lane, out,
                    a.G + (rowt + row0) * a.gtot + a.goff[l], a.gtot};
      mfma_layer<T>(in, mlp.width[l + 1], mlp.width[l], a.wt[l], a.wtkm[l], wave, lane, epi);
      __syncthreads();
      in = out;
      pq ^= 1;
    }
    if (stepper) {  // dL/dx_t = direct part + G_0 * s_0 (a_0 = beta_0 + x * s_0)
#pragma unroll
      for (int m = 0; m < M; ++m)
        lam[m] = gxd[m] + (own.valid(m) ? in[g * kNnLd + own.j(m)] * s0[m] : T(0));
    }
    __syncthreads();
  }
  if (a.g_x0 && live) own.store(a.g_x0 + lc.b * D, lam);
}

template <typename T, class E, int D, int SCHEME, bool COST, int KB, bool FAST, bool MASK = false>
__global__ __launch_bounds__(kNnThreads) void k_rollout_nn(const E eq, const DevConsts<T> c,
                                                          const NnMlp<T> mlp,
                                                          const NnRolloutArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC;
  using TR = Transition<T, E, SCHEME>;
  __shared__ T s_x0[kNnRows * kNnLd];   // BN_0(x_t)
  __shared__ T s_pq[2][kNnRows * kNnLd];
  if (a.guard && !x3_status_set(a.guard)) return;  // a fallback launch: only once the x3 kernel fell back
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
  // fast path: the narrow layers' weights in registers for the whole launch
  NarrowIn res_in;
  NarrowOut res_out;
  WidePre pre;
  static_assert(!FAST || std::is_same<T, float>::value, "the fast path is float-only");
  if constexpr (FAST) {  // launched only when mlp.fast (nn_fast_host)
    load_narrow_in(res_in, mlp.wkm[0], mlp.width[0], mlp.width[1], wave, lane);
    load_narrow_out(res_out, mlp.wkm[L], mlp.width[L], mlp.width[L + 1], wave, lane);
  }
  __syncthreads();  // padding zeroed before the first a0 write
  write_a0(x);

  auto load = [&](int t, DwFrame<T, M>& fr) { sx.load(rs_dw, fr.dw, (uint32_t)t * slab); };
  auto body = [&](int t, DwFrame<T, M>& fr, auto) {
    __syncthreads();  // a0 of step t is in s_x0; the previous step's reads are done
    NN_MARK(t, 0);
    // ---- actor MLP on MFMA (all four wavefronts) ----
    const T* in = s_x0;
    int pq = 0;
    for (int l = 0; l <= (DPAC_NN_ABLATE == 2 ? -1 : L); ++l) {  // ablation 2: no MLP (timing)
      T* out = s_pq[pq];
      FwdEpi<T> epi{mlp.scale[l + 1], mlp.shift[l + 1], l == L ? mlp.bias : nullptr, l < L, out,
                    a.save_z ? a.save_z + ((int64_t)t * a.B + row0) * mlp.ztot + mlp.zoff[l + 1] : nullptr,
                    mlp.ztot, rows_live};
      if constexpr (FAST) {
        if (MASK && l < L) {  // hidden output with its sign bits
          FwdEpiM<T> epm;
          static_cast<FwdEpi<T>&>(epm) = epi;
          epm.mask = a.save_mask + ((int64_t)t * ((a.B + 15) >> 4) + (row0 >> 4)) * a.mb + 13 * 64 * l;
          epm.nib = 0;
          if (l == 0) {
            if (L >= 2) load_wide_pre(pre, mlp.wkm[1], mlp.width[1], mlp.width[2], wave, lane);
            nn_layer_narrow_in(in, mlp.width[0], mlp.width[1], res_in, wave, lane, epm);
          } else {
            nn_layer_wide(in, mlp.width[l + 1], mlp.wkm[l], pre, wave, lane, epm, [&]() {
              if (l + 1 < L) load_wide_pre(pre, mlp.wkm[l + 1], mlp.width[l + 1], mlp.width[l + 2], wave, lane);
            });
          }
        } else if (l == 0) {
          if (L >= 2) load_wide_pre(pre, mlp.wkm[1], mlp.width[1], mlp.width[2], wave, lane);
          nn_layer_narrow_in(in, mlp.width[0], mlp.width[1], res_in, wave, lane, epi,
                             [&](int pt) { NN_MARK(t, pt); });
        } else if (l == L) {
          nn_layer_narrow_out(in, mlp.width[L], mlp.width[L + 1], res_out, wave, lane, epi);
        } else {
          nn_layer_wide(in, mlp.width[l + 1], mlp.wkm[l], pre, wave, lane, epi, [&]() {
            if (l + 1 < L) load_wide_pre(pre, mlp.wkm[l + 1], mlp.width[l + 1], mlp.width[l + 2], wave, lane);
          });
        }
      } else {
        mfma_layer<T>(in, mlp.width[l], mlp.width[l + 1], mlp.weight[l], mlp.wkm[l], wave, lane, epi);
      }
      NN_MARK(t, 1 + 2 * l);
      __syncthreads();
      NN_MARK(t, 2 + 2 * l);
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
    NN_MARK(t, 15);
  };
  pipelined<KB, DwFrame<T, M>>(0, a.N, load, body);
  if constexpr (COST) {
    if (live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
}
