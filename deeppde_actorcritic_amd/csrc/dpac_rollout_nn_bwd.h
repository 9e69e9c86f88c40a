// dpac_rollout_nn_bwd.h — the actor's BPTT (k_rollout_nn_bwd's reverse time loop and
// MLP input-gradient chain, solver.py:92-97 differentiated) with the memory traffic
// taken off the MFMA wavefronts.
//
// Measured on k_rollout_nn_bwd (lqr_d20 actor, B = 2048, N = 100, 16.1 us per reverse
// step; profiles/r02_bptt_ablation_base.txt): dropping the epilogue's z loads saves 1.7 us
// per step, the G stores 1.0, the step lanes' input loads 0.8.  gfx950 counts vector
// loads and stores in one in-order vmcnt, so each of those waits behind (or holds up)
// the weight-ring loads of the MFMA waves.  Here the workgroup gets two more wavefronts:
//   * the STAGER (wave kNnWaves) copies step t-1's inputs — the rows of x, dw, u, flag,
//     disc and (when it fits) the saved pre-BN outputs z — into an LDS parity buffer
//     with global_load_lds while step t computes, and waits for them once, before the
//     step's last barrier;
//   * the WRITER (wave kNnWaves + 1) stores each layer's G block from the LDS image the
//     next layer reads anyway, right after the barrier that completes it, and never waits.
// The MFMA waves' vmcnt then holds only their weight loads; the BN scales and shifts are
// copied to LDS once.  Barriers are s_barrier after lgkmcnt(0) (nn_bar): the stager's
// LDS-DMA stays in flight across them.  Results are bitwise those of k_rollout_nn_bwd
// (same products, same order).
#pragma once
// Included by dpac_kernels.h inside namespace dpac, after dpac_rollout_nn.h.

constexpr int kNnBwdThreads = kNnThreads + 128;  // + stager + writer
#ifndef DPAC_BWD2_GNT
#define DPAC_BWD2_GNT 0  // timing knob: non-temporal G stores from the writer wave
#endif
#ifndef DPAC_BWD2_DMA_NT
#define DPAC_BWD2_DMA_NT 0  // timing knob: the stager's LDS-DMA with the nt cache policy
#endif
#if DPAC_BWD2_DMA_NT
#define DPAC_BWD2_DMA_POL " nt"
#else
#define DPAC_BWD2_DMA_POL ""
#endif
#ifndef DPAC_BWD2_ZREG
#define DPAC_BWD2_ZREG 0  // timing knob: stage z through the stager's VGPRs instead of LDS-DMA
#endif
#ifndef DPAC_BWD2_ABLATE
#define DPAC_BWD2_ABLATE 0  // timing-only builds (bits): 1 = the stager copies nothing, 2 = the writer
                           // does nothing, 4 = the writer reads LDS but stores nothing
#endif

__device__ __forceinline__ void nn_bar() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// One wave copies `bytes` contiguous bytes from global src to LDS dst (both SZ-aligned)
// with global_load_lds: piece k, lane l moves bytes [SZ(64k + l), +SZ).  Lanes past the
// end read the first SZ bytes again (in bounds); dst must hold roundup(bytes, 64 SZ).
// Issued as inline asm: the compiler's wait insertion, which cannot tell the stager wave
// from the others, would otherwise guard every later LDS read of EVERY wave with a
// vmcnt(0) for the DMA (and so drain the MFMA waves' weight ring).  The caller waits with
// an explicit s_waitcnt vmcnt(0) before the barrier that publishes the data.
// part / parts: this call issues the part-th of `parts` equal shares of the pieces (the
// stager spreads the z rows over the step's first phases).
template <int SZ>
__device__ __forceinline__ void wave_copy_lds(const void* src, uint32_t bytes, unsigned char* dst,
                                              int lane, uint32_t part = 0, uint32_t parts = 1) {
  static_assert(SZ == 16 || SZ == 4, "global_load_lds_dwordx4 / _dword");
  const char* s = (const char*)src;
  const uint32_t pieces = (bytes + 64 * SZ - 1) / (64 * SZ);
  const uint32_t lds0 = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)dst;
  const uint32_t k0 = pieces * part / parts, k1 = pieces * (part + 1) / parts;
  for (uint32_t k = k0; k < k1; ++k) {
    const uint32_t off = (k * 64 + (uint32_t)lane) * SZ;
    const char* gp = s + (off < bytes ? off : 0);
    const uint32_t m0 = __builtin_amdgcn_readfirstlane(lds0 + k * 64 * SZ);
    int keep;
    if constexpr (SZ == 16)
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off" DPAC_BWD2_DMA_POL "\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(gp), "s"(m0) : "memory");
    else
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(gp), "s"(m0) : "memory");
  }
}

constexpr uint32_t round_up(uint32_t v, uint32_t m) { return (v + m - 1) / m * m; }

// Dynamic-LDS plan of k_rollout_nn_bwd2 (host and device): BN scale/shift images, two
// parity buffers of step inputs, then (zst) two parity buffers of z rows.
template <typename T, int D, int CD>
struct BwdPlan {
  static constexpr int kSzX = (D * sizeof(T)) % 16 == 0 ? 16 : 4;
  static constexpr int kSzU = (CD * sizeof(T)) % 16 == 0 ? 16 : 4;
  static constexpr uint32_t kX = 0;
  static constexpr uint32_t kDw = kX + round_up(kNnRows * D * sizeof(T), 64 * kSzX);
  static constexpr uint32_t kU = kDw + round_up(kNnRows * D * sizeof(T), 64 * kSzX);
  static constexpr uint32_t kDisc = kU + round_up(kNnRows * CD * sizeof(T), 64 * kSzU);
  static constexpr uint32_t kFlag = kDisc + round_up(kNnRows * sizeof(T), 256);
  static constexpr uint32_t kPar = kFlag + 256;  // one parity buffer of step inputs
  uint32_t bn, in, z, zpar, total;
  bool zst;
  // widths sum = Σ_i width[i] (the BN image: scale then shift); ztot = Σ_{i>=1} width[i];
  // mask_tile_bytes > 0: the parity buffers hold the sign-bit mask tile instead of z
  __host__ __device__ BwdPlan(int wsum, int ztot, bool want_z, int mask_tile_bytes = 0) {
    bn = 0;
    in = round_up(2u * (uint32_t)wsum * sizeof(T), 16);
    z = in + 2 * kPar;
    if (mask_tile_bytes > 0) {
      zst = false;
      zpar = round_up((uint32_t)mask_tile_bytes, 1024);
      total = z + 2 * zpar;
      return;
    }
    zpar = round_up((uint32_t)(kNnRows * ztot) * sizeof(T), 1024);
    zst = want_z && ((ztot * sizeof(T)) % 16 == 0) && z + 2 * zpar <= kMaxDyn;
    total = zst ? z + 2 * zpar : z;
  }
  // static __shared__ s_pq takes 2 x 16 x kNnLd x sizeof(T); the rest of 160 KB is dynamic
  static constexpr uint32_t kMaxDyn = 160 * 1024 - 2 * kNnRows * kNnLd * sizeof(T) - 1024;
};

// Backward epilogue (as BwdEpi) reading z and the BN constants from LDS and writing G_l
// only to the LDS image (the writer wave stores it).
template <typename T>
struct BwdEpiL {
  struct Col {
    T s, sh, z[4];
  };
  const T *scale, *shift;  // LDS, or null for l == 0
  const T* z;              // z_l of row 0 of the workgroup at this step (LDS or global)
  int z_stride, rows_live, lane;
  T* out;                  // LDS [16][kNnLd]
  __device__ __forceinline__ Col load(int col, bool valid) const {
    Col k{};
    if (scale) {
      k.s = valid ? scale[col] : T(0);
      k.sh = valid ? shift[col] : T(0);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = Mfma<T>::row(lane, i);
        k.z[i] = (valid && row < rows_live) ? z[row * z_stride + col] : T(0);
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
    out[row * kNnLd + col] = valid ? v : T(0);
  }
  __device__ __forceinline__ void store(int i, int row, int col, bool valid, T acc, const Col& k) const {
    T v = acc;
    if (scale) {
      const T yv = k.sh + k.z[i] * k.s;  // the forward's BN_l output, same expression
      v = acc * (yv > T(0) ? T(2) : T(1));  // d(y + relu(y))/dy
    }
    out[row * kNnLd + col] = valid ? v : T(0);
  }
};

// BwdEpiL with the activation factor from the forward's sign-bit mask (FwdEpiM) staged in
// LDS: 1 + bit, the value the z-based epilogue computes (same comparison, made once in the
// forward), so G is bitwise the same.  Used for the hidden layers (l >= 1) only.
template <typename T>
struct BwdEpiLM {
  struct Col {
    T f[4];
  };
  const uint8_t* m;  // LDS mask tile (FwdEpiM's layout) at this layer's offset
  int rows_live, lane;
  T* out;
  __device__ __forceinline__ Col load(int col, bool valid) const {
    Col k;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = Mfma<T>::row(lane, i);
      const uint32_t h = m[(col >> 4) * 64 + 16 * (row >> 2) + (col & 15)];
      k.f[i] = (valid && row < rows_live && ((h >> (row & 3)) & 1u)) ? T(2) : T(1);
    }
    return k;
  }
  __device__ __forceinline__ void store(int i, int row, int col, bool valid, T acc, const Col& k) const {
    out[row * kNnLd + col] = valid ? acc * k.f[i] : T(0);
  }
};

// The writer wave: G block `width` wide of the workgroup's rows from the LDS image `img`
// (row stride kNnLd) to G rows (stride gtot) at column offset goff.  Lane l owns vector
// q = l % per_row of rows l / per_row + k * (64 / per_row); four passes' LDS reads are in
// flight before their stores.  16-byte vectors when the block, the row stride and the
// offset allow it, else single elements.
template <typename T, int V>
__device__ __forceinline__ void write_G_rows(const T* img, int per_row, T* G, int64_t gtot, int goff,
                                             int rows_live, int lane) {
  typedef T vec __attribute__((ext_vector_type(V)));
  const int rpp = 64 / per_row;  // rows per pass
  const int r0 = lane / per_row, q = lane - r0 * per_row;
  const bool act = r0 < rpp;
  for (int rb = 0; rb < rows_live; rb += 4 * rpp) {
    vec v0, v1, v2, v3;  // the reads: clamped rows (in the image), so no branch
    const int ra = rb + r0, rb1 = ra + rpp, rc = ra + 2 * rpp, rd = ra + 3 * rpp;
    v0 = *reinterpret_cast<const vec*>(img + (ra < rows_live ? ra : 0) * kNnLd + q * V);
    v1 = *reinterpret_cast<const vec*>(img + (rb1 < rows_live ? rb1 : 0) * kNnLd + q * V);
    v2 = *reinterpret_cast<const vec*>(img + (rc < rows_live ? rc : 0) * kNnLd + q * V);
    v3 = *reinterpret_cast<const vec*>(img + (rd < rows_live ? rd : 0) * kNnLd + q * V);
#if DPAC_BWD2_ABLATE & 4
    asm volatile("" ::"v"(v0), "v"(v1), "v"(v2), "v"(v3));
    continue;
#endif
#if DPAC_BWD2_GNT  // timing knob: non-temporal G stores
    if (act && ra < rows_live) __builtin_nontemporal_store(v0, reinterpret_cast<vec*>(G + ra * gtot + goff + q * V));
    if (act && rb1 < rows_live) __builtin_nontemporal_store(v1, reinterpret_cast<vec*>(G + rb1 * gtot + goff + q * V));
    if (act && rc < rows_live) __builtin_nontemporal_store(v2, reinterpret_cast<vec*>(G + rc * gtot + goff + q * V));
    if (act && rd < rows_live) __builtin_nontemporal_store(v3, reinterpret_cast<vec*>(G + rd * gtot + goff + q * V));
#else
    if (act && ra < rows_live) *reinterpret_cast<vec*>(G + ra * gtot + goff + q * V) = v0;
    if (act && rb1 < rows_live) *reinterpret_cast<vec*>(G + rb1 * gtot + goff + q * V) = v1;
    if (act && rc < rows_live) *reinterpret_cast<vec*>(G + rc * gtot + goff + q * V) = v2;
    if (act && rd < rows_live) *reinterpret_cast<vec*>(G + rd * gtot + goff + q * V) = v3;
#endif
  }
}

template <typename T>
__device__ __forceinline__ void write_G_block(const T* img, int width, T* G, int64_t gtot, int goff,
                                              int rows_live, int lane) {
  constexpr int V = 16 / (int)sizeof(T);
  if (width % V == 0 && gtot % V == 0 && goff % V == 0 && width / V <= 64)
    write_G_rows<T, V>(img, width / V, G, gtot, goff, rows_live, lane);
  else if (width <= 64)
    write_G_rows<T, 1>(img, width, G, gtot, goff, rows_live, lane);
  else
    for (int c0 = 0; c0 < width; c0 += 64)  // wide blocks with odd widths: 64-column strips
      write_G_rows<T, 1>(img + c0, width - c0 < 64 ? width - c0 : 64, G, gtot, goff + c0, rows_live, lane);
}

template <typename T, class E, int D, int SCHEME, bool ZST, bool FAST, bool MASK = false>
__global__ __launch_bounds__(kNnBwdThreads) void k_rollout_nn_bwd2(const E eq, const DevConsts<T> c,
                                                                  const NnMlp<T> mlp,
                                                                  const NnBackArgs<T> a) {
  constexpr int P = E::kP, M = E::M, MC = E::MC, CD = E::CDIM;
  using PL = BwdPlan<T, D, CD>;
  __shared__ T s_pq[2][kNnRows * kNnLd];
  extern __shared__ __attribute__((aligned(16))) unsigned char s_dyn[];
  if (a.guard && !x3_status_set(a.guard)) return;  // a fallback launch: only once the x3 kernel fell back
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const bool stager = wave == kNnWaves && !(DPAC_BWD2_ABLATE & 1);
  const bool writer = wave == kNnWaves + 1 && !(DPAC_BWD2_ABLATE & 2);
  const int64_t row0 = (int64_t)blockIdx.x * kNnRows;
  const int rows_live = (int)((a.B - row0) < kNnRows ? (a.B - row0) : kNnRows);
  const bool stepper = tid < kNnRows * P;
  const int g = stepper ? tid / P : 0;
  const LaneCoord<P> lc(a.B, stepper ? tid % P : 0, row0 + g);
  const bool live = stepper && lc.live;
  const Own<D, P> own(lc.p);
  const Own<CD, P> ownu(lc.p);
  const int L = mlp.L;
  int wsum = 0;
  for (int i = 0; i <= L + 1; ++i) wsum += mlp.width[i];
  static_assert(!MASK || (FAST && !ZST), "the mask replaces z staging on the fast path");
  const PL pl(wsum, mlp.ztot, ZST, MASK ? a.mb : 0);
  T* s_bn = reinterpret_cast<T*>(s_dyn + pl.bn);  // [scale image | shift image], column goff[i]
  auto s_in = [&](int par) { return s_dyn + pl.in + (uint32_t)par * PL::kPar; };
  auto s_z = [&](int par) { return reinterpret_cast<const T*>(s_dyn + pl.z + (uint32_t)par * pl.zpar); };

  // step ts's inputs -> parity buffer par (stager wave): the step lanes' rows, then the z
  // rows in kZParts shares, one per phase, so no phase's barrier waits on the stager
  constexpr uint32_t kZParts = 3;
  auto stage_in = [&](int ts, int par) {
    const int64_t rt = (int64_t)ts * a.B + row0;
    unsigned char* b = s_dyn + pl.in + (uint32_t)par * PL::kPar;
    wave_copy_lds<PL::kSzX>(a.x + rt * D, (uint32_t)(rows_live * D * sizeof(T)), b + PL::kX, lane);
    wave_copy_lds<PL::kSzX>(a.dw + rt * D, (uint32_t)(rows_live * D * sizeof(T)), b + PL::kDw, lane);
    wave_copy_lds<PL::kSzU>(a.u + rt * CD, (uint32_t)(rows_live * CD * sizeof(T)), b + PL::kU, lane);
    wave_copy_lds<4>(a.disc_t + rt, (uint32_t)(rows_live * sizeof(T)), b + PL::kDisc, lane);
    wave_copy_lds<4>(a.flag + rt, (uint32_t)(rows_live * 4), b + PL::kFlag, lane);
  };
  auto stage_z = [&](int ts, int par, uint32_t part) {
    if constexpr (MASK) {  // the sign-bit tile (mb bytes, padded rows included): one share
      if (part == 0)
        wave_copy_lds<16>(a.mask + ((int64_t)ts * ((a.B + 15) >> 4) + (row0 >> 4)) * a.mb,
                          (uint32_t)a.mb, s_dyn + pl.z + (uint32_t)par * pl.zpar, lane);
    }
    if constexpr (ZST) {
      const int64_t rt = (int64_t)ts * a.B + row0;
#if DPAC_BWD2_ZREG
      // timing knob: the z share through the stager's VGPRs (dwordx4 loads, ds_write_b128)
      // instead of LDS-DMA
      const uint32_t bytes = (uint32_t)(rows_live * mlp.ztot * sizeof(T));
      const uint32_t pieces = (bytes + 1023) / 1024;
      const uint32_t k0 = pieces * part / kZParts, k1 = pieces * (part + 1) / kZParts;
      const __amdgpu_buffer_rsrc_t rz = make_rsrc(a.z + rt * mlp.ztot, bytes);
      unsigned char* dst = s_dyn + pl.z + (uint32_t)par * pl.zpar;
      typedef uint32_t u4 __attribute__((ext_vector_type(4)));
      u4 v[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const uint32_t off = ((k0 + q) * 64 + (uint32_t)lane) * 16;
        uint32_t w[4];
        buf_load_dwords<4>(rz, (k0 + q < k1) ? off : kOOB, w);
        v[q] = u4{w[0], w[1], w[2], w[3]};
      }
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (k0 + q < k1) *reinterpret_cast<u4*>(dst + ((k0 + q) * 64 + (uint32_t)lane) * 16) = v[q];
#else
      wave_copy_lds<16>(a.z + rt * mlp.ztot, (uint32_t)(rows_live * mlp.ztot * sizeof(T)),
                        s_dyn + pl.z + (uint32_t)par * pl.zpar, lane, part, kZParts);
#endif
    }
  };

  for (int i = tid; i < kNnRows * kNnLd; i += kNnBwdThreads) {
    s_pq[0][i] = T(0);
    s_pq[1][i] = T(0);
  }
  for (int i = 0; i <= L + 1; ++i)  // BN constants: LDS copies the epilogues read
    for (int j = tid; j < mlp.width[i]; j += kNnBwdThreads) {
      s_bn[a.goff[i] + j] = mlp.scale[i][j];
      s_bn[wsum + a.goff[i] + j] = mlp.shift[i][j];
    }
  T s0[M], lam[M], gxd[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    s0[m] = own.valid(m) ? mlp.scale[0][own.j(m)] : T(0);
    lam[m] = T(0);
    gxd[m] = T(0);
  }
  // fast path: the narrow products' weights in registers for the whole launch
  NarrowIn res_in;
  NarrowOut res_out;
  WidePre pre;
  static_assert(!FAST || std::is_same<T, float>::value, "the fast path is float-only");
  if constexpr (FAST) {  // launched only when a.fast (nn_fast_host)
    if (wave < kNnWaves) {
      load_narrow_in(res_in, a.wtkm[L], mlp.width[L + 1], mlp.width[L], wave, lane);
      load_narrow_out(res_out, a.wtkm[0], mlp.width[1], mlp.width[0], wave, lane);
    }
  }
  if (a.g_xN && stepper) own.load_masked(a.g_xN + lc.b * D, lam);
  T gD = (a.g_disc && stepper) ? a.g_disc[lc.b] : T(0);
  const T gy = (a.g_y && stepper) ? a.g_y[lc.b] : T(0);
  if (stager) {
    stage_in(a.N - 1, (a.N - 1) & 1);
    for (uint32_t k = 0; k < kZParts; ++k) stage_z(a.N - 1, (a.N - 1) & 1, k);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  nn_bar();
  for (int t = a.N - 1; t >= 0; --t) {
    const int64_t rowt = (int64_t)t * a.B;
    const int par = t & 1;
    NN_MARK(t, 0);
    if (stager && t > 0) stage_in(t - 1, par ^ 1);  // lands while step t computes
    if (stepper) {
      const unsigned char* bi = s_in(par);
      const T* xr = reinterpret_cast<const T*>(bi + PL::kX) + g * D;
      const T* dwr = reinterpret_cast<const T*>(bi + PL::kDw) + g * D;
      const T* ur = reinterpret_cast<const T*>(bi + PL::kU) + g * CD;
      T x[M], u[MC], dwv[M], gu[MC], gdn;
      own.load_masked(xr, x);
      own.load_masked(dwr, dwv);
      ownu.load_masked(ur, u);
      const Flags fl = Flags::decode(reinterpret_cast<const int32_t*>(bi + PL::kFlag)[g]);
      const T dsc = reinterpret_cast<const T*>(bi + PL::kDisc)[g];
      step_vjp<T, E, SCHEME>(eq, c, x, u, dwv, fl, dsc, lam, gD, gy, gxd, gu, gdn);
      gD = gdn;
      T* lrow = s_pq[0] + g * kNnLd;
      if (mlp.ekn) {  // gradient at the network output, through the Eikonal head (solver.py:272-274)
        const T* zr = ZST ? s_z(par) + g * mlp.ztot + mlp.zoff[L + 1]
                          : a.z + (rowt + lc.b) * mlp.ztot + mlp.zoff[L + 1];
        const T* sL = s_bn + a.goff[L + 1];
        const T* shL = s_bn + wsum + a.goff[L + 1];
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
        if (lc.p == 0) lrow[CD] = oc > T(0) ? -k : T(0);
      }
#pragma unroll
      for (int m = 0; m < MC; ++m)
        if (ownu.valid(m)) lrow[ownu.j(m)] = gu[m];
    }
    NN_MARK(t, 1);
    nn_bar();
    NN_MARK(t, 2);
    if (stager && t > 0) stage_z(t - 1, par ^ 1, 0);
    if (writer)
      write_G_block(s_pq[0], mlp.width[L + 1], a.G + (rowt + row0) * a.gtot, a.gtot, a.goff[L + 1],
                    rows_live, lane);
    // ---- input-gradient chain through the MLP (the MFMA wavefronts) ----
    const T* in = s_pq[0];
    int pq = 1;
    for (int l = L; l >= 0; --l) {
      T* out = s_pq[pq];
      const int K = mlp.width[l + 1], Nout = mlp.width[l];
      if (wave < kNnWaves) {
        BwdEpiL<T> epi{l >= 1 ? s_bn + a.goff[l] : nullptr, l >= 1 ? s_bn + wsum + a.goff[l] : nullptr,
                       ZST ? s_z(par) + mlp.zoff[l] : a.z + (rowt + row0) * mlp.ztot + mlp.zoff[l],
                       mlp.ztot, rows_live, lane, out};
        if constexpr (MASK) {
          if (l >= 1) {  // hidden layer l: its mask rows sit at halfword 13 (l - 1)
            BwdEpiLM<T> epm{reinterpret_cast<const uint8_t*>(s_dyn + pl.z + (uint32_t)par * pl.zpar) + 13 * 64 * (l - 1),
                            rows_live, lane, out};
            if (l == L) {
              if (L >= 2) load_wide_pre(pre, a.wtkm[L - 1], mlp.width[L], mlp.width[L - 1], wave, lane);
              nn_layer_narrow_in(in, K, Nout, res_in, wave, lane, epm);
            } else {
              nn_layer_wide(in, Nout, a.wtkm[l], pre, wave, lane, epm, [&]() {
                if (l >= 2) load_wide_pre(pre, a.wtkm[l - 1], mlp.width[l], mlp.width[l - 1], wave, lane);
              });
            }
          } else {
            nn_layer_narrow_out(in, K, Nout, res_out, wave, lane, epi);
          }
        } else if constexpr (FAST) {
          if (l == L) {
            if (L >= 2) load_wide_pre(pre, a.wtkm[L - 1], mlp.width[L], mlp.width[L - 1], wave, lane);
            nn_layer_narrow_in(in, K, Nout, res_in, wave, lane, epi);
          } else if (l == 0) {
            nn_layer_narrow_out(in, K, Nout, res_out, wave, lane, epi);
          } else {
            nn_layer_wide(in, Nout, a.wtkm[l], pre, wave, lane, epi, [&]() {
              if (l >= 2) load_wide_pre(pre, a.wtkm[l - 1], mlp.width[l], mlp.width[l - 1], wave, lane);
            });
          }
        } else {
          mfma_layer<T>(in, K, Nout, a.wt[l], a.wtkm[l], wave, lane, epi);
        }
      } else if (nn_splitk_layer(K, Nout)) {
        nn_bar();  // the split-K product's two internal barriers
        nn_bar();
      }
      NN_MARK(t, 3 + 2 * (L - l));
      nn_bar();
      NN_MARK(t, 4 + 2 * (L - l));
      if (stager && t > 0 && L - l + 1 < (int)kZParts) stage_z(t - 1, par ^ 1, (uint32_t)(L - l + 1));
      if (writer) write_G_block(out, Nout, a.G + (rowt + row0) * a.gtot, a.gtot, a.goff[l], rows_live, lane);
      in = out;
      pq ^= 1;
    }
    if (stepper) {  // dL/dx_t = direct part + G_0 * s_0 (a_0 = beta_0 + x * s_0)
#pragma unroll
      for (int m = 0; m < M; ++m)
        lam[m] = gxd[m] + (own.valid(m) ? in[g * kNnLd + own.j(m)] * s0[m] : T(0));
    }
    if (stager) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // step t-1's inputs landed
    NN_MARK(t, 13);
    nn_bar();
    NN_MARK(t, 14);
  }
  if (a.g_x0 && live) own.store(a.g_x0 + lc.b * D, lam);
}
