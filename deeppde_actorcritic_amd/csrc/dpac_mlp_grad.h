// dpac_mlp_grad.h — parameter gradients of a DeepNN (solver.py:227-278) from the
// backward chain's G and the forward's saved pre-BN outputs, over R independent
// rows (the actor's N*B BPTT rows or the critic G network's N*B rows).
//
// With s_i = gamma_i/sqrt(1+eps), a_0 = BN_0(x), a_i = y_i + relu(y_i),
// y_i = beta_i + z_i*s_i (i = 1..L) and G_i = dL/d(output of BN_i):
//   dW_i     = Σ_r a_i[r]^T (G_{i+1}[r] ⊙ s_{i+1})          [w_i x w_{i+1}]
//   dbeta_i  = Σ_r G_i[r]
//   dgamma_i = rs · Σ_r G_i[r] ⊙ zin_i[r],  zin_0 = x, zin_i = z_i, zin_{L+1} = z_{L+1} + b
//   db       = s_{L+1} ⊙ dbeta_{L+1}
// (what the reference's GradientTape produces for the trainable variables of
// DeepNN, solver.py:88,95).
//
// k_param_grads: workgroup (chunk c, column group g, layer i) = 4 wavefronts.
// Rows of the chunk are staged SR at a time through LDS — a_i (BN + activation
// applied while loading z_i) as the MFMA A operand (transposed: the reduction
// runs over rows) and G_{i+1} ⊙ s_{i+1} for the group's CW columns as B — and
// every wavefront accumulates its 16 x NTJ output tiles of dW_i in registers
// across the whole chunk.  The BN column sums ride on the same loads.  Each
// workgroup writes its chunk's partial; k_param_grads_reduce sums the chunks in
// a fixed order (deterministic, no atomics) and applies rs and s_{L+1}.
#pragma once

#include "dpac_device.h"

namespace dpac {

#ifndef DPAC_PG_SR
#define DPAC_PG_SR 16  // rows staged per sub-chunk
#endif
constexpr int kPgThreads = 256;
constexpr int kPgQ = DPAC_MLP_MAX_WIDTH / 64;  // A-stage columns per thread

// Rows staged per sub-chunk (4 row phases of the 4 wavefronts).
template <typename T>
struct PgCfg {
  static constexpr int SR = DPAC_PG_SR;
};

template <typename T>
struct PgArgs {
  int64_t rows, rows_per_chunk;
  int L;
  int width[DPAC_MLP_MAX_HIDDEN + 2];
  const T* scale[DPAC_MLP_MAX_HIDDEN + 2];
  const T* shift[DPAC_MLP_MAX_HIDDEN + 2];
  const T* bias;
  const T *x, *z, *G;
  int ldx, ztot, gtot;
  int zoff[DPAC_MLP_MAX_HIDDEN + 2];  // column of z_i in a z row (i >= 1)
  int goff[DPAC_MLP_MAX_HIDDEN + 2];  // column of G_i in a G row
  int64_t ptot;                       // elements per chunk partial (= flat size without b)
  int64_t off_gamma[DPAC_MLP_MAX_HIDDEN + 2], off_beta[DPAC_MLP_MAX_HIDDEN + 2];
  int64_t off_W[DPAC_MLP_MAX_HIDDEN + 1];
  T* part;  // [nchunks][ptot]
  uint32_t* status;       // split-fp16 kernel: the range guard (dpac.h dpac_mlp.status), or null
  const uint32_t* guard;  // f32 kernel as the fallback of a split-fp16 launch: run only once this
                          // word is set, every layer in one launch (blockIdx.z); null = always run
};

// One sub-chunk's global loads, issued before the MFMA phase of the previous one.
template <typename T, int SR, int QB>
struct PgStage {
  T a[SR / 4][kPgQ];  // zin_l (A source) at rows wave + 4m, columns lane + 64q
  T g0[SR / 4];       // layer 0 only: G_0 at column lane (BN_0 sums)
  T gb[SR / 4][QB];   // G_{l+1} at columns col0 + lane + 64q
  T zb[SR / 4][QB];   // zin_{l+1} (pre-bias) at the same places
};

// Workgroup (chunk c, column group g) of layer l: the chunk's partial of dW_l
// for B columns [g*CW, (g+1)*CW), plus the BN_{l+1} column sums of those
// columns (and, layer 0 / group 0, the BN_0 sums).  The 4 wavefronts form a
// WI x WJ grid over the output tiles: wave (wi, wj) owns row tiles wi + WI*m
// (m < NTI) and column tiles wj + WJ*j (j < NTJ), so NTI*WI*16 >= K and
// CW = NTJ*WJ*16.  Wide layers use WI = 1, WJ = 4; the narrow output layer
// (H <= 32) WI = 4, WJ = 1, so no wavefront multiplies padding columns.
// NTI / NTJ are compile-time: the MFMA loop is straight-line code.
template <typename T, int NTI, int NTJ, int WI>
__device__ __forceinline__ void pg_block(const PgArgs<T>& a, const int l, const int grp, const int64_t chunk);

// l_arg >= 0: layer l_arg, chunk blockIdx.x, column group blockIdx.y.  l_arg < 0: the guarded f32
// fallback of a split-fp16 launch over every layer, -l_arg column groups: a 1-D grid strides over
// the (chunk, group, layer) blocks (round 5: a small grid, so the launch costs little when the
// status word is clear and it exits at once — the (chunks x groups x layers) grid took 46 us to
// dispatch and retire its empty workgroups on the lqr_d20 G network)
template <typename T, int NTI, int NTJ, int WI>
__global__ __launch_bounds__(kPgThreads) void k_param_grads(const PgArgs<T> a, const int l_arg) {
  if (a.guard && !x3_status_set(a.guard)) return;  // a fallback launch: only once the x3 kernel fell back
  if (l_arg >= 0) {
    pg_block<T, NTI, NTJ, WI>(a, l_arg, (int)blockIdx.y, (int64_t)blockIdx.x);
    return;
  }
  const int64_t nch = (a.rows + a.rows_per_chunk - 1) / a.rows_per_chunk, ngrp = -l_arg;
  const int64_t nblk = nch * ngrp * (a.L + 1);
  for (int64_t vb = blockIdx.x; vb < nblk; vb += gridDim.x) {
    if (vb != (int64_t)blockIdx.x) __syncthreads();  // the previous block's LDS reads are done
    pg_block<T, NTI, NTJ, WI>(a, (int)(vb / (nch * ngrp)), (int)((vb / nch) % ngrp), vb % nch);
  }
}

template <typename T, int NTI, int NTJ, int WI>
__device__ __forceinline__ void pg_block(const PgArgs<T>& a, const int l, const int grp, const int64_t chunk) {
  using MF = Mfma<T>;
  constexpr int WJ = 4 / WI;
  constexpr int SR = PgCfg<T>::SR;
  constexpr int CW = 16 * NTJ * WJ;               // B columns per workgroup
  constexpr int QB = (CW + 63) / 64;              // B columns per thread
  constexpr int LDA = DPAC_MLP_MAX_WIDTH + 16;    // row strides: lanes of a k-quad
  constexpr int LDB = (CW < 64 ? 64 : CW) + 16;   // land 16 words apart
  constexpr int kpad = 16 * NTI * WI;             // staged A columns
  static_assert(kpad <= DPAC_MLP_MAX_WIDTH, "A image");
  constexpr uint32_t ES = sizeof(T);
  __shared__ T sA[SR * LDA];
  __shared__ T sB[SR * LDB];
  const int K = a.width[l], H = a.width[l + 1];
  const int col0 = grp * CW;
  if (col0 >= H) return;  // whole workgroup: no barrier reached yet
  const int tid = threadIdx.x, lane = tid % 64;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64);
  const int wi = wave / WJ, wj = wave % WJ;
  const int64_t r_begin = chunk * a.rows_per_chunk;
  const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
  const bool first = l == 0 && grp == 0;  // also sums BN_0
  const bool last = l == a.L;             // zin_{L+1} = z_{L+1} + bias
  const T* srcA = l == 0 ? a.x : a.z + a.zoff[l];
  const int64_t ldA = l == 0 ? a.ldx : a.ztot;
  const T* gA = a.G + a.goff[0];
  const T* gB = a.G + a.goff[l + 1] + col0;
  const T* zB = a.z + a.zoff[l + 1] + col0;

  // per-thread constants: A columns lane + 64q, B columns col0 + lane + 64q
  T sa[kPgQ], ha[kPgQ], sbv[QB], bbv[QB];
  uint32_t offA[kPgQ], offB[QB];
#pragma unroll
  for (int q = 0; q < kPgQ; ++q) {
    const int k = lane + 64 * q;
    sa[q] = k < K ? a.scale[l][k] : T(0);
    ha[q] = k < K ? a.shift[l][k] : T(0);
    offA[q] = k < K ? (uint32_t)k * ES : kOOB;
  }
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const int c = lane + 64 * q, h = col0 + c;
    const bool v = c < CW && h < H;
    sbv[q] = v ? a.scale[l + 1][h] : T(0);
    bbv[q] = (v && last) ? a.bias[h] : T(0);
    offB[q] = v ? (uint32_t)c * ES : kOOB;
  }
  const uint32_t offG0 = (first && lane < K) ? (uint32_t)lane * ES : kOOB;
  T cs0_b = 0, cs0_s = 0, csb_b[QB], csb_s[QB];
#pragma unroll
  for (int q = 0; q < QB; ++q) csb_b[q] = csb_s[q] = T(0);
  typename MF::acc_t acc[NTI][NTJ];
#pragma unroll
  for (int ti = 0; ti < NTI; ++ti)
#pragma unroll
    for (int jj = 0; jj < NTJ; ++jj) acc[ti][jj] = typename MF::acc_t{0, 0, 0, 0};

  // Loads of the SR rows starting at r0: descriptors based at row r0 whose range
  // ends at the chunk's last row, so rows past it read 0; masked columns carry
  // kOOB offsets (kOOB + a row offset < 2^32 stays out of range).  Every load is
  // unconditional: a select on a load result would force its wait right there.
  auto issue = [&](int64_t r0, PgStage<T, SR, QB>& st) {
    const int64_t nr = r_end - r0;  // >= 1
    const auto rA = make_rsrc(srcA + r0 * ldA, (uint32_t)(((nr - 1) * ldA + K) * ES));
    const auto rG = make_rsrc(gA + r0 * a.gtot, (uint32_t)(((nr - 1) * a.gtot + K) * ES));
    const auto rB = make_rsrc(gB + r0 * a.gtot, (uint32_t)(((nr - 1) * a.gtot + (H - col0)) * ES));
    const auto rZ = make_rsrc(zB + r0 * a.ztot, (uint32_t)(((nr - 1) * a.ztot + (H - col0)) * ES));
#pragma unroll
    for (int m = 0; m < SR / 4; ++m) {
      const uint32_t rl = (uint32_t)(wave + 4 * m);
#pragma unroll
      for (int q = 0; q < kPgQ; ++q)
        if (64 * q < kpad) st.a[m][q] = buf_load_elem<T>(rA, offA[q] + rl * (uint32_t)ldA * ES);
      st.g0[m] = buf_load_elem<T>(rG, offG0 + rl * (uint32_t)a.gtot * ES);
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        st.gb[m][q] = buf_load_elem<T>(rB, offB[q] + rl * (uint32_t)a.gtot * ES);
        st.zb[m][q] = buf_load_elem<T>(rZ, offB[q] + rl * (uint32_t)a.ztot * ES);
      }
    }
  };

  PgStage<T, SR, QB> st;
  issue(r_begin, st);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += SR) {
    __syncthreads();  // the previous sub-chunk's MFMA reads are done
#pragma unroll
    for (int m = 0; m < SR / 4; ++m) {
      const int rl = wave + 4 * m;
#pragma unroll
      for (int q = 0; q < kPgQ; ++q) {
        const int k = lane + 64 * q;
        if (64 * q >= kpad) continue;  // compile-time
        const T zi = st.a[m][q];
        const T y = ha[q] + zi * sa[q];  // the forward's expression (FwdEpi / write_a0)
        const T v = l == 0 ? y : y + fmax(y, T(0));
        if (k < kpad) sA[rl * LDA + k] = k < K ? v : T(0);  // rows past the end: z = 0 gives
      }                                                      // a = shift, masked by G = 0
      cs0_b += st.g0[m];  // G_0 reads 0 unless layer 0 / group 0
      cs0_s += st.g0[m] * st.a[m][0];
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        const T gv = st.gb[m][q];
        if (lane + 64 * q < CW) sB[rl * LDB + lane + 64 * q] = gv * sbv[q];
        csb_b[q] += gv;
        csb_s[q] += gv * (st.zb[m][q] + bbv[q]);  // bbv = 0 unless the output layer
      }
    }
    __syncthreads();
    if (r0 + SR < r_end) issue(r0 + SR, st);  // in flight during the MFMA phase
    const int kk = lane >> 4, ii = lane & 15;
#pragma unroll
    for (int ks = 0; ks < SR / 4; ++ks) {
      T bf[NTJ], af[NTI];
#pragma unroll
      for (int jj = 0; jj < NTJ; ++jj) bf[jj] = sB[(4 * ks + kk) * LDB + (wj + WJ * jj) * 16 + ii];
#pragma unroll
      for (int ti = 0; ti < NTI; ++ti) af[ti] = sA[(4 * ks + kk) * LDA + (wi + WI * ti) * 16 + ii];
#pragma unroll
      for (int ti = 0; ti < NTI; ++ti)
#pragma unroll
        for (int jj = 0; jj < NTJ; ++jj) acc[ti][jj] = MF::mma(af[ti], bf[jj], acc[ti][jj]);
    }
  }

  // ---- this chunk's partial dW_l ----
  T* part = a.part + chunk * a.ptot;
#pragma unroll
  for (int ti = 0; ti < NTI; ++ti) {
#pragma unroll
    for (int jj = 0; jj < NTJ; ++jj) {
      const int h = col0 + (wj + WJ * jj) * 16 + (lane & 15);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int k = (wi + WI * ti) * 16 + MF::row(lane, v);
        if (k < K && h < H) part[a.off_W[l] + (int64_t)k * H + h] = acc[ti][jj][v];
      }
    }
  }
  // ---- BN column sums: combine the 4 wavefronts (row phases) through LDS ----
  __syncthreads();  // LDS reuse
  T* red = sA;  // [4 waves][2][64*QB] (B side), then [4 waves][2][64] (BN_0)
  constexpr int RW = 64 * QB;
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    red[(wave * 2 + 0) * RW + lane + 64 * q] = csb_b[q];
    red[(wave * 2 + 1) * RW + lane + 64 * q] = csb_s[q];
  }
  T* red0 = sA + 8 * RW;
  red0[(wave * 2 + 0) * 64 + lane] = cs0_b;
  red0[(wave * 2 + 1) * 64 + lane] = cs0_s;
  __syncthreads();
  if (tid < CW && col0 + tid < H) {
    T sb = 0, ss = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red[(w * 2 + 0) * RW + tid];
      ss += red[(w * 2 + 1) * RW + tid];
    }
    part[a.off_beta[l + 1] + col0 + tid] = sb;
    part[a.off_gamma[l + 1] + col0 + tid] = ss;
  }
  if (first && tid < K) {
    T sb = 0, ss = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red0[(w * 2 + 0) * 64 + tid];
      ss += red0[(w * 2 + 1) * 64 + tid];
    }
    part[a.off_beta[0] + tid] = sb;
    part[a.off_gamma[0] + tid] = ss;
  }
}

// out[p] = Σ_c part[c][p]; gamma entries times rs; the bias gradient db = s_{L+1} ⊙ dbeta_{L+1}
// appended at out[ptot ...].  A workgroup owns kRedCols consecutive entries; its kRedSlices
// wavefront halves each sum the chunks c ≡ slice (mod kRedSlices), 8 loads in flight, and the
// slices are added in slice order through LDS (a fixed order: deterministic).  One thread per
// entry summing all chunks in turn waited out nchunks / 8 load latencies (tens of µs at 256
// chunks, the V network's reduce on the critic's critical path).
constexpr int kRedCols = 32, kRedSlices = 8;  // 256 threads
template <typename T>
__global__ __launch_bounds__(256) void k_param_grads_reduce(const PgArgs<T> a, int nchunks,
                                                            T gamma_scale, T* out) {
  // a deferred fallback's reduce (dpac.h guard_phase 2): only once an x3 kernel fell back
  if (a.guard && !x3_status_set(a.guard)) return;
  __shared__ T s_part[kRedSlices][kRedCols];
  const int col = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int64_t p = (int64_t)blockIdx.x * kRedCols + col;
  const int L = a.L, Hout = a.width[L + 1];
  const bool valid = p < a.ptot + Hout;
  const bool is_b = p >= a.ptot;
  const int64_t src = !valid ? 0 : is_b ? a.off_beta[L + 1] + (p - a.ptot) : p;
  const T* col_p = a.part + src;
  T s = 0;
  if (valid) {
    int c = sl;
    for (; c + 7 * kRedSlices < nchunks; c += 8 * kRedSlices) {  // 8 loads in flight
      T v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = col_p[(int64_t)(c + u * kRedSlices) * a.ptot];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
    for (; c < nchunks; c += kRedSlices) s += col_p[(int64_t)c * a.ptot];
  }
  s_part[sl][col] = s;
  __syncthreads();
  if (sl != 0 || !valid) return;
  s = s_part[0][col];
#pragma unroll
  for (int k = 1; k < kRedSlices; ++k) s += s_part[k][col];
  if (is_b) {
    s = a.scale[L + 1][p - a.ptot] * s;
  } else if (p < a.off_beta[0]) {  // gamma block comes first
    s = gamma_scale * s;
  }
  out[p] = s;
}

}  // namespace dpac
