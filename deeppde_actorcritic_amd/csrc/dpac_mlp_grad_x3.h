// dpac_mlp_grad_x3.h — k_param_grads (dpac_mlp_grad.h) on split-fp16 MFMA, for float
// networks whose caller asked for split-fp16 products (dpac_mlp.weight_x3 given).
//
// The same sums as k_param_grads (the trainable-variable gradients of DeepNN, solver.py:
// 227-278, as the GradientTape of solver.py:88,95 forms them):
//   dW_l = Σ_r a_l[r]^T (G_{l+1}[r] ⊙ s_{l+1}),  dbeta_i = Σ_r G_i[r],  dgamma_i = rs Σ_r G_i ⊙ zin_i
// with the reduction over rows as the MFMA's K dimension: one v_mfma_f32_16x16x32_f16 step
// covers 32 rows.  Operands are split as in dpac_mlp_x3.h (a = hi + lo 2^-12, three MFMAs
// hi*hi, hi*lo, lo*hi accumulated in f32), so every product is the f32 product
// to within the f32 accumulation error; the BN column sums stay plain f32 adds.
// Gradients are small (O(1/B) and far below it in early steps and inner layers), and a value
// under fp16's normal range (6.1e-5) keeps only an ABSOLUTE error of ~2^-37 through its lo
// half, so the B operand (G ⊙ s) carries a per-column power of two: each sub-chunk's column
// max raises a running exponent E_c, the column is staged times 2^(3 - E_c) (|values| < 8),
// the lane's accumulator of that column is rescaled by 2^(E_old - E_new) when E_c rises
// (exact), and the partial is unscaled by 2^(E_c - 3) when written.  (A per-row scale, as the
// backward chains use, cannot be undone after a reduction over rows.)  With |B| < 8 the three
// products share ONE accumulator: acc += A_hi (2^12 B_hi) + A_hi B_lo + A_lo B_hi (= 2^12 A B;
// 2^12 B_hi < 32768 is an exact fp16 number), half the accumulator registers of two chains.
//
// Workgroup (chunk c, column group g, layer l) = 8 wavefronts; a sub-chunk of 32 rows is
// staged through LDS per step:
//  * staging: thread (rb = tid / 128, f = tid % 128) loads rows 8 rb .. 8 rb + 7 of A feature
//    f (+128) and of B column f (+128) — coalesced dword loads along the row — applies BN and the
//    activation (A) or the BN scale (B), splits, and writes each 8-row run as ONE 16-byte LDS
//    write per part: the images are [part][row block][feature][8 rows] halves, which is
//    exactly the MFMA fragment order (lane l reads feature l & 15, row block l >> 4), so a
//    fragment read is 4 runs of 256 contiguous bytes;
//  * MFMA: wave (wi, wj) of a WI x WJ grid owns row tiles wi + WI ti (features of layer l)
//    and column tiles wj + WJ jj of the group.  Wide layers: WI = 1, WJ = 8, one column tile
//    per wave (CW = 128 columns, 2 groups at H = 200; NTJ = 2 would stage A once per chunk
//    but needs > 256 VGPRs at 13 input tiles); outputs of <= 32 columns: WI = 8, WJ = 1 (the
//    waves split the row tiles).
// Partials go to the same [chunk][ptot] layout k_param_grads_reduce sums.
#pragma once

#include "dpac_mlp_grad.h"

namespace dpac {

typedef _Float16 pgh8 __attribute__((ext_vector_type(8)));
typedef float pgf4 __attribute__((ext_vector_type(4)));

constexpr int kPgxThreads = 512;
constexpr int kPgxWaves = 8;
constexpr int kPgxSR = 32;  // rows per sub-chunk = the MFMA's K
#ifndef DPAC_PGX_DEPTH
#define DPAC_PGX_DEPTH 1  // register stages of loads in flight (2 measured: no gain, 0.628 vs 0.628 ms at 204 800 rows)
#endif
constexpr int kPgxDepth = DPAC_PGX_DEPTH;
#ifndef DPAC_PGX_ROWDESC
#define DPAC_PGX_ROWDESC 0  // timing knob: per-row buffer descriptors in the staging loads
#endif
static_assert(kPgxDepth == 1 || kPgxDepth == 2, "1 or 2 stages");
constexpr float kPgxLo = 4096.f, kPgxLoInv = 1.f / 4096.f;
#ifndef DPAC_PGW_EARLY
#define DPAC_PGW_EARLY 1  // issue the next sub-chunk's loads before the column scaling (round 6)
#endif

// staged values of one sub-chunk (registers; loaded before the previous sub-chunk's MFMAs)
template <int QA, int QB, bool L0>
struct PgxStage {
  float a[QA][8];             // zin_l at rows 8 rb + i, features f + 128 q
  float g0[L0 ? QA : 1][8];   // layer 0: G_0 at the same places (BN_0 sums)
  float gb[QB][8];            // G_{l+1} at columns col0 + f + 128 q
  float zb[QB][8];            // zin_{l+1} (pre-bias) at the same places
};

__device__ __forceinline__ void pgx_split8(const float (&v)[8], pgh8& h, pgh8& l) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    h[i] = (_Float16)v[i];
    l[i] = (_Float16)((v[i] - (float)h[i]) * kPgxLo);
  }
}

// The layout of one workgroup of NW wavefronts (8: 512 threads; a 16-wavefront register-staged
// build spilled, round 4: the wide layers' one-group kernel is k_param_grads_x3w below).
// Shared with the host (dynamic LDS size).
template <int NTI, int NTJ, int WI, bool L0, int NW>
struct PgxPlan {
  static constexpr int kThreads = 64 * NW;
  static constexpr int FL = kThreads / 4;               // staging threads per 8-row block
  static constexpr int WJ = NW / WI;
  static constexpr int CW = 16 * NTJ * WJ;             // B columns per workgroup (<= 256)
  static constexpr int KP = 16 * NTI * WI;             // staged A features
  static constexpr int QA = (KP + FL - 1) / FL;        // A features per staging thread
  static constexpr int QB = (CW + FL - 1) / FL;        // B columns per staging thread
  // LDS: the images, halves A [2 parts][4 row blocks][KP][8], B [3][4][CW][8] (hi, lo,
  // 2^12 hi); after the row loop the same bytes hold the BN column sums' reduction ([4 rb][2][CW]
  // floats for the B side, then [4 rb][2][FL QA] for BN_0 on the input layer); then the column
  // scaling: sub-chunk maxima [4 rb][CW], rescale factors [CW], exponents [CW]
  static constexpr int kImgBytes = (2 * KP + 3 * CW) * 4 * 8 * 2;
  static constexpr int kRedFloats = 4 * 2 * CW + (L0 ? 4 * 2 * FL * QA : 0);
  static constexpr int kMain = kImgBytes > kRedFloats * 4 ? kImgBytes : kRedFloats * 4;
  static constexpr int kSmem = kMain + (4 * CW + 2 * CW) * 4;
};

// One workgroup's work: chunk `chunk` of the rows, column group `grp` of layer l (the kernel
// k_param_grads_x3 below with its block indices; k_param_grads_x3_seg runs several layers'
// grids in one launch).
template <int NTI, int NTJ, int WI, bool L0, int NW = kPgxWaves>
__device__ __forceinline__ void pgx_body(const PgArgs<float>& a, const int l, const int64_t chunk, const int grp) {
  using PL = PgxPlan<NTI, NTJ, WI, L0, NW>;
  constexpr int WJ = PL::WJ, CW = PL::CW, KP = PL::KP, QA = PL::QA, QB = PL::QB, FL = PL::FL;
  static_assert(CW <= 256 && KP <= DPAC_MLP_MAX_WIDTH, "staging map: 256 columns, 256 features");
  static_assert(CW <= PL::kThreads, "one thread per column in the BN sums' reduction");
  constexpr int kMain = PL::kMain;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // PL::kSmem bytes (dynamic)
  _Float16* const sA = reinterpret_cast<_Float16*>(smem);
  _Float16* const sB = sA + 2 * 4 * KP * 8;
  float* const s_cmax = reinterpret_cast<float*>(smem + kMain);
  float* const s_cfac = s_cmax + 4 * CW;
  int* const s_cexp = reinterpret_cast<int*>(s_cfac + CW);
  if (x3_status_set(a.status)) return;  // fell back: the f32 kernel after this one does the work
  bool bad = false;  // a split operand outside the range (dpac.h dpac_mlp.status)
  const int K = a.width[l], H = a.width[l + 1];
  const int col0 = grp * CW;
  if (col0 >= H) return;  // whole workgroup, before any barrier
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wi = wave / WJ, wj = wave % WJ;
  const int rb = tid / FL, fl = tid % FL;
  static_assert(FL % 64 == 0, "a wave's lanes share one row block");
  const int rbu = __builtin_amdgcn_readfirstlane(rb);
  (void)rbu;
  const int64_t r_begin = chunk * a.rows_per_chunk;
  const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
  const bool first = L0 && grp == 0;  // also sums BN_0 (L0: l == 0)
  const bool last = l == a.L;             // zin_{L+1} = z_{L+1} + bias
  const float* srcA = l == 0 ? a.x : a.z + a.zoff[l];
  const int64_t ldA = l == 0 ? a.ldx : a.ztot;
  const float* gA = a.G + a.goff[0];
  const float* gB = a.G + a.goff[l + 1] + col0;
  const float* zB = a.z + a.zoff[l + 1] + col0;

  // per-thread constants: A features fl + 128 q, B column col0 + fl
  float sa[QA], ha[QA];
  uint32_t offA[QA], offG0[QA];
#pragma unroll
  for (int q = 0; q < QA; ++q) {
    const int k = fl + FL * q;
    const bool v = k < K;
    sa[q] = v ? a.scale[l][k] : 0.f;
    ha[q] = v ? a.shift[l][k] : 0.f;
    offA[q] = v ? (uint32_t)k * 4u : kOOB;
    offG0[q] = (v && first) ? (uint32_t)k * 4u : kOOB;
  }
  float sbv[QB], bbv[QB], csb_b[QB], csb_s[QB];
  uint32_t offB[QB];
  int cexp[QB];  // the columns' running exponents (B staging threads)
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const int c = fl + FL * q, hcol = col0 + c;
    const bool bv = c < CW && hcol < H;
    sbv[q] = bv ? a.scale[l + 1][hcol] : 0.f;
    bbv[q] = (bv && last) ? a.bias[hcol] : 0.f;
    offB[q] = bv ? (uint32_t)c * 4u : kOOB;
    csb_b[q] = csb_s[q] = 0.f;
    cexp[q] = -100;
  }
  float cs0_b[QA], cs0_s[QA];
#pragma unroll
  for (int q = 0; q < QA; ++q) cs0_b[q] = cs0_s[q] = 0.f;
  pgf4 acc[NTI][NTJ];  // 2^12 x (the column-scaled) dW tile
#pragma unroll
  for (int ti = 0; ti < NTI; ++ti)
#pragma unroll
    for (int jj = 0; jj < NTJ; ++jj) acc[ti][jj] = pgf4{0.f, 0.f, 0.f, 0.f};

#if DPAC_PGX_ROWDESC
  // loads of the 32 rows at r0: one descriptor per row (wave-uniform: a wave's lanes share
  // rb), based at the row and sized to it (0 past the chunk's end, so those rows read 0 and
  // add nothing); the lane offsets are the column offsets alone, so no per-row VGPR offsets
  // are hoisted out of the row loop (208 -> 180 VGPRs for the wide layers)
  auto issue = [&](int64_t r0, PgxStage<QA, QB, L0>& st) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = r0 + 8 * rbu + i;
      const bool in = row < r_end;
      const auto rA = make_rsrc(srcA + row * ldA, in ? (uint32_t)K * 4u : 0u);
      const auto rG = make_rsrc(gA + row * a.gtot, (in && L0) ? (uint32_t)K * 4u : 0u);
      const auto rB = make_rsrc(gB + row * a.gtot, in ? (uint32_t)(H - col0) * 4u : 0u);
      const auto rZ = make_rsrc(zB + row * a.ztot, in ? (uint32_t)(H - col0) * 4u : 0u);
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        st.a[q][i] = buf_load_elem<float>(rA, offA[q]);
        if constexpr (L0) st.g0[q][i] = first ? buf_load_elem<float>(rG, offG0[q]) : 0.f;
      }
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        st.gb[q][i] = buf_load_elem<float>(rB, offB[q]);
        st.zb[q][i] = buf_load_elem<float>(rZ, offB[q]);
      }
    }
  };
#else
  // loads of the 32 rows at r0: descriptors based at row r0 ending at the chunk's last row
  // (rows past it read 0, so their G is 0 and they add nothing); masked columns carry kOOB
  auto issue = [&](int64_t r0, PgxStage<QA, QB, L0>& st) {
    const int64_t nr = r_end - r0;  // >= 1
    const auto rA = make_rsrc(srcA + r0 * ldA, (uint32_t)(((nr - 1) * ldA + K) * 4));
    const auto rG = make_rsrc(gA + r0 * a.gtot, (uint32_t)(((nr - 1) * a.gtot + K) * 4));
    const auto rB = make_rsrc(gB + r0 * a.gtot, (uint32_t)(((nr - 1) * a.gtot + (H - col0)) * 4));
    const auto rZ = make_rsrc(zB + r0 * a.ztot, (uint32_t)(((nr - 1) * a.ztot + (H - col0)) * 4));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint32_t r = (uint32_t)(8 * rb + i);
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        st.a[q][i] = buf_load_elem<float>(rA, offA[q] + r * (uint32_t)ldA * 4u);
        if constexpr (L0) st.g0[q][i] = first ? buf_load_elem<float>(rG, offG0[q] + r * (uint32_t)a.gtot * 4u) : 0.f;
      }
#pragma unroll
      for (int q = 0; q < QB; ++q) {
        st.gb[q][i] = buf_load_elem<float>(rB, offB[q] + r * (uint32_t)a.gtot * 4u);
        st.zb[q][i] = buf_load_elem<float>(rZ, offB[q] + r * (uint32_t)a.ztot * 4u);
      }
    }
  };
#endif

  const int fq = lane >> 4, fi = lane & 15;  // fragment: row block, feature / column in the tile
  // one sub-chunk of 32 rows from its staged registers `st`, which are then refilled with
  // the sub-chunk kPgxDepth ahead (kPgxDepth register stages in flight)
  auto sub = [&](int64_t r0, PgxStage<QA, QB, L0>& st) {
    __syncthreads();  // the previous sub-chunk's fragment reads are done
#pragma unroll
    for (int q = 0; q < QA; ++q) {
      const int k = fl + FL * q;
      if (k >= KP) continue;  // compile-time for q = 0 when KP >= FL
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float zi = st.a[q][i];
        const float y = ha[q] + zi * sa[q];  // the forward's expression (FwdEpi / write_a0)
        v[i] = k < K ? (l == 0 ? y : y + fmaxf(y, 0.f)) : 0.f;  // rows past the end: a = shift,
        if constexpr (L0) {                                       // masked by G = 0
          cs0_b[q] += st.g0[q][i];
          cs0_s[q] += st.g0[q][i] * zi;
        }
      }
      pgh8 h, lo;
      pgx_split8(v, h, lo);
      bad |= x3_bad4(v[0], v[1], v[2], v[3]) | x3_bad4(v[4], v[5], v[6], v[7]);
      *reinterpret_cast<pgh8*>(sA + ((0 * 4 + rb) * KP + k) * 8) = h;
      *reinterpret_cast<pgh8*>(sA + ((1 * 4 + rb) * KP + k) * 8) = lo;
    }
    float vb[QB][8];
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int c = fl + FL * q;
      if (c >= CW) continue;  // compile-time for q = 0 when CW >= FL
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gv = st.gb[q][i];
        vb[q][i] = gv * sbv[q];
        m = fmaxf(m, fabsf(vb[q][i]));
        csb_b[q] += gv;
        csb_s[q] += gv * (st.zb[q][i] + bbv[q]);  // bbv = 0 unless the output layer
      }
      s_cmax[rb * CW + c] = m;
    }
    // round 6: the register stage is consumed (A into the image, B into vb and the sums), so the
    // sub-chunk kPgxDepth ahead is issued now, under the column scaling as well as the MFMAs
    if (DPAC_PGW_EARLY && r0 + kPgxDepth * kPgxSR < r_end) issue(r0 + kPgxDepth * kPgxSR, st);
    __syncthreads();  // the column maxima of the sub-chunk
#pragma unroll
    for (int q = 0; q < QB; ++q) {
      const int c = fl + FL * q;
      if (c >= CW) continue;
      const float m = fmaxf(fmaxf(s_cmax[c], s_cmax[CW + c]), fmaxf(s_cmax[2 * CW + c], s_cmax[3 * CW + c]));
      int e = cexp[q];
      if (m > 0.f && m < 3.0e38f) {
        int em = 0;
        (void)frexpf(m, &em);  // m in [2^(em-1), 2^em)
        e = em > cexp[q] ? em : cexp[q];
      }
      const float sc = ldexpf(1.f, 3 - e);  // the column's values times sc: |v| < 8
#pragma unroll
      for (int i = 0; i < 8; ++i) vb[q][i] *= sc;
      pgh8 h, lo, h12;
      pgx_split8(vb[q], h, lo);
      bad |= x3_bad4(vb[q][0], vb[q][1], vb[q][2], vb[q][3]) | x3_bad4(vb[q][4], vb[q][5], vb[q][6], vb[q][7]);
#pragma unroll
      for (int i = 0; i < 8; ++i) h12[i] = h[i] * (_Float16)kPgxLo;  // exact: |h| < 8
      *reinterpret_cast<pgh8*>(sB + ((0 * 4 + rb) * CW + c) * 8) = h;
      *reinterpret_cast<pgh8*>(sB + ((1 * 4 + rb) * CW + c) * 8) = lo;
      *reinterpret_cast<pgh8*>(sB + ((2 * 4 + rb) * CW + c) * 8) = h12;
      if (rb == 0) {
        s_cfac[c] = ldexpf(1.f, cexp[q] - e);  // the accumulated column, to the new scale (exact)
        s_cexp[c] = e;
      }
      cexp[q] = e;
    }
    __syncthreads();
    if (!DPAC_PGW_EARLY && r0 + kPgxDepth * kPgxSR < r_end) issue(r0 + kPgxDepth * kPgxSR, st);  // lands kPgxDepth sub-chunks later
    pgh8 bh[NTJ], bl[NTJ], b12[NTJ];
#pragma unroll
    for (int jj = 0; jj < NTJ; ++jj) {
      const int c = (wj + WJ * jj) * 16 + fi;
      bh[jj] = *reinterpret_cast<const pgh8*>(sB + ((0 * 4 + fq) * CW + c) * 8);
      bl[jj] = *reinterpret_cast<const pgh8*>(sB + ((1 * 4 + fq) * CW + c) * 8);
      b12[jj] = *reinterpret_cast<const pgh8*>(sB + ((2 * 4 + fq) * CW + c) * 8);
      const float f = s_cfac[c];
      if (__any(f != 1.f)) {  // a column's exponent rose: rescale what it accumulated
#pragma unroll
        for (int ti = 0; ti < NTI; ++ti) acc[ti][jj] *= f;
      }
    }
    auto fragA = [&](int ti, int part) {
      const int k = (wi + WI * ti) * 16 + fi;
      return *reinterpret_cast<const pgh8*>(sA + ((part * 4 + fq) * KP + k) * 8);
    };
    pgh8 xh = fragA(0, 0), xl = fragA(0, 1);
#pragma unroll
    for (int ti = 0; ti < NTI; ++ti) {  // A fragments one tile ahead (pinned: not all hoisted)
      pgh8 nh = xh, nl = xl;
      if (ti + 1 < NTI) {
        nh = fragA(ti + 1, 0);
        nl = fragA(ti + 1, 1);
      }
#pragma unroll
      for (int jj = 0; jj < NTJ; ++jj) {
        acc[ti][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, b12[jj], acc[ti][jj], 0, 0, 0);
        acc[ti][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, bl[jj], acc[ti][jj], 0, 0, 0);
        acc[ti][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, bh[jj], acc[ti][jj], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      xh = nh;
      xl = nl;
    }
  };
  PgxStage<QA, QB, L0> st0;
  issue(r_begin, st0);
  if constexpr (kPgxDepth == 1) {
    for (int64_t r0 = r_begin; r0 < r_end; r0 += kPgxSR) sub(r0, st0);
  } else {
    PgxStage<QA, QB, L0> st1;
    if (r_begin + kPgxSR < r_end) issue(r_begin + kPgxSR, st1);
    for (int64_t r0 = r_begin; r0 < r_end; r0 += 2 * kPgxSR) {
      sub(r0, st0);
      if (r0 + kPgxSR < r_end) sub(r0 + kPgxSR, st1);
    }
  }

  // ---- this chunk's partial dW_l: lane holds features 4 fq .. +3 of its row tile, column fi ----
  float* part = a.part + chunk * a.ptot;
#pragma unroll
  for (int ti = 0; ti < NTI; ++ti) {
#pragma unroll
    for (int jj = 0; jj < NTJ; ++jj) {
      const int h = col0 + (wj + WJ * jj) * 16 + fi;
      // undo 2^12 and the column scale 2^(3 - E_c)
      const float us = ldexpf(1.f, s_cexp[(wj + WJ * jj) * 16 + fi] - 3 - 12);
      const pgf4 c = acc[ti][jj] * us;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int k = (wi + WI * ti) * 16 + 4 * fq + v;
        if (k < K && h < H) part[a.off_W[l] + (int64_t)k * H + h] = c[v];
      }
    }
  }
  // ---- BN column sums: combine the 4 row blocks through LDS (reusing the images) ----
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  float* red0 = red + 4 * 2 * CW;
#pragma unroll
  for (int q = 0; q < QB; ++q) {
    const int c = fl + FL * q;
    if (c < CW) {
      red[(rb * 2 + 0) * CW + c] = csb_b[q];
      red[(rb * 2 + 1) * CW + c] = csb_s[q];
    }
  }
  if constexpr (L0) {
    if (first) {
#pragma unroll
      for (int q = 0; q < QA; ++q) {
        red0[(rb * 2 + 0) * FL * QA + fl + FL * q] = cs0_b[q];
        red0[(rb * 2 + 1) * FL * QA + fl + FL * q] = cs0_s[q];
      }
    }
  }
  __syncthreads();
  if (tid < CW && col0 + tid < H) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red[(w * 2 + 0) * CW + tid];
      ss += red[(w * 2 + 1) * CW + tid];
    }
    part[a.off_beta[l + 1] + col0 + tid] = sb;
    part[a.off_gamma[l + 1] + col0 + tid] = ss;
  }
  if (L0 && first && tid < K && tid < FL * QA) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red0[(w * 2 + 0) * FL * QA + tid];
      ss += red0[(w * 2 + 1) * FL * QA + tid];
    }
    part[a.off_beta[0] + tid] = sb;
    part[a.off_gamma[0] + tid] = ss;
  }
  if (bad) x3_flag(a.status);
}


// ---------------------------------------------------------------------------------------------
// k_param_grads_x3w: the wide hidden layers (K in (32, 208], H in (32, 256], l >= 1) and the
// input layer into a wide layer (L0: K <= 32, A = the network input, plus BN_0's sums from G_0)
// with ONE 256-column group per chunk, so the A operand is read once per chunk instead of once
// per 128-column group (round 4; the two-group kernel read 0.78 GB per 204 800-row layer for
// 0.49 GB of A, G and z).  The same sums, splits, column scaling and partial layout as
// k_param_grads_x3, in the same order: bitwise its results.
//
// 16 wavefronts (1 024 threads, one column tile each).  A 1 024-thread workgroup has 128 VGPRs
// per lane, too few to hold the 13 accumulator tiles AND a register stage of A, G and z (the
// register-staged 16-wave build spilled).  So z_l (A) and z_{l+1} (for the BN scale sums) reach
// LDS by LDS-DMA (global_load_lds_dwordx4, one instruction per row and wavefront: 32 rows over
// 16 wavefronts), and only G_{l+1} goes through registers (8 per lane).  Rows past the chunk's
// end DMA the chunk's last row again (finite values; their G loads read 0, so they add nothing).
// LDS: images A [2][4][KP][8] + B [3][4][256][8] halves, raw A and raw z [32][256] floats, the
// column maxima / factors / exponents: 145 KB at KP = 208.
// Requires 16-byte aligned rows: ztot, zoff[l], zoff[l+1] multiples of 4 (launch() checks).
constexpr int kPgwThreads = 1024;
constexpr int kPgwCW = 256;
template <int NTI, int NTJ, int WI, bool L0, int NW = kPgxWaves>
__global__ __launch_bounds__(64 * NW) void k_param_grads_x3(const PgArgs<float> a, const int l) {
  pgx_body<NTI, NTJ, WI, L0, NW>(a, l, blockIdx.x, blockIdx.y);
}

// Several layers' grids of the 8-wavefront split-fp16 kernel in ONE launch (round 6): segment
// i runs layer s[i].l with configuration s[i].cfg over blocks [s[i].b0, s[i].b0 + nch * ngrp),
// chunk-major.  For small row counts (the critic's V network over 3 B rows: 24 chunks) each
// layer's grid covers a fraction of the CUs and its launch is latency-bound, so the layers run
// side by side instead of one after another; every layer writes its own partial columns.
enum PgxCfg : int {
  kPgxIn1 = 0, kPgxIn2, kPgxW1, kPgxW2, kPgxW4, kPgxW8, kPgxW13, kPgxN11, kPgxN12, kPgxN21, kPgxN22, kPgxNCfg
};
struct PgxSeg {
  int l, cfg, ngrp;
  int64_t b0;
};
struct PgxSegs {
  int n;
  PgxSeg s[DPAC_MLP_MAX_HIDDEN + 1];
};
template <int CFG>
struct PgxCfgT;
template <> struct PgxCfgT<kPgxIn1> { using PL = PgxPlan<1, 1, 1, true, kPgxWaves>; };
template <> struct PgxCfgT<kPgxIn2> { using PL = PgxPlan<2, 1, 1, true, kPgxWaves>; };
template <> struct PgxCfgT<kPgxW1> { using PL = PgxPlan<1, 1, 1, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxW2> { using PL = PgxPlan<2, 1, 1, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxW4> { using PL = PgxPlan<4, 1, 1, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxW8> { using PL = PgxPlan<8, 1, 1, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxW13> { using PL = PgxPlan<13, 1, 1, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxN11> { using PL = PgxPlan<1, 1, 8, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxN12> { using PL = PgxPlan<1, 2, 8, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxN21> { using PL = PgxPlan<2, 1, 8, false, kPgxWaves>; };
template <> struct PgxCfgT<kPgxN22> { using PL = PgxPlan<2, 2, 8, false, kPgxWaves>; };
// the configurations k_param_grads_x3_seg runs
inline bool pgx_seg_cfg_ok(int cfg) {
  return cfg == kPgxIn1 || cfg == kPgxIn2 || cfg == kPgxW13 || cfg == kPgxN11 || cfg == kPgxN21;
}
// the dynamic LDS of a configuration (host)
inline int pgx_cfg_smem(int cfg) {
  switch (cfg) {
    case kPgxIn1: return PgxCfgT<kPgxIn1>::PL::kSmem;
    case kPgxIn2: return PgxCfgT<kPgxIn2>::PL::kSmem;
    case kPgxW1: return PgxCfgT<kPgxW1>::PL::kSmem;
    case kPgxW2: return PgxCfgT<kPgxW2>::PL::kSmem;
    case kPgxW4: return PgxCfgT<kPgxW4>::PL::kSmem;
    case kPgxW8: return PgxCfgT<kPgxW8>::PL::kSmem;
    case kPgxW13: return PgxCfgT<kPgxW13>::PL::kSmem;
    case kPgxN11: return PgxCfgT<kPgxN11>::PL::kSmem;
    case kPgxN12: return PgxCfgT<kPgxN12>::PL::kSmem;
    case kPgxN21: return PgxCfgT<kPgxN21>::PL::kSmem;
    default: return PgxCfgT<kPgxN22>::PL::kSmem;
  }
}

__global__ __launch_bounds__(64 * kPgxWaves) void k_param_grads_x3_seg(const PgArgs<float> a, const PgxSegs sg) {
  const int64_t b = blockIdx.x;
  int i = 0;
  while (i + 1 < sg.n && b >= sg.s[i + 1].b0) ++i;  // segments in block order
  const PgxSeg& g = sg.s[i];
  const int64_t r = b - g.b0;
  const int64_t chunk = r / g.ngrp;
  const int grp = (int)(r - chunk * g.ngrp);
  switch (g.cfg) {  // the critic V network's shapes (pgx_seg_cfg_ok); more cases spill
    case kPgxIn1: pgx_body<1, 1, 1, true>(a, g.l, chunk, grp); break;
    case kPgxIn2: pgx_body<2, 1, 1, true>(a, g.l, chunk, grp); break;
    case kPgxW13: pgx_body<13, 1, 1, false>(a, g.l, chunk, grp); break;
    case kPgxN11: pgx_body<1, 1, 8, false>(a, g.l, chunk, grp); break;
    default: pgx_body<2, 1, 8, false>(a, g.l, chunk, grp); break;
  }
}

template <int NTI, bool L0 = false>
struct PgwPlan {
  static constexpr int KP = 16 * NTI;
  static constexpr int kImgA = 2 * 4 * KP * 8 * 2;           // bytes
  static constexpr int kImgB = 3 * 4 * kPgwCW * 8 * 2;
  static constexpr int kRaw = kPgxSR * kPgwCW * 4;            // one raw [32][256] float block
  static constexpr int kRawA = kImgA + kImgB;
  static constexpr int kRawZ = kRawA + kRaw;
  static constexpr int kRawG0 = kRawZ + kRaw;                 // L0: G_0 rows (the BN_0 sums)
  static constexpr int kCol = kRawG0 + (L0 ? kRaw : 0);       // s_cmax [4][256], s_cfac, s_cexp
  static constexpr int kSmem = kCol + (4 * kPgwCW + 2 * kPgwCW) * 4;
  static_assert(4 * 2 * kPgwCW * 4 + 4 * 2 * KP * 4 <= kRawA, "BN sums' reduction fits the image bytes");
  static_assert(kSmem <= 160 * 1024, "LDS");
};

// One wavefront copies one row (bytes <= 1 024, a multiple of 16) from global src to LDS dst
// with global_load_lds_dwordx4: lane l moves bytes [16 l, 16 l + 16); lanes past the end read
// the row's first 16 bytes again (in bounds) into their own slot of the 1 KB destination.
// Inline asm (M0 holds the LDS base): the compiler cannot see the LDS write, so the caller
// waits with s_waitcnt vmcnt(0) before the barrier that publishes the row.
// The row address is wave-uniform (an SGPR pair, the saddr form); the lane's 32-bit offset
// `voff` (16 l, or 0 past the row's end) is the only VGPR operand.
__device__ __forceinline__ uint32_t pgw_lane_off(uint32_t bytes, int lane) {
  const uint32_t off = (uint32_t)lane * 16u;
  return off < bytes ? off : 0u;
}
__device__ __forceinline__ void pgw_row_dma(const float* src, uint32_t voff, unsigned char* dst) {
  const uint32_t m0 = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)dst);
  // readfirstlane returns int: widen through uint32_t (a sign-extended low word would set the
  // high 32 bits of the address)
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)src);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)((uintptr_t)src >> 32));
  const uint64_t base = lo | (hi << 32);
  int keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %3\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(m0), "s"(base) : "memory");
}

// The same copy of a row of at most 128 bytes into a compact 128-byte slot: only the lanes
// inside the row (and lane 0) issue, so nothing lands past dst + 128.
__device__ __forceinline__ void pgw_row_dma_128(const float* src, uint32_t bytes, int lane, unsigned char* dst) {
  if ((uint32_t)lane * 16u < bytes || lane == 0) pgw_row_dma(src, (uint32_t)lane * 16u, dst);
}
constexpr int kPgwRawG0c = kPgxSR * 128;  // merged launches: G_0 rows in compact 128-byte slots (K <= 32)

// lsel >= 0: layer lsel, chunk blockIdx.x.  lsel < 0 (round 5, L0 = false): -lsel = l0 + 8 nl,
// layers l0 .. l0 + nl - 1 in ONE launch, XCD-aware: each group of 8 nl workgroups holds 8 chunks
// x the nl layers, and a chunk's workgroups are 8 apart (the dispatcher deals workgroups
// round-robin over the 8 XCDs, so they share an XCD and run together): z_{l+1}, layer l's BN
// operand and layer l+1's A, is read by both at about the same time and the second read can hit
// L2 / the Infinity Cache.  A merged launch may start at the input layer (l0 = 0, K <= 32): its
// workgroups run the L0 variant's arithmetic at run time (BN_0 only, BN_0's sums from G_0 rows,
// which land in compact slots after the plan's LDS: the launch adds kPgwRawG0c bytes), bitwise
// k_param_grads_x3w<NTI, true>'s results.
// MODE 0: one layer (lsel >= 0); 1: a merged launch of wide / output layers; 2: a merged launch
// that starts at the input layer (run-time L0 workgroups).  Separate instantiations: the run-time
// L0 state costs registers the one-layer kernel does not have to spare (128 VGPRs at 1 024
// threads; round 5 measured a 54-VGPR spill when every launch carried it).
template <int NTI, bool L0 = false, int MODE = 0>
__global__ __launch_bounds__(kPgwThreads) void k_param_grads_x3w(const PgArgs<float> a, const int lsel) {
  using PL = PgwPlan<NTI, L0>;
  static_assert(MODE == 0 || !L0, "merged launches use the run-time input layer");
  constexpr int KP = PL::KP, CW = kPgwCW;
  static_assert(KP <= 256, "one staging thread per feature");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // PL::kSmem bytes (dynamic)
  _Float16* const sA = reinterpret_cast<_Float16*>(smem);
  _Float16* const sB = reinterpret_cast<_Float16*>(smem + PL::kImgA);
  const float* const rawA = reinterpret_cast<const float*>(smem + PL::kRawA);
  const float* const rawZ = reinterpret_cast<const float*>(smem + PL::kRawZ);
  float* const s_cmax = reinterpret_cast<float*>(smem + PL::kCol);
  float* const s_cfac = s_cmax + 4 * CW;
  int* const s_cexp = reinterpret_cast<int*>(s_cfac + CW);
  if (x3_status_set(a.status)) return;  // fell back: the f32 kernel after this one does the work
  const int64_t bx = blockIdx.x;
  const int nl = MODE == 0 ? 1 : (-lsel) >> 3;
  const int l = MODE == 0 ? lsel : ((-lsel) & 7) + (int)((bx >> 3) % nl);
  const int64_t chunk = MODE == 0 ? bx : (bx / (8 * nl)) * 8 + (bx & 7);
  if (chunk * a.rows_per_chunk >= a.rows) return;  // past the last chunk (merged grid), before any barrier
  bool bad = false;
  const int K = a.width[l], H = a.width[l + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // = the column tile
  const int rb = tid >> 8, fl = tid & 255;                     // staging: 8-row block, feature / column
  const int rbu = __builtin_amdgcn_readfirstlane(rb);
  const int64_t r_begin = chunk * a.rows_per_chunk;
  const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
  const bool last = l == a.L;
  const bool rt0 = MODE == 2 && l == 0;   // the input layer inside a merged launch (see above)
  const bool in0 = L0 || rt0;
  const float* srcA = in0 ? a.x : a.z + a.zoff[l];  // L0: the network input (l = 0)
  const int64_t ldA = in0 ? a.ldx : a.ztot;
  const float* const rawG0 = reinterpret_cast<const float*>(smem + (L0 ? PL::kRawG0 : PL::kSmem));
  const int g0ld = L0 ? CW : 32;  // floats per G_0 slot
  const float* gB = a.G + a.goff[l + 1];
  const float* zB = a.z + a.zoff[l + 1];
  const int64_t ld = a.ztot;
  const bool fa = fl < K, fb = fl < H;
  const float sa = fa ? a.scale[l][fl] : 0.f, ha = fa ? a.shift[l][fl] : 0.f;
  const float sbv = fb ? a.scale[l + 1][fl] : 0.f, bbv = (fb && last) ? a.bias[fl] : 0.f;
  const uint32_t offB = fb ? (uint32_t)fl * 4u : kOOB;
  float csb_b = 0.f, csb_s = 0.f;
  float cs0_b = 0.f, cs0_s = 0.f;  // L0: BN_0's sums, feature fl (rows of this thread's block)
  int cexp = -100;
  pgf4 acc[NTI];  // 2^12 x (the column-scaled) dW tile: features 16 t + 4 fq .., column 16 wave + fi
#pragma unroll
  for (int t = 0; t < NTI; ++t) acc[t] = pgf4{0.f, 0.f, 0.f, 0.f};
  float gst[8];  // G_{l+1} at rows 8 rb + i, column fl (the register stage)
  const uint32_t voffA = pgw_lane_off((uint32_t)K * 4u, lane), voffZ = pgw_lane_off((uint32_t)H * 4u, lane);

  // the 32 rows at r0: z_l and z_{l+1} rows by LDS-DMA (wavefront w: rows 2w, 2w + 1),
  // G_{l+1} through registers with one descriptor per row (wave-uniform rb)
  auto issue_dma = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * wave + j;
      const int64_t row = min(r0 + i, r_end - 1);
      pgw_row_dma(srcA + row * ldA, voffA, smem + PL::kRawA + i * CW * 4);
      pgw_row_dma(zB + row * ld, voffZ, smem + PL::kRawZ + i * CW * 4);
      if constexpr (L0) pgw_row_dma(a.G + a.goff[0] + row * a.gtot, voffA, smem + PL::kRawG0 + i * CW * 4);
      else if (rt0) pgw_row_dma_128(a.G + a.goff[0] + row * a.gtot, (uint32_t)K * 4u, lane, smem + PL::kSmem + i * 128);
    }
  };
  auto issue_g = [&](int64_t r0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = r0 + 8 * rbu + i;
      const auto rB = make_rsrc(gB + row * a.gtot, row < r_end ? (uint32_t)H * 4u : 0u);
      gst[i] = buf_load_elem<float>(rB, offB);
    }
  };
  auto issue = [&](int64_t r0) {
    issue_dma(r0);
    issue_g(r0);
  };

  const int fq = lane >> 4, fi = lane & 15;
  const _Float16* const aBase = sA + (fq * KP + fi) * 8;  // + (part 4 KP + 16 t) 8: immediates
  const int cT = wave * 16 + fi;                           // this lane's column in the group (past H: 0)
  const _Float16* const bBase = sB + (fq * CW + cT) * 8;
  issue(r_begin);
  for (int64_t r0 = r_begin; r0 < r_end; r0 += kPgxSR) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wavefront's row DMA (and G loads)
    __syncthreads();  // raw rows in LDS; the previous sub-chunk's fragment reads are done
    {  // A: feature fl of rows 8 rb .. + 7, the forward's BN and activation, split
      if (fl < KP) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xv = rawA[(8 * rb + i) * CW + fl];
          const float y = ha + xv * sa;
          if (in0) {  // BN_0 only (solver.py:260-262); its sums over the chunk's rows
            v[i] = fa ? y : 0.f;
            if (fa && r0 + 8 * rb + i < r_end) {
              const float g0 = rawG0[(8 * rb + i) * g0ld + fl];
              cs0_b += g0;
              cs0_s += g0 * xv;
            }
          } else {
            v[i] = fa ? y + fmaxf(y, 0.f) : 0.f;  // l >= 1: hidden activations
          }
        }
        pgh8 h, lo;
        pgx_split8(v, h, lo);
        bad |= x3_bad4(v[0], v[1], v[2], v[3]) | x3_bad4(v[4], v[5], v[6], v[7]);
        *reinterpret_cast<pgh8*>(sA + ((0 * 4 + rb) * KP + fl) * 8) = h;
        *reinterpret_cast<pgh8*>(sA + ((1 * 4 + rb) * KP + fl) * 8) = lo;
      }
    }
    float vb[8];
    {  // B: column fl, its sums and the sub-chunk's column max
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gv = gst[i];
        vb[i] = gv * sbv;
        m = fmaxf(m, fabsf(vb[i]));
        csb_b += gv;
        csb_s += gv * (rawZ[(8 * rb + i) * CW + fl] + bbv);  // bbv = 0 unless the output layer
      }
      s_cmax[rb * CW + fl] = m;
    }
    __syncthreads();  // the column maxima; every raw row read
    // round 6: the next sub-chunk's raw rows (LDS-DMA: no registers) are issued here, as soon as
    // every raw row is read, so they land during the column scaling and split as well as the
    // MFMAs; its G rows (a register stage) after the split as before (DPAC_PGW_EARLY=0: all after
    // the split, rounds 4-5)
    if (DPAC_PGW_EARLY && r0 + kPgxSR < r_end) issue_dma(r0 + kPgxSR);
    {
      const float m = fmaxf(fmaxf(s_cmax[fl], s_cmax[CW + fl]), fmaxf(s_cmax[2 * CW + fl], s_cmax[3 * CW + fl]));
      int e = cexp;
      if (m > 0.f && m < 3.0e38f) {
        int em = 0;
        (void)frexpf(m, &em);
        e = em > cexp ? em : cexp;
      }
      const float sc = ldexpf(1.f, 3 - e);
#pragma unroll
      for (int i = 0; i < 8; ++i) vb[i] *= sc;
      pgh8 h, lo, h12;
      pgx_split8(vb, h, lo);
      bad |= x3_bad4(vb[0], vb[1], vb[2], vb[3]) | x3_bad4(vb[4], vb[5], vb[6], vb[7]);
#pragma unroll
      for (int i = 0; i < 8; ++i) h12[i] = h[i] * (_Float16)kPgxLo;  // exact: |h| < 8
      *reinterpret_cast<pgh8*>(sB + ((0 * 4 + rb) * CW + fl) * 8) = h;
      *reinterpret_cast<pgh8*>(sB + ((1 * 4 + rb) * CW + fl) * 8) = lo;
      *reinterpret_cast<pgh8*>(sB + ((2 * 4 + rb) * CW + fl) * 8) = h12;
      if (rb == 0) {
        s_cfac[fl] = ldexpf(1.f, cexp - e);
        s_cexp[fl] = e;
      }
      cexp = e;
    }
    // the next sub-chunk's rows (the raw rows are read; vb no longer needs gst): they land
    // during this sub-chunk's MFMAs
    if (r0 + kPgxSR < r_end) {
      if (DPAC_PGW_EARLY) issue_g(r0 + kPgxSR);  // the G register stage: live only from here
      else issue(r0 + kPgxSR);
    }
    __syncthreads();  // the images
    {
      const pgh8 bh = *reinterpret_cast<const pgh8*>(bBase);
      const pgh8 bl = *reinterpret_cast<const pgh8*>(bBase + 4 * CW * 8);
      const pgh8 b12 = *reinterpret_cast<const pgh8*>(bBase + 2 * 4 * CW * 8);
      const float f = s_cfac[cT];
      if (__any(f != 1.f)) {
#pragma unroll
        for (int t = 0; t < NTI; ++t) acc[t] *= f;
      }
#pragma unroll
      for (int t = 0; t < NTI; ++t) {
        const pgh8 xh = *reinterpret_cast<const pgh8*>(aBase + 16 * t * 8);
        const pgh8 xl = *reinterpret_cast<const pgh8*>(aBase + (4 * KP + 16 * t) * 8);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, b12, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, bl, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, bh, acc[t], 0, 0, 0);
      }
    }
  }

  // ---- this chunk's partial dW_l: lane holds features 16 t + 4 fq .. +3, column cT ----
  float* part = a.part + chunk * a.ptot;
  {
    const float us = ldexpf(1.f, s_cexp[cT] - 3 - 12);  // undo 2^12 and the column scale
#pragma unroll
    for (int t = 0; t < NTI; ++t) {
      const pgf4 c = acc[t] * us;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int k = 16 * t + 4 * fq + v;
        if (k < K && cT < H) part[a.off_W[l] + (int64_t)k * H + cT] = c[v];
      }
    }
  }
  // ---- BN column sums: combine the 4 row blocks through LDS (reusing the images) ----
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  red[(rb * 2 + 0) * CW + fl] = csb_b;
  red[(rb * 2 + 1) * CW + fl] = csb_s;
  float* red0 = red + 4 * 2 * CW;  // L0: [4 rb][2][KP]
  if (in0 && fl < KP) {
    red0[(rb * 2 + 0) * KP + fl] = cs0_b;
    red0[(rb * 2 + 1) * KP + fl] = cs0_s;
  }
  __syncthreads();
  if (in0 && tid < K) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red0[(w * 2 + 0) * KP + tid];
      ss += red0[(w * 2 + 1) * KP + tid];
    }
    part[a.off_beta[0] + tid] = sb;
    part[a.off_gamma[0] + tid] = ss;
  }
  if (tid < CW && tid < H) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red[(w * 2 + 0) * CW + tid];
      ss += red[(w * 2 + 1) * CW + tid];
    }
    part[a.off_beta[l + 1] + tid] = sb;
    part[a.off_gamma[l + 1] + tid] = ss;
  }
  if (bad) x3_flag(a.status);
}

// ---------------------------------------------------------------------------------------------
// k_param_grads_x3d (round 6): k_param_grads_x3w's sums, with the next
// sub-chunk's loads in flight during this one's staging as well as its MFMAs.  x3w's 1 024-thread
// workgroup has 128 VGPRs per lane and no LDS for a second raw block, so it issues the next loads
// only after staging (measured: 3.7 TB/s of operand rows against 5.4 TB/s for the same row slices in
// a plain streaming kernel, profiles/r05_call22_slice_bw.txt).  Here:
//  * 8 wavefronts (512 threads, 256 VGPRs per lane), wave w owning the column tiles w and w + 8
//    (NTI x 2 accumulator tiles), so each wave reads every A fragment for two column tiles and the
//    A-image reads per sub-chunk halve;
//  * G_{l+1} through registers and A's raw rows by LDS-DMA into two raw blocks: two stages (an
//    unrolled pair of sub-chunks), each stage's loads issued as soon as its previous contents are
//    consumed, so they are in flight through a whole sub-chunk; z_{l+1} (only the BN sums read it)
//    by LDS-DMA into one raw block, issued once it is read (as x3w's), two phases ahead of use; the
//    2^12 hi B operand is formed in registers (no third B image): 160 KiB of LDS at 13 tiles.
// Arithmetic, order of every sum and partial layout are x3w's: bitwise its results.
constexpr int kPgdThreads = 512;
template <int NTI, bool L0 = false>
struct PgdPlan {
  static constexpr int KP = 16 * NTI;
  static constexpr int kImgA = 2 * 4 * KP * 8 * 2;          // A hi, lo halves
  static constexpr int kImgB = 2 * 4 * kPgwCW * 8 * 2;      // B hi, lo halves
  static constexpr int kRaw = kPgxSR * kPgwCW * 4;          // one raw A block [32][256] floats
  static constexpr int kRawA = kImgA + kImgB;               // two raw A blocks
  static constexpr int kRawZ = kRawA + 2 * kRaw;            // one raw z_{l+1} block
  static constexpr int kRawG0 = kRawZ + kRaw;               // L0: two compact G_0 blocks [32][32]
  static constexpr int kCol = kRawG0 + (L0 ? 2 * kPgwRawG0c : 0);
  static constexpr int kSmem = kCol + (4 * kPgwCW + 2 * kPgwCW) * 4;
  static_assert(4 * 2 * kPgwCW * 4 + 4 * 2 * KP * 4 <= kRawA, "BN sums' reduction fits the image bytes");
  static_assert(kSmem <= 160 * 1024, "LDS");
};

template <int NTI, bool L0 = false, int MODE = 0>
__global__ __launch_bounds__(kPgdThreads) void k_param_grads_x3d(const PgArgs<float> a, const int lsel) {
  using PL = PgdPlan<NTI, L0>;
  constexpr int KP = PL::KP, CW = kPgwCW;
  static_assert(MODE == 0 || !L0, "merged launches hold wide layers only");
  static_assert(!L0 || KP <= 32, "the input layer: K <= 32");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];  // PL::kSmem bytes (dynamic)
  _Float16* const sA = reinterpret_cast<_Float16*>(smem);
  _Float16* const sB = reinterpret_cast<_Float16*>(smem + PL::kImgA);
  float* const s_cmax = reinterpret_cast<float*>(smem + PL::kCol);
  float* const s_cfac = s_cmax + 4 * CW;
  int* const s_cexp = reinterpret_cast<int*>(s_cfac + CW);
  if (x3_status_set(a.status)) return;  // fell back: the f32 kernel after this one does the work
  const int64_t bx = blockIdx.x;
  const int nl = MODE == 0 ? 1 : (-lsel) >> 3;
  const int l = MODE == 0 ? lsel : ((-lsel) & 7) + (int)((bx >> 3) % nl);
  const int64_t chunk = MODE == 0 ? bx : (bx / (8 * nl)) * 8 + (bx & 7);
  if (chunk * a.rows_per_chunk >= a.rows) return;  // past the last chunk (merged grid), before any barrier
  bool bad = false;
  const int K = a.width[l], H = a.width[l + 1];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // column tiles wave, wave + 8
  const int rb = tid >> 7, fl = tid & 127;                     // staging: 8-row block; features / columns fl, fl + 128
  const int rbu = __builtin_amdgcn_readfirstlane(rb);
  const int64_t r_begin = chunk * a.rows_per_chunk;
  const int64_t r_end = min(a.rows, r_begin + a.rows_per_chunk);
  const bool last = l == a.L;
  const float* srcA = L0 ? a.x : a.z + a.zoff[l];
  const int64_t ldA = L0 ? a.ldx : a.ztot;
  const float* gB = a.G + a.goff[l + 1];
  const float* zB = a.z + a.zoff[l + 1];
  float sa[2], ha[2], sbv[2], bbv[2], csb_b[2], csb_s[2];
  uint32_t offB[2];
  bool fa[2];
  int cexp[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int k = fl + 128 * h;
    fa[h] = k < K;
    sa[h] = fa[h] ? a.scale[l][k] : 0.f;
    ha[h] = fa[h] ? a.shift[l][k] : 0.f;
    const bool fb = k < H;
    sbv[h] = fb ? a.scale[l + 1][k] : 0.f;
    bbv[h] = (fb && last) ? a.bias[k] : 0.f;
    offB[h] = fb ? (uint32_t)k * 4u : kOOB;
    csb_b[h] = csb_s[h] = 0.f;
    cexp[h] = -100;
  }
  float cs0_b = 0.f, cs0_s = 0.f;  // L0: BN_0's sums, feature fl
  pgf4 acc[NTI][2];  // 2^12 x (the column-scaled) dW tiles: features 16 t + 4 fq .., columns 16 (wave + 8 j) + fi
#pragma unroll
  for (int t = 0; t < NTI; ++t) acc[t][0] = acc[t][1] = pgf4{0.f, 0.f, 0.f, 0.f};
  float gst[2][2][8];  // [stage][h][row]: G_{l+1} at rows 8 rb + i, columns fl + 128 h
  const uint32_t voffA = pgw_lane_off((uint32_t)K * 4u, lane), voffZ = pgw_lane_off((uint32_t)H * 4u, lane);
  const float* const rawZ = reinterpret_cast<const float*>(smem + PL::kRawZ);

  // z_{l+1}'s 32 rows at r0 into the raw z block, wave w copying rows 4 w .. 4 w + 3 (past the
  // chunk: its last row again; times G = 0 it adds nothing)
  auto issue_z = [&](int64_t r0) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * wave + j;
      pgw_row_dma(zB + min(r0 + i, r_end - 1) * a.ztot, voffZ, smem + PL::kRawZ + i * CW * 4);
    }
  };
  // the 32 rows at r0 into stage S: G rows through registers, then the raw A rows (and G_0 rows)
  // by LDS-DMA, wave w copying rows 4 w .. 4 w + 3.  Rows past the chunk: G reads 0, the DMA
  // repeats the chunk's last row.
  auto issue = [&](int64_t r0, auto sidx) {
    constexpr int S = decltype(sidx)::value;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int64_t row = r0 + 8 * rbu + i;
      const auto rB = make_rsrc(gB + row * a.gtot, row < r_end ? (uint32_t)H * 4u : 0u);
#pragma unroll
      for (int h = 0; h < 2; ++h) gst[S][h][i] = buf_load_elem<float>(rB, offB[h]);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * wave + j;
      const int64_t row = min(r0 + i, r_end - 1);
      pgw_row_dma(srcA + row * ldA, voffA, smem + PL::kRawA + S * PL::kRaw + i * CW * 4);
      if constexpr (L0)
        pgw_row_dma_128(a.G + a.goff[0] + row * a.gtot, (uint32_t)K * 4u, lane,
                        smem + PL::kRawG0 + S * kPgwRawG0c + i * 128);
    }
  };
  constexpr int kIssueOps = 16 + 4 * (L0 ? 2 : 1);  // vector memory instructions per wave and issue

  const int fq = lane >> 4, fi = lane & 15;
  const _Float16* const aBase = sA + (fq * KP + fi) * 8;  // + (part 4 KP + 16 t) 8
  auto sub = [&](int64_t r0, auto sidx) {
    constexpr int S = decltype(sidx)::value;
    const float* const rawA = reinterpret_cast<const float*>(smem + PL::kRawA + S * PL::kRaw);
    const float* const rawG0 = reinterpret_cast<const float*>(smem + PL::kRawG0 + S * kPgwRawG0c);
    // this sub-chunk's rows have landed once only the issue made right after its z rows is
    // outstanding: issues come in the order (G, A)_k .. z_k, (G, A)_{k+1}, so that is the next
    // sub-chunk's (if any)
    if (r0 + kPgxSR < r_end) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(kIssueOps) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // raw rows in LDS; the previous sub-chunk's fragment reads are done
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // A: features fl + 128 h of rows 8 rb .. + 7, BN and the activation, split
      const int k = fl + 128 * h;
      if (h == 1 && 128 >= KP) continue;  // compile-time: no second feature
      if (k < KP) {
        float v[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float xv = rawA[(8 * rb + i) * CW + k];
          const float y = ha[h] + xv * sa[h];
          if constexpr (L0) {  // BN_0 only (solver.py:260-262); its sums over the chunk's rows
            v[i] = fa[h] ? y : 0.f;
            if (fa[h] && r0 + 8 * rb + i < r_end) {
              const float g0 = rawG0[(8 * rb + i) * 32 + k];
              cs0_b += g0;
              cs0_s += g0 * xv;
            }
          } else {
            v[i] = fa[h] ? y + fmaxf(y, 0.f) : 0.f;  // hidden activations
          }
        }
        pgh8 hh, lo;
        pgx_split8(v, hh, lo);
        bad |= x3_bad4(v[0], v[1], v[2], v[3]) | x3_bad4(v[4], v[5], v[6], v[7]);
        *reinterpret_cast<pgh8*>(sA + ((0 * 4 + rb) * KP + k) * 8) = hh;
        *reinterpret_cast<pgh8*>(sA + ((1 * 4 + rb) * KP + k) * 8) = lo;
      }
    }
    float vb[2][8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {  // B: columns fl + 128 h, their sums and the sub-chunk's column max
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float gv = gst[S][h][i];
        vb[h][i] = gv * sbv[h];
        m = fmaxf(m, fabsf(vb[h][i]));
        csb_b[h] += gv;
        csb_s[h] += gv * (rawZ[(8 * rb + i) * CW + fl + 128 * h] + bbv[h]);  // bbv = 0 unless the output layer
      }
      s_cmax[rb * CW + fl + 128 * h] = m;
    }
    __syncthreads();  // the column maxima; every raw row of this stage read
    if (r0 + kPgxSR < r_end) issue_z(r0 + kPgxSR);              // the raw z block is free: the next sub-chunk's
    if (r0 + 2 * kPgxSR < r_end) issue(r0 + 2 * kPgxSR, sidx);  // this stage is free: two sub-chunks ahead
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int c = fl + 128 * h;
      const float m = fmaxf(fmaxf(s_cmax[c], s_cmax[CW + c]), fmaxf(s_cmax[2 * CW + c], s_cmax[3 * CW + c]));
      int e = cexp[h];
      if (m > 0.f && m < 3.0e38f) {
        int em = 0;
        (void)frexpf(m, &em);
        e = em > cexp[h] ? em : cexp[h];
      }
      const float sc = ldexpf(1.f, 3 - e);
#pragma unroll
      for (int i = 0; i < 8; ++i) vb[h][i] *= sc;
      pgh8 hh, lo;
      pgx_split8(vb[h], hh, lo);
      bad |= x3_bad4(vb[h][0], vb[h][1], vb[h][2], vb[h][3]) | x3_bad4(vb[h][4], vb[h][5], vb[h][6], vb[h][7]);
      *reinterpret_cast<pgh8*>(sB + ((0 * 4 + rb) * CW + c) * 8) = hh;
      *reinterpret_cast<pgh8*>(sB + ((1 * 4 + rb) * CW + c) * 8) = lo;
      if (rb == 0) {
        s_cfac[c] = ldexpf(1.f, cexp[h] - e);
        s_cexp[c] = e;
      }
      cexp[h] = e;
    }
    __syncthreads();  // the images
    pgh8 bh[2], bl[2], b12[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int cT = (wave + 8 * j) * 16 + fi;
      bh[j] = *reinterpret_cast<const pgh8*>(sB + (fq * CW + cT) * 8);
      bl[j] = *reinterpret_cast<const pgh8*>(sB + ((4 + fq) * CW + cT) * 8);
      b12[j] = bh[j] * (_Float16)kPgxLo;  // exact: |hi| < 8
      const float f = s_cfac[cT];
      if (__any(f != 1.f)) {
#pragma unroll
        for (int t = 0; t < NTI; ++t) acc[t][j] *= f;
      }
    }
#pragma unroll
    for (int t = 0; t < NTI; ++t) {
      const pgh8 xh = *reinterpret_cast<const pgh8*>(aBase + 16 * t * 8);
      const pgh8 xl = *reinterpret_cast<const pgh8*>(aBase + (4 * KP + 16 * t) * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, b12[j], acc[t][j], 0, 0, 0);
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh, bl[j], acc[t][j], 0, 0, 0);
        acc[t][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl, bh[j], acc[t][j], 0, 0, 0);
      }
    }
  };
  using S0 = std::integral_constant<int, 0>;
  using S1 = std::integral_constant<int, 1>;
  issue(r_begin, S0{});
  issue_z(r_begin);
  if (r_begin + kPgxSR < r_end) issue(r_begin + kPgxSR, S1{});
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 2 * kPgxSR) {
    sub(r0, S0{});
    if (r0 + kPgxSR < r_end) sub(r0 + kPgxSR, S1{});
  }

  // ---- this chunk's partial dW_l: lane holds features 16 t + 4 fq .. +3, columns cT_j ----
  float* part = a.part + chunk * a.ptot;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int cT = (wave + 8 * j) * 16 + fi;
    const float us = ldexpf(1.f, s_cexp[cT] - 3 - 12);  // undo 2^12 and the column scale
#pragma unroll
    for (int t = 0; t < NTI; ++t) {
      const pgf4 c = acc[t][j] * us;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int k = 16 * t + 4 * fq + v;
        if (k < K && cT < H) part[a.off_W[l] + (int64_t)k * H + cT] = c[v];
      }
    }
  }
  // ---- BN column sums: combine the 4 row blocks through LDS (reusing the images) ----
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    red[(rb * 2 + 0) * CW + fl + 128 * h] = csb_b[h];
    red[(rb * 2 + 1) * CW + fl + 128 * h] = csb_s[h];
  }
  float* red0 = red + 4 * 2 * CW;  // L0: [4 rb][2][KP]
  if (L0 && fl < KP) {
    red0[(rb * 2 + 0) * KP + fl] = cs0_b;
    red0[(rb * 2 + 1) * KP + fl] = cs0_s;
  }
  __syncthreads();
  if (L0 && tid < K) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red0[(w * 2 + 0) * KP + tid];
      ss += red0[(w * 2 + 1) * KP + tid];
    }
    part[a.off_beta[0] + tid] = sb;
    part[a.off_gamma[0] + tid] = ss;
  }
  if (tid < CW && tid < H) {
    float sb = 0.f, ss = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      sb += red[(w * 2 + 0) * CW + tid];
      ss += red[(w * 2 + 1) * CW + tid];
    }
    part[a.off_beta[l + 1] + tid] = sb;
    part[a.off_gamma[l + 1] + tid] = ss;
  }
  if (bad) x3_flag(a.status);
}

}  // namespace dpac
