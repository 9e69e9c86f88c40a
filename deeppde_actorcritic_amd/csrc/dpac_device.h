// dpac_device.h — device building blocks shared by every libdpac kernel:
//   * the lane ownership model: a trajectory is owned by P consecutive lanes of
//     a 64-wide wavefront; lane p owns components j = p + m*P (m < M), so one
//     wave instruction touches P consecutive floats of a trajectory row;
//   * lane-group reductions over the P lanes (DPP only, no LDS);
//   * the Brownian-increment stream (rocRAND Philox4x32-10 + Box–Muller);
//   * the four equation families as device functors (coefficients, analytic
//     solutions and the vector-Jacobian products the rollout backward needs).
//
// Reference: equation.py:5-311 (Equation, LQR, VDP, ekn, LQR_var).
#pragma once

#include <hip/hip_runtime.h>
#include <rocrand/rocrand_kernel.h>
#include <stdint.h>

#include "dpac.h"
#include "dpac_mfma.h"

namespace dpac {

// ---------------------------------------------------------------------------
// Lane split.  P lanes per trajectory, M = ceil(D/P) components per lane with
// P = min(16, next_pow2(ceil(D/2))): at most 2 components per lane up to d = 32,
// so the per-step instruction stream of a wave is short and B = 4096, d = 20
// gives 1024 wavefronts — one per SIMD of the 256-CU chip.
// ---------------------------------------------------------------------------
__host__ __device__ constexpr int pow2_at_least(int v) {
  int p = 1;
  while (p < v) p *= 2;
  return p;
}
// Timing experiments only: DPAC_LANE_CAP / DPAC_LANE_COMPS change the split.
#ifndef DPAC_LANE_CAP
#define DPAC_LANE_CAP 16
#endif
#ifndef DPAC_LANE_COMPS
#define DPAC_LANE_COMPS 2
#endif
__host__ __device__ constexpr int lanes_for_dim(int D) {
  return pow2_at_least((D + DPAC_LANE_COMPS - 1) / DPAC_LANE_COMPS) < DPAC_LANE_CAP
             ? pow2_at_least((D + DPAC_LANE_COMPS - 1) / DPAC_LANE_COMPS)
             : DPAC_LANE_CAP;
}
__host__ __device__ constexpr int comps_per_lane(int D) {
  return (D + lanes_for_dim(D) - 1) / lanes_for_dim(D);
}
// The lane split of each equation family's kernels (the TUs dpac_eqn_*.hip instantiate the
// functors with it; the fused TD1 row kernels must use the same one).  VDP's cyclic coupling
// keeps a trajectory in one lane.
__host__ __device__ constexpr int eqn_lanes(int eqn, int D) {
  return eqn == DPAC_EQN_VDP ? 1 : lanes_for_dim(D);
}

// Ownership of one lane: the CONTIGUOUS components j = p*M + m (m < M), so a
// lane moves one M-element vector per row and a group's lanes cover the row
// [b*d, b*d + d) in order — one fully coalesced instruction per row slab.
// Lanes (or, for odd d, single elements) past d own nothing: their loads read
// zero and their stores are dropped (buffer descriptors, see BufSlab), and every
// componentwise equation maps zero components to zero contributions.
template <int D, int P>
struct Own {
  static constexpr int M = (D + P - 1) / P;
  static constexpr bool kFull = (D % M) == 0;  // every lane is either full or empty
  int p;
  __device__ __forceinline__ explicit Own(int p_) : p(p_) {}
  __device__ __forceinline__ int j(int m) const { return p * M + m; }
  __device__ __forceinline__ bool valid(int m) const { return p * M + m < D; }
  __device__ __forceinline__ bool active() const { return p * M < D; }
  template <typename T>
  __device__ __forceinline__ void mask(T (&v)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) v[m] = valid(m) ? v[m] : T(0);
  }
  // plain-pointer forms (predicated) for the single-step kernels
  template <typename T>
  __device__ __forceinline__ void load_masked(const T* __restrict__ row, T (&v)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) v[m] = valid(m) ? row[p * M + m] : T(0);
  }
  template <typename T>
  __device__ __forceinline__ void store(T* __restrict__ row, const T (&v)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (valid(m)) row[p * M + m] = v[m];
  }
};

// ---------------------------------------------------------------------------
// Buffer-descriptor access to [steps][rows][d] arrays (x / dw / u / G).  One
// descriptor covers the whole array (num_records = its bytes, < 2 GiB — the
// host checks); the per-lane voffset addresses the lane's elements inside one
// step's slab and the wave-uniform soffset selects the step, so the time loop
// spends one scalar add per array and step.  An out-of-range voffset (kOOB)
// reads 0 and drops the store whether or not the hardware counts soffset in
// the range check: inactive lanes and padding elements need no branch.
// ---------------------------------------------------------------------------
// Host description of the fused TD1 operands (dpac_mlp_rows_fwd_td1 / _bwd_td1).
struct TdRows {
  const void *x, *u, *dw;
  int64_t ldx;
  int ldu, p;
  double sa, sb;
  void* gdot;
  const void* g_gdot;
};

constexpr uint32_t kOOB = 0x80000000u;
constexpr int kRsrcFlags = 0x00020000;  // gfx950 raw-buffer descriptor word 3 (guide T8)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)bytes, kRsrcFlags);
}

// ---- the split-fp16 range guard (dpac.h dpac_mlp.status) ----
// An f32 operand a is split as hi = fp16(a), lo = fp16((a - hi) 2^12).  For |a| < 2^15,
// |hi| <= 2^15 and |a - hi| <= 8 (half an fp16 ulp), so |lo| <= 2^15: both finite.  Past it
// lo (from 2^15) or hi (from 65520) overflows.
constexpr float kX3Range = 32768.f;
// whether any of four split operands lies outside the range (also inf / NaN)
__device__ __forceinline__ bool x3_bad4(float a, float b, float c, float d) {
  return !(fabsf(a) < kX3Range) | !(fabsf(b) < kX3Range) | !(fabsf(c) < kX3Range) | !(fabsf(d) < kX3Range);
}
__device__ __forceinline__ bool x3_bad(float a) { return !(fabsf(a) < kX3Range); }
// sticky status word: set (a vector atomic to L2, agent scope) / read at agent scope
__device__ __forceinline__ void x3_flag(uint32_t* st) {
  if (st) __hip_atomic_fetch_or(st, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ bool x3_status_set(const uint32_t* st) {
  return st && __hip_atomic_load(const_cast<uint32_t*>(st), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u;
}

// AUX: the cache-policy immediate of the buffer instruction (0 = default; 2 = nt).
template <int K, int AUX = 0>
__device__ __forceinline__ void buf_load_dwords(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                uint32_t (&w)[K], uint32_t soff = 0) {
  constexpr int k4 = K / 4 * 4;
#pragma unroll
  for (int k = 0; k < k4; k += 4) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(voff + 4 * k), (int)soff, AUX);
    w[k] = q[0]; w[k + 1] = q[1]; w[k + 2] = q[2]; w[k + 3] = q[3];
  }
  if constexpr (K - k4 == 3) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b96(r, (int)(voff + 4 * k4), (int)soff, AUX);
    w[k4] = q[0]; w[k4 + 1] = q[1]; w[k4 + 2] = q[2];
  } else if constexpr (K - k4 == 2) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, (int)(voff + 4 * k4), (int)soff, AUX);
    w[k4] = q[0]; w[k4 + 1] = q[1];
  } else if constexpr (K - k4 == 1) {
    w[k4] = __builtin_amdgcn_raw_buffer_load_b32(r, (int)(voff + 4 * k4), (int)soff, AUX);
  }
}

template <int K, int AUX = 0>
__device__ __forceinline__ void buf_store_dwords(__amdgpu_buffer_rsrc_t r, uint32_t voff,
                                                 const uint32_t (&w)[K], uint32_t soff = 0) {
  constexpr int k4 = K / 4 * 4;
#pragma unroll
  for (int k = 0; k < k4; k += 4) {
    __attribute__((ext_vector_type(4))) unsigned int q = {w[k], w[k + 1], w[k + 2], w[k + 3]};
    __builtin_amdgcn_raw_buffer_store_b128(q, r, (int)(voff + 4 * k), (int)soff, AUX);
  }
  if constexpr (K - k4 == 3) {
    __attribute__((ext_vector_type(3))) unsigned int q = {w[k4], w[k4 + 1], w[k4 + 2]};
    __builtin_amdgcn_raw_buffer_store_b96(q, r, (int)(voff + 4 * k4), (int)soff, AUX);
  } else if constexpr (K - k4 == 2) {
    __attribute__((ext_vector_type(2))) unsigned int q = {w[k4], w[k4 + 1]};
    __builtin_amdgcn_raw_buffer_store_b64(q, r, (int)(voff + 4 * k4), (int)soff, AUX);
  } else if constexpr (K - k4 == 1) {
    __builtin_amdgcn_raw_buffer_store_b32(w[k4], r, (int)(voff + 4 * k4), (int)soff, AUX);
  }
}

template <typename T>
__device__ __forceinline__ T buf_load_elem(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  uint32_t w[sizeof(T) / 4];
  buf_load_dwords<sizeof(T) / 4>(r, voff, w);
  T v;
  __builtin_memcpy(&v, &w[0], sizeof(T));
  return v;
}

// Rows [row0, row0 + live) of a [rows][ld] array as a buffer descriptor (round 6, VERDICT r05
// item 6): element (r, k) sits at byte offset ((r - row0) ld + k) sizeof(T), and a row outside
// the range reads 0 (a store to it is dropped) instead of reaching memory past the array.
template <typename T>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const T* base, int64_t row0, int live, int64_t ld) {
  const bool any = base != nullptr && live > 0;
  return make_rsrc(any ? base + row0 * ld : nullptr, any ? (uint32_t)((int64_t)live * ld * (int64_t)sizeof(T)) : 0u);
}

// DPAC_CHECK_BOUNDS=1 (a test build, `make bounds`): every row-indexed load of the row kernels'
// TD operands and prologues checks that its row is live; a violation prints one line per wave
// and reads 0 (the descriptors' behaviour), so a test run reports it without faulting the GPU.
#ifndef DPAC_CHECK_BOUNDS
#define DPAC_CHECK_BOUNDS 0
#endif
#if DPAC_CHECK_BOUNDS
#define DPAC_CHECK_ROW(off, live)                                                                  \
  do {                                                                                             \
    if (!((int64_t)(off) >= 0 && (int64_t)(off) < (int64_t)(live)))                                \
      printf("dpac bounds violation: row offset %lld of %d live rows at %s:%d\n",                 \
             (long long)(off), (int)(live), __FILE__, __LINE__);                                   \
  } while (0)
#else
#define DPAC_CHECK_ROW(off, live) ((void)0)
#endif

template <typename T>
__device__ __forceinline__ void buf_store_scalar(__amdgpu_buffer_rsrc_t r, uint32_t voff, T v,
                                                 uint32_t soff = 0) {
  uint32_t w[sizeof(T) / 4];
  __builtin_memcpy(&w[0], &v, sizeof(T));
  buf_store_dwords<sizeof(T) / 4>(r, voff, w, soff);
}

// A lane's view of a [rows][D] slab: the byte offset of its M elements of row b
// (kOOB when the lane owns nothing or the row is a padding duplicate).  Full
// lanes move one vector; for odd D each element has its own offset.
template <typename T, int D, int P>
struct BufSlab {
  static constexpr int M = Own<D, P>::M;
  static constexpr bool kVec = Own<D, P>::kFull;
  static constexpr int K = M * (int)sizeof(T) / 4;
  uint32_t off[kVec ? 1 : M];
  __device__ __forceinline__ BufSlab(const Own<D, P>& own, int64_t b, bool live) {
    if constexpr (kVec) {
      off[0] = (live && own.active()) ? (uint32_t)((b * D + own.p * M) * (int64_t)sizeof(T)) : kOOB;
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m)
        off[m] = (live && own.valid(m)) ? (uint32_t)((b * D + own.j(m)) * (int64_t)sizeof(T)) : kOOB;
    }
  }
  // soff: wave-uniform byte offset of the row block (the step), in soffset.
  template <int AUX = 0>
  __device__ __forceinline__ void load(__amdgpu_buffer_rsrc_t r, T (&v)[M], uint32_t soff = 0) const {
    if constexpr (kVec) {
      uint32_t w[K];
      buf_load_dwords<K, AUX>(r, off[0], w, soff);
      __builtin_memcpy(&v[0], &w[0], sizeof(w));
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        uint32_t w[sizeof(T) / 4];
        buf_load_dwords<sizeof(T) / 4, AUX>(r, off[m], w, soff);
        __builtin_memcpy(&v[m], &w[0], sizeof(T));
      }
    }
  }
  template <int AUX = 0>
  __device__ __forceinline__ void store(__amdgpu_buffer_rsrc_t r, const T (&v)[M], uint32_t soff = 0) const {
    if constexpr (kVec) {
      uint32_t w[K];
      __builtin_memcpy(&w[0], &v[0], sizeof(w));
      buf_store_dwords<K, AUX>(r, off[0], w, soff);
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) {
        uint32_t w[sizeof(T) / 4];
        __builtin_memcpy(&w[0], &v[m], sizeof(T));
        buf_store_dwords<sizeof(T) / 4, AUX>(r, off[m], w, soff);
      }
    }
  }
};

// ---------------------------------------------------------------------------
// Lane-group all-reduce over groups of P consecutive lanes, DPP only:
// quad_perm xor1 / xor2, then row_half_mirror (8 lanes) and row_mirror (16).
// Each level adds two operands in commutative order, so every lane of the
// group ends with the same bits.
// ---------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __builtin_bit_cast(float, dpp_i32<CTRL>(__builtin_bit_cast(int, v)));
}
template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
  const long long b = __builtin_bit_cast(long long, v);
  const int lo = dpp_i32<CTRL>(static_cast<int>(b));
  const int hi = dpp_i32<CTRL>(static_cast<int>(b >> 32));
  return __builtin_bit_cast(double,
                            (static_cast<long long>(hi) << 32) | static_cast<unsigned int>(lo));
}
enum : int {
  kDppXor1 = 0xB1,        // quad_perm(1,0,3,2)
  kDppXor2 = 0x4E,        // quad_perm(2,3,0,1)
  kDppHalfMirror = 0x141, // row_half_mirror: lane i <-> 7-i within 8
  kDppMirror = 0x140,     // row_mirror: lane i <-> 15-i within 16
};

// Rows 2k and 2k+1 (16 lanes each) exchanged by v_permlane16_swap (gfx950):
// the two results hold the even-row and the odd-row value in both rows.
__device__ __forceinline__ float row_pair_sum(float v) {
  const unsigned u = __builtin_bit_cast(unsigned, v);
  const auto sw = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}
__device__ __forceinline__ double row_pair_sum(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)u, hi = (unsigned)(u >> 32);
  const auto sl = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto sh = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double a = __builtin_bit_cast(double, ((unsigned long long)(unsigned)sh[0] << 32) | (unsigned)sl[0]);
  const double b = __builtin_bit_cast(double, ((unsigned long long)(unsigned)sh[1] << 32) | (unsigned)sl[1]);
  return a + b;
}

// Shift register inside each lane group: lane p takes lane p-1's `keep`, the
// group's first lane takes `v`.  One v_mov_dpp row_shr:1 whose source-less lane
// (lane 0 of each 16-lane row) keeps `old` = v; groups shorter than a row also
// select v on their first lane.
template <int P, typename T>
__device__ __forceinline__ T group_shift_in(T keep, T v, bool group_start) {
  if constexpr (P == 1) {
    return v;
  } else {
    constexpr int kRowShr1 = 0x111;
    T sh;
    if constexpr (sizeof(T) == 4) {
      sh = __builtin_bit_cast(T, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, v),
                                                            __builtin_bit_cast(int, keep),
                                                            kRowShr1, 0xF, 0xF, false));
    } else {
      const long long vb = __builtin_bit_cast(long long, v), kb = __builtin_bit_cast(long long, keep);
      const int lo = __builtin_amdgcn_update_dpp((int)vb, (int)kb, kRowShr1, 0xF, 0xF, false);
      const int hi = __builtin_amdgcn_update_dpp((int)(vb >> 32), (int)(kb >> 32), kRowShr1, 0xF, 0xF,
                                                 false);
      sh = __builtin_bit_cast(T, ((long long)hi << 32) | (unsigned int)lo);
    }
    if constexpr (P < 16) sh = group_start ? v : sh;
    return sh;
  }
}

template <int P>
struct Lanes {
  static_assert(P == 1 || P == 2 || P == 4 || P == 8 || P == 16 || P == 32, "bad group size");
  template <typename T>
  __device__ __forceinline__ static T sum(T v) {
    if constexpr (P >= 2) v = v + dpp<kDppXor1>(v);
    if constexpr (P >= 4) v = v + dpp<kDppXor2>(v);
    if constexpr (P >= 8) v = v + dpp<kDppHalfMirror>(v);
    if constexpr (P >= 16) v = v + dpp<kDppMirror>(v);
    if constexpr (P >= 32) v = row_pair_sum(v);
    return v;
  }
};

// ---------------------------------------------------------------------------
// Brownian increments: rocRAND Philox4x32-10, subsequence = global trajectory
// index g, key = seed.  With P = lanes_for_dim(d), M = comps_per_lane(d) and PB the
// values one counter block yields (4 float normals, 2 double normals, 4 bounded values):
//  * paired layout, when 2M <= PB (round 6; e.g. float at d = 20: M = 2, PB = 4): lane slot
//    p draws the increments of TWO steps from one block, (tag << 48) | ((t/2)*P + p); value
//    (t % 2)*M + m of the block is component j = p*M + m of step t.  Every value drawn is
//    used (rounds 1-5 drew a block per step and kept M of its PB values);
//  * otherwise (2M > PB: float64 normals at M >= 2, VDP's one-lane groups): component
//    j = p*M + m of step t is element (m % PB) of block (tag << 48) | ((t*P + p)*BPL + m/PB),
//    BPL = ceil(M / PB).
// A lane draws exactly the components it owns, and the stream is a fixed function of
// (seed, g, t, j) for every GPU count and batch split.
// Normal: rocRAND's Box–Muller (float: box_muller_hw below; double:
// normal_distribution_double2).  Bounded: k = floor(6·u32 / 2^32) ∈ {0..5},
// value floor((k-1)/4)·√3 (equation.py:31-32).
// ---------------------------------------------------------------------------
enum : uint64_t { kTagDw = 0, kTagDir = 1, kTagRadius = 2, kTagBdry = 3 };

__device__ __forceinline__ uint4 philox_block(uint64_t seed, uint64_t subseq, uint64_t block) {
  rocrand_state_philox4x32_10 st;
  rocrand_init(seed, subseq, block * 4ull, &st);
  return rocrand4(&st);  // the 4 words of counter `block`; the engine copy dies here
}

// rocRAND's float Box–Muller mapping (rocrand_normal.h box_muller: u in (0,1],
// angle in (0, 2pi]) with the hardware v_log_f32 / v_sqrt_f32 / v_sin,cos_f32
// instead of the correctly-rounded expansions (~1 ulp).
__device__ __forceinline__ void box_muller_hw(unsigned int x, unsigned int y, float& a, float& b) {
  const float u = ROCRAND_2POW32_INV + (x * ROCRAND_2POW32_INV);
  const float v = ROCRAND_2POW32_INV_2PI + (y * ROCRAND_2POW32_INV_2PI);
  const float s = __builtin_amdgcn_sqrtf(-2.0f * __logf(u));
  float sn, cs;
  __sincosf(v, &sn, &cs);
  a = sn * s;
  b = cs * s;
}

template <typename T>
struct Rng;
template <>
struct Rng<float> {
  static constexpr int kNormalPerBlock = 4;
  __device__ __forceinline__ static void normals(uint4 v, float (&o)[4]) {
    box_muller_hw(v.x, v.y, o[0], o[1]);
    box_muller_hw(v.z, v.w, o[2], o[3]);
  }
};
template <>
struct Rng<double> {
  static constexpr int kNormalPerBlock = 2;
  __device__ __forceinline__ static void normals(uint4 v, double (&o)[2]) {
    const double2 n = rocrand_device::detail::normal_distribution_double2(v);
    o[0] = n.x;
    o[1] = n.y;
  }
};

template <typename T>
__device__ __forceinline__ T bounded_value(unsigned int w) {
  const unsigned int k = static_cast<unsigned int>((static_cast<unsigned long long>(w) * 6ull) >> 32);
  const T s3 = static_cast<T>(1.7320508075688772);  // np.sqrt(3.0)
  return k == 0u ? -s3 : (k == 5u ? s3 : static_cast<T>(0));
}

template <typename T>
__host__ __device__ constexpr int dw_per_block(int sample_type) {
  return sample_type == DPAC_SAMPLE_BOUNDED ? 4 : (sizeof(T) == 4 ? 4 : 2);
}

// Steps whose increments a lane slot draws from one counter block (the layout above): 2 when
// both steps' M values fit one block, else 1.
template <typename T>
__host__ __device__ constexpr int dw_steps_per_block(int M, int sample_type) {
  return 2 * M <= dw_per_block<T>(sample_type) ? 2 : 1;
}

// The values of one counter block of the dw stream (PB of them; the rest unset).
template <typename T>
__device__ __forceinline__ void dw_block_values(uint64_t seed, uint64_t traj, uint64_t block,
                                                int sample_type, T (&v)[4]) {
  const uint4 w = philox_block(seed, traj, (kTagDw << 48) | block);
  if (sample_type == DPAC_SAMPLE_BOUNDED) {
    v[0] = bounded_value<T>(w.x); v[1] = bounded_value<T>(w.y);
    v[2] = bounded_value<T>(w.z); v[3] = bounded_value<T>(w.w);
  } else {
    T n[Rng<T>::kNormalPerBlock];
    Rng<T>::normals(w, n);
#pragma unroll
    for (int e = 0; e < Rng<T>::kNormalPerBlock; ++e) v[e] = n[e];
  }
}

// Paired layout (dw_steps_per_block == 2): lane slot p's increments of steps 2q (out[0 .. M))
// and 2q + 1 (out[M .. 2M)), one counter block.
template <typename T, int D>
__device__ __forceinline__ void draw_slot_pair(uint64_t seed, uint64_t traj, int q, int p, int sample_type,
                                               T (&out)[2 * comps_per_lane(D)]) {
  constexpr int P = lanes_for_dim(D), M = comps_per_lane(D);
  static_assert(2 * M <= 4, "a block holds at most 4 values");
  T v[4];
  dw_block_values<T>(seed, traj, (uint64_t)q * P + p, sample_type, v);
#pragma unroll
  for (int i = 0; i < 2 * M; ++i) out[i] = v[i];
}

// The M increments of lane slot p (components p*M + m) at step t.
template <typename T, int D>
__device__ __forceinline__ void draw_slot(uint64_t seed, uint64_t traj, int t, int p,
                                          int sample_type, T (&out)[comps_per_lane(D)]) {
  constexpr int P = lanes_for_dim(D), M = comps_per_lane(D);
  if constexpr (2 * M <= 4) {
    if (dw_steps_per_block<T>(M, sample_type) == 2) {  // the paired layout: this step's half
      T v[2 * M];
      draw_slot_pair<T, D>(seed, traj, t >> 1, p, sample_type, v);
      const bool odd = (t & 1) != 0;
#pragma unroll
      for (int m = 0; m < M; ++m) out[m] = odd ? v[M + m] : v[m];
      return;
    }
  }
  if (sample_type == DPAC_SAMPLE_BOUNDED) {
    constexpr int PB = 4, BPL = (M + PB - 1) / PB;
    const uint64_t base = ((uint64_t)t * P + p) * BPL;
#pragma unroll
    for (int blk = 0; blk < BPL; ++blk) {
      const uint4 v = philox_block(seed, traj, (kTagDw << 48) | (base + blk));
      const unsigned int w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < PB; ++e)
        if (blk * PB + e < M) out[blk * PB + e] = bounded_value<T>(w[e]);
    }
  } else {
    constexpr int PB = Rng<T>::kNormalPerBlock, BPL = (M + PB - 1) / PB;
    const uint64_t base = ((uint64_t)t * P + p) * BPL;
#pragma unroll
    for (int blk = 0; blk < BPL; ++blk) {
      T n[PB];
      Rng<T>::normals(philox_block(seed, traj, (kTagDw << 48) | (base + blk)), n);
#pragma unroll
      for (int e = 0; e < PB; ++e)
        if (blk * PB + e < M) out[blk * PB + e] = n[e];
    }
  }
}

// All D increments of step t in component order (for one-lane-per-trajectory kernels).
template <typename T, int D>
__device__ __forceinline__ void draw_all(uint64_t seed, uint64_t traj, int t, int sample_type,
                                         T (&out)[D]) {
  constexpr int P = lanes_for_dim(D), M = comps_per_lane(D);
#pragma unroll
  for (int p = 0; p < P; ++p) {
    T s[M];
    draw_slot<T, D>(seed, traj, t, p, sample_type, s);
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (p * M + m < D) out[p * M + m] = s[m];
  }
}

// ---------------------------------------------------------------------------
// Equation functors.  Methods see a lane's owned slice (M components, zero in
// slots past d) and, where the equation needs it, the trajectory's norm r = |x|
// (hot path) or both S = |x|^2 and r (analytic solutions).  Constants are
// computed on the host in double, in the reference's evaluation order, then
// rounded to T.
// ---------------------------------------------------------------------------
struct HostConsts {  // double-precision constants shared by all equations
  double gamma, R, sigma_up, dt0, sqrt_dt0, dt_min, den, c_layer, R2;
};

// LQR — equation.py:144-176
template <typename T, int D, int P>
struct EqLQR {
  static constexpr int M = (D + P - 1) / P, MC = M, kP = P, CDIM = D;
  static constexpr bool kNeedsNorm = false;
  T p, q, beta, kappa, two_kd, kR2, sqrt2, two_k, k, two_p, two_q;
  static EqLQR make(const dpac_eqn_params& e) {
    EqLQR r;
    r.p = (T)e.p; r.q = (T)e.q; r.beta = (T)e.beta; r.k = (T)e.k;
    r.kappa = (T)(-e.beta * e.k / e.q);     // u_true: -beta*k/q*x (:164)
    r.two_kd = (T)(2.0 * e.k * e.dim);      // w: ... - 2*k*dim (:155)
    r.kR2 = (T)(e.k * (e.R * e.R));         // Z = k*R^2 (:158)
    r.sqrt2 = (T)1.4142135623730951;        // np.sqrt(2.0) (:170)
    r.two_k = (T)(2.0 * e.k);               // V_grad = 2*k*x (:167)
    r.two_p = (T)(2.0 * e.p); r.two_q = (T)(2.0 * e.q);
    return r;
  }
  __device__ __forceinline__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = kappa * x[m];
  }
  __device__ __forceinline__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = beta * u[m];
  }
  __device__ __forceinline__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  // sigma() as sa * (1 + sb * x_j * u_j) for the fused TD1 row kernels (host side)
  static void sigma_form(const dpac_eqn_params&, double& sa, double& sb) { sa = 1.4142135623730951; sb = 0.0; }
  __device__ __forceinline__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T a = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) a += p * (x[m] * x[m]) + q * (u[m] * u[m]);
    return a;
  }
  __device__ __forceinline__ T w_finish(T s) const { return s - two_kd; }
  __device__ __forceinline__ T V_true(const T (&x)[M], T S, T r) const { return S * k; }
  __device__ __forceinline__ T Z(const T (&x)[M], T S, T r) const { return kR2; }
  __device__ __forceinline__ void V_grad(const T (&x)[M], T S, T r, T (&g)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = two_k * x[m];
  }
  // VJPs: accumulate a·∂drift/∂(x,u), a·∂sigma/∂(x,u), gw·∂w/∂(x,u)
  __device__ __forceinline__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T r, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) gu[m] += beta * a[m];
  }
  __device__ __forceinline__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M], T (&gx)[M],
                            T (&gu)[MC]) const {}
  __device__ __forceinline__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gx[m] += gw * (two_p * x[m]);
      gu[m] += gw * (two_q * u[m]);
    }
  }
};

// LQR_var — equation.py:278-311 (state- and control-dependent diagonal sigma)
template <typename T, int D, int P>
struct EqLQRVar {
  static constexpr int M = (D + P - 1) / P, MC = M, kP = P, CDIM = D;
  static constexpr bool kNeedsNorm = false;
  T q, beta, eps, k, c1, c2, gk, two_kd, kR2, sqrt2, bpe, qk, e2, two_k, two_q, two_gk, sqrt2_eps,
      two_c1q;
  static EqLQRVar make(const dpac_eqn_params& e) {
    EqLQRVar r;
    r.q = (T)e.q; r.beta = (T)e.beta; r.eps = (T)e.epsilon; r.k = (T)e.k;
    const double bpe = e.beta + 2.0 * e.epsilon;
    r.c1 = (T)(e.k * e.k * (bpe * bpe));             // k**2*(beta+2eps)**2 (:289)
    r.c2 = (T)(2.0 * e.k * (e.epsilon * e.epsilon));  // 2*k*eps**2 (:289)
    r.gk = (T)(e.gamma * e.k);                        // gamma*k (:290)
    r.two_kd = (T)(2.0 * e.k * e.dim);
    r.kR2 = (T)(e.k * (e.R * e.R));
    r.sqrt2 = (T)1.4142135623730951;
    r.bpe = (T)bpe;                                   // u_true numerator (:299)
    r.qk = (T)(e.q / e.k);
    r.e2 = (T)(2.0 * (e.epsilon * e.epsilon));
    r.two_k = (T)(2.0 * e.k); r.two_q = (T)(2.0 * e.q); r.two_gk = (T)(2.0 * e.gamma * e.k);
    r.sqrt2_eps = (T)(1.4142135623730951 * e.epsilon);
    r.two_c1q = (T)(2.0 * (e.k * e.k * (bpe * bpe)) * e.q);
    return r;
  }
  __device__ __forceinline__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = (-bpe * x[m]) / (qk + e2 * (x[m] * x[m]));
  }
  __device__ __forceinline__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = beta * u[m];
  }
  __device__ __forceinline__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2 * (1 + (eps * x[m]) * u[m]);
  }
  static void sigma_form(const dpac_eqn_params& e, double& sa, double& sb) {
    sa = 1.4142135623730951;  // sqrt2 * (1 + eps * x * u) (equation.py:305)
    sb = e.epsilon;
  }
  __device__ __forceinline__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T a = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const T x2 = x[m] * x[m];
      a += (c1 * x2) / (q + c2 * x2) + (gk * x2 + q * (u[m] * u[m]));
    }
    return a;
  }
  __device__ __forceinline__ T w_finish(T s) const { return s - two_kd; }
  __device__ __forceinline__ T V_true(const T (&x)[M], T S, T r) const { return S * k; }
  __device__ __forceinline__ T Z(const T (&x)[M], T S, T r) const { return kR2; }
  __device__ __forceinline__ void V_grad(const T (&x)[M], T S, T r, T (&g)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = two_k * x[m];
  }
  __device__ __forceinline__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T r, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) gu[m] += beta * a[m];
  }
  __device__ __forceinline__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M], T (&gx)[M],
                            T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gx[m] += a[m] * (sqrt2_eps * u[m]);
      gu[m] += a[m] * (sqrt2_eps * x[m]);
    }
  }
  __device__ __forceinline__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) {
      const T den = q + c2 * (x[m] * x[m]);
      gx[m] += gw * (two_c1q * x[m] / (den * den) + two_gk * x[m]);
      gu[m] += gw * (two_q * u[m]);
    }
  }
};

// ekn (configs say "EKN") — diffusive Eikonal, equation.py:240-276
template <typename T, int D, int P>
struct EqEKN {
  static constexpr int M = (D + P - 1) / P, MC = M, kP = P, CDIM = D;
  static constexpr bool kNeedsNorm = true;
  T a2, a3, K, two_a2, three_a3, sqrt2;
  static EqEKN make(const dpac_eqn_params& e) {
    EqEKN r;
    r.a2 = (T)e.a2; r.a3 = (T)e.a3;
    r.K = (T)(3.0 * (e.dim + 1) * e.a3 / 2.0 / e.a2 / e.dim);  // (:272) numerator chain
    r.two_a2 = (T)(2.0 * e.a2); r.three_a3 = (T)(3.0 * e.a3);
    r.sqrt2 = (T)1.4142135623730951;
    return r;
  }
  __device__ __forceinline__ void u_true(const T (&x)[M], T r, T (&u)[MC]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) u[m] = x[m] / r;  // x / |x| (:261)
  }
  __device__ __forceinline__ void drift(const T (&x)[M], const T (&u)[MC], T r, T (&f)[M]) const {
    const T c = K / (two_a2 - three_a3 * r);
#pragma unroll
    for (int m = 0; m < M; ++m) f[m] = c * u[m];
  }
  __device__ __forceinline__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  static void sigma_form(const dpac_eqn_params&, double& sa, double& sb) { sa = 1.4142135623730951; sb = 0.0; }
  __device__ __forceinline__ T w_part(const T (&x)[M], const T (&u)[MC]) const { return 0; }
  __device__ __forceinline__ T w_finish(T) const { return 1; }  // 0*sum(x) + 1 (:250)
  __device__ __forceinline__ T V_true(const T (&x)[M], T S, T r) const { return a3 * (r * r * r) - a2 * (r * r); }
  __device__ __forceinline__ T Z(const T (&x)[M], T S, T r) const { return V_true(x, S, r); }
  __device__ __forceinline__ void V_grad(const T (&x)[M], T S, T r, T (&g)[M]) const {
    const T c = three_a3 * r - two_a2;
#pragma unroll
    for (int m = 0; m < M; ++m) g[m] = c * x[m];
  }
  __device__ __forceinline__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T r, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
    const T den = two_a2 - three_a3 * r;
    const T c = K / den;
    T au = 0;
#pragma unroll
    for (int m = 0; m < M; ++m) {
      gu[m] += c * a[m];
      au += a[m] * u[m];
    }
    au = Lanes<P>::sum(au);
    // d c / d r = K*3a3/den^2 ; d r / d x = x / r
    const T f = au * (K * three_a3 / (den * den)) / r;
#pragma unroll
    for (int m = 0; m < M; ++m) gx[m] += f * x[m];
  }
  __device__ __forceinline__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M], T (&gx)[M],
                            T (&gu)[MC]) const {}
  __device__ __forceinline__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M], T (&gu)[MC]) const {}
};

// VDP — stochastic Van der Pol oscillator, equation.py:179-238.  x = (x1, x2),
// c = d/2; px/nx are the cyclic shifts inside each half (:192-195).  The
// coupling between halves keeps the whole state in one lane (P = 1).
template <typename T, int D, int P>
struct EqVDP {
  static_assert(P == 1 && D % 2 == 0, "VDP keeps a trajectory in one lane");
  static constexpr int M = D, C = D / 2, MC = D / 2, kP = 1, CDIM = D / 2;
  static constexpr bool kNeedsNorm = false;
  T a, eps, q, gamma, geps, ga, two_ad, sqrt2, two_a, inv2q, two_ga, two_q;
  static EqVDP make(const dpac_eqn_params& e) {
    EqVDP r;
    r.a = (T)e.a; r.eps = (T)e.epsilon; r.q = (T)e.q; r.gamma = (T)e.gamma;
    r.geps = (T)(-e.gamma * e.epsilon);  // -gamma*epsl (:198)
    r.ga = (T)(e.gamma * e.a);           // gamma*a (:199)
    r.two_ad = (T)(2.0 * e.a * e.dim);   // 2*a*dim (:199)
    r.sqrt2 = (T)1.4142135623730951;
    r.two_a = (T)(2.0 * e.a);
    r.inv2q = (T)(1.0 / (2.0 * e.q));
    r.two_ga = (T)(2.0 * e.gamma * e.a);
    r.two_q = (T)(2.0 * e.q);
    return r;
  }
  __device__ __forceinline__ static constexpr int nxt(int i) { return (i + 1) % C; }
  __device__ __forceinline__ static constexpr int prv(int i) { return (i + C - 1) % C; }
  // dv = 2a*v - eps*(px + nx) on one half (:196-197, :217, :227)
  __device__ __forceinline__ void Lop(const T* v, T* o) const {
#pragma unroll
    for (int i = 0; i < C; ++i) o[i] = two_a * v[i] - eps * (v[nxt(i)] + v[prv(i)]);
  }
  __device__ __forceinline__ void u_true(const T (&x)[M], T, T (&u)[MC]) const {
    T dv2[C];
    Lop(x + C, dv2);
#pragma unroll
    for (int i = 0; i < C; ++i) u[i] = -dv2[i] / 2 / q;  // (:217)
  }
  __device__ __forceinline__ void drift(const T (&x)[M], const T (&u)[MC], T, T (&f)[M]) const {
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      f[i] = x2;
      f[C + i] = (1 - x1 * x1) * x2 - x1 + u[i];  // (:235)
    }
  }
  __device__ __forceinline__ void sigma(const T (&x)[M], const T (&u)[MC], T (&s)[M]) const {
#pragma unroll
    for (int m = 0; m < M; ++m) s[m] = sqrt2;
  }
  static void sigma_form(const dpac_eqn_params&, double& sa, double& sb) { sa = 1.4142135623730951; sb = 0.0; }
  __device__ __forceinline__ T w_part(const T (&x)[M], const T (&u)[MC]) const {
    T dv1[C], dv2[C];
    Lop(x, dv1);
    Lop(x + C, dv2);
    T acc = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      const T px1 = x[nxt(i)], px2 = x[C + nxt(i)];
      const T temp = geps * (x1 * px1 + x2 * px2) + (dv2[i] * dv2[i]) / 4 / q - x2 * dv1[i] -
                     ((1 - x1 * x1) * x2 - x1) * dv2[i];
      acc += temp + q * (u[i] * u[i]) + ga * (x1 * x1 + x2 * x2);
    }
    return acc;
  }
  __device__ __forceinline__ T w_finish(T s) const { return s - two_ad; }
  __device__ __forceinline__ T V_true(const T (&x)[M], T S, T r) const {  // (:210)
    T cross = 0;
#pragma unroll
    for (int i = 0; i < C; ++i) cross += x[i] * x[nxt(i)] + x[C + i] * x[C + nxt(i)];
    return a * S - eps * cross;
  }
  __device__ __forceinline__ T Z(const T (&x)[M], T S, T r) const { return V_true(x, S, r); }
  __device__ __forceinline__ void V_grad(const T (&x)[M], T S, T r, T (&g)[M]) const {  // (:227)
    Lop(x, g);
    Lop(x + C, g + C);
  }
  __device__ __forceinline__ void drift_vjp(const T (&x)[M], const T (&u)[MC], T r, const T (&a)[M],
                            T (&gx)[M], T (&gu)[MC]) const {
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i], a1 = a[i], a2v = a[C + i];
      gx[i] += a2v * (-2 * x1 * x2 - 1);
      gx[C + i] += a1 + a2v * (1 - x1 * x1);
      gu[i] += a2v;
    }
  }
  __device__ __forceinline__ void sigma_vjp(const T (&x)[M], const T (&u)[MC], const T (&a)[M], T (&gx)[M],
                            T (&gu)[MC]) const {}
  // gradient of w (derivation in DESIGN.md §4.3): with L v = 2a v - eps(px v + nx v),
  // g = (1 - x1^2) x2 - x1:
  //   dw/dx1 = -gamma*eps*(px1+nx1) + 2 x1 x2 dv2 + 2 gamma a x1
  //   dw/dx2 = -gamma*eps*(px2+nx2) + L(dv2)/(2q) - dv1 - (1 - x1^2) dv2 - L(g) + 2 gamma a x2
  __device__ __forceinline__ void w_vjp(const T (&x)[M], const T (&u)[MC], T gw, T (&gx)[M], T (&gu)[MC]) const {
    T dv1[C], dv2[C], g[C], Ldv2[C], Lg[C];
    Lop(x, dv1);
    Lop(x + C, dv2);
#pragma unroll
    for (int i = 0; i < C; ++i) g[i] = (1 - x[i] * x[i]) * x[C + i] - x[i];
    Lop(dv2, Ldv2);
    Lop(g, Lg);
#pragma unroll
    for (int i = 0; i < C; ++i) {
      const T x1 = x[i], x2 = x[C + i];
      const T s1 = x[nxt(i)] + x[prv(i)], s2 = x[C + nxt(i)] + x[C + prv(i)];
      const T d1 = geps * s1 + 2 * x1 * x2 * dv2[i] + two_ga * x1;
      const T d2 = geps * s2 + Ldv2[i] * inv2q - dv1[i] - (1 - x1 * x1) * dv2[i] - Lg[i] + two_ga * x2;
      gx[i] += gw * d1;
      gx[C + i] += gw * d2;
      gu[i] += gw * (two_q * u[i]);
    }
  }
};

}  // namespace dpac
