// dpac_mlp_x3.h — the row-parallel MLP kernels (dpac_mlp_rows.h) on split-fp16 MFMA.
//
// gfx950 runs v_mfma_f32_16x16x32_f16 at 16 times the FLOP rate of the f32-input
// v_mfma_f32_16x16x4_f32 (16 cycles per 16x16x32 vs 32 per 16x16x4).  An f32 operand
// a is carried as two fp16 numbers,
//     hi = fp16(a),   lo = fp16((a - hi) * 2^12),   a = hi + lo * 2^-12 (+ <= 2^-22 |a|),
// and a product of two such operands as three MFMAs accumulated in f32:
//     acc_hi += A_hi B_hi,   acc_lo += A_hi B_lo + A_lo B_hi,   C = acc_hi + acc_lo * 2^-12
// (the dropped A_lo B_lo term is below 2^-24 |a b|).  That is the f32 product to within
// the f32 accumulation error (DESIGN.md §4.3 measures both against the float64 oracle)
// at 3 x 16 = 48 cycles per 16x16x32 step instead of 8 x 32 = 256: 5.3x fewer MFMA
// cycles.  lo scaled by 2^12 stays a normal fp16 number wherever hi is; the backward
// chain, whose gradients are small (~1/B), is scaled per row by a power of two first
// (exact, undone when G is stored).  Range: |a| (and |a| times the row scale) < 2^15: every
// split reports an operand outside it, and the kernel then sets the caller's status word
// (dpac.h dpac_mlp.status), after which the f32 kernel of the same launch recomputes every
// output (dpac_mlp.hip); a kernel that finds the word already set does no work.
//
// Every product is formed transposed, C^T = W^T act^T: the weight image is the MFMA's A
// operand (lane l: output feature l&15 of the tile, k = 32c + 8(l>>4) .. +7), the LDS
// activation image its B operand (lane l: batch row l&15, the same 8 k), so the
// accumulator gives lane l the FOUR CONSECUTIVE features 4(l>>4) .. +3 of batch row l&15:
// the epilogue stores each row's z / G as one 16-byte store and writes the next layer's
// operand as two 8-byte LDS writes (hi, lo), with no cross-lane exchange.
//
// Layouts.  A row's activations live in LDS as 32-wide k chunks of 64 halves,
// [hi(k0..k0+31) | lo(k0..k0+31)], row stride kX3Ld halves (264 dwords = 8 mod 64:
// conflict-free ds_read_b128 as in dpac_mlp_rows.h).  The weight images
// (dpac_mlp.weight_x3 / weight_t_x3, written by dpac_mlp_prepare) are fragment-major:
// per 16-feature tile, chunk and part (hi, lo) the 64 lanes' A operands, lane-ordered, so
// one buffer_load_dwordx4 of a wave reads 1 KB of contiguous memory (8 cache lines; the
// feature-major image of round 3's first build touched 16 half-used lines per quarter-wave,
// and in the fused NN rollout those loads, not the MFMAs, set the step time).
//
// Workgroup: 8 wavefronts over kX3Rows = 64 rows (4 row tiles); the waves split the
// 16-feature tiles (wave, wave + 8); every weight fragment serves the 4 row tiles, so the
// weights stream from L2 once per 64 rows (4x less than the 16-row f32 kernel).
#pragma once

#include "dpac_mlp_rows.h"

namespace dpac {

typedef _Float16 x3h8 __attribute__((ext_vector_type(8)));
typedef _Float16 x3h4 __attribute__((ext_vector_type(4)));
typedef float x3f4 __attribute__((ext_vector_type(4)));

constexpr int kX3Waves = 8;
constexpr int kX3Threads = 64 * kX3Waves;
#ifndef DPAC_X3_RT
#define DPAC_X3_RT 4  // row tiles per workgroup of the forward (timing knob)
#endif
#ifndef DPAC_X3_RT_BWD
#define DPAC_X3_RT_BWD 2  // of the backward chain: at 4 it needs > 256 VGPRs and spills 432 B per lane
#endif
constexpr int kX3RT = DPAC_X3_RT;         // row tiles per workgroup (forward)
constexpr int kX3Rows = 16 * kX3RT;       // 64 rows
constexpr int kX3RTB = DPAC_X3_RT_BWD;    // row tiles per workgroup (backward)
constexpr int kX3RowsB = 16 * kX3RTB;     // 32 rows
constexpr int kX3MaxChunks = (DPAC_MLP_MAX_WIDTH + 31) / 32;  // 8
#ifndef DPAC_X3_LDPAD
#define DPAC_X3_LDPAD 16  // halves of padding per LDS row (a multiple of 8: 16-byte rows)
#endif
constexpr int kX3Ld = 64 * kX3MaxChunks + DPAC_X3_LDPAD;      // halves per LDS row (1056 B at 16)
constexpr float kX3LoScale = 4096.f;      // 2^12
constexpr float kX3LoInv = 1.f / 4096.f;
constexpr int kX3MaxNT = (DPAC_MLP_MAX_WIDTH / 16 + kX3Waves - 1) / kX3Waves;  // 2
static_assert(kX3MaxNT == 2, "the dispatch below covers 1..2 feature tiles per wave");

__host__ __device__ constexpr int x3_chunks(int k) { return (k + 31) / 32; }

// Timing-only builds (-DDPAC_X3_TRACE=1): lane 0 of every wavefront of the first 256
// workgroups records the shader clock at fixed points (start, prologue done, then per layer
// K loop done / layer barrier passed) into g_x3_trace, read by dpac_debug_x3_trace.
#ifndef DPAC_X3_TRACE
#define DPAC_X3_TRACE 0
#endif
#if DPAC_X3_TRACE
__device__ uint32_t g_x3_trace[256 * 8 * 16];  // [block][wave][point]
#define X3_MARK(pt)                                                                          \
  do {                                                                                       \
    if (blockIdx.x < 256 && (threadIdx.x & 63) == 0)                                         \
      g_x3_trace[(blockIdx.x * 8 + threadIdx.x / 64) * 16 + (pt)] = (uint32_t)__builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define X3_MARK(pt) \
  do {              \
  } while (0)
#endif

#ifndef DPAC_X3_SPF
#define DPAC_X3_SPF 2  // chunks of weights in flight ahead of the one being multiplied (forward)
#endif
#ifndef DPAC_X3_SPF_BWD
#define DPAC_X3_SPF_BWD 2  // the same for the backward chain
#endif
#ifndef DPAC_X3_BWD_MINB
#define DPAC_X3_BWD_MINB 1  // min waves per SIMD the backward is compiled for (launch bounds; timing knob)
#endif
#ifndef DPAC_X3_MASK_EARLY
#define DPAC_X3_MASK_EARLY 1  // the backward's sign-bit word loaded before the K loop (1) or after it (0)
#endif

__device__ __forceinline__ void x3_split(float a, _Float16& hi, _Float16& lo) {
  hi = (_Float16)a;
  lo = (_Float16)((a - (float)hi) * kX3LoScale);
}

// one element into a split LDS image (prologue); true if it is outside the split range
__device__ __forceinline__ bool x3_put(_Float16* img, int row, int col, float v) {
  _Float16 h, l;
  x3_split(v, h, l);
  _Float16* p = img + row * kX3Ld + (col >> 5) * 64 + (col & 31);
  p[0] = h;
  p[32] = l;
  return x3_bad(v);
}

// four consecutive features f0..f0+3 (f0 % 4 == 0) of one row: two 8-byte LDS writes; true
// if one of them is outside the split range
__device__ __forceinline__ bool x3_put4(_Float16* img, int row, int f0, x3f4 v) {
  x3h4 h, l;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (_Float16)v[e];
    l[e] = (_Float16)((v[e] - (float)h[e]) * kX3LoScale);
  }
  _Float16* p = img + row * kX3Ld + (f0 >> 5) * 64 + (f0 & 31);
  *reinterpret_cast<x3h4*>(p) = h;
  *reinterpret_cast<x3h4*>(p + 32) = l;
  return x3_bad4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ x3f4 x3_mma(x3h8 a, x3h8 b, x3f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

// four consecutive floats at element offset `off` of the workgroup's rows of an array
// (buffer descriptor r over them, plain pointer p to their start): one 16-byte buffer
// store when all four features exist (rows past the live ones fall outside r and are
// dropped), else plain stores of the existing ones in live rows
__device__ __forceinline__ void x3_store4(__amdgpu_buffer_rsrc_t r, float* p, uint32_t off, int nvalid, bool live,
                                          x3f4 v) {
  if (nvalid >= 4) {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v), r,
                                           (int)(off * 4), 0, 0);
  } else if (live) {
#pragma unroll
    for (int e = 0; e < 3; ++e)
      if (e < nvalid) p[off + e] = v[e];
  }
}

__device__ __forceinline__ x3f4 x3_load4(__amdgpu_buffer_rsrc_t r, const float* p, uint32_t off, int nvalid, bool live) {
  if (nvalid >= 4) return __builtin_bit_cast(x3f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(off * 4), 0, 0));
  x3f4 v{0, 0, 0, 0};
  if (live) {
#pragma unroll
    for (int e = 0; e < 3; ++e)
      if (e < nvalid) v[e] = p[off + e];
  }
  return v;
}

// acc[RT][NT] = (in[64 x K] @ W[K x Nout])^T for this wave's NT feature tiles (tile
// wave + 8j), then epi.store(j, rt, z) with z the lane's four features of its row.  NCH
// = ceil(K / 32) as a template constant (straight-line code, counted waits) or 0
// (runtime K, single-buffered).  epi.pre<NT>() runs before the K loop, epi.post<NT>()
// after it.  Returns whether a stored operand left the split range (epi.store's result).
template <int NT, int NCH, int RT, int SPF, class EPI>
__device__ __forceinline__ bool x3_layer_t(const _Float16* in, int K, int Nout, const _Float16* Wx3, int wave,
                                           int lane, EPI& epi) {
  const int col_l = lane & 15, q = lane >> 4;
  const int nch = NCH ? NCH : x3_chunks(K);
  const int ntiles = (Nout + 15) / 16;
  const __amdgpu_buffer_rsrc_t rW = make_rsrc(Wx3, (uint32_t)(ntiles * nch * 2048));
  uint32_t voff[NT];
  x3f4 ah[RT][NT], al[RT][NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int tile = wave + kX3Waves * j;
    voff[j] = tile < ntiles ? (uint32_t)(tile * nch * 2048 + 16 * lane) : kOOB;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ah[rt][j] = al[rt][j] = x3f4{0, 0, 0, 0};
  }
  (void)col_l;
  auto loadW = [&](int c, int j, int part) {  // part 0: hi, 1: lo; one contiguous KB per wave
    return __builtin_bit_cast(x3h8, __builtin_amdgcn_raw_buffer_load_b128(
                                        rW, (int)(voff[j] + (uint32_t)(c * 2048 + 1024 * part)), 0, 0));
  };
  const _Float16* arow = in + col_l * kX3Ld + 8 * q;
  auto loadX = [&](int c, int rt, int part) {
    return *reinterpret_cast<const x3h8*>(arow + rt * 16 * kX3Ld + c * 64 + 32 * part);
  };
  auto step = [&](const x3h8 (&wh)[NT], const x3h8 (&wl)[NT], const x3h8 (&xh)[RT], const x3h8 (&xl)[RT]) {
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        ah[rt][j] = x3_mma(wh[j], xh[rt], ah[rt][j]);
        al[rt][j] = x3_mma(wh[j], xl[rt], al[rt][j]);
        al[rt][j] = x3_mma(wl[j], xh[rt], al[rt][j]);
      }
  };
  if constexpr (NCH > 0) {
    constexpr int PF = SPF < NCH ? SPF : NCH;
    x3h8 wh[PF][NT], wl[PF][NT];
#pragma unroll
    for (int f = 0; f < PF; ++f)
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        wh[f][j] = loadW(f, j, 0);
        wl[f][j] = loadW(f, j, 1);
      }
    epi.template pre<NT>(wave, lane);
    x3h8 xh[2][RT], xl[2][RT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) {
      xh[0][rt] = loadX(0, rt, 0);
      xl[0][rt] = loadX(0, rt, 1);
    }
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      const int sx = c & 1, sw = c % PF;
      if (c + 1 < NCH) {
#pragma unroll
        for (int rt = 0; rt < RT; ++rt) {
          xh[sx ^ 1][rt] = loadX(c + 1, rt, 0);
          xl[sx ^ 1][rt] = loadX(c + 1, rt, 1);
        }
      }
      x3h8 ch[NT], cl[NT];
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        ch[j] = wh[sw][j];
        cl[j] = wl[sw][j];
        if (c + PF < NCH) {  // refill the slot just taken
          wh[sw][j] = loadW(c + PF, j, 0);
          wl[sw][j] = loadW(c + PF, j, 1);
        }
      }
      step(ch, cl, xh[sx], xl[sx]);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads where they are issued
    }
  } else {
    epi.template pre<NT>(wave, lane);
    x3h8 wh[NT], wl[NT], xh[RT], xl[RT];
    for (int c = 0; c < nch; ++c) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        wh[j] = loadW(c, j, 0);
        wl[j] = loadW(c, j, 1);
      }
#pragma unroll
      for (int rt = 0; rt < RT; ++rt) {
        xh[rt] = loadX(c, rt, 0);
        xl[rt] = loadX(c, rt, 1);
      }
      step(wh, wl, xh, xl);
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  X3_MARK(epi.mark);
  epi.template post<NT>(wave, lane);
  bool bad = false;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) bad |= epi.store(j, rt, ah[rt][j] + al[rt][j] * kX3LoInv, wave, lane);
  epi.finish(lane);
  return bad;
}

template <int RT = kX3RT, int SPF = DPAC_X3_SPF, class EPI>
__device__ __forceinline__ bool x3_layer(const _Float16* in, int K, int Nout, const _Float16* Wx3, int wave,
                                         int lane, EPI& epi) {
  const int ntiles = (Nout + 15) / 16;
  const int mine = ntiles > wave ? (ntiles - wave + kX3Waves - 1) / kX3Waves : 0;
  const int nch = x3_chunks(K);
  // straight-line layers for the shipped shapes (d <= 32: one chunk; 193..224 wide: seven)
  if (nch == 1) {
    if (mine == 1) return x3_layer_t<1, 1, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
    if (mine == 2) return x3_layer_t<2, 1, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
  } else if (nch == 7) {
    if (mine == 1) return x3_layer_t<1, 7, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
    if (mine == 2) return x3_layer_t<2, 7, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
  } else if (mine == 1) {
    return x3_layer_t<1, 0, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
  } else if (mine == 2) {
    return x3_layer_t<2, 0, RT, SPF>(in, K, Nout, Wx3, wave, lane, epi);
  }
  epi.finish(lane);  // a wave without tiles: its (zero) sign-bit mask word
  return false;
}

struct X3Args {
  int64_t rows;
  int L;
  int width[DPAC_MLP_MAX_HIDDEN + 2];
  const float* scale[DPAC_MLP_MAX_HIDDEN + 2];
  const float* shift[DPAC_MLP_MAX_HIDDEN + 2];
  const _Float16* wx3[DPAC_MLP_MAX_HIDDEN + 1];  // forward: weight_x3; backward: weight_t_x3
  const float* bias;
  int zoff[DPAC_MLP_MAX_HIDDEN + 2], goff[DPAC_MLP_MAX_HIDDEN + 2];
  int ztot, gtot;
  const float* x;
  int64_t ldx;
  float* out;
  float* z;
  const float* g_out;
  float* G;
  float* g_x;
  // TD1 fused (as MrArgs)
  const float *td_x, *td_u, *td_dw;
  int64_t td_ldx;
  int td_ldu, td_p;
  float td_sa, td_sb;
  float* gdot;
  const float* g_gdot;
  uint32_t* status;  // the range guard (dpac_mlp.status), or null
  // the hidden activations' sign bits (dpac.h dpac_mlp_rows_fwd_masked): per hidden layer h
  // (1..L) and 64-row block b, 512 words; word ((h - 1) nblk + b) 512 + 64 w + 16 q + r holds at
  // bit 4 (2 rt + j) + e whether BN_h's output of row 64 b + 16 rt + r, feature 16 (w + 8 j) +
  // 4 q + e, is > 0 — exactly the nibbles lane 16 q + r of wave w holds in the 64-row forward
  // (x3_f0), so each lane writes one word per layer.  Written by the forward, read by the
  // backward instead of z (null: not written / z read).
  uint32_t* mask;
  int64_t nblk;  // ceil(rows / 64)
};
constexpr int kX3MaskWords = 512;  // per hidden layer and 64-row block
static_assert(4 % kX3RTB == 0, "a backward workgroup's row tiles lie in one 64-row mask block");
static_assert(kX3Waves == 8 && kX3MaxNT == 2, "the mask word holds 2 tiles x 4 row tiles of one lane");

// the lane's feature quad f0 = 16 tile + 4 (l >> 4) and how many of its features exist
__device__ __forceinline__ int x3_f0(int wave, int j, int lane) { return (wave + kX3Waves * j) * 16 + 4 * (lane >> 4); }
__device__ __forceinline__ int x3_nvalid(int f0, int Nout) { return Nout - f0 < 0 ? 0 : (Nout - f0 > 4 ? 4 : Nout - f0); }

// Forward epilogue of dense layer l: z -> save -> BN(z (+ b)) -> then by MODE: [y + relu(y)]
// split into the next LDS image (hidden), the f32 rows of the TD1 dot (stage), or `out`.
enum { kX3Hidden = 0, kX3Stage = 1, kX3Out = 2 };
template <int MODE>
struct X3FwdEpi {
  int mark;                  // trace point of this layer's K loop end (DPAC_X3_TRACE)
  const float *scale, *shift, *bias;
  int rows_live, Nout;
  _Float16* img;             // hidden: next layer's input image
  float* stage;              // stage: [64][kMrLd] f32 (overlays the free image)
  __amdgpu_buffer_rsrc_t rz; // saves of the workgroup's rows at this layer (num_records: live rows)
  bool save;
  int z_ld;                  // floats
  __amdgpu_buffer_rsrc_t ro; // out: the workgroup's rows
  float *zp, *op;            // the same rows as plain pointers (x3_store4's partial quads)
  uint32_t* mp;              // hidden: the layer's mask words of the workgroup's 64-row block, or null
  uint32_t mword;            // the lane's sign nibbles, bit 4 (2 rt + j) + e
  x3f4 s[kX3MaxNT], sh[kX3MaxNT], bb[kX3MaxNT];
  template <int NT>
  __device__ __forceinline__ void pre(int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int f0 = x3_f0(wave, j, lane);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool v = f0 + e < Nout;
        s[j][e] = v ? scale[f0 + e] : 0.f;
        sh[j][e] = v ? shift[f0 + e] : 0.f;
        bb[j][e] = (v && MODE != kX3Hidden) ? bias[f0 + e] : 0.f;
      }
    }
  }
  template <int NT>
  __device__ __forceinline__ void post(int, int) {}
  __device__ __forceinline__ void finish(int lane) {  // one mask word per lane and layer
    if (MODE == kX3Hidden && mp) mp[lane] = mword;
  }
  __device__ __forceinline__ bool store(int j, int rt, x3f4 zv, int wave, int lane) {
    const int f0 = x3_f0(wave, j, lane), nv = x3_nvalid(f0, Nout);
    const int row = rt * 16 + (lane & 15);
    if (save) x3_store4(rz, zp, (uint32_t)(row * z_ld + f0), nv, row < rows_live, zv);
    x3f4 y = zv;
    if (MODE != kX3Hidden) y = y + bb[j];  // addmm(b, y, W) (solver.py:270)
    y = sh[j] + y * s[j];                  // addcmul(beta, y, gamma/sqrt(1+eps))
    if (MODE == kX3Hidden) {
      uint32_t nib = 0;  // the sign bits the backward's activation factor needs (MASKED)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        nib |= (e < nv && y[e] > 0.f) ? 1u << e : 0u;
        y[e] = e < nv ? y[e] + fmaxf(y[e], 0.f) : 0.f;  // y + relu(y) (solver.py:269)
      }
      if (row < rows_live) mword |= nib << (4 * (2 * rt + j));
      return x3_put4(img, row, f0, y);
    } else if (MODE == kX3Stage) {
#pragma unroll
      for (int e = 0; e < 4; ++e) y[e] = e < nv ? y[e] : 0.f;
      *reinterpret_cast<x3f4*>(stage + row * kMrLd + f0) = y;
    } else {
      x3_store4(ro, op, (uint32_t)(row * Nout + f0), nv, row < rows_live, y);
    }
    return false;
  }
};

// Backward epilogue of g = G_{l+1} @ (W_l diag s_{l+1})^T: times 1 + [BN_l(z_l) > 0] for
// l >= 1 (FIRST = false), the sign from the forward's saved z or (MASKED) from its sign-bit
// bytes; G_l (unscaled by the row's power of two) to global; scaled and split into LDS; for
// l == 0 (FIRST) also dL/dx = G_0 * s_0.
template <bool FIRST, bool MASKED = false, int RT = kX3RTB>
struct X3BwdEpi {
  int mark;                    // trace point of this layer's K loop end (DPAC_X3_TRACE)
  const float *scale, *shift;  // BN_l (l >= 1)
  int rows_live, Nout;
  _Float16* img;
  __amdgpu_buffer_rsrc_t rz;   // the forward's z_l of the workgroup's rows
  int z_ld;
  __amdgpu_buffer_rsrc_t rg;   // G_l
  int g_ld;
  __amdgpu_buffer_rsrc_t rx;   // dL/dx (FIRST, optional)
  bool gx;
  const float* s0;
  const float* rinv;           // LDS: 2^-e of each row (undoes the chain's row scale)
  const float* zp;             // plain pointers to the same rows (partial quads)
  float *gp, *xp;
  const uint32_t* mp;          // MASKED: layer l's mask words of the workgroup's 64-row block
  int mshift;                  // MASKED: 4 * 2 * (the workgroup's first row tile within the block)
  x3f4 s[kX3MaxNT], sh[kX3MaxNT];
  float ri[RT];
  x3f4 zz[MASKED ? 1 : kX3MaxNT][MASKED ? 1 : RT];  // z_l of the lane's quads, loaded in post()
  uint32_t mword;              // MASKED: the lane's mask word (loaded in post())
  template <int NT>
  __device__ __forceinline__ void pre(int wave, int lane) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int f0 = x3_f0(wave, j, lane);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool v = f0 + e < Nout;
        s[j][e] = !v ? 0.f : (FIRST ? s0[f0 + e] : scale[f0 + e]);
        sh[j][e] = (v && !FIRST) ? shift[f0 + e] : 0.f;
      }
    }
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) ri[rt] = rinv[rt * 16 + (lane & 15)];
    if constexpr (!FIRST && MASKED && DPAC_X3_MASK_EARLY) mword = mp[lane] >> mshift;
  }
  template <int NT>
  __device__ __forceinline__ void post(int wave, int lane) {  // every z load, then one wait
    if constexpr (!FIRST && MASKED) {
      if constexpr (!DPAC_X3_MASK_EARLY) mword = mp[lane] >> mshift;
    } else if constexpr (!FIRST) {
#pragma unroll
      for (int j = 0; j < NT; ++j) {
        const int f0 = x3_f0(wave, j, lane), nv = x3_nvalid(f0, Nout);
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
          zz[j][rt] = x3_load4(rz, zp, (uint32_t)((rt * 16 + (lane & 15)) * z_ld + f0), nv,
                               rt * 16 + (lane & 15) < rows_live);
      }
    }
  }
  __device__ __forceinline__ void finish(int) {}
  __device__ __forceinline__ bool store(int j, int rt, x3f4 v, int wave, int lane) {
    const int f0 = x3_f0(wave, j, lane), nv = x3_nvalid(f0, Nout);
    const int row = rt * 16 + (lane & 15);
    if constexpr (!FIRST && MASKED) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] * (((mword >> (4 * (2 * rt + j) + e)) & 1u) ? 2.f : 1.f);  // d(y + relu(y))/dy
    } else if constexpr (!FIRST) {
      const x3f4 y = sh[j] + zz[j][rt] * s[j];  // the forward's BN_l output
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = v[e] * (y[e] > 0.f ? 2.f : 1.f);  // d(y + relu(y))/dy
    }
    const x3f4 vt = v * ri[rt];                  // exact: a power of two
    x3_store4(rg, gp, (uint32_t)(row * g_ld + f0), nv, row < rows_live, vt);
    if (FIRST && gx) x3_store4(rx, xp, (uint32_t)(row * Nout + f0), nv, row < rows_live, vt * s[j]);  // G_0 * s_0
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = e < nv ? v[e] : 0.f;
    return x3_put4(img, row, f0, v);
  }
};

template <int ROWS = kX3Rows>
__device__ __forceinline__ void x3_zero(_Float16* img, int tid) {
  uint4* p = reinterpret_cast<uint4*>(img);
  constexpr int n = ROWS * kX3Ld * 2 / 16;
  for (int e = tid; e < n; e += kX3Threads) p[e] = uint4{0, 0, 0, 0};
}

// LDS of the x3 row kernels: two split images (the output layer's f32 rows for the TD1 dot
// reuse the free one: 64 x kMrLd floats = one image) + the backward's row scales (132 KB)
constexpr uint32_t kX3ImgBytes = kX3Rows * kX3Ld * 2;
static_assert(kX3Rows * kMrLd * 4 <= kX3ImgBytes, "the f32 staging rows fit in one split image");
constexpr uint32_t kX3LdsBytes = 2 * kX3ImgBytes + kX3Rows * 4;
constexpr uint32_t kX3ImgBytesB = kX3RowsB * kX3Ld * 2;  // the backward's (kX3RTB row tiles)
constexpr uint32_t kX3LdsBytesB = 2 * kX3ImgBytesB + kX3RowsB * 4;

// rows [row0, row0 + live) of a [rows][ld] float array as a buffer descriptor
__device__ __forceinline__ __amdgpu_buffer_rsrc_t x3_rows_rsrc(const float* base, int64_t row0, int live, int ld) {
  return make_rsrc(base ? base + row0 * ld : nullptr, base ? (uint32_t)(live * ld * 4) : 0u);
}

// x[row0 + r][k] of the forward's row block through its row descriptor (0 past the block)
__device__ __forceinline__ float x3_x_at(__amdgpu_buffer_rsrc_t rx, int r, int k, int64_t ldx, int live) {
  DPAC_CHECK_ROW(r, live);
  return buf_load_elem<float>(rx, (uint32_t)(r * ldx + k) * 4u);
}

__global__ __launch_bounds__(kX3Threads) void k_mlp_rows_fwd_x3(const X3Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char x3_lds[];
  _Float16* const img0 = reinterpret_cast<_Float16*>(x3_lds);
  _Float16* const img1 = reinterpret_cast<_Float16*>(x3_lds + kX3ImgBytes);
  auto img = [&](int i) { return i ? img1 : img0; };
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  if (x3_status_set(a.status)) return;  // fell back: the f32 kernel after this one does the work
  const int64_t row0 = (int64_t)blockIdx.x * kX3Rows;
  const int rows_live = (int)((a.rows - row0) < kX3Rows ? (a.rows - row0) : kX3Rows);
  const int d = a.width[0];
  const __amdgpu_buffer_rsrc_t rx0 = rows_rsrc(a.x, row0, rows_live, a.ldx);
  bool bad = false;  // an operand outside the split range (dpac.h dpac_mlp.status)
  X3_MARK(0);
  // a_0 = BN_0(x) (solver.py:265): for d <= 32 the loads go first, their latency under the
  // LDS clear (64 rows x 32 features = 4 per thread)
  constexpr int kPro = kX3Rows * 32 / kX3Threads;
  const bool narrow = d <= 32;
  float xv[kPro];
#pragma unroll
  for (int t = 0; t < kPro; ++t) {
    const int e = tid + t * kX3Threads, r = e / d, k = e % d;
    xv[t] = (narrow && e < kX3Rows * d && r < rows_live) ? x3_x_at(rx0, r, k, a.ldx, rows_live) : 0.f;
  }
  x3_zero(img0, tid);
  x3_zero(img1, tid);
  __syncthreads();
  if (narrow) {
#pragma unroll
    for (int t = 0; t < kPro; ++t) {
      const int e = tid + t * kX3Threads, r = e / d, k = e % d;
      if (e < kX3Rows * d) bad |= x3_put(img0, r, k, r < rows_live ? a.shift[0][k] + xv[t] * a.scale[0][k] : 0.f);
    }
  } else {
    for (int e = tid; e < kX3Rows * d; e += kX3Threads) {
      const int r = e / d, k = e % d;
      bad |= x3_put(img0, r, k, r < rows_live ? a.shift[0][k] + x3_x_at(rx0, r, k, a.ldx, rows_live) * a.scale[0][k] : 0.f);
    }
  }
  MrArgs<float> ta{};  // the TD1 operands, as dpac_mlp_rows.h's td_dot_rows reads them
  ta.td_x = a.td_x; ta.td_u = a.td_u; ta.td_dw = a.td_dw; ta.td_ldx = a.td_ldx; ta.td_ldu = a.td_ldu;
  ta.td_p = a.td_p; ta.td_sa = a.td_sa; ta.td_sb = a.td_sb; ta.gdot = a.gdot;
  __syncthreads();
  X3_MARK(1);
  int pq = 0;
  for (int l = 0; l <= a.L; ++l) {
    const int Nout = a.width[l + 1];
    const __amdgpu_buffer_rsrc_t rz = x3_rows_rsrc(a.z ? a.z + a.zoff[l + 1] : nullptr, row0, rows_live, a.ztot);
    float* zp = a.z ? a.z + a.zoff[l + 1] + row0 * a.ztot : nullptr;
    if (l < a.L) {
      X3FwdEpi<kX3Hidden> epi{2 + 2 * l, a.scale[l + 1], a.shift[l + 1], nullptr, rows_live, Nout, img(pq ^ 1),
                              nullptr, rz, a.z != nullptr, a.ztot, make_rsrc(nullptr, 0), zp, nullptr,
                              a.mask ? a.mask + ((int64_t)l * a.nblk + blockIdx.x) * kX3MaskWords + wave * 64
                                     : nullptr,
                              0u};
      bad |= x3_layer(img(pq), a.width[l], Nout, a.wx3[l], wave, lane, epi);
    } else if (a.gdot) {
      X3FwdEpi<kX3Stage> epi{2 + 2 * l, a.scale[l + 1], a.shift[l + 1], a.bias, rows_live, Nout, nullptr,
                             reinterpret_cast<float*>(img(pq ^ 1)), rz, a.z != nullptr, a.ztot, make_rsrc(nullptr, 0),
                             zp, nullptr, nullptr, 0u};
      x3_layer(img(pq), a.width[l], Nout, a.wx3[l], wave, lane, epi);
    } else {
      X3FwdEpi<kX3Out> epi{2 + 2 * l, a.scale[l + 1], a.shift[l + 1], a.bias, rows_live, Nout, nullptr, nullptr,
                           rz, a.z != nullptr, a.ztot, x3_rows_rsrc(a.out, row0, rows_live, Nout), zp,
                           a.out + row0 * Nout, nullptr, 0u};
      x3_layer(img(pq), a.width[l], Nout, a.wx3[l], wave, lane, epi);
    }
    __syncthreads();
    X3_MARK(3 + 2 * l);
    pq ^= 1;
  }
  if (a.gdot && tid < kMrThreads) {  // the TD1 dot per row (k_td's lane split and DPP tree)
    const float* stage = reinterpret_cast<const float*>(img(pq));
    const int dd = a.width[a.L + 1];
    float pre[kTdPre];
    for (int r0 = 0; r0 < kX3Rows; r0 += kMrThreads / 16)
      td_dot_rows<float, kMrThreads / 16>(ta, stage + r0 * kMrLd, row0 + r0, rows_live - r0 < 0 ? 0 : rows_live - r0,
                                          dd, tid, false, pre);
  }
  if (bad) x3_flag(a.status);
}

// MASKED: the activation factors from the forward's sign-bit bytes (a.mask) instead of z
template <bool MASKED>
__global__ __launch_bounds__(kX3Threads, DPAC_X3_BWD_MINB) void k_mlp_rows_bwd_x3(const X3Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char x3_lds[];
  _Float16* const img0 = reinterpret_cast<_Float16*>(x3_lds);
  _Float16* const img1 = reinterpret_cast<_Float16*>(x3_lds + kX3ImgBytesB);
  auto img = [&](int i) { return i ? img1 : img0; };
  float* rinv = reinterpret_cast<float*>(x3_lds + 2 * kX3ImgBytesB);
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  if (x3_status_set(a.status)) return;  // fell back: the f32 kernel after this one does the work
  const int64_t row0 = (int64_t)blockIdx.x * kX3RowsB;
  const int rows_live = (int)((a.rows - row0) < kX3RowsB ? (a.rows - row0) : kX3RowsB);
  const int L = a.L, hout = a.width[L + 1];
  bool bad = false;
  X3_MARK(0);
  MrArgs<float> ta{};
  ta.td_x = a.td_x; ta.td_u = a.td_u; ta.td_dw = a.td_dw; ta.td_ldx = a.td_ldx; ta.td_ldu = a.td_ldu;
  ta.td_sa = a.td_sa; ta.td_sb = a.td_sb;
  // G_{L+1} = dL/d out, row by row (8 lanes per row): to G unscaled, and times the row's
  // power of two 2^e (max |G_{L+1}| of the row in [1, 2)) split into image 0.  Round 6: for
  // hout <= 32 (the G network's d) the loads are issued first and kept in registers, their
  // latency under the LDS clear (rounds 3-5 loaded every element twice, after the clear).
  {
    const int r = tid / 8, sub = tid % 8;  // 8 lanes per row (kX3RowsB rows: the first 8 kX3RowsB threads)
    const bool live = r < rows_live;
    const int64_t gr = row0 + (live ? r : 0);
    const TdSrc<float> src = td_src(ta, row0, rows_live, hout);
    const __amdgpu_buffer_rsrc_t rgd = rows_rsrc(a.g_gdot, row0, rows_live, 1);
    const __amdgpu_buffer_rsrc_t rgo = rows_rsrc(a.g_out, row0, rows_live, hout);
    auto g_top = [&](int k) {  // dL/d out of row gr, column k (0 for a dead row)
      DPAC_CHECK_ROW(gr - row0, rows_live);
      const uint32_t o = (uint32_t)(gr - row0);
      return a.g_gdot ? buf_load_elem<float>(rgd, o * 4u) * td_sdw(src, gr, k)
                      : buf_load_elem<float>(rgo, (o * (uint32_t)hout + (uint32_t)k) * 4u);
    };
    constexpr int kTopReg = 4;
    const bool inreg = hout <= 8 * kTopReg;
    float gv[kTopReg];
#pragma unroll
    for (int i = 0; i < kTopReg; ++i) {
      const int k = sub + 8 * i;
      gv[i] = (inreg && live && k < hout) ? g_top(k) : 0.f;
    }
    x3_zero<kX3RowsB>(img0, tid);
    x3_zero<kX3RowsB>(img1, tid);
    float mx = 0.f;
    if (inreg) {
#pragma unroll
      for (int i = 0; i < kTopReg; ++i) {
        const int k = sub + 8 * i;
        if (live && k < hout) a.G[gr * a.gtot + a.goff[L + 1] + k] = gv[i];
        mx = fmaxf(mx, fabsf(gv[i]));
      }
    } else {
      for (int k = sub; k < hout; k += 8) {
        const float v = live ? g_top(k) : 0.f;
        if (live) a.G[gr * a.gtot + a.goff[L + 1] + k] = v;
        mx = fmaxf(mx, fabsf(v));
      }
    }
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) mx = fmaxf(mx, __shfl_xor(mx, m, 64));
    int e = 0;
    if (mx > 0.f && mx < 3.0e38f) (void)frexpf(mx, &e);  // mx in [2^(e-1), 2^e)
    const float sc = ldexpf(1.f, 1 - e);                   // max |G| * sc in [1, 2)
    __syncthreads();  // the images are clear
    if (inreg) {
#pragma unroll
      for (int i = 0; i < kTopReg; ++i) {
        const int k = sub + 8 * i;
        if (r < kX3RowsB && k < hout) bad |= x3_put(img0, r, k, gv[i] * sc);
      }
    } else {
      for (int k = sub; k < hout; k += 8) {
        const float v = live ? g_top(k) : 0.f;
        if (r < kX3RowsB) bad |= x3_put(img0, r, k, v * sc);
      }
    }
    if (sub == 0 && r < kX3RowsB) rinv[r] = ldexpf(1.f, e - 1);
  }
  __syncthreads();
  X3_MARK(1);
  int pq = 0;
  for (int l = L; l >= 0; --l) {
    const __amdgpu_buffer_rsrc_t rg = x3_rows_rsrc(a.G + a.goff[l], row0, rows_live, a.gtot);
    float* gp = a.G + a.goff[l] + row0 * a.gtot;
    if (l >= 1) {
      X3BwdEpi<false, MASKED> epi{2 + 2 * (L - l), a.scale[l], a.shift[l], rows_live, a.width[l], img(pq ^ 1),
                                  x3_rows_rsrc(MASKED ? nullptr : a.z + a.zoff[l], row0, rows_live, a.ztot), a.ztot,
                                  rg, a.gtot, make_rsrc(nullptr, 0), false, nullptr, rinv,
                                  a.z + a.zoff[l] + row0 * a.ztot, gp, nullptr,
                                  MASKED ? a.mask + ((int64_t)(l - 1) * a.nblk + (row0 >> 6)) * kX3MaskWords + wave * 64
                                         : nullptr,
                                  8 * (int)((row0 & 63) >> 4)};
      bad |= x3_layer<kX3RTB, DPAC_X3_SPF_BWD>(img(pq), a.width[l + 1], a.width[l], a.wx3[l], wave, lane, epi);
    } else {
      X3BwdEpi<true> epi{2 + 2 * L, nullptr, nullptr, rows_live, a.width[0], img(pq ^ 1), make_rsrc(nullptr, 0), 0, rg, a.gtot,
                         x3_rows_rsrc(a.g_x, row0, rows_live, a.width[0]), a.g_x != nullptr, a.scale[0], rinv,
                         nullptr, gp, a.g_x ? a.g_x + row0 * a.width[0] : nullptr, nullptr, 0};
      x3_layer<kX3RTB, DPAC_X3_SPF_BWD>(img(pq), a.width[1], a.width[0], a.wx3[0], wave, lane, epi);  // dL/dx: not split again
    }
    __syncthreads();
    X3_MARK(3 + 2 * (L - l));
    pq ^= 1;
  }
  if (bad) x3_flag(a.status);
}

}  // namespace dpac
