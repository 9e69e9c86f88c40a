// dpac_rollout_nn_x3.h — the fused NN rollout (k_rollout_nn) and the actor's BPTT
// (k_rollout_nn_bwd2) on split-fp16 MFMA, for float actors of the fast-path shape
// (d, c <= 32, hidden layers 193..208 wide: SURVEY §8(f) rank 1, solver.py:92-97, 260-278).
//
// Why.  At lqr_d20's B = 2048 the f32 kernels run 128 workgroups whose per-step chain of
// five dense layers is latency-bound (profiles/r02_nn_phase_trace_fast.json: 30 k cycles per
// forward step, 9.5-10 k of them in each 200x200 layer, 6.7 k of which are the SIMD's
// v_mfma_f32_16x16x4_f32 work).  The split-fp16 product of dpac_mlp_x3.h — operands
// a = hi + lo * 2^-12 as two fp16 numbers, three v_mfma_f32_16x16x32_f16 per 32-k step
// (hi*hi, hi*lo, lo*hi) accumulated in f32 — does the same product in 48 MFMA cycles per
// 32 k instead of 256, at f32 accuracy.
//
// Layout (as dpac_mlp_x3.h): every product is formed transposed, C^T = W^T act^T, with the
// weight image (dpac_mlp.weight_x3 / weight_t_x3) as the A operand (lane l: output feature
// l & 15 of a 16-feature tile, k = 32c + 8 (l >> 4) .. +7) and the LDS activation image as
// B (lane l: trajectory l & 15, the same 8 k), so lane l's accumulator holds the FOUR
// CONSECUTIVE features 4 (l >> 4) .. +3 of trajectory l & 15: one 16-byte z / G store per
// tile and two 8-byte LDS writes of the next operand, no cross-lane exchange.  Activation
// images hold per 32-wide k chunk 32 hi halves then 32 lo halves.
//
// Workgroup: 8 wavefronts, 16 trajectories (one tile of rows), for all N steps.
//  * Every wave takes the feature tiles (wave, wave + 8) of a 13-tile hidden layer (tiles
//    past the layer multiply zeros: the SIMD holding waves 0 and 4 has four real tiles
//    either way, so the uniform pair costs no wall time and keeps one code path).
//  * The narrow-K product (d or c <= 32 inputs: one chunk) and the split-K product into the
//    narrow output (wave w multiplies chunk w for both output tiles) keep their weights in
//    VGPRs for the whole launch; a wide layer's seven chunks are loaded into VGPRs right
//    after the previous wide layer's MFMAs, so their L2 latency hides behind that layer's
//    epilogue and barrier (no ring, every wait a counted vmcnt).
//  * The split-K partials of the narrow output go to LDS and the step lanes sum their own
//    components (fixed wave order) — no reduction phase, no extra barrier.
//  * No stager or writer wavefronts: the step lanes prefetch their next step's inputs into
//    registers and the epilogues store z / G directly; the weight loads of a layer are
//    issued before its predecessor's stores, so the in-order vmcnt never makes them wait
//    on a store.
// The sign-bit mask keeps FwdEpiM's byte layout (dpac.h): the x3 accumulator groups four
// features of one row per lane, the f32 one four rows of one feature, and a 4x4 bit
// transpose inside each lane quad (two DPP ORs) converts between them, so a mask written by
// either forward kernel serves either BPTT kernel.
#pragma once
// Included by dpac_kernels.h inside namespace dpac, after dpac_rollout_nn_bwd.h.

typedef _Float16 nxh8 __attribute__((ext_vector_type(8)));
typedef _Float16 nxh4 __attribute__((ext_vector_type(4)));
typedef float nxf4 __attribute__((ext_vector_type(4)));

#ifndef DPAC_NX_LDPAD
#define DPAC_NX_LDPAD 16  // halves of padding per image row (a multiple of 8: 16-byte rows)
#endif
constexpr int kNxLd = 64 * 8 + DPAC_NX_LDPAD;  // halves per row of a hidden image (K <= 256): 264 dwords = 8 mod 64
constexpr int kNxLd0 = 64 + 8;       // halves per row of the narrow input image (K <= 32): 36 dwords
constexpr int kNxPartLd = 36;        // floats per row of a split-K partial (conflict-free b128 writes)
constexpr int kNxWide = 7;           // 32-k chunks of a 193..224-wide K
#ifndef DPAC_NX_RING
#define DPAC_NX_RING 4               // wide layers: chunks of weights in flight (VGPR budget: 16 per chunk)
#endif
constexpr int kNxRing = DPAC_NX_RING;
#ifndef DPAC_NX_ABLATE
#define DPAC_NX_ABLATE 0  // timing-only builds (bits): 1 = no weight loads (constant weights), 2 = no z / G /
                          // mask stores, 4 = no LDS B-operand reads (constant activations)
#endif
constexpr int kNxBnHalf = DPAC_MLP_MAX_WIDTH;      // shift offset inside a layer's LDS BN image
constexpr int kNxBnLd = 2 * DPAC_MLP_MAX_WIDTH;    // floats per hidden layer: scale | shift
constexpr float kNxLo = 4096.f;      // 2^12
constexpr float kNxLoInv = 1.f / 4096.f;
static_assert(kNnWaves == 8 && kNnRows == 16, "the x3 kernels assume 8 wavefronts over 16 rows");
static_assert(DPAC_MLP_MAX_WIDTH <= 256, "8 chunks per hidden image");

// Dynamic LDS of both kernels (bytes): two hidden images, the narrow input image, the
// split-K partials, the hidden layers' BN constants (forward) and the rows' gradient scales
// (BPTT).
struct NxLds {
  static constexpr uint32_t kImg = kNnRows * kNxLd * 2;                    // 16 896
  static constexpr uint32_t kImg0 = kNnRows * kNxLd0 * 2;                  //  2 304
  static constexpr uint32_t kPart = kNnWaves * kNnRows * kNxPartLd * 4;    // 18 432
  static constexpr uint32_t kBn = DPAC_MLP_MAX_HIDDEN * kNxBnLd * 4;       //  8 192
  static constexpr uint32_t img0 = 0, img1 = kImg, in0 = 2 * kImg, part = in0 + kImg0, bn = part + kPart,
                            rinv = bn + kBn, total = rinv + 64;
};

__device__ __forceinline__ nxf4 nx_mma(nxh8 a, nxh8 b, nxf4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

#ifndef DPAC_NX_FOLD
#define DPAC_NX_FOLD 1  // the narrow product after the last wide layer folded into its epilogue (round 5)
#endif

// four values split into hi / lo halves; true if one of them is outside the split range
// (dpac.h dpac_mlp.status)
__device__ __forceinline__ bool nx_split4(nxf4 v, nxh4& h, nxh4& l) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[e] = (_Float16)v[e];
    l[e] = (_Float16)((v[e] - (float)h[e]) * kNxLo);
  }
  return x3_bad4(v[0], v[1], v[2], v[3]);
}

// Bank-conflict-free hidden images (round 6).  A row holds, per 32-k chunk,
// 32 hi halves then 32 lo halves: eight 16-byte blocks.  The B-operand reads (lane l: row l & 15,
// k block l >> 4, ds_read_b128) were conflict-free at the 264-dword row stride, but the
// epilogue's two 8-byte writes per tile (ds_write_b64: 16 contiguous lanes = the 16 rows at one
// k quad, banks (a/4) mod 32, row stride 8 mod 32) hit 4 distinct bank pairs: 4-way conflicts,
// the bulk of the kernels' measured lds_conflict_frac (0.32 / 0.36).  Now:
//  * the 16-byte blocks of rows 4..7 and 12..15 swap in pairs (block index XOR ((row >> 2) & 1));
//  * a v_permlane16_swap per dword gives the lanes of even 16-lane rows (k quads 0, 2) the hi
//    halves of their quad AND the next quad, and the odd rows the lo halves of both, so each
//    lane stores ONE 16-byte block (ds_write_b128, 8 contiguous lanes per bank cycle).
// Both the reads and the writes are then conflict-free under gfx950's LDS lane grouping
// (MI355X_MICROARCH.md §LDS; checked exhaustively for every tile and chunk offline).
#ifndef DPAC_NX_SWZ
#define DPAC_NX_SWZ 0  // 0: unswizzled images, two 8-byte writes per tile (4-way write conflicts);
                       // 1: swizzled, two 8-byte writes (2-way); 2: swizzled + permlane16 swap, one
                       // 16-byte write (conflict-free)
#endif
__device__ __forceinline__ int nx_swz(int row) { return DPAC_NX_SWZ ? (row >> 2) & 1 : 0; }

// four consecutive features f0..f0+3 (f0 % 4 == 0) of one row, split; the wave's lanes exchange
// halves (above) and each stores one 16-byte block.  ld = kNxLd (the swizzled hidden images).
// True if one of the values is outside the split range (dpac.h dpac_mlp.status).
__device__ __forceinline__ bool nx_put4(_Float16* img, int ld, int row, int f0, nxf4 v, int lane) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  nxh4 h, l;
  const bool bad = nx_split4(v, h, l);
  if constexpr (DPAC_NX_SWZ < 2) {  // two 8-byte writes: hi at block (f0 % 32) / 8, lo 4 blocks on
    const int blk = ((f0 & 31) >> 3) ^ nx_swz(row);  // (a 4-feature quad is half a block)
    _Float16* p = img + row * ld + (f0 >> 5) * 64 + 8 * blk + (f0 & 4);
    *reinterpret_cast<nxh4*>(p) = h;
    *reinterpret_cast<nxh4*>(p + 32) = l;
    return bad;
  }
  u32x2 hw = __builtin_bit_cast(u32x2, h), lw = __builtin_bit_cast(u32x2, l);
  // odd 16-lane rows of hw <-> even rows of lw: even rows keep [h(q) | h(q + 1)], odd rows
  // [l(q - 1) | l(q)]
  const auto s0 = __builtin_amdgcn_permlane16_swap(hw[0], lw[0], false, false);
  const auto s1 = __builtin_amdgcn_permlane16_swap(hw[1], lw[1], false, false);
  const int q = lane >> 4;
  _Float16* p = img + row * ld + (f0 >> 5) * 64 + 32 * (q & 1) + 16 * ((f0 >> 4) & 1) + 8 * ((q >> 1) ^ nx_swz(row));
  *reinterpret_cast<uint4*>(p) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
  return bad;
}

// The narrow product that follows the last 13-tile layer (the forward's output layer, the
// BPTT's gradient into a_0), folded into that layer's epilogue (round 5): wave w already holds,
// for row l & 15, the features 16 w + 4 q + e (its tile w) and 16 (w + 8) + 4 q + e (tile w + 8),
// q = l >> 4, e = 0..3 — exactly the 8 k of a B fragment if the wave's 32-k "chunk" is those 32
// features in that order.  So each wave multiplies its own activations, straight from registers,
// by the matching rows of the weight: A fragments (output column l & 15 of output tile t, the
// same permuted k) gathered once per launch from the fragment-major image W (Nout columns over
// nch 32-k chunks; rows past the layer and missing chunks read 0).  Wave w's partial of output
// tile t goes to the split-K partial slot w: no LDS image of the last layer, no barrier before
// the narrow product.
__device__ __forceinline__ void nx_fold_w(nxh8 (&fh)[2], nxh8 (&fl)[2], const _Float16* W, int Nout, int nch,
                                          int wave, int lane) {
  typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
  const int ntiles = (Nout + 15) / 16;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(W, (uint32_t)(ntiles * nch * 2048));
  const int q = lane >> 4;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
#pragma unroll
    for (int sd = 0; sd < 2; ++sd) {
      const int tile = wave + 8 * sd;              // the 16-feature tile of the layer's k
      const int c = tile >> 1;                     // its 32-k chunk in the image
      const int qq = 2 * (tile & 1) + (q >> 1);    // the image lane group holding k = 16 tile + 4 q ..
      const uint32_t off = (t < ntiles && c < nch)
                               ? (uint32_t)((t * nch + c) * 2048 + (qq * 16 + (lane & 15)) * 16 + 8 * (q & 1))
                               : kOOB;
      const nxh4 h = __builtin_bit_cast(nxh4, __builtin_amdgcn_raw_buffer_load_b64(r, (int)off, 0, 0));
      const nxh4 l = __builtin_bit_cast(nxh4, __builtin_amdgcn_raw_buffer_load_b64(r, (int)(off + 1024u), 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        fh[t][4 * sd + e] = h[e];
        fl[t][4 * sd + e] = l[e];
      }
    }
  }
}

// the folded narrow product of a wave's split activations (bh, bl: the permuted B fragment) into
// its split-K partial slot (kNxPartLd floats per row, output tile t at column 16 t)
__device__ __forceinline__ void nx_fold_prod(const nxh8 (&fh)[2], const nxh8 (&fl)[2], nxh8 bh, nxh8 bl,
                                             float* part, int wave, int lane) {
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    nxf4 a[3] = {nxf4{0.f, 0.f, 0.f, 0.f}, nxf4{0.f, 0.f, 0.f, 0.f}, nxf4{0.f, 0.f, 0.f, 0.f}};
    a[0] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[t], bh, a[0], 0, 0, 0);
    a[1] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fh[t], bl, a[1], 0, 0, 0);
    a[2] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fl[t], bh, a[2], 0, 0, 0);
    *reinterpret_cast<nxf4*>(part + (wave * 16 + (lane & 15)) * kNxPartLd + 16 * t + 4 * (lane >> 4)) =
        a[0] + (a[1] + a[2]) * kNxLoInv;
  }
}

__device__ __forceinline__ bool nx_put1(_Float16* img, int ld, int row, int col, float v) {
  const _Float16 h = (_Float16)v;
  _Float16* p = img + row * ld + (col >> 5) * 64 + (col & 31);
  p[0] = h;
  p[32] = (_Float16)((v - (float)h) * kNxLo);
  return x3_bad(v);
}

// A operands of chunks [c0, c0 + NC) of the feature tiles tA, tB of a fragment-major split-fp16
// image ([tile][chunk][hi|lo][lane][8] halves, Nout features over nch chunks: one contiguous
// KB per wave and load); tiles or chunks that do not exist read 0 (kOOB).
template <int NC>
__device__ __forceinline__ void nx_loadw(nxh8 (&wh)[NC][2], nxh8 (&wl)[NC][2], const _Float16* W, int Nout,
                                         int nch, int c0, int tA, int tB, int lane) {
  const int ntiles = (Nout + 15) / 16;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(W, (uint32_t)(ntiles * nch * 2048));
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tile = j ? tB : tA;
    const bool ok = tile < ntiles;
    const uint32_t base = (uint32_t)(tile * nch * 2048 + 16 * lane);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint32_t o = (ok && c0 + c < nch) ? base + (uint32_t)((c0 + c) * 2048) : kOOB;
#if DPAC_NX_ABLATE & 1
      wh[c][j] = nxh8{(_Float16)(0.01f * c), (_Float16)0.02f, 0, 0, 0, 0, (_Float16)(0.001f * j), 0};
      wl[c][j] = wh[c][j];
      (void)o;
      continue;
#endif
      wh[c][j] = __builtin_bit_cast(nxh8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0));
      wl[c][j] = __builtin_bit_cast(nxh8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(o + 1024u), 0, 0));
    }
  }
}

// acc[j] = the three partial products of chunks [c0, c0 + NC) of the image `in` (row stride
// LD halves) against tile j's A operands: [0] hi*hi, [1] hi*lo, [2] lo*hi (three independent
// accumulation chains).  The B operands come from LDS one chunk ahead.
//   Resident form (RING = 0): wh / wl hold all NC chunks.
//   Ring form (RING = PF > 0): wh / wl hold the first PF chunks; after chunk c's MFMAs the
//   slot is refilled with chunk c + PF of image W (tiles tA, tB; Nout x nch), so PF chunks of
//   weights stay in flight.  The ring is free (and stale) on return.
template <int NC, int LD, int RING, int NS>
__device__ __forceinline__ void nx_prod(const _Float16* in, int c0, nxh8 (&wh)[NS][2], nxh8 (&wl)[NS][2],
                                        nxf4 (&acc)[2][3], int lane, const _Float16* W = nullptr, int Nout = 0,
                                        int nch = 0, int tA = 0, int tB = 0) {
  static_assert(RING ? NS == RING : NS == NC, "resident: one slot per chunk");
  // the hidden images' 16-byte blocks are swizzled by row (nx_swz); the narrow input image is not
  const int kq = LD == kNxLd ? ((lane >> 4) ^ nx_swz(lane & 15)) : (lane >> 4);
  const _Float16* b = in + (lane & 15) * LD + c0 * 64 + 8 * kq;
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int q = 0; q < 3; ++q) acc[j][q] = nxf4{0.f, 0.f, 0.f, 0.f};
  const int ntiles = (Nout + 15) / 16;
  const __amdgpu_buffer_rsrc_t r = make_rsrc(W, RING > 0 ? (uint32_t)(ntiles * nch * 2048) : 0u);
  uint32_t base[2] = {kOOB, kOOB};
  if constexpr (RING > 0) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int tile = j ? tB : tA;
      base[j] = tile < ntiles ? (uint32_t)(tile * nch * 2048 + 16 * lane) : kOOB;
    }
  }
#if DPAC_NX_ABLATE & 4
  nxh8 bh = nxh8{(_Float16)0.5f, 0, 0, (_Float16)(0.25f * c0), 0, 0, 0, 0}, bl = bh;
  (void)b;
#else
  nxh8 bh = *reinterpret_cast<const nxh8*>(b), bl = *reinterpret_cast<const nxh8*>(b + 32);
#endif
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    constexpr int kS = RING > 0 ? RING : NC;
    const int sl = c % kS;
    nxh8 nh = bh, nl = bl;
    if (c + 1 < NC && !(DPAC_NX_ABLATE & 4)) {
      nh = *reinterpret_cast<const nxh8*>(b + (c + 1) * 64);
      nl = *reinterpret_cast<const nxh8*>(b + (c + 1) * 64 + 32);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      acc[j][0] = nx_mma(wh[sl][j], bh, acc[j][0]);
      acc[j][1] = nx_mma(wh[sl][j], bl, acc[j][1]);
      acc[j][2] = nx_mma(wl[sl][j], bh, acc[j][2]);
    }
    if constexpr (RING > 0) {
      if (c + RING < NC && !(DPAC_NX_ABLATE & 1)) {  // refill the slot just used
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const uint32_t o = base[j] + (uint32_t)((c + RING) * 2048);
          wh[sl][j] = __builtin_bit_cast(nxh8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)o, 0, 0));
          wl[sl][j] = __builtin_bit_cast(nxh8, __builtin_amdgcn_raw_buffer_load_b128(r, (int)(o + 1024u), 0, 0));
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // keep the refill where it is issued
    }
    bh = nh;
    bl = nl;
  }
}

__device__ __forceinline__ nxf4 nx_sum(const nxf4 (&a)[3]) { return a[0] + (a[1] + a[2]) * kNxLoInv; }

// Sign bits: this lane's 4-bit nibble (features e of its row) -> the FwdEpiM byte it writes
// (column 4 (l >> 4) + (l & 3) of the tile, rows 4 ((l & 15) >> 2) .. +3 at bits 0..3), and
// back.  Both are a 4x4 bit transpose inside the lane quad.
__device__ __forceinline__ uint32_t nx_quad_gather(uint32_t v, int lane) {
  uint32_t w = v << (4 * (lane & 3));
  w |= (uint32_t)dpp_i32<kDppXor1>((int)w);
  w |= (uint32_t)dpp_i32<kDppXor2>((int)w);
  return w;
}
__device__ __forceinline__ uint32_t nx_pick4(uint32_t w, int i) {  // bits 4k + i, k = 0..3
  return ((w >> i) & 1u) | (((w >> (4 + i)) & 1u) << 1) | (((w >> (8 + i)) & 1u) << 2) |
         (((w >> (12 + i)) & 1u) << 3);
}
__device__ __forceinline__ int nx_mask_idx(int lane) {  // byte of the tile this lane owns
  return 16 * ((lane & 15) >> 2) + 4 * (lane >> 4) + (lane & 3);
}

// Forward epilogue of a hidden layer (pre-BN z of hidden layer h): save z, BN, the sign bit,
// y + relu(y) split into the next image, the mask byte.  bn: LDS [scale | shift] of layer h,
// zero past Nout.  Tiles past the layer are skipped (wave-uniform).  Returns whether a split
// operand left the range.
// FOLD: the last hidden layer: instead of the next image, its activations multiply the folded
// output weights (fh, fl; nx_fold_w) into the wave's split-K partial slot of `part`.
template <bool SAVE, bool MASK, bool FOLD = false>
__device__ __forceinline__ bool nx_fwd_epi(const nxf4 (&acc)[2][3], int wave, int lane, int Nout, const float* bn,
                                           _Float16* out, float* zrow0, int ztot, bool zvec, int rows_live,
                                           uint8_t* mtile, bool mrow, const nxh8 (*fh)[2] = nullptr,
                                           const nxh8 (*fl)[2] = nullptr, float* part = nullptr) {
  const int row = lane & 15;
  bool bad = false;
  nxh8 bh = nxh8{0, 0, 0, 0, 0, 0, 0, 0}, bl = bh;  // FOLD: the wave's permuted B fragment
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tl = wave + 8 * j;
    if (tl * 16 >= Nout) continue;
    const int f0 = tl * 16 + 4 * (lane >> 4);
    const int nv = Nout - f0 < 0 ? 0 : (Nout - f0 > 4 ? 4 : Nout - f0);
    const nxf4 z = nx_sum(acc[j]);
    if (SAVE && row < rows_live && !(DPAC_NX_ABLATE & 2)) {
      float* zp = zrow0 + row * ztot + f0;
      if (nv == 4 && zvec) {
        *reinterpret_cast<nxf4*>(zp) = z;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < nv) zp[e] = z[e];
      }
    }
    const nxf4 s = *reinterpret_cast<const nxf4*>(bn + f0), sh = *reinterpret_cast<const nxf4*>(bn + kNxBnHalf + f0);
    nxf4 y = z * s;
    y = sh + y;  // addcmul(beta, y, gamma/sqrt(1+eps)) (solver.py:266-268), as FwdEpi rounds it
    uint32_t nib = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      nib |= (e < nv && y[e] > 0.f) ? 1u << e : 0u;
      y[e] = e < nv ? y[e] + fmaxf(y[e], 0.f) : 0.f;  // y + relu(y) (solver.py:269)
    }
    if constexpr (FOLD) {
      nxh4 h, l;
      bad |= nx_split4(y, h, l);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bh[4 * j + e] = h[e];
        bl[4 * j + e] = l[e];
      }
    } else {
      bad |= nx_put4(out, kNxLd, row, f0, y, lane);
    }
    if constexpr (MASK && !(DPAC_NX_ABLATE & 2)) {
      const uint32_t w = nx_quad_gather(nib, lane);
      if (mrow) mtile[64 * tl + nx_mask_idx(lane)] = (uint8_t)nx_pick4(w, lane & 3);
    }
  }
  if constexpr (FOLD) nx_fold_prod(*fh, *fl, bh, bl, part, wave, lane);
  return bad;
}

// BPTT epilogue of hidden layer h: the activation factor 1 + [y_h > 0] from the forward's
// mask bytes, G_h = v * 2^(e-1) (the row's scale undone) to global, v split into the next image.
// Returns whether a split operand left the range.
// FOLD: hidden layer 1: instead of the next image, the (scaled) gradient multiplies the folded
// weights of the product into a_0's gradient (fh, fl; nx_fold_w) into the wave's partial slot.
template <bool FOLD = false>
__device__ __forceinline__ bool nx_bwd_epi(const nxf4 (&acc)[2][3], int wave, int lane, int Nout,
                                           const uint32_t (&mb)[2], _Float16* out, float* grow0, int gtot,
                                           bool gvec, int rows_live, float ri, const nxh8 (*fh)[2] = nullptr,
                                           const nxh8 (*fl)[2] = nullptr, float* part = nullptr) {
  const int row = lane & 15, i = lane & 3;
  bool bad = false;
  nxh8 bh = nxh8{0, 0, 0, 0, 0, 0, 0, 0}, bl = bh;  // FOLD: the wave's permuted B fragment
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int tl = wave + 8 * j;
    if (tl * 16 >= Nout) continue;
    const int f0 = tl * 16 + 4 * (lane >> 4);
    const int nv = Nout - f0 < 0 ? 0 : (Nout - f0 > 4 ? 4 : Nout - f0);
    nxf4 v = nx_sum(acc[j]);
    const uint32_t w = nx_quad_gather(mb[j], lane);
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = e < nv ? v[e] * (((w >> (4 * e + i)) & 1u) ? 2.f : 1.f) : 0.f;
    if (row < rows_live && !(DPAC_NX_ABLATE & 2)) {
      const nxf4 gv = v * ri;  // exact: a power of two
      float* gp = grow0 + row * gtot + f0;
      if (nv == 4 && gvec) {
        *reinterpret_cast<nxf4*>(gp) = gv;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (e < nv) gp[e] = gv[e];
      }
    }
    if constexpr (FOLD) {
      nxh4 h, l;
      bad |= nx_split4(v, h, l);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        bh[4 * j + e] = h[e];
        bl[4 * j + e] = l[e];
      }
    } else {
      bad |= nx_put4(out, kNxLd, row, f0, v, lane);
    }
  }
  if constexpr (FOLD) nx_fold_prod(*fh, *fl, bh, bl, part, wave, lane);
  return bad;
}

__device__ __forceinline__ void nx_lds_zero(unsigned char* lds, uint32_t bytes, int tid, int nthreads) {
  uint4* p = reinterpret_cast<uint4*>(lds);
  for (uint32_t e = tid; e < bytes / 16; e += nthreads) p[e] = uint4{0, 0, 0, 0};
}

// Whether the x3 kernels serve a float network (host side, per launch): the actor-shape fast
// path (nn_fast_host) with every split-fp16 image of the direction; DPAC_NN_X3=0 forces the
// f32 kernels (tests compare the two).
inline bool nn_x3_host(int L, const int* width, const void* const* x3, int kin, int kout) {
  const char* e = getenv("DPAC_NN_X3");  // read per launch
  if (e && e[0] == '0') return false;
  if (L < 1 || kin > 32 || kout > 32) return false;
  for (int i = 1; i <= L; ++i)
    if ((width[i] + 15) / 16 != 13 || (width[i] + 31) / 32 != kNxWide) return false;
  for (int i = 0; i <= L; ++i)
    if (!x3[i]) return false;
  return true;
}

// group max over the P lanes of a trajectory (DPP, as Lanes<P>::sum)
template <int P>
__device__ __forceinline__ float nx_group_max(float v) {
  if constexpr (P >= 2) v = fmaxf(v, dpp<kDppXor1>(v));
  if constexpr (P >= 4) v = fmaxf(v, dpp<kDppXor2>(v));
  if constexpr (P >= 8) v = fmaxf(v, dpp<kDppHalfMirror>(v));
  if constexpr (P >= 16) v = fmaxf(v, dpp<kDppMirror>(v));
  static_assert(P <= 16, "lane groups of at most 16");
  return v;
}

// ---------------------------------------------------------------------------
// Forward: k_rollout_nn's step with the MLP on split-fp16 MFMA.
// ---------------------------------------------------------------------------
template <class E, int D, int SCHEME, bool COST, bool SAVE, bool MASK>
__global__ __launch_bounds__(kNnThreads) void k_rollout_nn_x3(const E eq, const DevConsts<float> c,
                                                             const NnMlp<float> mlp,
                                                             const NnRolloutArgs<float> a) {
  using T = float;
  constexpr int P = E::kP, M = E::M, MC = E::MC, CD = E::CDIM;
  using TR = Transition<T, E, SCHEME>;
  extern __shared__ __attribute__((aligned(16))) unsigned char nx_lds[];
  _Float16* const img0 = reinterpret_cast<_Float16*>(nx_lds + NxLds::img0);
  _Float16* const img1 = reinterpret_cast<_Float16*>(nx_lds + NxLds::img1);
  _Float16* const in0 = reinterpret_cast<_Float16*>(nx_lds + NxLds::in0);
  float* const part = reinterpret_cast<float*>(nx_lds + NxLds::part);
  float* const s_bn = reinterpret_cast<float*>(nx_lds + NxLds::bn);
  auto img = [&](int i) { return (i & 1) ? img1 : img0; };
  if (x3_status_set(mlp.status)) return;  // fell back: the f32 kernel after this one does the work
  bool bad = false;                       // a split operand outside the range (dpac.h dpac_mlp.status)
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int tr = a.tr == 8 ? 8 : kNnRows;  // trajectories per workgroup: 16, or 8 (rows 8..15 of the tile stay zero)
  const int64_t row0 = (int64_t)blockIdx.x * tr;
  const int rows_live = (int)((a.B - row0) < tr ? (a.B - row0) : tr);
  const bool stepper = tid < tr * P;
  // sign-bit mask bytes: a byte holds 4 rows of one feature of a 16-row tile (FwdEpiM's layout);
  // an 8-row workgroup at row0 % 16 == 8 owns the tile's row groups 2, 3 (+32 bytes)
  const int moff = (int)(row0 & 15) * 4;
  const bool mrow = (lane & 15) < tr;
  const int g = stepper ? tid / P : 0;
  const LaneCoord<P> lc(a.B, stepper ? tid % P : 0, row0 + g);
  const bool live = stepper && lc.live;
  const Own<D, P> own(lc.p);
  const Own<CD, P> ownu(lc.p);
  const BufSlab<T, D, P> sx(own, lc.b, live);
  const BufSlab<T, CD, P> su(ownu, lc.b, live);
  const uint32_t slab = (uint32_t)(a.B * D * sizeof(T));
  const uint32_t slab_u = (uint32_t)(a.B * CD * sizeof(T));
  const __amdgpu_buffer_rsrc_t rs_x = make_rsrc(a.x, slab * (uint32_t)(a.N + 1));
  const __amdgpu_buffer_rsrc_t rs_dw = make_rsrc(a.dw, slab * (uint32_t)a.N);
  const __amdgpu_buffer_rsrc_t rs_u = make_rsrc(a.u, a.u ? slab_u * (uint32_t)a.N : 0u);
  const int L = mlp.L, c_out = mlp.width[L + 1];
  const int nch_out = (mlp.width[L] + 31) / 32;  // split-K: wave w < nch_out multiplies chunk w
  constexpr bool kFold = DPAC_NX_FOLD != 0;
  const int nparts = kFold ? kNnWaves : nch_out;  // split-K partials the step lanes add
  int zalign = mlp.ztot;  // 16-byte z saves where every hidden block starts 4-aligned
  for (int h = 1; h <= L; ++h) zalign |= mlp.zoff[h];
  const bool zvec = (zalign & 3) == 0;
  const int64_t ntile = (a.B + 15) >> 4;

  nx_lds_zero(nx_lds, NxLds::bn, tid, kNnThreads);
  for (int h = 1; h <= L; ++h)  // BN of the hidden layers, zero past the width
    for (int f = tid; f < DPAC_MLP_MAX_WIDTH; f += kNnThreads) {
      const bool v = f < mlp.width[h];
      s_bn[(h - 1) * kNxBnLd + f] = v ? mlp.scale[h][f] : 0.f;
      s_bn[(h - 1) * kNxBnLd + kNxBnHalf + f] = v ? mlp.shift[h][f] : 0.f;
    }
  // step lanes: BN_0 of the owned state components, the output layer's constants of the
  // owned control components (+ the Eikonal column CD)
  T s0[M], b0[M], oS[MC], oSh[MC], oB[MC];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    const int j = own.j(m);
    s0[m] = own.valid(m) ? mlp.scale[0][j] : T(0);
    b0[m] = own.valid(m) ? mlp.shift[0][j] : T(0);
  }
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    const int j = ownu.j(m);
    oS[m] = ownu.valid(m) ? mlp.scale[L + 1][j] : T(0);
    oSh[m] = ownu.valid(m) ? mlp.shift[L + 1][j] : T(0);
    oB[m] = ownu.valid(m) ? mlp.bias[j] : T(0);
  }
  const T eS = mlp.ekn ? mlp.scale[L + 1][CD] : T(0), eSh = mlp.ekn ? mlp.shift[L + 1][CD] : T(0),
          eB = mlp.ekn ? mlp.bias[CD] : T(0);
  // weights: the narrow products' for the whole launch, the first wide layer's
  nxh8 rih[1][2], ril[1][2], roh[1][2], rol[1][2], wh[kNxRing][2], wl[kNxRing][2];
  nx_loadw<1>(rih, ril, mlp.wx3[0], mlp.width[1], 1, 0, wave, wave + 8, lane);
  if constexpr (kFold)
    nx_fold_w(roh[0], rol[0], mlp.wx3[L], c_out, nch_out, wave, lane);  // the output layer, folded
  else
    nx_loadw<1>(roh, rol, mlp.wx3[L], c_out, nch_out, wave, 0, 1, lane);
  if (L >= 2) nx_loadw<kNxRing>(wh, wl, mlp.wx3[1], mlp.width[2], kNxWide, 0, wave, wave + 8, lane);

  auto write_a0 = [&](const T (&xv)[M]) {  // addcmul(beta0, x, gamma0/sqrt(1+eps)), solver.py:265
    if (stepper) {
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (own.valid(m)) bad |= nx_put1(in0, kNxLd0, g, own.j(m), b0[m] + xv[m] * s0[m]);
    }
  };
  T x[M];
  sx.load(make_rsrc(a.x0, slab), x);
  sx.store(rs_x, x);
  T r = TR::kRadius ? dsqrt(Lanes<P>::sum(sumsq(x))) : T(0);
  Flags fl = SCHEME == DPAC_SCHEME_ADAPTIVE ? region(r, c) : Flags{true, false};
  T disc = 1, y = 0;
  __syncthreads();  // LDS zeroed before the first a0 write
  write_a0(x);

  auto load = [&](int t, DwFrame<T, M>& fr) { sx.load(rs_dw, fr.dw, (uint32_t)t * slab); };
  auto body = [&](int t, DwFrame<T, M>& fr, auto) {
    __syncthreads();  // a0 of step t is in in0; the previous step's partial reads are done
    NN_MARK(t, 0);
    const int64_t rowt = (int64_t)t * a.B + row0;
    uint8_t* mt = MASK ? a.save_mask + ((int64_t)t * ntile + (row0 >> 4)) * a.mb + moff : nullptr;
    {  // hidden layer 1 from a0 (narrow K, resident weights)
      nxf4 acc[2][3];
      nx_prod<1, kNxLd0, 0>(in0, 0, rih, ril, acc, lane);
      if (kFold && L == 1)
        bad |= nx_fwd_epi<SAVE, MASK, kFold>(acc, wave, lane, mlp.width[1], s_bn, img(0),
                                             SAVE ? a.save_z + rowt * mlp.ztot + mlp.zoff[1] : nullptr, mlp.ztot,
                                             zvec, rows_live, mt, mrow, &roh[0], &rol[0], part);
      else
        bad |= nx_fwd_epi<SAVE, MASK>(acc, wave, lane, mlp.width[1], s_bn, img(0),
                                      SAVE ? a.save_z + rowt * mlp.ztot + mlp.zoff[1] : nullptr, mlp.ztot, zvec,
                                      rows_live, mt, mrow);
    }
    NN_MARK(t, 1);
    __syncthreads();
    NN_MARK(t, 2);
    for (int l = 1; l < L; ++l) {  // hidden layer l + 1 (wide)
      nxf4 acc[2][3];
      nx_prod<kNxWide, kNxLd, kNxRing>(img(l - 1), 0, wh, wl, acc, lane, mlp.wx3[l], mlp.width[l + 1], kNxWide,
                                       wave, wave + 8);
#if DPAC_NN_TRACE
      asm volatile("" ::"v"(acc[1][2]));
      NN_MARK(t, 11 + l);  // products done
#endif
      const int ln = l + 1 < L ? l + 1 : 1;  // the next wide layer (this step's or the next one's first)
      nx_loadw<kNxRing>(wh, wl, mlp.wx3[ln], mlp.width[ln + 1], kNxWide, 0, wave, wave + 8, lane);
      if (kFold && l + 1 == L)  // the last hidden layer: the output layer in its epilogue
        bad |= nx_fwd_epi<SAVE, MASK, kFold>(acc, wave, lane, mlp.width[l + 1], s_bn + l * kNxBnLd, img(l),
                                             SAVE ? a.save_z + rowt * mlp.ztot + mlp.zoff[l + 1] : nullptr,
                                             mlp.ztot, zvec, rows_live, MASK ? mt + 13 * 64 * l : nullptr, mrow,
                                             &roh[0], &rol[0], part);
      else
        bad |= nx_fwd_epi<SAVE, MASK>(acc, wave, lane, mlp.width[l + 1], s_bn + l * kNxBnLd, img(l),
                                      SAVE ? a.save_z + rowt * mlp.ztot + mlp.zoff[l + 1] : nullptr, mlp.ztot,
                                      zvec, rows_live, MASK ? mt + 13 * 64 * l : nullptr, mrow);
      NN_MARK(t, 1 + 2 * l);
      __syncthreads();
      NN_MARK(t, 2 + 2 * l);
    }
    if (!kFold) {
      if (wave < nch_out) {  // output layer: chunk `wave` of hidden layer L for both output tiles
        nxf4 acc[2][3];
        nx_prod<1, kNxLd, 0>(img(L - 1), wave, roh, rol, acc, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<nxf4*>(part + (wave * 16 + (lane & 15)) * kNxPartLd + 16 * j + 4 * (lane >> 4)) =
              nx_sum(acc[j]);
      }
      NN_MARK(t, 1 + 2 * L);
      __syncthreads();
      NN_MARK(t, 2 + 2 * L);
    }
    if (!stepper) return;
    // ---- u_t from the partials (fixed wave order), then the transition (step lanes) ----
    const float* pr = part + g * kNxPartLd;
    float* zrow = SAVE ? a.save_z + ((int64_t)t * a.B + lc.b) * mlp.ztot + mlp.zoff[L + 1] : nullptr;
    T u[MC];
#pragma unroll
    for (int m = 0; m < MC; ++m) {
      const int j = ownu.valid(m) ? ownu.j(m) : 0;
      T z = pr[j];
      for (int w = 1; w < nparts; ++w) z += pr[w * 16 * kNxPartLd + j];
      if (SAVE && live && ownu.valid(m)) zrow[j] = z;
      T yv = z + oB[m];     // addmm(b, y, W) (solver.py:270)
      yv = yv * oS[m];
      u[m] = ownu.valid(m) ? oSh[m] + yv : T(0);  // BN_last (solver.py:271)
    }
    if (mlp.ekn) {  // y[:, :d] / (1e-15 + relu(y[:, d]) + |y[:, :d]|) (solver.py:272-274)
      T zc = pr[CD];
      for (int w = 1; w < nparts; ++w) zc += pr[w * 16 * kNxPartLd + CD];
      if (SAVE && live && lc.p == 0) zrow[CD] = zc;
      T yc = zc + eB;
      yc = eSh + yc * eS;
      const T nrm = dsqrt(Lanes<P>::sum(sumsq(u)));
      const T den = (T(1e-15) + fmax(yc, T(0))) + nrm;
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
    disc = disc * disc_factor(tr.dt, cf, c);
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
  pipelined<1, DwFrame<T, M>>(0, a.N, load, body);
  if constexpr (COST) {
    if (live && lc.p == 0) {
      a.y[lc.b] = y;
      a.disc[lc.b] = disc;
    }
  }
  if (bad) x3_flag(mlp.status);
}

// ---------------------------------------------------------------------------
// BPTT: k_rollout_nn_bwd2's reverse loop with the input-gradient chain on split-fp16 MFMA.
// The gradient entering the network output is scaled per trajectory by a power of two (max
// |component| in [1, 2)) before it is split (the fp16 parts of O(1/B) gradients would lose
// bits to subnormals); the chain carries the scale and every stored G is unscaled exactly.
// Needs the forward's sign-bit mask.
// ---------------------------------------------------------------------------
template <class E, int D, int SCHEME>
__global__ __launch_bounds__(kNnThreads) void k_rollout_nn_bwd_x3(const E eq, const DevConsts<float> c,
                                                                 const NnMlp<float> mlp,
                                                                 const NnBackArgs<float> a) {
  using T = float;
  constexpr int P = E::kP, M = E::M, MC = E::MC, CD = E::CDIM;
  extern __shared__ __attribute__((aligned(16))) unsigned char nx_lds[];
  _Float16* const img0 = reinterpret_cast<_Float16*>(nx_lds + NxLds::img0);
  _Float16* const img1 = reinterpret_cast<_Float16*>(nx_lds + NxLds::img1);
  _Float16* const in0 = reinterpret_cast<_Float16*>(nx_lds + NxLds::in0);
  float* const part = reinterpret_cast<float*>(nx_lds + NxLds::part);
  float* const s_rinv = reinterpret_cast<float*>(nx_lds + NxLds::rinv);
  auto img = [&](int i) { return (i & 1) ? img1 : img0; };
  if (x3_status_set(mlp.status)) return;  // fell back: the f32 kernel after this one does the work
  bool bad = false;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
  const int tr = a.tr == 8 ? 8 : kNnRows;  // trajectories per workgroup: 16, or 8 (rows 8..15 of the tile stay zero)
  const int64_t row0 = (int64_t)blockIdx.x * tr;
  const int rows_live = (int)((a.B - row0) < tr ? (a.B - row0) : tr);
  const bool stepper = tid < tr * P;
  // sign-bit mask bytes: a byte holds 4 rows of one feature of a 16-row tile (FwdEpiM's layout);
  // an 8-row workgroup at row0 % 16 == 8 owns the tile's row groups 2, 3 (+32 bytes)
  const int moff = (int)(row0 & 15) * 4;
  const bool mrow = (lane & 15) < tr;
  const int g = stepper ? tid / P : 0;
  const LaneCoord<P> lc(a.B, stepper ? tid % P : 0, row0 + g);
  const bool live = stepper && lc.live;
  const Own<D, P> own(lc.p);
  const Own<CD, P> ownu(lc.p);
  const int L = mlp.L;
  const int nch0 = (mlp.width[1] + 31) / 32;  // split-K of the product into a_0's gradient
  constexpr bool kFold = DPAC_NX_FOLD != 0;
  const int nparts = kFold ? kNnWaves : nch0;  // split-K partials the step lanes add
  int galign = a.gtot;  // 16-byte G stores where every hidden block starts 4-aligned
  for (int h = 1; h <= L; ++h) galign |= a.goff[h];
  const bool gvec = (galign & 3) == 0;
  const int64_t ntile = (a.B + 15) >> 4;

  nx_lds_zero(nx_lds, NxLds::total, tid, kNnThreads);
  T s0[M], lam[M], gxd[M];
#pragma unroll
  for (int m = 0; m < M; ++m) {
    s0[m] = own.valid(m) ? mlp.scale[0][own.j(m)] : T(0);
    lam[m] = T(0);
    gxd[m] = T(0);
  }
  // the Eikonal head's constants of the owned components (+ column CD)
  T oS[MC], oSh[MC], oB[MC];
#pragma unroll
  for (int m = 0; m < MC; ++m) {
    const int j = ownu.j(m);
    const bool v = mlp.ekn && ownu.valid(m);
    oS[m] = v ? mlp.scale[L + 1][j] : T(0);
    oSh[m] = v ? mlp.shift[L + 1][j] : T(0);
    oB[m] = v ? mlp.bias[j] : T(0);
  }
  const T eS = mlp.ekn ? mlp.scale[L + 1][CD] : T(0), eSh = mlp.ekn ? mlp.shift[L + 1][CD] : T(0),
          eB = mlp.ekn ? mlp.bias[CD] : T(0);
  // weights of the transposed chain (weight_t_x3[i]: [width[i]][ceil(width[i+1] / 32)][64])
  nxh8 rih[1][2], ril[1][2], roh[1][2], rol[1][2], wh[kNxRing][2], wl[kNxRing][2];
  nx_loadw<1>(rih, ril, a.wtx3[L], mlp.width[L], 1, 0, wave, wave + 8, lane);
  if constexpr (kFold)
    nx_fold_w(roh[0], rol[0], a.wtx3[0], mlp.width[0], nch0, wave, lane);  // a_0's gradient, folded
  else
    nx_loadw<1>(roh, rol, a.wtx3[0], mlp.width[0], nch0, wave, 0, 1, lane);
  if (L >= 2) nx_loadw<kNxRing>(wh, wl, a.wtx3[L - 1], mlp.width[L - 1], kNxWide, 0, wave, wave + 8, lane);
  if (a.g_xN && stepper) own.load_masked(a.g_xN + lc.b * D, lam);
  T gD = (a.g_disc && stepper) ? a.g_disc[lc.b] : T(0);
  const T gy = (a.g_y && stepper) ? a.g_y[lc.b] : T(0);
  // step inputs and mask bytes, one step ahead in registers
  T px[M] = {}, pdw[M] = {}, pu[MC] = {}, pdisc = 0;
  int pflag = 0;
  uint32_t pmb[DPAC_MLP_MAX_HIDDEN][2];
  auto fetch = [&](int ts) {
    const int64_t rt = (int64_t)ts * a.B;
    if (stepper) {
      own.load_masked(a.x + (rt + lc.b) * D, px);
      own.load_masked(a.dw + (rt + lc.b) * D, pdw);
      ownu.load_masked(a.u + (rt + lc.b) * CD, pu);
      pflag = a.flag[rt + lc.b];
      pdisc = a.disc_t[rt + lc.b];
    }
    const uint8_t* mt = a.mask + ((int64_t)ts * ntile + (row0 >> 4)) * a.mb + moff + nx_mask_idx(lane);
#pragma unroll
    for (int h = 0; h < DPAC_MLP_MAX_HIDDEN; ++h)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        pmb[h][j] = (mrow && h < L && wave + 8 * j < 13) ? (uint32_t)mt[13 * 64 * h + 64 * (wave + 8 * j)] : 0u;
  };
  fetch(a.N - 1);
  __syncthreads();  // LDS zeroed
  for (int t = a.N - 1; t >= 0; --t) {
    NN_MARK(t, 0);
    const int64_t rowt = (int64_t)t * a.B;
    T x[M], u[MC], dwv[M];
#pragma unroll
    for (int m = 0; m < M; ++m) {
      x[m] = px[m];
      dwv[m] = pdw[m];
    }
#pragma unroll
    for (int m = 0; m < MC; ++m) u[m] = pu[m];
    const int cflag = pflag;
    const T dsc = pdisc;
    uint32_t mb[DPAC_MLP_MAX_HIDDEN][2];
#pragma unroll
    for (int h = 0; h < DPAC_MLP_MAX_HIDDEN; ++h) {
      mb[h][0] = pmb[h][0];
      mb[h][1] = pmb[h][1];
    }
    fetch(t > 0 ? t - 1 : 0);  // lands while step t computes (t = 0: an unused re-read)
    if (stepper) {
      T gu[MC], gdn;
      step_vjp<T, E, SCHEME>(eq, c, x, u, dwv, Flags::decode(cflag), dsc, lam, gD, gy, gxd, gu, gdn);
      gD = gdn;
      T goc = 0;
      if (mlp.ekn) {  // gradient at the network output, through the Eikonal head (solver.py:272-274)
        const T* zr = a.z + (rowt + lc.b) * mlp.ztot + mlp.zoff[L + 1];
        T o[MC];
#pragma unroll
        for (int m = 0; m < MC; ++m) {
          const int j = ownu.j(m);
          T ov = ownu.valid(m) ? zr[j] : T(0);
          ov = ov + oB[m];
          o[m] = ownu.valid(m) ? oSh[m] + ov * oS[m] : T(0);
        }
        T oc = zr[CD] + eB;
        oc = eSh + oc * eS;
        const T nrm = dsqrt(Lanes<P>::sum(sumsq(o)));
        const T den = (T(1e-15) + fmax(oc, T(0))) + nrm;
        T dot = 0;
#pragma unroll
        for (int m = 0; m < MC; ++m) dot += gu[m] * o[m];
        const T k = Lanes<P>::sum(dot) / (den * den);
#pragma unroll
        for (int m = 0; m < MC; ++m) gu[m] = gu[m] / den - (k / nrm) * o[m];
        goc = oc > T(0) ? -k : T(0);
      }
      // the row's power-of-two scale: max |gradient| in [1, 2)
      T mx = T(0);
#pragma unroll
      for (int m = 0; m < MC; ++m) mx = ownu.valid(m) ? fmaxf(mx, fabsf(gu[m])) : mx;
      if (mlp.ekn && lc.p == 0) mx = fmaxf(mx, fabsf(goc));
      mx = nx_group_max<P>(mx);
      int ex = 0;
      if (mx > 0.f && mx < 3.0e38f) (void)frexpf(mx, &ex);
      const T sc = ldexpf(1.f, 1 - ex);
      T* grow = a.G + (rowt + lc.b) * a.gtot + a.goff[L + 1];
#pragma unroll
      for (int m = 0; m < MC; ++m)
        if (ownu.valid(m)) {
          bad |= nx_put1(in0, kNxLd0, g, ownu.j(m), gu[m] * sc);
          if (live) grow[ownu.j(m)] = gu[m];
        }
      if (mlp.ekn && lc.p == 0) {
        bad |= nx_put1(in0, kNxLd0, g, CD, goc * sc);
        if (live) grow[CD] = goc;
      }
      if (lc.p == 0) s_rinv[g] = ldexpf(1.f, ex - 1);
    }
    NN_MARK(t, 1);
    __syncthreads();
    NN_MARK(t, 2);
    const float ri = s_rinv[lane & 15];
    {  // hidden layer L from the output's gradient (narrow K, resident weights)
      nxf4 acc[2][3];
      nx_prod<1, kNxLd0, 0>(in0, 0, rih, ril, acc, lane);
      if (kFold && L == 1)
        bad |= nx_bwd_epi<kFold>(acc, wave, lane, mlp.width[L], mb[L - 1], img(0),
                                 a.G + (rowt + row0) * a.gtot + a.goff[L], a.gtot, gvec, rows_live, ri, &roh[0],
                                 &rol[0], part);
      else
        bad |= nx_bwd_epi(acc, wave, lane, mlp.width[L], mb[L - 1], img(0), a.G + (rowt + row0) * a.gtot + a.goff[L],
                          a.gtot, gvec, rows_live, ri);
    }
    NN_MARK(t, 3);
    __syncthreads();
    NN_MARK(t, 4);
    for (int l = L - 1; l >= 1; --l) {  // hidden layer l (wide)
      nxf4 acc[2][3];
      nx_prod<kNxWide, kNxLd, kNxRing>(img(L - 1 - l), 0, wh, wl, acc, lane, a.wtx3[l], mlp.width[l], kNxWide,
                                       wave, wave + 8);
#if DPAC_NN_TRACE
      asm volatile("" ::"v"(acc[1][2]));
      NN_MARK(t, 11 + l);  // products done
#endif
      const int ln = l - 1 >= 1 ? l - 1 : L - 1;  // the next wide layer (this step's or the next one's first)
      nx_loadw<kNxRing>(wh, wl, a.wtx3[ln], mlp.width[ln], kNxWide, 0, wave, wave + 8, lane);
      if (kFold && l == 1)  // hidden layer 1: the product into a_0's gradient in its epilogue
        bad |= nx_bwd_epi<kFold>(acc, wave, lane, mlp.width[l], mb[l - 1], img(L - l),
                                 a.G + (rowt + row0) * a.gtot + a.goff[l], a.gtot, gvec, rows_live, ri, &roh[0],
                                 &rol[0], part);
      else
        bad |= nx_bwd_epi(acc, wave, lane, mlp.width[l], mb[l - 1], img(L - l),
                          a.G + (rowt + row0) * a.gtot + a.goff[l], a.gtot, gvec, rows_live, ri);
      NN_MARK(t, 3 + 2 * (L - l));
      __syncthreads();
      NN_MARK(t, 4 + 2 * (L - l));
    }
    if (!kFold) {
      if (wave < nch0) {  // dL/d a_0: chunk `wave` of hidden layer 1's gradient for both tiles
        nxf4 acc[2][3];
        nx_prod<1, kNxLd, 0>(img(L - 1), wave, roh, rol, acc, lane);
#pragma unroll
        for (int j = 0; j < 2; ++j)
          *reinterpret_cast<nxf4*>(part + (wave * 16 + (lane & 15)) * kNxPartLd + 16 * j + 4 * (lane >> 4)) =
              nx_sum(acc[j]);
      }
      NN_MARK(t, 3 + 2 * L);
      __syncthreads();
      NN_MARK(t, 4 + 2 * L);
    }
    if (stepper) {  // G_0 and dL/dx_t = direct part + G_0 * s_0 (a_0 = beta_0 + x * s_0)
      const float* pr = part + g * kNxPartLd;
      const T rg = s_rinv[g];
      T* g0 = a.G + (rowt + lc.b) * a.gtot + a.goff[0];
#pragma unroll
      for (int m = 0; m < M; ++m) {
        const int j = own.valid(m) ? own.j(m) : 0;
        T v = pr[j];
        for (int w = 1; w < nparts; ++w) v += pr[w * 16 * kNxPartLd + j];
        v = v * rg;
        if (live && own.valid(m)) g0[j] = v;
        lam[m] = gxd[m] + (own.valid(m) ? v * s0[m] : T(0));
      }
    }
    NN_MARK(t, 13);
  }
  if (a.g_x0 && live) own.store(a.g_x0 + lc.b * D, lam);
  if (bad) x3_flag(mlp.status);
}
