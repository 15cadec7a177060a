// K2 of libptzba for gfx950: the reduced camera system of the Schur complement (SURVEY §8a row a4,
// the exact replacement of scipy's dense trf solve at bundle_adjustment.py:200-202).
// Compiled without SLP vectorisation: packing the per-lane FMA chains into v_pk_* operations with
// register shuffles serialises them (dependent pk_mul -> pk_fma -> pk_add chains with s_nop hazards).
#include <cstdlib>
#include <string>

#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

// ------------------------------------------------------------------------------------------------
// K2: reduced camera system  S = U - sum_l W_l V~_l^-1 W_l^T   (damping added after the exchange),
//                            b = -g_pose + sum_l W_l V~_l^-1 g_l
// Two launches:
//   k_schur        the coupling blocks, register-blocked with LDS-staged operands (below); chunk-0
//                  items also sum the diagonal terms (U, g_pose, W V~^-1 g) of their frames;
//   k_schur_reduce sums the split partials of each tile, adds U on the diagonal, writes S (lower
//                  triangle, system order) and b | g_pose | diag U.
// k_schur work item = (tile: block F1 of 32 consecutive free frames x chunk of 64 partner frames,
// split of the tile's landmark list).  Lane = partner frame f2; wave w owns the 4 frames f1 = f1b+4w..
// of F1, so a lane accumulates the four 3x3 blocks S_{f1,f2} in registers (no atomics, no scatter).
// W lives in the dense landmark x frame slot table (slot = toff_l + f - first_l, written by K1; slots
// of frames that do not see the landmark stay zero).  Per batch of SNB landmarks the workgroup stages
// in LDS, double-buffered with the next batch's loads in flight during the current batch's FMAs:
//   * the landmarks' W rows over the chunk's 64 frames (coalesced: consecutive slots) -- loaded once
//     and read by all 8 waves (32 frames of reuse per load);
//   * Y = W_{f1,l} V~_l^-1 for every (landmark, f1 in F1) pair (zero where f1 does not see l), so the
//     batch's FMAs run straight-line without branches.
// Products are accumulated in the record precision per batch and flushed to fp64 registers; each
// split writes its fp64 blocks to a partial buffer [item][32 f1][9][64 f2] (coalesced), reduced by
// k_schur_reduce in a fixed order (deterministic).
// ------------------------------------------------------------------------------------------------
#ifndef S2_DU
#define S2_DU 4  // diagonal-term loads in flight per thread (chunk-0 items)
#endif
constexpr int SF = SCHUR_F1;   // frames per F1 block
constexpr int SFW = SF / 8;    // f1 frames per wave (8 waves)

// Bijection block -> item that gives each XCD group (b mod 8) a contiguous run of items.
__device__ __forceinline__ int xcd_swizzle(int b, int nb) {
  const int c = b & 7, idx = b >> 3;
  int start = 0;
  for (int q = 0; q < c; ++q) start += (nb - q + 7) >> 3;
  return start + idx;
}

// chunk-0 items: diagonal terms of the F1 frames over this split's landmarks: U, g_pose and W V~^-1 g,
// read from the dense slots (thread = (landmark j0 + 16 k, frame i): consecutive threads, consecutive
// slots), reduced through `red` ([512][12] doubles of LDS that is free until staging) into part_diag.
template <typename real>
__device__ __forceinline__ void schur_diag_terms(const SchurArgs& a, const int4* sL, int nl, int f1b, int item,
                                                 bool alt, double* red) {
  const int t = threadIdx.x;
  const real* __restrict__ w_slot = (const real*)(alt ? a.w_slot1 : a.w_slot);
  const real* __restrict__ ug_slot = (const real*)(alt ? a.ug_slot1 : a.ug_slot);
  const int i = t & (SF - 1), f = f1b + i;
  double acc[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) acc[k] = 0;
  // DU landmarks per thread and step, all loads issued before any is consumed (clamped, branch-free)
  constexpr int DU = S2_DU, JS = 512 / SF;
  for (int j0 = t >> 5; j0 < nl; j0 += DU * JS) {
    real u[DU][9], w[DU][6];
    double vg[DU][2];
    bool in[DU];
#pragma unroll
    for (int d = 0; d < DU; ++d) {
      const int j = j0 + d * JS;
      const int4 m = sL[min(j, nl - 1)];
      in[d] = j < nl && f >= m.y && f <= m.z;
      const int64_t slot = m.w + min(max(f - m.y, 0), m.z - m.y);
      slot_load6(w[d], w_slot + slot * W_STRIDE);
      slot_load9(u[d], ug_slot + slot * UG_STRIDE);
      const double* vi = a.lm_aux + (int64_t)m.x * 8;
      vg[d][0] = vi[3];
      vg[d][1] = vi[4];
    }
#pragma unroll
    for (int d = 0; d < DU; ++d) {
      if (in[d]) {
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[k] += (double)u[d][k];
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[9 + q] += (double)w[d][2 * q] * vg[d][0] + (double)w[d][2 * q + 1] * vg[d][1];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) red[t * 12 + k] = acc[k];
  __syncthreads();
  if (t < SF * 12) {
    double v = 0;
    for (int j0 = 0; j0 < 512 / SF; ++j0) v += red[j0 * SF * 12 + t];
    a.part_diag[(int64_t)item * SF * 12 + t] = v;
  }
  __syncthreads();
}

#ifdef SK_TIMING
__device__ long long g_sk[16][16];
__device__ long long g_sk_items[4096][4];  // per item: start, end (s_memrealtime, 100 MHz), chunk, nl
#define SK_T(k) do { if (skrec) sk[k] = clock64(); } while (0)
#define SK_ACC(k, t0) do { if (skrec) sk[k] += clock64() - (t0); } while (0)
#define SK_NOW(t0) do { if (skrec) t0 = clock64(); } while (0)
#else
#define SK_T(k) do { } while (0)
#define SK_ACC(k, t0) do { } while (0)
#define SK_NOW(t0) do { } while (0)
#endif
template <typename real>
__global__ __launch_bounds__(512) void k_schur(SchurArgs a) {
  // fp64 (parity path) stages half as many landmarks per batch to stay inside 160 KiB of LDS
  constexpr int SNB = sizeof(real) == 4 ? 16 : 8;
  constexpr int WP = sizeof(real) == 4 ? 8 : 6;  // 16-B aligned row pitch for 6 values
  __shared__ real sW[2][SNB][6][WAVE];                             // W rows of the chunk's frames (SoA)
  // Y of (landmark, f1), 0 if unobserved.  fp32: frames (2p, 2p+1) interleaved per component, so one
  // 8-byte read gives the pair's value for the packed FMAs; fp64: one row of 6 per frame.
  __shared__ __attribute__((aligned(16))) real sY[2][SNB][SF][WP];
  __shared__ int4 sL[SCHUR_LMAX];                                    // the item's landmark list
  if (a.skip_if && *a.skip_if) return;
#ifdef SK_TIMING
  const bool skrec = threadIdx.x == 0 && blockIdx.x < 16;
  long long* sk = g_sk[blockIdx.x & 15];
  if (skrec)
    for (int k = 0; k < 16; ++k) sk[k] = 0;
#endif
  long long skt = 0;
  (void)skt;
  SK_T(0);
  const int item = xcd_swizzle(blockIdx.x, gridDim.x);
  const int4 it = a.items[item];
#ifdef SK_TIMING
  if (threadIdx.x == 0 && item < 4096) {
    g_sk_items[item][0] = __builtin_amdgcn_s_memrealtime();
    g_sk_items[item][2] = it.y;
    g_sk_items[item][3] = it.w - it.z;
  }
#endif
  const int f1b = it.x, chunk = it.y, lb = it.z, nl = it.w - it.z;
  const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const int f2base = f1b + WAVE * chunk;
  const bool alt = a.sel && *a.sel;  // device-chosen linearisation slot
  const real* __restrict__ w_slot = (const real*)(alt ? a.w_slot1 : a.w_slot);
  for (int k = t; k < nl; k += 512) sL[k] = a.item_lm[lb + k];
  __syncthreads();
  SK_T(1);

  if (chunk == 0) schur_diag_terms<real>(a, sL, nl, f1b, item, alt, reinterpret_cast<double*>(&sW[0][0][0][0]));
  SK_T(2);

  // ---- staging registers: W slots (e = t, t + 512 over [SNB][64]) and one Y pair (j = t / SF, i = t % SF;
  // fp64: threads >= SNB*SF repeat a pair and do not stage it).  Branch-free, so the loads stay in flight
  // until stage() consumes them after the current batch's FMAs.
  constexpr int NSL = SNB * WAVE / 512;  // W slots per thread per batch (2 fp32, 1 fp64)
  real rw[NSL][6];
  bool rwin[NSL];
  real ryw[6];
  double rvi[3];
  bool ryin;
  const int yj = (t / SF) & (SNB - 1), yi = t & (SF - 1);
  auto fetch = [&](int p) {  // landmarks [p, p + SNB) of the list
#pragma unroll
    for (int q = 0; q < NSL; ++q) {
      const int e = t + 512 * q, j = e >> 6, ln = e & 63;
      const int4 m = sL[min(p + j, nl - 1)];  // {landmark, first frame, last frame, slot offset}
      const int idx = f2base + ln - m.y;
      rwin[q] = (p + j < nl) && idx >= 0 && f2base + ln <= m.z;
      slot_load6(rw[q], w_slot + (int64_t)(m.w + min(max(idx, 0), m.z - m.y)) * W_STRIDE);
    }
    const int f = f1b + yi;
    const int4 m = sL[min(p + yj, nl - 1)];
    ryin = (p + yj < nl) && f >= m.y && f <= m.z;
    slot_load6(ryw, w_slot + (int64_t)(m.w + min(max(f - m.y, 0), m.z - m.y)) * W_STRIDE);
    const double* vi = a.lm_aux + (int64_t)m.x * 8;
    rvi[0] = vi[0]; rvi[1] = vi[1]; rvi[2] = vi[2];
  };
  auto stage = [&](int buf) {
#pragma unroll
    for (int q = 0; q < NSL; ++q) {
      const int e = t + 512 * q, j = e >> 6, ln = e & 63;
      if constexpr (sizeof(real) == 4) {
        // fp32: W as component pairs (w_2r, w_2r+1) per lane, so the packed FMAs take one half of a
        // loaded pair for both result halves (op_sel) instead of building splat pairs with moves
        float2* w2p = reinterpret_cast<float2*>(&sW[0][0][0][0]) + ((buf * SNB + j) * 3) * WAVE + ln;
#pragma unroll
        for (int r = 0; r < 3; ++r)
          w2p[r * WAVE] = rwin[q] ? make_float2(rw[q][2 * r], rw[q][2 * r + 1]) : make_float2(0.f, 0.f);
      } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) sW[buf][j][k][ln] = rwin[q] ? rw[q][k] : (real)0;
      }
    }
    if (t < SNB * SF) {
      // pair layout (fp32): element (frame 2p + h, component k) at [2p][0] + 2 k + h of the pair's 16 reals
      real* y = sizeof(real) == 4 ? &sY[buf][yj][yi & ~1][0] + (yi & 1) : sY[buf][yj][yi];
      const int ks = sizeof(real) == 4 ? 2 : 1;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double W0 = ryin ? (double)ryw[2 * q] : 0.0, W1 = ryin ? (double)ryw[2 * q + 1] : 0.0;
        y[ks * (2 * q)] = (real)-(W0 * rvi[0] + W1 * rvi[1]);  // staged negated: the FMAs accumulate -Y W^T
        y[ks * (2 * q + 1)] = (real)-(W0 * rvi[1] + W1 * rvi[2]);
      }
    }
  };

  double acc[SFW][9];
#pragma unroll
  for (int i = 0; i < SFW; ++i)
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[i][k] = 0;

  if (nl > 0) {
    fetch(0);
    stage(0);
  }
  __syncthreads();
  SK_T(3);
#ifdef SK_TIMING
  if (skrec) {
    sk[8] = nl;
    sk[9] = chunk;
  }
#endif
  int buf = 0;
  for (int p = 0; p < nl; p += SNB) {
    const bool more = p + SNB < nl;  // block-uniform
    fetch(p + SNB);  // next batch's loads in flight during this batch's FMAs (unconditional: no phi
                     // at a join forces an early wait; past the list the lanes load clamped slots)
    real accr[SFW][9];
#pragma unroll
    for (int i = 0; i < SFW; ++i)
#pragma unroll
      for (int k = 0; k < 9; ++k) accr[i][k] = 0;
    SK_NOW(skt);
    // straight-line over the whole batch: slots past the list and unobserved (landmark, f1) pairs were
    // staged as zeros, so no branch (and no wait at a branch) interrupts the LDS reads and the FMAs
    if constexpr (sizeof(real) == 4) {
      // packed: one v_pk_fma_f32 updates the same block entry of two frames (2p, 2p+1)
      typedef float f2 __attribute__((ext_vector_type(2)));
      f2 accp[SFW / 2][9];
#pragma unroll
      for (int pp = 0; pp < SFW / 2; ++pp)
#pragma unroll
        for (int k = 0; k < 9; ++k) accp[pp][k] = f2{0.f, 0.f};
#pragma unroll 2
      for (int j = 0; j < SNB; ++j) {
        const f2* wsrc = reinterpret_cast<const f2*>(&sW[0][0][0][0]) + ((buf * SNB + j) * 3) * WAVE + lane;
        f2 wp[3];
#pragma unroll
        for (int r = 0; r < 3; ++r) wp[r] = wsrc[r * WAVE];
#pragma unroll
        for (int pp = 0; pp < SFW / 2; ++pp) {
          const f2* ys = reinterpret_cast<const f2*>(&sY[buf][j][SFW * wv + 2 * pp][0]);
          f2 y[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) y[k] = ys[k];
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              accp[pp][3 * q + r] = __builtin_elementwise_fma(y[2 * q], __builtin_shufflevector(wp[r], wp[r], 0, 0),
                                                              accp[pp][3 * q + r]);
              accp[pp][3 * q + r] = __builtin_elementwise_fma(y[2 * q + 1], __builtin_shufflevector(wp[r], wp[r], 1, 1),
                                                              accp[pp][3 * q + r]);
            }
        }
      }
#pragma unroll
      for (int pp = 0; pp < SFW / 2; ++pp)
#pragma unroll
        for (int k = 0; k < 9; ++k) {
          acc[2 * pp][k] += (double)accp[pp][k].x;
          acc[2 * pp + 1][k] += (double)accp[pp][k].y;
        }
    } else {
#pragma unroll 2
      for (int j = 0; j < SNB; ++j) {
        real w2[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) w2[k] = sW[buf][j][k][lane];
#pragma unroll
        for (int i = 0; i < SFW; ++i) {
          const real* ys = sY[buf][j][SFW * wv + i];
          real y[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) y[k] = ys[k];
#pragma unroll
          for (int q = 0; q < 3; ++q)
#pragma unroll
            for (int r = 0; r < 3; ++r) {
              accr[i][3 * q + r] = fma(y[2 * q], w2[2 * r], accr[i][3 * q + r]);
              accr[i][3 * q + r] = fma(y[2 * q + 1], w2[2 * r + 1], accr[i][3 * q + r]);
            }
        }
      }
#pragma unroll
      for (int i = 0; i < SFW; ++i)
#pragma unroll
        for (int k = 0; k < 9; ++k) acc[i][k] += (double)accr[i][k];
    }
    SK_ACC(4, skt);  // compute
    SK_NOW(skt);
    if (more) stage(buf ^ 1);
    SK_ACC(5, skt);  // stage (waits for the prefetched loads)
    SK_NOW(skt);
    __syncthreads();
    SK_ACC(6, skt);  // barrier
    buf ^= 1;
  }
  SK_T(7);
  // partial blocks of this split: part[item][f1 local][k][f2 lane]
  // split partials in the record precision: half the bytes of fp64 for the fp32 path (each is a sum of
  // fp64-flushed batches, rounded once; the reduce sums them in fp64)
  real* out = (real*)a.part + (int64_t)item * (SF * 9 * WAVE);
#pragma unroll
  for (int i = 0; i < SFW; ++i)
#pragma unroll
    for (int k = 0; k < 9; ++k) out[((SFW * wv + i) * 9 + k) * WAVE + lane] = (real)acc[i][k];
  SK_T(10);
#ifdef SK_TIMING
  __syncthreads();
  if (threadIdx.x == 0 && item < 4096) g_sk_items[item][1] = __builtin_amdgcn_s_memrealtime();
#endif
}
// ------------------------------------------------------------------------------------------------
// K2 on the matrix cores (fp32 path, the default): the same work items, split partials and diagonal
// terms as k_schur; each batch of 16 landmarks is one k-step (K = 16 landmarks x 2 ray dimensions) of
// v_mfma_f32_16x16x32_f16 over the item's 96 x 192 block S(F1 dofs, chunk dofs) -- 72 output blocks of
// 16 x 16, nine per wave (3 row blocks x 3 column blocks).  Zero products (a landmark covers ~19 % of a
// tile) cost matrix-core cycles instead of VALU issue.
// Precision: every operand is split x = hi + lo into two fp16 (22 significant bits) and a product is
// hi*hi + hi*lo + lo*hi (the dropped lo*lo is ~2^-22 of it), accumulated in fp32 over the item's batches
// and stored as the fp32 split partial (the reduce sums the splits in fp64).  Range: W (~1e4 px^2) and Y = -W V~^-1 (~1) would not both fit fp16, so row
// k = (landmark, d) of W is scaled by g_l = 2^round(log2 sqrt(tr V~_l^-1)) and the same row of Y by
// 1 / g_l: the product Y^T W is unchanged (powers of two: exact), both factors ~ sqrt(|W| |Y|).
typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f4v __attribute__((ext_vector_type(4)));
constexpr int MKP = 40;
#ifndef MF_DIAG_FUSED
#define MF_DIAG_FUSED 1  // chunk-0 diagonal terms inside the batch pipeline (0: a phase before it)
#endif
// (k pitch of an operand row in halves: 80-B rows keep the 16-B fragment reads aligned)

// (x0, x1) -> hi + lo, each a packed pair of fp16 (v_cvt_pkrtz: toward zero; x - hi is exact in fp32 and
// has at most 13 significant bits, of which lo keeps 11)
typedef __fp16 hp2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_pk(float x0, float x1, hp2v& h, hp2v& l) {
  h = __builtin_amdgcn_cvt_pkrtz(x0, x1);
  l = __builtin_amdgcn_cvt_pkrtz(x0 - (float)h[0], x1 - (float)h[1]);
}

template <typename real, bool AGENT>
__device__ __forceinline__ void schur_reduce_elem(const SchurArgs& a, const int4 g, int e);
template <bool AGENT>
__device__ __forceinline__ void schur_reduce_vec(const SchurArgs& a, const int4 g, int tid);

__global__ __launch_bounds__(512) void k_schur_mf(SchurArgs a) {
  constexpr int SNB = 16;                // landmarks per batch
  constexpr int NSL = SNB * WAVE / 512;  // W slots staged per thread per batch
  __shared__ __attribute__((aligned(16))) _Float16 sY[2][2][3 * SF][MKP];     // [buf][hi|lo][q*32 + f1][2j + d]
  __shared__ __attribute__((aligned(16))) _Float16 sWt[2][2][3 * WAVE][MKP];  // [buf][hi|lo][r*64 + f2][2j + d]
  __shared__ int4 sL[SCHUR_LMAX];
  __shared__ float sG[SCHUR_LMAX];  // g_l per landmark of the list
  if (a.skip_if && *a.skip_if) return;
#ifdef SK_TIMING
  const bool skrec = threadIdx.x == 0 && blockIdx.x < 16;
  long long* sk = g_sk[blockIdx.x & 15];
  if (skrec)
    for (int k = 0; k < 16; ++k) sk[k] = 0;
#endif
  long long skt = 0;
  (void)skt;
  SK_T(0);
  const int item = xcd_swizzle(blockIdx.x, gridDim.x);
  const int4 it = a.items[item];
#ifdef SK_TIMING
  if (threadIdx.x == 0 && item < 4096) {
    g_sk_items[item][0] = __builtin_amdgcn_s_memrealtime();
    g_sk_items[item][2] = it.y;
    g_sk_items[item][3] = it.w - it.z;
  }
#endif
  const int f1b = it.x, chunk = it.y, lb = it.z, nl = it.w - it.z;
  const int t = threadIdx.x, lane = lane_id(), wv = t >> 6;
  const int f2base = f1b + WAVE * chunk;
  const bool alt = a.sel && *a.sel;  // device-chosen linearisation slot
  const float* __restrict__ w_slot = (const float*)(alt ? a.w_slot1 : a.w_slot);
  for (int k = t; k < nl; k += 512) {
    const int4 m = a.item_lm[lb + k];
    sL[k] = m;
    const double* vi = a.lm_aux + (int64_t)m.x * 8;
    int e = 0;
    (void)frexp(vi[0] + vi[2], &e);
    sG[k] = ldexpf(1.f, e / 2);
  }
  __syncthreads();
  SK_T(1);
#if !MF_DIAG_FUSED
  if (chunk == 0) schur_diag_terms<float>(a, sL, nl, f1b, item, alt, reinterpret_cast<double*>(&sWt[0][0][0][0]));
#endif

  // staging registers of one batch (two sets: the loads of batch p + 2 are issued while batch p is
  // multiplied and batch p + 1 staged, so each load has two batches of MFMA time to arrive)
  struct Pre {
    float rw[NSL][6], rgw[NSL], ryw[6], ryg, rvi[3];
    bool rwin[NSL], ryin;
  };
  const int yj = t / SF, yi = t & (SF - 1);
  auto fetch = [&](Pre& P, int p) {  // landmarks [p, p + SNB) of the list (clamped, branch-free)
#pragma unroll
    for (int q = 0; q < NSL; ++q) {
      const int e = t + 512 * q, j = e >> 6, ln = e & 63;
      const int jj = min(p + j, nl - 1);
      const int4 m = sL[jj];
      const int idx = f2base + ln - m.y;
      P.rwin[q] = (p + j < nl) && idx >= 0 && f2base + ln <= m.z;
      P.rgw[q] = sG[jj];
      slot_load6(P.rw[q], w_slot + (int64_t)(m.w + min(max(idx, 0), m.z - m.y)) * W_STRIDE);
    }
    const int f = f1b + yi, jj = min(p + yj, nl - 1);
    const int4 m = sL[jj];
    P.ryin = (p + yj < nl) && f >= m.y && f <= m.z;
    P.ryg = sG[jj];
    slot_load6(P.ryw, w_slot + (int64_t)(m.w + min(max(f - m.y, 0), m.z - m.y)) * W_STRIDE);
    const double* vi = a.lm_aux + (int64_t)m.x * 8;
    P.rvi[0] = (float)vi[0]; P.rvi[1] = (float)vi[1]; P.rvi[2] = (float)vi[2];
  };
  auto stage = [&](const Pre& P, int buf) {
#pragma unroll
    for (int q = 0; q < NSL; ++q) {
      const int e = t + 512 * q, j = e >> 6, ln = e & 63;
      const float gq = P.rwin[q] ? P.rgw[q] : 0.f;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        hp2v h, l;
        split_pk(P.rw[q][2 * r] * gq, P.rw[q][2 * r + 1] * gq, h, l);
        *reinterpret_cast<hp2v*>(&sWt[buf][0][r * WAVE + ln][2 * j]) = h;
        *reinterpret_cast<hp2v*>(&sWt[buf][1][r * WAVE + ln][2 * j]) = l;
      }
    }
    // Y / g = -(W / g) V~^-1, staged negated: the products accumulate -Y W^T (fp32 is exact enough: the
    // operand keeps 22 bits).  1 / g is a power of two: exact.
    const float gi = P.ryin ? 1.f / P.ryg : 0.f;
    const float v0 = P.rvi[0] * gi, v1 = P.rvi[1] * gi, v2 = P.rvi[2] * gi;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      const float W0 = P.ryw[2 * q], W1 = P.ryw[2 * q + 1];
      hp2v h, l;
      split_pk(-fmaf(W0, v0, W1 * v1), -fmaf(W0, v1, W1 * v2), h, l);
      *reinterpret_cast<hp2v*>(&sY[buf][0][q * SF + yi][2 * yj]) = h;
      *reinterpret_cast<hp2v*>(&sY[buf][1][q * SF + yi][2 * yj]) = l;
    }
  };

  const int rg = wv >> 2, cg = wv & 3;             // row blocks 3rg.., column blocks 3cg..
  const int fr = lane & 15, fk = (lane >> 4) * 8;  // fragment row / column and k offset of this lane
  // the item's products accumulate in fp32 over all its batches (<= 32 of 16 landmarks); the split partial is
  // stored in fp32 anyway, and round 6 measured fp64 flushes every 4 batches (72 more VGPRs: spills, and an early
  // vmcnt(0) in the loop) as no more accurate: max |S32 - S64| / sqrt(S_ii S_jj) 2.87e-7 / 4.24e-7 at configs 2 / 3
  // against 2.90e-7 / 3.93e-7, 3 us faster per build (profiles/r06_k2_ab.json)
  f4v c[3][3];
#pragma unroll
  for (int x = 0; x < 3; ++x)
#pragma unroll
    for (int y = 0; y < 3; ++y) c[x][y] = f4v{0.f, 0.f, 0.f, 0.f};
  auto compute = [&](int buf) {
    h8v bh[3], bl[3];
#pragma unroll
    for (int y = 0; y < 3; ++y) {
      const int col = 16 * (3 * cg + y) + fr;
      bh[y] = *reinterpret_cast<const h8v*>(&sWt[buf][0][col][fk]);
      bl[y] = *reinterpret_cast<const h8v*>(&sWt[buf][1][col][fk]);
    }
#pragma unroll
    for (int x = 0; x < 3; ++x) {
      const int row = 16 * (3 * rg + x) + fr;
      const h8v ah = *reinterpret_cast<const h8v*>(&sY[buf][0][row][fk]);
      const h8v al = *reinterpret_cast<const h8v*>(&sY[buf][1][row][fk]);
#pragma unroll
      for (int y = 0; y < 3; ++y) {
        c[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[y], c[x][y], 0, 0, 0);
        c[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[y], c[x][y], 0, 0, 0);
        c[x][y] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[y], c[x][y], 0, 0, 0);
      }
    }
  };
  SK_T(2);
#if MF_DIAG_FUSED
  // chunk-0 items: the diagonal terms (U, g_pose, W V~^-1 g of the F1 frames; HBM-bound, ~100 MB per
  // build) ride in the batch pipeline instead of a phase of their own: the thread that stages Y of
  // (landmark, f1) also sums that pair's terms, its U|g loads issued one batch ahead, under the MFMAs.
  const bool diag = chunk == 0;
  const float* __restrict__ ug_slot = (const float*)(alt ? a.ug_slot1 : a.ug_slot);
  float du[9];
  double dvg[2];  // converted where they are consumed (daccum): a conversion here would wait for the load at once
  float dacc[12];  // fp32 over the item's <= 32 batches: one term per batch (the reduction below is fp64)
#pragma unroll
  for (int k = 0; k < 12; ++k) dacc[k] = 0.f;
  auto dfetch = [&](int p) {
    const int4 m = sL[min(p + yj, nl - 1)];
    const int64_t slot = m.w + min(max(f1b + yi - m.y, 0), m.z - m.y);
    slot_load9(du, ug_slot + slot * UG_STRIDE);
    const double* vi = a.lm_aux + (int64_t)m.x * 8;
    dvg[0] = vi[3];
    dvg[1] = vi[4];
  };
  auto daccum = [&](const Pre& P) {
    if (P.ryin) {
      const float g0 = (float)dvg[0], g1 = (float)dvg[1];
#pragma unroll
      for (int k = 0; k < 9; ++k) dacc[k] += du[k];
#pragma unroll
      for (int q = 0; q < 3; ++q) dacc[9 + q] += fmaf(P.ryw[2 * q], g0, P.ryw[2 * q + 1] * g1);
    }
  };
#else
  constexpr bool diag = false;
  auto dfetch = [&](int) {};
  auto daccum = [&](const Pre&) {};
#endif
  Pre A, B;
  if (nl > 0) {
    if (diag) dfetch(0);
    fetch(A, 0);
    fetch(B, SNB);
    stage(A, 0);
    if (diag) daccum(A);
  }
  __syncthreads();
  SK_T(3);
#ifdef SK_TIMING
  if (skrec) {
    sk[8] = nl;
    sk[9] = chunk;
  }
#endif
  // batch p in buffer 0 from set A, batch p + SNB in buffer 1 from set B (block-uniform control flow)
  for (int p = 0; p < nl; p += 2 * SNB) {
    SK_NOW(skt);
    if (diag && p + SNB < nl) dfetch(p + SNB);
    fetch(A, p + 2 * SNB);
    compute(0);
    SK_ACC(4, skt);
    SK_NOW(skt);
    if (p + SNB < nl) {
      stage(B, 1);
      if (diag) daccum(B);
    }
    SK_ACC(5, skt);
    SK_NOW(skt);
    __syncthreads();
    SK_ACC(6, skt);
    if (p + SNB >= nl) break;
    SK_NOW(skt);
    if (diag && p + 2 * SNB < nl) dfetch(p + 2 * SNB);
    fetch(B, p + 3 * SNB);
    compute(1);
    SK_ACC(4, skt);
    SK_NOW(skt);
    if (p + 2 * SNB < nl) {
      stage(A, 0);
      if (diag) daccum(A);
    }
    SK_ACC(5, skt);
    SK_NOW(skt);
    __syncthreads();
    SK_ACC(6, skt);
  }
  SK_T(7);
#if MF_DIAG_FUSED
  if (diag) {  // fixed-order reduction over the 16 landmark lanes of each frame (as schur_diag_terms)
    double* red = reinterpret_cast<double*>(&sWt[0][0][0][0]);  // free after the last batch's barrier
#pragma unroll
    for (int k = 0; k < 12; ++k) red[(yj * SF + yi) * 12 + k] = (double)dacc[k];
    __syncthreads();
    if (t < SF * 12) {
      double v = 0;
      for (int j0 = 0; j0 < 512 / SF; ++j0) v += red[j0 * SF * 12 + t];
      a.part_diag[(int64_t)item * SF * 12 + t] = v;
    }
  }
#endif
  // partial blocks of this split: part[item][f1 local][3q + r][f2], as k_schur writes them
  float* out = (float*)a.part + (int64_t)item * (SF * 9 * WAVE);
#pragma unroll
  for (int x = 0; x < 3; ++x)
#pragma unroll
    for (int y = 0; y < 3; ++y)
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int row = 16 * (3 * rg + x) + (lane >> 4) * 4 + v, col = 16 * (3 * cg + y) + fr;
        const int q = row / SF, i = row % SF, r = col / WAVE, f2 = col % WAVE;
        out[(i * 9 + 3 * q + r) * WAVE + f2] = c[x][y][v];
      }
  SK_T(10);
#ifdef SK_TIMING
  __syncthreads();
  if (threadIdx.x == 0 && item < 4096) g_sk_items[item][1] = __builtin_amdgcn_s_memrealtime();
#endif
}


#ifdef SK_TIMING
extern "C" int ptzba_debug_sk(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk), sizeof(g_sk)) == hipSuccess ? 0 : -1;
}
extern "C" int ptzba_debug_sk_items(long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sk_items), sizeof(g_sk_items)) == hipSuccess ? 0 : -1;
}
#endif

// split-partial loads of the tile reduction (AGENT: agent-scope loads; the reduce launch uses plain ones).  Round 3-4
// also reduced each tile in its LAST split (k_schur_mf "folded reduce", counters per tile): 258 us per build with an
// acq_rel counter, not faster with write-through partials; removed in round 5 with the chunk-pair k_schur_mf2 (103 vs
// 70 us per build, r03ab).
template <typename real, bool AGENT>
__device__ __forceinline__ real part_load(const real* p) {
  if constexpr (AGENT) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <typename real, bool AGENT>
__device__ __forceinline__ void schur_reduce_elem(const SchurArgs& a, const int4 g, int e) {
  constexpr int NE = SF * 9 * WAVE;
  const int f1b = g.x, chunk = g.y;
  const int ln = e & 63, ik = e >> 6, i = ik / 9, k = ik - 9 * i, q = k / 3, r = k - 3 * q;
  const int f1 = f1b + i, f2 = f1b + WAVE * chunk + ln;
  // the window bound and both frames' system positions in one round trip (clamped indices: a thread outside the
  // window reads a valid entry and leaves)
  const int f1c = min(f1, a.n_pose - 1), f2c = min(f2, a.n_pose - 1);
  const int whi = a.frame_win_hi[f1c];
  const int64_t col0 = a.frame_pos[f1c], pf2 = a.frame_pos[f2c];
  if (!(f1 < a.n_pose && f2 >= f1 && f2 <= whi)) return;
  const real* p = (const real*)a.part + e;
  double v = 0;
  int it = g.z;
  // up to 8 splits' partials in flight (a tile has ~8 at config 3: one round trip), summed in item order
  for (; it + 8 <= g.w; it += 8) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = part_load<real, AGENT>(p + (int64_t)(it + u) * NE);
#pragma unroll
    for (int u = 0; u < 8; ++u) v += x[u];
  }
  if (it < g.w) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = it + u < g.w ? (double)part_load<real, AGENT>(p + (int64_t)(it + u) * NE) : 0.0;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (it + u < g.w) v += x[u];
  }
  if (f2 == f1) {  // chunk 0: U of the frame, summed over the tile's splits
    const int ui = q <= r ? (q == 0 ? r : (q == 1 ? 2 + r : 5)) : (r == 0 ? q : (r == 1 ? 2 + q : 5));
    double du = 0;  // diag U as the chunk-0 vector block sums it (fresh, item order): the damping's scale
    for (int it2 = g.z; it2 < g.w; ++it2) {
      const double uu = part_load<double, AGENT>(a.part_diag + ((int64_t)it2 * SF + i) * 12 + ui);
      v += uu;
      du += uu;
    }
    if (a.prep.pad && q == r) {  // fused prepare: Marquardt damping of the pose row (k_chol_prepare's rule)
      const double lambda = a.prep.lam_dev ? *a.prep.lam_dev : a.prep.lambda;
      double* D = a.prep.D_pose + 3 * (int64_t)f1 + q;
      const double d = fmax(*D, fmax(du, 1e-12));
      *D = d;
      const int64_t row = col0 + q;
      a.S[row * a.ld + row] = v;
      a.S[row * a.ld + row] += lambda * d;
      return;
    }
  }
  const int64_t ld = a.ld;
  if (pf2 >= col0) a.S[(pf2 + r) * ld + col0 + q] = v;
  else a.S[(col0 + q) * ld + pf2 + r] = v;
}
template <bool AGENT>
__device__ __forceinline__ void schur_reduce_vec(const SchurArgs& a, const int4 g, int tid) {
  const int f1b = g.x;
  const int i2 = tid / 3, q2 = tid - 3 * i2, f = f1b + i2;
  if (f >= a.n_pose) return;
  double d[12];
  for (int k = 0; k < 12; ++k) d[k] = 0;
  for (int it2 = g.z; it2 < g.w; ++it2)
    for (int k = 0; k < 12; ++k) d[k] += part_load<double, AGENT>(a.part_diag + ((int64_t)it2 * SF + i2) * 12 + k);
  const int c0 = a.frame_pos[f];
  const double bv = -d[6 + q2] + d[9 + q2];
  a.b[c0 + q2] = bv;
  a.g_pose[c0 + q2] = d[6 + q2];
  a.dU[c0 + q2] = d[q2 == 0 ? 0 : (q2 == 1 ? 3 : 5)];
  if (a.prep.pad) a.S[a.prep.n_aug * a.ld + c0 + q2] = bv;  // fused prepare: the augmented row b^T
}

// (Four elements per reduce thread with 16-B partial loads, `SR_VEC`, and four independent elements with all their
// partials in flight, measured slower (r03v: 77-78 vs 71 us; r05ac: 93 vs 72 us per build), are gone since round 5.)

// tile reduction: fixed-order sum of the splits, U on the diagonal blocks, write the lower triangle in the
// system order (mirror when f2 precedes f1); chunk-0 tiles also write b | g_pose | diag U of their frames.
// fp32 partials: thread = four elements of a tile (grid: tile x 18 blocks of 256); fp64: one element
// (tile x 72 blocks).
template <typename real>
__global__ __launch_bounds__(256) void k_schur_reduce(SchurArgs a) {
  if (a.skip_if && *a.skip_if) return;
  const int4 g = a.groups[blockIdx.y];  // {f1b, chunk, first item, end item}
  schur_reduce_elem<real, false>(a, g, blockIdx.x * 256 + threadIdx.x);
  if (g.y == 0 && blockIdx.x == 0 && threadIdx.x < SF * 3) schur_reduce_vec<false>(a, g, threadIdx.x);
}

template <typename real>
void launch_schur(const SchurArgs& a, int n_items, int n_groups, int n_fixed, hipStream_t st) {
  const int n_free = a.n_pose - n_fixed;
  if (n_free <= 0) return;
  // fp32: the matrix cores (k_schur_mf, fp16 hi/lo splits); fp64: the VALU kernel
  if (n_items > 0) {
    if (sizeof(real) == 4) hipLaunchKernelGGL(k_schur_mf, dim3(n_items), dim3(512), 0, st, a);
    else hipLaunchKernelGGL(k_schur<real>, dim3(n_items), dim3(512), 0, st, a);
  }
  if (n_groups > 0)
    hipLaunchKernelGGL(k_schur_reduce<real>, dim3(SF * 9 * WAVE / 256, n_groups),
                       dim3(256), 0, st, a);
}

template void launch_schur<float>(const SchurArgs&, int, int, int, hipStream_t);
template void launch_schur<double>(const SchurArgs&, int, int, int, hipStream_t);

}  // namespace ptzba
