// Dense-tile fp64 Cholesky solve of the reduced camera system (gfx950).
//
// The reduced camera system S (SPD, block-banded: keyframes couple only to pan neighbours) replaces
// scipy's dense SVD of the full Jacobian (trf.py:467 via bundle_adjustment.py:200).
//
// Storage: row-major [ld][ld] lower triangle in the solver's system order (api.hip: natural frame
// order, or nested dissection [A | B reversed | C] with each part padded to whole 32-row tiles;
// padding rows are identity).  Row n_aug holds b^T (augmented right-hand side) with a huge diagonal,
// so row n_aug of the factor is y = L^-1 b: the forward substitution comes out of the factorisation.
//
// Factorisation: 32x32 tiles, one launch per LEVEL of the tile-column elimination tree ("delayed
// update"; natural order = one column per level, nested dissection = the A and B chains side by side).
// A task carries its tile (i, j) and up to two update panels p from the previous level:
//   panel task (i, k):   D <- A_kk - sum_p L_kp L_kp^T,  T <- A_ik - sum_p L_ip L_kp^T,
//                        then the workgroup factors D and solves L_ik = T L_kk^-T in the same sweep
//                        (wg_potrf_trsm32_df)   [i == k: L_kk -> Ldiag]
//   trailing task (i,j): A_ij <- A_ij - sum_p L_ip L_jp^T   (column j is factored at a later level)
// Every update (i, j, p) is applied exactly once, at the level after p's: by the trailing tasks, or by
// column j's panel tasks when j is factored at that very level.  Only structurally nonzero tiles
// (symbolic fill on the tile graph) are visited.
// Back substitution L^T x = y: one 1024-thread workgroup per chain of tile columns (nested
// dissection: C then A, C then B), right-looking updates of an LDS-resident right-hand side.
#include <algorithm>

#include <cstdlib>
#include <cstring>

#include "ptzba_common.h"
#include "ptzba_kernels.h"

namespace ptzba {

constexpr int NB = CHOL_NB;
constexpr double AUG_DIAG = 1e300;

__device__ __forceinline__ double bcast(double v, int j) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

// augmented row / padding: A[n][j] = b[j], A[n][n] = huge, A[i][i] = 1 for padding rows (pad[i], i < n)
// and for every row after n.  With PoseDamp (BA solve): also the Marquardt damping of the pose rows,
// D_f = max(D_f, diag U_f), S_ff += lambda D_f (scipy x_scale='jac', common.py:598-612) -- disjoint
// rows from the padding, so one launch does both.
struct PoseDamp {
  const double* dU;
  double* D_pose;
  const int32_t* frame_pos;
  int n_pose, n_fixed;
  double lambda;
  const double* lam_dev;
  // part-owned solve (api.hip): row_phase[r] = 1 rows of this rank's part, 2 separator rows, 0 rows of the
  // other part; phase 1 prepares the part's rows and writes the right-hand side of the part and of C (C's is
  // this rank's partial, summed by the separator exchange), phase 2 the separator's rows and the augmented
  // diagonal after that exchange.  phase 0: every row (replicated solve).
  const uint8_t* row_phase;
  int phase;
};
__global__ void k_chol_prepare(double* __restrict__ A, int64_t ld, int n, const double* __restrict__ b,
                               const uint8_t* __restrict__ pad, int* info, PoseDamp pd) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int ph = pd.phase;
  if (i == 0 && ph <= 1) info[0] = 0;  // (a part-owned solve's first phase: later phases keep the earlier verdict)
  if (i < n) {
    if (ph == 0 || (ph == 1 && pd.row_phase[i] != 0)) A[(int64_t)n * ld + i] = b[i];
    if (pad && pad[i] && (ph == 0 || pd.row_phase[i] == ph)) A[i * ld + i] = 1.0;
  }
  if (ph != 1) {
    if (i == n) A[i * ld + i] = AUG_DIAG;
    if (i > n && i < ld) A[i * ld + i] = 1.0;
  }
  if (pd.dU && i < 3 * (int64_t)(pd.n_pose - pd.n_fixed)) {
    const int f = pd.n_fixed + (int)(i / 3);
    const int64_t row = pd.frame_pos[f] + i % 3;
    if (ph != 0 && pd.row_phase[row] != ph) return;
    const double lambda = pd.lam_dev ? *pd.lam_dev : pd.lambda;
    double* D = pd.D_pose + 3 * pd.n_fixed + i;
    const double d = fmax(*D, fmax(pd.dU[row], 1e-12));
    *D = d;
    A[row * ld + row] += lambda * d;
  }
}

void launch_chol_prepare(double* A, int64_t ld, int n, double* b, const uint8_t* pad, int* info, hipStream_t st) {
  hipLaunchKernelGGL(k_chol_prepare, dim3((unsigned)((ld + 255) / 256)), dim3(256), 0, st, A, ld, n, b, pad, info,
                     PoseDamp{nullptr, nullptr, nullptr, 0, 0, 0.0, nullptr, nullptr, 0});
}
void launch_chol_prepare_damped(double* A, int64_t ld, int n, double* b, const uint8_t* pad, int* info,
                                const double* dU, double* D_pose, const int32_t* frame_pos, int n_pose, int n_fixed,
                                double lambda, const double* lam_dev, hipStream_t st, const uint8_t* row_phase,
                                int phase) {
  const int64_t m = std::max<int64_t>(ld, 3 * (int64_t)(n_pose - n_fixed));
  hipLaunchKernelGGL(k_chol_prepare, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, A, ld, n, b, pad, info,
                     PoseDamp{dU, D_pose, frame_pos, n_pose, n_fixed, lambda, lam_dev, row_phase, phase});
}

// Batched tile staging: every thread fetches its 4 elements of each tile into registers first (all global
// loads of a task in flight together: one memory round trip per task instead of one per update panel),
// then writes them to LDS.  256 threads per workgroup.
// COH (the SPD level launches' default): tiles are read with agent-scope loads that miss this XCD's L2 and written
// through with agent-scope stores (MI355X_MICROARCH.md, inter-workgroup hand-off table, first row), so the next
// level's workgroups on other XCDs find them in the Infinity Cache; plain accesses otherwise.
template <bool COH>
__device__ __forceinline__ double gld(const double* p) {
  if constexpr (COH) return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool COH>
__device__ __forceinline__ void gst(double* p, double v) {
  if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else *p = v;
}
// A thread stages two pairs of adjacent elements of a tile (pair p = threadIdx.x + 256 q: row p >> 4, columns
// 2 (p & 15) and 2 (p & 15) + 1) with 16-B loads -- half the load instructions of one element per load; COH: `sc1`
// buffer loads (aux 16), as the agent-scope loads above (tiles and ld are 16-B aligned: ld, the tile offsets and the
// pair columns are even)
typedef int v4i32 __attribute__((ext_vector_type(4)));
template <bool COH = false>
__device__ __forceinline__ void fetch_tile(double (&v)[4], const double* __restrict__ src, int64_t ld) {
  if constexpr (COH) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(src), 0,
                                                                       (int)((31 * ld + NB) * 8), 0x00020000);
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = threadIdx.x + 256 * q;
      const v4i32 x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(((p >> 4) * ld + 2 * (p & 15)) * 8), 0, 16);
      const double2 d = __builtin_bit_cast(double2, x);
      v[2 * q] = d.x;
      v[2 * q + 1] = d.y;
    }
  } else {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int p = threadIdx.x + 256 * q;
      const double2 d = *reinterpret_cast<const double2*>(src + (int64_t)(p >> 4) * ld + 2 * (p & 15));
      v[2 * q] = d.x;
      v[2 * q + 1] = d.y;
    }
  }
}
// The tile stores in the same pair order: 16-B stores of get(row, col), get(row, col + 1); COH: `sc1` buffer stores
// (write-through, as gst)
template <bool COH, typename F>
__device__ __forceinline__ void store_tile(double* __restrict__ dst, int64_t ld, F get) {
  __amdgpu_buffer_rsrc_t rs;
  if constexpr (COH) rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)((31 * ld + NB) * 8), 0x00020000);
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = threadIdx.x + 256 * q, r = p >> 4, c = 2 * (p & 15);
    const double2 d{get(r, c), get(r, c + 1)};
    if constexpr (COH) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4i32, d), rs, (int)((r * ld + c) * 8), 0, 16);
    else *reinterpret_cast<double2*>(dst + (int64_t)r * ld + c) = d;
  }
}
__device__ __forceinline__ void put_tile(double (*dst)[NB + 1], const double (&v)[4]) {
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int p = threadIdx.x + 256 * q;
    dst[p >> 4][2 * (p & 15)] = v[2 * q];
    dst[p >> 4][2 * (p & 15) + 1] = v[2 * q + 1];
  }
}

// C -= A B^T for 32x32 tiles in LDS on the fp64 matrix cores: 256 threads = 4 waves, wave w owns the
// 16x16 block (16 (w>>1), 16 (w&1)) and runs 8 v_mfma_f64_16x16x4_f64 (k = 4 per step).  Operand lane
// maps (gfx950): A[i = l&15][k = l>>4], B[k = l>>4][j = l&15]; D[row = (l>>4) + 4 r][col = l&15].
typedef double v4f64 __attribute__((ext_vector_type(4)));
// SG: C -= A Sigma B^T with Sigma = diag(sg) (the signed factor of an indefinite system, see k_chol_step)
// The level tasks keep C in registers instead (blk_acc_*): wave w's block, the 4 values of the MFMA D layout.
template <bool SG = false>
__device__ __forceinline__ void blk_gemm_nt_sub(v4f64& acc, const double (*A)[NB + 1], const double (*B)[NB + 1],
                                                const double* sg = nullptr) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const int bi = (w >> 1) * 16, bj = (w & 1) * 16;
  const int li = l & 15, lk = l >> 4;
#pragma unroll
  for (int s = 0; s < NB / 4; ++s) {
    const double a = -A[bi + li][4 * s + lk];
    double b = B[bj + li][4 * s + lk];
    if constexpr (SG) b *= sg[4 * s + lk];
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
  }
}
// wave w's 16 x 16 block of a 32 x 32 tile (rows 16 (w >> 1) + lk + 4 r, columns 16 (w & 1) + li) from / to memory
// or LDS
template <bool COH>
__device__ __forceinline__ void blk_acc_load(v4f64& acc, const double* __restrict__ tile, int64_t ld) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const double* p = tile + (int64_t)((w >> 1) * 16 + (l >> 4)) * ld + (w & 1) * 16 + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) acc[r] = gld<COH>(p + (int64_t)(4 * r) * ld);
}
template <bool COH>
__device__ __forceinline__ void blk_acc_store(double* __restrict__ tile, int64_t ld, const v4f64& acc) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double* p = tile + (int64_t)((w >> 1) * 16 + (l >> 4)) * ld + (w & 1) * 16 + (l & 15);
#pragma unroll
  for (int r = 0; r < 4; ++r) gst<COH>(p + (int64_t)(4 * r) * ld, acc[r]);
}
__device__ __forceinline__ void blk_acc_put(double (*C)[NB + 1], const v4f64& acc) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < 4; ++r) C[(w >> 1) * 16 + (l >> 4) + 4 * r][(w & 1) * 16 + (l & 15)] = acc[r];
}

// fp64 reciprocal and reciprocal square root: hardware estimate + two Newton steps (full double
// precision, a much shorter dependent chain than IEEE division / sqrt on the pivot critical path)
__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  return fma(r, fma(-d, r, 1.0), r);
}
__device__ __forceinline__ double rsq_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y * fma(-0.5 * d * y, y, 1.5);
}

#ifdef CS_TIMING
__device__ long long g_cs_stamps[64][6];
__device__ long long g_cs_wg[64][10];
__device__ int g_cs_level;
// sweep accounting (round 6): per level, block 0's wave 0 stamps eight points of every 4-pivot block, the helpers the
// time they publish each block (tools/chol_timing.py --sweep)
__device__ long long g_cs_blk[64][8][8];
__device__ long long g_cs_hlp[64][8][3];
// the level timeline in s_memrealtime (100 MHz, one clock for every XCD): block 0's task start, sweep end, factor
// stores complete; and the last workgroup of the level to finish its task (atomicMax)
__device__ long long g_cs_rt[64][4];
#define CSB(s_, k_) do { if (wrec0 && (s_) < 8) { __builtin_amdgcn_s_waitcnt(0xc07f); cs_blk[s_][k_] = clock64(); } } while (0)
#else
#define CSB(s_, k_) do { } while (0)
#endif
#ifndef BS_LOADERS
#define BS_LOADERS 1  // loader waves of the lookahead back-solve (2: ring positions alternate; measured neutral)
#endif
#ifndef LA_BW
#define LA_BW 4  // pivot block of the lookahead form
#endif
// reciprocal square root by a series step on the hardware estimate: e = 1 - d y0^2 (|e| ~ 5e-8),
// y = y0 (1 + e/2 + 3e^2/8) -- full double precision in 4 dependent operations (rsq_nr: 6)
__device__ __forceinline__ double rsq_fast(double d) {
  const double y0 = __builtin_amdgcn_rsq(d);
  const double e = fma(-d * y0, y0, 1.0);
  return fma(y0 * e, fma(e, 0.375, 0.5), y0);
}

// The pivot sweep (round 2-4 history: single-wave, 4-wave and barrier-per-stage lookahead forms): wave 0
// runs the critical chain one pivot block of BW columns at a time, waves 1-3 bring the next block up to date, and
// no workgroup barrier separates the stages.  LDS counters carry the two dependencies instead:
//   nl = number of factor blocks wave 0 has published (waves 1-3 wait for block t-1 before stage t),
//   nu[t] = helper waves that have brought block t+1 up to date (wave 0 waits for all 3 before it
//           starts block t+1).
__device__ __forceinline__ int lds_poll(const int* p) {
  return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
}
// LDS-only hand-off between waves of one workgroup without release/acquire semantics (those also wait
// for the wave's outstanding global loads, i.e. for its prefetches): the producer waits for its own LDS
// writes (lgkmcnt) and stores the counter; the consumer polls it and its later LDS reads stay behind
// the poll (LDS operations of a wave execute in order; compiler barrier against reordering).
__device__ __forceinline__ void lds_signal(int* p, int v) {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
  __builtin_amdgcn_wave_barrier();
  if (lane_id() == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const int* p, int v, int sleep) {
  while (__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < v) {
    if (sleep) __builtin_amdgcn_s_sleep(1);
  }
  asm volatile("" ::: "memory");
}
// SG (signed, for the indefinite EKF innovation matrix): factor A = L Sigma L^T, Sigma = diag(+-1) --
// a pivot d < 0 gives L_jj = sqrt(|d|), sigma_j = -1 (Sylvester: as many negative pivots as negative
// eigenvalues; no pivoting, as np.linalg.inv of the reference would not need); every update carries the
// sign of its pivot.  The signs go to sig[NB] (LDS) for the caller.  SG = false is the SPD factor.
template <int BW, bool SG = false>
__device__ __forceinline__ void wg_potrf_trsm32_df(double (*D)[NB + 1], double (*T)[NB + 1],
                                                   double (*Lb)[2 * NB][BW], double (*Pb)[BW], int* flags,
                                                   int* info, double* sig = nullptr) {
  constexpr int NS = NB / BW;
  const int w = threadIdx.x >> 6, lane = lane_id();
  const bool isT = lane >= NB;
  const int r = lane & (NB - 1);
  const bool have = !isT || T != nullptr;
  double* row = (isT && T) ? T[r] : D[r];
  int* nl = flags;
  int* nu = flags + 1;  // [NS]
  if (threadIdx.x <= NS) flags[threadIdx.x] = 0;
  __syncthreads();
#ifdef CS_TIMING
  long long* wst = g_cs_wg[g_cs_level < 64 ? g_cs_level : 63];
  const bool wrec = threadIdx.x == 0 && blockIdx.x == 0;
  if (wrec) wst[0] = clock64();
  const int cs_l = g_cs_level < 64 ? g_cs_level : 63;
  const bool wrec0 = lane == 0 && w == 0 && blockIdx.x == 0;
  long long (*cs_blk)[8] = g_cs_blk[cs_l];
  if (wrec0) { cs_blk[0][1] = __builtin_amdgcn_s_memrealtime(); cs_blk[2][1] = clock64(); }
#endif
  if (w == 0) {
    bool bad = false;
    double lp[BW];  // this lane's factor values of the last block (SG: sigma_k L_rk, the update operand)
#pragma unroll
    for (int k = 0; k < BW; ++k) lp[k] = 0.0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const int kb = s * BW;
      CSB(s, 0);
      // the previous block's factor rows kb..kb+BW-1 (this wave's own stores) are read before the wait for the
      // helpers: their LDS round trip overlaps the poll's instead of following it
      double pl[BW][BW];
      if (s > 0) {
#pragma unroll
        for (int j = 0; j < BW; ++j)
#pragma unroll
          for (int k = 0; k < BW; ++k) pl[j][k] = Lb[s - 1][kb + j][k];
      }
      double a[BW];
      if (s >= 2) {
        while (lds_poll(&nu[s - 1]) < 3) __builtin_amdgcn_s_sleep(0);
      }
      CSB(s, 2);
#pragma unroll
      for (int j = 0; j < BW; ++j) a[j] = row[kb + j];
      CSB(s, 3);
      if (s > 0) {
#pragma unroll
        for (int j = 0; j < BW; ++j) {
          double acc = a[j];
#pragma unroll
          for (int k = 0; k < BW; ++k) acc = fma(-lp[k], pl[j][k], acc);
          a[j] = acc;
        }
      }
      double P[BW][BW], y[BW], sg[BW];
      // the BW x BW diagonal block lives in lanes kb..kb+BW-1 of this wave: read it lane to lane
      // (v_readlane, uniform lane indices) instead of a round trip through LDS
#pragma unroll
      for (int i = 0; i < BW; ++i)
#pragma unroll
        for (int j = 0; j <= i; ++j) P[i][j] = bcast(a[j], kb + i);
#ifdef CS_TIMING
      if (wrec0 && s < 8) {  // consume P so the stamp follows the gathers
        double t = 0.0;
#pragma unroll
        for (int i = 0; i < BW; ++i) t += P[i][i];
        if (t == 12345.678) cs_blk[s][7] = 1;
      }
#endif
      CSB(s, 4);
      {
#pragma unroll
      for (int j = 0; j < BW; ++j) {
        double d = P[j][j];
        sg[j] = 1.0;
        if constexpr (SG) {
          if (d < 0.0) {
            sg[j] = -1.0;
            d = -d;
          }
        }
        if (!(d > 0.0)) {
          bad = true;
          d = 1e-300;
        }
        y[j] = rsq_fast(d);
#pragma unroll
        for (int i = j + 1; i < BW; ++i) P[i][j] *= y[j];  // = sigma_j L_ij
#pragma unroll
        for (int i = j + 1; i < BW; ++i)
#pragma unroll
          for (int m = j + 1; m <= i; ++m) {
            if constexpr (SG) P[i][m] = fma(-sg[j] * P[i][j], P[m][j], P[i][m]);
            else P[i][m] = fma(-P[i][j], P[m][j], P[i][m]);
          }
      }
#ifdef CS_TIMING
      if (wrec0 && s < 8 && y[BW - 1] == 12345.678) cs_blk[s][7] = 1;
#endif
      CSB(s, 5);
#pragma unroll
      for (int j = 0; j < BW; ++j) {
        const double x = a[j] * y[j];  // sigma_j L_rj
        lp[j] = x;
#pragma unroll
        for (int i = j + 1; i < BW; ++i) {
          if constexpr (SG) a[i] = fma(-sg[j] * P[i][j], x, a[i]);
          else a[i] = fma(-P[i][j], x, a[i]);
        }
      }
      }
#ifdef CS_TIMING
      if (wrec0 && s < 8 && lp[BW - 1] == 12345.678) cs_blk[s][7] = 1;
#endif
      CSB(s, 6);
#pragma unroll
      for (int j = 0; j < BW; ++j) Lb[s][lane][j] = SG ? sg[j] * lp[j] : lp[j];  // L_rj
      if constexpr (SG) {
        if (lane == 0) {
#pragma unroll
          for (int j = 0; j < BW; ++j) sig[kb + j] = sg[j];
        }
      }
      if (s + 2 < NS) {
        __builtin_amdgcn_s_waitcnt(0xc07f);
        __builtin_amdgcn_wave_barrier();
        if (lane == 0) __hip_atomic_store(nl, s + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      CSB(s, 7);
#ifdef CS_TIMING
      if (wrec && s < 9) wst[1 + s] = clock64();
#endif
    }
    if (bad && lane == 0) atomicOr(info, 1);
#ifdef CS_TIMING
    if (wrec0) { cs_blk[1][1] = __builtin_amdgcn_s_memrealtime(); cs_blk[3][1] = clock64(); }
#endif
  } else {
    // helpers, left-looking: during wave 0's stage t they bring block t+1 up to date with the factor
    // blocks 0..t-1 (wave 0 adds block t itself), so each block is written once and wave 0 never waits
    // for bulk updates.  Column m belongs to wave 1 + m % 3.
    const int u = w - 1;  // 0..2
    double lr[NS][BW];    // this lane's row of the published factor blocks
#pragma unroll
    for (int t = 1; t + 1 < NS; ++t) {
      const int kb = t * BW;
      while (lds_poll(nl) < t) __builtin_amdgcn_s_sleep(0);
#pragma unroll
      for (int k = 0; k < BW; ++k) {
        lr[t - 1][k] = Lb[t - 1][lane][k];
        if constexpr (SG) lr[t - 1][k] *= sig[(t - 1) * BW + k];  // published before nl (same LDS order)
      }
#pragma unroll
      for (int m = kb + BW; m < kb + 2 * BW; ++m) {
        if (m % 3 != u) continue;
        double acc = row[m];
#pragma unroll
        for (int b = 0; b < t; ++b)
#pragma unroll
          for (int k = 0; k < BW; ++k) acc = fma(-lr[b][k], Lb[b][m][k], acc);
        if (have) row[m] = acc;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      if (lane == 0) __hip_atomic_fetch_add(&nu[t], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
#ifdef CS_TIMING
      if (lane == 0 && blockIdx.x == 0 && t < 8) g_cs_hlp[cs_l][t][u] = clock64();
#endif
    }
  }
  __syncthreads();
}

#ifdef CS_TIMING
#define CS_STAMP(k) do { if (threadIdx.x == 0 && blockIdx.x == 0 && cs_lvl < 64) g_cs_stamps[cs_lvl][k] = clock64(); } while (0)
#define CS_RT(k) do { if (threadIdx.x == 0 && blockIdx.x == 0 && cs_lvl < 64) g_cs_rt[cs_lvl][k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#define CS_RT_END() do { if (threadIdx.x == 0 && cs_lvl < 64) { __builtin_amdgcn_s_waitcnt(0); atomicMax((unsigned long long*)&g_cs_rt[cs_lvl][3], (unsigned long long)__builtin_amdgcn_s_memrealtime()); } } while (0)
#else
#define CS_STAMP(k) do { } while (0)
#define CS_RT(k) do { } while (0)
#define CS_RT_END() do { } while (0)
#endif
// SG: signed factor A = L Sigma L^T (indefinite systems: the EKF innovation block, ekf.hip); sgn[ld] holds
// sigma per factored row, written by each column's diagonal task and applied to the update panels
// A level's tasks: by value in the kernel arguments when they fit (the workgroup's first dependent global
// load -- tasks[blockIdx.x] before any tile address is known -- disappears from the level's critical path),
// else a device array.
// M = L^-1 of one 32 x 32 lower factor tile (row-major), by the whole workgroup: stage L in LDS, diagonal
// reciprocals, then one wave: lane j computes column j by forward substitution against e_j, right-looking
// (after m_k is known every later row's running sum takes its term at once: the dependent chain is one
// multiply and one FMA per row).  Shared by k_tile_inv and the type-2 tasks of the level launches.
template <bool COH = false>
__device__ __forceinline__ void tile_inv_wave(const double* __restrict__ src, double* __restrict__ dst,
                                              double (*Lt)[NB + 1], double* rinv) {
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) Lt[e >> 5][e & 31] = gld<COH>(src + e);
  __syncthreads();
  if (threadIdx.x < NB) rinv[threadIdx.x] = rcp_nr(Lt[threadIdx.x][threadIdx.x]);
  __syncthreads();
  if (threadIdx.x >= WAVE) return;
  const int lane = threadIdx.x, j = lane & (NB - 1);
  double acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = (i == j) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double mk = (k >= j) ? acc[k] * rinv[k] : 0.0;  // m_k (0 above the diagonal)
    acc[k] = mk;
#pragma unroll
    for (int i = k + 1; i < NB; ++i) acc[i] = fma(-Lt[i][k], mk, acc[i]);
  }
  if (lane < NB) {
#pragma unroll
    for (int i = 0; i < NB; ++i) dst[i * NB + lane] = acc[i];
  }
}

// Trailing block task (type 3, plans with delayed updates): output tiles (i0 + a, j0 + b), a, b in {0, 1}, present
// where bit 2a + b of mask is set; wave 2a + b owns tile (a, b) whole, its four 16 x 16 blocks as MFMA
// accumulators read from and written back to memory directly.  Per update panel p (ascending, the same order as
// the per-tile tasks) the workgroup stages the four row tiles L_{i0,p}, L_{i0+1,p} (A side) and L_{j0,p},
// L_{j0+1,p} (B side) in LDS -- each loaded once for the (up to) two output tiles that use it -- with the next
// panel's tiles in flight in registers.  Same MFMA sequence per output tile as tile_gemm_nt_sub: bitwise the
// result of one task per tile.
template <bool COH = false>
__device__ __forceinline__ void chol_trail_block(double* __restrict__ A, int64_t ld, int i0, int j0, int mask, int up0,
                                                 int up1, int up2, int up3, double (*sA)[NB][NB + 1],
                                                 double (*sB)[NB][NB + 1]) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63, li = l & 15, lk = l >> 4;
  const int64_t NBl = NB;
  const bool mine = (mask >> w) & 1;
  const int ta = w >> 1, tb = w & 1;
  // which staged tiles some present output tile needs
  const bool needA[2] = {(mask & 3) != 0, (mask & 12) != 0};
  const bool needB[2] = {(mask & 5) != 0, (mask & 10) != 0};
  double* C = A + (i0 + ta) * NBl * ld + (j0 + tb) * NBl;
  v4f64 acc[2][2];
  if (mine) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[x][y][r] = gld<COH>(C + (int64_t)(16 * x + lk + 4 * r) * ld + 16 * y + li);
  }
  const int ups[4] = {up0, up1, up2, up3};
  double ra[2][4], rb[2][4];  // one register set: the next panel's tiles are fetched once this one is in LDS
  auto fetch = [&](int p) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (needA[t]) fetch_tile<COH>(ra[t], A + (i0 + t) * NBl * ld + p * NBl, ld);
      if (needB[t]) fetch_tile<COH>(rb[t], A + (j0 + t) * NBl * ld + p * NBl, ld);
    }
  };
  int u = 0;
  while (u < 4 && ups[u] < 0) ++u;
  if (u < 4) fetch(ups[u]);
  while (u < 4) {
    int un = u + 1;
    while (un < 4 && ups[un] < 0) ++un;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      if (needA[t]) put_tile(sA[t], ra[t]);
      if (needB[t]) put_tile(sB[t], rb[t]);
    }
    if (un < 4) fetch(ups[un]);  // in flight during this panel's MFMAs (the LDS writes above read the registers first)
    __syncthreads();
    if (mine) {
      const double (*At)[NB + 1] = sA[ta];
      const double (*Bt)[NB + 1] = sB[tb];
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int s4 = 0; s4 < NB / 4; ++s4) {
            const double av = -At[16 * x + li][4 * s4 + lk];
            const double bv = Bt[16 * y + li][4 * s4 + lk];
            acc[x][y] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc[x][y], 0, 0, 0);
          }
    }
    __syncthreads();
    u = un;
  }
  if (mine) {
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int r = 0; r < 4; ++r) gst<COH>(C + (int64_t)(16 * x + lk + 4 * r) * ld + 16 * y + li, acc[x][y][r]);
  }
}

struct CholTaskPtr {
  const int4* p;
  __device__ int4 get(int b) const { return p[b]; }
};
// the level's first CHOL_KT tasks by value in the kernel arguments (its panel tasks -- the critical path -- come
// first in every level's list), the rest from the device array (trailing tasks of the wide levels)
struct CholTaskVal {
  int4 t[CHOL_KT];
  const int4* rest;
  __device__ int4 get(int b) const { return b < CHOL_KT ? t[b] : rest[b - CHOL_KT]; }
};
// P2: plans with delayed trailing updates (a second pair of update panels per task, api.hip make_plan)
// One factorisation task (api.hip make_plan: panel / trailing / inverse / trailing block) by the workgroup: the
// body of a level launch (k_chol_step).
template <bool SG, bool P2, bool COH>
__device__ __forceinline__ void chol_task(double* __restrict__ A, int64_t ld, const int4 tk, double* __restrict__ Ldiag,
                                          int* info, double* __restrict__ sgn, double* __restrict__ Minv) {
  static_assert(!(COH && SG), "coherent tile accesses: SPD level launches only");
  // Four tiles of LDS: the update panels' row tiles while the task's target tiles accumulate in registers (wave w
  // owns one 16 x 16 block of each: blk_acc_*); after the last update the panel task parks D and T in sP[2] / sP[3]
  // for the sweep, whose block buffer overlays sP[0..1].  34 KB per workgroup: four workgroups per CU (three with
  // round 5's six LDS tiles, 51 KB) -- config 4's trailing levels carry 800-1,900 tasks each.
  __shared__ __attribute__((aligned(16))) double sP[4][NB][NB + 1];
  double (*const sA)[NB][NB + 1] = sP;      // L_ip (panel task: of the T side) of the two update panels in LDS
  double (*const sB)[NB][NB + 1] = sP + 2;  // L_kp or L_jp of the two update panels
  double (*const sD)[NB + 1] = sP[2];       // after the updates: D -> L_kk (the sweep)
  double (*const sC)[NB + 1] = sP[3];       // after the updates: T_ik
  static_assert((NB / LA_BW) * 2 * NB * LA_BW <= 2 * NB * (NB + 1), "block buffer must fit the panel tiles");
  double (*s_lb)[2 * NB][LA_BW] = reinterpret_cast<double (*)[2 * NB][LA_BW]>(&sP[0][0][0]);
  __shared__ __attribute__((aligned(16))) double s_pb[LA_BW][LA_BW];
  __shared__ int s_flags[NB / LA_BW + 1];
  __shared__ double s_sgp[2][NB];  // SG: signs of the two update panels' columns
  __shared__ double s_sig[NB];     // SG: signs of this column's pivots
  if ((tk.x & 3) == 2) {  // inverse of a diagonal factor tile of the previous level (see tile_inv_wave)
    if (tk.y < 0) return;  // (no-op slot)
    __shared__ double s_rinv[NB];
    tile_inv_wave<COH>(Ldiag + (int64_t)tk.y * NB * NB, Minv + (int64_t)tk.y * NB * NB, sD, s_rinv);
    return;
  }
  const int type = tk.x & 3, i = tk.y, j = tk.z;
  const int up0 = (tk.w & 0x3fff) - 1;
  const int up1 = ((tk.w >> 14) & 0x3fff) - 1;
  const int tmask = (tk.w >> 28) & 3;  // panel: which updates also apply to T
  // delayed trailing updates (api.hip make_plan, period 2): a second pair of update panels rides in x
  const int up2 = P2 ? (int)(((unsigned)tk.x >> 2) & 0x3fff) - 1 : -1;
  const int up3 = P2 ? (int)(((unsigned)tk.x >> 16) & 0x3fff) - 1 : -1;
  const int tmask2 = P2 ? (int)((unsigned)tk.x >> 30) : 0;
  const bool pass2 = P2 && (up2 >= 0 || up3 >= 0);
  const int64_t NBl = NB;
#ifdef CS_TIMING
  const int cs_lvl = g_cs_level;
  if (threadIdx.x == 0 && blockIdx.x == 0 && cs_lvl < 64) g_cs_stamps[cs_lvl][5] = type;
#endif
  CS_STAMP(0);
  CS_RT(0);
  if constexpr (P2 && !SG) {
    if (type == 3) {  // 2 x 2 block of trailing tiles (api.hip make_plan): A_ij -= sum_p L_ip L_jp^T
      chol_trail_block<COH>(A, ld, i, j, ((tk.w >> 28) & 3) | (((unsigned)tk.x >> 30) << 2), up0, up1, up2, up3, sA, sB);
      return;
    }
  }
  double v1[4], v2[4], v3[4], v4[4], v5[4], w2[4], w3[4], w4[4], w5[4];
  auto load_signs = [&](int ua, int ub) {  // SG: signs of the update panels' columns
    if constexpr (SG) {
      if (threadIdx.x < 2 * NB) {
        const int q = threadIdx.x >> 5, up = q ? ub : ua;
        s_sgp[q][threadIdx.x & 31] = up >= 0 ? sgn[(int64_t)up * NB + (threadIdx.x & 31)] : 1.0;
      }
    }
  };
  // the update panels' row tiles through LDS, in pairs (the second pair of a delayed plan in the same buffers, a
  // barrier between); the target blocks accumulate in registers: per output element the same MFMA sequence in the
  // same panel order as round 5's LDS-resident targets (bitwise the same factor)
  auto stage_pair = [&](const double (&ra0)[4], const double (&rb0)[4], const double (&ra1)[4],
                        const double (&rb1)[4], bool a0, bool b0, bool a1, bool b1) {
    if (a0) put_tile(sA[0], ra0);
    if (b0) put_tile(sB[0], rb0);
    if (a1) put_tile(sA[1], ra1);
    if (b1) put_tile(sB[1], rb1);
  };
  if (type == 1) {
    // trailing: A_ij -= sum_p L_ip L_jp^T
    double* C = A + i * NBl * ld + j * NBl;
    v4f64 acc;
    blk_acc_load<COH>(acc, C, ld);
    if (up0 >= 0) {
      fetch_tile<COH>(v1, A + i * NBl * ld + up0 * NBl, ld);
      fetch_tile<COH>(v2, A + j * NBl * ld + up0 * NBl, ld);
    }
    if (up1 >= 0) {
      fetch_tile<COH>(v3, A + i * NBl * ld + up1 * NBl, ld);
      fetch_tile<COH>(v4, A + j * NBl * ld + up1 * NBl, ld);
    }
    if (up2 >= 0) {
      fetch_tile<COH>(w2, A + i * NBl * ld + up2 * NBl, ld);
      fetch_tile<COH>(w3, A + j * NBl * ld + up2 * NBl, ld);
    }
    if (up3 >= 0) {
      fetch_tile<COH>(w4, A + i * NBl * ld + up3 * NBl, ld);
      fetch_tile<COH>(w5, A + j * NBl * ld + up3 * NBl, ld);
    }
    stage_pair(v1, v2, v3, v4, up0 >= 0, up0 >= 0, up1 >= 0, up1 >= 0);
    load_signs(up0, up1);
    __syncthreads();
    if (up0 >= 0) blk_gemm_nt_sub<SG>(acc, sA[0], sB[0], s_sgp[0]);
    if (up1 >= 0) blk_gemm_nt_sub<SG>(acc, sA[1], sB[1], s_sgp[1]);
    if (pass2) {  // the second pair through the same panel buffers
      __syncthreads();
      stage_pair(w2, w3, w4, w5, up2 >= 0, up2 >= 0, up3 >= 0, up3 >= 0);
      load_signs(up2, up3);
      __syncthreads();
      if (up2 >= 0) blk_gemm_nt_sub<SG>(acc, sA[0], sB[0], s_sgp[0]);
      if (up3 >= 0) blk_gemm_nt_sub<SG>(acc, sA[1], sB[1], s_sgp[1]);
    }
    blk_acc_store<COH>(C, ld, acc);
    return;
  }
  // panel task (i, k = j)
  const int k = j;
  const bool diag_only = (i == k);
  const bool updT0 = !diag_only && (tmask & 1), updT1 = !diag_only && (tmask & 2);
  const bool updT2 = !diag_only && (tmask2 & 1), updT3 = !diag_only && (tmask2 & 2);
  v4f64 accD, accT;
  blk_acc_load<COH>(accD, A + (int64_t)k * NBl * ld + k * NBl, ld);
  if (!diag_only) blk_acc_load<COH>(accT, A + i * NBl * ld + k * NBl, ld);
  if (up0 >= 0) fetch_tile<COH>(v2, A + (int64_t)k * NBl * ld + up0 * NBl, ld);
  if (updT0 && up0 >= 0) fetch_tile<COH>(v3, A + i * NBl * ld + up0 * NBl, ld);
  if (up1 >= 0) fetch_tile<COH>(v4, A + (int64_t)k * NBl * ld + up1 * NBl, ld);
  if (updT1 && up1 >= 0) fetch_tile<COH>(v5, A + i * NBl * ld + up1 * NBl, ld);
  if (up2 >= 0) fetch_tile<COH>(w2, A + (int64_t)k * NBl * ld + up2 * NBl, ld);
  if (updT2 && up2 >= 0) fetch_tile<COH>(w3, A + i * NBl * ld + up2 * NBl, ld);
  if (up3 >= 0) fetch_tile<COH>(w4, A + (int64_t)k * NBl * ld + up3 * NBl, ld);
  if (updT3 && up3 >= 0) fetch_tile<COH>(w5, A + i * NBl * ld + up3 * NBl, ld);
  const bool any_up = up0 >= 0 || up1 >= 0;
  if (any_up) {
    stage_pair(v3, v2, v5, v4, updT0 && up0 >= 0, up0 >= 0, updT1 && up1 >= 0, up1 >= 0);
    load_signs(up0, up1);
    __syncthreads();
  }
  CS_STAMP(1);
  if (up0 >= 0) {
    blk_gemm_nt_sub<SG>(accD, sB[0], sB[0], s_sgp[0]);
    if (updT0) blk_gemm_nt_sub<SG>(accT, sA[0], sB[0], s_sgp[0]);
  }
  if (up1 >= 0) {
    blk_gemm_nt_sub<SG>(accD, sB[1], sB[1], s_sgp[1]);
    if (updT1) blk_gemm_nt_sub<SG>(accT, sA[1], sB[1], s_sgp[1]);
  }
  if (pass2) {  // the delayed pair (api.hip make_plan) through the same panel buffers
    if (any_up) __syncthreads();
    stage_pair(w3, w2, w5, w4, updT2 && up2 >= 0, up2 >= 0, updT3 && up3 >= 0, up3 >= 0);
    load_signs(up2, up3);
    __syncthreads();
    if (up2 >= 0) {
      blk_gemm_nt_sub<SG>(accD, sB[0], sB[0], s_sgp[0]);
      if (updT2) blk_gemm_nt_sub<SG>(accT, sA[0], sB[0], s_sgp[0]);
    }
    if (up3 >= 0) {
      blk_gemm_nt_sub<SG>(accD, sB[1], sB[1], s_sgp[1]);
      if (updT3) blk_gemm_nt_sub<SG>(accT, sA[1], sB[1], s_sgp[1]);
    }
  }
  if (any_up || pass2) __syncthreads();  // the panel tiles are read: D and T take their place
  blk_acc_put(sD, accD);
  if (!diag_only) blk_acc_put(sC, accT);
  __syncthreads();
  CS_STAMP(2);
  wg_potrf_trsm32_df<LA_BW, SG>(sD, diag_only ? nullptr : sC, s_lb, s_pb, s_flags, info, s_sig);
  __syncthreads();  // (the flag-synchronised sweep ends in a barrier of its own)
  CS_STAMP(3);
  CS_RT(1);
#ifdef CS_TIMING
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    CS_STAMP(4);
    g_cs_level = cs_lvl + 1;
  }
#endif
  // the factor goes to memory straight from the sweep's block buffer (rows 0..31: D, 32..63: T)
  if (diag_only) {
    store_tile<COH>(Ldiag + (int64_t)k * NB * NB, NB,
                    [&](int r, int m) { return m <= r ? s_lb[m / LA_BW][r][m % LA_BW] : 0.0; });
    if constexpr (SG) {
      if (threadIdx.x < NB) sgn[(int64_t)k * NB + threadIdx.x] = s_sig[threadIdx.x];
    }
#ifdef CS_TIMING
    if (threadIdx.x == 0 && blockIdx.x == 0 && cs_lvl < 64) {
      __builtin_amdgcn_s_waitcnt(0);
      g_cs_rt[cs_lvl][2] = __builtin_amdgcn_s_memrealtime();
    }
    CS_RT_END();
#endif
    return;
  }
  // (A_kk itself stays untouched: other panel workgroups of this launch are still reading it)
  store_tile<COH>(A + i * NBl * ld + k * NBl, ld, [&](int r, int m) { return s_lb[m / LA_BW][NB + r][m % LA_BW]; });
#ifdef CS_TIMING
  if (threadIdx.x == 0 && blockIdx.x == 0 && cs_lvl < 64) {
    __builtin_amdgcn_s_waitcnt(0);
    g_cs_rt[cs_lvl][2] = __builtin_amdgcn_s_memrealtime();
  }
  CS_RT_END();
#endif
}

template <bool SG, typename TaskArg, bool P2 = false, bool COH = false>
__global__ __launch_bounds__(256) void k_chol_step(double* __restrict__ A, int64_t ld, const TaskArg tasks,
                                                   double* __restrict__ Ldiag, int* info, double* __restrict__ sgn,
                                                   double* __restrict__ Minv) {
  chol_task<SG, P2, COH>(A, ld, tasks.get(blockIdx.x), Ldiag, info, sgn, Minv);
}

// (Rounds 4 tried every level of a factorisation in ONE launch -- one workgroup per task, a task of level L waiting
// on level L - 1's completion counter: bitwise the same factor, 338-425 us per trial against ~232 with one launch per
// level; removed in round 5.)
// SPD factorisations write their tiles through (agent-scope stores) and read them past this XCD's L2 (COH): the next
// level's workgroups, mostly on other XCDs, find the tiles in the Infinity Cache at once (same-box A/B r04e:
// cholesky_solve 240 -> 232 us per trial at config 3; the plain-access knob PTZBA_CHOL_COH=0 was removed in round 6).
// The signed (EKF) factor keeps plain accesses.
template <typename TaskArg>
static void launch_chol_level(const TaskArg& ta, int n, double* A, int64_t ld, double* Ldiag, int* info, double* sgn,
                              double* Minv, bool delayed, hipStream_t st) {
  if (sgn)
    hipLaunchKernelGGL((k_chol_step<true, TaskArg, false, false>), dim3(n), dim3(256), 0, st, A, ld, ta, Ldiag, info, sgn, Minv);
  else if (delayed)
    hipLaunchKernelGGL((k_chol_step<false, TaskArg, true, true>), dim3(n), dim3(256), 0, st, A, ld, ta, Ldiag, info, sgn, Minv);
  else
    hipLaunchKernelGGL((k_chol_step<false, TaskArg, false, true>), dim3(n), dim3(256), 0, st, A, ld, ta, Ldiag, info, sgn, Minv);
}
void launch_cholesky(double* A, int64_t ld, const int4* tasks, const int* task_off_host, int n_launch, double* Ldiag,
                     int* info, hipStream_t st, double* sgn, const int4* tasks_host, double* Minv, int first_level,
                     bool delayed) {
  // a level's first CHOL_KT tasks travel by value in the kernel arguments (the rest through a pointer): the
  // workgroup's first dependent load disappears (round 2 A/B: 313 -> 308 us per trial at config 3)
  for (int L = first_level; L < n_launch; ++L) {
    const int n = task_off_host[L + 1] - task_off_host[L];
    if (n <= 0) continue;
    if (tasks_host) {
      CholTaskVal tv;
      std::memcpy(tv.t, tasks_host + task_off_host[L], std::min(n, CHOL_KT) * sizeof(int4));
      tv.rest = tasks + task_off_host[L] + CHOL_KT;
      launch_chol_level<CholTaskVal>(tv, n, A, ld, Ldiag, info, sgn, Minv, delayed, st);
      continue;
    }
    launch_chol_level<CholTaskPtr>(CholTaskPtr{tasks + task_off_host[L]}, n, A, ld, Ldiag, info, sgn, Minv, delayed, st);
  }
}

// ---------------------------------------------------------------------------------------------
// inverses of the diagonal factor tiles: M_kt = L_kt,kt^-1 (lower), row-major [kt][32][32].  One wave
// per tile: lane j computes column j by forward substitution against e_j, right-looking (after m_k is
// known, every later row's running sum takes its term at once), so the dependent chain is one
// multiply and one FMA per row; the diagonal reciprocals are formed up front, off the chain.
__global__ __launch_bounds__(64) void k_tile_inv(const double* __restrict__ Ldiag, double* __restrict__ Minv) {
  __shared__ __attribute__((aligned(16))) double Lt[NB][NB];
  __shared__ double rinv[NB];
  const int kt = blockIdx.x, lane = threadIdx.x, j = lane & (NB - 1);
  const double* src = Ldiag + (int64_t)kt * NB * NB;
  for (int e = lane; e < NB * NB; e += WAVE) Lt[e >> 5][e & 31] = src[e];
  __syncthreads();
  if (lane < NB) rinv[lane] = rcp_nr(Lt[lane][lane]);
  __syncthreads();
  double acc[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) acc[i] = (i == j) ? 1.0 : 0.0;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double mk = (k >= j) ? acc[k] * rinv[k] : 0.0;  // m_k (0 above the diagonal)
    acc[k] = mk;
#pragma unroll
    for (int i = k + 1; i < NB; ++i) acc[i] = fma(-Lt[i][k], mk, acc[i]);
  }
  if (lane < NB) {
    double* dst = Minv + (int64_t)kt * NB * NB + lane;
#pragma unroll
    for (int i = 0; i < NB; ++i) dst[i * NB] = acc[i];
  }
}

#ifdef BS_TIMING
__device__ long long g_bs_stamps[2][128][6];
__device__ long long g_bs_edges[2][4];
#endif
// Back substitution L^T x = y (y = row n of the factor, x written to xout[0..n)) with a lookahead chain wave, one
// workgroup per chain of tile columns (nested dissection: C then A, C then B), no workgroup barrier in the column loop
// (round 1's barrier-per-column form k_chol_backsolve was removed in round 6):
//   * wave 0 walks the chain: x_kt = M_kt^T r_kt, publishes x (LDS counter xcnt), then at once forms the
//     contribution of x_kt to the NEXT column's right-hand side (L_kt,next^T x_kt, in registers), so
//     the next solve waits only for the older contributions;
//   * the BS_HELPERS other waves own the right-hand-side tiles (tile j -> helper j % BS_HELPERS) and
//     apply every other update r_j -= L_kt,j^T x_kt, walking a host-built task list (position, tile) in
//     column order with the L tiles of the next two tasks in flight, and publish their progress
//     (prog[w] = first column not yet done);
//   * before solving position q the chain wave waits until the owner of its tile has finished the
//     columns up to q-2 (column q-1's part is the lookahead).
// Each r_j is summed in a fixed order (owner's columns in order, then the lookahead): deterministic.
// A loader wave streams each position's M and lookahead L blocks into an LDS ring up to 3 positions
// ahead, so the chain wave issues no global loads.
// la_tasks = [lookahead tile per position (-1: none) | task offsets per (chain, helper) | tasks q<<16|j].
__global__ __launch_bounds__(64 * (BS_HELPERS + 1 + BS_LOADERS)) void k_chol_backsolve_la(
    const double* __restrict__ L, int64_t ld, int n, const int* __restrict__ chain_off,
    const int* __restrict__ chain_cols, const int* __restrict__ la_tasks, const double* __restrict__ Ldiag,
    const double* __restrict__ Minv, double* __restrict__ xout) {
  constexpr int NH = BS_HELPERS, RING = 3;
  extern __shared__ __attribute__((aligned(16))) double xv[];  // [ld] r / x | cols [nq] | la [nq] | tasks (int)
  __shared__ int s_xcnt, s_prog[NH], s_toff[NH + 1], s_ready[RING], s_cdone;  // s_ready: per ring slot, position + 1
  __shared__ double s_ring[RING][2][NB * NB];  // M_kt | L_kt,next of the chain's coming positions
  const int nq = chain_off[gridDim.x];
  const int* toff_g = la_tasks + nq;
  const int* task_g = toff_g + gridDim.x * NH + 1;
  int* s_cc = reinterpret_cast<int*>(xv + ld);
  int* s_la = s_cc + nq;
  int* s_task = s_la + nq;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c = lane & 31, h = lane >> 5;  // column of the tile, row half
#ifdef BS_TIMING
  if (t == 0) g_bs_edges[blockIdx.x & 1][0] = clock64();
#define BSL_STAMP(q, k) do { if (t == 0 && (q) - q0 < 128) g_bs_stamps[blockIdx.x & 1][(q) - q0][k] = clock64(); } while (0)
#else
#define BSL_STAMP(q, k) do { } while (0)
#endif
  const int tn = n / NB, rn = n - tn * NB;
  const int q0 = chain_off[blockIdx.x], q1 = chain_off[blockIdx.x + 1];
  const int tb = toff_g[blockIdx.x * NH], te = toff_g[blockIdx.x * NH + NH];
  for (int i = t; i < ld; i += blockDim.x)
    xv[i] = (i >= n) ? 0.0 : (i < tn * NB ? L[(int64_t)n * ld + i] : Ldiag[((int64_t)tn * NB + rn) * NB + (i - tn * NB)]);
  for (int i = t; i < nq; i += blockDim.x) {
    s_cc[i] = chain_cols[i];
    s_la[i] = la_tasks[i];
  }
  for (int i = t; i < te - tb; i += blockDim.x) s_task[i] = task_g[tb + i];
  if (t <= NH) s_toff[t] = toff_g[blockIdx.x * NH + t] - tb;
  if (t == 0) {
    s_xcnt = q0;
    for (int k = 0; k < RING; ++k) s_ready[k] = q0;
    s_cdone = q0;
  }
  if (t < NH) {  // columns before a helper's first task are trivially done
    const int k0 = toff_g[blockIdx.x * NH + t], k1 = toff_g[blockIdx.x * NH + t + 1];
    s_prog[t] = k0 < k1 ? (task_g[k0] >> 16) : q1;
  }
  __syncthreads();
#ifdef BS_TIMING
  if (t == 0) g_bs_edges[blockIdx.x & 1][1] = clock64();
#endif
  if (wv == 0) {
    double la_c = 0.0;  // lookahead contribution to the current tile's r (column c)
    for (int q = q0; q < q1; ++q) {
      const int kt = s_cc[q];
      const int64_t c0 = (int64_t)kt * NB;
      const double* sm = s_ring[(q - q0) % RING][0];
      const double* sl = s_ring[(q - q0) % RING][1];
      BSL_STAMP(q, 0);
      // this position's M and L blocks from the ring into registers first: the reads overlap the wait
      // for the owner of the tile
      lds_wait_ge(&s_ready[(q - q0) % RING], q + 1, 0);
      BSL_STAMP(q, 1);
      double mv[NB / 2], lv[NB / 2];
#pragma unroll
      for (int i = 0; i < NB / 2; ++i) {
        mv[i] = sm[(h * (NB / 2) + i) * NB + c];
        lv[i] = sl[(h * (NB / 2) + i) * NB + c];
      }
      lds_wait_ge(&s_prog[kt % NH], q - 1, 0);
      BSL_STAMP(q, 2);
      const double r = xv[c0 + c] - la_c;
      if (h == 0) xv[c0 + c] = r;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      double s4[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < NB / 2; ++i)
        s4[i & 3] = fma(mv[i], xv[c0 + h * (NB / 2) + i], s4[i & 3]);
      double xs = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      xs += __shfl_xor(xs, 32, WAVE);
      if (h == 0) {
        xv[c0 + c] = xs;
        if (c0 + c < n) xout[c0 + c] = xs;
      }
      lds_signal(&s_xcnt, q + 1);
      BSL_STAMP(q, 3);
      la_c = 0.0;
      if (s_la[q] >= 0) {
        double u4[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < NB / 2; ++i)
          u4[i & 3] = fma(lv[i], xv[c0 + h * (NB / 2) + i], u4[i & 3]);
        la_c = (u4[0] + u4[1]) + (u4[2] + u4[3]);
        la_c += __shfl_xor(la_c, 32, WAVE);
      }
      lds_signal(&s_cdone, q + 1);  // ring slot free
      BSL_STAMP(q, 4);
    }
#ifdef BS_TIMING
    if (t == 0) g_bs_edges[blockIdx.x & 1][2] = clock64();
#endif
  } else if (wv >= NH + 1) {
    // loaders: M_kt and L_kt,next of position q into ring slot (q - q0) % RING, up to RING positions ahead;
    // BS_LOADERS waves take turns by position, so one loader's memory round trip overlaps the other's
    for (int q = q0 + (wv - NH - 1); q < q1; q += BS_LOADERS) {
      lds_wait_ge(&s_cdone, q - RING + 1, 1);
      const int kt = s_cc[q], la = max(s_la[q], 0);
      double vm[NB * NB / WAVE], vl[NB * NB / WAVE];
#pragma unroll
      for (int i = 0; i < NB * NB / WAVE; ++i) {
        const int e = lane + WAVE * i;
        vm[i] = Minv[(int64_t)kt * NB * NB + e];
        vl[i] = L[((int64_t)kt * NB + (e >> 5)) * ld + (int64_t)la * NB + (e & 31)];
      }
      double* sm = s_ring[(q - q0) % RING][0];
      double* sl = s_ring[(q - q0) % RING][1];
#pragma unroll
      for (int i = 0; i < NB * NB / WAVE; ++i) {
        sm[lane + WAVE * i] = vm[i];
        sl[lane + WAVE * i] = vl[i];
      }
      lds_signal(&s_ready[(q - q0) % RING], q + 1);
    }
  } else {
    const int me = wv - 1, k0 = s_toff[me], k1 = s_toff[me + 1];
    if (k0 < k1) {
      double tA[NB / 2], tB[NB / 2];
      auto fetch = [&](int k, double (&lt)[NB / 2]) {  // L_kt,j of task k (clamped)
        const int tk = s_task[min(k, k1 - 1)], kt = s_cc[tk >> 16], j = tk & 0xffff;
        const double* lp = L + ((int64_t)kt * NB + h * (NB / 2)) * ld + (int64_t)j * NB + c;
#pragma unroll
        for (int i = 0; i < NB / 2; ++i) lt[i] = lp[(int64_t)i * ld];
      };
      auto run = [&](int k, const double (&lt)[NB / 2]) {
        const int tk = s_task[k], q = tk >> 16, j = tk & 0xffff;
        const int64_t c0 = (int64_t)s_cc[q] * NB;
        lds_wait_ge(&s_xcnt, q + 1, 1);
        double s4[4] = {0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < NB / 2; ++i) s4[i & 3] = fma(lt[i], xv[c0 + h * (NB / 2) + i], s4[i & 3]);
        double sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        sacc += __shfl_xor(sacc, 32, WAVE);
        if (h == 0) xv[(int64_t)j * NB + c] -= sacc;
        const int qn = k + 1 < k1 ? (s_task[k + 1] >> 16) : q1;
        if (qn > q) {
          lds_signal(&s_prog[me], qn);
        }
      };
      fetch(k0, tA);
      for (int k = k0; k < k1; k += 2) {
        fetch(k + 1, tB);
        run(k, tA);
        if (k + 1 >= k1) break;
        fetch(k + 2, tA);
        run(k + 1, tB);
      }
    }
  }
}

// Left-looking back substitution for systems whose update lists do not fit the lookahead kernel's LDS
// (multi-row keyframe grids: thousands of frames, a coupling band of ~60 tiles).  One 1024-thread
// workgroup per chain; x (init y) stays in LDS, the lists come from global memory.  Per chain position
// (column kt, descending): r_kt = y_kt - sum_i L_i,kt^T x_i over the already-solved row tiles i coupled
// to kt (lo_off / lo_tiles: host-built, ascending i) -- wave w takes tiles w, w + 16, ..., lane =
// (column c, row half h), 16 independent loads per tile; the per-wave partials are summed in a fixed
// order (deterministic) and wave 0 solves x_kt = M_kt^T r_kt.
constexpr int BSL_WAVES = 16;
__global__ __launch_bounds__(64 * BSL_WAVES) void k_chol_backsolve_ll(
    const double* __restrict__ L, int64_t ld, int n, const int* __restrict__ chain_off,
    const int* __restrict__ chain_cols, const int* __restrict__ lo_off, const int* __restrict__ lo_tiles,
    const double* __restrict__ Ldiag, const double* __restrict__ Minv, double* __restrict__ xout) {
  extern __shared__ __attribute__((aligned(16))) double xv[];  // [ld]
  __shared__ double red[BSL_WAVES][NB];
  __shared__ double rk[NB];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int c = lane & 31, h = lane >> 5;
  const int tn = n / NB, rn = n - tn * NB;
  for (int i = t; i < ld; i += blockDim.x)
    xv[i] = (i >= n) ? 0.0 : (i < tn * NB ? L[(int64_t)n * ld + i] : Ldiag[((int64_t)tn * NB + rn) * NB + (i - tn * NB)]);
  __syncthreads();
  const int q0 = chain_off[blockIdx.x], q1 = chain_off[blockIdx.x + 1];
  for (int q = q0; q < q1; ++q) {
    const int kt = chain_cols[q];
    const int64_t c0 = (int64_t)kt * NB;
    const int e0 = lo_off[q], e1 = lo_off[q + 1];
    double acc = 0.0;
    for (int e = e0 + wv; e < e1; e += 2 * BSL_WAVES) {
      const bool two = e + BSL_WAVES < e1;  // wave-uniform
      const int i0 = lo_tiles[e], i1 = lo_tiles[two ? e + BSL_WAVES : e];
      const double* p0 = L + ((int64_t)i0 * NB + h * (NB / 2)) * ld + c0 + c;
      const double* p1 = L + ((int64_t)i1 * NB + h * (NB / 2)) * ld + c0 + c;
      double a0[NB / 2], a1[NB / 2];
#pragma unroll
      for (int r = 0; r < NB / 2; ++r) a0[r] = p0[(int64_t)r * ld];
#pragma unroll
      for (int r = 0; r < NB / 2; ++r) a1[r] = p1[(int64_t)r * ld];
      const double* x0 = xv + (int64_t)i0 * NB + h * (NB / 2);
      const double* x1 = xv + (int64_t)i1 * NB + h * (NB / 2);
#pragma unroll
      for (int r = 0; r < NB / 2; ++r) acc = fma(a0[r], x0[r], acc);
      if (two) {
#pragma unroll
        for (int r = 0; r < NB / 2; ++r) acc = fma(a1[r], x1[r], acc);
      }
    }
    acc += __shfl_xor(acc, 32, WAVE);
    if (h == 0) red[wv][c] = acc;
    __syncthreads();
    if (wv == 0) {
      double s = 0.0;
#pragma unroll
      for (int w = 0; w < BSL_WAVES; ++w) s += red[w][c];
      if (h == 0) rk[c] = xv[c0 + c] - s;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      const double* m = Minv + (int64_t)kt * NB * NB + c;  // x_c = sum_k M[k][c] r_k
      double s4[4] = {0, 0, 0, 0};
#pragma unroll
      for (int k = 0; k < NB / 2; ++k) {
        const int kk = h * (NB / 2) + k;
        s4[k & 3] = fma(m[kk * NB], rk[kk], s4[k & 3]);
      }
      double x = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      x += __shfl_xor(x, 32, WAVE);
      if (h == 0) {
        xv[c0 + c] = x;
        if (c0 + c < n) xout[c0 + c] = x;
      }
    }
    __syncthreads();
  }
}

// Blocked right-looking back substitution for large systems (api.hip make_bs_steps).  The left-looking
// form above streams the whole factor through ONE CU per chain (config 4: 224 MB of L tiles, 2.4 ms); here
// every step is a launch of one workgroup per (block, target column t), so a step's L tiles are read by
// ~60-120 CUs at once.  Workgroup = BSB_P waves, wave k owns block column c_k:
//   * all of its tiles are requested up front: M_ck (= L_ck^-1, k_tile_inv), the intra-block tiles
//     L_cj,ck (j < k), the target tile L_ck,t, r_ck (or y_ck on its first touch) and, wave 0, r_t;
//   * the block solve runs down the waves: wave k waits for x_c0..x_c(k-1) (LDS counter, ordered
//     hand-off as everywhere in this file), r'_ck = r_ck - sum_j L_cj,ck^T x_cj (fixed order j), x_ck =
//     M_ck^T r'_ck, publishes x_ck; every workgroup of the step solves the block redundantly (~10 tiles
//     from L2) instead of paying a second launch;
//   * the target: r_t -= sum_k L_ck,t^T x_ck (fixed order k), a plain read-modify-write: no other task of
//     the step touches t and steps are stream-ordered, so every r_t is summed in a fixed order
//     (deterministic, no atomics).  The task flagged writer stores the block's x.
// Lane = (column c, row half h) of a tile, 16 strided loads per tile as in the left-looking form.
__global__ __launch_bounds__(64 * BSB_P) void k_chol_backsolve_blk(
    const double* __restrict__ L, int64_t ld, int n, const int4* __restrict__ tasks,
    const double* __restrict__ Ldiag, const double* __restrict__ Minv, double* __restrict__ r,
    double* __restrict__ xout) {
  __shared__ double xs[BSB_P][NB];  // x of the block columns
  __shared__ double rs[BSB_P][NB];  // r' of a block column (before M^T)
  __shared__ double ps[BSB_P][NB];  // the target's partial sums per block column
  __shared__ int s_cnt;             // block columns published
  const int lane = threadIdx.x & 63, k = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  if (threadIdx.x == 0) s_cnt = 0;
  // task record (3 int4, independent loads): block columns | {p, intra-block bits, first-touch bits} |
  // {target t (-1: none), flags: target bits per block column, 0x100 writer, 0x200 t's first touch}
  const int4 bc = tasks[3 * blockIdx.x], bm = tasks[3 * blockIdx.x + 1], tk = tasks[3 * blockIdx.x + 2];
  const int p = bm.x, imask = bm.y, ftouch = bm.z, t = tk.x, tmask = tk.y & 0xff;
  const bool writer = (tk.y & 0x100) != 0, tfirst = (tk.y & 0x200) != 0;
  const int64_t tnNB = (int64_t)(n / NB) * NB, rn = n - tnNB;
  auto yval = [&](int64_t i) -> double {  // forward-substitution result: the factor's augmented row
    return i < tnNB ? L[(int64_t)n * ld + i] : (i < n ? Ldiag[(tnNB + rn) * NB + (i - tnNB)] : 0.0);
  };
  const int ck = k == 0 ? bc.x : (k == 1 ? bc.y : (k == 2 ? bc.z : bc.w));
  const bool act = k < p;
  const int64_t cc = (int64_t)ck * NB;
  double m[NB / 2], lj[BSB_P - 1][NB / 2], lt[NB / 2], rk = 0.0, rt = 0.0;
  if (act) {
    const double* mp = Minv + cc * NB + (int64_t)(h * (NB / 2)) * NB + c;  // M[kk][c], kk = h * 16 + i
#pragma unroll
    for (int i = 0; i < NB / 2; ++i) m[i] = mp[i * NB];
#pragma unroll
    for (int j = 0; j < BSB_P - 1; ++j) {
      const int cj = j == 0 ? bc.x : (j == 1 ? bc.y : bc.z);
      if (j < k && ((imask >> (j * 4 + k)) & 1)) {
        const double* lp = L + ((int64_t)cj * NB + h * (NB / 2)) * ld + cc + c;
#pragma unroll
        for (int i = 0; i < NB / 2; ++i) lj[j][i] = lp[(int64_t)i * ld];
      }
    }
    if ((tmask >> k) & 1) {
      const double* lp = L + (cc + h * (NB / 2)) * ld + (int64_t)t * NB + c;
#pragma unroll
      for (int i = 0; i < NB / 2; ++i) lt[i] = lp[(int64_t)i * ld];
    }
    rk = ((ftouch >> k) & 1) ? yval(cc + c) : r[cc + c];
    if (k == 0 && t >= 0) rt = tfirst ? yval((int64_t)t * NB + c) : r[(int64_t)t * NB + c];
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): s_cnt's init (global loads stay in flight)
  __builtin_amdgcn_s_barrier();
  if (act) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < BSB_P - 1; ++j) {
      if (j < k) {
        lds_wait_ge(&s_cnt, j + 1, 0);
        if ((imask >> (j * 4 + k)) & 1) {
          double a4[4] = {0, 0, 0, 0};
#pragma unroll
          for (int i = 0; i < NB / 2; ++i) a4[i & 3] = fma(lj[j][i], xs[j][h * (NB / 2) + i], a4[i & 3]);
          s += (a4[0] + a4[1]) + (a4[2] + a4[3]);
        }
      }
    }
    s += __shfl_xor(s, 32, WAVE);
    if (h == 0) rs[k][c] = rk - s;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    double x4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NB / 2; ++i) x4[i & 3] = fma(m[i], rs[k][h * (NB / 2) + i], x4[i & 3]);
    double x = (x4[0] + x4[1]) + (x4[2] + x4[3]);
    x += __shfl_xor(x, 32, WAVE);
    if (h == 0) xs[k][c] = x;
    lds_signal(&s_cnt, k + 1);  // waits for this wave's LDS stores first
    if (writer && h == 0 && cc + c < n) xout[cc + c] = x;
    if ((tmask >> k) & 1) {
      double a4[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < NB / 2; ++i) a4[i & 3] = fma(lt[i], xs[k][h * (NB / 2) + i], a4[i & 3]);
      double a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      a += __shfl_xor(a, 32, WAVE);
      if (h == 0) ps[k][c] = a;
    }
  }
  __syncthreads();
  if (k == 0 && t >= 0 && h == 0) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < BSB_P; ++j)
      if ((tmask >> j) & 1) s += ps[j][c];
    r[(int64_t)t * NB + c] = rt - s;
  }
}

// Persistent form of the blocked back substitution: every step's tasks in ONE launch (blockIdx order = step order,
// all resident: <= 512 workgroups), the launch boundaries between steps replaced by per-column update counters.
// A task first requests every immutable operand it needs (M_ck, the intra-block L tiles, L_ck,t: written by the
// factorisation, a previous launch), then waits -- per block column the wave that owns it, for the target wave 0 --
// until the column's counter shows the updates of all earlier steps (counter >= epoch * tot[col] + expect), and only
// then loads r with sc1 loads.  The target's r_t is stored sc1 by wave 0 (the only wave that stores it), drained
// (vmcnt(0)), and lane 0 of that wave adds 1 to the target's counter (MI355X_MICROARCH.md, inter-workgroup hand-off
// table, first row).  The arithmetic and the summation order are k_chol_backsolve_blk's: bitwise the same x.
constexpr int BSP_SPIN = 1 << 22;  // polls before a wait gives up (err = 1): ~seconds, never a hang
__device__ __forceinline__ bool bsp_wait(const unsigned* c, unsigned target) {
  for (int k = 0; k < BSP_SPIN; ++k) {
    if ((int)(__hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - target) >= 0) return true;
    __builtin_amdgcn_s_sleep(1);
  }
  return false;
}
__global__ __launch_bounds__(64 * BSB_P) void k_chol_backsolve_pst(
    const double* __restrict__ L, int64_t ld, int n, const int4* __restrict__ tasks, const int4* __restrict__ expect,
    const double* __restrict__ Ldiag, const double* __restrict__ Minv, double* __restrict__ r, double* __restrict__ xout,
    unsigned* __restrict__ cnt, const int* __restrict__ tot, uint32_t epoch, int* __restrict__ err) {
  __shared__ double xs[BSB_P][NB];
  __shared__ double rs[BSB_P][NB];
  __shared__ double ps[BSB_P][NB];
  __shared__ int s_cnt;
  const int lane = threadIdx.x & 63, k = threadIdx.x >> 6, c = lane & 31, h = lane >> 5;
  if (threadIdx.x == 0) s_cnt = 0;
  const int4 bc = tasks[3 * blockIdx.x], bm = tasks[3 * blockIdx.x + 1], tk = tasks[3 * blockIdx.x + 2];
  const int4 ex = expect[2 * blockIdx.x], ex2 = expect[2 * blockIdx.x + 1];
  const int p = bm.x, imask = bm.y, ftouch = bm.z, t = tk.x, tmask = tk.y & 0xff;
  const bool writer = (tk.y & 0x100) != 0, tfirst = (tk.y & 0x200) != 0;
  const int64_t tnNB = (int64_t)(n / NB) * NB, rn = n - tnNB;
  auto yval = [&](int64_t i) -> double {
    return i < tnNB ? L[(int64_t)n * ld + i] : (i < n ? Ldiag[(tnNB + rn) * NB + (i - tnNB)] : 0.0);
  };
  const int ck = k == 0 ? bc.x : (k == 1 ? bc.y : (k == 2 ? bc.z : bc.w));
  const int eck = k == 0 ? ex.x : (k == 1 ? ex.y : (k == 2 ? ex.z : ex.w));
  const bool act = k < p;
  const int64_t cc = (int64_t)ck * NB;
  double m[NB / 2], lj[BSB_P - 1][NB / 2], lt[NB / 2], rk = 0.0, rt = 0.0;
  bool ok = true;
  if (act) {  // the immutable operands first: their latency overlaps the waits below
    const double* mp = Minv + cc * NB + (int64_t)(h * (NB / 2)) * NB + c;
#pragma unroll
    for (int i = 0; i < NB / 2; ++i) m[i] = mp[i * NB];
#pragma unroll
    for (int j = 0; j < BSB_P - 1; ++j) {
      const int cj = j == 0 ? bc.x : (j == 1 ? bc.y : bc.z);
      if (j < k && ((imask >> (j * 4 + k)) & 1)) {
        const double* lp = L + ((int64_t)cj * NB + h * (NB / 2)) * ld + cc + c;
#pragma unroll
        for (int i = 0; i < NB / 2; ++i) lj[j][i] = lp[(int64_t)i * ld];
      }
    }
    if ((tmask >> k) & 1) {
      const double* lp = L + (cc + h * (NB / 2)) * ld + (int64_t)t * NB + c;
#pragma unroll
      for (int i = 0; i < NB / 2; ++i) lt[i] = lp[(int64_t)i * ld];
    }
    if ((ftouch >> k) & 1) {
      rk = yval(cc + c);
    } else {
      ok = bsp_wait(cnt + ck, epoch * (unsigned)tot[ck] + (unsigned)eck);
      // acquire after the counter observation: the r load below cannot be reordered above the poll (by the compiler
      // or a later toolchain) and misses this CU's vector cache; the L2 is not written back by it
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      rk = __hip_atomic_load(r + cc + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (k == 0 && t >= 0) {
      if (tfirst) {
        rt = yval((int64_t)t * NB + c);
      } else {
        ok = bsp_wait(cnt + t, epoch * (unsigned)tot[t] + (unsigned)ex2.x) && ok;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // as above
        rt = __hip_atomic_load(r + (int64_t)t * NB + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!ok && lane == 0) __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // pinned host flag
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): s_cnt's init
  __builtin_amdgcn_s_barrier();
  if (act) {
    double s = 0.0;
#pragma unroll
    for (int j = 0; j < BSB_P - 1; ++j) {
      if (j < k) {
        lds_wait_ge(&s_cnt, j + 1, 0);
        if ((imask >> (j * 4 + k)) & 1) {
          double a4[4] = {0, 0, 0, 0};
#pragma unroll
          for (int i = 0; i < NB / 2; ++i) a4[i & 3] = fma(lj[j][i], xs[j][h * (NB / 2) + i], a4[i & 3]);
          s += (a4[0] + a4[1]) + (a4[2] + a4[3]);
        }
      }
    }
    s += __shfl_xor(s, 32, WAVE);
    if (h == 0) rs[k][c] = rk - s;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    double x4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < NB / 2; ++i) x4[i & 3] = fma(m[i], rs[k][h * (NB / 2) + i], x4[i & 3]);
    double x = (x4[0] + x4[1]) + (x4[2] + x4[3]);
    x += __shfl_xor(x, 32, WAVE);
    if (h == 0) xs[k][c] = x;
    lds_signal(&s_cnt, k + 1);
    if (writer && h == 0 && cc + c < n) xout[cc + c] = x;
    if ((tmask >> k) & 1) {
      double a4[4] = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < NB / 2; ++i) a4[i & 3] = fma(lt[i], xs[k][h * (NB / 2) + i], a4[i & 3]);
      double a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      a += __shfl_xor(a, 32, WAVE);
      if (h == 0) ps[k][c] = a;
    }
  }
  __syncthreads();
  if (k == 0 && t >= 0) {
    if (h == 0) {
      double sum = 0.0;
#pragma unroll
      for (int j = 0; j < BSB_P; ++j)
        if ((tmask >> j) & 1) sum += ps[j][c];
      __hip_atomic_store(r + (int64_t)t * NB + c, rt - sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // wave 0's r_t stores have landed (write-through, sc1) before the counter add; the asm's memory clobber keeps the
    // compiler from moving the add above the stores.  No agent-scope release: it would write back this XCD's L2
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(cnt + t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

__global__ void k_tile_inv_list(const double* __restrict__ Ldiag, double* __restrict__ Minv,
                                const int* __restrict__ tiles);
void launch_chol_backsolve_pst(const double* L, int64_t ld, int n, const int4* tasks, const int4* expect, int n_tasks,
                               const double* Ldiag, double* Minv, double* r, double* xout, unsigned* cnt,
                               const int* tot, uint32_t epoch, int* err, hipStream_t st, const int* tinv_list,
                               int n_tinv) {
  if (n_tinv > 0) hipLaunchKernelGGL(k_tile_inv_list, dim3(n_tinv), dim3(64), 0, st, Ldiag, Minv, tinv_list);
  if (n_tasks > 0)
    hipLaunchKernelGGL(k_chol_backsolve_pst, dim3(n_tasks), dim3(64 * BSB_P), 0, st, L, ld, n, tasks, expect, Ldiag,
                       Minv, r, xout, cnt, tot, epoch, err);
}
void launch_chol_backsolve_blk(const double* L, int64_t ld, int n, const int4* tasks, const int* step_off_host,
                               int n_steps, const double* Ldiag, double* Minv, double* r, double* xout,
                               hipStream_t st, const int* tinv_list, int n_tinv) {
  if (n_tinv > 0) hipLaunchKernelGGL(k_tile_inv_list, dim3(n_tinv), dim3(64), 0, st, Ldiag, Minv, tinv_list);
  for (int s = 0; s < n_steps; ++s) {
    const int t0 = step_off_host[s], nt = step_off_host[s + 1] - t0;
    if (nt > 0)
      hipLaunchKernelGGL(k_chol_backsolve_blk, dim3(nt), dim3(64 * BSB_P), 0, st, L, ld, n, tasks + 3 * t0, Ldiag,
                         Minv, r, xout);
  }
}

#ifdef CS_TIMING
extern "C" int ptzba_debug_cs_stamps(long long* out) {
  const int zero = 0;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cs_stamps), sizeof(g_cs_stamps)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 64 * 6, HIP_SYMBOL(g_cs_wg), sizeof(g_cs_wg)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 64 * 16, HIP_SYMBOL(g_cs_blk), sizeof(g_cs_blk)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 64 * 16 + 64 * 64, HIP_SYMBOL(g_cs_hlp), sizeof(g_cs_hlp)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 64 * 16 + 64 * 64 + 64 * 24, HIP_SYMBOL(g_cs_rt), sizeof(g_cs_rt)) != hipSuccess) return -1;
  static long long zero_rt[64][4];
  if (hipMemcpyToSymbol(HIP_SYMBOL(g_cs_rt), zero_rt, sizeof(zero_rt)) != hipSuccess) return -1;
  return hipMemcpyToSymbol(HIP_SYMBOL(g_cs_level), &zero, sizeof(int)) == hipSuccess ? 0 : -1;
}
#endif
#ifdef BS_TIMING
extern "C" int ptzba_debug_bs_stamps(long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bs_stamps), sizeof(g_bs_stamps)) != hipSuccess) return -1;
  return hipMemcpyFromSymbol(out + 2 * 128 * 6, HIP_SYMBOL(g_bs_edges), sizeof(g_bs_edges)) == hipSuccess ? 0 : -1;
}
#endif

// the diagonal tiles listed in `tiles` (the last elimination level's; the others were inverted by type-2
// tasks of the level launches)
__global__ __launch_bounds__(64) void k_tile_inv_list(const double* __restrict__ Ldiag, double* __restrict__ Minv,
                                                      const int* __restrict__ tiles) {
  __shared__ double Lt[NB][NB + 1];
  __shared__ double rinv[NB];
  const int kt = tiles[blockIdx.x];
  tile_inv_wave(Ldiag + (int64_t)kt * NB * NB, Minv + (int64_t)kt * NB * NB, Lt, rinv);
}

void launch_chol_backsolve(const double* L, int64_t ld, int n, int n_chain, int n_pos, const int* chain_off,
                           const int* chain_cols, const int* upd_off, const int* upd_tiles, int n_upd,
                           const int* la_tasks, int n_tasks, const double* Ldiag, double* Minv, double* xout,
                           const int* lo_off, const int* lo_tiles, hipStream_t st, const int* tinv_list,
                           int n_tinv) {
  const int tx = (n + NB - 1) / NB;
  if (tinv_list) {
    if (n_tinv > 0) hipLaunchKernelGGL(k_tile_inv_list, dim3(n_tinv), dim3(64), 0, st, Ldiag, Minv, tinv_list);
  } else {
    hipLaunchKernelGGL(k_tile_inv, dim3(tx), dim3(64), 0, st, Ldiag, Minv);
  }
  if (lo_off) {  // large systems: left-looking form (api.hip chooses it when the lookahead lists exceed LDS)
    hipLaunchKernelGGL(k_chol_backsolve_ll, dim3(n_chain), dim3(64 * BSL_WAVES), (size_t)ld * sizeof(double), st, L,
                       ld, n, chain_off, chain_cols, lo_off, lo_tiles, Ldiag, Minv, xout);
    return;
  }
  const size_t lds = (size_t)ld * sizeof(double) + (size_t)(2 * n_pos + n_tasks) * sizeof(int);
  hipLaunchKernelGGL(k_chol_backsolve_la, dim3(n_chain), dim3(64 * (BS_HELPERS + 1 + BS_LOADERS)), lds, st, L, ld, n, chain_off,
                     chain_cols, la_tasks, Ldiag, Minv, xout);
}

// packed exchange: the lower tiles the Schur kernel can write (xt[k] = (ti, tj)) and the three
// length-ld vectors b | g_pose | dU, copied between the system matrix and a contiguous buffer
// (unpack != 0: buffer -> matrix).  Block k < n_tiles moves tile k; the last block moves the vectors.
__global__ void k_pack_exchange(double* __restrict__ S, int64_t ld, const int2* __restrict__ xt, int n_tiles,
                                double* __restrict__ vec, double* __restrict__ buf, int unpack) {
  const int k = blockIdx.x;
  if (k < n_tiles) {
    const int2 t = xt[k];
    double* tile = S + (int64_t)t.x * NB * ld + (int64_t)t.y * NB;
    double* b = buf + (int64_t)k * NB * NB;
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
      double* m = tile + (int64_t)(e >> 5) * ld + (e & 31);
      if (unpack) *m = b[e];
      else b[e] = *m;
    }
    return;
  }
  double* b = buf + (int64_t)n_tiles * NB * NB;
  for (int64_t e = threadIdx.x; e < 3 * ld; e += blockDim.x) {
    if (unpack) vec[e] = b[e];
    else b[e] = vec[e];
  }
}

// zero the listed 32x32 tiles of S (block k < n_tiles) and n_vec doubles at vec (last block)
__global__ __launch_bounds__(256) void k_zero_tiles(double* __restrict__ S, int64_t ld, const int2* __restrict__ zt,
                                                    int n_tiles, double* __restrict__ vec, int64_t n_vec) {
  if ((int)blockIdx.x < n_tiles) {
    const int2 tij = zt[blockIdx.x];
    double* T = S + (int64_t)tij.x * NB * ld + (int64_t)tij.y * NB;
    for (int e = threadIdx.x; e < NB * NB / 2; e += blockDim.x)
      *reinterpret_cast<double2*>(T + (int64_t)(e >> 4) * ld + 2 * (e & 15)) = make_double2(0.0, 0.0);
  } else {
    for (int64_t e = threadIdx.x; e < n_vec; e += blockDim.x) vec[e] = 0.0;
  }
}
void launch_zero_tiles(double* S, int64_t ld, const int2* zt, int n_tiles, double* vec, int64_t n_vec, hipStream_t st) {
  hipLaunchKernelGGL(k_zero_tiles, dim3(n_tiles + 1), dim3(256), 0, st, S, ld, zt, n_tiles, vec, n_vec);
}

void launch_pack_exchange(double* S, int64_t ld, const int2* xt, int n_tiles, double* vec, double* buf, int unpack,
                          hipStream_t st) {
  hipLaunchKernelGGL(k_pack_exchange, dim3(n_tiles + 1), dim3(256), 0, st, S, ld, xt, n_tiles, vec, buf, unpack);
}

// part-owned exchanges: a tile list and up to three vector ranges (offsets into vec) moved between the
// system and a contiguous buffer.  mode 0: pack, 1: unpack, 2: pack zeros (a group's non-leader ranks take
// part in the separator sum with nothing: their leader already contributes the group's values).
__global__ void k_pack_region(double* __restrict__ S, int64_t ld, const int2* __restrict__ xt, int n_tiles,
                              double* __restrict__ vec, VecRanges vr, double* __restrict__ buf, int mode) {
  const int k = blockIdx.x;
  if (k < n_tiles) {
    const int2 t = xt[k];
    double* tile = S + (int64_t)t.x * NB * ld + (int64_t)t.y * NB;
    double* b = buf + (int64_t)k * NB * NB;
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
      double* m = tile + (int64_t)(e >> 5) * ld + (e & 31);
      if (mode == 1) *m = b[e];
      else b[e] = mode == 2 ? 0.0 : *m;
    }
    return;
  }
  double* b = buf + (int64_t)n_tiles * NB * NB;
  for (int q = 0; q < vr.n; ++q) {
    for (int64_t e = threadIdx.x; e < vr.count[q]; e += blockDim.x) {
      double* m = vec + vr.off[q] + e;
      if (mode == 1) *m = b[e];
      else b[e] = mode == 2 ? 0.0 : *m;
    }
    b += vr.count[q];
  }
}

void launch_pack_region(double* S, int64_t ld, const int2* xt, int n_tiles, double* vec, const VecRanges& vr,
                        double* buf, int mode, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_region, dim3(n_tiles + 1), dim3(256), 0, st, S, ld, xt, n_tiles, vec, vr, buf, mode);
}

}  // namespace ptzba
