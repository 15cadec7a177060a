// Microbenchmark: 32x32 fp64 tile Cholesky (potrf) and triangular solve (TRSM, X = T L^-T) variants
// for the fused k_chol_step.  Each workgroup (256 threads) repeats potrf+trsm REPS times on its own
// SPD tile; grid = many workgroups; reports us per (potrf, trsm) and checks results vs variant 0.
//   hipcc -O3 --offload-arch=gfx950 tools/potrf_bench.hip -o tools/potrf_bench && tools/potrf_bench
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int NB = 32, WAVE = 64, REPS = 16;

__device__ __forceinline__ double bcast(double v, int j) {
  int lo = __builtin_amdgcn_readlane(__double2loint(v), j);
  int hi = __builtin_amdgcn_readlane(__double2hiint(v), j);
  return __hiloint2double(hi, lo);
}

// ---- V0: rows in registers, pivot column by readlane (current library code)
__device__ void potrf_v0(double (*D)[NB + 1], double* rdg) {
  const int lane = threadIdx.x & 63;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = D[lane & 31][m];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double d = bcast(row[j], j);
    const double r = 1.0 / sqrt(d);
    if (lane == j) rdg[j] = r;
    const double li = row[j] / d;
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * bcast(row[j], m);
  }
  if (lane < NB) {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V1: readlanes of the whole pivot column first (distinct SGPRs), then the FMAs
__device__ void potrf_v1(double (*D)[NB + 1], double* rdg) {
  const int lane = threadIdx.x & 63;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = D[lane & 31][m];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    double c[NB];
#pragma unroll
    for (int m = j; m < NB; ++m) c[m] = bcast(row[j], m);
    const double d = c[j];
    const double r = 1.0 / sqrt(d);
    if (lane == j) rdg[j] = r;
    const double li = row[j] / d;
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * c[m];
  }
  if (lane < NB) {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V2: rows in registers, pivot column broadcast through LDS (uniform-address reads)
__device__ void potrf_v2(double (*D)[NB + 1], double* rdg, double* col) {
  const int lane = threadIdx.x & 63;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = D[lane & 31][m];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    if (lane < NB) col[lane] = row[j];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const double d = col[j];
    const double li = row[j] / d;
    if (lane == j) rdg[j] = 1.0 / sqrt(d);
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * col[m];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
  if (lane < NB) {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V3: two lanes per row (lane 2r: columns 0..15, lane 2r+1: columns 16..31), LDS broadcast
__device__ void potrf_v3(double (*D)[NB + 1], double* rdg, double* col) {
  const int lane = threadIdx.x & 63;
  const int r = lane >> 1, h = lane & 1;
  double row[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) row[m] = D[r][16 * h + m];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    // owner of column j publishes A_rj for its row
    if (h == (j >> 4)) col[r] = row[j & 15];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const double d = col[j];
    const double li = col[r] / d;
    if (lane == 2 * j) rdg[j] = 1.0 / sqrt(d);
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      const int gm = 16 * h + m;
      if (gm > j) row[m] -= li * col[gm];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  }
#pragma unroll
  for (int m = 0; m < 16; ++m) D[r][16 * h + m] = row[m];
}


__device__ __forceinline__ double rcp_nr(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = fma(r, fma(-d, r, 1.0), r);
  r = fma(r, fma(-d, r, 1.0), r);
  return r;
}
__device__ __forceinline__ double rsq_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * fma(-0.5 * d * y, y, 1.5);
  y = y * fma(-0.5 * d * y, y, 1.5);
  return y;
}

// ---- V8: fused potrf + TRSM on one wave: lanes 0..31 hold the rows of D, lanes 32..63 the rows of T.
// Right-looking step j: v[m] -= (v[j] / d_j) * A_mj (m > j) is the Cholesky update for D rows and the
// forward substitution for T rows alike.  Pivot column by readlane, fast rcp/rsq + Newton.
template <bool FAST>
__device__ void potrf_trsm_v8(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
  double rs[NB];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double d = bcast(row[j], j);
    const double inv = FAST ? rcp_nr(d) : 1.0 / d;
    rs[j] = FAST ? rsq_nr(d) : 1.0 / sqrt(d);
    const double li = row[j] * inv;
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * bcast(row[j], m);
  }
  // scale: L_ij = row_i[j] rs_j (j < i), rdg_j = rs_j; X_rj = x_j rs_j
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rs[m];
  if (lane < NB) rdg[lane] = 0;  // placeholder, rdg below
  if (lane == 0) {
#pragma unroll
    for (int m = 0; m < NB; ++m) rdg[m] = rs[m];
  }
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}


// ---- V10: fused potrf + TRSM with the pivot column broadcast through LDS, software-pipelined:
// in step j every lane first updates its element j+1, publishes it to colbuf[(j+1)&1], then does the
// rest of the step; step j+1 reads the column with wide uniform-address loads.  One scheduling
// barrier per step keeps the compiler from hoisting later steps' reads (register spills).
__device__ void potrf_trsm_v10(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg, double (*colbuf)[NB]) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
  if (!isT) colbuf[0][lane] = row[0];
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double* col = colbuf[j & 1];
    const double d = col[j];
    if (lane == 0) rdg[j] = rsq_nr(d);
    const double li = row[j] * rcp_nr(d);
    if (j + 1 < NB) {
      row[j + 1] -= li * col[j + 1];
      if (!isT) colbuf[(j + 1) & 1][lane] = row[j + 1];
    }
#pragma unroll
    for (int m = j + 2; m < NB; ++m) row[m] -= li * col[m];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V11: V8 (readlane broadcast) with rs kept in LDS
__device__ void potrf_trsm_v11(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const double d = bcast(row[j], j);
    if (lane == 0) rdg[j] = rsq_nr(d);
    const double li = row[j] * rcp_nr(d);
#pragma unroll
    for (int m = j + 1; m < NB; ++m) row[m] -= li * bcast(row[j], m);
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V12<B>: fused potrf + TRSM, pivots in blocks of B.  Inside a block the pivot column moves by readlane
// (B(B-1)/2 elements); after the block the D lanes publish their B block values to LDS once, and the
// trailing rank-B update of every row reads them with uniform-address (broadcast) 16-byte loads.
template <int B>
__device__ void potrf_trsm_v12(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg, double (*cb)[B]) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
#pragma unroll
  for (int kb = 0; kb < NB; kb += B) {
    double w[B];
#pragma unroll
    for (int j = kb; j < kb + B; ++j) {
      const double d = bcast(row[j], j);
      if (lane == 0) rdg[j] = rsq_nr(d);
      const double li = row[j] * rcp_nr(d);
      w[j - kb] = li;
#pragma unroll
      for (int m = j + 1; m < kb + B; ++m) row[m] -= li * bcast(row[j], m);
    }
    if (kb + B < NB) {
      if (!isT) {
#pragma unroll
        for (int k = 0; k < B; ++k) cb[lane][k] = row[kb + k];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int m = kb + B; m < NB; ++m) {
        double s = row[m];
#pragma unroll
        for (int k = 0; k < B; ++k) s -= w[k] * cb[m][k];
        row[m] = s;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V15<B, MC>: V12 with the trailing update software-pipelined in chunks of MC rows (the reads of chunk
// c+1 issue before the FMAs of chunk c) and a scheduling barrier per chunk (no hoisting, no spills).
template <int B, int MC>
__device__ void potrf_trsm_v15(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg, double (*cb)[B]) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
#pragma unroll
  for (int kb = 0; kb < NB; kb += B) {
    double w[B];
#pragma unroll
    for (int j = kb; j < kb + B; ++j) {
      const double d = bcast(row[j], j);
      if (lane == 0) rdg[j] = rsq_nr(d);
      const double li = row[j] * rcp_nr(d);
      w[j - kb] = li;
#pragma unroll
      for (int m = j + 1; m < kb + B; ++m) row[m] -= li * bcast(row[j], m);
    }
    if (kb + B < NB) {
      if (!isT) {
#pragma unroll
        for (int k = 0; k < B; ++k) cb[lane][k] = row[kb + k];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_sched_barrier(0);
      constexpr int M0 = 0;
      const int m0 = kb + B;
      double nxt[MC][B];
#pragma unroll
      for (int q = 0; q < MC; ++q)
#pragma unroll
        for (int k = 0; k < B; ++k) nxt[q][k] = (m0 + q < NB) ? cb[m0 + q][k] : 0.0;
#pragma unroll
      for (int mc = m0; mc < NB; mc += MC) {
        double cur[MC][B];
#pragma unroll
        for (int q = 0; q < MC; ++q)
#pragma unroll
          for (int k = 0; k < B; ++k) cur[q][k] = nxt[q][k];
        if (mc + MC < NB) {
#pragma unroll
          for (int q = 0; q < MC; ++q)
#pragma unroll
            for (int k = 0; k < B; ++k) nxt[q][k] = (mc + MC + q < NB) ? cb[mc + MC + q][k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < MC; ++q) {
          if (mc + q < NB) {
            double s = row[mc + q];
#pragma unroll
            for (int k = 0; k < B; ++k) s -= w[k] * cur[q][k];
            row[mc + q] = s;
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      (void)M0;
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- V19<B, MC>: V15 with every updated row value pinned by an empty asm (the FMAs otherwise float past
// the scheduling barriers in the DAG and keep every LDS operand live: spills).
template <int B, int MC>
__device__ void potrf_trsm_v19(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg, double (*cb)[B]) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
#pragma unroll
  for (int kb = 0; kb < NB; kb += B) {
    double w[B];
#pragma unroll
    for (int j = kb; j < kb + B; ++j) {
      const double d = bcast(row[j], j);
      if (lane == 0) rdg[j] = rsq_nr(d);
      const double li = row[j] * rcp_nr(d);
      w[j - kb] = li;
#pragma unroll
      for (int m = j + 1; m < kb + B; ++m) row[m] -= li * bcast(row[j], m);
    }
    if (kb + B < NB) {
      if (!isT) {
#pragma unroll
        for (int k = 0; k < B; ++k) cb[lane][k] = row[kb + k];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      const int m0 = kb + B;
      double nxt[MC][B];
#pragma unroll
      for (int q = 0; q < MC; ++q)
#pragma unroll
        for (int k = 0; k < B; ++k) nxt[q][k] = (m0 + q < NB) ? cb[m0 + q][k] : 0.0;
#pragma unroll
      for (int mc = m0; mc < NB; mc += MC) {
        double cur[MC][B];
#pragma unroll
        for (int q = 0; q < MC; ++q)
#pragma unroll
          for (int k = 0; k < B; ++k) cur[q][k] = nxt[q][k];
        if (mc + MC < NB) {
#pragma unroll
          for (int q = 0; q < MC; ++q)
#pragma unroll
            for (int k = 0; k < B; ++k) nxt[q][k] = (mc + MC + q < NB) ? cb[mc + MC + q][k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < MC; ++q) {
          if (mc + q < NB) {
            double s = row[mc + q];
#pragma unroll
            for (int k = 0; k < B; ++k) s -= w[k] * cur[q][k];
            row[mc + q] = s;
            asm volatile("" : "+v"(row[mc + q]));
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

template <int B, int MC>
__device__ void potrf_trsm_v24(double (*D)[NB + 1], double (*C)[NB + 1], double* rdg, double (*cb)[B]) {
  const int lane = threadIdx.x & 63;
  const bool isT = lane >= NB;
  double row[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] = isT ? C[lane - NB][m] : D[lane][m];
  double dm = 1.0;  // lane j keeps pivot d_j; the 32 rsq run once, vectorised, at the end
#pragma unroll
  for (int kb = 0; kb < NB; kb += B) {
    double w[B];
#pragma unroll
    for (int j = kb; j < kb + B; ++j) {
      const double d = bcast(row[j], j);
      dm = (lane == j) ? d : dm;
      const double li = row[j] * rcp_nr(d);
      w[j - kb] = li;
#pragma unroll
      for (int m = j + 1; m < kb + B; ++m) row[m] -= li * bcast(row[j], m);
    }
    if (kb + B < NB) {
      if (!isT) {
#pragma unroll
        for (int k = 0; k < B; ++k) cb[lane][k] = row[kb + k];
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
      const int m0 = kb + B;
      double nxt[MC][B];
#pragma unroll
      for (int q = 0; q < MC; ++q)
#pragma unroll
        for (int k = 0; k < B; ++k) nxt[q][k] = (m0 + q < NB) ? cb[m0 + q][k] : 0.0;
#pragma unroll
      for (int mc = m0; mc < NB; mc += MC) {
        double cur[MC][B];
#pragma unroll
        for (int q = 0; q < MC; ++q)
#pragma unroll
          for (int k = 0; k < B; ++k) cur[q][k] = nxt[q][k];
        if (mc + MC < NB) {
#pragma unroll
          for (int q = 0; q < MC; ++q)
#pragma unroll
            for (int k = 0; k < B; ++k) nxt[q][k] = (mc + MC + q < NB) ? cb[mc + MC + q][k] : 0.0;
        }
#pragma unroll
        for (int q = 0; q < MC; ++q) {
          if (mc + q < NB) {
            double s = row[mc + q];
#pragma unroll
            for (int k = 0; k < B; ++k) s -= w[k] * cur[q][k];
            row[mc + q] = s;
            asm volatile("" : "+v"(row[mc + q]));
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);
      __builtin_amdgcn_wave_barrier();
    }
  }
  if (lane < NB) rdg[lane] = rsq_nr(dm);
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int m = 0; m < NB; ++m) row[m] *= rdg[m];
  if (isT) {
#pragma unroll
    for (int m = 0; m < NB; ++m) C[lane - NB][m] = row[m];
  } else {
#pragma unroll
    for (int m = 0; m < NB; ++m) D[lane][m] = row[m];
  }
}

// ---- TRSM variants: X = T L^-T with L = D (scaled on the fly: L_mj = D[m][j] * rdg[j] for m > j, L_jj = 1/rdg)
// T0: lane per row, sched_barrier per step (library)
__device__ void trsm_t0(double (*C)[NB + 1], double (*D)[NB + 1], const double* rdg) {
  const int r = threadIdx.x;
  if (r >= NB) return;
  double x[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) x[m] = C[r][m];
#pragma unroll
  for (int jj = 0; jj < NB; ++jj) {
    x[jj] *= rdg[jj];
#pragma unroll
    for (int m = jj + 1; m < NB; ++m) x[m] -= x[jj] * D[m][jj];
    __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m) C[r][m] = x[m];
}

// T1: lane per row, no scheduling barrier (compiler free to pipeline LDS reads)
__device__ void trsm_t1(double (*C)[NB + 1], double (*D)[NB + 1], const double* rdg) {
  const int r = threadIdx.x;
  if (r >= NB) return;
  double x[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) x[m] = C[r][m];
#pragma unroll
  for (int jj = 0; jj < NB; ++jj) {
    x[jj] *= rdg[jj];
#pragma unroll
    for (int m = jj + 1; m < NB; ++m) x[m] -= x[jj] * D[m][jj];
    if ((jj & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m) C[r][m] = x[m];
}

// T2: 4 waves, 8 lanes per row?  -> instead: 2 waves x 32 lanes, each wave half the rows, D transposed
// in LDS (Dt[jj][m]) so the per-step column is a contiguous, vectorisable read
__device__ void trsm_t2(double (*C)[NB + 1], double (*Dt)[NB + 1], const double* rdg) {
  const int r = threadIdx.x;
  if (r >= NB) return;
  double x[NB];
#pragma unroll
  for (int m = 0; m < NB; ++m) x[m] = C[r][m];
#pragma unroll
  for (int jj = 0; jj < NB; ++jj) {
    x[jj] *= rdg[jj];
#pragma unroll
    for (int m = jj + 1; m < NB; ++m) x[m] -= x[jj] * Dt[jj][m];
    if ((jj & 3) == 3) __builtin_amdgcn_sched_barrier(0);
  }
#pragma unroll
  for (int m = 0; m < NB; ++m) C[r][m] = x[m];
}

template <int PV, int TV>
__global__ __launch_bounds__(256) void k_bench(const double* __restrict__ A, const double* __restrict__ T,
                                               double* __restrict__ L, double* __restrict__ X) {
  __shared__ double sD[NB][NB + 1];
  __shared__ double sDt[NB][NB + 1];
  __shared__ double sC[NB][NB + 1];
  __shared__ double rdg[NB];
  __shared__ double col[NB];
  __shared__ double colbuf[2][NB];
  __shared__ __attribute__((aligned(16))) double cb4[NB][4];
  __shared__ __attribute__((aligned(16))) double cb8[NB][8];
  const double* a = A + (size_t)blockIdx.x * NB * NB;
  const double* t = T + (size_t)blockIdx.x * NB * NB;
  for (int rep = 0; rep < REPS; ++rep) {
    for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
      sD[e >> 5][e & 31] = a[e];
      sC[e >> 5][e & 31] = t[e];
    }
    __syncthreads();
    if (threadIdx.x < WAVE) {
      if (PV == 0) potrf_v0(sD, rdg);
      if (PV == 1) potrf_v1(sD, rdg);
      if (PV == 2) potrf_v2(sD, rdg, col);
      if (PV == 3) potrf_v3(sD, rdg, col);
      if (PV == 7) potrf_v0(sD, rdg);
      if (PV == 8) potrf_trsm_v8<true>(sD, sC, rdg);
      if (PV == 9) potrf_trsm_v8<false>(sD, sC, rdg);
      if (PV == 10) potrf_trsm_v10(sD, sC, rdg, colbuf);
      if (PV == 11) potrf_trsm_v11(sD, sC, rdg);
      if (PV == 12) potrf_trsm_v12<4>(sD, sC, rdg, cb4);
      if (PV == 13) potrf_trsm_v12<8>(sD, sC, rdg, cb8);
      if (PV == 14) potrf_trsm_v12<2>(sD, sC, rdg, (double(*)[2])cb4);
      if (PV == 15) potrf_trsm_v15<4, 4>(sD, sC, rdg, cb4);
      if (PV == 16) potrf_trsm_v15<8, 2>(sD, sC, rdg, cb8);
      if (PV == 17) potrf_trsm_v15<4, 2>(sD, sC, rdg, cb4);
      if (PV == 18) potrf_trsm_v15<2, 4>(sD, sC, rdg, (double(*)[2])cb4);
      if (PV == 19) potrf_trsm_v19<4, 4>(sD, sC, rdg, cb4);
      if (PV == 20) potrf_trsm_v19<8, 2>(sD, sC, rdg, cb8);
      if (PV == 21) potrf_trsm_v19<4, 2>(sD, sC, rdg, cb4);
      if (PV == 22) potrf_trsm_v19<8, 4>(sD, sC, rdg, cb8);
      if (PV == 23) potrf_trsm_v19<2, 4>(sD, sC, rdg, (double(*)[2])cb4);
      if (PV == 24) potrf_trsm_v24<4, 4>(sD, sC, rdg, cb4);
      if (PV == 25) potrf_trsm_v24<8, 2>(sD, sC, rdg, cb8);
      if (PV == 26) potrf_trsm_v24<8, 4>(sD, sC, rdg, cb8);
    }
    __syncthreads();
    if (TV == 2) {
      for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) sDt[e & 31][e >> 5] = sD[e >> 5][e & 31];
      __syncthreads();
    }
    if (TV == 0) trsm_t0(sC, sD, rdg);
    if (TV == 1) trsm_t1(sC, sD, rdg);
    if (TV == 2) trsm_t2(sC, sDt, rdg);
    __syncthreads();
  }
  double* l = L + (size_t)blockIdx.x * NB * NB;
  double* x = X + (size_t)blockIdx.x * NB * NB;
  for (int e = threadIdx.x; e < NB * NB; e += blockDim.x) {
    const int i = e >> 5, j = e & 31;
    if (PV >= 8) l[e] = (j < i) ? sD[i][j] : (j == i ? 1.0 / rdg[i] : 0.0);
    else l[e] = (j < i) ? sD[i][j] * rdg[j] : (j == i ? 1.0 / rdg[i] : 0.0);
    x[e] = sC[i][j];
  }
}

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

template <int PV, int TV>
double run(int nb, double* dA, double* dT, double* dL, double* dX, std::vector<double>& L, std::vector<double>& X) {
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  hipLaunchKernelGGL((k_bench<PV, TV>), dim3(nb), dim3(256), 0, 0, dA, dT, dL, dX);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(e0));
  for (int it = 0; it < 5; ++it) hipLaunchKernelGGL((k_bench<PV, TV>), dim3(nb), dim3(256), 0, 0, dA, dT, dL, dX);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  L.resize((size_t)nb * NB * NB);
  X.resize((size_t)nb * NB * NB);
  CK(hipMemcpy(L.data(), dL, L.size() * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(X.data(), dX, X.size() * 8, hipMemcpyDeviceToHost));
  return ms * 1e3 / 5 / REPS;  // us per (load + potrf + trsm), all workgroups concurrent
}

int main() {
  const int nb = 64;  // workgroups (one tile each) -> runs concurrently, time = per-tile latency
  std::vector<double> A((size_t)nb * NB * NB), T((size_t)nb * NB * NB);
  srand(1);
  for (int b = 0; b < nb; ++b) {
    std::vector<double> B(NB * NB);
    for (auto& x : B) x = (double)rand() / RAND_MAX - 0.5;
    for (int i = 0; i < NB; ++i)
      for (int j = 0; j < NB; ++j) {
        double s = (i == j) ? NB : 0.0;
        for (int k = 0; k < NB; ++k) s += B[i * NB + k] * B[j * NB + k];
        A[(size_t)b * NB * NB + i * NB + j] = s;
        T[(size_t)b * NB * NB + i * NB + j] = (double)rand() / RAND_MAX - 0.5;
      }
  }
  double *dA, *dT, *dL, *dX;
  CK(hipMalloc(&dA, A.size() * 8));
  CK(hipMalloc(&dT, T.size() * 8));
  CK(hipMalloc(&dL, A.size() * 8));
  CK(hipMalloc(&dX, A.size() * 8));
  CK(hipMemcpy(dA, A.data(), A.size() * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dT, T.data(), T.size() * 8, hipMemcpyHostToDevice));
  std::vector<double> L0, X0, L, X;
  auto cmp = [&](const char* name, double us) {
    double el = 0, ex = 0;
    for (size_t i = 0; i < L.size(); ++i) el = fmax(el, fabs(L[i] - L0[i]));
    // X vs a CPU forward substitution X L^T = T with the reference L0
    for (int b = 0; b < nb; ++b)
      for (int r = 0; r < NB; ++r) {
        double x[NB];
        for (int c = 0; c < NB; ++c) {
          double s = T[(size_t)b * NB * NB + r * NB + c];
          for (int m = 0; m < c; ++m) s -= x[m] * L0[(size_t)b * NB * NB + c * NB + m];
          x[c] = s / L0[(size_t)b * NB * NB + c * NB + c];
          ex = fmax(ex, fabs(x[c] - X[(size_t)b * NB * NB + r * NB + c]));
        }
      }
    printf("%-22s %8.3f us   max|dL| %.2e  max|dX| %.2e\n", name, us, el, ex);
  };
  double us = run<0, 0>(nb, dA, dT, dL, dX, L0, X0);
  L = L0; X = X0;
  cmp("potrf v0 + trsm t0", us);
  cmp("potrf v1 + trsm t0", run<1, 0>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v2 + trsm t0", run<2, 0>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v3 + trsm t0", run<3, 0>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v0 + trsm t1", run<0, 1>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v0 + trsm t2", run<0, 2>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v2 + trsm t1", run<2, 1>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v3 + trsm t2", run<3, 2>(nb, dA, dT, dL, dX, L, X));
  cmp("potrf v0 only (no trsm)", run<7, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("load only", run<6, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v8 fast rcp", run<8, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v9 ieee div", run<9, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v10 lds pipelined", run<10, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v11 readlane, rs in lds", run<11, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v12 blocked B=4", run<12, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v13 blocked B=8", run<13, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v14 blocked B=2", run<14, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v15 pipelined B=4 MC=4", run<15, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v16 pipelined B=8 MC=2", run<16, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v17 pipelined B=4 MC=2", run<17, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v18 pipelined B=2 MC=4", run<18, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v19 pinned B=4 MC=4", run<19, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v20 pinned B=8 MC=2", run<20, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v21 pinned B=4 MC=2", run<21, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v22 pinned B=8 MC=4", run<22, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v23 pinned B=2 MC=4", run<23, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v24 pinned+rsq end B=4 MC=4", run<24, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v25 pinned+rsq end B=8 MC=2", run<25, 9>(nb, dA, dT, dL, dX, L, X));
  cmp("fused v26 pinned+rsq end B=8 MC=4", run<26, 9>(nb, dA, dT, dL, dX, L, X));
  return 0;
}
