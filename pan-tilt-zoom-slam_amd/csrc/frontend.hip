// Feature front-end on the GPU: the matching half of image_process.match_sift_features
// (image_process.py:178-234) -- brute-force 2-nearest-neighbour search in L2 (cv.BFMatcher().knnMatch(k=2))
// and the homography RANSAC behind it (homography_ransac, image_process.py:418-441, cv.findHomography with
// RANSAC) -- pyramidal LK (optical_flow_matching, :393-415) and cross-checked Hamming matching (:237-310).
// SIFT detection is sift.hip.  Every entry point holds device_work_lock while it uses the per-device work
// buffers (host_util.h): thread-safe, serialised per device.
//
//   ptz_match_knn2         one 64x64 tile of squared L2 distances per workgroup (fp32, 4x4 outputs per
//                          thread, descriptors staged through LDS in k-chunks of 16), then one wave per query
//                          keeps the two nearest (distance, index), ties to the lower index.  For SIFT's
//                          integer-valued descriptors (0..255, 128-d) every partial sum is an exact fp32
//                          integer, so the distances equal any other summation order bit for bit.
//   ptz_homography_ransac  hypotheses from counter-keyed 4-point samples (the sampling stream is a function of
//                          (seed, hypothesis, draw) only), one lane per hypothesis solves the 8x8 DLT system
//                          (normalised coordinates, partial pivoting), a workgroup of 256 scores 64 hypotheses
//                          against every point, the best (most inliers, then lowest index) is kept with a 64-bit
//                          atomic max; one workgroup refits H by linear least squares on its inliers and writes
//                          the final mask.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/ptzba.h"
#include "host_util.h"
#include "ptzba_common.h"

namespace ptzba {

constexpr int KT = 64, KC = 16;  // distance tile, k-chunk

__global__ __launch_bounds__(256) void k_sqdist(int n1, int n2, int dim, const float* __restrict__ a,
                                                const float* __restrict__ b, float* __restrict__ d) {
  __shared__ float sa[KC][KT + 4], sb[KC][KT + 4];
  const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
  const int q0 = blockIdx.y * KT, j0 = blockIdx.x * KT;
  float acc[4][4] = {};
  for (int k0 = 0; k0 < dim; k0 += KC) {
#pragma unroll
    for (int p = 0; p < 4; ++p) {  // 64 rows x 16 dims each for a and b: 1024 values, 4 per thread
      const int e = t + 256 * p, r = e >> 4, k = e & 15;
      const int qa = q0 + r, jb = j0 + r, kk = k0 + k;
      sa[k][r] = (qa < n1 && kk < dim) ? a[(int64_t)qa * dim + kk] : 0.f;
      sb[k][r] = (jb < n2 && kk < dim) ? b[(int64_t)jb * dim + kk] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      float av[4], bv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        av[i] = sa[k][ty * 4 + i];
        bv[i] = sb[k][tx * 4 + i];
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float df = av[i] - bv[j];
          acc[i][j] = fmaf(df, df, acc[i][j]);
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int q = q0 + ty * 4 + i;
    if (q >= n1) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int jj = j0 + tx * 4 + j;
      if (jj < n2) d[(int64_t)q * n2 + jj] = acc[i][j];
    }
  }
}

// (d, idx) lexicographic: smaller distance first, then smaller index
__device__ __forceinline__ bool lt(float d1, int i1, float d2, int i2) { return d1 < d2 || (d1 == d2 && i1 < i2); }

__global__ __launch_bounds__(256) void k_top2(int n1, int n2, const float* __restrict__ d, int* __restrict__ idx,
                                              float* __restrict__ dist) {
  const int q = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (q >= n1) return;
  float b1 = INFINITY, b2 = INFINITY;
  int i1 = 0x7fffffff, i2 = 0x7fffffff;
  for (int j = lane; j < n2; j += 64) {
    const float v = d[(int64_t)q * n2 + j];
    if (lt(v, j, b1, i1)) {
      b2 = b1; i2 = i1; b1 = v; i1 = j;
    } else if (lt(v, j, b2, i2)) {
      b2 = v; i2 = j;
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const float ob1 = __shfl_xor(b1, off), ob2 = __shfl_xor(b2, off);
    const int oi1 = __shfl_xor(i1, off), oi2 = __shfl_xor(i2, off);
    // merge two sorted pairs {b1 <= b2}, {ob1 <= ob2}
    float n1v, n2v;
    int n1i, n2i;
    if (lt(b1, i1, ob1, oi1)) {
      n1v = b1; n1i = i1;
      if (lt(b2, i2, ob1, oi1)) { n2v = b2; n2i = i2; } else { n2v = ob1; n2i = oi1; }
    } else {
      n1v = ob1; n1i = oi1;
      if (lt(b1, i1, ob2, oi2)) { n2v = b1; n2i = i1; } else { n2v = ob2; n2i = oi2; }
    }
    b1 = n1v; i1 = n1i; b2 = n2v; i2 = n2i;
  }
  if (lane == 0) {
    idx[2 * q] = i1;
    idx[2 * q + 1] = n2 > 1 ? i2 : -1;
    dist[2 * q] = sqrtf(b1);
    dist[2 * q + 1] = n2 > 1 ? sqrtf(b2) : INFINITY;
  }
}

// kNN-2 on the matrix cores for integer-valued 128-d descriptors (SIFT's: integers 0..255): one workgroup per 64 query
// rows (a wave per 16), the train set streamed through LDS in tiles of 64 as f16 (exact: integers with 2 dim v^2 < 2^24, |v| <= 255 at 128-d), the
// dot products on v_mfma_f32_16x16x32_f16 (products exact, sums exact integers below 2^24), d^2 = |q|^2 + |t|^2 - 2 q.t
// exact -- the same integer k_sqdist's fp32 sum of (a - b)^2 gives -- and each lane keeps a running (distance, index)
// top 2 for its four rows over its columns (ascending), merged across the 16 lanes of a row at the end with k_top2's
// lexicographic rule: bit for bit k_sqdist + k_top2's output, without the n1 x n2 distance matrix.
typedef _Float16 kn_h8 __attribute__((ext_vector_type(8)));
typedef float kn_f4 __attribute__((ext_vector_type(4)));
constexpr int KN_DIM = 128, KN_TC = 64, KN_LD = KN_DIM + 8;  // train tile columns, f16 row pitch (272 B)
__global__ __launch_bounds__(256) void k_knn2_mf(int n1, int n2, const float* __restrict__ a, const float* __restrict__ b,
                                                 int* __restrict__ idx, float* __restrict__ dist) {
  __shared__ __attribute__((aligned(16))) _Float16 sb[KN_TC][KN_LD];
  __shared__ float snb[KN_TC];
  __shared__ float sna[4][16];
  const int t = threadIdx.x, w = t >> 6, lane = t & 63, fr = lane & 15, fk = (lane >> 4) * 8;
  const int q0 = blockIdx.x * 64 + 16 * w;
  // this wave's 16 query rows as MFMA A operands (row fr, dims 32 c + fk .. + 7) and their squared norms
  kn_h8 qa[KN_DIM / 32];
  {
    const int q = min(q0 + fr, n1 - 1);
    const float* src = a + (int64_t)q * KN_DIM;
#pragma unroll
    for (int c = 0; c < KN_DIM / 32; ++c) {
      const float4 u0 = reinterpret_cast<const float4*>(src + 32 * c + fk)[0];
      const float4 u1 = reinterpret_cast<const float4*>(src + 32 * c + fk)[1];
      qa[c] = kn_h8{(_Float16)u0.x, (_Float16)u0.y, (_Float16)u0.z, (_Float16)u0.w,
                    (_Float16)u1.x, (_Float16)u1.y, (_Float16)u1.z, (_Float16)u1.w};
    }
    if (lane < 16) {
      float s = 0.f;
      for (int k = 0; k < KN_DIM; ++k) s = fmaf(src[k], src[k], s);  // exact integer
      sna[w][fr] = s;
    }
  }
  float b1[4], b2[4];
  int i1[4], i2[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    b1[v] = b2[v] = INFINITY;
    i1[v] = i2[v] = 0x7fffffff;
  }
  for (int j0 = 0; j0 < n2; j0 += KN_TC) {
    __syncthreads();  // (the previous tile's reads are done)
    {  // stage 64 train rows as f16: thread = (row t >> 2, quarter t & 3 of the dims); their squared norms
      const int r = t >> 2, qd = (t & 3) * (KN_DIM / 4), j = j0 + r;
      float s = 0.f;
      const float* src = b + (int64_t)min(j, n2 - 1) * KN_DIM + qd;
#pragma unroll
      for (int k = 0; k < KN_DIM / 4; k += 4) {
        const float4 u = reinterpret_cast<const float4*>(src + k)[0];
        sb[r][qd + k] = (_Float16)u.x;
        sb[r][qd + k + 1] = (_Float16)u.y;
        sb[r][qd + k + 2] = (_Float16)u.z;
        sb[r][qd + k + 3] = (_Float16)u.w;
        s = fmaf(u.x, u.x, s);
        s = fmaf(u.y, u.y, s);
        s = fmaf(u.z, u.z, s);
        s = fmaf(u.w, u.w, s);
      }
      s += __shfl_xor(s, 1);
      s += __shfl_xor(s, 2);
      if ((t & 3) == 0) snb[r] = s;
    }
    __syncthreads();
#pragma unroll
    for (int y = 0; y < KN_TC / 16; ++y) {
      kn_f4 c = kn_f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kc = 0; kc < KN_DIM / 32; ++kc) {
        const kn_h8 bv = *reinterpret_cast<const kn_h8*>(&sb[16 * y + fr][32 * kc + fk]);
        c = __builtin_amdgcn_mfma_f32_16x16x32_f16(qa[kc], bv, c, 0, 0, 0);
      }
      const int jl = 16 * y + fr, j = j0 + jl;
      if (j >= n2) continue;
      const float nb = snb[jl];
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float d = (sna[w][(lane >> 4) * 4 + v] + nb) - 2.f * c[v];
        if (lt(d, j, b1[v], i1[v])) {
          b2[v] = b1[v]; i2[v] = i1[v]; b1[v] = d; i1[v] = j;
        } else if (lt(d, j, b2[v], i2[v])) {
          b2[v] = d; i2[v] = j;
        }
      }
    }
  }
  // merge the 16 lanes of each row group (lanes with the same lane >> 4): the k_top2 merge
#pragma unroll
  for (int v = 0; v < 4; ++v) {
#pragma unroll
    for (int off = 8; off > 0; off >>= 1) {
      const float ob1 = __shfl_xor(b1[v], off), ob2 = __shfl_xor(b2[v], off);
      const int oi1 = __shfl_xor(i1[v], off), oi2 = __shfl_xor(i2[v], off);
      float n1v, n2v;
      int n1i, n2i;
      if (lt(b1[v], i1[v], ob1, oi1)) {
        n1v = b1[v]; n1i = i1[v];
        if (lt(b2[v], i2[v], ob1, oi1)) { n2v = b2[v]; n2i = i2[v]; } else { n2v = ob1; n2i = oi1; }
      } else {
        n1v = ob1; n1i = oi1;
        if (lt(b1[v], i1[v], ob2, oi2)) { n2v = b1[v]; n2i = i1[v]; } else { n2v = ob2; n2i = oi2; }
      }
      b1[v] = n1v; i1[v] = n1i; b2[v] = n2v; i2[v] = n2i;
    }
    const int q = q0 + (lane >> 4) * 4 + v;
    if (fr == 0 && q < n1) {
      idx[2 * q] = i1[v];
      idx[2 * q + 1] = n2 > 1 ? i2[v] : -1;
      dist[2 * q] = sqrtf(b1[v]);
      dist[2 * q + 1] = n2 > 1 ? sqrtf(b2[v]) : INFINITY;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// homography RANSAC
// ---------------------------------------------------------------------------------------------
__device__ __host__ inline uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// draw k of hypothesis h: a function of (seed, h, k, attempt) only
__device__ __host__ inline uint32_t ransac_draw(uint64_t seed, uint32_t h, uint32_t k, uint32_t attempt, uint32_t n) {
  const uint64_t z = mix64(seed * 0x9E3779B97F4A7C15ull + ((uint64_t)h << 20) + ((uint64_t)attempt << 4) + k + 1);
  return (uint32_t)(z % n);
}

struct Norm {
  double c1x, c1y, s1, c2x, c2y, s2;  // p' = s (p - c)
};

// solve the 8x8 system M x = r (row-major M[8][9] augmented) by Gaussian elimination with partial
// pivoting; false if singular
__device__ __host__ inline bool solve8(double (&M)[8][9], double (&x)[8]) {
  for (int c = 0; c < 8; ++c) {
    int p = c;
    double best = fabs(M[c][c]);
    for (int r = c + 1; r < 8; ++r)
      if (fabs(M[r][c]) > best) { best = fabs(M[r][c]); p = r; }
    if (!(best > 1e-12)) return false;
    if (p != c)
      for (int k = 0; k < 9; ++k) { const double tmp = M[c][k]; M[c][k] = M[p][k]; M[p][k] = tmp; }
    const double inv = 1.0 / M[c][c];
    for (int r = c + 1; r < 8; ++r) {
      const double f = M[r][c] * inv;
      for (int k = c; k < 9; ++k) M[r][k] -= f * M[c][k];
    }
  }
  for (int c = 7; c >= 0; --c) {
    double s = M[c][8];
    for (int k = c + 1; k < 8; ++k) s -= M[c][k] * x[k];
    x[c] = s / M[c][c];
  }
  return true;
}

// the two DLT rows of one correspondence (h33 = 1) in normalised coordinates
__device__ __host__ inline void dlt_rows(double x, double y, double u, double v, double (&r0)[9], double (&r1)[9]) {
  r0[0] = x; r0[1] = y; r0[2] = 1; r0[3] = 0; r0[4] = 0; r0[5] = 0; r0[6] = -u * x; r0[7] = -u * y; r0[8] = u;
  r1[0] = 0; r1[1] = 0; r1[2] = 0; r1[3] = x; r1[4] = y; r1[5] = 1; r1[6] = -v * x; r1[7] = -v * y; r1[8] = v;
}

// H (pixel coordinates) from the normalised solution h: H = T2^-1 Hn T1
__device__ __host__ inline void denormalise(const double (&h)[8], const Norm& N, double (&H)[9]) {
  const double Hn[9] = {h[0], h[1], h[2], h[3], h[4], h[5], h[6], h[7], 1.0};
  // Hn T1: T1 = [[s1, 0, -s1 c1x], [0, s1, -s1 c1y], [0, 0, 1]]
  double A[9];
  for (int r = 0; r < 3; ++r) {
    A[3 * r + 0] = Hn[3 * r + 0] * N.s1;
    A[3 * r + 1] = Hn[3 * r + 1] * N.s1;
    A[3 * r + 2] = Hn[3 * r + 2] - Hn[3 * r + 0] * N.s1 * N.c1x - Hn[3 * r + 1] * N.s1 * N.c1y;
  }
  // T2^-1 = [[1/s2, 0, c2x], [0, 1/s2, c2y], [0, 0, 1]]
  for (int c = 0; c < 3; ++c) {
    H[0 + c] = A[0 + c] / N.s2 + N.c2x * A[6 + c];
    H[3 + c] = A[3 + c] / N.s2 + N.c2y * A[6 + c];
    H[6 + c] = A[6 + c];
  }
}

__device__ __host__ inline double reproj_err2(const double (&H)[9], double x, double y, double u, double v) {
  const double w = H[6] * x + H[7] * y + H[8];
  const double px = (H[0] * x + H[1] * y + H[2]) / w, py = (H[3] * x + H[4] * y + H[5]) / w;
  return (px - u) * (px - u) + (py - v) * (py - v);
}

constexpr int RH = 64;  // hypotheses per workgroup

// batched form (ptz_homography_ransac_batch): set blockIdx.y of n_sets, its points at [off[y], off[y + 1]), its own
// normalisation and best key; the single-set call passes off = nullptr (the kernel arguments are the set)
struct RansacSets {
  const int64_t* off;  // [n_sets + 1] or nullptr
  const Norm* norm;    // [n_sets]
};
__global__ __launch_bounds__(256) void k_ransac_score(int n, const double* __restrict__ p1, const double* __restrict__ p2,
                                                      Norm N, double thr2, int n_hyp, uint64_t seed,
                                                      unsigned long long* __restrict__ best, RansacSets rs) {
  if (rs.off) {  // batched: set blockIdx.y
    const int y = blockIdx.y;
    const int64_t a = rs.off[y];
    n = (int)(rs.off[y + 1] - a);
    p1 += 2 * a;
    p2 += 2 * a;
    N = rs.norm[y];
    best += y;
  }
  __shared__ double sH[RH][9];
  __shared__ int sOk[RH];
  __shared__ int sCnt[4][RH];
  const int t = threadIdx.x, h0 = blockIdx.x * RH;
  if (t < RH) {
    const int h = h0 + t;
    bool ok = h < n_hyp;
    double H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 1};
    if (ok) {
      uint32_t s[4];
      for (int k = 0; k < 4; ++k) {
        uint32_t att = 0, v;
        bool dup;
        do {
          v = ransac_draw(seed, (uint32_t)h, (uint32_t)k, att++, (uint32_t)n);
          dup = false;
          for (int m = 0; m < k; ++m) dup |= (s[m] == v);
        } while (dup && att < 64);
        s[k] = v;
      }
      double M[8][9];
      for (int k = 0; k < 4; ++k) {
        const double x = N.s1 * (p1[2 * s[k]] - N.c1x), y = N.s1 * (p1[2 * s[k] + 1] - N.c1y);
        const double u = N.s2 * (p2[2 * s[k]] - N.c2x), v = N.s2 * (p2[2 * s[k] + 1] - N.c2y);
        dlt_rows(x, y, u, v, M[2 * k], M[2 * k + 1]);
      }
      double hv[8];
      ok = solve8(M, hv);
      if (ok) denormalise(hv, N, H);
    }
    for (int k = 0; k < 9; ++k) sH[t][k] = H[k];
    sOk[t] = ok ? 1 : 0;
  }
  __syncthreads();
  const int hl = t & (RH - 1), part = t >> 6;
  double H[9];
  for (int k = 0; k < 9; ++k) H[k] = sH[hl][k];
  int cnt = 0;
  if (sOk[hl])
    for (int i = part; i < n; i += 4)
      cnt += reproj_err2(H, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) < thr2 ? 1 : 0;
  sCnt[part][hl] = cnt;
  __syncthreads();
  if (t < RH && sOk[t] && h0 + t < n_hyp) {
    const int c = sCnt[0][t] + sCnt[1][t] + sCnt[2][t] + sCnt[3][t];
    const unsigned long long key = ((unsigned long long)c << 32) | (0xffffffffu - (unsigned)(h0 + t));
    atomicMax(best, key);
  }
}

// one workgroup: the best hypothesis' H, its inliers, a linear least-squares refit on them (normal
// equations of the DLT rows in normalised coordinates, fixed-order reduction), the final mask
__global__ __launch_bounds__(256) void k_ransac_refine(int n, const double* __restrict__ p1, const double* __restrict__ p2,
                                                       Norm N, double thr2, uint64_t seed,
                                                       const unsigned long long* __restrict__ best,
                                                       uint8_t* __restrict__ mask, double* __restrict__ Hout,
                                                       int* __restrict__ nin, RansacSets rs) {
  if (rs.off) {  // batched: set blockIdx.x
    const int y = blockIdx.x;
    const int64_t a = rs.off[y];
    n = (int)(rs.off[y + 1] - a);
    p1 += 2 * a;
    p2 += 2 * a;
    N = rs.norm[y];
    best += y;
    mask += a;
    Hout += 9 * y;
    nin += y;
  }
  __shared__ double sH[9];
  __shared__ double red[256][45];  // 8x9 augmented normal equations (upper part of the 9x9 Gram matrix)
  __shared__ int sOk;
  const int t = threadIdx.x;
  const unsigned long long key = *best;
  if (t == 0) {
    const uint32_t h = 0xffffffffu - (uint32_t)(key & 0xffffffffu);
    uint32_t s[4];
    for (int k = 0; k < 4; ++k) {
      uint32_t att = 0, v;
      bool dup;
      do {
        v = ransac_draw(seed, h, (uint32_t)k, att++, (uint32_t)n);
        dup = false;
        for (int m = 0; m < k; ++m) dup |= (s[m] == v);
      } while (dup && att < 64);
      s[k] = v;
    }
    double M[8][9], hv[8], H[9] = {0, 0, 0, 0, 0, 0, 0, 0, 1};
    for (int k = 0; k < 4; ++k) {
      const double x = N.s1 * (p1[2 * s[k]] - N.c1x), y = N.s1 * (p1[2 * s[k] + 1] - N.c1y);
      const double u = N.s2 * (p2[2 * s[k]] - N.c2x), v = N.s2 * (p2[2 * s[k] + 1] - N.c2y);
      dlt_rows(x, y, u, v, M[2 * k], M[2 * k + 1]);
    }
    sOk = key != 0 && solve8(M, hv);
    if (sOk) denormalise(hv, N, H);
    for (int k = 0; k < 9; ++k) sH[k] = H[k];
  }
  __syncthreads();
  if (!sOk) {
    for (int i = t; i < n; i += 256) mask[i] = 0;
    if (t < 9) Hout[t] = 0.0;
    if (t == 0) *nin = 0;
    return;
  }
  double H[9];
  for (int k = 0; k < 9; ++k) H[k] = sH[k];
  double g[45];
  for (int k = 0; k < 45; ++k) g[k] = 0.0;
  for (int i = t; i < n; i += 256) {
    if (!(reproj_err2(H, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) < thr2)) continue;
    double r0[9], r1[9];
    const double x = N.s1 * (p1[2 * i] - N.c1x), y = N.s1 * (p1[2 * i + 1] - N.c1y);
    const double u = N.s2 * (p2[2 * i] - N.c2x), v = N.s2 * (p2[2 * i + 1] - N.c2y);
    dlt_rows(x, y, u, v, r0, r1);
    int e = 0;
    for (int a = 0; a < 8; ++a)
      for (int b = a; b < 9; ++b) g[e++] += r0[a] * r0[b] + r1[a] * r1[b];
  }
  for (int k = 0; k < 44; ++k) red[t][k] = g[k];
  __syncthreads();
  if (t < 44) {
    double s = 0.0;
    for (int q = 0; q < 256; ++q) s += red[q][t];
    red[0][t] = s;
  }
  __syncthreads();
  if (t == 0) {
    double M[8][9], hv[8];
    int e = 0;
    for (int a = 0; a < 8; ++a)
      for (int b = a; b < 9; ++b) {
        M[a][b] = red[0][e++];
        if (b < 8) M[b][a] = M[a][b];
      }
    if (solve8(M, hv)) {
      double Hr[9];
      denormalise(hv, N, Hr);
      for (int k = 0; k < 9; ++k) sH[k] = Hr[k];
    }
  }
  __syncthreads();
  for (int k = 0; k < 9; ++k) H[k] = sH[k];
  int cnt = 0;
  for (int i = t; i < n; i += 256) {
    const uint8_t m = reproj_err2(H, p1[2 * i], p1[2 * i + 1], p2[2 * i], p2[2 * i + 1]) < thr2 ? 1 : 0;
    mask[i] = m;
    cnt += m;
  }
  __shared__ int sc[256];
  sc[t] = cnt;
  __syncthreads();
  if (t == 0) {
    int c = 0;
    for (int q = 0; q < 256; ++q) c += sc[q];
    *nin = c;
  }
  if (t < 9) Hout[t] = H[t] / H[8];
}

}  // namespace ptzba

using namespace ptzba;

int ptz_match_knn2(int device, int64_t n1, int64_t n2, int32_t dim, const float* des1, const float* des2,
                   int32_t* idx_out, float* dist_out) {
  if (n1 < 0 || n2 < 0 || dim <= 0) return fail("bad sizes n1=%lld n2=%lld dim=%d", (long long)n1, (long long)n2, dim);
  if (n1 == 0) return 0;
  if (!des1 || !idx_out || !dist_out || (n2 > 0 && !des2)) return fail("null argument");
  if (n1 * n2 > ((int64_t)1 << 31)) return fail("distance matrix %lld x %lld too large", (long long)n1, (long long)n2);
  if (n2 == 0) {
    for (int64_t i = 0; i < n1; ++i) {
      idx_out[2 * i] = idx_out[2 * i + 1] = -1;
      dist_out[2 * i] = dist_out[2 * i + 1] = INFINITY;
    }
    return 0;
  }
  if (select_device(device)) return -1;
  struct KnnWork {
    DBuf a, b, d, idx, dist;
  };
  auto guard = device_work_lock(device);
  KnnWork& Wk = work_for<KnnWork>(device);  // kept across calls: a keyframe matches ~15 pairs
  DBuf &a = Wk.a, &b = Wk.b, &d = Wk.d, &idx = Wk.idx, &dist = Wk.dist;
  if (a.reserve((size_t)n1 * dim * 4) || b.reserve((size_t)n2 * dim * 4) || d.reserve((size_t)n1 * n2 * 4) ||
      idx.reserve((size_t)n1 * 8) || dist.reserve((size_t)n1 * 8))
    return -1;
  HIPCHK(hipMemcpy(a.p, des1, (size_t)n1 * dim * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(b.p, des2, (size_t)n2 * dim * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_sqdist, dim3((unsigned)((n2 + KT - 1) / KT), (unsigned)((n1 + KT - 1) / KT)), dim3(256), 0, nullptr,
                     (int)n1, (int)n2, dim, a.as<float>(), b.as<float>(), d.as<float>());
  hipLaunchKernelGGL(k_top2, dim3((unsigned)((n1 + 3) / 4)), dim3(256), 0, nullptr, (int)n1, (int)n2, d.as<float>(),
                     idx.as<int>(), dist.as<float>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(idx_out, idx.p, (size_t)n1 * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(dist_out, dist.p, (size_t)n1 * 8, hipMemcpyDeviceToHost));
  return 0;
}

// Device-resident descriptor sets (ptz_desc_put / ptz_desc_drop) and kNN-2 of several resident query sets against a
// resident train set (ptz_match_knn2_sets): a sliding keyframe window matches its new keyframe against ~29 older
// ones per call, whose descriptors (~22 MB of fp32 at 1500 x 128 each) would otherwise be concatenated and copied
// host -> device again at every call.  The query sets are gathered device to device into the work buffer and run
// through the same two kernels as ptz_match_knn2 on their concatenation: the same result bit for bit.
struct DescSet {
  DBuf buf;
  int64_t n = 0;
  int32_t dim = 0;
  bool integral = false;  // every value an integer with 2 dim v^2 < 2^24 (exact in f16 sums: k_knn2_mf applies)
};
struct DescStore {
  std::vector<std::pair<uint64_t, DescSet*>> sets;
  DescSet* find(uint64_t key) {
    for (auto& e : sets)
      if (e.first == key) return e.second;
    return nullptr;
  }
  ~DescStore() {
    for (auto& e : sets) delete e.second;
  }
};

int ptz_desc_put(int device, uint64_t key, int64_t n, int32_t dim, const float* des) {
  if (n < 0 || dim <= 0 || (n > 0 && !des)) return fail("ptz_desc_put: bad arguments n=%lld dim=%d", (long long)n, dim);
  if (select_device(device)) return -1;
  auto guard = device_work_lock(device);
  DescStore& S = work_for<DescStore>(device);
  DescSet* d = S.find(key);
  if (!d) {
    d = new DescSet;
    S.sets.emplace_back(key, d);
  }
  if (d->buf.reserve((size_t)std::max<int64_t>(n, 1) * dim * 4)) return -1;
  d->n = n;
  d->dim = dim;
  // the matrix-core kNN (k_knn2_mf) is exact while every f16 product and every distance sum stays an exact integer
  // below 2^24: 2 * dim * v^2 < 2^24, i.e. |v| <= 255 for 128-d (SIFT) rows
  const float vmax = std::floor(std::sqrt((float)((1 << 23) - 1) / (float)std::max(dim, 1)));
  bool integral = true;
  for (int64_t e = 0; e < n * dim && integral; ++e) integral = des[e] == std::nearbyint(des[e]) && std::fabs(des[e]) <= vmax;
  d->integral = integral;
  if (n) HIPCHK(hipMemcpy(d->buf.p, des, (size_t)n * dim * 4, hipMemcpyHostToDevice));
  return 0;
}

int ptz_desc_drop(int device, int32_t n_keys, const uint64_t* keys) {
  if (n_keys < 0 || (n_keys > 0 && !keys)) return fail("ptz_desc_drop: bad arguments");
  if (select_device(device)) return -1;
  auto guard = device_work_lock(device);
  DescStore& S = work_for<DescStore>(device);
  for (int32_t k = 0; k < n_keys; ++k)
    for (size_t q = 0; q < S.sets.size(); ++q)
      if (S.sets[q].first == keys[k]) {
        delete S.sets[q].second;
        S.sets.erase(S.sets.begin() + q);
        break;
      }
  return 0;
}

int ptz_match_knn2_sets(int device, int32_t n_sets, const uint64_t* query_keys, uint64_t train_key, int64_t n_rows,
                        int32_t* idx_out, float* dist_out) {
  if (n_sets < 0 || (n_sets > 0 && (!query_keys || !idx_out || !dist_out))) return fail("ptz_match_knn2_sets: bad arguments");
  if (select_device(device)) return -1;
  auto guard = device_work_lock(device);
  DescStore& S = work_for<DescStore>(device);
  const DescSet* tr = S.find(train_key);
  if (!tr) return fail("ptz_match_knn2_sets: no descriptor set under train key %llu", (unsigned long long)train_key);
  const int32_t dim = tr->dim;
  const int64_t n2 = tr->n;
  int64_t n1 = 0;
  for (int32_t q = 0; q < n_sets; ++q) {
    const DescSet* d = S.find(query_keys[q]);
    if (!d) return fail("ptz_match_knn2_sets: no descriptor set under query key %llu", (unsigned long long)query_keys[q]);
    if (d->n > 0 && n2 > 0 && d->dim != dim) return fail("ptz_match_knn2_sets: query set %d has dim %d, train %d", q, d->dim, dim);
    n1 += d->n;
  }
  if (n1 != n_rows) return fail("ptz_match_knn2_sets: the query sets hold %lld rows, the output %lld", (long long)n1, (long long)n_rows);
  if (n1 == 0) return 0;
  if (n1 * n2 > ((int64_t)1 << 31)) return fail("distance matrix %lld x %lld too large", (long long)n1, (long long)n2);
  if (n2 == 0) {
    for (int64_t i = 0; i < n1; ++i) {
      idx_out[2 * i] = idx_out[2 * i + 1] = -1;
      dist_out[2 * i] = dist_out[2 * i + 1] = INFINITY;
    }
    return 0;
  }
  struct KnnSetsWork {
    DBuf a, d, idx, dist;
  };
  KnnSetsWork& Wk = work_for<KnnSetsWork>(device);
  // integer-valued 128-d sets (SIFT's): the matrix-core kernel, no distance matrix (PTZ_KNN_MF=0: the fp32 pair, A/B)
  bool mf = dim == KN_DIM && tr->integral;
  for (int32_t q = 0; q < n_sets && mf; ++q) mf = S.find(query_keys[q])->integral;
  const char* mfe = getenv("PTZ_KNN_MF");
  if (mfe && atoi(mfe) == 0) mf = false;
  if (Wk.a.reserve((size_t)n1 * dim * 4) || (!mf && Wk.d.reserve((size_t)n1 * n2 * 4)) || Wk.idx.reserve((size_t)n1 * 8) ||
      Wk.dist.reserve((size_t)n1 * 8))
    return -1;
  int64_t o = 0;
  for (int32_t q = 0; q < n_sets; ++q) {
    const DescSet* d = S.find(query_keys[q]);
    if (d->n) HIPCHK(hipMemcpyAsync(Wk.a.as<char>() + o * dim * 4, d->buf.p, (size_t)d->n * dim * 4, hipMemcpyDeviceToDevice, nullptr));
    o += d->n;
  }
  if (mf) {
    hipLaunchKernelGGL(k_knn2_mf, dim3((unsigned)((n1 + 63) / 64)), dim3(256), 0, nullptr, (int)n1, (int)n2,
                       Wk.a.as<float>(), tr->buf.as<float>(), Wk.idx.as<int>(), Wk.dist.as<float>());
  } else {
    hipLaunchKernelGGL(k_sqdist, dim3((unsigned)((n2 + KT - 1) / KT), (unsigned)((n1 + KT - 1) / KT)), dim3(256), 0, nullptr,
                       (int)n1, (int)n2, dim, Wk.a.as<float>(), tr->buf.as<float>(), Wk.d.as<float>());
    hipLaunchKernelGGL(k_top2, dim3((unsigned)((n1 + 3) / 4)), dim3(256), 0, nullptr, (int)n1, (int)n2, Wk.d.as<float>(),
                       Wk.idx.as<int>(), Wk.dist.as<float>());
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(idx_out, Wk.idx.p, (size_t)n1 * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(dist_out, Wk.dist.p, (size_t)n1 * 8, hipMemcpyDeviceToHost));
  return 0;
}

// Hartley normalisation of each point set (centroid, mean distance sqrt(2)); host, O(n)
static Norm hartley(int64_t n, const double* pts1, const double* pts2) {
  Norm N{};
  double sx1 = 0, sy1 = 0, sx2 = 0, sy2 = 0;
  for (int64_t i = 0; i < n; ++i) {
    sx1 += pts1[2 * i]; sy1 += pts1[2 * i + 1]; sx2 += pts2[2 * i]; sy2 += pts2[2 * i + 1];
  }
  N.c1x = sx1 / n; N.c1y = sy1 / n; N.c2x = sx2 / n; N.c2y = sy2 / n;
  double d1 = 0, d2 = 0;
  for (int64_t i = 0; i < n; ++i) {
    d1 += std::sqrt((pts1[2 * i] - N.c1x) * (pts1[2 * i] - N.c1x) + (pts1[2 * i + 1] - N.c1y) * (pts1[2 * i + 1] - N.c1y));
    d2 += std::sqrt((pts2[2 * i] - N.c2x) * (pts2[2 * i] - N.c2x) + (pts2[2 * i + 1] - N.c2y) * (pts2[2 * i + 1] - N.c2y));
  }
  N.s1 = d1 > 0 ? std::sqrt(2.0) * n / d1 : 1.0;
  N.s2 = d2 > 0 ? std::sqrt(2.0) * n / d2 : 1.0;
  return N;
}

int ptz_homography_ransac(int device, int64_t n, const double* pts1, const double* pts2, double threshold,
                          int32_t n_hyp, uint64_t seed, uint8_t* mask_out, double* H_out, int32_t* n_inliers_out) {
  if (n < 4) return fail("homography RANSAC needs at least 4 correspondences (got %lld)", (long long)n);
  if (!pts1 || !pts2 || !mask_out || !H_out || !n_inliers_out) return fail("null argument");
  if (!(threshold > 0) || n_hyp < 1) return fail("bad threshold / hypothesis count");
  if (n >= ((int64_t)1 << 31)) return fail("too many correspondences");
  const Norm N = hartley(n, pts1, pts2);
  if (select_device(device)) return -1;
  struct RansacWork {
    DBuf p1, p2, best, mask, H, nin;
  };
  auto guard = device_work_lock(device);
  RansacWork& Wk = work_for<RansacWork>(device);
  DBuf &p1 = Wk.p1, &p2 = Wk.p2, &best = Wk.best, &mask = Wk.mask, &H = Wk.H, &nin = Wk.nin;
  if (p1.reserve((size_t)n * 16) || p2.reserve((size_t)n * 16) || best.reserve(8) || mask.reserve((size_t)n) ||
      H.reserve(72) || nin.reserve(4))
    return -1;
  HIPCHK(hipMemcpy(p1.p, pts1, (size_t)n * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(p2.p, pts2, (size_t)n * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(best.p, 0, 8));
  const double thr2 = threshold * threshold;
  hipLaunchKernelGGL(k_ransac_score, dim3((unsigned)((n_hyp + RH - 1) / RH)), dim3(256), 0, nullptr, (int)n,
                     p1.as<double>(), p2.as<double>(), N, thr2, n_hyp, seed, best.as<unsigned long long>(),
                     RansacSets{nullptr, nullptr});
  hipLaunchKernelGGL(k_ransac_refine, dim3(1), dim3(256), 0, nullptr, (int)n, p1.as<double>(), p2.as<double>(), N, thr2,
                     seed, best.as<unsigned long long>(), mask.as<uint8_t>(), H.as<double>(), nin.as<int>(),
                     RansacSets{nullptr, nullptr});
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(mask_out, mask.p, (size_t)n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(H_out, H.p, 72, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(n_inliers_out, nin.p, 4, hipMemcpyDeviceToHost));
  return 0;
}

// n_sets independent RANSACs in two launches (a keyframe's pairwise matches): set s has the correspondences
// [off[s], off[s + 1]) of pts1 / pts2; per set exactly the result of ptz_homography_ransac with the same seed (the
// hypotheses are keyed by (seed, hypothesis, draw), the set's normalisation and best key are its own)
int ptz_homography_ransac_batch(int device, int32_t n_sets, const int64_t* off, const double* pts1, const double* pts2,
                                double threshold, int32_t n_hyp, uint64_t seed, uint8_t* mask_out, double* H_out,
                                int32_t* n_inliers_out) {
  if (n_sets < 0 || (n_sets > 0 && (!off || !pts1 || !pts2 || !mask_out || !H_out || !n_inliers_out)))
    return fail("null argument");
  if (n_sets == 0) return 0;
  if (!(threshold > 0) || n_hyp < 1) return fail("bad threshold / hypothesis count");
  if (n_sets > 65535) return fail("too many sets (%d)", n_sets);
  if (off[0] != 0) return fail("off[0] must be 0");
  std::vector<Norm> norms(n_sets);
  for (int s = 0; s < n_sets; ++s) {
    const int64_t n = off[s + 1] - off[s];
    if (n < 4) return fail("set %d: homography RANSAC needs at least 4 correspondences (got %lld)", s, (long long)n);
    if (n >= ((int64_t)1 << 31)) return fail("set %d: too many correspondences", s);
    norms[s] = hartley(n, pts1 + 2 * off[s], pts2 + 2 * off[s]);
  }
  const int64_t nt = off[n_sets];
  if (select_device(device)) return -1;
  struct RansacBatchWork {
    DBuf p1, p2, best, mask, H, nin, off, norm;
  };
  auto guard = device_work_lock(device);
  RansacBatchWork& Wk = work_for<RansacBatchWork>(device);
  if (Wk.p1.reserve((size_t)nt * 16) || Wk.p2.reserve((size_t)nt * 16) || Wk.best.reserve(8 * (size_t)n_sets) ||
      Wk.mask.reserve((size_t)nt) || Wk.H.reserve(72 * (size_t)n_sets) || Wk.nin.reserve(4 * (size_t)n_sets) ||
      Wk.off.reserve(8 * (size_t)(n_sets + 1)) || Wk.norm.reserve(sizeof(Norm) * (size_t)n_sets))
    return -1;
  HIPCHK(hipMemcpy(Wk.p1.p, pts1, (size_t)nt * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(Wk.p2.p, pts2, (size_t)nt * 16, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(Wk.off.p, off, 8 * (size_t)(n_sets + 1), hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(Wk.norm.p, norms.data(), sizeof(Norm) * (size_t)n_sets, hipMemcpyHostToDevice));
  HIPCHK(hipMemset(Wk.best.p, 0, 8 * (size_t)n_sets));
  const double thr2 = threshold * threshold;
  const RansacSets rs{Wk.off.as<int64_t>(), Wk.norm.as<Norm>()};
  hipLaunchKernelGGL(k_ransac_score, dim3((unsigned)((n_hyp + RH - 1) / RH), (unsigned)n_sets), dim3(256), 0, nullptr, 0,
                     Wk.p1.as<double>(), Wk.p2.as<double>(), Norm{}, thr2, n_hyp, seed,
                     Wk.best.as<unsigned long long>(), rs);
  hipLaunchKernelGGL(k_ransac_refine, dim3((unsigned)n_sets), dim3(256), 0, nullptr, 0, Wk.p1.as<double>(),
                     Wk.p2.as<double>(), Norm{}, thr2, seed, Wk.best.as<unsigned long long>(), Wk.mask.as<uint8_t>(),
                     Wk.H.as<double>(), Wk.nin.as<int>(), rs);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(mask_out, Wk.mask.p, (size_t)nt, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(H_out, Wk.H.p, 72 * (size_t)n_sets, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(n_inliers_out, Wk.nin.p, 4 * (size_t)n_sets, hipMemcpyDeviceToHost));
  return 0;
}

// The batched SIFT matcher of a new keyframe in one call (image_process.match_sift_features_batch when the pairs share
// one resident train set): ptz_match_knn2_sets over the query sets, Lowe's ratio test d1 < 0.7 d2 in float32 per set
// (match_sift_features, image_process.py:178-234), the survivors' points gathered from the callers' keypoint
// arrays, one ptz_homography_ransac_batch over the sets with more than 8 survivors, and their inliers as index
// pairs -- per set exactly match_sift_features' (index1, index2).  status_out[s] = 1: 8 or fewer survivors (the
// caller prints the reference's warning), 0 otherwise; out_off [n_sets + 1] into out_i1 / out_i2 (capacity: the
// query rows).
int ptz_match_sets_ransac(int device, int32_t n_sets, const uint64_t* query_keys, const int64_t* query_rows,
                          uint64_t train_key, int64_t train_rows, const double* query_xy, const double* train_xy,
                          double threshold, int32_t n_hyp, uint64_t seed, int32_t* status_out, int64_t* out_off,
                          int32_t* out_i1, int32_t* out_i2) {
  if (n_sets < 0 || (n_sets > 0 && (!query_keys || !query_rows || !query_xy || !status_out || !out_off || !out_i1 || !out_i2)))
    return fail("ptz_match_sets_ransac: bad arguments");
  out_off[0] = 0;
  if (n_sets == 0) return 0;
  std::vector<int64_t> qoff(n_sets + 1, 0);
  for (int32_t q = 0; q < n_sets; ++q) qoff[q + 1] = qoff[q] + query_rows[q];
  const int64_t n1 = qoff[n_sets];
  std::vector<int32_t> idx(2 * std::max<int64_t>(n1, 1));
  std::vector<float> dist(2 * std::max<int64_t>(n1, 1));
  if (ptz_match_knn2_sets(device, n_sets, query_keys, train_key, n1, idx.data(), dist.data())) return -1;
  // ratio test and the candidate point sets
  std::vector<int64_t> coff(1, 0);
  std::vector<int32_t> cset, ci1, ci2;
  std::vector<double> p1, p2;
  for (int32_t q = 0; q < n_sets; ++q) {
    const size_t c0 = ci1.size();
    if (train_rows >= 2)
      for (int64_t r = 0; r < query_rows[q]; ++r) {
        const int64_t g = qoff[q] + r;
        if (dist[2 * g] < 0.7f * dist[2 * g + 1]) {
          const int32_t j = idx[2 * g];
          if (j < 0 || j >= train_rows) return fail("ptz_match_sets_ransac: train index %d out of range", j);
          ci1.push_back((int32_t)r);
          ci2.push_back(j);
          p1.push_back(query_xy[2 * g]);
          p1.push_back(query_xy[2 * g + 1]);
          p2.push_back(train_xy[2 * (int64_t)j]);
          p2.push_back(train_xy[2 * (int64_t)j + 1]);
        }
      }
    if (ci1.size() - c0 <= 8) {  // too few survivors: no RANSAC for this set
      status_out[q] = 1;
      ci1.resize(c0);
      ci2.resize(c0);
      p1.resize(2 * c0);
      p2.resize(2 * c0);
      continue;
    }
    status_out[q] = 0;
    cset.push_back(q);
    coff.push_back((int64_t)ci1.size());
  }
  const int32_t nc = (int32_t)cset.size();
  std::vector<uint8_t> mask(std::max<size_t>(ci1.size(), 1));
  std::vector<double> H(9 * std::max(nc, 1));
  std::vector<int32_t> nin(std::max(nc, 1));
  if (nc && ptz_homography_ransac_batch(device, nc, coff.data(), p1.data(), p2.data(), threshold, n_hyp, seed,
                                        mask.data(), H.data(), nin.data()))
    return -1;
  int64_t o = 0, c = 0;
  for (int32_t q = 0; q < n_sets; ++q) {
    if (status_out[q] == 0) {
      for (int64_t e = coff[c]; e < coff[c + 1]; ++e)
        if (mask[e]) {
          out_i1[o] = ci1[e];
          out_i2[o] = ci2[e];
          ++o;
        }
      ++c;
    }
    out_off[q + 1] = o;
  }
  return 0;
}

namespace ptzba {
// ---------------------------------------------------------------------------------------------
// pyramidal Lucas-Kanade point tracking (cv.calcOpticalFlowPyrLK(img, next_img, points, None,
// winSize=(31, 31)) as called by optical_flow_matching, image_process.py:393-415)
//   pyramid: level l+1 = 5x5 binomial [1 4 6 4 1]/16 blur of level l (reflect-101 border), every
//            second pixel (cv.pyrDown); gradients: Scharr 3x3 / 32 (reflect-101)
//   per point, one 256-thread workgroup: from the coarsest level down, the window's samples of the
//   first image and its gradients (bilinear, clamped to the image) give G = sum [Ix Iy]^T [Ix Iy];
//   Newton steps d += G^-1 sum (I - J(x + g + d)) [Ix Iy] until |delta| < eps or max_iter; the
//   guess doubles to the next level.  status 0 when G's smaller eigenvalue / window area < min_eig at
//   any level or the point leaves the image; err = mean |I - J| over the window at the final position.
// Sums are fp64 with a fixed-order LDS reduction (deterministic).
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

__global__ void k_u8_to_f32(int n, const uint8_t* __restrict__ src, float* __restrict__ dst) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}

__global__ void k_pyr_down(int sw, int sh, const float* __restrict__ src, int dw, int dh, float* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw || y >= dh) return;
  const float k[5] = {1.f, 4.f, 6.f, 4.f, 1.f};
  float s = 0.f;
  for (int i = 0; i < 5; ++i) {
    const int yy = refl101(2 * y + i - 2, sh);
    float r = 0.f;
    for (int j = 0; j < 5; ++j) r += k[j] * src[(int64_t)yy * sw + refl101(2 * x + j - 2, sw)];
    s += k[i] * r;
  }
  dst[(int64_t)y * dw + x] = s * (1.f / 256.f);
}

__global__ void k_scharr(int w, int h, const float* __restrict__ src, float* __restrict__ gx, float* __restrict__ gy) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const int xm = refl101(x - 1, w), xp = refl101(x + 1, w), ym = refl101(y - 1, h), yp = refl101(y + 1, h);
  auto P = [&](int yy, int xx) { return src[(int64_t)yy * w + xx]; };
  gx[(int64_t)y * w + x] = (3.f * (P(ym, xp) - P(ym, xm)) + 10.f * (P(y, xp) - P(y, xm)) + 3.f * (P(yp, xp) - P(yp, xm))) *
                           (1.f / 32.f);
  gy[(int64_t)y * w + x] = (3.f * (P(yp, xm) - P(ym, xm)) + 10.f * (P(yp, x) - P(ym, x)) + 3.f * (P(yp, xp) - P(ym, xp))) *
                           (1.f / 32.f);
}

__device__ __forceinline__ double bil(const float* __restrict__ im, int w, int h, double x, double y) {
  x = fmin(fmax(x, 0.0), (double)(w - 1));
  y = fmin(fmax(y, 0.0), (double)(h - 1));
  const int x0 = min((int)x, w - 2 < 0 ? 0 : w - 2), y0 = min((int)y, h - 2 < 0 ? 0 : h - 2);
  const int x1 = min(x0 + 1, w - 1), y1 = min(y0 + 1, h - 1);
  const double ax = x - x0, ay = y - y0;
  const double a = im[(int64_t)y0 * w + x0], b = im[(int64_t)y0 * w + x1], c = im[(int64_t)y1 * w + x0],
               d = im[(int64_t)y1 * w + x1];
  return (1 - ay) * ((1 - ax) * a + ax * b) + ay * ((1 - ax) * c + ax * d);
}

constexpr int LK_MAXLV = 6;
struct LkPyr {
  const float* I[LK_MAXLV];
  const float* J[LK_MAXLV];
  const float* gx[LK_MAXLV];
  const float* gy[LK_MAXLV];
  int w[LK_MAXLV], h[LK_MAXLV];
  int levels;
};

// block-wide fixed-order sum of NV doubles (256 threads)
template <int NV>
__device__ __forceinline__ void block_sum(double (&v)[NV], double (*red)[NV]) {
  const int t = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NV; ++k) red[t][k] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s)
#pragma unroll
      for (int k = 0; k < NV; ++k) red[t][k] += red[t + s][k];
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < NV; ++k) v[k] = red[0][k];
  __syncthreads();
}

__global__ __launch_bounds__(256) void k_lk_track(LkPyr P, int n, const float* __restrict__ pts, int half, int max_iter,
                                                  double eps, double min_eig, float* __restrict__ out_pts,
                                                  uint8_t* __restrict__ status, float* __restrict__ err) {
  __shared__ double red[256][3];
  const int q = blockIdx.x, t = threadIdx.x;
  if (q >= n) return;
  const int win = 2 * half + 1, area = win * win;
  constexpr int SPT = 4;  // window samples per thread (31 x 31 = 961 <= 1024)
  const double px = pts[2 * q], py = pts[2 * q + 1];
  double gxv = 0.0, gyv = 0.0;  // guess at the current level
  bool ok = true;
  double dx = 0.0, dy = 0.0;
  for (int L = P.levels - 1; L >= 0 && ok; --L) {
    const double sc = 1.0 / (double)(1 << L);
    const double cx = px * sc, cy = py * sc;
    const int w = P.w[L], h = P.h[L];
    double Iv[SPT], Ixv[SPT], Iyv[SPT];
    double g[3] = {0.0, 0.0, 0.0};
#pragma unroll
    for (int s = 0; s < SPT; ++s) {
      const int e = t + 256 * s;
      Iv[s] = Ixv[s] = Iyv[s] = 0.0;
      if (e < area) {
        const double x = cx + (e % win - half), y = cy + (e / win - half);
        Iv[s] = bil(P.I[L], w, h, x, y);
        Ixv[s] = bil(P.gx[L], w, h, x, y);
        Iyv[s] = bil(P.gy[L], w, h, x, y);
        g[0] += Ixv[s] * Ixv[s];
        g[1] += Ixv[s] * Iyv[s];
        g[2] += Iyv[s] * Iyv[s];
      }
    }
    block_sum<3>(g, red);
    const double tr = g[0] + g[2], det = g[0] * g[2] - g[1] * g[1];
    const double mineig = 0.5 * (tr - sqrt(fmax((g[0] - g[2]) * (g[0] - g[2]) + 4.0 * g[1] * g[1], 0.0))) / area;
    if (!(mineig >= min_eig) || !(det > 0)) {
      ok = false;
      break;
    }
    dx = dy = 0.0;
    for (int it = 0; it < max_iter; ++it) {
      double b[3] = {0.0, 0.0, 0.0};
#pragma unroll
      for (int s = 0; s < SPT; ++s) {
        const int e = t + 256 * s;
        if (e < area) {
          const double x = cx + (e % win - half) + gxv + dx, y = cy + (e / win - half) + gyv + dy;
          const double ediff = Iv[s] - bil(P.J[L], w, h, x, y);
          b[0] += ediff * Ixv[s];
          b[1] += ediff * Iyv[s];
        }
      }
      block_sum<3>(b, red);
      const double ddx = (g[2] * b[0] - g[1] * b[1]) / det, ddy = (g[0] * b[1] - g[1] * b[0]) / det;
      dx += ddx;
      dy += ddy;
      if (ddx * ddx + ddy * ddy < eps * eps) break;
    }
    if (L > 0) {
      gxv = 2.0 * (gxv + dx);
      gyv = 2.0 * (gyv + dy);
    }
  }
  const double nx = px + gxv + dx, ny = py + gyv + dy;
  double e1[3] = {0.0, 0.0, 0.0};
  if (ok) {
    const int w = P.w[0], h = P.h[0];
    for (int e = t; e < area; e += 256) {
      const double ox = (e % win - half), oy = (e / win - half);
      e1[0] += fabs(bil(P.I[0], w, h, px + ox, py + oy) - bil(P.J[0], w, h, nx + ox, ny + oy));
    }
  }
  block_sum<3>(e1, red);
  if (t == 0) {
    const bool inside = nx >= 0 && ny >= 0 && nx <= P.w[0] - 1 && ny <= P.h[0] - 1;
    out_pts[2 * q] = (float)nx;
    out_pts[2 * q + 1] = (float)ny;
    status[q] = (ok && inside) ? 1 : 0;
    err[q] = ok ? (float)(e1[0] / area) : INFINITY;
  }
}

}  // namespace ptzba

int ptz_lk_track(int device, int32_t width, int32_t height, const uint8_t* img0, const uint8_t* img1, int64_t n,
                 const float* pts0, int32_t levels, int32_t win, int32_t max_iter, double eps, double min_eig,
                 float* pts1_out, uint8_t* status_out, float* err_out) {
  using namespace ptzba;
  if (width < 2 || height < 2 || !img0 || !img1) return fail("bad image");
  if (n < 0 || (n > 0 && (!pts0 || !pts1_out || !status_out || !err_out))) return fail("bad point list");
  if (levels < 1 || levels > LK_MAXLV || win < 3 || (win & 1) == 0 || win > 31 || max_iter < 1)
    return fail("bad LK parameters (levels 1..%d, odd win 3..31)", LK_MAXLV);
  if (n == 0) return 0;
  if (select_device(device)) return -1;
  const int64_t np = (int64_t)width * height;
  std::vector<int> W(levels), H(levels);
  W[0] = width; H[0] = height;
  int64_t tot = 0;
  for (int l = 0; l < levels; ++l) {
    if (l > 0) { W[l] = (W[l - 1] + 1) / 2; H[l] = (H[l - 1] + 1) / 2; }
    tot += (int64_t)W[l] * H[l];
  }
  // work buffers kept across calls (a stream tracks every frame): one set per device, grown, never shrunk
  struct LkWork {
    DBuf u8, bufI, bufJ, bufX, bufY, dp, dout, dst, derr;
  };
  auto guard = device_work_lock(device);
  LkWork& Wk = work_for<LkWork>(device);
  DBuf &u8 = Wk.u8, &bufI = Wk.bufI, &bufJ = Wk.bufJ, &bufX = Wk.bufX, &bufY = Wk.bufY, &dp = Wk.dp, &dout = Wk.dout;
  DBuf &dst = Wk.dst, &derr = Wk.derr;
  if (u8.reserve((size_t)np * 2) || bufI.reserve((size_t)tot * 4) || bufJ.reserve((size_t)tot * 4) ||
      bufX.reserve((size_t)tot * 4) || bufY.reserve((size_t)tot * 4) || dp.reserve((size_t)n * 8) ||
      dout.reserve((size_t)n * 8) || dst.reserve((size_t)n) || derr.reserve((size_t)n * 4))
    return -1;
  HIPCHK(hipMemcpy(u8.p, img0, (size_t)np, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(u8.as<uint8_t>() + np, img1, (size_t)np, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dp.p, pts0, (size_t)n * 8, hipMemcpyHostToDevice));
  LkPyr P{};
  P.levels = levels;
  int64_t off = 0;
  for (int l = 0; l < levels; ++l) {
    P.I[l] = bufI.as<float>() + off; P.J[l] = bufJ.as<float>() + off;
    P.gx[l] = bufX.as<float>() + off; P.gy[l] = bufY.as<float>() + off;
    P.w[l] = W[l]; P.h[l] = H[l];
    off += (int64_t)W[l] * H[l];
  }
  hipLaunchKernelGGL(k_u8_to_f32, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, nullptr, (int)np, u8.as<uint8_t>(),
                     (float*)P.I[0]);
  hipLaunchKernelGGL(k_u8_to_f32, dim3((unsigned)((np + 255) / 256)), dim3(256), 0, nullptr, (int)np,
                     u8.as<uint8_t>() + np, (float*)P.J[0]);
  for (int l = 1; l < levels; ++l) {
    const dim3 g((unsigned)((W[l] + 127) / 128), (unsigned)H[l]);
    hipLaunchKernelGGL(k_pyr_down, g, dim3(128), 0, nullptr, W[l - 1], H[l - 1], P.I[l - 1], W[l], H[l], (float*)P.I[l]);
    hipLaunchKernelGGL(k_pyr_down, g, dim3(128), 0, nullptr, W[l - 1], H[l - 1], P.J[l - 1], W[l], H[l], (float*)P.J[l]);
  }
  for (int l = 0; l < levels; ++l)
    hipLaunchKernelGGL(k_scharr, dim3((unsigned)((W[l] + 127) / 128), (unsigned)H[l]), dim3(128), 0, nullptr, W[l], H[l],
                       P.I[l], (float*)P.gx[l], (float*)P.gy[l]);
  hipLaunchKernelGGL(k_lk_track, dim3((unsigned)n), dim3(256), 0, nullptr, P, (int)n, dp.as<float>(), win / 2, max_iter,
                     eps, min_eig, dout.as<float>(), dst.as<uint8_t>(), derr.as<float>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(pts1_out, dout.p, (size_t)n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(status_out, dst.p, (size_t)n, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(err_out, derr.p, (size_t)n * 4, hipMemcpyDeviceToHost));
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Hamming nearest neighbours both ways (cv.BFMatcher(cv.NORM_HAMMING, crossCheck=True).match, the matching
// step of match_orb_features / match_latch_features, image_process.py:237-310): one wave per query keeps the
// nearest train descriptor (ties to the lower index); the host keeps the mutual pairs.
// ---------------------------------------------------------------------------------------------
namespace ptzba {
constexpr int HAM_MAXW = 16;  // descriptor words (<= 64 bytes)

__global__ __launch_bounds__(256) void k_hamming_nn(int nq, int nt, int words, const uint32_t* __restrict__ q,
                                                    const uint32_t* __restrict__ t, int* __restrict__ idx,
                                                    int* __restrict__ dist) {
  const int qi = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (qi >= nq) return;
  uint32_t qv[HAM_MAXW];
#pragma unroll
  for (int k = 0; k < HAM_MAXW; ++k) qv[k] = k < words ? q[(int64_t)qi * words + k] : 0u;
  int bd = 0x7fffffff, bi = 0x7fffffff;
  for (int j = lane; j < nt; j += 64) {
    int d = 0;
#pragma unroll
    for (int k = 0; k < HAM_MAXW; ++k)
      if (k < words) d += __popc(qv[k] ^ t[(int64_t)j * words + k]);
    if (d < bd) { bd = d; bi = j; }  // j ascends per lane: the first minimum
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const int od = __shfl_xor(bd, off), oi = __shfl_xor(bi, off);
    if (od < bd || (od == bd && oi < bi)) { bd = od; bi = oi; }
  }
  if (lane == 0) {
    idx[qi] = nt > 0 ? bi : -1;
    dist[qi] = nt > 0 ? bd : -1;
  }
}
}  // namespace ptzba

int ptz_match_hamming(int device, int64_t n1, int64_t n2, int32_t nbytes, const uint8_t* des1, const uint8_t* des2,
                      int32_t* idx12, int32_t* dist12, int32_t* idx21) {
  using namespace ptzba;
  if (n1 < 0 || n2 < 0 || nbytes <= 0 || nbytes % 4 || nbytes > 4 * HAM_MAXW)
    return fail("bad descriptor shape (bytes per descriptor: a multiple of 4, at most %d)", 4 * HAM_MAXW);
  if ((n1 && (!des1 || !idx12 || !dist12)) || (n2 && (!des2 || !idx21))) return fail("null buffer");
  if (n1 == 0 && n2 == 0) return 0;
  if (select_device(device)) return -1;
  const int words = nbytes / 4;
  DBuf a, b, i12, d12, i21, d21;
  if (a.alloc((size_t)std::max<int64_t>(n1, 1) * nbytes) || b.alloc((size_t)std::max<int64_t>(n2, 1) * nbytes) ||
      i12.alloc((size_t)std::max<int64_t>(n1, 1) * 4) || d12.alloc((size_t)std::max<int64_t>(n1, 1) * 4) ||
      i21.alloc((size_t)std::max<int64_t>(n2, 1) * 4) || d21.alloc((size_t)std::max<int64_t>(n2, 1) * 4))
    return -1;
  if (n1) HIPCHK(hipMemcpy(a.p, des1, (size_t)n1 * nbytes, hipMemcpyHostToDevice));
  if (n2) HIPCHK(hipMemcpy(b.p, des2, (size_t)n2 * nbytes, hipMemcpyHostToDevice));
  if (n1)
    hipLaunchKernelGGL(k_hamming_nn, dim3((unsigned)((n1 + 3) / 4)), dim3(256), 0, nullptr, (int)n1, (int)n2, words,
                       a.as<uint32_t>(), b.as<uint32_t>(), i12.as<int>(), d12.as<int>());
  if (n2)
    hipLaunchKernelGGL(k_hamming_nn, dim3((unsigned)((n2 + 3) / 4)), dim3(256), 0, nullptr, (int)n2, (int)n1, words,
                       b.as<uint32_t>(), a.as<uint32_t>(), i21.as<int>(), d21.as<int>());
  HIPCHK(hipGetLastError());
  if (n1) {
    HIPCHK(hipMemcpy(idx12, i12.p, (size_t)n1 * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(dist12, d12.p, (size_t)n1 * 4, hipMemcpyDeviceToHost));
  }
  if (n2) HIPCHK(hipMemcpy(idx21, i21.p, (size_t)n2 * 4, hipMemcpyDeviceToHost));
  return 0;
}

// ------------------------------------------------------------------------------------------------
// Shi-Tomasi corner response (cv.cornerMinEigenVal(img, blockSize=3, ksize=3), the measure of
// cv.goodFeaturesToTrack as detect_harris_corner_grid calls it, image_process.py:352-390): 3x3 Sobel
// derivatives scaled by 1 / (4 * 3 * 255) (OpenCV's scale for 8-bit input, ksize 3, blockSize 3), the
// products dx^2, dx dy, dy^2 summed over a 3x3 block (unnormalised box filter), and the smaller eigenvalue
// (a + c) - sqrt((a - c)^2 + b^2) with a = sum dx^2 / 2, c = sum dy^2 / 2, b = sum dx dy.  Every border is
// reflect-101 (the source for the derivatives, the product image for the block sum).  fp32 throughout
// (every operation rounded separately: the oracle repeats it in numpy float32).  A second pass flags the
// 3x3 local maxima (eig == max of its neighbourhood, eig > 0, not on the one-pixel image border): the
// candidates goodFeaturesToTrack keeps after its dilation.
// ------------------------------------------------------------------------------------------------
namespace ptzba {
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void k_min_eig(int w, int h, const uint8_t* __restrict__ img, float scale,
                                                 float* __restrict__ eig) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= w || y >= h) return;
  float sa = 0.f, sb = 0.f, sc = 0.f;
  for (int by = -1; by <= 1; ++by)
    for (int bx = -1; bx <= 1; ++bx) {
      const int cx = refl101(x + bx, w), cy = refl101(y + by, h);  // the product image is reflected here
      int gx = 0, gy = 0;
      for (int j = -1; j <= 1; ++j) {
        const int wj = j == 0 ? 2 : 1;
        const int yy = refl101(cy + j, h), xx = refl101(cx + j, w);
        gx += wj * ((int)img[(int64_t)yy * w + refl101(cx + 1, w)] - (int)img[(int64_t)yy * w + refl101(cx - 1, w)]);
        gy += wj * ((int)img[(int64_t)refl101(cy + 1, h) * w + xx] - (int)img[(int64_t)refl101(cy - 1, h) * w + xx]);
      }
      const float dx = (float)gx * scale, dy = (float)gy * scale;
      sa = sa + dx * dx;
      sb = sb + dx * dy;
      sc = sc + dy * dy;
    }
  const float a = sa * 0.5f, b = sb, c = sc * 0.5f;
  const float d = (a - c) * (a - c) + b * b;
  eig[(int64_t)y * w + x] = (a + c) - sqrtf(d);
}
#pragma clang fp contract(on)
__global__ __launch_bounds__(256) void k_local_max3(int w, int h, const float* __restrict__ eig, uint8_t* __restrict__ flag) {
  const int x = blockIdx.x * 16 + (threadIdx.x & 15), y = blockIdx.y * 16 + (threadIdx.x >> 4);
  if (x >= w || y >= h) return;
  uint8_t f = 0;
  if (x >= 1 && y >= 1 && x < w - 1 && y < h - 1) {
    const float v = eig[(int64_t)y * w + x];
    bool mx = v > 0.f;
    for (int dy = -1; dy <= 1 && mx; ++dy)
      for (int dx = -1; dx <= 1; ++dx)
        if (eig[(int64_t)(y + dy) * w + x + dx] > v) mx = false;
    f = mx ? 1 : 0;
  }
  flag[(int64_t)y * w + x] = f;
}
}  // namespace ptzba

int ptz_corner_min_eig(int device, int32_t width, int32_t height, const uint8_t* img, float* eig_out, uint8_t* locmax_out) {
  using namespace ptzba;
  if (width < 1 || height < 1 || !img || !eig_out) return fail("bad image / output");
  if (select_device(device)) return -1;
  const size_t np = (size_t)width * height;
  struct EigWork {
    DBuf u8, eig, flag;
  };
  auto guard = device_work_lock(device);
  EigWork& Wk = work_for<EigWork>(device);
  if (Wk.u8.reserve(np) || Wk.eig.reserve(np * 4) || Wk.flag.reserve(np)) return -1;
  HIPCHK(hipMemcpy(Wk.u8.p, img, np, hipMemcpyHostToDevice));
  const dim3 grid((unsigned)((width + 15) / 16), (unsigned)((height + 15) / 16));
  const float scale = (float)(1.0 / (4.0 * 3.0 * 255.0));
  hipLaunchKernelGGL(k_min_eig, grid, dim3(256), 0, nullptr, width, height, Wk.u8.as<uint8_t>(), scale, Wk.eig.as<float>());
  if (locmax_out)
    hipLaunchKernelGGL(k_local_max3, grid, dim3(256), 0, nullptr, width, height, Wk.eig.as<float>(), Wk.flag.as<uint8_t>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(eig_out, Wk.eig.p, np * 4, hipMemcpyDeviceToHost));
  if (locmax_out) HIPCHK(hipMemcpy(locmax_out, Wk.flag.p, np, hipMemcpyDeviceToHost));
  return 0;
}
