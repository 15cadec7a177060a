// SIFT keypoints + descriptors on the GPU (detection half of the front-end):
// cv.xfeatures2d.SIFT_create(nfeatures).detectAndCompute as detect_compute_sift calls it
// (image_process.py:56-79).  Lowe's algorithm with OpenCV's defaults: the image doubled (bilinear), 3 layers
// per octave, sigma 1.6 (input blur 0.5), contrast threshold 0.04, edge ratio 10, 36-bin orientation
// histograms (peaks >= 0.8 max), 4 x 4 x 8 descriptors clipped at 0.2 and scaled to integers 0..255.
//   pyramid     k_sift_up (2x bilinear), separable Gaussian blur (row / column launches, reflect-101,
//               float32 mul-then-add in kernel order: no contraction, so the pyramid is bit-identical to
//               the oracle's), k_sift_down, k_sift_dog
//   extrema     k_sift_extrema: one thread per pixel of the 3 inner DoG layers, 26-neighbour test, then the
//               sub-pixel refinement (fp64, at most 5 steps), contrast and edge tests; survivors are
//               appended to a candidate list
//   orientation k_sift_orient: one wave per candidate, 36-bin histogram in LDS (adds of one wave only),
//               smoothing and peak interpolation by lane 0; every peak is a keypoint
//   selection   host: keypoints ordered by (-response, y, x, angle), cut to nfeatures
//   descriptor  k_sift_descr: one wave per keypoint, the (d+2)^2 (n+2) trilinear histogram in LDS (fp64
//               adds of one wave), normalise / clip / renormalise / round by the wave
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "../../include/ptzba.h"
#include "host_util.h"
#include "ptzba_common.h"

// Every float / double operation of this file rounds separately (no fused multiply-add): the pyramid is
// bit-identical to the oracle's float32 numpy and the refinement follows its fp64 evaluation order.
#pragma clang fp contract(off)

namespace ptzba {

constexpr int SIFT_S = 3, SIFT_BORDER = 5, SIFT_MAXI = 5, SIFT_OB = 36, SIFT_D = 4, SIFT_N = 8;
constexpr double SIFT_SIG = 1.6, SIFT_CONTR = 0.04, SIFT_EDGE = 10.0;
constexpr int SIFT_HB = (SIFT_D + 2) * (SIFT_D + 2) * (SIFT_N + 2);  // 360 descriptor histogram bins

struct SiftCand {
  int o, l, r, c;
  double xi, xr, xc, contr;
};
struct SiftKp {
  float x, y, size, angle, response, scl;
  int o, l, r, c, pad0, pad1;
};

__device__ __forceinline__ int refl101(int i, int n) {
  if (n == 1) return 0;
  const int p = 2 * n - 2;
  i = abs(i) % p;
  return i >= n ? p - i : i;
}

__global__ void k_sift_up(int w, int h, const uint8_t* __restrict__ src, float* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  const int W = 2 * w;
  if (x >= W) return;
  auto coord = [](int d, int n, int& i0, int& i1, float& a) {
    const float s = (((float)d * 0.5f) - 0.25f);
    i0 = (int)floorf(s);
    a = (s - (float)i0);
    if (i0 < 0) { i0 = 0; a = 0.f; }
    if (i0 >= n - 1) { i0 = n - 1; a = 0.f; }
    i1 = min(i0 + 1, n - 1);
  };
  int x0, x1, y0, y1;
  float ax, ay;
  coord(x, w, x0, x1, ax);
  coord(y, h, y0, y1, ay);
  auto P = [&](int yy, int xx) { return (float)src[(int64_t)yy * w + xx]; };
  const float bx = (1.f - ax), by = (1.f - ay);
  const float top = ((bx * P(y0, x0)) + (ax * P(y0, x1)));
  const float bot = ((bx * P(y1, x0)) + (ax * P(y1, x1)));
  dst[(int64_t)y * W + x] = ((by * top) + (ay * bot));
}

// separable blur through LDS: a row segment (+ halo) / a column tile (+ halo rows) is read once; the
// accumulation order over k is unchanged (bit-identical to the per-pixel form and to the oracle)
constexpr int BLUR_RMAX = 32, BLUR_TX = 256, BLUR_CT = 64, BLUR_CR = 64;
__global__ __launch_bounds__(BLUR_TX) void k_sift_blur_rows(int w, int h, const float* __restrict__ src,
                                                             float* __restrict__ dst, const float* __restrict__ wt, int K) {
  __shared__ float tile[BLUR_TX + 2 * BLUR_RMAX];
  __shared__ float sw[2 * BLUR_RMAX + 1];
  const int x0 = blockIdx.x * BLUR_TX, y = blockIdx.y, r = K / 2, t = threadIdx.x;
  const float* row = src + (int64_t)y * w;
  for (int i = t; i < BLUR_TX + 2 * r; i += BLUR_TX) tile[i] = row[refl101(x0 + i - r, w)];
  if (t < K) sw[t] = wt[t];
  __syncthreads();
  const int x = x0 + t;
  if (x >= w) return;
  float acc = 0.f;
  for (int k = 0; k < K; ++k) acc = acc + sw[k] * tile[t + k];
  dst[(int64_t)y * w + x] = acc;
}

// Column pass with a sliding window (round 4): thread (tx, ty) produces the 16 consecutive output rows 16 ty .. 16 ty + 15
// of its column, keeping the 16 inputs the current tap needs in registers -- one LDS read per 16 products instead of
// one per product (1.816 -> 1.776 ms per 1080p detection against one output per thread, r04t).  Per output the same
// products in the same order (mul, then add; k ascending) as the oracle's sift_blur: bit-identical.
// Measured slower and removed in round 5: a sliding-window row pass (2.00 vs 1.81 ms, r04v), a row pass over 4 rows
// per workgroup (1.86 vs 1.81 ms, r04z8), both passes + the DoG in one launch (2.29 vs 2.23 ms, r04i).
__global__ __launch_bounds__(256) void k_sift_blur_cols_sw(int w, int h, const float* __restrict__ src,
                                                            float* __restrict__ dst, const float* __restrict__ wt, int K) {
  __shared__ float tile[BLUR_CR + 2 * BLUR_RMAX][BLUR_CT + 1];
  __shared__ float sw[2 * BLUR_RMAX + 1];
  const int tx = threadIdx.x & (BLUR_CT - 1), ty = threadIdx.x / BLUR_CT;  // 64 x 4
  const int x0 = blockIdx.x * BLUR_CT, y0 = blockIdx.y * BLUR_CR, r = K / 2;
  const int x = x0 + tx;
  const int nrow = BLUR_CR + 2 * r;
  for (int i = ty; i < nrow; i += 256 / BLUR_CT)
    tile[i][tx] = x < w ? src[(int64_t)refl101(y0 + i - r, h) * w + x] : 0.f;
  if (threadIdx.x < K) sw[threadIdx.x] = wt[threadIdx.x];
  __syncthreads();
  if (x >= w) return;
  constexpr int R = BLUR_CR / 4;  // 16 output rows per thread
  const int ra = R * ty;
  float acc[R], win[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    acc[j] = 0.f;
    win[j] = tile[ra + j][tx];
  }
  for (int k = 0; k < K; ++k) {
    const float wk = sw[k];
#pragma unroll
    for (int j = 0; j < R; ++j) acc[j] = acc[j] + wk * win[j];
    if (k + 1 == K) break;
#pragma unroll
    for (int j = 0; j + 1 < R; ++j) win[j] = win[j + 1];
    win[R - 1] = tile[ra + R + k][tx];  // row ra + R + k <= BLUR_CR - 1 + K - 1: inside the staged rows
  }
#pragma unroll
  for (int j = 0; j < R; ++j)
    if (y0 + ra + j < h) dst[(int64_t)(y0 + ra + j) * w + x] = acc[j];
}

__global__ void k_sift_down(int sw, const float* __restrict__ src, int dw, int dh, float* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw || y >= dh) return;
  dst[(int64_t)y * dw + x] = src[(int64_t)(2 * y) * sw + 2 * x];
}

__global__ void k_sift_dog(int64_t n, const float* __restrict__ g, float* __restrict__ d) {
  // n pixels per level; S + 2 DoG levels from S + 3 Gaussian levels (contiguous per octave)
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n * (SIFT_S + 2)) return;
  const int64_t lv = i / n, p = i - lv * n;
  d[i] = (g[(lv + 1) * n + p] - g[lv * n + p]);
}

// [[a b c] [b d e] [c e f]] x = y by the adjugate (the oracle's _solve3_sym)
__device__ bool solve3_sym(double a, double b, double c, double d, double e, double f, const double* y, double* x) {
#pragma clang fp contract(off)
  const double A0 = d * f - e * e, A1 = c * e - b * f, A2 = b * e - c * d;
  const double det = a * A0 + b * A1 + c * A2;
  if (det == 0.0) return false;
  const double B1 = a * f - c * c, B2 = b * c - a * e, C2 = a * d - b * b;
  const double inv = 1.0 / det;
  x[0] = (A0 * y[0] + A1 * y[1] + A2 * y[2]) * inv;
  x[1] = (A1 * y[0] + B1 * y[1] + B2 * y[2]) * inv;
  x[2] = (A2 * y[0] + B2 * y[1] + C2 * y[2]) * inv;
  return true;
}

// one thread per pixel (x, y) of DoG layer l = 1 + blockIdx.z of octave `o` (dog: S + 2 levels of w x h)
__global__ void k_sift_extrema(int o, int w, int h, const float* __restrict__ dog, float thr, SiftCand* __restrict__ out,
                               int* __restrict__ count, int cap) {
#pragma clang fp contract(off)
  const int c0 = blockIdx.x * blockDim.x + threadIdx.x + SIFT_BORDER, r0 = blockIdx.y + SIFT_BORDER;
  const int l0 = 1 + blockIdx.z;
  if (c0 >= w - SIFT_BORDER || r0 >= h - SIFT_BORDER) return;
  const int64_t n = (int64_t)w * h;
  auto D = [&](int l, int r, int c) { return dog[l * n + (int64_t)r * w + c]; };
  const float v = D(l0, r0, c0);
  if (!(fabsf(v) > thr)) return;
  bool mx = v > 0.f, mn = v < 0.f;
  for (int dl = -1; dl <= 1; ++dl)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dx = -1; dx <= 1; ++dx) {
        if (!dl && !dy && !dx) continue;
        const float u = D(l0 + dl, r0 + dy, c0 + dx);
        mx = mx && v >= u;
        mn = mn && v <= u;
      }
  if (!(mx || mn)) return;
  // sub-pixel refinement (fp64)
  const double sc = 1.0 / 255.0, ds = sc * 0.5, s2 = sc, cs = sc * 0.25;
  int l = l0, r = r0, c = c0;
  double xi = 0, xr = 0, xc = 0;
  bool ok = false;
  for (int it = 0; it < SIFT_MAXI; ++it) {
    auto C = [&](int rr, int cc) { return (double)D(l, rr, cc); };
    auto P = [&](int rr, int cc) { return (double)D(l - 1, rr, cc); };
    auto N = [&](int rr, int cc) { return (double)D(l + 1, rr, cc); };
    const double dD[3] = {(C(r, c + 1) - C(r, c - 1)) * ds, (C(r + 1, c) - C(r - 1, c)) * ds, (N(r, c) - P(r, c)) * ds};
    const double v2 = C(r, c) * 2;
    const double dxx = (C(r, c + 1) + C(r, c - 1) - v2) * s2;
    const double dyy = (C(r + 1, c) + C(r - 1, c) - v2) * s2;
    const double dss = (N(r, c) + P(r, c) - v2) * s2;
    const double dxy = (C(r + 1, c + 1) - C(r + 1, c - 1) - C(r - 1, c + 1) + C(r - 1, c - 1)) * cs;
    const double dxs = (N(r, c + 1) - N(r, c - 1) - P(r, c + 1) + P(r, c - 1)) * cs;
    const double dys = (N(r + 1, c) - N(r - 1, c) - P(r + 1, c) + P(r - 1, c)) * cs;
    double X[3];
    if (!solve3_sym(dxx, dxy, dxs, dyy, dys, dss, dD, X)) return;
    xc = -X[0]; xr = -X[1]; xi = -X[2];
    if (fabs(xi) < 0.5 && fabs(xr) < 0.5 && fabs(xc) < 0.5) {
      ok = true;
      break;
    }
    if (fabs(xi) > 1e6 || fabs(xr) > 1e6 || fabs(xc) > 1e6) return;
    c += (int)rint(xc);
    r += (int)rint(xr);
    l += (int)rint(xi);
    if (l < 1 || l > SIFT_S || c < SIFT_BORDER || c >= w - SIFT_BORDER || r < SIFT_BORDER || r >= h - SIFT_BORDER) return;
  }
  if (!ok) return;
  auto C = [&](int rr, int cc) { return (double)D(l, rr, cc); };
  auto P = [&](int rr, int cc) { return (double)D(l - 1, rr, cc); };
  auto N = [&](int rr, int cc) { return (double)D(l + 1, rr, cc); };
  const double dD0 = (C(r, c + 1) - C(r, c - 1)) * ds, dD1 = (C(r + 1, c) - C(r - 1, c)) * ds, dD2 = (N(r, c) - P(r, c)) * ds;
  const double t = dD0 * xc + dD1 * xr + dD2 * xi;
  const double contr = C(r, c) * sc + t * 0.5;
  if (fabs(contr) * SIFT_S < SIFT_CONTR) return;
  const double v2 = C(r, c) * 2;
  const double dxx = (C(r, c + 1) + C(r, c - 1) - v2) * s2;
  const double dyy = (C(r + 1, c) + C(r - 1, c) - v2) * s2;
  const double dxy = (C(r + 1, c + 1) - C(r + 1, c - 1) - C(r - 1, c + 1) + C(r - 1, c - 1)) * cs;
  const double tr = dxx + dyy, det = dxx * dyy - dxy * dxy;
  if (det <= 0 || tr * tr * SIFT_EDGE >= (SIFT_EDGE + 1) * (SIFT_EDGE + 1) * det) return;
  const int k = atomicAdd(count, 1);
  if (k < cap) out[k] = SiftCand{o, l, r, c, xi, xr, xc, contr};
}

// one wave per candidate: orientation histogram of the Gaussian image of its (octave, layer)
__global__ __launch_bounds__(256) void k_sift_orient(const SiftCand* __restrict__ cand, const int* __restrict__ n_cand,
                                                     const float* const* __restrict__ gauss, const int* __restrict__ ow,
                                                     const int* __restrict__ oh, SiftKp* __restrict__ kp,
                                                     int* __restrict__ n_kp, int cap) {
#pragma clang fp contract(off)
  __shared__ float hist[4][SIFT_OB];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + wv;
  if (q >= min(*n_cand, cap)) return;
  const SiftCand cd = cand[q];
  const int w = ow[cd.o], h = oh[cd.o];
  const float* img = gauss[cd.o * (SIFT_S + 3) + cd.l];
  const double scl = SIFT_SIG * pow(2.0, (cd.l + cd.xi) / SIFT_S);
  const int rad = (int)rint(3 * 1.5 * scl);
  const double sig = 1.5 * scl;
  const float es = (float)(-1.0 / (2.0 * sig * sig));
  float* hs = hist[wv];
  for (int b = lane; b < SIFT_OB; b += 64) hs[b] = 0.f;
  __builtin_amdgcn_wave_barrier();
  const int side = 2 * rad + 1, ns = side * side;
  for (int s = lane; s < ns; s += 64) {
    const int i = s / side - rad, j = s % side - rad;
    const int y = cd.r + i, x = cd.c + j;
    if (y <= 0 || y >= h - 1 || x <= 0 || x >= w - 1) continue;
    const float dx = (img[(int64_t)y * w + x + 1] - img[(int64_t)y * w + x - 1]);
    const float dy = (img[(int64_t)(y - 1) * w + x] - img[(int64_t)(y + 1) * w + x]);
    const float wgt = expf(((float)(i * i + j * j) * es));
    float ori = (float)(atan2((double)dy, (double)dx) * 57.29577951308232);
    if (ori < 0.f) ori = (ori + 360.f);
    const float mag = sqrtf(((dx * dx) + (dy * dy)));
    int bn = (int)rintf(((float)(SIFT_OB / 360.0) * ori));
    bn = bn >= SIFT_OB ? bn - SIFT_OB : (bn < 0 ? bn + SIFT_OB : bn);
    atomicAdd(&hs[bn], (wgt * mag));
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  if (lane != 0) return;
  float sm[SIFT_OB];
  for (int i = 0; i < SIFT_OB; ++i) {
    const float a = (hs[(i + SIFT_OB - 2) % SIFT_OB] + hs[(i + 2) % SIFT_OB]);
    const float b = (hs[(i + SIFT_OB - 1) % SIFT_OB] + hs[(i + 1) % SIFT_OB]);
    sm[i] = (((a * 1.f / 16.f) + (b * 4.f / 16.f)) + (hs[i] * 6.f / 16.f));
  }
  float omax = sm[0];
  for (int i = 1; i < SIFT_OB; ++i) omax = fmaxf(omax, sm[i]);
  const float thr = (omax * 0.8f);
  const double scale = ldexp(1.0, cd.o - 1);
  const float px = (float)((cd.c + cd.xc) * scale), py = (float)((cd.r + cd.xr) * scale);
  const float size = (float)(SIFT_SIG * pow(2.0, (cd.l + cd.xi) / SIFT_S) * ldexp(1.0, cd.o) * 2 * 0.5);
  for (int j = 0; j < SIFT_OB; ++j) {
    const float lf = sm[(j + SIFT_OB - 1) % SIFT_OB], rg = sm[(j + 1) % SIFT_OB];
    if (!(sm[j] > lf && sm[j] > rg && sm[j] >= thr)) continue;
    float bn = ((float)j + (0.5f * ((lf - rg) / ((lf - (2.f * sm[j])) + rg))));
    bn = bn < 0.f ? (bn + (float)SIFT_OB) : (bn >= (float)SIFT_OB ? (bn - (float)SIFT_OB) : bn);
    float ang = (360.f - ((float)(360.0 / SIFT_OB) * bn));
    if (fabsf((ang - 360.f)) < 1.2e-7f) ang = 0.f;
    const int k = atomicAdd(n_kp, 1);
    if (k < cap) kp[k] = SiftKp{px, py, size, ang, (float)fabs(cd.contr), (float)scl, cd.o, cd.l, cd.r, cd.c, 0, 0};
  }
}

// one wave per keypoint: the descriptor (calcSIFTDescriptor's sampling and trilinear binning)
__global__ __launch_bounds__(256) void k_sift_descr(const SiftKp* __restrict__ kps, int n, const float* const* __restrict__ gauss,
                                                    const int* __restrict__ ow, const int* __restrict__ oh,
                                                    float* __restrict__ des) {
#pragma clang fp contract(off)
  __shared__ double hist[4][SIFT_HB];
  const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int q = blockIdx.x * 4 + wv;
  if (q >= n) return;
  const SiftKp k = kps[q];
  const int w = ow[k.o], h = oh[k.o];
  const float* img = gauss[k.o * (SIFT_S + 3) + k.l];
  const double s = ldexp(1.0, k.o - 1);
  const double xo = (double)k.x / s, yo = (double)k.y / s;
  double ori = 360.0 - (double)k.angle;
  if (fabs(ori - 360.0) < 1.2e-7) ori = 0.0;
  const double hist_w = 3.0 * (double)k.scl;
  int rad = (int)rint(hist_w * sqrt(2.0) * (SIFT_D + 1) * 0.5);
  rad = min(rad, (int)sqrt((double)h * h + (double)w * w));
  const double cos_t = cos(ori * (M_PI / 180.0)) / hist_w, sin_t = sin(ori * (M_PI / 180.0)) / hist_w;
  const int px = (int)rint(xo), py = (int)rint(yo);
  double* hs = hist[wv];
  for (int b = lane; b < SIFT_HB; b += 64) hs[b] = 0.0;
  __builtin_amdgcn_wave_barrier();
  const double es = -1.0 / (SIFT_D * SIFT_D * 0.5), bpr = SIFT_N / 360.0;
  const int side = 2 * rad + 1, ns = side * side;
  for (int sidx = lane; sidx < ns; sidx += 64) {
    const int i = sidx / side - rad, j = sidx % side - rad;
    const double c_rot = j * cos_t - i * sin_t, r_rot = j * sin_t + i * cos_t;
    const double rbin = r_rot + SIFT_D / 2 - 0.5, cbin = c_rot + SIFT_D / 2 - 0.5;
    const int r = py + i, c = px + j;
    if (!(rbin > -1 && rbin < SIFT_D && cbin > -1 && cbin < SIFT_D && r > 0 && r < h - 1 && c > 0 && c < w - 1)) continue;
    const double dx = (double)(img[(int64_t)r * w + c + 1] - img[(int64_t)r * w + c - 1]);
    const double dy = (double)(img[(int64_t)(r - 1) * w + c] - img[(int64_t)(r + 1) * w + c]);
    const double wgt = exp((c_rot * c_rot + r_rot * r_rot) * es);
    double o = atan2(dy, dx) * 57.29577951308232;
    if (o < 0) o = o + 360;
    const double mag = sqrt(dx * dx + dy * dy) * wgt;
    const double obin = (o - ori) * bpr;
    const int r0 = (int)floor(rbin), c0 = (int)floor(cbin);
    int o0 = (int)floor(obin);
    const double rb = rbin - r0, cb = cbin - c0, ob = obin - o0;
    o0 = o0 < 0 ? o0 + SIFT_N : (o0 >= SIFT_N ? o0 - SIFT_N : o0);
    for (int dr = 0; dr < 2; ++dr) {
      const double wr = dr ? rb : 1 - rb;
      for (int dc = 0; dc < 2; ++dc) {
        const double wc = dc ? cb : 1 - cb;
        for (int dO = 0; dO < 2; ++dO) {
          const double wo = dO ? ob : 1 - ob;
          atomicAdd(&hs[((r0 + 1 + dr) * (SIFT_D + 2) + (c0 + 1 + dc)) * (SIFT_N + 2) + o0 + dO], mag * wr * wc * wo);
        }
      }
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);
  __builtin_amdgcn_wave_barrier();
  // 128 values, two per lane: v = hist[i+1][j+1][k] (+ the wrapped bins n, n+1 for k = 0, 1)
  double v[2];
  for (int t = 0; t < 2; ++t) {
    const int e = lane * 2 + t, i = e / (SIFT_D * SIFT_N), j = (e / SIFT_N) % SIFT_D, kk = e % SIFT_N;
    const int base = ((i + 1) * (SIFT_D + 2) + (j + 1)) * (SIFT_N + 2);
    v[t] = hs[base + kk];
    if (kk < 2) v[t] += hs[base + SIFT_N + kk];
  }
  double ss = v[0] * v[0] + v[1] * v[1];
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  const double thr = sqrt(ss) * 0.2;
  v[0] = fmin(v[0], thr);
  v[1] = fmin(v[1], thr);
  ss = v[0] * v[0] + v[1] * v[1];
  for (int off = 32; off > 0; off >>= 1) ss += __shfl_xor(ss, off, 64);
  const double nrm = 512.0 / fmax(sqrt(ss), 1.2e-7);
  for (int t = 0; t < 2; ++t) des[(int64_t)q * 128 + lane * 2 + t] = (float)fmin(fmax(rint(v[t] * nrm), 0.0), 255.0);
}

}  // namespace ptzba

namespace {
// Device work buffers kept across calls (one set per device; grown, never shrunk; deliberately not freed at
// exit): a stream calls SIFT on every frame, and allocating ~0.5 GB of pyramid per call cost more than
// the kernels.
struct SiftWork {
  ptzba::DBuf dimg, dg, dd, dtmp, dk, dcand, dcnt, dkp, dptr, dow, doh, dsel, ddes;
  // the last call's image (host copy) and its oriented keypoints before the top-n cut: the pyramid in dg / dptr
  // belongs to it, so a call on the same image (a stream detects each frame with 500 features, then the same frame
  // again with 1500 when it becomes a keyframe) re-selects and computes descriptors only
  std::vector<uint8_t> last_img;
  int32_t last_w = 0, last_h = 0;
  std::vector<ptzba::SiftKp> last_kps;
  bool last_valid = false;
  // the blur kernels, octave sizes and level pointers uploaded for (width, height, pyramid buffer): constant per
  // stream, so a frame of the same size skips their four synchronous copies
  int32_t tab_w = 0, tab_h = 0;
  void* tab_p[5] = {};  // dg, dk, dow, doh, dptr when the tables were uploaded
  // pinned staging of the 8-bit image (the H2D copy is asynchronous; the call synchronises before it returns)
  uint8_t* pin = nullptr;
  size_t pin_cap = 0;
};
SiftWork& sift_work(int device) { return ptzba::work_for<SiftWork>(device); }  // under device_work_lock

std::vector<float> sift_kernel(double sigma) {
  int k = (int)std::nearbyint(sigma * 8 + 1) | 1;
  const int r = k / 2;
  std::vector<double> w(k);
  double s = 0;
  for (int i = 0; i < k; ++i) {
    const double x = i - r;
    w[i] = std::exp(-x * x / (2.0 * sigma * sigma));
    s += w[i];
  }
  std::vector<float> f(k);
  for (int i = 0; i < k; ++i) f[i] = (float)(w[i] / s);
  return f;
}
}  // namespace

int ptz_sift(int device, int32_t width, int32_t height, const uint8_t* img, int32_t nfeatures, int32_t max_kp,
             float* kp_out, float* response_out, float* des_out, int32_t* n_out) {
  using namespace ptzba;
  if (width < 8 || height < 8 || !img || !n_out) return fail("bad image");
  if (max_kp < 0 || (max_kp > 0 && (!kp_out || !des_out))) return fail("bad output buffers");
  if (select_device(device)) return -1;
  const int W0 = 2 * width, H0 = 2 * height;
  const int n_oct = (int)std::nearbyint(std::log2((double)std::min(W0, H0)) - 2);
  if (n_oct < 1) return fail("image too small");
  std::vector<int> ow(n_oct), oh(n_oct);
  std::vector<int64_t> goff(n_oct), doff(n_oct);
  int64_t gtot = 0, dtot = 0;
  for (int o = 0; o < n_oct; ++o) {
    ow[o] = o ? ow[o - 1] / 2 : W0;
    oh[o] = o ? oh[o - 1] / 2 : H0;
    if (ow[o] < 1 || oh[o] < 1) return fail("octave %d empty", o);
    goff[o] = gtot;
    doff[o] = dtot;
    gtot += (int64_t)ow[o] * oh[o] * (SIFT_S + 3);
    dtot += (int64_t)ow[o] * oh[o] * (SIFT_S + 2);
  }
  const double kf = std::pow(2.0, 1.0 / SIFT_S);
  std::vector<std::vector<float>> kern(SIFT_S + 3);
  kern[0] = sift_kernel(std::sqrt(std::max(SIFT_SIG * SIFT_SIG - 1.0, 0.01)));  // input blur 0.5, doubled
  size_t kmax = kern[0].size();
  for (int i = 1; i < SIFT_S + 3; ++i) {
    const double prev = std::pow(kf, i - 1) * SIFT_SIG;
    kern[i] = sift_kernel(std::sqrt((prev * kf) * (prev * kf) - prev * prev));
    kmax = std::max(kmax, kern[i].size());
  }
  if ((int)kmax / 2 > BLUR_RMAX) return fail("blur radius %d exceeds %d", (int)kmax / 2, BLUR_RMAX);
  const int CAP = 1 << 17;
  auto guard = device_work_lock(device);
  SiftWork& Wk = sift_work(device);
  DBuf &dimg = Wk.dimg, &dg = Wk.dg, &dd = Wk.dd, &dtmp = Wk.dtmp, &dk = Wk.dk, &dcand = Wk.dcand, &dcnt = Wk.dcnt;
  DBuf &dkp = Wk.dkp, &dptr = Wk.dptr, &dow = Wk.dow, &doh = Wk.doh, &dsel = Wk.dsel, &ddes = Wk.ddes;
  if (dimg.reserve((size_t)width * height) || dg.reserve((size_t)gtot * 4) || dd.reserve((size_t)dtot * 4) ||
      dtmp.reserve((size_t)W0 * H0 * 4) || dk.reserve((SIFT_S + 3) * kmax * 4) || dcand.reserve(CAP * sizeof(SiftCand)) ||
      dcnt.reserve(16) || dkp.reserve(CAP * sizeof(SiftKp)) || dptr.reserve(n_oct * (SIFT_S + 3) * sizeof(float*)) ||
      dow.reserve(n_oct * 4) || doh.reserve(n_oct * 4))
    return -1;
  // PTZ_SIFT_REUSE=0: always rebuild the pyramid (read per call; the reuse test compares both)
  const char* rue = getenv("PTZ_SIFT_REUSE");
  const bool reuse = !(rue && atoi(rue) == 0);
  const size_t img_bytes = (size_t)width * height;
  std::vector<SiftKp> kps;
  if (reuse && Wk.last_valid && Wk.last_w == width && Wk.last_h == height && std::memcmp(Wk.last_img.data(), img, img_bytes) == 0) {
    kps = Wk.last_kps;  // the same image as the last call: its pyramid and keypoints are still on hand
  } else {
    Wk.last_valid = false;
    if (Wk.pin_cap < img_bytes) {
      if (Wk.pin) (void)hipHostFree(Wk.pin);
      Wk.pin = nullptr;
      Wk.pin_cap = 0;
      HIPCHK(hipHostMalloc((void**)&Wk.pin, img_bytes, hipHostMallocDefault));
      Wk.pin_cap = img_bytes;
    }
    HIPCHK(hipStreamSynchronize(nullptr));  // (a previous call that failed midway may still be reading it)
    std::memcpy(Wk.pin, img, img_bytes);
    HIPCHK(hipMemcpyAsync(dimg.p, Wk.pin, img_bytes, hipMemcpyHostToDevice, nullptr));
    std::vector<float*> gptr(n_oct * (SIFT_S + 3));
    float* G = dg.as<float>();
    float* Dg = dd.as<float>();
    float* T = dtmp.as<float>();
    for (int o = 0; o < n_oct; ++o)
      for (int i = 0; i < SIFT_S + 3; ++i) gptr[o * (SIFT_S + 3) + i] = G + goff[o] + (int64_t)i * ow[o] * oh[o];
    void* const tabs[5] = {dg.p, dk.p, dow.p, doh.p, dptr.p};
    if (Wk.tab_w != width || Wk.tab_h != height || !std::equal(tabs, tabs + 5, Wk.tab_p)) {
      Wk.tab_w = 0;  // (stays invalid if a copy below fails)
      std::vector<float> kflat((SIFT_S + 3) * kmax, 0.f);
      for (int i = 0; i < SIFT_S + 3; ++i) std::copy(kern[i].begin(), kern[i].end(), kflat.begin() + i * kmax);
      HIPCHK(hipMemcpy(dk.p, kflat.data(), kflat.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(dow.p, ow.data(), n_oct * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(doh.p, oh.data(), n_oct * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(dptr.p, gptr.data(), gptr.size() * sizeof(float*), hipMemcpyHostToDevice));
      Wk.tab_w = width;
      Wk.tab_h = height;
      std::copy(tabs, tabs + 5, Wk.tab_p);
    }
    HIPCHK(hipMemsetAsync(dcnt.p, 0, 16, nullptr));
    auto blur = [&](int w, int h, const float* src, float* dst, int ki) {
      const int K = (int)kern[ki].size();
      hipLaunchKernelGGL(k_sift_blur_rows, dim3((unsigned)((w + BLUR_TX - 1) / BLUR_TX), (unsigned)h), dim3(BLUR_TX), 0,
                         nullptr, w, h, src, T, dk.as<float>() + ki * kmax, K);
      hipLaunchKernelGGL(k_sift_blur_cols_sw, dim3((unsigned)((w + BLUR_CT - 1) / BLUR_CT), (unsigned)((h + BLUR_CR - 1) / BLUR_CR)),
                         dim3(256), 0, nullptr, w, h, T, dst, dk.as<float>() + ki * kmax, K);
    };
    // base: doubled image, then the blur from the assumed input blur to sigma
    hipLaunchKernelGGL(k_sift_up, dim3((unsigned)((W0 + 127) / 128), (unsigned)H0), dim3(128), 0, nullptr, width, height,
                       dimg.as<uint8_t>(), gptr[1]);
    blur(W0, H0, gptr[1], gptr[0], 0);
    const float thr = (float)std::floor(0.5 * SIFT_CONTR / SIFT_S * 255);
    for (int o = 0; o < n_oct; ++o) {
      const int w = ow[o], h = oh[o];
      if (o > 0)
        hipLaunchKernelGGL(k_sift_down, dim3((unsigned)((w + 127) / 128), (unsigned)h), dim3(128), 0, nullptr, ow[o - 1],
                           gptr[(o - 1) * (SIFT_S + 3) + SIFT_S], w, h, gptr[o * (SIFT_S + 3)]);
      const int64_t np = (int64_t)w * h;
      for (int i = 1; i < SIFT_S + 3; ++i) blur(w, h, gptr[o * (SIFT_S + 3) + i - 1], gptr[o * (SIFT_S + 3) + i], i);
      hipLaunchKernelGGL(k_sift_dog, dim3((unsigned)((np * (SIFT_S + 2) + 255) / 256)), dim3(256), 0, nullptr, np,
                         G + goff[o], Dg + doff[o]);
      if (w > 2 * SIFT_BORDER && h > 2 * SIFT_BORDER)
        hipLaunchKernelGGL(k_sift_extrema, dim3((unsigned)((w - 2 * SIFT_BORDER + 63) / 64), (unsigned)(h - 2 * SIFT_BORDER), SIFT_S),
                           dim3(64), 0, nullptr, o, w, h, Dg + doff[o], thr, dcand.as<SiftCand>(), dcnt.as<int>(), CAP);
    }
    HIPCHK(hipGetLastError());
    int cnt[2];
    HIPCHK(hipMemcpy(cnt, dcnt.p, 8, hipMemcpyDeviceToHost));
    if (cnt[0] > CAP) return fail("%d SIFT extrema exceed the candidate list (%d)", cnt[0], CAP);
    const int nc = cnt[0];
    if (nc > 0)
      hipLaunchKernelGGL(k_sift_orient, dim3((unsigned)((nc + 3) / 4)), dim3(256), 0, nullptr, dcand.as<SiftCand>(),
                         dcnt.as<int>(), (const float* const*)dptr.p, dow.as<int>(), doh.as<int>(), dkp.as<SiftKp>(),
                         dcnt.as<int>() + 1, CAP);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(cnt, dcnt.p, 8, hipMemcpyDeviceToHost));
    if (cnt[1] > CAP) return fail("%d SIFT keypoints exceed the keypoint list (%d)", cnt[1], CAP);
    const int nk1 = cnt[1];
    kps.resize(nk1);
    if (nk1) HIPCHK(hipMemcpy(kps.data(), dkp.p, (size_t)nk1 * sizeof(SiftKp), hipMemcpyDeviceToHost));
    if (reuse) {
      Wk.last_img.assign(img, img + img_bytes);
      Wk.last_w = width;
      Wk.last_h = height;
      Wk.last_kps = kps;
      Wk.last_valid = true;
    }
  }
  const int nk = (int)kps.size();
  // strongest first (ties: y, x, angle, then detection order -- a total order, so selecting the first n and sorting
  // only them gives exactly the stable sort's first n)
  int n = nk;
  if (nfeatures > 0) n = std::min(n, (int)nfeatures);
  {
    std::vector<int> ord(nk);
    for (int i = 0; i < nk; ++i) ord[i] = i;
    auto before = [&](int ia, int ib) {
      const SiftKp &a = kps[ia], &b = kps[ib];
      if (a.response != b.response) return a.response > b.response;
      if (a.y != b.y) return a.y < b.y;
      if (a.x != b.x) return a.x < b.x;
      if (a.angle != b.angle) return a.angle < b.angle;
      return ia < ib;
    };
    if (n < nk) std::nth_element(ord.begin(), ord.begin() + n, ord.end(), before);
    std::sort(ord.begin(), ord.begin() + n, before);
    std::vector<SiftKp> top(n);
    for (int i = 0; i < n; ++i) top[i] = kps[ord[i]];
    kps.swap(top);
  }
  *n_out = n;
  n = std::min(n, (int)max_kp);
  if (n <= 0) return 0;
  if (dsel.reserve((size_t)n * sizeof(SiftKp)) || ddes.reserve((size_t)n * 128 * 4)) return -1;
  HIPCHK(hipMemcpy(dsel.p, kps.data(), (size_t)n * sizeof(SiftKp), hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_sift_descr, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, nullptr, dsel.as<SiftKp>(), n,
                     (const float* const*)dptr.p, dow.as<int>(), doh.as<int>(), ddes.as<float>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(des_out, ddes.p, (size_t)n * 128 * 4, hipMemcpyDeviceToHost));
  for (int i = 0; i < n; ++i) {
    kp_out[4 * i] = kps[i].x;
    kp_out[4 * i + 1] = kps[i].y;
    kp_out[4 * i + 2] = kps[i].size;
    kp_out[4 * i + 3] = kps[i].angle;
    if (response_out) response_out[i] = kps[i].response;
  }
  return 0;
}
