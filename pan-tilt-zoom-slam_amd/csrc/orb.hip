// ORB and LATCH detection + description on the GPU (image_process.detect_compute_orb and
// detect_compute_latch, image_process.py:105-155, which call cv.ORB_create(nfeatures) and
// cv.xfeatures2d.LATCH_create(64) with their defaults).  OpenCV is not part of this image, so this restates
// OpenCV's published ORB pipeline (opencv 3.4 features2d/orb.cpp, xfeatures2d/latch.cpp) with the same
// parameters; its two learned tables (ORB's bit_pattern_31 and LATCH's triplets) are not available and are
// replaced by generated ones (see orb_tables): descriptors follow the same construction but are not
// OpenCV's bits -- parity is against oracle/ptz_oracle.py's restatement (parity unpinned against cv2).
//
//   pyramid      8 levels, scale 1.2: level l is resized from level l-1 to round(w / 1.2^l) (bilinear,
//                11-bit fixed-point weights as OpenCV's 8-bit INTER_LINEAR; integer, so bit-exact)
//   FAST-9       threshold 20 on every level: score = the largest threshold at which the pixel is still a
//                corner (9 contiguous circle pixels all brighter or all darker), 3x3 non-maximum
//                suppression (strictly greater than all 8 neighbours), points closer than 31 px to the
//                level's border dropped; per level the 2 n_l best FAST scores are kept (ties at the cut
//                kept, as KeyPointsFilter::retainBest does)
//   Harris       7x7 block of Sobel products at each kept point (integer sums, the float response of
//                OpenCV's HarrisResponses: k = 0.04, scale (1 / (4 * 7 * 255))^4); per level the n_l best
//                responses are kept (ties at the cut kept); n_l = OpenCV's geometric split of nfeatures
//   orientation  intensity centroid over the radius-15 disc (OpenCV's umax rows): integer moments, angle =
//                atan2(m01, m10) in degrees [0, 360)
//   ORB bits     level image blurred 7x7, sigma 2 (reflect-101, 8-bit result); 256 point pairs rotated by
//                the angle, positions rounded half to even; bit i = I(p0) < I(p1), byte i / 8, bit i % 8
//   LATCH bits   the level-0 image blurred 13x13, sigma 2 (GaussianBlur(Size(0, 0), 2, 2)); points within
//                27 px (48 / 2 + 3) of the border dropped; 512 triplets (anchor, c1, c2) rotated by the
//                angle; bit = SSD(7x7 at anchor, 7x7 at c1) < SSD(anchor, c2); 64 bytes
// Output order: level ascending, then response descending, then y, x (OpenCV's order within a level is
// nth_element's, i.e. unspecified).  Keypoints are (x, y) * 1.2^l in level-0 pixels, size 31 * 1.2^l.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>

#include "../../include/ptzba.h"
#include "host_util.h"

namespace ptzba {
namespace {

constexpr int ORB_LEVELS = 8, ORB_EDGE = 31, ORB_HALF = 15, ORB_FAST_T = 20, ORB_PAIRS = 256;
constexpr int LATCH_BITS = 512, LATCH_HALF_SSD = 3, LATCH_BORDER = 48 / 2 + LATCH_HALF_SSD;
constexpr int BLUR_MAXK = 13;
constexpr float HARRIS_K = 0.04f;

__constant__ int8_t c_orb_pattern[ORB_PAIRS * 4];  // (x0, y0, x1, y1) per pair
__constant__ int8_t c_latch_trip[LATCH_BITS * 6];  // (ax, ay, c1x, c1y, c2x, c2y) per bit
__constant__ int c_umax[ORB_HALF + 2];
__constant__ float c_blur[2][BLUR_MAXK];  // ORB 7-tap, LATCH 13-tap Gaussian (sigma 2), centred

__device__ __host__ inline uint64_t orb_mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// The generated tables (host; oracle/ptz_oracle.py orb_tables repeats them).  ORB: each coordinate is the
// sum of four uniform integers in [-5, 5] (sigma ~6.3, BRIEF's Gaussian G II sampling for a 31-px patch),
// clipped to [-13, 13] as OpenCV's learned pattern is.  LATCH: points uniform in the radius-19 disc by
// rejection (rotated 7x7 windows stay inside the 48-px patch).
void orb_tables(std::vector<int8_t>& pattern, std::vector<int8_t>& trip) {
  pattern.resize(ORB_PAIRS * 4);
  uint64_t k = 0;
  for (int i = 0; i < ORB_PAIRS * 4; ++i) {
    int s = 0;
    for (int r = 0; r < 4; ++r) s += (int)(orb_mix64(0x0B5EEDull * 0x9E3779B97F4A7C15ull + (k++)) % 11) - 5;
    pattern[i] = (int8_t)std::max(-13, std::min(13, s));
  }
  trip.resize(LATCH_BITS * 6);
  uint64_t c = 0;
  for (int i = 0; i < LATCH_BITS * 3; ++i) {
    int x, y;
    do {
      x = (int)(orb_mix64(0x1A7C4ull * 0x9E3779B97F4A7C15ull + (c++)) % 39) - 19;
      y = (int)(orb_mix64(0x1A7C4ull * 0x9E3779B97F4A7C15ull + (c++)) % 39) - 19;
    } while (x * x + y * y > 19 * 19);
    trip[2 * i] = (int8_t)x;
    trip[2 * i + 1] = (int8_t)y;
  }
}

// OpenCV's circular-patch row ends (features2d/orb.cpp, made symmetric)
std::vector<int> orb_umax() {
  std::vector<int> umax(ORB_HALF + 2, 0);
  const int vmax = (int)std::floor(ORB_HALF * std::sqrt(2.f) / 2 + 1);
  const int vmin = (int)std::ceil(ORB_HALF * std::sqrt(2.f) / 2);
  for (int v = 0; v <= vmax; ++v) umax[v] = (int)std::lrint(std::sqrt((double)ORB_HALF * ORB_HALF - v * v));
  for (int v = ORB_HALF, v0 = 0; v >= vmin; --v) {
    while (umax[v0] == umax[v0 + 1]) ++v0;
    umax[v] = v0;
    ++v0;
  }
  return umax;
}

// cv::getGaussianKernel(n, sigma) in float (the sum is normalised in double)
std::vector<float> gauss_taps(int n, double sigma) {
  std::vector<double> w(n);
  double s = 0;
  for (int i = 0; i < n; ++i) {
    const double x = i - (n - 1) * 0.5;
    w[i] = std::exp(-x * x / (2 * sigma * sigma));
    s += w[i];
  }
  std::vector<float> f(BLUR_MAXK, 0.f);
  for (int i = 0; i < n; ++i) f[i] = (float)(w[i] / s);
  return f;
}

__device__ __forceinline__ int refl(int i, int n) {
  if (n == 1) return 0;
  while (i < 0 || i >= n) i = i < 0 ? -i : 2 * n - 2 - i;
  return i;
}

#pragma clang fp contract(off)
// bilinear resize of an 8-bit image, OpenCV INTER_LINEAR geometry (pixel centres) and 11-bit weights
__global__ void k_orb_resize(int sw, int sh, const uint8_t* __restrict__ src, int dw, int dh, uint8_t* __restrict__ dst) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= dw) return;
  const double fxs = ((double)x + 0.5) * ((double)sw / (double)dw) - 0.5;
  const double fys = ((double)y + 0.5) * ((double)sh / (double)dh) - 0.5;
  int x0 = (int)floor(fxs), y0 = (int)floor(fys);
  int ax = (int)rint((fxs - x0) * 2048.0), ay = (int)rint((fys - y0) * 2048.0);
  if (x0 < 0) { x0 = 0; ax = 0; }
  if (y0 < 0) { y0 = 0; ay = 0; }
  if (x0 >= sw - 1) { x0 = sw - 1; ax = 0; }
  if (y0 >= sh - 1) { y0 = sh - 1; ay = 0; }
  const int x1 = min(x0 + 1, sw - 1), y1 = min(y0 + 1, sh - 1);
  const int64_t r0 = (int64_t)y0 * sw, r1 = (int64_t)y1 * sw;
  const int t = src[r0 + x0] * (2048 - ax) + src[r0 + x1] * ax;
  const int b = src[r1 + x0] * (2048 - ax) + src[r1 + x1] * ax;
  dst[(int64_t)y * dw + x] = (uint8_t)((t * (2048 - ay) + b * ay + (1 << 21)) >> 22);
}

// separable Gaussian, reflect-101, fp32 in a fixed order, rounded to 8 bits (rows pass to fp32, columns to u8)
__global__ void k_orb_blur_rows(int w, int h, const uint8_t* __restrict__ src, float* __restrict__ tmp, int which, int n) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const int r = n / 2;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s = s + c_blur[which][i] * (float)src[(int64_t)y * w + refl(x + i - r, w)];
  tmp[(int64_t)y * w + x] = s;
}
__global__ void k_orb_blur_cols(int w, int h, const float* __restrict__ tmp, uint8_t* __restrict__ dst, int which, int n) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  const int r = n / 2;
  float s = 0.f;
  for (int i = 0; i < n; ++i) s = s + c_blur[which][i] * tmp[(int64_t)refl(y + i - r, h) * w + x];
  dst[(int64_t)y * w + x] = (uint8_t)min(255, max(0, (int)rintf(s)));
}
#pragma clang fp contract(on)

// FAST-9 score (0 = not a corner): the largest t for which 9 contiguous circle pixels are all < p - t or all
// > p + t, i.e. max over arcs of the arc's minimum of (p - I) resp. (I - p), minus one
__global__ void k_fast_score(int w, int h, const uint8_t* __restrict__ img, int thr, uint8_t* __restrict__ score) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x >= w) return;
  int s = 0;
  if (x >= 3 && y >= 3 && x < w - 3 && y < h - 3) {
    const int dx[16] = {0, 1, 2, 3, 3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1};
    const int dy[16] = {3, 3, 2, 1, 0, -1, -2, -3, -3, -3, -2, -1, 0, 1, 2, 3};
    const int p = img[(int64_t)y * w + x];
    int d[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) d[k] = p - (int)img[(int64_t)(y + dy[k]) * w + x + dx[k]];
    int a = -1000, b = -1000;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      int mn = 1000, mx = -1000;
#pragma unroll
      for (int m = 0; m < 9; ++m) {
        const int v = d[(k + m) & 15];
        mn = min(mn, v);
        mx = max(mx, v);
      }
      a = max(a, mn);   // darker arc: every p - I > t
      b = max(b, -mx);  // brighter arc: every I - p > t
    }
    const int t = max(a, b) - 1;
    s = t >= thr ? t : 0;
  }
  score[(int64_t)y * w + x] = (uint8_t)s;
}

struct OrbCand {
  int x, y, level, score;  // score: FAST, later replaced by index into the Harris list
};

__global__ void k_fast_nms(int w, int h, const uint8_t* __restrict__ score, int level, OrbCand* __restrict__ out,
                           int* __restrict__ cnt, int cap) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x, y = blockIdx.y;
  if (x < ORB_EDGE || y < ORB_EDGE || x >= w - ORB_EDGE || y >= h - ORB_EDGE) return;
  const int s = score[(int64_t)y * w + x];
  if (s == 0) return;
  for (int j = -1; j <= 1; ++j)
    for (int i = -1; i <= 1; ++i)
      if ((i || j) && score[(int64_t)(y + j) * w + x + i] >= s) return;
  const int k = atomicAdd(cnt, 1);
  if (k < cap) out[k] = OrbCand{x, y, level, s};
}

struct OrbLevels {
  const uint8_t* img[ORB_LEVELS];
  const uint8_t* blur[ORB_LEVELS];
  int w[ORB_LEVELS], h[ORB_LEVELS];
  float scale[ORB_LEVELS];  // (float) 1.2^l, computed in double on the host as OpenCV's getScale
};
float orb_scale(int l) { return (float)std::pow(1.2, (double)l); }

#pragma clang fp contract(off)
__global__ void k_orb_harris(OrbLevels L, const OrbCand* __restrict__ c, int n, float* __restrict__ resp) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const OrbCand q = c[k];
  const uint8_t* im = L.img[q.level];
  const int w = L.w[q.level];
  int a = 0, b = 0, cc = 0;
  for (int v = -3; v <= 3; ++v)
    for (int u = -3; u <= 3; ++u) {
      const uint8_t* p = im + (int64_t)(q.y + v) * w + q.x + u;
      const int ix = (p[1] - p[-1]) * 2 + (p[-w + 1] - p[-w - 1]) + (p[w + 1] - p[w - 1]);
      const int iy = (p[w] - p[-w]) * 2 + (p[w - 1] - p[-w - 1]) + (p[w + 1] - p[-w + 1]);
      a += ix * ix;
      b += iy * iy;
      cc += ix * iy;
    }
  const float sc = 1.f / (4 * 7 * 255.f), s4 = sc * sc * sc * sc;
  const float fa = (float)a, fb = (float)b, fc = (float)cc;
  resp[k] = (fa * fb - fc * fc - HARRIS_K * (fa + fb) * (fa + fb)) * s4;
}
#pragma clang fp contract(on)

// one wave per keypoint: intensity-centroid angle, then the descriptor bits (ORB pairs or LATCH triplets)
struct OrbKp {
  int x, y, level, pad;  // level pixel position
};
__global__ __launch_bounds__(256) void k_orb_describe(OrbLevels L, const OrbKp* __restrict__ kp, int n, int latch,
                                                      const uint8_t* __restrict__ lblur, int W0, int H0,
                                                      float* __restrict__ angle_out, uint8_t* __restrict__ des) {
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (wv >= n) return;
  const OrbKp q = kp[wv];
  const uint8_t* im = L.img[q.level];
  const int w = L.w[q.level];
  // moments: lane v + 15 takes row v (31 rows)
  long long m01 = 0, m10 = 0;
  if (lane < 2 * ORB_HALF + 1) {
    const int v = lane - ORB_HALF, d = c_umax[v < 0 ? -v : v];
    const uint8_t* row = im + (int64_t)(q.y + v) * w + q.x;
    for (int u = -d; u <= d; ++u) {
      m10 += (long long)u * row[u];
      m01 += (long long)v * row[u];
    }
  }
  for (int o = 32; o >= 1; o >>= 1) {
    m01 += __shfl_xor(m01, o, 64);
    m10 += __shfl_xor(m10, o, 64);
  }
  double ang = atan2((double)m01, (double)m10) * (180.0 / 3.14159265358979323846);
  if (ang < 0) ang += 360.0;
  const double rad = ang * (3.14159265358979323846 / 180.0), ca = cos(rad), sa = sin(rad);
  if (lane == 0) angle_out[wv] = (float)ang;
  auto rot = [&](int px, int py, int& ox, int& oy) {
    ox = (int)rint(px * ca - py * sa);
    oy = (int)rint(px * sa + py * ca);
  };
  if (!latch) {
    const uint8_t* bl = L.blur[q.level];
    // lane owns pairs lane, lane + 64, ..., (4 pairs); bit of pair i -> byte i / 8
    unsigned long long mask[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = lane + 64 * r;
      int x0, y0, x1, y1;
      rot(c_orb_pattern[4 * i], c_orb_pattern[4 * i + 1], x0, y0);
      rot(c_orb_pattern[4 * i + 2], c_orb_pattern[4 * i + 3], x1, y1);
      const int v0 = bl[(int64_t)(q.y + y0) * w + q.x + x0], v1 = bl[(int64_t)(q.y + y1) * w + q.x + x1];
      mask[r] = __ballot(v0 < v1);
    }
    if (lane < 32) {  // byte b = bits 8b..8b+7 of the 256-bit string
      const int r = lane / 8, sh = (lane % 8) * 8;
      des[(int64_t)wv * 32 + lane] = (uint8_t)((mask[r] >> sh) & 0xff);
    }
    return;
  }
  // LATCH on the blurred level-0 image at the rounded level-0 position
  const float X = (float)q.x * L.scale[q.level], Y = (float)q.y * L.scale[q.level];
  const int cx = (int)rintf(X), cy = (int)rintf(Y);
  unsigned long long mask[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int i = lane + 64 * r;
    int ax, ay, bx, by, ex, ey;
    rot(c_latch_trip[6 * i], c_latch_trip[6 * i + 1], ax, ay);
    rot(c_latch_trip[6 * i + 2], c_latch_trip[6 * i + 3], bx, by);
    rot(c_latch_trip[6 * i + 4], c_latch_trip[6 * i + 5], ex, ey);
    int s1 = 0, s2 = 0;
    for (int v = -LATCH_HALF_SSD; v <= LATCH_HALF_SSD; ++v)
      for (int u = -LATCH_HALF_SSD; u <= LATCH_HALF_SSD; ++u) {
        const int va = lblur[(int64_t)(cy + ay + v) * W0 + cx + ax + u];
        const int d1 = va - lblur[(int64_t)(cy + by + v) * W0 + cx + bx + u];
        const int d2 = va - lblur[(int64_t)(cy + ey + v) * W0 + cx + ex + u];
        s1 += d1 * d1;
        s2 += d2 * d2;
      }
    mask[r] = __ballot(s1 < s2);
  }
  (void)H0;
  const int r = lane / 8, sh = (lane % 8) * 8;
  des[(int64_t)wv * 64 + lane] = (uint8_t)((mask[r] >> sh) & 0xff);
}

struct OrbWork {
  DBuf tmp, score, cand, cnt, resp, kp, ang, des, lblur;
  DBuf lev[ORB_LEVELS], blur[ORB_LEVELS];
};

// OpenCV's per-level feature split (features2d/orb.cpp): geometric with factor 1 / scale
std::vector<int> orb_level_counts(int nfeatures) {
  std::vector<int> n(ORB_LEVELS);
  const double factor = 1.0 / 1.2;
  double nd = nfeatures * (1 - factor) / (1 - std::pow(factor, (double)ORB_LEVELS));
  int sum = 0;
  for (int l = 0; l < ORB_LEVELS - 1; ++l) {
    n[l] = (int)std::lrint(nd);
    sum += n[l];
    nd *= factor;
  }
  n[ORB_LEVELS - 1] = std::max(nfeatures - sum, 0);
  return n;
}

// KeyPointsFilter::retainBest: the m best, plus every point tied with the m-th (order: value desc, y, x)
template <typename T>
void retain_best(std::vector<T>& v, int m, float (*val)(const T&)) {
  std::stable_sort(v.begin(), v.end(), [&](const T& a, const T& b) {
    if (val(a) != val(b)) return val(a) > val(b);
    if (a.y != b.y) return a.y < b.y;
    return a.x < b.x;
  });
  if ((int)v.size() <= m) return;
  if (m <= 0) {
    v.clear();
    return;
  }
  const float cut = val(v[m - 1]);
  size_t e = m;
  while (e < v.size() && val(v[e]) >= cut) ++e;
  v.resize(e);
}

struct HostKp {
  int x, y, level;
  float fast, harris;
};

}  // namespace
}  // namespace ptzba

int ptz_orb(int device, int32_t width, int32_t height, const uint8_t* img, int32_t nfeatures, int32_t descriptor,
            int32_t max_kp, float* kp_out, uint8_t* des_out, int32_t* n_out) {
  using namespace ptzba;
  if (width < 2 * ORB_EDGE + 1 || height < 2 * ORB_EDGE + 1 || !img || !n_out) return fail("bad image (needs > 62 x 62)");
  if (nfeatures <= 0) return fail("nfeatures must be > 0");
  if (descriptor != 0 && descriptor != 1) return fail("descriptor must be 0 (ORB) or 1 (LATCH)");
  if (max_kp < 0 || (max_kp > 0 && (!kp_out || !des_out))) return fail("bad output buffers");
  if (select_device(device)) return -1;
  static std::once_flag once;
  static int init_rc = 0;
  std::call_once(once, [] {
    std::vector<int8_t> pat, trip;
    orb_tables(pat, trip);
    const std::vector<int> umax = orb_umax();
    std::vector<float> bl(2 * BLUR_MAXK);
    const std::vector<float> b7 = gauss_taps(7, 2.0), b13 = gauss_taps(13, 2.0);
    std::copy(b7.begin(), b7.end(), bl.begin());
    std::copy(b13.begin(), b13.end(), bl.begin() + BLUR_MAXK);
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_orb_pattern), pat.data(), pat.size()) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_latch_trip), trip.data(), trip.size()) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_umax), umax.data(), umax.size() * 4) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_blur), bl.data(), bl.size() * 4) != hipSuccess)
      init_rc = -1;
  });
  if (init_rc) return fail("ORB constant tables could not be uploaded");
  // level sizes as OpenCV: round(cols / scale) with the float scale
  int lw[ORB_LEVELS], lh[ORB_LEVELS];
  int nlev = 0;
  for (int l = 0; l < ORB_LEVELS; ++l) {
    const float sc = orb_scale(l);
    lw[l] = (int)std::lrint((float)width / sc);
    lh[l] = (int)std::lrint((float)height / sc);
    nlev = l + 1;
  }
  const std::vector<int> per = orb_level_counts(nfeatures);
  const int CAP = 1 << 18;
  auto guard = device_work_lock(device);
  OrbWork& Wk = work_for<OrbWork>(device);
  const size_t np = (size_t)width * height;
  if (Wk.tmp.reserve(np * 4) || Wk.score.reserve(np) || Wk.cand.reserve(CAP * sizeof(OrbCand)) || Wk.cnt.reserve(16))
    return -1;
  for (int l = 0; l < nlev; ++l)
    if (Wk.lev[l].reserve((size_t)lw[l] * lh[l]) || Wk.blur[l].reserve((size_t)lw[l] * lh[l])) return -1;
  HIPCHK(hipMemcpy(Wk.lev[0].p, img, np, hipMemcpyHostToDevice));
  OrbLevels L{};
  for (int l = 0; l < nlev; ++l) {
    if (l > 0)
      hipLaunchKernelGGL(k_orb_resize, dim3((unsigned)((lw[l] + 127) / 128), (unsigned)lh[l]), dim3(128), 0, nullptr,
                         lw[l - 1], lh[l - 1], Wk.lev[l - 1].as<uint8_t>(), lw[l], lh[l], Wk.lev[l].as<uint8_t>());
    L.img[l] = Wk.lev[l].as<uint8_t>();
    L.blur[l] = Wk.blur[l].as<uint8_t>();
    L.w[l] = lw[l];
    L.h[l] = lh[l];
    L.scale[l] = orb_scale(l);
  }
  HIPCHK(hipMemset(Wk.cnt.p, 0, 16));
  for (int l = 0; l < nlev; ++l) {
    if (lw[l] <= 2 * ORB_EDGE || lh[l] <= 2 * ORB_EDGE) continue;
    const dim3 g((unsigned)((lw[l] + 127) / 128), (unsigned)lh[l]);
    hipLaunchKernelGGL(k_fast_score, g, dim3(128), 0, nullptr, lw[l], lh[l], L.img[l], ORB_FAST_T, Wk.score.as<uint8_t>());
    hipLaunchKernelGGL(k_fast_nms, g, dim3(128), 0, nullptr, lw[l], lh[l], Wk.score.as<uint8_t>(), l, Wk.cand.as<OrbCand>(),
                       Wk.cnt.as<int>(), CAP);
  }
  HIPCHK(hipGetLastError());
  int nc = 0;
  HIPCHK(hipMemcpy(&nc, Wk.cnt.p, 4, hipMemcpyDeviceToHost));
  if (nc > CAP) return fail("%d FAST corners exceed the candidate list (%d)", nc, CAP);
  std::vector<OrbCand> cand(nc);
  if (nc) HIPCHK(hipMemcpy(cand.data(), Wk.cand.p, (size_t)nc * sizeof(OrbCand), hipMemcpyDeviceToHost));
  // per level: the 2 n_l best FAST scores (ties kept)
  std::vector<std::vector<HostKp>> lv(ORB_LEVELS);
  for (const OrbCand& c : cand) lv[c.level].push_back(HostKp{c.x, c.y, c.level, (float)c.score, 0.f});
  std::vector<OrbCand> keep;
  for (int l = 0; l < ORB_LEVELS; ++l) {
    retain_best<HostKp>(lv[l], 2 * per[l], [](const HostKp& k) { return k.fast; });
    for (const HostKp& k : lv[l]) keep.push_back(OrbCand{k.x, k.y, k.level, 0});
  }
  const int nk = (int)keep.size();
  std::vector<float> hr(nk);
  if (nk) {
    if (Wk.cand.reserve((size_t)nk * sizeof(OrbCand)) || Wk.resp.reserve((size_t)nk * 4)) return -1;
    HIPCHK(hipMemcpy(Wk.cand.p, keep.data(), (size_t)nk * sizeof(OrbCand), hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_orb_harris, dim3((unsigned)((nk + 255) / 256)), dim3(256), 0, nullptr, L, Wk.cand.as<OrbCand>(), nk,
                       Wk.resp.as<float>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpy(hr.data(), Wk.resp.p, (size_t)nk * 4, hipMemcpyDeviceToHost));
  }
  std::vector<HostKp> fin;
  {
    std::vector<std::vector<HostKp>> hv(ORB_LEVELS);
    for (int k = 0; k < nk; ++k) hv[keep[k].level].push_back(HostKp{keep[k].x, keep[k].y, keep[k].level, 0.f, hr[k]});
    for (int l = 0; l < ORB_LEVELS; ++l) {
      retain_best<HostKp>(hv[l], per[l], [](const HostKp& k) { return k.harris; });
      fin.insert(fin.end(), hv[l].begin(), hv[l].end());
    }
  }
  if (descriptor == 1) {  // LATCH drops points whose 48-px patch (+ SSD half window) leaves the image
    std::vector<HostKp> in;
    for (const HostKp& k : fin) {
      const float sc = orb_scale(k.level), X = (float)k.x * sc, Y = (float)k.y * sc;
      if (X >= LATCH_BORDER && Y >= LATCH_BORDER && X < width - LATCH_BORDER && Y < height - LATCH_BORDER) in.push_back(k);
    }
    fin.swap(in);
  }
  const int n = (int)fin.size();
  *n_out = n;
  const int m = std::min(n, (int)max_kp);
  if (m <= 0) return 0;
  const int nb = descriptor ? 64 : 32;
  std::vector<OrbKp> kq(m);
  for (int i = 0; i < m; ++i) kq[i] = OrbKp{fin[i].x, fin[i].y, fin[i].level, 0};
  if (Wk.kp.reserve((size_t)m * sizeof(OrbKp)) || Wk.ang.reserve((size_t)m * 4) || Wk.des.reserve((size_t)m * nb)) return -1;
  HIPCHK(hipMemcpy(Wk.kp.p, kq.data(), (size_t)m * sizeof(OrbKp), hipMemcpyHostToDevice));
  auto blur = [&](int w, int h, const uint8_t* src, uint8_t* dst, int which, int taps) {
    const dim3 g((unsigned)((w + 127) / 128), (unsigned)h);
    hipLaunchKernelGGL(k_orb_blur_rows, g, dim3(128), 0, nullptr, w, h, src, Wk.tmp.as<float>(), which, taps);
    hipLaunchKernelGGL(k_orb_blur_cols, g, dim3(128), 0, nullptr, w, h, Wk.tmp.as<float>(), dst, which, taps);
  };
  const uint8_t* lb = nullptr;
  if (descriptor == 0) {
    for (int l = 0; l < nlev; ++l) blur(lw[l], lh[l], L.img[l], Wk.blur[l].as<uint8_t>(), 0, 7);
  } else {
    if (Wk.lblur.reserve(np)) return -1;
    blur(width, height, L.img[0], Wk.lblur.as<uint8_t>(), 1, 13);
    lb = Wk.lblur.as<uint8_t>();
  }
  hipLaunchKernelGGL(k_orb_describe, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, nullptr, L, Wk.kp.as<OrbKp>(), m,
                     descriptor, lb, width, height, Wk.ang.as<float>(), Wk.des.as<uint8_t>());
  HIPCHK(hipGetLastError());
  std::vector<float> ang(m);
  HIPCHK(hipMemcpy(ang.data(), Wk.ang.p, (size_t)m * 4, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(des_out, Wk.des.p, (size_t)m * nb, hipMemcpyDeviceToHost));
  for (int i = 0; i < m; ++i) {
    const float sc = orb_scale(fin[i].level);
    kp_out[6 * i] = (float)fin[i].x * sc;
    kp_out[6 * i + 1] = (float)fin[i].y * sc;
    kp_out[6 * i + 2] = 31.f * sc;
    kp_out[6 * i + 3] = ang[i];
    kp_out[6 * i + 4] = fin[i].harris;
    kp_out[6 * i + 5] = (float)fin[i].level;
  }
  return 0;
}
