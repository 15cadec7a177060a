// Synthetic multi-row keyframe grid (BASELINE configs[3]: 5000 keyframes x 200k rays in 10 tilt rows) --
// the input generator of the config-4 tests and bench, NOT part of the solver: it stands in for the
// camera + SIFT front-end (image_process.py:509-667) the way synthetic.py does for configs 1-3, and
// writes the reference's own pair-form data (bundle_adjustment.py:67-99 residual order).
//
// Same rules as synthetic.py: per-row pans linspace(lo, hi), tilt = row + U[-1, 1],
// f ~ U[2500, 3500]; rays theta ~ U[lo - 14, hi + 14], phi ~ U[min row - 7, max row + 7] (|phi| <= 80);
// visibility 0 < x < 1280, 0 < y < 720, q2 > 0; keypoint noise N(0, 0.5 px); initial poses frame 0
// exact, others + N(0, [0.5, 0.2, 40]); pairs i < j with overlap_pan_angle > 5 on the INITIAL poses
// (bundle_adjustment.py:135-144) and > 20 shared rays (image_process.py:590), capped at 200 matches
// per pair by a seeded shuffle; landmark ids by first occurrence in (i, j) pair order
// (image_process.py:611-639); ray init = from_image_to_ray of the last src observation with the
// initial pose (bundle_adjustment.py:184-194).
// The numpy generator needs ~6 minutes and ~35 GB for this size (one Python-level step per pair); this
// one is threaded and deterministic (per-frame / per-pair counter-based random streams, independent of
// the thread count).  Its random streams differ from numpy's, so the counts differ from a numpy run of
// the same spec by sampling noise only.
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr double DEG = M_PI / 180.0;

struct Rng {  // splitmix64 stream
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }
  double uni(double a, double b) { return a + (b - a) * uni(); }
  double normal() {  // Box-Muller (one value per call, the pair's second half is dropped)
    double u1 = uni();
    while (u1 <= 0) u1 = uni();
    const double u2 = uni();
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
  }
  uint64_t below(uint64_t n) { return next() % n; }
};

uint64_t mix(uint64_t a, uint64_t b, uint64_t c = 0) {
  Rng r(a * 0x9E3779B97F4A7C15ull ^ (b + 0x632BE59BD9B4E019ull) * 0xD1B54A32D192ED03ull ^ c * 0x8CB92BA72F3D8DD7ull);
  r.next();
  return r.next();
}

// closed-form BA projection (q form, |q2| in y: transformation.py:99-135)
inline void project(double u, double v, double f, double pan, double tilt, double th, double ph, double& x, double& y,
                    double& q2) {
  const double a = pan * DEG, b = tilt * DEG;
  const double p0 = std::tan(th * DEG);
  const double p1 = -std::tan(ph * DEG) * std::sqrt(p0 * p0 + 1.0);
  const double ca = std::cos(a), sa = std::sin(a), cb = std::cos(b), sb = std::sin(b);
  const double w0 = ca * p0 - sa, w2 = sa * p0 + ca;
  const double q1 = cb * p1 + sb * w2;
  q2 = -sb * p1 + cb * w2;
  x = u + f * w0 / q2;
  y = v + f * q1 / std::fabs(q2);
}

// back-projection (transformation.py:137-175), closed form
inline void image_to_ray(double u, double v, double f, double pan, double tilt, double x, double y, double& th,
                         double& ph) {
  const double a = pan * DEG, b = tilt * DEG;
  const double ca = std::cos(a), sa = std::sin(a), cb = std::cos(b), sb = std::sin(b);
  const double c0 = (x - u) / f, c1 = (y - v) / f;
  const double e0 = c0, e1 = cb * c1 - sb, e2 = sb * c1 + cb;
  const double d0 = ca * e0 + sa * e2, d1 = e1, d2 = -sa * e0 + ca * e2;
  th = std::atan(d0 / d2) / DEG;
  ph = std::atan(-d1 / std::sqrt(d0 * d0 + d2 * d2)) / DEG;
}

inline double overlap_pan(double f1, double p1, double f2, double p2, double width) {  // util.py:49-72
  const double w = width / 2.0;
  const double d1 = std::atan(w / f1) / DEG, d2 = std::atan(w / f2) / DEG;
  return std::max(0.0, std::min(p1 + d1, p2 + d2) - std::max(p1 - d1, p2 - d2));
}

template <typename F>
void parallel_for(int n, int threads, F&& fn) {
  std::atomic<int> next{0};
  std::vector<std::thread> pool;
  const int nt = std::max(1, std::min(threads, n));
  for (int t = 0; t < nt; ++t)
    pool.emplace_back([&] {
      for (int i; (i = next.fetch_add(1)) < n;) fn(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

struct ptzsynth_params {
  int32_t n_kf, n_rays, n_rows, threads;
  double pan_lo, pan_hi;
  const double* rows;  // [n_rows] row tilts (deg); frames are row-major: frame = row * (n_kf / n_rows) + k
  uint64_t seed;
  double noise, sig_pan, sig_tilt, sig_f;
  int32_t min_match, max_match;
  double overlap_deg;
};

struct ptzsynth_result {
  int64_t n_pose, n_landmark, n_rec, n_pairs;
  std::vector<int32_t> frame, landmark;
  std::vector<double> xy, init_ptz, gt_ptz, init_rays, gt_rays;
};

void* ptzsynth_grid_new(const ptzsynth_params* P) {
  if (!P || P->n_rows < 1 || P->n_kf < P->n_rows || P->n_rays < 1) return nullptr;
  const double U = 640.0, V = 360.0, W = 1280.0, H = 720.0;
  const int per = P->n_kf / P->n_rows, N = per * P->n_rows, M0 = P->n_rays;
  const int threads = std::max(1, P->threads);
  auto* R = new ptzsynth_result();
  // ---- cameras and rays (one sequential stream)
  Rng g(mix(P->seed, 1));
  std::vector<double> gt(3 * N), init(3 * N);
  double rmin = 1e9, rmax = -1e9;
  for (int r = 0; r < P->n_rows; ++r) {
    rmin = std::min(rmin, P->rows[r]);
    rmax = std::max(rmax, P->rows[r]);
    for (int k = 0; k < per; ++k) {
      const int f = r * per + k;
      gt[3 * f] = per > 1 ? P->pan_lo + (P->pan_hi - P->pan_lo) * k / (per - 1) : P->pan_lo;
      gt[3 * f + 1] = P->rows[r] + g.uni(-1.0, 1.0);
    }
  }
  for (int f = 0; f < N; ++f) gt[3 * f + 2] = g.uni(2500.0, 3500.0);
  const double phi_lo = std::max(rmin - 7.0, -80.0), phi_hi = std::min(rmax + 7.0, 80.0);
  std::vector<double> th(M0), ph(M0);
  for (int i = 0; i < M0; ++i) th[i] = g.uni(P->pan_lo - 14.0, P->pan_hi + 14.0);
  for (int i = 0; i < M0; ++i) ph[i] = g.uni(phi_lo, phi_hi);
  init = gt;
  const double sig[3] = {P->sig_pan, P->sig_tilt, P->sig_f};
  for (int f = 1; f < N; ++f)
    for (int c = 0; c < 3; ++c) init[3 * f + c] += g.normal() * sig[c];
  std::vector<int32_t> by_th(M0);
  for (int i = 0; i < M0; ++i) by_th[i] = i;
  std::stable_sort(by_th.begin(), by_th.end(), [&](int a, int b) { return th[a] < th[b]; });
  std::vector<double> th_sorted(M0);
  for (int i = 0; i < M0; ++i) th_sorted[i] = th[by_th[i]];

  // ---- keypoints per frame: visible rays in ascending ray id, projected with the TRUE pose + noise
  std::vector<std::vector<int32_t>> kray(N);
  std::vector<std::vector<double>> kxy(N);
  std::vector<double> box(4 * N);  // theta / phi range of the frame's visible rays
  parallel_for(N, threads, [&](int f) {
    const double pan = gt[3 * f], tilt = gt[3 * f + 1], fl = gt[3 * f + 2];
    const double b = tilt * DEG, c0 = std::max(U, W - U) / fl, c1 = std::max(V, H - V) / fl;
    const double den = std::cos(b) - std::fabs(std::sin(b)) * c1;
    std::vector<int32_t> cand;
    if (den <= 1e-3) {
      cand.resize(M0);
      for (int i = 0; i < M0; ++i) cand[i] = i;
    } else {
      const double half = std::atan(c0 / den) / DEG + 0.5;
      const auto lo = std::lower_bound(th_sorted.begin(), th_sorted.end(), pan - half) - th_sorted.begin();
      const auto hi = std::upper_bound(th_sorted.begin(), th_sorted.end(), pan + half) - th_sorted.begin();
      cand.assign(by_th.begin() + lo, by_th.begin() + hi);
      std::sort(cand.begin(), cand.end());
    }
    Rng rn(mix(P->seed, 2, (uint64_t)f));
    double tmin = 1e9, tmax = -1e9, pmin = 1e9, pmax = -1e9;
    for (int id : cand) {
      double x, y, q2;
      project(U, V, fl, pan, tilt, th[id], ph[id], x, y, q2);
      if (!(q2 > 0 && x > 0 && x < W && y > 0 && y < H)) continue;
      kray[f].push_back(id);
      kxy[f].push_back(x + rn.normal() * P->noise);
      kxy[f].push_back(y + rn.normal() * P->noise);
      tmin = std::min(tmin, th[id]); tmax = std::max(tmax, th[id]);
      pmin = std::min(pmin, ph[id]); pmax = std::max(pmax, ph[id]);
    }
    box[4 * f] = tmin; box[4 * f + 1] = tmax; box[4 * f + 2] = pmin; box[4 * f + 3] = pmax;
  });

  // ---- matched pairs (i < j), in (i, j) order; per pair the positions in frame i and frame j
  struct Pair { int32_t j; int64_t off; int32_t n; };
  std::vector<std::vector<Pair>> pairs(N);
  std::vector<std::vector<int32_t>> pidx(N);  // per frame i: (a, b) interleaved for its pairs
  parallel_for(N, threads, [&](int i) {
    std::vector<int32_t> a, b;
    for (int j = i + 1; j < N; ++j) {
      if (!(overlap_pan(init[3 * i + 2], init[3 * i], init[3 * j + 2], init[3 * j], W) > P->overlap_deg)) continue;
      if (box[4 * i] > box[4 * j + 1] || box[4 * j] > box[4 * i + 1] || box[4 * i + 2] > box[4 * j + 3] ||
          box[4 * j + 2] > box[4 * i + 3])
        continue;
      const auto &ri = kray[i], &rj = kray[j];
      a.clear();
      b.clear();
      for (size_t p = 0, q = 0; p < ri.size() && q < rj.size();) {
        if (ri[p] < rj[q]) ++p;
        else if (ri[p] > rj[q]) ++q;
        else { a.push_back((int32_t)p); b.push_back((int32_t)q); ++p; ++q; }
      }
      const int n = (int)a.size();
      if (n <= P->min_match) continue;
      int keep = n;
      if (n > P->max_match) {  // seeded shuffle, keep the first max_match (image_process.py:592-597)
        Rng rs(mix(P->seed, 3, ((uint64_t)i << 32) | (uint64_t)j));
        for (int k = n - 1; k > 0; --k) {
          const int s = (int)rs.below((uint64_t)k + 1);
          std::swap(a[k], a[s]);
          std::swap(b[k], b[s]);
        }
        keep = P->max_match;
      }
      pairs[i].push_back({j, (int64_t)pidx[i].size(), keep});
      for (int k = 0; k < keep; ++k) {
        pidx[i].push_back(a[k]);
        pidx[i].push_back(b[k]);
      }
    }
  });

  // ---- records in the reference residual order, first-seen landmark ids, last-writer ray init
  int64_t n_match = 0, n_pairs = 0;
  for (int i = 0; i < N; ++i) {
    n_pairs += (int64_t)pairs[i].size();
    n_match += (int64_t)pidx[i].size() / 2;
  }
  R->n_pose = N;
  R->n_pairs = n_pairs;
  R->n_rec = 2 * n_match;
  R->frame.resize(2 * n_match);
  R->landmark.resize(2 * n_match);
  R->xy.resize(4 * n_match);
  std::vector<int32_t> relabel(M0, -1), src_frame, src_kp, order_ray;
  int64_t m = 0;
  for (int i = 0; i < N; ++i) {
    for (const Pair& pr : pairs[i]) {
      const int j = pr.j;
      for (int k = 0; k < pr.n; ++k, ++m) {
        const int a = pidx[i][pr.off + 2 * k], b = pidx[i][pr.off + 2 * k + 1];
        const int ray = kray[i][a];
        int l = relabel[ray];
        if (l < 0) {
          l = relabel[ray] = (int32_t)order_ray.size();
          order_ray.push_back(ray);
          src_frame.push_back(i);
          src_kp.push_back(a);
        }
        src_frame[l] = i;  // last writer wins
        src_kp[l] = a;
        R->frame[2 * m] = i;
        R->frame[2 * m + 1] = j;
        R->landmark[2 * m] = l;
        R->landmark[2 * m + 1] = l;
        R->xy[4 * m] = kxy[i][2 * a];
        R->xy[4 * m + 1] = kxy[i][2 * a + 1];
        R->xy[4 * m + 2] = kxy[j][2 * b];
        R->xy[4 * m + 3] = kxy[j][2 * b + 1];
      }
    }
    std::vector<Pair>().swap(pairs[i]);
    std::vector<int32_t>().swap(pidx[i]);
  }
  const int M = (int)order_ray.size();
  R->n_landmark = M;
  R->gt_rays.resize(2 * (size_t)M);
  R->init_rays.resize(2 * (size_t)M);
  for (int l = 0; l < M; ++l) {
    R->gt_rays[2 * l] = th[order_ray[l]];
    R->gt_rays[2 * l + 1] = ph[order_ray[l]];
    const int f = src_frame[l], a = src_kp[l];
    image_to_ray(U, V, init[3 * f + 2], init[3 * f], init[3 * f + 1], kxy[f][2 * a], kxy[f][2 * a + 1],
                 R->init_rays[2 * l], R->init_rays[2 * l + 1]);
  }
  R->gt_ptz = std::move(gt);
  R->init_ptz = std::move(init);
  return R;
}

int ptzsynth_counts(void* h, int64_t* out4) {
  if (!h || !out4) return -1;
  auto* R = static_cast<ptzsynth_result*>(h);
  out4[0] = R->n_pose;
  out4[1] = R->n_landmark;
  out4[2] = R->n_rec;
  out4[3] = R->n_pairs;
  return 0;
}

// copies the problem into caller-owned arrays sized by ptzsynth_counts (any pointer may be null)
int ptzsynth_fetch(void* h, int32_t* frame, int32_t* landmark, double* xy, double* init_ptz, double* gt_ptz,
                   double* init_rays, double* gt_rays) {
  if (!h) return -1;
  auto* R = static_cast<ptzsynth_result*>(h);
  auto cp = [](void* dst, const auto& v) {
    if (dst && !v.empty()) std::memcpy(dst, v.data(), v.size() * sizeof(v[0]));
  };
  cp(frame, R->frame);
  cp(landmark, R->landmark);
  cp(xy, R->xy);
  cp(init_ptz, R->init_ptz);
  cp(gt_ptz, R->gt_ptz);
  cp(init_rays, R->init_rays);
  cp(gt_rays, R->gt_rays);
  return 0;
}

void ptzsynth_free(void* h) { delete static_cast<ptzsynth_result*>(h); }

}  // extern "C"
