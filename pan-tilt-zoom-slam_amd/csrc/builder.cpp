// Correspondence -> packed-observation builder (host, native).  SURVEY §8f-2.
//
// The reference assembles the BA problem in Python loops (image_process.py:568-667,
// bundle_adjustment.py:167-197, 214-248).  Three of its steps carry interpreter-defined ordering that the
// results depend on bit for bit; they are reproduced here exactly, so a native build is a drop-in:
//
//   * the 200-match cap draws `random.shuffle` from the GLOBAL Mersenne Twister (image_process.py:592-597):
//     ptz_py_shuffle_prefix replays CPython's shuffle / _randbelow / getrandbits on that generator's
//     state (random.getstate() in, random.setstate() out);
//   * keyframe features are the iteration order of `set(pairs)` over (local, global) tuples
//     (bundle_adjustment.py:222-239): ptz_keyframe_features inserts the same tuple sequence into an
//     open-addressing table with CPython's tuple hash (xxHash lanes, 3.8+) and set probing (linear
//     probes + perturbation, resize policy), then reads the table in slot order;
//   * x0 rays come from the src observation of the LAST match of each landmark (bundle_adjustment.py:
//     186-195): ptz_pack_records reports that record per landmark while packing.
//
// Python verifies the two interpreter-defined emulations against the live interpreter once per process
// (correspondence.py:_self_check) and uses the interpreter itself if they ever disagree.
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <vector>

#include "../../include/ptzba.h"
#include "host_util.h"

using ptzba::fail;

namespace {

// ---- MT19937 exactly as CPython's _randommodule.c (genrand_uint32) ----
constexpr int MT_N = 624, MT_M = 397;

struct MT {
  uint32_t s[MT_N];
  uint32_t t[MT_N];  // the tempered outputs of the current block (formed in one vectorisable pass per twist)
  int idx;
  void twist() {
    int kk = 0;
    for (; kk < MT_N - MT_M; kk++) {
      const uint32_t y = (s[kk] & 0x80000000u) | (s[kk + 1] & 0x7fffffffu);
      s[kk] = s[kk + MT_M] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    for (; kk < MT_N - 1; kk++) {
      const uint32_t y = (s[kk] & 0x80000000u) | (s[kk + 1] & 0x7fffffffu);
      s[kk] = s[kk + (MT_M - MT_N)] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
    }
    const uint32_t y = (s[MT_N - 1] & 0x80000000u) | (s[0] & 0x7fffffffu);
    s[MT_N - 1] = s[MT_M - 1] ^ (y >> 1) ^ ((0u - (y & 1u)) & 0x9908b0dfu);
  }
  void temper_from(int i0) {
    for (int i = i0; i < MT_N; ++i) {
      uint32_t y = s[i];
      y ^= (y >> 11);
      y ^= (y << 7) & 0x9d2c5680u;
      y ^= (y << 15) & 0xefc60000u;
      y ^= (y >> 18);
      t[i] = y;
    }
  }
  // state as CPython keeps it (mt[624], index); `t` is derived
  void load(const uint32_t* st, int index) {
    memcpy(s, st, sizeof(s));
    idx = index;
    if (idx < MT_N) temper_from(idx);
  }
  __attribute__((always_inline)) inline uint32_t next() {
    if (__builtin_expect(idx >= MT_N, 0)) {
      twist();
      temper_from(0);
      idx = 0;
    }
    return t[idx++];
  }
  // Random._randbelow_with_getrandbits(n), n < 2^31: k = n.bit_length(); r = getrandbits(k) until r < n
  uint32_t below(uint32_t n) {
    const int k = 32 - __builtin_clz(n);
    uint32_t r;
    do {
      r = next() >> (32 - k);
    } while (r >= n);
    return r;
  }
};

// ---- CPython 3.8+ tuple hash of a 2-tuple of non-negative ints (< 2^61 - 1, so hash(int) == int) ----
inline uint64_t tuple2_hash(uint64_t a, uint64_t b) {
  const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P5 = 2870177450012600261ull;
  uint64_t acc = P5;
  acc += a * P2;
  acc = (acc << 31) | (acc >> 33);
  acc *= P1;
  acc += b * P2;
  acc = (acc << 31) | (acc >> 33);
  acc *= P1;
  acc += 2ull ^ (P5 ^ 3527539ull);
  if (acc == ~0ull) return 1546275796ull;
  return acc;
}

// ---- CPython set (Objects/setobject.c): insertion-only table, iteration = slot order ----
// A slot is (a, b) as two int32 (a < 0: empty; the hash is recomputed when a resize re-inserts), the two table
// buffers are reused across sets and resizes, and a table is cleared with one memset: a 30-keyframe window's
// per-keyframe sets (~6 resizes each, up to 32K slots) cost ~0.1 us per insert instead of ~50 (r04 host bench).
struct PySetEmu {
  static constexpr size_t LINEAR_PROBES = 9, PERTURB_SHIFT = 5, MINSIZE = 8;
  struct Slot {
    int32_t a, b;
  };
  std::vector<Slot> buf[2];
  Slot* t = nullptr;  // the current table: buf[cur]
  int cur = 0;
  size_t mask = MINSIZE - 1, fill = 0;

  static Slot* clear(std::vector<Slot>& v, size_t n) {
    if (v.size() < n) v.resize(n);
    memset(v.data(), 0xff, n * sizeof(Slot));  // a = b = -1
    return v.data();
  }
  void reset() {
    t = clear(buf[cur], MINSIZE);
    mask = MINSIZE - 1;
    fill = 0;
  }
  static void insert_clean(Slot* tab, size_t m, const Slot& e) {
    const uint64_t h = tuple2_hash((uint64_t)e.a, (uint64_t)e.b);
    size_t perturb = h, i = h & m;
    for (;;) {
      if (tab[i].a < 0) {
        tab[i] = e;
        return;
      }
      if (i + LINEAR_PROBES <= m) {
        for (size_t j = 1; j <= LINEAR_PROBES; ++j)
          if (tab[i + j].a < 0) {
            tab[i + j] = e;
            return;
          }
      }
      perturb >>= PERTURB_SHIFT;
      i = (i * 5 + 1 + perturb) & m;
    }
  }
  void resize(size_t minused) {
    size_t ns = MINSIZE;
    while (ns <= minused) ns <<= 1;
    Slot* nt = clear(buf[cur ^ 1], ns);
    for (size_t k = 0; k <= mask; ++k)
      if (t[k].a >= 0) insert_clean(nt, ns - 1, t[k]);
    cur ^= 1;
    t = nt;
    mask = ns - 1;
  }
  // a, b in [0, 2^31)
  void add(int64_t a64, int64_t b64) {
    const int32_t a = (int32_t)a64, b = (int32_t)b64;
    const uint64_t h = tuple2_hash((uint64_t)a64, (uint64_t)b64);
    size_t i = h & mask, perturb = h;
    size_t slot;
    if (t[i].a < 0) {
      slot = i;
    } else {
      for (;;) {
        if (t[i].a == a && t[i].b == b) return;  // already present (equal tuples: equal hashes)
        bool found = false;
        if (i + LINEAR_PROBES <= mask) {
          for (size_t j = 1; j <= LINEAR_PROBES; ++j) {
            const Slot& e = t[i + j];
            if (e.a < 0) {
              slot = i + j;
              found = true;
              break;
            }
            if (e.a == a && e.b == b) return;
          }
        }
        if (found) break;
        perturb >>= PERTURB_SHIFT;
        i = (i * 5 + 1 + perturb) & mask;
        if (t[i].a < 0) {
          slot = i;
          break;
        }
      }
    }
    t[slot] = Slot{a, b};
    ++fill;  // no deletions: fill == used
    if (fill * 5 < mask * 3) return;
    resize(fill > 50000 ? fill * 2 : fill * 4);
  }
};

}  // namespace

extern "C" {

int ptz_py_shuffle_prefix(uint32_t* mt_state, int64_t n_lists, const int64_t* lens, int64_t keep,
                          int64_t* out) {
  if (!mt_state || n_lists < 0 || keep < 0) return fail("ptz_py_shuffle_prefix: bad arguments");
  if (mt_state[MT_N] > (uint32_t)MT_N) return fail("ptz_py_shuffle_prefix: bad generator index");
  MT g;
  g.load(mt_state, (int)mt_state[MT_N]);
  std::vector<int64_t> perm;
  int64_t o = 0;
  for (int64_t l = 0; l < n_lists; ++l) {
    const int64_t n = lens[l];
    if (n < 0 || n >= (int64_t)1 << 31) return fail("ptz_py_shuffle_prefix: list %lld length %lld", (long long)l,
                                                    (long long)n);
    perm.resize((size_t)n);
    for (int64_t k = 0; k < n; ++k) perm[k] = k;
    // random.shuffle: for i in reversed(range(1, len(x))): j = _randbelow(i + 1); swap
    for (int64_t i = n - 1; i >= 1; --i) {
      const int64_t j = g.below((uint32_t)(i + 1));
      const int64_t t = perm[i];
      perm[i] = perm[j];
      perm[j] = t;
    }
    const int64_t m = n < keep ? n : keep;
    for (int64_t k = 0; k < m; ++k) out[o + k] = perm[k];
    o += m;
  }
  memcpy(mt_state, g.s, sizeof(g.s));
  mt_state[MT_N] = (uint32_t)g.idx;
  return 0;
}

int ptz_set_order_pairs(int64_t n, const int64_t* a, const int64_t* b, int64_t* out_a, int64_t* out_b,
                        int64_t* n_out) {
  PySetEmu s;
  s.reset();
  for (int64_t k = 0; k < n; ++k) {
    if (a[k] < 0 || b[k] < 0) return fail("ptz_set_order_pairs: negative value");
    if (a[k] > INT32_MAX || b[k] > INT32_MAX) return fail("ptz_set_order_pairs: value above 2^31 - 1");
    s.add(a[k], b[k]);
  }
  int64_t o = 0;
  for (size_t k = 0; k <= s.mask; ++k)
    if (s.t[k].a >= 0) {
      out_a[o] = s.t[k].a;
      out_b[o] = s.t[k].b;
      ++o;
    }
  *n_out = o;
  return 0;
}

int ptz_keyframe_features(int32_t n_frames, int64_t n_matches, const int32_t* m_i, const int32_t* m_j,
                          const int64_t* k1, const int64_t* k2, const int64_t* lm, int64_t* out_off,
                          int64_t* out_local, int64_t* out_global) {
  if (n_frames < 0 || n_matches < 0) return fail("ptz_keyframe_features: bad sizes");
  // matches must be in the reference's pair order: (i, j) lexicographic, i < j
  for (int64_t k = 0; k < n_matches; ++k) {
    if (m_i[k] < 0 || m_j[k] >= n_frames || m_i[k] >= m_j[k])
      return fail("ptz_keyframe_features: match %lld has bad frames (%d, %d)", (long long)k, m_i[k], m_j[k]);
    if (k && (m_i[k] < m_i[k - 1] || (m_i[k] == m_i[k - 1] && m_j[k] < m_j[k - 1])))
      return fail("ptz_keyframe_features: matches not in (i, j) order at %lld", (long long)k);
    if (k1[k] < 0 || k2[k] < 0 || lm[k] < 0) return fail("ptz_keyframe_features: negative index at %lld",
                                                          (long long)k);
    if (k1[k] > INT32_MAX || k2[k] > INT32_MAX || lm[k] > INT32_MAX)
      return fail("ptz_keyframe_features: index above 2^31 - 1 at %lld", (long long)k);
  }
  // src role of frame f: matches with m_i == f (contiguous, j ascending); dst role: matches with
  // m_j == f in global order (= m_i ascending) -> stable counting sort by m_j
  std::vector<int64_t> src_off(n_frames + 1, 0), dst_off(n_frames + 1, 0), dst_list(n_matches);
  for (int64_t k = 0; k < n_matches; ++k) {
    src_off[m_i[k] + 1]++;
    dst_off[m_j[k] + 1]++;
  }
  for (int f = 0; f < n_frames; ++f) {
    src_off[f + 1] += src_off[f];
    dst_off[f + 1] += dst_off[f];
  }
  {
    std::vector<int64_t> cur(dst_off.begin(), dst_off.end() - 1);
    for (int64_t k = 0; k < n_matches; ++k) dst_list[cur[m_j[k]]++] = k;
  }
  // the keyframes' sets are independent: host threads take keyframes from a shared counter, each keeps its own
  // table, and the per-keyframe lists are concatenated in keyframe order (the same output as one thread)
  std::vector<std::vector<int32_t>> res(n_frames);
  std::atomic<int> next{0};
  auto work = [&] {
    PySetEmu s;
    for (int f; (f = next.fetch_add(1)) < n_frames;) {
      s.reset();
      for (int64_t k = src_off[f]; k < src_off[f + 1]; ++k) s.add(k1[k], lm[k]);
      for (int64_t q = dst_off[f]; q < dst_off[f + 1]; ++q) {
        const int64_t k = dst_list[q];
        s.add(k2[k], lm[k]);
      }
      auto& r = res[f];
      r.reserve(2 * s.fill);
      for (size_t k = 0; k <= s.mask; ++k)
        if (s.t[k].a >= 0) {
          r.push_back(s.t[k].a);
          r.push_back(s.t[k].b);
        }
    }
  };
  const int T = (int)std::min<int64_t>({(int64_t)n_frames, 16, 1 + n_matches / 16384,
                                         (int64_t)std::max(1u, std::thread::hardware_concurrency())});
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  int64_t o = 0;
  out_off[0] = 0;
  for (int f = 0; f < n_frames; ++f) {
    const auto& r = res[f];
    for (size_t q = 0; q < r.size(); q += 2) {
      out_local[o] = r[q];
      out_global[o] = r[q + 1];
      ++o;
    }
    out_off[f + 1] = o;
  }
  return 0;
}

// Number of distinct (local keypoint, landmark) pairs per keyframe -- len() of ptz_keyframe_features' per-keyframe
// lists without their set() order (bundle_adjustment.py:238's verbose print).  Keyframes over host threads; per
// keyframe a keypoint map gives the count directly (first-seen landmark ids give a keypoint one landmark unless the
// matching was inconsistent), and only a keyframe with a keypoint seen under two landmarks sorts its pairs.
int ptz_keyframe_feature_counts(int32_t n_frames, int64_t n_matches, const int32_t* m_i, const int32_t* m_j,
                                const int64_t* k1, const int64_t* k2, const int64_t* lm, int64_t* counts_out) {
  if (n_frames < 0 || n_matches < 0) return fail("ptz_keyframe_feature_counts: bad sizes");
  int64_t kmax = 0;
  for (int64_t k = 0; k < n_matches; ++k) {
    if (m_i[k] < 0 || m_i[k] >= n_frames || m_j[k] < 0 || m_j[k] >= n_frames || k1[k] < 0 || k2[k] < 0 || lm[k] < 0 ||
        k1[k] > INT32_MAX || k2[k] > INT32_MAX || lm[k] > INT32_MAX)
      return fail("ptz_keyframe_feature_counts: match %lld out of range", (long long)k);
    kmax = std::max(kmax, std::max(k1[k], k2[k]));
  }
  // a window's keyframes (cells of one frame x keypoint table fit 64 MiB): one sequential pass over the matches
  // marks each (keyframe, keypoint) cell with its first landmark and counts it; a side whose keypoint already carries
  // another landmark (inconsistent matching) is set aside as (cell, first landmark) and (cell, landmark), and those
  // are deduplicated in one open-addressing table: every distinct (cell, landmark) beyond the cell's first is one
  // more pair of its keyframe (no sort: the container's branchy sorts of ~15K triples cost more than the pass)
  if ((int64_t)n_frames * (kmax + 1) <= ((int64_t)1 << 24)) {
    const int64_t kw = kmax + 1;
    std::vector<int32_t> tab((size_t)n_frames * kw, -1);
    std::vector<uint64_t> ex;  // cell << 32 | landmark
    for (int f = 0; f < n_frames; ++f) counts_out[f] = 0;
    for (int64_t k = 0; k < n_matches; ++k) {
      const int32_t l = (int32_t)lm[k];
      const size_t c1 = (size_t)m_i[k] * kw + k1[k], c2 = (size_t)m_j[k] * kw + k2[k];
      int32_t& a1 = tab[c1];
      if (a1 < 0) {
        a1 = l;
        ++counts_out[m_i[k]];
      } else if (a1 != l) {
        ex.push_back(((uint64_t)c1 << 32) | (uint32_t)a1);
        ex.push_back(((uint64_t)c1 << 32) | (uint32_t)l);
      }
      int32_t& a2 = tab[c2];
      if (a2 < 0) {
        a2 = l;
        ++counts_out[m_j[k]];
      } else if (a2 != l) {
        ex.push_back(((uint64_t)c2 << 32) | (uint32_t)a2);
        ex.push_back(((uint64_t)c2 << 32) | (uint32_t)l);
      }
    }
    if (!ex.empty()) {
      size_t hs = 16;
      while (hs < 2 * ex.size()) hs <<= 1;
      std::vector<uint64_t> h(hs, ~0ull);
      for (const uint64_t key : ex) {
        size_t i = (size_t)((key * 0x9E3779B97F4A7C15ull) >> 20) & (hs - 1);
        while (h[i] != ~0ull && h[i] != key) i = (i + 1) & (hs - 1);
        if (h[i] == key) continue;
        h[i] = key;  // a new (cell, landmark)
        const size_t cell = (size_t)(key >> 32);
        const int f = (int)(cell / (size_t)kw);
        if (tab[cell] != -2) {  // the cell's first distinct landmark is already counted
          tab[cell] = -2;
        } else {
          ++counts_out[f];
        }
      }
    }
    return 0;
  }
  // per keyframe its (keypoint, landmark) sides: a counting sort of the 2 n_matches sides by keyframe
  std::vector<int64_t> off(n_frames + 1, 0);
  for (int64_t k = 0; k < n_matches; ++k) {
    off[m_i[k] + 1]++;
    off[m_j[k] + 1]++;
  }
  for (int f = 0; f < n_frames; ++f) off[f + 1] += off[f];
  std::vector<uint64_t> key(2 * (size_t)n_matches);  // keypoint << 32 | landmark
  {
    std::vector<int64_t> cur(off.begin(), off.end() - 1);
    for (int64_t k = 0; k < n_matches; ++k) {
      key[cur[m_i[k]]++] = ((uint64_t)k1[k] << 32) | (uint64_t)lm[k];
      key[cur[m_j[k]]++] = ((uint64_t)k2[k] << 32) | (uint64_t)lm[k];
    }
  }
  const bool mapped = kmax < ((int64_t)1 << 26);  // keypoint map per thread: (kmax + 1) int32
  std::atomic<int> next{0};
  auto work = [&] {
    std::vector<int32_t> lm_of(mapped ? (size_t)kmax + 1 : 0, -1);
    for (int f; (f = next.fetch_add(1)) < n_frames;) {
      uint64_t* b = key.data() + off[f];
      uint64_t* e = key.data() + off[f + 1];
      bool conflict = !mapped;
      int64_t c = 0;
      if (mapped) {
        for (uint64_t* p = b; p < e && !conflict; ++p) {
          int32_t& m = lm_of[(size_t)(*p >> 32)];
          const int32_t l = (int32_t)(*p & 0xffffffffu);
          if (m < 0) {
            m = l;
            ++c;
          } else if (m != l) {
            conflict = true;
          }
        }
        for (uint64_t* p = b; p < e; ++p) lm_of[(size_t)(*p >> 32)] = -1;  // reset for the next keyframe
      }
      if (conflict) {
        std::sort(b, e);
        c = std::unique(b, e) - b;
      }
      counts_out[f] = c;
    }
  };
  const int T = (int)std::min<int64_t>({(int64_t)n_frames, 16, 1 + n_matches / 16384,
                                         (int64_t)std::max(1u, std::thread::hardware_concurrency())});
  std::vector<std::thread> th;
  for (int t = 1; t < T; ++t) th.emplace_back(work);
  work();
  for (auto& x : th) x.join();
  return 0;
}

int ptz_pack_records(int32_t n_frames, int64_t n_matches, const int32_t* m_i, const int32_t* m_j,
                     const int64_t* k1, const int64_t* k2, const int64_t* lm, const int64_t* kp_off,
                     const double* kp_xy, int64_t n_landmark, int32_t* rec_frame, int32_t* rec_landmark,
                     double* rec_xy, int64_t* landmark_src_rec) {
  if (n_frames < 0 || n_matches < 0 || n_landmark < 0) return fail("ptz_pack_records: bad sizes");
  for (int64_t l = 0; l < n_landmark; ++l) landmark_src_rec[l] = -1;
  for (int64_t k = 0; k < n_matches; ++k) {
    const int i = m_i[k], j = m_j[k];
    if (i < 0 || i >= n_frames || j < 0 || j >= n_frames) return fail("ptz_pack_records: match %lld frame", (long long)k);
    const int64_t a = k1[k], b = k2[k], l = lm[k];
    if (a < 0 || a >= kp_off[i + 1] - kp_off[i] || b < 0 || b >= kp_off[j + 1] - kp_off[j])
      return fail("ptz_pack_records: match %lld keypoint out of range", (long long)k);
    if (l < 0 || l >= n_landmark) return fail("ptz_pack_records: match %lld landmark out of range", (long long)k);
    const double* p = kp_xy + 2 * (kp_off[i] + a);
    const double* q = kp_xy + 2 * (kp_off[j] + b);
    rec_frame[2 * k] = i;
    rec_frame[2 * k + 1] = j;
    rec_landmark[2 * k] = rec_landmark[2 * k + 1] = (int32_t)l;
    rec_xy[4 * k + 0] = p[0];
    rec_xy[4 * k + 1] = p[1];
    rec_xy[4 * k + 2] = q[0];
    rec_xy[4 * k + 3] = q[1];
    landmark_src_rec[l] = 2 * k;  // last writer wins
  }
  return 0;
}

}  // extern "C"
