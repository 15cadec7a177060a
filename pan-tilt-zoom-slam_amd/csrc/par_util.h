// Host-thread helpers for the O(records) passes of ptzba_set_problem (config 4: 410 M pair records): a chunked
// parallel-for and a stable parallel counting sort.  Plain std::thread, no HIP dependency; every result is
// identical to the sequential pass (the sort is stable, chunks are contiguous and combined in order).
#pragma once
#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <thread>
#include <vector>

namespace ptzba {

// worker threads for a pass over n items: at most 16 (the GPU box's CPU share per GPU), one per 256 K items (a config-5 window's ~170K records stay on one thread: 2 threads measured slower there,
// sort 0.6 -> 1.1 ms, segments 1.0 -> 1.5 ms, r04t)
inline int host_threads(int64_t n) {
  static const int cap = [] {
    int c = 16;
    const int hw = (int)std::thread::hardware_concurrency();
    if (hw > 0) c = std::min(c, hw);
    return std::max(1, c);
  }();
  return (int)std::max<int64_t>(1, std::min<int64_t>(cap, n >> 18));
}

// fn(lo, hi, t) over T contiguous chunks of [0, n), chunk t = [n t / T, n (t + 1) / T)
template <typename F>
inline void parallel_chunks(int64_t n, int T, F&& fn) {
  if (T <= 1) {
    fn((int64_t)0, n, 0);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(T - 1);
  for (int t = 1; t < T; ++t) th.emplace_back([&, t] { fn(n * t / T, n * (t + 1) / T, t); });
  fn((int64_t)0, n / T, 0);
  for (auto& x : th) x.join();
}

// Stable counting sort of the items in[0..n) (in == nullptr: the identity 0..n-1) by key(item) in [0, K): out[0..n)
// receives the items in (key, position in `in`) order -- exactly the sequential counting sort's result.
template <typename Key, typename Item = int64_t>
inline void parallel_counting_sort(int64_t n, int64_t K, const Item* in, Item* out, Key key) {
  const int T = host_threads(n);
  std::vector<std::vector<int64_t>> cnt(T, std::vector<int64_t>(K, 0));
  parallel_chunks(n, T, [&](int64_t lo, int64_t hi, int t) {
    int64_t* c = cnt[t].data();
    for (int64_t k = lo; k < hi; ++k) c[key(in ? in[k] : (Item)k)]++;
  });
  // bucket-major, then chunk order: the start of (bucket b, chunk t)
  int64_t run = 0;
  for (int64_t b = 0; b < K; ++b)
    for (int t = 0; t < T; ++t) {
      const int64_t c = cnt[t][b];
      cnt[t][b] = run;
      run += c;
    }
  parallel_chunks(n, T, [&](int64_t lo, int64_t hi, int t) {
    int64_t* c = cnt[t].data();
    for (int64_t k = lo; k < hi; ++k) {
      const Item item = in ? in[k] : (Item)k;
      out[c[key(item)]++] = item;
    }
  });
}

}  // namespace ptzba
