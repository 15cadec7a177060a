// GPU front of ptzba_set_problem for large problems (config 3's 14.6M and config 4's 410M pair records): the
// (landmark, frame, original record) order, the segment runs and the device-resident record arrays, built where
// they are used instead of by host passes over the records (round 4: 2.6 s of host sorting and segment scans at
// config 4, then a 6 GB pageable upload of the results).
//
//   setup_sort_runs      one stable LSD radix sort (rocPRIM) of the 32-bit composite key landmark * n_pose + frame with
//                        the record index as value -- exactly the order of the host's two stable counting sorts (by
//                        frame, then by landmark: ties keep the input order); run starts flagged and inclusive-scanned
//                        into the record -> segment map
//   setup_fill_segments  per segment its frame, landmark and first record (and the end record), the first segment of
//                        every landmark
//   setup_records        the per-segment base observation (fp64, the segment's first record), the records as deltas
//                        from it in the record precision, weights, K1's 1-byte window keys, the sorted -> original
//                        permutation
// The host keeps what its structure passes read (segment frame / landmark / first record); nothing here depends on
// the host's thread count, so the result is the same bit for bit as the host path's.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "host_util.h"
#include "ptzba_kernels.h"

namespace ptzba {

namespace {

__global__ void k_setup_keys(int64_t n, int n_pose, const int32_t* __restrict__ frame, const int32_t* __restrict__ lm,
                             uint32_t* __restrict__ key, uint32_t* __restrict__ idx) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    key[k] = (uint32_t)lm[k] * (uint32_t)n_pose + (uint32_t)frame[k];
    idx[k] = (uint32_t)k;
  }
}

__global__ void k_setup_flags(int64_t n, const uint32_t* __restrict__ key, int32_t* __restrict__ flag) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x)
    flag[k] = (k == 0 || key[k] != key[k - 1]) ? 1 : 0;
}

// rec_seg holds the inclusive scan of the run flags (1-based); it leaves as the 0-based segment id
__global__ void k_setup_segments(int64_t n, int n_pose, const uint32_t* __restrict__ key, int32_t* __restrict__ rec_seg,
                                 int32_t* __restrict__ seg_frame, int32_t* __restrict__ seg_lm,
                                 int64_t* __restrict__ seg_rec_begin) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = rec_seg[k] - 1;
    rec_seg[k] = s;
    if (k == 0 || key[k] != key[k - 1]) {
      seg_frame[s] = (int32_t)(key[k] % (uint32_t)n_pose);
      seg_lm[s] = (int32_t)(key[k] / (uint32_t)n_pose);
      seg_rec_begin[s] = k;
    }
    if (k == n - 1) seg_rec_begin[s + 1] = n;
  }
}

__global__ void k_setup_lm_first(int64_t n_seg, const int32_t* __restrict__ seg_lm, int32_t* __restrict__ lm_first) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_seg; s += (int64_t)gridDim.x * blockDim.x)
    if (s == 0 || seg_lm[s] != seg_lm[s - 1]) lm_first[seg_lm[s]] = (int32_t)s;
}

__global__ void k_setup_seg_base(int64_t n_seg, const uint32_t* __restrict__ order, const int64_t* __restrict__ seg_rec_begin,
                                 const double2* __restrict__ xy, double2* __restrict__ base) {
  for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < n_seg; s += (int64_t)gridDim.x * blockDim.x)
    base[s] = xy[order[seg_rec_begin[s]]];
}

template <typename real>
__global__ void k_setup_records(int64_t n, const uint32_t* __restrict__ order, const int32_t* __restrict__ rec_seg,
                                const int32_t* __restrict__ seg_lm, const int32_t* __restrict__ lm_first,
                                const double2* __restrict__ xy, const double* __restrict__ w, const double2* __restrict__ base,
                                real* __restrict__ rec_xy, real* __restrict__ rec_w, uint8_t* __restrict__ rec_key,
                                int64_t* __restrict__ perm) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t r = order[k];
    const int32_t s = rec_seg[k];
    const double2 o = xy[r], b = base[s];
    rec_xy[2 * k] = (real)(o.x - b.x);
    rec_xy[2 * k + 1] = (real)(o.y - b.y);
    if (w) rec_w[k] = (real)w[r];
    rec_key[k] = (uint8_t)((s - lm_first[seg_lm[s]]) % K1_SEGW);
    perm[k] = r;
  }
}

dim3 grid_for(int64_t n) { return dim3((unsigned)std::min<int64_t>((n + 255) / 256, 8192)); }

}  // namespace

int setup_sort_runs(hipStream_t st, int64_t n, int n_pose, int n_lm, const int32_t* frame, const int32_t* lm,
                    uint32_t* order, uint32_t* key_sorted, int32_t* rec_seg, int64_t* n_seg) {
  *n_seg = 0;
  if (n <= 0) return 0;
  DBuf key_in, idx_in, temp;
  if (key_in.alloc(4 * (size_t)n) || idx_in.alloc(4 * (size_t)n)) return -1;
  hipLaunchKernelGGL(k_setup_keys, grid_for(n), dim3(256), 0, st, n, n_pose, frame, lm, key_in.as<uint32_t>(),
                     idx_in.as<uint32_t>());
  HIPCHK(hipGetLastError());
  const uint64_t kmax = (uint64_t)n_lm * (uint64_t)n_pose;
  unsigned end_bit = 1;
  while (end_bit < 32 && (1ull << end_bit) < kmax) ++end_bit;
  size_t tb = 0;
  HIPCHK(rocprim::radix_sort_pairs(nullptr, tb, key_in.as<uint32_t>(), key_sorted, idx_in.as<uint32_t>(), order,
                                   (size_t)n, 0u, end_bit, st));
  if (temp.alloc(tb)) return -1;
  HIPCHK(rocprim::radix_sort_pairs(temp.p, tb, key_in.as<uint32_t>(), key_sorted, idx_in.as<uint32_t>(), order, (size_t)n,
                                   0u, end_bit, st));
  int32_t* flag = key_in.as<int32_t>();  // the unsorted keys are dead
  hipLaunchKernelGGL(k_setup_flags, grid_for(n), dim3(256), 0, st, n, key_sorted, flag);
  HIPCHK(hipGetLastError());
  size_t sb = 0;
  HIPCHK(rocprim::inclusive_scan(nullptr, sb, flag, rec_seg, (size_t)n, rocprim::plus<int32_t>(), st));
  if (sb > temp.bytes && temp.alloc(sb)) return -1;
  HIPCHK(rocprim::inclusive_scan(temp.p, sb, flag, rec_seg, (size_t)n, rocprim::plus<int32_t>(), st));
  int32_t last = 0;
  HIPCHK(hipMemcpyAsync(&last, rec_seg + (n - 1), 4, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));  // (also: the temporaries above die at return)
  *n_seg = last;
  return 0;
}

int setup_fill_segments(hipStream_t st, int64_t n, int n_pose, int64_t n_seg, const uint32_t* key_sorted, int32_t* rec_seg,
                        int32_t* seg_frame, int32_t* seg_lm, int64_t* seg_rec_begin, int32_t* lm_first) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_setup_segments, grid_for(n), dim3(256), 0, st, n, n_pose, key_sorted, rec_seg, seg_frame, seg_lm,
                     seg_rec_begin);
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL(k_setup_lm_first, grid_for(n_seg), dim3(256), 0, st, n_seg, seg_lm, lm_first);
  HIPCHK(hipGetLastError());
  return 0;
}

template <typename real>
int setup_records(hipStream_t st, int64_t n, int64_t n_seg, const uint32_t* order, const int32_t* rec_seg,
                  const int32_t* seg_lm, const int64_t* seg_rec_begin, const int32_t* lm_first, const double* xy,
                  const double* w, double* seg_base, real* rec_xy, real* rec_w, uint8_t* rec_key, int64_t* perm) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_setup_seg_base, grid_for(n_seg), dim3(256), 0, st, n_seg, order, seg_rec_begin,
                     reinterpret_cast<const double2*>(xy), reinterpret_cast<double2*>(seg_base));
  HIPCHK(hipGetLastError());
  hipLaunchKernelGGL((k_setup_records<real>), grid_for(n), dim3(256), 0, st, n, order, rec_seg, seg_lm, lm_first,
                     reinterpret_cast<const double2*>(xy), w, reinterpret_cast<const double2*>(seg_base), rec_xy, rec_w,
                     rec_key, perm);
  HIPCHK(hipGetLastError());
  return 0;
}

template int setup_records<float>(hipStream_t, int64_t, int64_t, const uint32_t*, const int32_t*, const int32_t*,
                                  const int64_t*, const int32_t*, const double*, const double*, double*, float*, float*,
                                  uint8_t*, int64_t*);
template int setup_records<double>(hipStream_t, int64_t, int64_t, const uint32_t*, const int32_t*, const int32_t*,
                                   const int64_t*, const int32_t*, const double*, const double*, double*, double*,
                                   double*, uint8_t*, int64_t*);

}  // namespace ptzba
