// libptzba C-ABI (see include/ptzba.h): host-side problem preparation (native C++: stable counting
// sorts into landmark-major records, segment / landmark / frame CSR, work ordering), device buffer
// ownership, and the Levenberg-Marquardt step sequence over the gfx950 kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iterator>
#include <map>
#include <numeric>
#include <string>
#include <utility>
#include <vector>

#include "../../include/ptzba.h"
#include "ptzba_common.h"
#include "ptzba_kernels.h"
#include "host_util.h"
#include "par_util.h"

using namespace ptzba;

static size_t g_total_bytes(std::initializer_list<const DBuf*> l) {
  size_t s = 0;
  for (auto* b : l) s += b->bytes;
  return s;
}

enum { TM_K1 = 0, TM_SCHUR = 1, TM_CHOL = 2, TM_BACK = 3, TM_N = 4 };
constexpr int LM_RING = 4;
constexpr int TM_POOL = 512;
constexpr int COMM_POOL = 2048;  // timed exchanges per reset_kernel_times

struct ptzba_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t st = nullptr;
  // problem
  bool have_problem = false;
  int n_pose = 0, n_lm = 0, n_fixed = 1, precision = PTZBA_FP64, loss = PTZBA_LOSS_LINEAR;
  double fs = 1.0;
  double hcurv = 1.0;  // huber curvature weight beyond the unit, in units of rho' (LinArgs::hcurv), host-driven LM
  std::vector<std::pair<const char*, double>> setup_phases;  // the last set_problem's host phases (name, ms)
  bool lm_curv_pending = false;  // device-driven LM: the huber curvature switch has not happened yet
  bool lm_relin_mode = false;    // LMParams::relin_mode of the current run
  DBuf curv_pred;                // [8] the curvature-mode reduction's output (the trial's landmark-part prediction)
  int64_t n_rec = 0, n_seg = 0;
  int n_work = 0, max_seg_per_lm = 0;
  int n_sys = 0;
  int64_t ld = 0;
  double u = 0, v = 0;
  bool weighted = false;
  std::vector<int64_t> perm_host;  // sorted -> original record index
  bool perm_uploaded = false;
  // device: structure
  DBuf rec_xy, rec_seg, rec_w, perm, rec_key;
  DBuf seg_frame, seg_lm, seg_rec_begin, lm_seg_begin, lm_order;
  DBuf frame_seg_begin, frame_seg_list, frame_win_hi;
  DBuf s2_items, s2_groups, s2_lm, lm_meta;  // K2 work items / tiles / lists, slot ranges
  DBuf s2_part, part_diag;                                    // K2 split partials (blocks, diagonal terms)
  int n_s2_items = 0, n_s2_groups = 0;
  int64_t n_slot = 0;  // dense landmark x frame slots (W table rows)
  // device: state
  DBuf ptz, rays, ptz_trial, rays_trial, D_pose, D_ray;
  DBuf ptz_saved, rays_saved;  // ptzba_save_state / ptzba_restore_state (device-resident restart point)
  DBuf ft, rt, ft64, rt64, seg_base;
  DBuf ug_slot[2], w_slot[2], lm_out[2];
  int cur = 0;
  DBuf lm_aux, lm_red, red_scratch;
  DBuf sys;  // [S ld*ld | b ld | g_pose ld | dU ld]
  DBuf scal, info;  // scal: [8 partial scalars | 8 pose partials ("loc")], contiguous for one exchange
  DBuf scal_pack;               // device block [scal 8 | loc 8 | info]
  double* scal_host = nullptr;   // pinned host copy of scal_pack
  uint8_t* out_pin = nullptr;    // pinned landing buffer of ptzba_get_state (grown, kept)
  size_t out_pin_cap = 0;
  DBuf chol_tasks, Ldiag, Minv, dpose;  // Minv: inverses of the diagonal factor tiles (back-substitution)
  std::vector<int> chol_task_off;  // host: per elimination level, offsets into chol_tasks
  std::vector<int32_t> chol_tasks_host;  // host copy of chol_tasks (int4 records)
  DBuf tinv_tail;                        // diagonal tiles inverted after the factorisation
  int n_tinv_tail = 0;
  int chol_levels = 0, n_aug = 0, n_chain = 1;
  bool nested = false;
  int nd_depth = 0;  // dissection levels of the system order (SysOrder::nd_depth)
  DBuf frame_pos, row_pad, bs_chain_off, bs_chain_cols, bs_upd_off, bs_upd_tiles, bs_la_tasks;
  int bs_nupd = 0, bs_npos = 0, bs_ntasks = 0;
  DBuf bs_lo_off, bs_lo_tiles;  // left-looking back substitution lists (large systems)
  DBuf bsb_tasks, bsb_r;  // blocked back substitution (large systems): plan + r scratch [ld]
  std::vector<int> bsb_step_off;
  // persistent blocked back substitution (one launch, per-column update counters): expected counts, per-column
  // totals, the counters (zeroed at set_problem, advanced by one solve's totals per launch: epoch), error flag
  DBuf bsp_expect, bsp_tot, bsp_cnt;
  int* bsp_err = nullptr;  // pinned host flag a persistent kernel sets when a wait gave up (checked by lm_wait)
  // pinned staging of set_problem's small uploads (bump allocated, reset once the stream has drained them)
  uint8_t* stage = nullptr;
  size_t stage_cap = 0, stage_used = 0;
  // set_problem queues its staged uploads and zero fills here and lands them with ONE copy of the staging range into
  // stage_dev plus one scatter launch (flush_stage) instead of ~50 hipMemcpyAsync / hipMemsetAsync calls
  struct StageOp {
    void* dst;
    size_t off;  // offset in the staging buffer; SIZE_MAX: zero fill
    size_t n;
  };
  std::vector<StageOp> stage_ops;
  bool stage_batch = false;
  DBuf stage_dev;
  bool bs_pst = false;
  uint32_t bsp_epoch = 0;
  bool bs_ll = false, bs_blk = false;
  bool chol_delayed = false;  // the plan delays trailing updates (make_plan, DT = 2)
  DBuf xtiles, xbuf;  // packed exchange: tile list, buffer
  int n_xtiles = 0;
  DBuf ztiles;  // tiles zeroed before each build (the rest of the system region stays zero)
  int n_ztiles = 0;
  double lambda = 0;
  // device-driven LM: state, pinned record ring, events
  DBuf lmdev;
  LMDev* lm_host = nullptr;
  // device-driven LM: the value of LMDev::cur at which (ptz, rays) -- not (ptz_trial, rays_trial) -- hold the current
  // state (BacksubArgs::state_xor); lm_wait swaps the pointers when the device's decisions moved it
  int state_base = 0;
  // single-GPU device-driven LM: the trial-cost reduction waits for ptzba_lm_decide, which fuses the decision into it
  bool scal_deferred = false;
  bool scal_exported = false;  // ptzba_exchange handed out the scalar buffer (a caller-run scalar exchange)
  // timing
  int timing = 0;  // bitmask of timed kernel groups (1 K1, 2 Schur, 4 Cholesky solve, 8 back-substitution)
  std::vector<hipEvent_t> ev[TM_N];
  int ev_used[TM_N] = {0, 0, 0, 0};
  int64_t tm_seen[TM_N] = {0, 0, 0, 0};
  bool tm_sampled[TM_N] = {false, false, false, false};
  int tm_stride = 1;
  bool tm_flush = false;  // cold-cache timing: stream a scratch buffer through the caches before each timed K1
  bool tm_flush_read = false;  // ... by reading it (clean lines) instead of writing it
  DBuf flush_buf;
  int64_t gpu_setup_min = -1;  // set_problem's device front from this many records (-1: GPU_SETUP_MIN_REC)
  // collective timing (enable bit PTZBA_TIME_COMM): an event pair around every exchange, its kind and size
  std::vector<hipEvent_t> cev;
  int cev_used = 0;
  std::vector<std::pair<int, int64_t>> clog;

  // multi-GPU (include/ptzba.h): exchanges done by the library, part-owned solve state
  ptzba_comm comm = nullptr;        // attached, not owned
  // communicators of the rank tree's groups, one per tree depth (split off comm at the first exchange; owned)
  ptzba_comm group_comms[4] = {nullptr, nullptr, nullptr, nullptr};
  bool groups_split = false;
  ptzba_exchange_fn hook = nullptr;
  void* hook_ctx = nullptr;
  int dist_world = 1, dist_rank = 0;
  int dist_mode = 0;  // 1: part-owned solve
  // rank-tree phases (make_plan_tree): factorisation levels, the exchange before each phase (kind, rank group,
  // tree depth of its communicator), exchanged tiles / vector ranges and their packing buffer
  struct DistPhase {
    int lv0 = 0, lv1 = 0, kind = 0, r0 = 0, nr = 1, depth = 0, node = -1, n_tiles = 0;
    VecRanges vr{};
    int64_t n_buf = 0;
  };
  static constexpr int MAX_PHASES = 4;
  DistPhase ph[MAX_PHASES];
  DBuf ph_tiles[MAX_PHASES], ph_buf[MAX_PHASES];
  int n_phase = 0, base_node = -1, tree_depth = 0;
  std::vector<int32_t> tree_groups;  // (r0, nr, depth) of every tree group of >= 2 ranks below the root
  DBuf row_phase, fmask;  // [n_aug] phase + 1 of each system row (0: not this rank's), [n_pose] bit 0 owned / bit 1 counted
  std::vector<uint8_t> owned_host;
  void drop_groups() {
    for (auto& c : group_comms)
      if (c) {
        ptzba_comm_delete(c);
        c = nullptr;
      }
    groups_split = false;
  }

  int elem() const { return precision == PTZBA_FP32 ? 4 : 8; }
  double* locp() const { return scal.as<double>() + 8; }
  bool has_exchange() const { return hook != nullptr || comm != nullptr; }
  bool ext_exchange = false;   // the caller ran its own exchange protocol (ptzba_exchange / _packed) once
  bool f1_covered = false;     // every 32-frame block has a chunk-0 Schur tile (all diagonals written by K2)
  // single-GPU builds fold k_chol_prepare into the build (FusedPrep, ptzba_kernels.h)
  bool no_fused_prep = false;  // PTZBA_NO_FUSED_PREP (A/B knob, read at set_problem)
  bool fused_prep() const { return !no_fused_prep && !dist_mode && !has_exchange() && !ext_exchange && f1_covered; }
  double* S() const { return sys.as<double>(); }
  double* bvec() const { return sys.as<double>() + ld * ld; }
  double* gpose() const { return sys.as<double>() + ld * ld + ld; }
  double* dU() const { return sys.as<double>() + ld * ld + 2 * ld; }
  int64_t sys_count() const { return ld * ld + 3 * ld; }
};

// Cold-cache K1 timing: 16-B vector stores over a scratch buffer larger than L2 + Infinity Cache (256 MB
// MALL, MI355X_MICROARCH.md) evict the record stream before the timed launch, so K1 reads from HBM.
// ptzba_restore_state: state <- snapshot, Marquardt scales <- 0
__global__ void __launch_bounds__(256) k_restore_state(double* __restrict__ ptz, const double* __restrict__ ptz_saved,
                                                       int64_t n_ptz, double* __restrict__ rays,
                                                       const double* __restrict__ rays_saved, int64_t n_rays,
                                                       double* __restrict__ D_pose, int64_t n_dp,
                                                       double* __restrict__ D_ray, int64_t n_dr) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_ptz) ptz[i] = ptz_saved[i];
  if (i < n_rays) rays[i] = rays_saved[i];
  if (i < n_dp) D_pose[i] = 0.0;
  if (i < n_dr) D_ray[i] = 0.0;
}

__global__ void __launch_bounds__(256) k_flush_caches(float4* buf, int64_t n16, float v) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
    buf[i] = make_float4(v, v, v, v);
}
// the read flush: streams the scratch buffer (filled once by k_flush_caches) through the caches, leaving clean lines;
// the sum is stored only if it equals an impossible value (the buffer holds small positive numbers), which keeps the
// loads alive
__global__ void __launch_bounds__(256) k_flush_caches_read(float4* buf, int64_t n16, float v) {
  float s = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x) {
    const float4 x = buf[i];
    s += x.x + x.y + x.z + x.w;
  }
  if (s == -v) buf[0] = make_float4(s, s, s, s);
}
constexpr size_t FLUSH_BYTES = (size_t)1 << 30;

// a timed group records an event pair around every tm_stride-th launch (each record adds a gap to the
// stream; sampling keeps that overhead out of most launches)
static void tm_begin(ptzba_ctx* h, int k) {
  h->tm_sampled[k] = false;
  if (!((h->timing >> k) & 1) || h->ev_used[k] + 2 > (int)h->ev[k].size()) return;
  if (h->tm_seen[k]++ % h->tm_stride != 0) return;
  h->tm_sampled[k] = true;
  if (k == TM_K1 && h->tm_flush && h->flush_buf.p) {
    if (h->tm_flush_read)
      k_flush_caches_read<<<4096, 256, 0, h->st>>>(h->flush_buf.as<float4>(), (int64_t)(h->flush_buf.bytes / 16), 1.0f);
    else
      k_flush_caches<<<4096, 256, 0, h->st>>>(h->flush_buf.as<float4>(), (int64_t)(h->flush_buf.bytes / 16),
                                               (float)h->tm_seen[k]);
  }
  if (k == TM_K1) return;  // K1 carries its event pair in its own launch (tm_k1_events)
  (void)hipEventRecord(h->ev[k][h->ev_used[k]], h->st);
}
static void tm_end(ptzba_ctx* h, int k) {
  if (!h->tm_sampled[k]) return;
  if (k != TM_K1) (void)hipEventRecord(h->ev[k][h->ev_used[k] + 1], h->st);
  h->ev_used[k] += 2;
  h->tm_sampled[k] = false;
}
// the event pair of a sampled K1 launch, for hipExtLaunchKernelGGL (the kernel packet's own start / end timestamps:
// the figure rocprofv3 reports, without the marker packets' dispatch gaps); nullptrs when this launch is not sampled
static hipEvent_t tm_k1_event(ptzba_ctx* h, int which) {
  return h->tm_sampled[TM_K1] ? h->ev[TM_K1][h->ev_used[TM_K1] + which] : nullptr;
}

const char* ptzba_last_error(void) { return g_err.c_str(); }
// 0.2 (round 6): ptzba_lm_opts carries huber_curvature / curvature_switch (11 fields; 0.1 had 9).  They are read
// for the Huber loss only, and huber_curvature 0 means the default 0.1, so a zero-filled tail keeps 0.1's behaviour.
const char* ptzba_version(void) { return "ptzba 0.2 gfx950 (ptzba_lm_opts: 11 fields)"; }

ptzba_handle ptzba_new(int device) {
  if (select_device(device)) return nullptr;
  auto* h = new ptzba_ctx();
  h->device = device;
  if (hipStreamCreateWithFlags(&h->own, hipStreamNonBlocking) != hipSuccess) {
    delete h;
    fail("hipStreamCreate failed");
    return nullptr;
  }
  h->st = h->own;
  return h;
}

void ptzba_delete(ptzba_handle h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->st) (void)hipStreamSynchronize(h->st);
  for (int k = 0; k < TM_N; ++k)
    for (auto e : h->ev[k]) (void)hipEventDestroy(e);
  for (auto e : h->cev) (void)hipEventDestroy(e);
  if (h->own) (void)hipStreamDestroy(h->own);
  if (h->scal_host) (void)hipHostFree(h->scal_host);
  if (h->out_pin) (void)hipHostFree(h->out_pin);
  if (h->bsp_err) (void)hipHostFree(h->bsp_err);
  if (h->stage) (void)hipHostFree(h->stage);
  h->drop_groups();
  if (h->lm_host) (void)hipHostFree(h->lm_host);
  delete h;
}

int ptzba_set_stream(ptzba_handle h, void* stream) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));  // work already queued on the previous stream completes first
  h->st = (hipStream_t)stream;          // NULL = the default stream (torch's current_stream() is often it)
  return 0;
}

int ptzba_use_own_stream(ptzba_handle h) { return h ? ptzba_set_stream(h, h->own) : fail("null handle"); }

// set_problem's uploads: a small array is copied into the handle's pinned staging buffer and its H2D copy queued on
// the handle's stream without waiting (a sliding-window map calls set_problem per keyframe: ~40 uploads, each a
// pageable copy plus a stream synchronisation before); large ones take the blocking path below.  The staging
// buffer is reused only after the stream has drained (set_problem synchronises before its first upload and at the
// end; a full buffer synchronises before wrapping).
constexpr size_t STAGE_MAX = 4u << 20, STAGE_MIN_CAP = 8u << 20;
constexpr int STAGE_OPS_PER_LAUNCH = 48;
struct StageScatterArgs {
  const uint8_t* src;
  int n_ops;
  uint8_t* dst[STAGE_OPS_PER_LAUNCH];
  uint64_t off[STAGE_OPS_PER_LAUNCH];  // ~0: zero fill
  uint64_t n[STAGE_OPS_PER_LAUNCH];
};
// every op's bytes over the grid: 16-B vectors when both ends are 16-B aligned (staging offsets and device
// allocations are 256-B aligned), the tail (or an unaligned op) byte by byte
__global__ __launch_bounds__(256) void k_stage_scatter(StageScatterArgs a) {
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (size_t)gridDim.x * blockDim.x;
  for (int q = 0; q < a.n_ops; ++q) {
    uint8_t* d = a.dst[q];
    const bool zero = a.off[q] == ~(uint64_t)0;
    const uint8_t* sp = zero ? nullptr : a.src + a.off[q];
    const bool vec = (((uintptr_t)d | (uintptr_t)sp) & 15) == 0;  // (a sub-buffer fill may start unaligned)
    const size_t n = a.n[q], n16 = vec ? n / 16 : 0;
    for (size_t i = tid; i < n16; i += nt)
      reinterpret_cast<uint4*>(d)[i] = zero ? make_uint4(0, 0, 0, 0) : reinterpret_cast<const uint4*>(sp)[i];
    for (size_t i = 16 * n16 + tid; i < n; i += nt) d[i] = zero ? 0 : sp[i];
  }
}
// lands the queued staged uploads and zero fills (stream-ordered after everything queued before)
static int flush_stage(ptzba_ctx* h) {
  if (h->stage_ops.empty()) return 0;
  bool any_copy = false;
  for (const auto& o : h->stage_ops) any_copy |= o.off != SIZE_MAX;
  if (any_copy) {
    if (h->stage_dev.reserve(h->stage_cap)) return -1;
    HIPCHK(hipMemcpyAsync(h->stage_dev.p, h->stage, h->stage_used, hipMemcpyHostToDevice, h->st));
  }
  size_t tot = 0;
  for (const auto& o : h->stage_ops) tot += o.n;
  const unsigned blocks = (unsigned)std::min<size_t>(1024, std::max<size_t>(1, tot / 32768));
  for (size_t q0 = 0; q0 < h->stage_ops.size(); q0 += STAGE_OPS_PER_LAUNCH) {
    StageScatterArgs a{};
    a.src = h->stage_dev.as<uint8_t>();
    a.n_ops = (int)std::min<size_t>(STAGE_OPS_PER_LAUNCH, h->stage_ops.size() - q0);
    for (int q = 0; q < a.n_ops; ++q) {
      const auto& o = h->stage_ops[q0 + q];
      a.dst[q] = (uint8_t*)o.dst;
      a.off[q] = o.off == SIZE_MAX ? ~(uint64_t)0 : (uint64_t)o.off;
      a.n[q] = o.n;
    }
    hipLaunchKernelGGL(k_stage_scatter, dim3(blocks), dim3(256), 0, h->st, a);
    HIPCHK(hipGetLastError());
  }
  h->stage_ops.clear();
  return 0;
}
// n zero bytes at p on the handle's stream (queued with the staged uploads while set_problem batches them)
static int zero_async(ptzba_ctx* h, void* p, size_t n) {
  if (!p || !n) return 0;
  if (h->stage_batch) {
    h->stage_ops.push_back({p, SIZE_MAX, n});
    return 0;
  }
  HIPCHK(hipMemsetAsync(p, 0, n, h->st));
  return 0;
}
// a pinned staging slot of n bytes for one queued copy (*out = nullptr when n is too large for the staging path)
static int stage_take(ptzba_ctx* h, size_t n, uint8_t** out) {
  *out = nullptr;
  if (n > STAGE_MAX) return 0;
  size_t off = (h->stage_used + 255) & ~(size_t)255;
  if (!h->stage || off + n > h->stage_cap) {
    if (flush_stage(h)) return -1;         // the queued copies read the staging buffer: land them first
    HIPCHK(hipStreamSynchronize(h->st));  // every staged copy so far has landed
    off = 0;
    if (!h->stage) {
      HIPCHK(hipHostMalloc((void**)&h->stage, STAGE_MIN_CAP, hipHostMallocDefault));
      h->stage_cap = STAGE_MIN_CAP;
    }
  }
  *out = h->stage + off;
  h->stage_used = off + n;
  return 0;
}
template <typename T>
static int upload(DBuf& b, const std::vector<T>& v, hipStream_t st);
template <typename T>
static int upload_st(ptzba_ctx* h, DBuf& b, const std::vector<T>& v) {
  const size_t n = v.size() * sizeof(T);
  if (n > STAGE_MAX) return upload(b, v, h->st);
  if (b.alloc(n)) return -1;
  if (n == 0) return 0;
  uint8_t* p = nullptr;
  if (stage_take(h, n, &p)) return -1;
  std::memcpy(p, v.data(), n);
  if (h->stage_batch) {
    h->stage_ops.push_back({b.p, (size_t)(p - h->stage), n});
    return 0;
  }
  HIPCHK(hipMemcpyAsync(b.p, p, n, hipMemcpyHostToDevice, h->st));
  return 0;
}

// ------------------------------------------------------------------------------------------------
// records hold obs - base(segment) in `real`; the per-segment base observation stays fp64, so the
// per-record arithmetic of K1 works on O(residual) magnitudes even in fp32
template <typename real>
static int upload_records(ptzba_ctx* h, const std::vector<int64_t>& order, const std::vector<int32_t>& rec_seg,
                          const std::vector<double>& base, const double* obs_xy, const double* w) {
  // the copies below read host vectors that die at return: every exit path (errors included) waits for the
  // handle's stream first (the stream does not order itself behind the legacy null stream, so every upload /
  // memset of set_problem goes on h->st)
  const size_t nxy = 2 * (size_t)h->n_rec, nw = w ? (size_t)h->n_rec : 0;
  // allocate everything before queuing any copy; padded by 8 records: K1's coarsened loads read whole groups
  if (h->rec_xy.alloc((nxy + 16) * sizeof(real))) return -1;
  if (w) {
    if (h->rec_w.alloc(nw * sizeof(real))) return -1;
  } else {
    h->rec_w.release();
  }
  // small problems (a sliding window's ~170K records) convert straight into the pinned staging buffer and queue the
  // copies; large ones convert into host vectors and copy with a synchronisation (the vectors die at return)
  uint8_t *pxy = nullptr, *pw = nullptr;
  if (stage_take(h, nxy * sizeof(real), &pxy)) return -1;
  if (pxy && w && stage_take(h, nw * sizeof(real), &pw)) return -1;
  const bool staged = pxy && (!w || pw);
  std::vector<real> vxy(staged ? 0 : nxy), vw(staged ? 0 : nw);
  struct SyncIf {  // the vector path: every exit waits for the copies reading the vectors (errors included)
    hipStream_t s;
    bool on;
    ~SyncIf() {
      if (on) (void)hipStreamSynchronize(s);
    }
  } sync_guard{h->st, !staged};
  real* xy = staged ? reinterpret_cast<real*>(pxy) : vxy.data();
  real* ww = staged ? reinterpret_cast<real*>(pw) : vw.data();
  parallel_chunks(h->n_rec, host_threads(h->n_rec), [&](int64_t lo, int64_t hi, int) {
    for (int64_t r = lo; r < hi; ++r) {
      const int32_t s = rec_seg[r];
      xy[2 * r] = (real)(obs_xy[2 * order[r]] - base[2 * s]);
      xy[2 * r + 1] = (real)(obs_xy[2 * order[r] + 1] - base[2 * s + 1]);
      if (w) ww[r] = (real)w[order[r]];
    }
  });
  if (staged && h->stage_batch) {  // queued with set_problem's other staged uploads
    h->stage_ops.push_back({h->rec_xy.p, (size_t)(pxy - h->stage), nxy * sizeof(real)});
    if (w) h->stage_ops.push_back({h->rec_w.p, (size_t)(pw - h->stage), nw * sizeof(real)});
    return zero_async(h, reinterpret_cast<real*>(h->rec_xy.p) + nxy, 16 * sizeof(real));
  }
  HIPCHK(hipMemcpyAsync(h->rec_xy.p, xy, nxy * sizeof(real), hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemsetAsync(reinterpret_cast<real*>(h->rec_xy.p) + nxy, 0, 16 * sizeof(real), h->st));
  if (w) HIPCHK(hipMemcpyAsync(h->rec_w.p, ww, nw * sizeof(real), hipMemcpyHostToDevice, h->st));
  return 0;
}

// blocking upload on stream st (nullptr: the null stream); returns after the copy has landed
template <typename T>
static int upload(DBuf& b, const std::vector<T>& v, hipStream_t st) {
  if (b.alloc(v.size() * sizeof(T))) return -1;
  if (!v.empty()) {
    HIPCHK(hipMemcpyAsync(b.p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
  }
  return 0;
}

// ------------------------------------------------------------------------------------------------
// system order of the reduced camera system and the tile-level factorisation plan
// ------------------------------------------------------------------------------------------------
static int pad_tile(int x) { return (x + CHOL_NB - 1) / CHOL_NB * CHOL_NB; }
static bool getenv_is(const char* name, const char* value) {
  const char* e = getenv(name);
  return e && std::string(e) == value;
}

struct SysOrder {
  std::vector<int32_t> pos;  // [n_pose] system row of the frame's pan (-1: fixed)
  std::vector<uint8_t> pad;  // [n_aug] identity padding rows
  int n_aug = 0;
  bool nested = false;
  int tiles_a = 0, tiles_b = 0;  // nested: tile columns of parts A and B (C follows)
  int split_m = 0, split_cend = 0;  // nested: A = [nf, m), C = [m, c_end), B = [c_end, n_pose)
  // separator tree of a nested order (tile-column ranges [t0, t1); parent -1 = the root separator): the
  // back-substitution chains are its root-to-leaf paths, the blocked back-solve's phases its depths
  struct Node { int t0, t1, parent, f0, f1; };  // (+ the node's frames [f0, f1))
  std::vector<Node> nodes;
  int nd_depth = 0;  // 0 natural, 1 = [A | B reversed | C], 2 = two dissection levels (nested_order2)
};

static SysOrder natural_order(int n_pose, int nf) {
  SysOrder o;
  o.pos.assign(n_pose, -1);
  for (int f = nf; f < n_pose; ++f) o.pos[f] = 3 * (f - nf);
  o.n_aug = 3 * (n_pose - nf);
  o.pad.assign(o.n_aug, 0);
  return o;
}

// One level of nested dissection of the frame chain: A = [nf, m), separator C = [m, c_end) with
// c_end past every frame A couples to, B = [c_end, n_pose) (decoupled from A).  System order
// [A | B reversed | C], each part padded to whole tiles: A and B factor side by side, their couplings
// to C are eliminated last, and the back-substitution splits into two chains after C.  Chosen only when
// it shortens the critical path of tile columns.
static bool nested_order(int n_pose, int nf, const std::vector<int32_t>& win, SysOrder& o, bool force) {
  const int nfree = n_pose - nf;
  if (nfree < (force ? 3 : 16)) return false;
  std::vector<int> pmax(n_pose + 1, -1);
  for (int f = nf; f < n_pose; ++f) pmax[f + 1] = std::max(pmax[f], (int)win[f]);
  const int nat = pad_tile(3 * nfree + 1) / CHOL_NB;
  int best_m = -1, best = nat;
  (void)force;
  for (int m = nf + 1; m < n_pose; ++m) {
    const int cend = std::max(m, pmax[m] + 1);
    if (cend >= n_pose) break;
    const int ta = pad_tile(3 * (m - nf)) / CHOL_NB, tb = pad_tile(3 * (n_pose - cend)) / CHOL_NB;
    const int tc = pad_tile(3 * (cend - m)) / CHOL_NB;
    const int chain = std::max(ta, tb) + tc + 1;
    if (chain < best) {
      best = chain;
      best_m = m;
    }
  }
  if (force) {  // testing: the most balanced split with a non-empty B, whatever the gain
    best_m = -1;
    int bal = INT32_MAX;
    for (int m = nf + 1; m < n_pose; ++m) {
      const int cend = std::max(m, pmax[m] + 1);
      if (cend >= n_pose) break;
      const int d = std::abs((m - nf) - (n_pose - cend));
      if (d < bal) { bal = d; best_m = m; }
    }
  }
  if (best_m < 0 || (!force && best + 2 > nat)) return false;
  const int m = best_m, cend = std::max(m, pmax[m] + 1);
  const int ar = 3 * (m - nf), br = 3 * (n_pose - cend), cr = 3 * (cend - m);
  const int ap = pad_tile(ar), bp = pad_tile(br), cp = pad_tile(cr);
  o.pos.assign(n_pose, -1);
  for (int f = nf; f < m; ++f) o.pos[f] = 3 * (f - nf);
  for (int f = n_pose - 1; f >= cend; --f) o.pos[f] = ap + 3 * (n_pose - 1 - f);
  for (int f = m; f < cend; ++f) o.pos[f] = ap + bp + 3 * (f - m);
  o.n_aug = ap + bp + cp;
  o.pad.assign(o.n_aug, 0);
  for (int r = ar; r < ap; ++r) o.pad[r] = 1;
  for (int r = ap + br; r < ap + bp; ++r) o.pad[r] = 1;
  for (int r = ap + bp + cr; r < o.n_aug; ++r) o.pad[r] = 1;
  o.nested = true;
  o.tiles_a = ap / CHOL_NB;
  o.tiles_b = bp / CHOL_NB;
  o.split_m = m;
  o.split_cend = cend;
  o.nd_depth = 1;
  const int c0 = o.tiles_a + o.tiles_b;
  o.nodes = {{c0, o.n_aug / CHOL_NB, -1, m, cend}, {0, o.tiles_a, 0, nf, m}, {o.tiles_a, c0, 0, cend, n_pose}};
  return true;
}

// Two levels of nested dissection (round 3): the top separator C2 = [m, cend) splits the chain into halves,
// each half is split again by its most balanced separator: A1 | C1 | A2 | C2 | A3 | C3 | A4.  System order
// [A1 | A2 | A3 | A4 reversed | C1 | C3 | C2], each part padded to whole tiles: the four leaves factor side by
// side, then C1 and C3, then C2 -- a critical path of max(leaf) + sub-separator + top separator tile columns
// instead of max(A, B) + C (config 3: 26 instead of 30 levels), and four back-substitution chains C2 -> C1 ->
// A1 / A2, C2 -> C3 -> A3 / A4.  A leaf couples only to its ancestors: A1 to C1, A2 to C1 and C2, A3 to C2
// and C3, A4 to C3 (and, where the window reaches that far, C2).  The top split minimises the estimated chain.
static bool nested_order2(int n_pose, int nf, const std::vector<int32_t>& win, SysOrder& o, bool halves = false) {
  if (n_pose - nf < 32) return false;
  std::vector<int> pmax(n_pose + 1, -1);
  for (int f = nf; f < n_pose; ++f) pmax[f + 1] = std::max(pmax[f], (int)win[f]);
  auto tiles = [](int a, int b) { return pad_tile(3 * (b - a)) / CHOL_NB; };
  // most balanced split of [lo, hi) by a separator [m1, c1) (running coupling max from lo); false if none
  auto balanced = [&](int lo, int hi, int& m1_out, int& c1_out) {
    int best = INT32_MAX, run = -1;
    for (int m1 = lo + 1; m1 < hi; ++m1) {
      run = std::max(run, (int)win[m1 - 1]);
      const int c1 = std::max(m1, run + 1);
      if (c1 >= hi) break;
      const int d = std::abs((m1 - lo) - (hi - c1));
      if (d < best) { best = d; m1_out = m1; c1_out = c1; }
    }
    return best != INT32_MAX;
  };
  int best = INT32_MAX, bm = -1, bc = -1, b1 = -1, bc1 = -1, b3 = -1, bc3 = -1;
  for (int m = nf + 2; m < n_pose - 1; ++m) {
    const int cend = std::max(m, pmax[m] + 1);
    if (cend >= n_pose - 1) break;
    int m1, c1, m3, c3;
    if (!balanced(nf, m, m1, c1) || !balanced(cend, n_pose, m3, c3)) continue;
    const int est = std::max(std::max(tiles(nf, m1), tiles(c1, m)) + tiles(m1, c1),
                             std::max(tiles(cend, m3), tiles(c3, n_pose)) + tiles(m3, c3)) + tiles(m, cend) + 1;
    if (est < best) { best = est; bm = m; bc = cend; b1 = m1; bc1 = c1; b3 = m3; bc3 = c3; }
  }
  if (bm < 0) return false;
  // parts in system order: {first frame, end frame, reversed}.  halves (part-owned multi-GPU solve): each half
  // contiguous, [A1 | A2 | C1 | A3 | A4 reversed | C3 | C2], so a rank group owns [A1 | A2 | C1] or [A3 | A4 | C3]
  // and C2 is the separator the groups exchange (the same dependencies, so the same levels)
  const int pa[7][3] = {{nf, b1, 0}, {bc1, bm, 0}, {bc, b3, 0}, {bc3, n_pose, 1}, {b1, bc1, 0}, {b3, bc3, 0}, {bm, bc, 0}};
  const int ph[7][3] = {{nf, b1, 0}, {bc1, bm, 0}, {b1, bc1, 0}, {bc, b3, 0}, {bc3, n_pose, 1}, {b3, bc3, 0}, {bm, bc, 0}};
  const int (*parts)[3] = halves ? ph : pa;
  o = SysOrder{};
  o.pos.assign(n_pose, -1);
  int row = 0, t[8];
  std::vector<std::pair<int, int>> pad_ranges;
  for (int p = 0; p < 7; ++p) {
    const int a = parts[p][0], b = parts[p][1], nr = 3 * (b - a);
    t[p] = row / CHOL_NB;
    for (int f = a; f < b; ++f) o.pos[f] = row + 3 * (parts[p][2] ? (b - 1 - f) : (f - a));
    pad_ranges.push_back({row + nr, row + pad_tile(nr)});
    row += pad_tile(nr);
  }
  t[7] = row / CHOL_NB;
  o.n_aug = row;
  o.pad.assign(o.n_aug, 0);
  for (auto& pr : pad_ranges)
    for (int r = pr.first; r < pr.second; ++r) o.pad[r] = 1;
  o.nested = true;
  o.nd_depth = 2;
  if (halves) {
    // nodes: 0 = C2 (root), 1 = C1, 2 = C3, 3..6 = A1..A4 (part-owned fields: the halves and C2's frames)
    o.nodes = {{t[6], t[7], -1, bm, bc}, {t[2], t[3], 0, b1, bc1}, {t[5], t[6], 0, b3, bc3},
               {t[0], t[1], 1, nf, b1}, {t[1], t[2], 1, bc1, bm}, {t[3], t[4], 2, bc, b3}, {t[4], t[5], 2, bc3, n_pose}};
    o.tiles_a = t[3];
    o.tiles_b = t[6] - t[3];
    o.split_m = bm;
    o.split_cend = bc;
    return true;
  }
  // nodes: 0 = C2 (root), 1 = C1, 2 = C3, 3..6 = A1..A4
  o.nodes = {{t[6], t[7], -1, bm, bc}, {t[4], t[5], 0, b1, bc1}, {t[5], t[6], 0, b3, bc3},
             {t[0], t[1], 1, nf, b1}, {t[1], t[2], 1, bc1, bm}, {t[2], t[3], 2, bc, b3}, {t[3], t[4], 2, bc3, n_pose}};
  return true;
}

// The split of a part-owned (multi-GPU) solve: nested_order's choice when it shortens the critical path,
// else its most balanced split; false when none exists (every frame couples to the last one).  A pure
// function of the coupling window, so ptzba_partition_landmarks and every rank's set_problem agree.
static bool dist_order(int n_pose, int nf, const std::vector<int32_t>& win, int world, SysOrder& o);  // after make_plan_tree

// Rank tree of a part-owned (multi-GPU) solve (round 4).  The separator tree of a nested order (one or two
// dissection levels) with the world's ranks dealt over it: a node with R >= 2 ranks gives ceil(R / 2) of them to its
// lower-frame child and the rest to the other; a node reached with one rank is that rank's OWN subtree; a leaf
// reached with R >= 2 ranks is SHARED by them.  A rank's phases: its base (own subtree, or shared leaf), then each
// ancestor separator up to the root.  Every subtree's tile columns and frames are contiguous in the orders used.
struct DistTree {
  struct N {
    int t0, t1, parent, f0, f1;  // separator / leaf columns and frames (SysOrder::Node)
    int st0, st1, sf0, sf1;      // the subtree's columns and frames
    int child[2], nch, depth;
    int r0, nr;                  // ranks [r0, r0 + nr) below this node
  };
  std::vector<N> n;
  int depth = 0;  // deepest node
};
static bool dist_tree(const SysOrder& o, int world, DistTree& T) {
  const int nn = (int)o.nodes.size();
  if (nn < 3 || world < 2) return false;
  T.n.assign(nn, DistTree::N{});
  for (int v = 0; v < nn; ++v) {
    const auto& a = o.nodes[v];
    T.n[v] = DistTree::N{a.t0, a.t1, a.parent, a.f0, a.f1, a.t0, a.t1, a.f0, a.f1, {-1, -1}, 0, 0, 0, 0};
  }
  for (int v = 0; v < nn; ++v) {
    const int p = T.n[v].parent;
    if (p < 0) continue;
    if (T.n[p].nch >= 2) return false;
    T.n[p].child[T.n[p].nch++] = v;
  }
  T.depth = 0;
  for (int v = 0; v < nn; ++v) {
    for (int u = T.n[v].parent; u >= 0; u = T.n[u].parent) T.n[v].depth++;
    T.depth = std::max(T.depth, T.n[v].depth);
    for (int u = T.n[v].parent; u >= 0; u = T.n[u].parent) {  // extend the ancestors' subtree ranges
      T.n[u].st0 = std::min(T.n[u].st0, T.n[v].t0);
      T.n[u].st1 = std::max(T.n[u].st1, T.n[v].t1);
      T.n[u].sf0 = std::min(T.n[u].sf0, T.n[v].f0);
      T.n[u].sf1 = std::max(T.n[u].sf1, T.n[v].f1);
    }
  }
  for (int v = 0; v < nn; ++v) {
    auto& x = T.n[v];
    if (x.nch == 1) return false;
    if (x.nch == 2 && T.n[x.child[0]].sf0 > T.n[x.child[1]].sf0) std::swap(x.child[0], x.child[1]);
  }
  // contiguity of every subtree (columns and frames): the sum of its nodes' sizes fills its range
  for (int v = 0; v < nn; ++v) {
    int64_t cols = 0, frames = 0;
    for (int u = 0; u < nn; ++u) {
      bool in = false;
      for (int w = u; w >= 0; w = T.n[w].parent) in = in || w == v;
      if (in) { cols += T.n[u].t1 - T.n[u].t0; frames += T.n[u].f1 - T.n[u].f0; }
    }
    if (cols != T.n[v].st1 - T.n[v].st0 || frames != T.n[v].sf1 - T.n[v].sf0) return false;
  }
  std::vector<std::pair<int, std::pair<int, int>>> stack{{0, {0, world}}};
  while (!stack.empty()) {
    const int v = stack.back().first, r0 = stack.back().second.first, nr = stack.back().second.second;
    stack.pop_back();
    T.n[v].r0 = r0;
    T.n[v].nr = nr;
    if (T.n[v].nch == 2) {
      const int k = nr >= 2 ? (nr + 1) / 2 : 1;
      stack.push_back({T.n[v].child[0], {r0, k}});
      stack.push_back({T.n[v].child[1], nr >= 2 ? std::make_pair(r0 + k, nr - k) : std::make_pair(r0, 1)});
    }
  }
  return true;
}
// a rank's base node (own subtree: nr == 1; shared leaf: nr >= 2) and its ancestors, bottom-up
static int dist_base(const DistTree& T, int rank, std::vector<int>* anc = nullptr) {
  int v = 0;
  while (T.n[v].nr >= 2 && T.n[v].nch == 2) {
    const auto& c = T.n[T.n[v].child[0]];
    v = (rank >= c.r0 && rank < c.r0 + c.nr) ? T.n[v].child[0] : T.n[v].child[1];
  }
  if (anc) {
    anc->clear();
    for (int u = T.n[v].parent; u >= 0; u = T.n[u].parent) anc->push_back(u);
  }
  return v;
}

struct CholPlan {
  std::vector<int32_t> tasks;  // int4 records
  std::vector<int> level_off;
  std::vector<int> chain_off, chain_cols, upd_off, upd_tiles;
  std::vector<int> la_tasks;  // lookahead back substitution: la [npos] | task_off [n_chain * BS_HELPERS + 1] | tasks
  int n_tasks = 0;
  std::vector<int> lo_off, lo_tiles;  // left-looking back substitution: per position the solved row tiles coupled to it
  std::vector<int32_t> xtiles;  // (ti, tj) pairs the Schur kernel can write (before fill), for the exchange
  std::vector<int32_t> ztiles;  // (ti, tj) lower tiles of the factor's pattern (incl. fill): zeroed per build
  std::vector<int32_t> tinv_tail;  // diagonal tiles inverted after the last level (the others: type-2 tasks)
  int n_levels = 0;
  bool delayed = false;  // tasks carry a second pair of update panels (delayed trailing updates, make_plan)
  // blocked back substitution (large systems): tasks of 3 int4 (block columns | {p, intra-block coupling
  // bits, first-touch bits, 0} | {target column, flags, 0, 0}) and the task offset of each step (one launch
  // per step); empty when no valid schedule exists
  std::vector<int32_t> bsb_tasks;
  std::vector<int> bsb_step_off;
  // persistent form (k_chol_backsolve_pst): per task the updates its block columns / target have received before
  // its step, {E_c0, E_c1, E_c2, E_c3, E_t, 0, 0, 0}, and per column the updates one solve applies to it
  std::vector<int32_t> bsb_expect, bsb_tot;
};

// Steps of the blocked right-looking back substitution (k_chol_backsolve_blk).  The chains' common prefix
// (the separator C of a nested order) is cut into blocks of BSB_P consecutive positions solved one block
// per step; the chains' remainders (A and B) then advance in lockstep, one block of each per step.  A step
// solves its blocks (every workgroup redundantly) and applies their contribution to every later column t
// coupled to them (one workgroup per (block, t): a plain read-modify-write of r_t, as no two tasks of a
// step share a target and steps are stream-ordered).  First-touch flags make a column's first read take
// the forward-substitution result y (the factor's augmented row) instead of r, so r needs no init launch.
// phases: the separator tree's depths (root separator first), each a list of sequences (tile columns in
// back-substitution order) that advance in lockstep.
typedef std::vector<std::vector<std::vector<int>>> BsPhases;
static void make_bs_steps(const std::vector<std::vector<uint8_t>>& nz, int Tx, CholPlan& P, const BsPhases& phases) {
  P.bsb_tasks.clear();
  P.bsb_step_off.assign(1, 0);
  const int T = (int)nz.size(), nch = (int)P.chain_off.size() - 1;
  if (nch < 1) return;
  std::vector<uint8_t> in_any(T, 0), solved(T, 0), touched(T, 0);
  for (int kt : P.chain_cols) in_any[kt] = 1;
  auto fail = [&]() {
    P.bsb_tasks.clear();
    P.bsb_step_off.assign(1, 0);
  };
  for (const auto& seqs : phases) {
    size_t len = 0;
    for (const auto& q : seqs) len = std::max(len, q.size());
    for (size_t q0 = 0; q0 < len; q0 += BSB_P) {
      std::vector<uint8_t> used(T, 0);  // block columns and targets of this step
      std::vector<int> step_targets;
      for (const auto& q : seqs) {
        if (q0 >= q.size()) continue;
        const int p = (int)std::min<size_t>(BSB_P, q.size() - q0);
        int cols[BSB_P] = {-1, -1, -1, -1}, imask = 0, ftouch = 0;
        for (int k = 0; k < p; ++k) {
          cols[k] = q[q0 + k];
          if (used[cols[k]] || solved[cols[k]]) return fail();
          used[cols[k]] = 1;
          if (!touched[cols[k]]) ftouch |= 1 << k;
          for (int j = 0; j < k; ++j) {
            if (cols[j] <= cols[k]) return fail();  // descending within a block
            if (nz[cols[j]][cols[k]]) imask |= 1 << (j * 4 + k);
          }
        }
        auto push_task = [&](int t, int flags) {
          P.bsb_tasks.insert(P.bsb_tasks.end(), {cols[0], cols[1], cols[2], cols[3], p, imask, ftouch, 0, t, flags, 0, 0});
        };
        std::vector<int> tmask(T, 0);
        for (int k = 0; k < p; ++k)
          for (int t = 0; t < cols[k]; ++t)
            if (in_any[t] && nz[cols[k]][t] && !(t == cols[0] || t == cols[1] || t == cols[2] || t == cols[3]))
              tmask[t] |= 1 << k;
        bool first = true;
        for (int t = 0; t < T; ++t) {
          if (!tmask[t]) continue;
          if (used[t] || solved[t]) return fail();
          used[t] = 1;
          step_targets.push_back(t);
          push_task(t, tmask[t] | (first ? 0x100 : 0) | (touched[t] ? 0 : 0x200));
          first = false;
        }
        if (first) push_task(-1, 0x100);
        for (int k = 0; k < p; ++k) solved[cols[k]] = touched[cols[k]] = 1;
      }
      for (int t : step_targets) touched[t] = 1;
      P.bsb_step_off.push_back((int)(P.bsb_tasks.size() / 12));
    }
  }
  for (int kt = 0; kt < Tx; ++kt)
    if (in_any[kt] && !solved[kt]) return fail();
  // expected update counts for the persistent form: replay the steps in order
  const int nt = (int)(P.bsb_tasks.size() / 12);
  P.bsb_expect.assign(8 * (size_t)nt, 0);
  std::vector<int32_t> done(T, 0);
  for (size_t st = 0; st + 1 < P.bsb_step_off.size(); ++st) {
    for (int q = P.bsb_step_off[st]; q < P.bsb_step_off[st + 1]; ++q) {
      const int32_t* tk = &P.bsb_tasks[12 * (size_t)q];
      for (int k = 0; k < 4; ++k) P.bsb_expect[8 * (size_t)q + k] = tk[k] >= 0 ? done[tk[k]] : 0;
      P.bsb_expect[8 * (size_t)q + 4] = tk[8] >= 0 ? done[tk[8]] : 0;
    }
    for (int q = P.bsb_step_off[st]; q < P.bsb_step_off[st + 1]; ++q) {
      const int t = P.bsb_tasks[12 * (size_t)q + 8];
      if (t >= 0) done[t]++;
    }
  }
  P.bsb_tot = done;
}

// Tile structure (coupled frame pairs + the dense augmented row + symbolic fill), elimination levels
// (at most two tile columns per level), tasks per level and back-substitution chains.
// Rank-tree restriction of make_plan (make_plan_tree, §7): the tile columns this rank factors, phase by phase (each
// phase's columns depend only on the same phase's; a flush level closes every phase but the last and is always a
// trailing level, so it applies the phase's pending panels to the later phases' tiles), and the exactly-once rule:
// an update from phase q's panels into a later phase's tile (i, j) is kept only by group member (i + j) mod size.
struct TreeSpec {
  std::vector<int8_t> col_phase;  // [T] phase of each tile column, -1 not this rank's
  std::vector<int> ph_nr, ph_me;  // per phase: group size, this rank's index in the group
  std::vector<int> chain;         // back-substitution chain (the phases from the root down, columns descending)
  std::vector<int> ph_lv0, ph_lv1;  // out: per phase its levels [lv0, lv1) (the closing flush level included)
};
static int tile_owner(int i, int j, int nr) { return (i + j) % nr; }
// (Round 4's supercolumn plans -- two chain columns per level task, measured slower: 0.31 vs 0.23 ms at config 3 --
// were removed in round 6 with their kernel; DESIGN.md §4.3 keeps the record.)
static bool make_plan(const SysOrder& o, int n_pose, int nf, const std::vector<int32_t>& win, int64_t ld, CholPlan& P,
                      int force_dt = 0, TreeSpec* ts = nullptr) {
  const int T = (int)(ld / CHOL_NB);
  std::vector<std::vector<uint8_t>> nz(T, std::vector<uint8_t>(T, 0));
  auto mark = [&](int r, int c) {
    int ti = r / CHOL_NB, tj = c / CHOL_NB;
    if (ti < tj) std::swap(ti, tj);
    nz[ti][tj] = 1;
  };
  for (int f1 = nf; f1 < n_pose; ++f1)
    for (int f2 = f1; f2 <= std::min(n_pose - 1, (int)win[f1]); ++f2) {
      const int p1 = o.pos[f1], p2 = o.pos[f2];
      mark(p2, p1); mark(p2 + 2, p1); mark(p2, p1 + 2); mark(p2 + 2, p1 + 2);
    }
  P.xtiles.clear();
  for (int i = 0; i < T; ++i)
    for (int j = 0; j <= i; ++j)
      if (nz[i][j] || i == j) { P.xtiles.push_back(i); P.xtiles.push_back(j); }
  const int ta = o.n_aug / CHOL_NB;  // tile holding the augmented row
  for (int j = 0; j <= ta; ++j) nz[ta][j] = 1;
  for (int i = 0; i < T; ++i) nz[i][i] = 1;
  for (int k = 0; k < T; ++k) {  // symbolic fill
    std::vector<int> R;
    for (int i = k + 1; i < T; ++i)
      if (nz[i][k]) R.push_back(i);
    for (size_t x = 0; x < R.size(); ++x)
      for (size_t y = 0; y <= x; ++y) nz[R[x]][R[y]] = 1;
  }
  auto own = [&](int t) { return !ts || ts->col_phase[t] >= 0; };
  auto phase = [&](int t) { return ts ? (int)ts->col_phase[t] : 0; };
  if (ts)
    for (int k = 0; k < T; ++k)  // a column this rank eliminates couples only to rows it holds
      if (own(k))
        for (int i = k + 1; i < T; ++i)
          if (nz[i][k] && !own(i)) return false;
  std::vector<int> level(T, ts ? -1 : 0), count;
  std::vector<uint8_t> flush_lv;
  auto place = [&](int k, int L0) {
    int L = L0;
    for (int p = 0; p < k; ++p)
      if (nz[k][p] && level[p] >= 0 && phase(p) == phase(k)) L = std::max(L, level[p] + 1);
    while (L < (int)count.size() && count[L] >= 4) ++L;  // at most four columns per launch
    if (L >= (int)count.size()) count.resize(L + 1, 0);
    count[L]++;
    level[k] = L;
  };
  if (!ts) {
    for (int k = 0; k < T; ++k) place(k, 0);
  } else {
    const int NP = (int)ts->ph_nr.size();
    ts->ph_lv0.assign(NP, 0);
    ts->ph_lv1.assign(NP, 0);
    for (int q = 0; q < NP; ++q) {
      ts->ph_lv0[q] = (int)count.size();
      for (int k = 0; k < T; ++k)
        if (phase(k) == q) place(k, ts->ph_lv0[q]);
      if (q + 1 < NP) {
        count.push_back(0);
        flush_lv.resize(count.size(), 0);
        flush_lv.back() = 1;
      }
      ts->ph_lv1[q] = (int)count.size();
    }
  }
  flush_lv.resize(count.size(), 0);
  P.ztiles.clear();
  for (int i = 0; i < T; ++i)
    for (int j = 0; j <= i; ++j)
      if (nz[i][j] && own(i) && own(j)) { P.ztiles.push_back(i); P.ztiles.push_back(j); }
  int nL = (int)count.size();
  std::vector<std::vector<int>> K(nL);
  for (int k = 0; k < T; ++k)
    if (level[k] >= 0) K[level[k]].push_back(k);
  P.tasks.clear();
  P.level_off.assign(nL + 1, 0);
  auto push = [&](int type, int i, int j, int w) {
    P.tasks.push_back(type); P.tasks.push_back(i); P.tasks.push_back(j); P.tasks.push_back(w);
  };
  // inverses of the diagonal factor tiles (for the back-substitution): the tiles of level L-1's columns are
  // inverted by type-2 tasks of level L, beside its panels (off the critical path); the last level's after
  // the factorisation (tinv_tail).  Columns >= n_inv (the augmented-row tile) need none.
  const int n_inv = (o.n_aug + CHOL_NB - 1) / CHOL_NB;
  const bool tinv_split = true;  // (round 2 A/B: every inverse after the factorisation instead: +4 us per trial)
  P.tinv_tail.clear();
  // Delayed trailing updates (period DT): trailing tasks run only at levels L = 0 mod DT and apply the
  // panels of levels [L - DT, L - 1] at once (rank <= 2 DT x 32: half the read-modify-writes of the band's
  // tiles at DT = 2); a panel task applies inline every update not yet applied to its tiles, the panels of
  // levels [F, L - 1] with F the last trailing level before L.  Worth it when the levels are dominated by
  // their trailing tasks (config 4: ~1,600 per level), not when they are chain-bound (config 3).
  int64_t trail = 0;
  for (int p = 0; p < T; ++p) {
    if (!own(p)) continue;
    int64_t r = 0;
    for (int i = p + 1; i < T; ++i) r += nz[i][p] && own(i);
    trail += r * (r + 1) / 2;
  }
  int DT = trail > 600 * (int64_t)nL ? 2 : 1;
  if (const char* e = getenv("PTZBA_CHOL_DELAY")) DT = std::max(1, std::min(2, atoi(e)));  // A/B knob
  if (force_dt) DT = force_dt;
  P.delayed = DT > 1;
  size_t max_pd = 0;  // update panels of one task: the P2 kernel takes up to four (any DT), the other two
  bool any_block = false;  // 2 x 2 trailing blocks (type 3) run in the P2 kernel only
  auto pack2 = [](int type, const std::vector<int>& pd, int tm) {  // int4 task: x (type + panels 2, 3), w (0, 1)
    return std::make_pair(chol_pack_type(type, pd.size() > 2 ? pd[2] : -1, pd.size() > 3 ? pd[3] : -1, (tm >> 2) & 3),
                          chol_pack_updates(pd.size() > 0 ? pd[0] : -1, pd.size() > 1 ? pd[1] : -1, tm & 3));
  };
  // trailing levels: every DT-th, and (rank-tree plans) every phase's flush level; a trailing level applies the
  // panels of the levels since the previous trailing level, a panel task inline those since the last one before it
  int last_trailing = 0;
  for (int L = 0; L < nL; ++L) {
    P.level_off[L] = (int)(P.tasks.size() / 4);
    const std::vector<int> none;
    const std::vector<int>& prev = L > 0 ? K[L - 1] : none;
    const bool trailing = L % DT == 0 || flush_lv[L];
    std::vector<int> inl;  // panels applied inline by this level's panel tasks
    if (L > 0)
      for (int l = last_trailing; l < L; ++l) inl.insert(inl.end(), K[l].begin(), K[l].end());
    for (int k : K[L]) {
      std::vector<int> pd;
      for (int pp : inl)
        if (pp < k && nz[k][pp]) pd.push_back(pp);
      for (int i = k; i < T; ++i) {
        if (!nz[i][k] || !own(i)) continue;
        int tm = 0;
        for (size_t u = 0; u < pd.size(); ++u)
          if (i == k || nz[i][pd[u]]) tm |= 1 << u;
        const auto w = pack2(0, pd, tm);
        push(w.first, i, k, w.second);
      }
      max_pd = std::max(max_pd, pd.size());
    }
    // trailing updates from the panels of levels [L - DT, L - 1] into tiles of columns factored after L
    std::vector<std::pair<int64_t, int>> upd;  // (tile key, panel)
    if (trailing && L > 0)
      for (int l = last_trailing; l < L; ++l)
        for (int pp : K[l]) {
          std::vector<int> R;
          for (int i = pp + 1; i < T; ++i)
            if (nz[i][pp] && own(i)) R.push_back(i);
          for (size_t x = 0; x < R.size(); ++x)
            for (size_t y = 0; y <= x; ++y) {
              if (level[R[y]] <= L) continue;
              // rank tree: into a later phase's tile only by its owner in this phase's group (exactly once)
              if (ts && phase(R[y]) != phase(pp) &&
                  tile_owner(R[x], R[y], ts->ph_nr[phase(pp)]) != ts->ph_me[phase(pp)])
                continue;
              upd.push_back({(int64_t)R[x] * T + R[y], pp});
            }
        }
    if (trailing) last_trailing = L;
    std::sort(upd.begin(), upd.end());
    // per tile its panels (ascending); with delayed updates the tiles are grouped into 2 x 2 blocks
    // (rows 2a, 2a + 1 x columns 2b, 2b + 1): one type-3 task per block stages each panel's four row tiles
    // once for up to four output tiles (~6 tile loads per output tile instead of ~10).  A block's panel set
    // is the union of its tiles' sets (at most four); a panel a tile is not coupled to has a zero L tile
    // there, so its product adds exact zeros -- the same arithmetic, in the same panel order, as one task
    // per tile.  PTZBA_CHOL_BLOCKS=0: one task per tile (A/B knob).
    std::map<int64_t, std::pair<int, std::vector<int>>> blocks;  // block key -> (tile mask, panel union)
    std::vector<std::pair<int, int>> single;                      // tiles emitted one by one (key index)
    std::vector<std::pair<int64_t, std::vector<int>>> tiles_pd;
    for (size_t x = 0; x < upd.size();) {
      size_t y = x + 1;
      while (y < upd.size() && upd[y].first == upd[x].first) ++y;
      std::vector<int> pd;
      for (size_t u = x; u < y; ++u) pd.push_back(upd[u].second);
      max_pd = std::max(max_pd, pd.size());
      tiles_pd.push_back({upd[x].first, pd});
      x = y;
    }
    const bool blocked = !getenv_is("PTZBA_CHOL_BLOCKS", "0");
    std::vector<uint8_t> in_block(tiles_pd.size(), 0);
    if (blocked) {
      for (size_t q = 0; q < tiles_pd.size(); ++q) {
        const int i = (int)(tiles_pd[q].first / T), j = (int)(tiles_pd[q].first % T);
        auto& b = blocks[(int64_t)(i / 2) * T + j / 2];
        b.first |= 1 << (2 * (i & 1) + (j & 1));
        for (int pp : tiles_pd[q].second)
          if (std::find(b.second.begin(), b.second.end(), pp) == b.second.end()) b.second.push_back(pp);
      }
      for (size_t q = 0; q < tiles_pd.size(); ++q) {
        const int i = (int)(tiles_pd[q].first / T), j = (int)(tiles_pd[q].first % T);
        const auto& b = blocks[(int64_t)(i / 2) * T + j / 2];
        in_block[q] = b.second.size() <= 4 && __builtin_popcount(b.first) >= 2;
      }
      for (auto& kv : blocks) {
        if (kv.second.second.size() > 4 || __builtin_popcount(kv.second.first) < 2) continue;
        std::vector<int> pd = kv.second.second;
        std::sort(pd.begin(), pd.end());
        const int a = (int)(kv.first / T), bcol = (int)(kv.first % T), mask = kv.second.first;
        push(chol_pack_type(3, pd.size() > 2 ? pd[2] : -1, pd.size() > 3 ? pd[3] : -1, (mask >> 2) & 3), 2 * a, 2 * bcol,
             chol_pack_updates(pd.size() > 0 ? pd[0] : -1, pd.size() > 1 ? pd[1] : -1, mask & 3));
        any_block = true;
      }
    }
    for (size_t q = 0; q < tiles_pd.size(); ++q) {
      if (in_block[q]) continue;
      const int i = (int)(tiles_pd[q].first / T), j = (int)(tiles_pd[q].first % T);
      const auto w = pack2(1, tiles_pd[q].second, 15);
      push(w.first, i, j, w.second);
    }
    // type 2: inverses of the previous level's diagonal tiles
    for (int pp : prev)
      if (tinv_split && pp < n_inv) push(2, pp, pp, 0);
  }
  for (int k = 0; k < n_inv && k < T; ++k)
    if (own(k) && (!tinv_split || level[k] == nL - 1)) P.tinv_tail.push_back(k);
  P.level_off[nL] = (int)(P.tasks.size() / 4);
  P.n_levels = nL;
  if (max_pd > 4) {  // too many panels for one task: DT = 1
    if (DT > 1) return make_plan(o, n_pose, nf, win, ld, P, 1, ts);
    return false;
  }
  if (max_pd > 2 || any_block) P.delayed = true;  // the P2 kernel (second panel pair, trailing blocks)
  // back-substitution: chains of tile columns holding unknowns and, per chain position, the chain's
  // later columns coupled to that row tile (right-looking updates).  Nested orders: one chain per leaf of
  // the separator tree (its root-to-leaf path, each node's columns descending); natural: one chain.
  const int Tx = (o.n_aug + CHOL_NB - 1) / CHOL_NB;
  P.chain_off.assign(1, 0);
  P.chain_cols.clear();
  BsPhases phases;
  if (ts) {  // rank tree: one chain, the phases from the root down
    P.chain_cols = ts->chain;
    P.chain_off.push_back((int)P.chain_cols.size());
    phases.push_back({P.chain_cols});
  } else if (o.nested && !o.nodes.empty()) {
    const int nn = (int)o.nodes.size();
    std::vector<int> depth(nn, 0), nchild(nn, 0);
    for (int v = 0; v < nn; ++v) {
      for (int u = o.nodes[v].parent; u >= 0; u = o.nodes[u].parent) ++depth[v];
      if (o.nodes[v].parent >= 0) ++nchild[o.nodes[v].parent];
    }
    auto desc = [&](int v) {
      std::vector<int> c;
      for (int kt = o.nodes[v].t1 - 1; kt >= o.nodes[v].t0; --kt) c.push_back(kt);
      return c;
    };
    for (int v = 0; v < nn; ++v) {
      if (nchild[v]) continue;  // leaf: the path root -> v
      std::vector<int> path;
      for (int u = v; u >= 0; u = o.nodes[u].parent) path.push_back(u);
      for (auto it = path.rbegin(); it != path.rend(); ++it)
        for (int kt : desc(*it)) P.chain_cols.push_back(kt);
      P.chain_off.push_back((int)P.chain_cols.size());
    }
    for (int v = 0; v < nn; ++v) {
      if ((int)phases.size() <= depth[v]) phases.resize(depth[v] + 1);
      phases[depth[v]].push_back(desc(v));
    }
    // every coupling of a chain column to a later column stays inside the chain (a leaf couples only to its
    // ancestors); otherwise this order is unusable
    for (size_t ch = 0; ch + 1 < P.chain_off.size(); ++ch) {
      std::vector<uint8_t> in_chain(T, 0);
      for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q) in_chain[P.chain_cols[q]] = 1;
      for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q)
        for (int i = P.chain_cols[q] + 1; i < Tx; ++i)
          if (nz[i][P.chain_cols[q]] && !in_chain[i]) return false;
    }
  } else {
    for (int kt = Tx - 1; kt >= 0; --kt) P.chain_cols.push_back(kt);
    P.chain_off.push_back((int)P.chain_cols.size());
    phases.push_back({P.chain_cols});
  }
  P.upd_off.assign(1, 0);
  P.upd_tiles.clear();
  for (size_t ch = 0; ch + 1 < P.chain_off.size(); ++ch) {
    std::vector<uint8_t> in_chain(T, 0);
    for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q) in_chain[P.chain_cols[q]] = 1;
    for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q) {
      const int kt = P.chain_cols[q];
      for (int j = 0; j < kt; ++j)
        if (in_chain[j] && nz[kt][j]) P.upd_tiles.push_back(j);
      P.upd_off.push_back((int)P.upd_tiles.size());
    }
  }
  P.lo_off.assign(1, 0);
  P.lo_tiles.clear();
  for (size_t ch = 0; ch + 1 < P.chain_off.size(); ++ch) {
    std::vector<uint8_t> in_chain(T, 0);
    for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q) in_chain[P.chain_cols[q]] = 1;
    for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q) {
      const int kt = P.chain_cols[q];
      for (int i = kt + 1; i < Tx; ++i)
        if (in_chain[i] && nz[i][kt]) P.lo_tiles.push_back(i);
      P.lo_off.push_back((int)P.lo_tiles.size());
    }
  }
  // lookahead back substitution: the next position's tile when the current row couples to it, and per
  // (chain, helper wave) the other updates (position, tile j with j % BS_HELPERS == helper) in order
  const int npos = (int)P.chain_cols.size(), nch = (int)P.chain_off.size() - 1;
  std::vector<int> la(npos, -1), toff(1, 0), tasks;
  for (int ch = 0; ch < nch; ++ch)
    for (int q = P.chain_off[ch]; q + 1 < P.chain_off[ch + 1]; ++q)
      for (int e = P.upd_off[q]; e < P.upd_off[q + 1]; ++e)
        if (P.upd_tiles[e] == P.chain_cols[q + 1]) la[q] = P.chain_cols[q + 1];
  for (int ch = 0; ch < nch; ++ch)
    for (int hw = 0; hw < BS_HELPERS; ++hw) {
      for (int q = P.chain_off[ch]; q < P.chain_off[ch + 1]; ++q)
        for (int e = P.upd_off[q]; e < P.upd_off[q + 1]; ++e) {
          const int j = P.upd_tiles[e];
          if (j % BS_HELPERS == hw && j != la[q]) tasks.push_back((q << 16) | j);
        }
      toff.push_back((int)tasks.size());
    }
  P.n_tasks = (int)tasks.size();
  P.la_tasks = la;
  P.la_tasks.insert(P.la_tasks.end(), toff.begin(), toff.end());
  P.la_tasks.insert(P.la_tasks.end(), tasks.begin(), tasks.end());
  make_bs_steps(nz, Tx, P, phases);
  return true;
}


// estimated factorisation time of a plan: per level the longer of the pivot chain (~7 us) and its tasks in
// rounds of the chip (~768 resident workgroups, ~6 us a round) -- fewer levels only pay when the extra fill
// and the wider levels do not turn them into throughput-bound ones (config 4: the two-level order has 189
// levels instead of 265 but up to 18K tasks per level, 7.9 vs 4.7 ms per trial)
static double plan_est_us(const CholPlan& P) {
  double t = 0;
  for (int L = 0; L < P.n_levels; ++L) {
    const int n = P.level_off[L + 1] - P.level_off[L];
    t += std::max(7.0, 6.0 * ((n + 767) / 768));
  }
  return t;
}

// System order and plan of a single-system solve: natural, or the one-level nested order, or two dissection
// levels when that plan has fewer levels (PTZBA_ND_DEPTH=1 / =2: A/B knob, one level only / two levels
// whenever valid).  Returns nonzero if no plan exists.
static int choose_order_plan(int n_pose, int nf, const std::vector<int32_t>& win, int ordering, SysOrder& so,
                             CholPlan& plan) {
  if (!(ordering != PTZBA_ORDER_NATURAL && nested_order(n_pose, nf, win, so, ordering == PTZBA_ORDER_NESTED_FORCE)))
    so = natural_order(n_pose, nf);
  if (!make_plan(so, n_pose, nf, win, pad_tile(so.n_aug + 1), plan)) return -1;
  const char* nde = getenv("PTZBA_ND_DEPTH");
  const int nd_env = nde ? atoi(nde) : 0;
  const auto est_us = plan_est_us;
  SysOrder s2;
  CholPlan p2;
  if (ordering == PTZBA_ORDER_NESTED && nd_env != 1 && nested_order2(n_pose, nf, win, s2) &&
      pad_tile(s2.n_aug + 1) <= CHOL_MAX_LD && make_plan(s2, n_pose, nf, win, pad_tile(s2.n_aug + 1), p2) &&
      ((p2.n_levels < plan.n_levels && est_us(p2) < est_us(plan)) || nd_env == 2)) {
    so = std::move(s2);
    plan = std::move(p2);
  }
  return 0;
}

// Rank-tree plan of a part-owned (multi-GPU) solve (api: ptzba_partition_landmarks, round 4).  A rank factors the
// tile columns of its phases in order -- its base (own subtree, or shared leaf), then each ancestor separator, the
// root's with the augmented column -- each phase closed by a flush level that applies its last panels to the later
// phases' tiles.  Between phases the library sums the next phase's columns over that node's rank group (X_SUB for an
// inner separator, X_SEP for the root; a shared leaf's columns before the first phase, X_PART), so a phase always
// starts from the complete sums of its columns.  Exactly-once rule: an update from a phase's panels into a LATER
// phase's tile is applied by one rank of the phase's group only -- tile (i, j) by group member (i + j) mod size --
// and the later exchange sums the members' tiles; inside the phase every member applies everything (they all factor
// the phase).  Each member's own Schur partials enter the sum once, as they are.  So the work on the separators'
// Schur complements is split over the group, not replicated.  Tasks, update rules and the panel packing are
// make_plan's (at most two columns per level, no delayed updates).
struct TreePhase {
  int lv0 = 0, lv1 = 0;      // factorisation levels [lv0, lv1) (incl. the closing flush level)
  int kind = PTZBA_X_PART;   // exchange BEFORE this phase (phase 0: X_PART when shared; later: X_SUB / X_SEP)
  int node = -1, r0 = 0, nr = 1, depth = 0;
  int c0 = 0, c1 = 0;        // tile columns
  std::vector<int32_t> xt;   // exchanged tiles (ti, tj) (phase 0: only when shared)
  VecRanges vr{};            // exchanged vector ranges of [b | g | dU]
};
struct TreePlan {
  std::vector<TreePhase> ph;
  std::vector<int8_t> col_phase;  // [T] phase of each tile column, -1 not this rank's
  int base = -1;
};
static bool make_plan_tree(const SysOrder& o, const DistTree& DT, int rank, int n_pose, int nf,
                           const std::vector<int32_t>& win, int64_t ld, CholPlan& P, TreePlan& Q) {
  const int T = (int)(ld / CHOL_NB), taug = o.n_aug / CHOL_NB;
  std::vector<int> anc;
  Q.base = dist_base(DT, rank, &anc);
  const auto& bn = DT.n[Q.base];
  const bool shared = bn.nr >= 2;
  Q.ph.clear();
  {
    TreePhase p0;
    p0.kind = PTZBA_X_PART;
    p0.node = Q.base;
    p0.r0 = shared ? bn.r0 : rank;
    p0.nr = shared ? bn.nr : 1;
    p0.depth = bn.depth;
    p0.c0 = shared ? bn.t0 : bn.st0;
    p0.c1 = shared ? bn.t1 : bn.st1;
    Q.ph.push_back(p0);
  }
  for (int u : anc) {
    TreePhase p;
    p.kind = DT.n[u].parent < 0 ? PTZBA_X_SEP : PTZBA_X_SUB;
    p.node = u;
    p.r0 = DT.n[u].r0;
    p.nr = DT.n[u].nr;
    p.depth = DT.n[u].depth;
    p.c0 = DT.n[u].t0;
    p.c1 = DT.n[u].parent < 0 ? T : DT.n[u].t1;  // the root's phase takes the augmented column too
    Q.ph.push_back(p);
  }
  const int NP = (int)Q.ph.size();
  if (Q.ph.back().c1 != T || taug != T - 1) return false;
  Q.col_phase.assign(T, -1);
  for (int q = 0; q < NP; ++q)
    for (int t = Q.ph[q].c0; t < Q.ph[q].c1; ++t) Q.col_phase[t] = (int8_t)q;
  auto own = [&](int t) { return Q.col_phase[t] >= 0; };
  std::vector<std::vector<uint8_t>> nz(T, std::vector<uint8_t>(T, 0));
  auto mark = [&](int r, int c) {
    int ti = r / CHOL_NB, tj = c / CHOL_NB;
    if (ti < tj) std::swap(ti, tj);
    nz[ti][tj] = 1;
  };
  for (int f1 = nf; f1 < n_pose; ++f1)
    for (int f2 = f1; f2 <= std::min(n_pose - 1, (int)win[f1]); ++f2) {
      const int p1 = o.pos[f1], p2 = o.pos[f2];
      mark(p2, p1); mark(p2 + 2, p1); mark(p2, p1 + 2); mark(p2 + 2, p1 + 2);
    }
  if (shared)  // a shared leaf's columns as the Schur kernels write them (before fill), summed before phase 0
    for (int j = Q.ph[0].c0; j < Q.ph[0].c1; ++j)
      for (int i = j; i < T; ++i)
        if ((nz[i][j] || i == j) && own(i)) { Q.ph[0].xt.push_back(i); Q.ph[0].xt.push_back(j); }
  for (int j = 0; j <= taug; ++j) nz[taug][j] = 1;
  for (int i = 0; i < T; ++i) nz[i][i] = 1;
  for (int k = 0; k < T; ++k) {  // symbolic fill (global)
    std::vector<int> R;
    for (int i = k + 1; i < T; ++i)
      if (nz[i][k]) R.push_back(i);
    for (size_t x = 0; x < R.size(); ++x)
      for (size_t y = 0; y <= x; ++y) nz[R[x]][R[y]] = 1;
  }
  for (int q = 1; q < NP; ++q)  // an ancestor's columns (its rows and the later phases' rows, the augmented row)
    for (int j = Q.ph[q].c0; j < std::min(Q.ph[q].c1, taug); ++j)
      for (int i = j; i < T; ++i)
        if (nz[i][j] && own(i)) { Q.ph[q].xt.push_back(i); Q.ph[q].xt.push_back(j); }
  for (int q = 0; q < NP; ++q) {
    const int64_t r0 = (int64_t)Q.ph[q].c0 * CHOL_NB, r1 = std::min<int64_t>((int64_t)Q.ph[q].c1 * CHOL_NB, o.n_aug);
    const int64_t cnt = std::max<int64_t>(r1 - r0, 0);
    if (q == 0)
      Q.ph[q].vr = VecRanges{{r0, ld + r0, 2 * ld + r0}, {cnt, cnt, cnt}, 3};  // b | g | dU of the shared leaf
    else
      Q.ph[q].vr = VecRanges{{ld + r0, 2 * ld + r0, 0}, {cnt, cnt, 0}, 2};  // g | dU (b rides in the augmented row)
  }
  // the factorisation tasks: make_plan restricted to this rank's phases (delayed trailing updates and 2 x 2
  // trailing blocks included), the exactly-once rule on the later phases' tiles
  TreeSpec ts;
  ts.col_phase = Q.col_phase;
  for (const auto& ph : Q.ph) {
    ts.ph_nr.push_back(ph.nr);
    ts.ph_me.push_back(rank - ph.r0);
  }
  const int n_inv = (o.n_aug + CHOL_NB - 1) / CHOL_NB;
  for (int q = NP - 1; q >= 0; --q)
    for (int kt = std::min(Q.ph[q].c1, n_inv) - 1; kt >= Q.ph[q].c0; --kt) ts.chain.push_back(kt);
  if (!make_plan(o, n_pose, nf, win, ld, P, 0, &ts)) return false;
  for (int q = 0; q < NP; ++q) {
    Q.ph[q].lv0 = ts.ph_lv0[q];
    Q.ph[q].lv1 = ts.ph_lv1[q];
  }
  P.xtiles = Q.ph[0].xt;
  return true;
}

// The order of a part-owned solve: one dissection level (nested_order's choice when it shortens the critical path,
// else its most balanced split) or the two-level order with contiguous halves, whichever gives the slowest rank the
// shorter estimated factorisation (PTZBA_ND_DEPTH=1 keeps one level); false when the chain has no split.  A pure
// function of the coupling window and the world size, so ptzba_partition_landmarks and every rank's set_problem agree.
static bool dist_order(int n_pose, int nf, const std::vector<int32_t>& win, int world, SysOrder& o) {
  if (!(nested_order(n_pose, nf, win, o, false) || nested_order(n_pose, nf, win, o, true))) return false;
  if (getenv_is("PTZBA_ND_DEPTH", "1")) return true;
  SysOrder o2;
  if (!nested_order2(n_pose, nf, win, o2, true) || pad_tile(o2.n_aug + 1) > CHOL_MAX_LD) return true;
  double e[2] = {0, 0};
  const SysOrder* os[2] = {&o, &o2};
  for (int v = 0; v < 2; ++v) {
    DistTree DT;
    if (!dist_tree(*os[v], world, DT)) {
      if (v == 0) return false;
      return true;
    }
    for (int r = 0; r < world; ++r) {
      // ranks sharing a base have the same plan shape: one per base
      if (r > 0 && dist_base(DT, r) == dist_base(DT, r - 1)) continue;
      CholPlan P;
      TreePlan Q;
      if (!make_plan_tree(*os[v], DT, r, n_pose, nf, win, pad_tile(os[v]->n_aug + 1), P, Q)) {
        if (v == 0) return false;
        return true;
      }
      e[v] = std::max(e[v], plan_est_us(P));
    }
  }
  if (e[1] < e[0]) o = std::move(o2);
  return true;
}

// set_problem's device front for large problems (setup_kernels.hip): the records' (landmark, frame, index) order,
// segments and device record arrays (rec_seg, seg_frame / seg_lm / seg_rec_begin, seg_base, rec_xy / rec_w, rec_key,
// perm), bit for bit what the host path uploads; returns the per-segment arrays the host passes read (seg_rec_begin
// with the end entry)
// From 64K records on (round 6; 4M before): a 30-keyframe window's ~170K records take 1.3 ms on the device front against
// 2.2 ms on the host (set_problem per keyframe, config 5: keyframe BA 8.7-9.2 -> 7.9-8.1 ms mean, profiles/r06f_*)
constexpr int64_t GPU_SETUP_MIN_REC = (int64_t)1 << 16;
static int gpu_front(ptzba_ctx* h, int64_t n, int n_pose, int n_lm, const int32_t* frame, const int32_t* lm,
                     const double* xy, const double* w, std::vector<int32_t>& seg_frame, std::vector<int32_t>& seg_lm,
                     std::vector<int64_t>& seg_rec_begin) {
  DBuf order, key;
  int64_t ns = 0;
  {
    DBuf d_frame, d_lm;
    if (d_frame.alloc(4 * (size_t)n) || d_lm.alloc(4 * (size_t)n) || order.alloc(4 * (size_t)n) ||
        key.alloc(4 * (size_t)n) || h->rec_seg.alloc(4 * (size_t)n))
      return -1;
    HIPCHK(hipMemcpyAsync(d_frame.p, frame, 4 * (size_t)n, hipMemcpyHostToDevice, h->st));
    HIPCHK(hipMemcpyAsync(d_lm.p, lm, 4 * (size_t)n, hipMemcpyHostToDevice, h->st));
    // (synchronises: the inputs die here)
    if (setup_sort_runs(h->st, n, n_pose, n_lm, d_frame.as<int32_t>(), d_lm.as<int32_t>(), order.as<uint32_t>(),
                        key.as<uint32_t>(), h->rec_seg.as<int32_t>(), &ns))
      return -1;
  }
  if (ns >= INT32_MAX - 1) return fail("too many segments");
  DBuf lm_first;
  if (h->seg_frame.alloc(4 * (size_t)ns) || h->seg_lm.alloc(4 * (size_t)ns) || h->seg_rec_begin.alloc(8 * (size_t)(ns + 1)) ||
      lm_first.alloc(4 * (size_t)std::max(n_lm, 1)))
    return -1;
  if (setup_fill_segments(h->st, n, n_pose, ns, key.as<uint32_t>(), h->rec_seg.as<int32_t>(), h->seg_frame.as<int32_t>(),
                          h->seg_lm.as<int32_t>(), h->seg_rec_begin.as<int64_t>(), lm_first.as<int32_t>()))
    return -1;
  seg_frame.resize(ns);
  seg_lm.resize(ns);
  seg_rec_begin.resize(ns + 1);
  HIPCHK(hipMemcpyAsync(seg_frame.data(), h->seg_frame.p, 4 * (size_t)ns, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(seg_lm.data(), h->seg_lm.p, 4 * (size_t)ns, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipMemcpyAsync(seg_rec_begin.data(), h->seg_rec_begin.p, 8 * (size_t)(ns + 1), hipMemcpyDeviceToHost, h->st));
  // the records: the raw observations up, the deltas from each segment's base in the record precision
  const size_t e = h->elem();
  DBuf d_xy, d_w;
  if (d_xy.alloc(16 * (size_t)n) || (w && d_w.alloc(8 * (size_t)n)) || h->seg_base.alloc(16 * (size_t)ns) ||
      h->rec_xy.alloc((2 * (size_t)n + 16) * e) || h->rec_key.alloc((size_t)n + 8) || h->perm.alloc(8 * (size_t)n))
    return -1;
  if (w) {
    if (h->rec_w.alloc((size_t)n * e)) return -1;
  } else {
    h->rec_w.release();
  }
  HIPCHK(hipMemcpyAsync(d_xy.p, xy, 16 * (size_t)n, hipMemcpyHostToDevice, h->st));
  if (w) HIPCHK(hipMemcpyAsync(d_w.p, w, 8 * (size_t)n, hipMemcpyHostToDevice, h->st));
  const int rc = h->precision == PTZBA_FP32
                     ? setup_records<float>(h->st, n, ns, order.as<uint32_t>(), h->rec_seg.as<int32_t>(),
                                            h->seg_lm.as<int32_t>(), h->seg_rec_begin.as<int64_t>(), lm_first.as<int32_t>(),
                                            d_xy.as<double>(), w ? d_w.as<double>() : nullptr, h->seg_base.as<double>(),
                                            h->rec_xy.as<float>(), w ? h->rec_w.as<float>() : nullptr,
                                            h->rec_key.as<uint8_t>(), h->perm.as<int64_t>())
                     : setup_records<double>(h->st, n, ns, order.as<uint32_t>(), h->rec_seg.as<int32_t>(),
                                             h->seg_lm.as<int32_t>(), h->seg_rec_begin.as<int64_t>(), lm_first.as<int32_t>(),
                                             d_xy.as<double>(), w ? d_w.as<double>() : nullptr, h->seg_base.as<double>(),
                                             h->rec_xy.as<double>(), w ? h->rec_w.as<double>() : nullptr,
                                             h->rec_key.as<uint8_t>(), h->perm.as<int64_t>());
  if (rc) return rc;
  HIPCHK(hipMemsetAsync(h->rec_xy.as<uint8_t>() + 2 * (size_t)n * e, 0, 16 * e, h->st));  // K1's padded record groups
  HIPCHK(hipMemsetAsync(h->rec_key.as<uint8_t>() + n, 0, 8, h->st));
  HIPCHK(hipStreamSynchronize(h->st));  // the temporaries and the host vectors' copies above complete here
  return 0;
}

int ptzba_set_problem(ptzba_handle h, int32_t n_pose, int32_t n_landmark, int64_t n_obs, const int32_t* obs_frame,
                      const int32_t* obs_landmark, const double* obs_xy, const double* obs_weight, double u, double v,
                      const ptzba_problem_opts* opts) {
  if (!h) return fail("null handle");
  // host phase times of this call (ptzba_setup_timing: where a config-4 set_problem spends its seconds)
  h->setup_phases.clear();
  auto st_t0 = std::chrono::steady_clock::now();
  auto st_mark = [&](const char* what) {
    const auto t = std::chrono::steady_clock::now();
    h->setup_phases.emplace_back(what, std::chrono::duration<double, std::milli>(t - st_t0).count());
    st_t0 = t;
  };
  if (n_pose < 1 || n_landmark < 0 || n_obs < 0) return fail("bad sizes n_pose=%d n_landmark=%d n_obs=%lld", n_pose, n_landmark, (long long)n_obs);
  if (n_obs > 0 && (!obs_frame || !obs_landmark || !obs_xy)) return fail("null observation pointer");
  ptzba_problem_opts o{PTZBA_FP64, PTZBA_LOSS_LINEAR, 1.0, 1, PTZBA_ORDER_NESTED, nullptr};
  if (opts) o = *opts;
  if (o.precision != PTZBA_FP64 && o.precision != PTZBA_FP32) return fail("bad precision %d", o.precision);
  if (o.loss != PTZBA_LOSS_LINEAR && o.loss != PTZBA_LOSS_HUBER) return fail("bad loss %d", o.loss);
  if (o.n_fixed < 0 || o.n_fixed > n_pose) return fail("bad n_fixed %d", o.n_fixed);
  if (o.loss == PTZBA_LOSS_HUBER && !(o.f_scale > 0)) return fail("huber needs f_scale > 0");
  if (o.ordering < PTZBA_ORDER_NATURAL || o.ordering > PTZBA_ORDER_NESTED_FORCE) return fail("bad ordering %d", o.ordering);
  if (o.frame_win_hi)
    for (int f = 0; f < n_pose; ++f)
      if (o.frame_win_hi[f] < f || o.frame_win_hi[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, o.frame_win_hi[f]);
  {
    // record validation over host threads; the error reported is the first bad record's, as a sequential scan's
    const int T = host_threads(n_obs);
    std::vector<int64_t> first_bad(T, n_obs);
    parallel_chunks(n_obs, T, [&](int64_t lo, int64_t hi, int t) {
      for (int64_t r = lo; r < hi; ++r)
        if (obs_frame[r] < 0 || obs_frame[r] >= n_pose || obs_landmark[r] < 0 || obs_landmark[r] >= n_landmark ||
            !std::isfinite(obs_xy[2 * r]) || !std::isfinite(obs_xy[2 * r + 1]) || (obs_weight && !(obs_weight[r] >= 0))) {
          first_bad[t] = r;
          return;
        }
    });
    const int64_t r = *std::min_element(first_bad.begin(), first_bad.end());
    if (r < n_obs) {
      if (obs_frame[r] < 0 || obs_frame[r] >= n_pose) return fail("record %lld: frame %d out of range", (long long)r, obs_frame[r]);
      if (obs_landmark[r] < 0 || obs_landmark[r] >= n_landmark)
        return fail("record %lld: landmark %d out of range", (long long)r, obs_landmark[r]);
      if (!std::isfinite(obs_xy[2 * r]) || !std::isfinite(obs_xy[2 * r + 1])) return fail("record %lld: non-finite observation", (long long)r);
      return fail("record %lld: negative weight", (long long)r);
    }
  }
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  h->have_problem = false;
  h->ptz_saved.release();
  h->rays_saved.release();
  h->n_pose = n_pose;
  h->n_lm = n_landmark;
  h->n_rec = n_obs;
  h->precision = o.precision;
  h->loss = o.loss;
  h->fs = o.f_scale;
  h->hcurv = 1.0;
  h->n_fixed = o.n_fixed;
  h->u = u;
  h->v = v;
  h->weighted = obs_weight != nullptr;

  st_mark("validate");
  // large problems (configs 3 and 4: 14.6M / 410M records): the order, the segment runs and the record arrays are
  // built on the device (setup_kernels.hip: one stable radix sort of the composite key landmark * n_pose + frame --
  // the same order as the host's two stable counting sorts); the host keeps only the per-segment arrays its
  // structure passes read.  Smaller ones (a sliding window's ~170K records) stay on the host.
  const bool gpu_setup = n_obs >= (h->gpu_setup_min >= 0 ? h->gpu_setup_min : GPU_SETUP_MIN_REC) && n_obs > 0 &&
                         n_obs < ((int64_t)1 << 31) &&
                         (uint64_t)n_landmark * (uint64_t)n_pose <= ((uint64_t)1 << 32);
  // ---- stable counting sorts: by frame, then by landmark -> (landmark, frame, original index)
  std::vector<int64_t> tmp, order(gpu_setup ? 0 : n_obs), lm_start;
  std::vector<int32_t> sorted_frame;  // single-thread path: obs_frame in sorted order
  // large problems (config 4: 410M records) sort on host threads: the same stable order (par_util.h)
  const bool par_host = !gpu_setup && host_threads(n_obs) > 1;
  if (gpu_setup) {
    // sorted in the segment phase below
  } else if (par_host) {
    tmp.resize(n_obs);
    parallel_counting_sort(n_obs, n_pose, (const int64_t*)nullptr, tmp.data(), [&](int64_t r) { return obs_frame[r]; });
    parallel_counting_sort(n_obs, n_landmark, tmp.data(), order.data(), [&](int64_t r) { return obs_landmark[r]; });
  } else {
    // two stable counting passes (by frame, then by landmark) -> (landmark, frame, record) order; the second pass
    // walks the records frame by frame, so each record's frame is known without a lookup and lands in sorted_frame
    // beside `order` -- the segment pass below then streams over it (per-landmark comparison sorts measured 2.4x
    // slower at a window's ~250 records per landmark)
    std::vector<int64_t> fo(n_pose + 1, 0);
    for (int64_t r = 0; r < n_obs; ++r) fo[obs_frame[r] + 1]++;
    for (int f = 0; f < n_pose; ++f) fo[f + 1] += fo[f];
    tmp.resize(n_obs);
    {
      std::vector<int64_t> c(fo.begin(), fo.end() - 1);
      for (int64_t r = 0; r < n_obs; ++r) tmp[c[obs_frame[r]]++] = r;
    }
    lm_start.assign(n_landmark + 1, 0);
    for (int64_t r = 0; r < n_obs; ++r) lm_start[obs_landmark[r] + 1]++;
    for (int l = 0; l < n_landmark; ++l) lm_start[l + 1] += lm_start[l];
    sorted_frame.resize(n_obs);
    {
      std::vector<int64_t> c(lm_start.begin(), lm_start.end() - 1);
      for (int f = 0; f < n_pose; ++f)
        for (int64_t k = fo[f]; k < fo[f + 1]; ++k) {
          const int64_t r = tmp[k];
          const int64_t q = c[obs_landmark[r]]++;
          order[q] = r;
          sorted_frame[q] = f;
        }
    }
  }
  st_mark("sort");
  // ---- segments (unique landmark, frame)
  std::vector<int32_t> seg_frame, seg_lm, rec_seg(gpu_setup ? 0 : n_obs);
  std::vector<int64_t> seg_rec_begin;
  std::vector<int32_t> lm_seg_begin(n_landmark + 1, 0);
  if (gpu_setup) {
    if (gpu_front(h, n_obs, n_pose, n_landmark, obs_frame, obs_landmark, obs_xy, obs_weight, seg_frame, seg_lm,
                  seg_rec_begin))
      return -1;
    // segments are landmark-ordered: each landmark's first segment, landmarks without one take the next's
    const int64_t ns = (int64_t)seg_frame.size();
    std::vector<int32_t> first(n_landmark + 1, -1);
    first[n_landmark] = (int32_t)ns;
    for (int64_t sg = 0; sg < ns; ++sg)
      if (sg == 0 || seg_lm[sg] != seg_lm[sg - 1]) first[seg_lm[sg]] = (int32_t)sg;
    for (int l = n_landmark - 1; l >= 0; --l)
      if (first[l] < 0) first[l] = first[l + 1];
    lm_seg_begin.assign(first.begin(), first.end());
  } else if (par_host) {
    // two passes over the same record chunks: count the segment starts per chunk, then fill at the prefix offsets
    const int T = host_threads(n_obs);
    auto is_start = [&](int64_t k) {
      return k == 0 || obs_landmark[order[k]] != obs_landmark[order[k - 1]] || obs_frame[order[k]] != obs_frame[order[k - 1]];
    };
    std::vector<int64_t> base(T + 1, 0);
    parallel_chunks(n_obs, T, [&](int64_t lo, int64_t hi, int t) {
      int64_t c = 0;
      for (int64_t k = lo; k < hi; ++k) c += is_start(k);
      base[t + 1] = c;
    });
    for (int t = 0; t < T; ++t) base[t + 1] += base[t];
    if (base[T] >= INT32_MAX - 1) return fail("too many segments");
    seg_frame.resize(base[T]);
    seg_lm.resize(base[T]);
    seg_rec_begin.resize(base[T]);
    parallel_chunks(n_obs, T, [&](int64_t lo, int64_t hi, int t) {
      int64_t sg = base[t] - 1;
      for (int64_t k = lo; k < hi; ++k) {
        if (is_start(k)) {
          const int64_t r = order[k];
          ++sg;
          seg_frame[sg] = obs_frame[r];
          seg_lm[sg] = obs_landmark[r];
          seg_rec_begin[sg] = k;
        }
        rec_seg[k] = (int32_t)sg;
      }
    });
    // segments are landmark-ordered: each landmark's first segment, landmarks without one take the next's
    std::vector<int32_t> first(n_landmark + 1, -1);
    first[n_landmark] = (int32_t)base[T];
    for (int64_t sg = 0; sg < base[T]; ++sg)
      if (sg == 0 || seg_lm[sg] != seg_lm[sg - 1]) first[seg_lm[sg]] = (int32_t)sg;
    for (int l = n_landmark - 1; l >= 0; --l)
      if (first[l] < 0) first[l] = first[l + 1];
    lm_seg_begin.assign(first.begin(), first.end());
  } else {
    seg_frame.reserve(n_obs / 4 + 16);
    seg_lm.reserve(n_obs / 4 + 16);
    seg_rec_begin.reserve(n_obs / 4 + 16);
    for (int l = 0; l < n_landmark; ++l) {
      lm_seg_begin[l] = (int32_t)seg_frame.size();
      for (int64_t k = lm_start[l]; k < lm_start[l + 1]; ++k) {
        if (k == lm_start[l] || sorted_frame[k] != sorted_frame[k - 1]) {
          if ((int64_t)seg_frame.size() >= INT32_MAX - 1) return fail("too many segments");
          seg_frame.push_back(sorted_frame[k]);
          seg_lm.push_back(l);
          seg_rec_begin.push_back(k);
        }
        rec_seg[k] = (int32_t)seg_frame.size() - 1;
      }
    }
    lm_seg_begin[n_landmark] = (int32_t)seg_frame.size();
  }
  const int64_t n_seg = (int64_t)seg_frame.size();
  if (!gpu_setup) seg_rec_begin.push_back(n_obs);  // (the device front returns the end entry with the segments)
  h->n_seg = n_seg;
  // ---- frame CSR over segments (stable: landmark ascending within a frame)
  std::vector<int32_t> frame_seg_begin(n_pose + 1, 0), frame_seg_list(n_seg), frame_win_hi(n_pose);
  for (int64_t s = 0; s < n_seg; ++s) frame_seg_begin[seg_frame[s] + 1]++;
  for (int f = 0; f < n_pose; ++f) frame_seg_begin[f + 1] += frame_seg_begin[f];
  if ((par_host || gpu_setup) && host_threads(n_seg) > 1) {
    parallel_counting_sort(n_seg, n_pose, (const int32_t*)nullptr, frame_seg_list.data(),
                           [&](int32_t sg) { return seg_frame[sg]; });
  } else {
    std::vector<int32_t> c(frame_seg_begin.begin(), frame_seg_begin.end() - 1);
    for (int64_t s = 0; s < n_seg; ++s) frame_seg_list[c[seg_frame[s]]++] = (int32_t)s;
  }
  parallel_chunks(n_pose, (par_host || gpu_setup) ? std::min(host_threads(n_obs), n_pose) : 1, [&](int64_t f0, int64_t f1, int) {
    for (int64_t f = f0; f < f1; ++f) {
      int hi = (int)f;
      for (int e = frame_seg_begin[f]; e < frame_seg_begin[f + 1]; ++e) {
        int l = seg_lm[frame_seg_list[e]];
        hi = std::max(hi, seg_frame[lm_seg_begin[l + 1] - 1]);
      }
      frame_win_hi[f] = hi;
    }
  });
  st_mark("segments+frame csr");
  // ---- register-blocked K2 structure: per landmark its frame range [first, last] and a dense W slot
  // per frame in it; K2 tiles (SCHUR_F1 frames x 64 partner frames) with the landmarks that reach them,
  std::vector<int32_t> lm_meta(4 * (size_t)std::max(n_landmark, 1), 0), s2_items, s2_groups,
      s2_lm;
  {
    int64_t toff = 0;
    for (int l = 0; l < n_landmark; ++l) {
      const int s0 = lm_seg_begin[l], s1 = lm_seg_begin[l + 1];
      if (s1 == s0) continue;
      const int lo = seg_frame[s0], hi = seg_frame[s1 - 1];  // segments are frame-ordered per landmark
      lm_meta[4 * l] = lo;
      lm_meta[4 * l + 1] = hi;
      lm_meta[4 * l + 2] = (int32_t)toff;
      toff += hi - lo + 1;
      if (toff >= INT32_MAX) return fail("landmark x frame slot table exceeds 2^31 rows");
    }
    h->n_slot = toff;
    // split size: about two work items per CU over the whole list volume, at least 64 landmarks
    std::vector<std::vector<int32_t>> tiles;
    std::vector<int32_t> tile_key;
    std::vector<int32_t> un;
    // the landmarks of an F1 block, ascending and unique: marked in a bitmap, then read out word by word between the
    // lowest and highest marked word (no sort: a config-5 window's single block holds ~100K segments)
    std::vector<uint64_t> lm_bits((size_t)n_landmark / 64 + 1, 0);
    for (int f1b = o.n_fixed; f1b < n_pose; f1b += SCHUR_F1) {
      un.clear();
      size_t w_lo = lm_bits.size(), w_hi = 0;
      for (int f = f1b; f < std::min(n_pose, f1b + SCHUR_F1); ++f)
        for (int e = frame_seg_begin[f]; e < frame_seg_begin[f + 1]; ++e) {
          const uint32_t l = (uint32_t)seg_lm[frame_seg_list[e]];
          lm_bits[l >> 6] |= 1ull << (l & 63);
          w_lo = std::min<size_t>(w_lo, l >> 6);
          w_hi = std::max<size_t>(w_hi, l >> 6);
        }
      for (size_t wd = w_lo; wd <= w_hi && w_lo < lm_bits.size(); ++wd) {
        uint64_t m = lm_bits[wd];
        lm_bits[wd] = 0;
        while (m) {
          un.push_back((int32_t)(wd * 64 + __builtin_ctzll(m)));
          m &= m - 1;
        }
      }
      int hi = f1b;
      for (int l : un) hi = std::max(hi, lm_meta[4 * l + 1]);
      const int nc = (hi - f1b) / WAVE + 1;
      for (int c = 0; c < nc; ++c) {
        // a landmark enters chunk c only when it sees a frame of the chunk (its frame set can have gaps:
        // on a multi-row keyframe grid a landmark seen by two tilt rows spans a whole row of frames)
        std::vector<int32_t> lst;
        const int c_lo = f1b + WAVE * c, c_hi = c_lo + WAVE - 1;
        for (int l : un) {
          if (c > 0) {
            if (lm_meta[4 * l + 1] < c_lo) continue;
            const int32_t* fb = seg_frame.data() + lm_seg_begin[l];
            const int32_t* fe = seg_frame.data() + lm_seg_begin[l + 1];
            const int32_t* it = std::lower_bound(fb, fe, c_lo);
            if (it == fe || *it > c_hi) continue;
          }
          lst.push_back(l);
        }
        if (lst.empty()) continue;
        tiles.push_back(std::move(lst));
        tile_key.push_back(f1b);
        tile_key.push_back(c);
      }
    }
    // split size: at most 256 work items (one round of one workgroup per CU) counting the per-tile rounding, at
    // least 64 landmarks, at most SCHUR_LMAX (the LDS list).  Chunk-0 items also sum the diagonal terms: their
    // lists are weighted (6 / 4; per-item clock stamps, tools/schur_items.py, put a chunk-0 landmark at 1.5-1.9x
    // the time of another's; 5 / 4 before round 5) so that the items of the round end together.
    int64_t W0 = 6;
    constexpr int64_t WD = 4;  // chunk-0 weight W0 / WD
    int64_t total_w = 0;
    for (size_t k = 0; k < tiles.size(); ++k)
      total_w += (int64_t)tiles[k].size() * (tile_key[2 * k + 1] == 0 ? W0 : WD);
    const int64_t n_tiles = (int64_t)tiles.size();
    // item target: at most 256 (ONE round of one 512-thread workgroup per CU: k_schur_mf's ~100 KB of LDS allows one
    // per CU) -- same-box A/B at config 3 (r04j, r04p): 256 items 64.7-64.8 us per build against 73.3-74.6 with 512
    // (two rounds), 68.0 with 192, 84.8 with 320; proportionally fewer for less work -- a rank's shard of a sharded
    // solve: each item's 74 KB split partial and the reduce over its tile's splits are fixed costs (measured at
    // config 3, tools/dist_model.py: N = 8 shard 44-66 -> 37-47 us with 64-128 items)
    int64_t target_items = std::min<int64_t>(256, std::max<int64_t>(64, (512 * total_w) / 480000));
    // the smallest split weight whose per-tile rounding still fits the target (binary search: the item count falls as
    // the split grows), so the items are as short -- and the one round as even -- as the target allows
    auto items_for = [&](int64_t sw) {
      int64_t c = 0;
      for (size_t k = 0; k < tiles.size(); ++k) {
        const int64_t n = (int64_t)tiles[k].size(), nw = n * (tile_key[2 * k + 1] == 0 ? W0 : WD);
        c += std::max<int64_t>((nw + sw - 1) / sw, (n + SCHUR_LMAX - 1) / SCHUR_LMAX);
      }
      return c;
    };
    int64_t sw_lo = 64 * WD, sw_hi = std::max<int64_t>(sw_lo, total_w);
    if (items_for(sw_lo) <= target_items) {
      sw_hi = sw_lo;
    } else {
      while (sw_hi - sw_lo > 1) {  // items_for(sw_lo) > target >= items_for(sw_hi)
        const int64_t mid = (sw_lo + sw_hi) / 2;
        if (items_for(mid) <= target_items) sw_hi = mid;
        else sw_lo = mid;
      }
    }
    (void)n_tiles;
    const int64_t split_w = sw_hi;
    for (size_t k = 0; k < tiles.size(); ++k) {
      const auto& lst = tiles[k];
      const int n = (int)lst.size();
      const int64_t nw = (int64_t)n * (tile_key[2 * k + 1] == 0 ? W0 : WD);
      const int nparts = (int)std::max<int64_t>((nw + split_w - 1) / split_w, (n + SCHUR_LMAX - 1) / SCHUR_LMAX);
      const int i0 = (int)(s2_items.size() / 4);
      for (int pp = 0; pp < nparts; ++pp) {
        const int a0 = (int)((int64_t)n * pp / nparts), a1 = (int)((int64_t)n * (pp + 1) / nparts);
        const int b0 = (int)(s2_lm.size() / 4);
        for (int q = a0; q < a1; ++q) {
          const int l = lst[q];
          s2_lm.insert(s2_lm.end(), {l, lm_meta[4 * l], lm_meta[4 * l + 1], lm_meta[4 * l + 2]});
        }
        s2_items.insert(s2_items.end(), {tile_key[2 * k], tile_key[2 * k + 1], b0, (int32_t)(s2_lm.size() / 4)});
      }
      s2_groups.insert(s2_groups.end(), {tile_key[2 * k], tile_key[2 * k + 1], i0, (int32_t)(s2_items.size() / 4)});
    }
    h->n_s2_groups = (int)(s2_groups.size() / 4);
    h->n_s2_items = (int)(s2_items.size() / 4);
    {
      std::vector<uint8_t> cov((n_pose + SCHUR_F1) / SCHUR_F1 + 1, 0);
      for (size_t g = 0; g < s2_groups.size(); g += 4)
        if (s2_groups[g + 1] == 0) cov[(s2_groups[g] - o.n_fixed) / SCHUR_F1] = 1;
      h->f1_covered = true;
      for (int f1b = o.n_fixed; f1b < n_pose; f1b += SCHUR_F1)
        if (!cov[(f1b - o.n_fixed) / SCHUR_F1]) h->f1_covered = false;
    }
  }
  st_mark("k2 structure");
  // ---- landmark work order: heaviest (most records) first
  std::vector<int32_t> lm_order;
  int max_seg = 0;
  for (int l = 0; l < n_landmark; ++l) {
    int ns = lm_seg_begin[l + 1] - lm_seg_begin[l];
    if (ns > 0) lm_order.push_back(l);
    max_seg = std::max(max_seg, ns);
  }
  {
    // heaviest first (LPT over the workgroup slots) at 1/8-octave resolution of the record count, and inside such a
    // size class by first frame: a K1 workgroup's landmarks then see neighbouring frames, so it stages ~a coupling
    // window of frame tables instead of the whole table (ba_kernels.hip FTL)
    auto nrec = [&](int l) { return seg_rec_begin[lm_seg_begin[l + 1]] - seg_rec_begin[lm_seg_begin[l]]; };
    auto size_class = [&](int l) {
      const uint64_t c = (uint64_t)nrec(l);
      if (c < 16) return (int)c;
      const int msb = 63 - __builtin_clzll(c);
      return 16 + 8 * (msb - 4) + (int)((c >> (msb - 3)) & 7);
    };
    std::vector<int64_t> key(n_landmark, 0);
    for (int l : lm_order) key[l] = ((int64_t)(1 << 20) - size_class(l)) * ((int64_t)1 << 40) + ((int64_t)lm_meta[4 * l] << 20);
    std::sort(lm_order.begin(), lm_order.end(), [&](int a, int b) { return key[a] != key[b] ? key[a] < key[b] : a < b; });
  }
  h->n_work = (int)lm_order.size();
  h->max_seg_per_lm = max_seg;
  if (n_obs >= ((int64_t)1 << 31)) return fail("n_obs %lld exceeds the 2^31 record limit of a handle (shard it)", (long long)n_obs);
  // K1 work descriptors, 32 B: {landmark, first segment, end segment, first record | first frame, last
  // frame, slot offset (lm_meta), end record of the first K1_SEGW-segment window}
  std::vector<int32_t> lm_work(8 * (size_t)h->n_work);
  for (int k = 0; k < h->n_work; ++k) {
    const int l = lm_order[k];
    lm_work[8 * k + 0] = l;
    lm_work[8 * k + 1] = lm_seg_begin[l];
    lm_work[8 * k + 2] = lm_seg_begin[l + 1];
    lm_work[8 * k + 3] = (int32_t)seg_rec_begin[lm_seg_begin[l]];
    for (int q = 0; q < 3; ++q) lm_work[8 * k + 4 + q] = lm_meta[4 * l + q];
    lm_work[8 * k + 7] = (int32_t)seg_rec_begin[std::min(lm_seg_begin[l + 1], lm_seg_begin[l] + K1_SEGW)];
  }
  h->n_sys = 3 * (n_pose - o.n_fixed);
  // system order and factorisation plan (from the coupling window; a sharded problem passes the global one)
  std::vector<int32_t> win(frame_win_hi);
  if (o.frame_win_hi)
    for (int f = 0; f < n_pose; ++f) win[f] = std::max(win[f], o.frame_win_hi[f]);
  // multi-GPU: part-owned solve when the frame chain splits (the landmarks partitioned accordingly by
  // ptzba_partition_landmarks), else every rank factors the whole summed system (replicated)
  const bool dist = o.dist_world >= 2;
  if (dist && (o.dist_rank < 0 || o.dist_rank >= o.dist_world))
    return fail("bad rank %d of %d", o.dist_rank, o.dist_world);
  if (dist && !o.frame_win_hi) return fail("a sharded solve needs the global coupling window (frame_win_hi)");
  SysOrder sorder;
  const bool part_mode = dist && dist_order(n_pose, o.n_fixed, win, o.dist_world, sorder);
  CholPlan plan;
  if (!part_mode && choose_order_plan(n_pose, o.n_fixed, win, o.ordering, sorder, plan))
    return fail("factorisation plan: an update task needs more than four panels");
  h->n_aug = sorder.n_aug;
  h->nested = sorder.nested;
  h->nd_depth = sorder.nd_depth;
  h->ld = pad_tile(h->n_aug + 1);  // + augmented rhs row
  // the back-substitution keeps x ([ld] doubles) in LDS
  if (h->ld > CHOL_MAX_LD) return fail("reduced system %d too large for the dense solver", h->n_sys);
  TreePlan tplan;
  h->dist_world = dist ? o.dist_world : 1;
  h->dist_rank = dist ? o.dist_rank : 0;
  h->dist_mode = part_mode ? 1 : 0;
  h->n_phase = 0;
  h->base_node = -1;
  h->tree_depth = 0;
  h->tree_groups.clear();
  std::vector<uint8_t> row_phase, fmask;
  h->owned_host.assign(n_pose, 1);
  if (part_mode) {
    DistTree DT;
    if (!dist_tree(sorder, o.dist_world, DT) ||
        !make_plan_tree(sorder, DT, o.dist_rank, n_pose, o.n_fixed, win, h->ld, plan, tplan))
      return fail("part-owned plan: the parts are coupled (bad coupling window)");
    if ((int)tplan.ph.size() > ptzba_ctx::MAX_PHASES) return fail("rank tree deeper than %d phases", ptzba_ctx::MAX_PHASES);
    h->base_node = tplan.base;
    h->tree_depth = DT.depth;
    for (int v = 1; v < (int)DT.n.size(); ++v)
      if (DT.n[v].nr >= 2 && (DT.n[v].nch == 2 || true)) {
        bool dup = false;
        for (size_t q = 0; q < h->tree_groups.size(); q += 3)
          dup = dup || (h->tree_groups[q] == DT.n[v].r0 && h->tree_groups[q + 1] == DT.n[v].nr);
        if (!dup) h->tree_groups.insert(h->tree_groups.end(), {DT.n[v].r0, DT.n[v].nr, DT.n[v].depth});
      }
    auto fphase = [&](int f) { return sorder.pos[f] < 0 ? -1 : (int)tplan.col_phase[sorder.pos[f] / CHOL_NB]; };
    for (int64_t r = 0; r < n_obs; ++r)
      if (obs_frame[r] >= o.n_fixed && fphase(obs_frame[r]) < 0)
        return fail("record %lld sees frame %d outside rank %d's part (partition the landmarks with "
                    "ptzba_partition_landmarks)", (long long)r, obs_frame[r], o.dist_rank);
    fmask.assign(n_pose, 0);
    for (int f = 0; f < n_pose; ++f) {
      const int q = f < o.n_fixed ? -1 : fphase(f);
      const bool owned = q >= 0;
      h->owned_host[f] = owned ? 1 : 0;
      // each frame's pose partials counted by one rank: its phase group's first rank (fixed frames: rank 0)
      const bool counted = f < o.n_fixed ? o.dist_rank == 0 : (owned && o.dist_rank == tplan.ph[q].r0);
      fmask[f] = (uint8_t)((owned ? 1 : 0) | (counted ? 2 : 0));
    }
    row_phase.assign(h->n_aug, 0);
    for (int r = 0; r < h->n_aug; ++r) row_phase[r] = (uint8_t)(tplan.col_phase[r / CHOL_NB] + 1);
    h->n_phase = (int)tplan.ph.size();
    for (int q = 0; q < h->n_phase; ++q) {
      const auto& tp = tplan.ph[q];
      auto& d = h->ph[q];
      d.lv0 = tp.lv0;
      d.lv1 = tp.lv1;
      d.kind = tp.kind;
      d.r0 = tp.r0;
      d.nr = tp.nr;
      d.depth = tp.depth;
      d.node = tp.node;
      d.n_tiles = (int)(tp.xt.size() / 2);
      d.vr = tp.vr;
      d.n_buf = (q == 0 && tp.nr < 2) ? 0 : (int64_t)d.n_tiles * CHOL_NB * CHOL_NB + tp.vr.count[0] + tp.vr.count[1] + tp.vr.count[2];
    }
  }
  h->chol_task_off = plan.level_off;
  h->chol_tasks_host = plan.tasks;
  h->n_tinv_tail = (int)plan.tinv_tail.size();
  h->chol_levels = plan.n_levels;
  h->chol_delayed = plan.delayed;
  h->n_chain = (int)plan.chain_off.size() - 1;
  frame_win_hi = win;  // K2 windows follow the same (possibly global) coupling
  h->perm_uploaded = gpu_setup;  // (the device front wrote the permutation itself)
  if (gpu_setup) h->perm_host.clear();

  st_mark("work order+plan");
  // ---- upload (staged: the stream has drained, so the staging buffer is free)
  HIPCHK(hipStreamSynchronize(h->st));
  h->stage_used = 0;
  h->stage_ops.clear();
  // the staged uploads / zero fills land with one copy + one scatter launch (0.73 -> 0.66 ms per config-5 call, r04z4)
  h->stage_batch = true;
  struct BatchOff {  // every exit (errors included) leaves the batching off
    ptzba_ctx* h;
    ~BatchOff() { h->stage_batch = false; }
  } batch_off{h};
  st_mark("pre-upload sync");
  if (!gpu_setup) {  // (the device front has built these on the device)
    std::vector<double> seg_base(2 * n_seg);
    for (int64_t s = 0; s < n_seg; ++s) {
      const int64_t r = order[seg_rec_begin[s]];
      seg_base[2 * s] = obs_xy[2 * r];
      seg_base[2 * s + 1] = obs_xy[2 * r + 1];
    }
    int rc = h->precision == PTZBA_FP32 ? upload_records<float>(h, order, rec_seg, seg_base, obs_xy, obs_weight)
                                        : upload_records<double>(h, order, rec_seg, seg_base, obs_xy, obs_weight);
    if (rc) return rc;
    if (upload_st(h, h->seg_base, seg_base)) return -1;
    {  // K1's 1-byte segment key: the record's segment within its landmark's window of K1_SEGW segments
      std::vector<uint8_t> key(n_obs + 8);  // + 8: K1 reads whole 8-record key groups
      for (int64_t k = 0; k < n_obs; ++k) {
        const int32_t sg = rec_seg[k];
        key[k] = (uint8_t)((sg - lm_seg_begin[seg_lm[sg]]) % K1_SEGW);
      }
      if (upload_st(h, h->rec_key, key)) return -1;
    }
    if (upload_st(h, h->rec_seg, rec_seg) || upload_st(h, h->seg_frame, seg_frame) || upload_st(h, h->seg_lm, seg_lm) ||
        upload_st(h, h->seg_rec_begin, seg_rec_begin))
      return -1;
    h->perm_host = std::move(order);
  }
  if (upload_st(h, h->lm_seg_begin, lm_seg_begin) ||
      upload_st(h, h->lm_order, lm_work) || upload_st(h, h->frame_seg_begin, frame_seg_begin) ||
      upload_st(h, h->frame_seg_list, frame_seg_list) || upload_st(h, h->frame_win_hi, frame_win_hi) ||
      upload_st(h, h->s2_items, s2_items) || upload_st(h, h->s2_groups, s2_groups) || upload_st(h, h->s2_lm, s2_lm) ||
      upload_st(h, h->lm_meta, lm_meta))
    return -1;
  const size_t e = h->elem();
  if (h->ptz.alloc(3 * n_pose * 8) || h->ptz_trial.alloc(3 * n_pose * 8) || h->rays.alloc(2 * (size_t)n_landmark * 8) ||
      h->rays_trial.alloc(2 * (size_t)n_landmark * 8) || h->D_pose.alloc(3 * n_pose * 8) ||
      h->D_ray.alloc(2 * (size_t)n_landmark * 8) || h->ft.alloc((size_t)n_pose * 8 * e) ||
      h->rt.alloc((size_t)n_landmark * 8 * e) || h->ft64.alloc((size_t)n_pose * 64) ||
      h->rt64.alloc((size_t)n_landmark * 64) || h->ug_slot[0].alloc((size_t)std::max<int64_t>(h->n_slot, 1) * UG_STRIDE * e) ||
      h->ug_slot[1].alloc((size_t)std::max<int64_t>(h->n_slot, 1) * UG_STRIDE * e) || h->w_slot[0].alloc((size_t)std::max<int64_t>(h->n_slot, 1) * W_STRIDE * e) ||
      h->w_slot[1].alloc((size_t)std::max<int64_t>(h->n_slot, 1) * W_STRIDE * e) || h->lm_out[0].alloc((size_t)n_landmark * 8 * 8) ||
      h->lm_out[1].alloc((size_t)n_landmark * 8 * 8) || h->lm_aux.alloc((size_t)n_landmark * 8 * 8) ||
      h->lm_red.alloc((size_t)n_landmark * 4 * 8) || h->sys.alloc((size_t)h->sys_count() * 8) ||
      h->scal.alloc(2 * PTZBA_NSCALARS * 8) || h->red_scratch.alloc(RED_SCRATCH * 8) || h->info.alloc(16) ||
      h->Ldiag.alloc((size_t)h->ld * CHOL_NB * 8) || h->Minv.alloc((size_t)h->ld * CHOL_NB * 8) ||
      h->dpose.alloc((size_t)h->ld * 8) ||
      h->s2_part.alloc((size_t)std::max(h->n_s2_items, 1) * SCHUR_F1 * 9 * WAVE * 8) ||
      h->part_diag.alloc((size_t)std::max(h->n_s2_items, 1) * SCHUR_F1 * 12 * 8))
    return -1;
  if (upload_st(h, h->chol_tasks, plan.tasks) || upload_st(h, h->tinv_tail, plan.tinv_tail) || upload_st(h, h->frame_pos, sorder.pos) || upload_st(h, h->row_pad, sorder.pad) ||
      upload_st(h, h->bs_chain_off, plan.chain_off) || upload_st(h, h->bs_chain_cols, plan.chain_cols) ||
      upload_st(h, h->bs_upd_off, plan.upd_off) || upload_st(h, h->bs_upd_tiles, plan.upd_tiles) || upload_st(h, h->xtiles, plan.xtiles) || upload_st(h, h->ztiles, plan.ztiles) ||
      upload_st(h, h->bs_la_tasks, plan.la_tasks) || upload_st(h, h->bs_lo_off, plan.lo_off) || upload_st(h, h->bs_lo_tiles, plan.lo_tiles))
    return -1;
  if (part_mode) {
    if (upload_st(h, h->row_phase, row_phase) || upload_st(h, h->fmask, fmask)) return -1;
    for (int q = 0; q < h->n_phase; ++q)
      if (upload_st(h, h->ph_tiles[q], tplan.ph[q].xt) || h->ph_buf[q].alloc((size_t)std::max<int64_t>(h->ph[q].n_buf, 1) * 8))
        return -1;
  } else {
    h->row_phase.release();
    h->fmask.release();
  }
  for (int q = h->n_phase; q < ptzba_ctx::MAX_PHASES; ++q) {
    h->ph_tiles[q].release();
    h->ph_buf[q].release();
  }
  if (zero_async(h, h->dpose.p, h->dpose.bytes)) return -1;  // rows a part-owned rank never solves
  h->n_xtiles = (int)(plan.xtiles.size() / 2);
  h->n_ztiles = (int)(plan.ztiles.size() / 2);
  if (zero_async(h, h->sys.p, h->sys.bytes)) return -1;  // outside the factor's tiles it is never written
  h->bs_nupd = (int)plan.upd_tiles.size();
  h->bs_npos = (int)plan.chain_cols.size();
  h->bs_ntasks = plan.n_tasks;
  // the back-substitution keeps r and its update lists in LDS (plus ~9 KiB of static staging)
  // (lookahead form: + 48 KiB ring of M / L blocks)
  // (lookahead form: + 48 KiB ring of M / L blocks); larger systems take the left-looking form, whose lists
  // stay in global memory
  h->bs_ll = h->ld * 8 + (std::max(h->bs_npos + 1 + h->bs_nupd, 2 * h->bs_npos + h->bs_ntasks)) * 4 > 100 * 1024;
  // systems of >= 512 rows take the blocked right-looking form (many CUs per step) when the plan has a valid
  // schedule: the lookahead form reads the whole band of L through one CU per chain (config 3, same-box A/B
  // r03ab: cholesky_solve 0.261 -> 0.248 ms per trial); smaller ones (sliding windows) keep the lookahead form.
  // Knobs: PTZBA_BACKSOLVE=la (lookahead while its lists fit LDS) / =ll (left-looking) / =blk (blocked, any size)
  const char* bse = getenv("PTZBA_BACKSOLVE");
  const std::string bsk = bse ? bse : "";
  const bool want_blk = bsk == "blk" || (bsk.empty() && (h->bs_ll || h->n_aug >= 512));
  h->bs_blk = (want_blk || (h->bs_ll && bsk != "ll")) && bsk != "ll" && !plan.bsb_tasks.empty();
  h->bs_ll = (h->bs_ll || bsk == "ll") && !h->bs_blk;
  h->bsb_step_off = plan.bsb_step_off;
  // persistent form: every step's tasks in one launch (all resident at <= 512 workgroups); PTZBA_BS_PERSIST=0 keeps
  // one launch per step (the bitwise schedule test compares both; same-box A/B r04a: cholesky_solve 245 -> 241 us
  // per trial at config 3)
  h->bs_pst = h->bs_blk && !getenv_is("PTZBA_BS_PERSIST", "0") &&
              plan.bsb_tasks.size() / 12 <= 512;  // (2 workgroups per CU resident: 190 VGPRs)
  h->bsp_epoch = 0;
  h->no_fused_prep = getenv("PTZBA_NO_FUSED_PREP") != nullptr;
  if (h->bs_pst && !h->bsp_err) HIPCHK(hipHostMalloc((void**)&h->bsp_err, sizeof(int), hipHostMallocDefault));
  if (h->bsp_err) *h->bsp_err = 0;  // (a wait that gave up under an earlier problem does not outlive it)
  if (h->bs_pst) {
    if (upload_st(h, h->bsp_expect, plan.bsb_expect) || upload_st(h, h->bsp_tot, plan.bsb_tot) ||
        h->bsp_cnt.alloc(4 * plan.bsb_tot.size()))
      return -1;
    if (zero_async(h, h->bsp_cnt.p, h->bsp_cnt.bytes)) return -1;
  }
  if (h->bs_blk) {
    if (upload_st(h, h->bsb_tasks, plan.bsb_tasks) ||
        h->bsb_r.alloc((size_t)h->ld * 8))
      return -1;
  } else {
    h->bsb_tasks.release();
    h->bsb_r.release();
  }
  h->xbuf.release();  // allocated on first ptzba_exchange_packed
  if (zero_async(h, h->D_pose.p, h->D_pose.bytes) || zero_async(h, h->D_ray.p, h->D_ray.bytes) ||
      zero_async(h, h->w_slot[0].p, h->w_slot[0].bytes) ||  // slots of unobserved frames stay zero
      zero_async(h, h->w_slot[1].p, h->w_slot[1].bytes) ||
      zero_async(h, h->lm_out[0].p, h->lm_out[0].bytes) ||  // landmarks without records keep zero rows
      zero_async(h, h->lm_out[1].p, h->lm_out[1].bytes) || zero_async(h, h->ug_slot[0].p, h->ug_slot[0].bytes) ||
      zero_async(h, h->ug_slot[1].p, h->ug_slot[1].bytes) || zero_async(h, h->ptz.p, h->ptz.bytes) ||
      zero_async(h, h->rays.p, h->rays.bytes) || zero_async(h, h->scal.p, h->scal.bytes) ||
      zero_async(h, h->red_scratch.p, h->red_scratch.bytes))
    return -1;
  if (flush_stage(h)) return -1;
  h->stage_batch = false;
  st_mark("upload+alloc");
  if (!h->scal_host) HIPCHK(hipHostMalloc((void**)&h->scal_host, 24 * sizeof(double), hipHostMallocDefault));
  if (!h->scal_pack.p && h->scal_pack.alloc(24 * sizeof(double))) return -1;
  h->cur = 0;
  h->lambda = 0;
  HIPCHK(hipStreamSynchronize(h->st));  // every initialisation above has landed before the handle is used
  st_mark("final sync");
  h->have_problem = true;
  h->drop_groups();  // the groups of the previous problem; split anew at the first exchange of this one
  // no collective here: a rank whose set_problem failed validation above must not leave the others blocked in a
  // split.  The group communicator is split by the first exchange (ensure_group_comm), which every rank reaches.
  return 0;
}

int ptzba_problem_info(ptzba_handle h, int64_t* info) {
  if (!h || !h->have_problem) return fail("no problem set");
  info[0] = h->n_pose;
  info[1] = h->n_lm;
  info[2] = h->n_rec;
  info[3] = h->n_seg;
  info[4] = h->n_sys;
  info[5] = h->n_work;
  info[6] = h->max_seg_per_lm;
  info[7] = (int64_t)g_total_bytes({&h->rec_xy, &h->rec_seg, &h->rec_w, &h->perm, &h->seg_frame, &h->seg_lm,
                                    &h->seg_base, &h->ft64, &h->rt64,
                                    &h->seg_rec_begin, &h->lm_seg_begin, &h->lm_order, &h->frame_seg_begin,
                                    &h->frame_seg_list, &h->frame_win_hi, &h->ptz, &h->rays, &h->ptz_trial,
                                    &h->rays_trial, &h->D_pose, &h->D_ray, &h->ft, &h->rt, &h->ug_slot[0],
                                    &h->ug_slot[1], &h->w_slot[0], &h->w_slot[1], &h->lm_out[0], &h->lm_out[1], &h->lm_aux, &h->lm_red, &h->sys,
                                    &h->scal});
  return 0;
}

// ------------------------------------------------------------------------------------------------
static void* ft_real(ptzba_ctx* h) { return h->precision == PTZBA_FP32 ? h->ft.p : h->ft64.p; }
static void* rt_real(ptzba_ctx* h) { return h->precision == PTZBA_FP32 ? h->rt.p : h->rt64.p; }

static void tables(ptzba_ctx* h, const double* ptz, const double* rays, const int* run_if = nullptr,
                   double* zero = nullptr, int n_zero = 0) {
  if (h->precision == PTZBA_FP32)
    launch_tables<float>(ptz, rays, h->n_pose, h->n_lm, h->ft64.p, h->rt64.p, h->ft.p, h->rt.p, run_if, h->st, zero,
                         n_zero);
  else
    launch_tables<double>(ptz, rays, h->n_pose, h->n_lm, h->ft64.p, h->rt64.p, h->ft64.p, h->rt64.p, run_if, h->st, zero,
                          n_zero);
}

// sel != nullptr (device-driven LM): the kernel writes slot (*sel ^ sel_xor), chosen on the device
// run_if != nullptr: a conditional re-linearisation of the current point (device-driven LM, after the curvature
// switch): the launch exits at once unless *run_if; not timed as a K1 launch (the roofline averages real ones)
// hc_dev: device-driven LM, the huber curvature weight from device memory (LMDev::hc / hc_trial); nullptr: h->hcurv
static void linearize_into(ptzba_ctx* h, int slot, const int* sel = nullptr, int sel_xor = 0,
                           const int* run_if = nullptr, const double* hc_dev = nullptr) {
  LinArgs a;
  a.lm_work = h->lm_order.as<int4>();
  a.n_work = h->n_work;
  a.lm_seg_begin = h->lm_seg_begin.as<int32_t>();
  a.seg_frame = h->seg_frame.as<int32_t>();
  a.seg_rec_begin = h->seg_rec_begin.as<int64_t>();
  a.rec_seg = h->rec_seg.as<int32_t>();
  a.rec_key = h->rec_key.as<uint8_t>();
  a.rec_xy = h->rec_xy.p;
  a.rec_w = h->weighted ? h->rec_w.p : nullptr;
  a.ft = ft_real(h);
  a.rt = rt_real(h);
  a.ft64 = h->ft64.p;
  a.rt64 = h->rt64.p;
  a.seg_base = h->seg_base.as<double2>();
  a.u = h->u;
  a.v = h->v;
  a.fs2 = h->fs * h->fs;
  a.inv_fs2 = 1.0 / (h->fs * h->fs);
  a.hcurv = h->hcurv;
  a.hcurv_dev = hc_dev;
  a.run_if = run_if;
  a.ug_slot = h->ug_slot[slot].p;
  a.w_slot = h->w_slot[slot].p;
  a.lm_meta = h->lm_meta.as<int4>();
  a.lm_out = h->lm_out[slot].as<double>();
  a.sel = sel;
  a.sel_xor = sel_xor;
  if (sel) {
    a.ug_slot = h->ug_slot[0].p;
    a.w_slot = h->w_slot[0].p;
    a.lm_out = h->lm_out[0].as<double>();
  }
  a.ug_slot1 = h->ug_slot[1].p;
  a.w_slot1 = h->w_slot[1].p;
  a.lm_out1 = h->lm_out[1].as<double>();
  a.n_pose = h->n_pose;
  if (!run_if) tm_begin(h, TM_K1);
  hipEvent_t e0 = run_if ? nullptr : tm_k1_event(h, 0), e1 = run_if ? nullptr : tm_k1_event(h, 1);
  if (h->precision == PTZBA_FP32)
    launch_linearize<float>(a, h->loss, h->st, e0, e1);
  else
    launch_linearize<double>(a, h->loss, h->st, e0, e1);
  if (!run_if) tm_end(h, TM_K1);
}

int ptzba_solver_info(ptzba_handle h, int64_t* info8) {
  if (!h || !h->have_problem) return fail("no problem set");
  info8[0] = h->n_aug;
  info8[1] = h->ld;
  info8[2] = h->chol_levels;
  info8[3] = (h->nested ? PTZBA_ORDER_NESTED : PTZBA_ORDER_NATURAL) | ((int64_t)h->nd_depth << 8);
  info8[4] = h->bs_blk ? 2 : (h->bs_ll ? 1 : 0);
  info8[5] = h->n_slot;
  info8[6] = h->n_s2_items;
  info8[7] = h->n_ztiles;
  return 0;
}

int ptzba_residual(ptzba_handle h, const double* x_full, double* r_out) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  if (!h->perm_uploaded) {
    if (upload(h->perm, h->perm_host, h->st)) return -1;
    h->perm_uploaded = true;
  }
  DBuf x, r;
  if (x.alloc((3 * (size_t)h->n_pose + 2 * (size_t)h->n_lm) * 8) || r.alloc(2 * (size_t)h->n_rec * 8)) return -1;
  SyncOnExit sync_guard{h->st};  // destroyed before x and r: queued work on them ends first, also on errors
  HIPCHK(hipMemcpyAsync(x.p, x_full, x.bytes, hipMemcpyHostToDevice, h->st));
  const double* px = x.as<double>();
  tables(h, px, px + 3 * h->n_pose);
  if (h->precision == PTZBA_FP32)
    launch_residual<float>(h->rec_seg.as<int32_t>(), h->seg_frame.as<int32_t>(), h->seg_lm.as<int32_t>(),
                           h->seg_base.as<double2>(), h->rec_xy.p, h->perm.as<int64_t>(), h->ft64.p, h->rt64.p, h->u,
                           h->v, h->n_rec, r.as<double>(), h->st);
  else
    launch_residual<double>(h->rec_seg.as<int32_t>(), h->seg_frame.as<int32_t>(), h->seg_lm.as<int32_t>(),
                            h->seg_base.as<double2>(), h->rec_xy.p, h->perm.as<int64_t>(), h->ft64.p, h->rt64.p, h->u,
                            h->v, h->n_rec, r.as<double>(), h->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(r_out, r.p, 2 * (size_t)h->n_rec * 8, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

int ptzba_set_state(ptzba_handle h, const double* ptz, const double* rays) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  SyncOnExit sync_guard{h->st};  // caller buffers: no copy outlives the call, also on errors
  HIPCHK(hipMemcpyAsync(h->ptz.p, ptz, 3 * (size_t)h->n_pose * 8, hipMemcpyHostToDevice, h->st));
  if (h->n_lm) HIPCHK(hipMemcpyAsync(h->rays.p, rays, 2 * (size_t)h->n_lm * 8, hipMemcpyHostToDevice, h->st));
  HIPCHK(hipMemsetAsync(h->D_pose.p, 0, h->D_pose.bytes, h->st));
  HIPCHK(hipMemsetAsync(h->D_ray.p, 0, h->D_ray.bytes, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

// device-resident restart point: snapshot the current state / restore it (stream-ordered, no host sync)
int ptzba_save_state(ptzba_handle h) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  if (h->ptz_saved.alloc(h->ptz.bytes) || h->rays_saved.alloc(std::max<size_t>(h->rays.bytes, 8))) return -1;
  HIPCHK(hipMemcpyAsync(h->ptz_saved.p, h->ptz.p, 3 * (size_t)h->n_pose * 8, hipMemcpyDeviceToDevice, h->st));
  if (h->n_lm)
    HIPCHK(hipMemcpyAsync(h->rays_saved.p, h->rays.p, 2 * (size_t)h->n_lm * 8, hipMemcpyDeviceToDevice, h->st));
  return 0;
}

int ptzba_restore_state(ptzba_handle h) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!h->ptz_saved.p) return fail("no saved state (ptzba_save_state)");
  HIPCHK(hipSetDevice(h->device));
  // one launch instead of two copies and two fills (four stream operations at ~4-5 us each)
  const int64_t n_ptz = 3 * (int64_t)h->n_pose, n_rays = 2 * (int64_t)h->n_lm;
  const int64_t n_dp = (int64_t)(h->D_pose.bytes / 8), n_dr = (int64_t)(h->D_ray.bytes / 8);
  const int64_t n = std::max(std::max(n_ptz, n_rays), std::max(n_dp, n_dr));
  if (n > 0)
    hipLaunchKernelGGL(k_restore_state, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, h->st, h->ptz.as<double>(),
                       h->ptz_saved.as<double>(), n_ptz, h->rays.as<double>(), h->rays_saved.as<double>(), n_rays,
                       h->D_pose.as<double>(), n_dp, h->D_ray.as<double>(), n_dr);
  HIPCHK(hipGetLastError());
  return 0;
}

int ptzba_get_state(ptzba_handle h, double* ptz, double* rays) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  SyncOnExit sync_guard{h->st};  // no copy outlives the call, also on errors
  // through a pinned landing buffer kept by the handle: a pageable destination sent the copy down the runtime's
  // pageable path, whose cost jumped at some sizes (a 30-KF stream's keyframe call: 0.4 -> 6 ms once)
  const size_t nb_ptz = ptz ? 3 * (size_t)h->n_pose * 8 : 0, nb_rays = (rays && h->n_lm) ? 2 * (size_t)h->n_lm * 8 : 0;
  if (nb_ptz + nb_rays == 0) return 0;
  if (h->out_pin_cap < nb_ptz + nb_rays) {
    if (h->out_pin) {
      HIPCHK(hipStreamSynchronize(h->st));
      HIPCHK(hipHostFree(h->out_pin));
      h->out_pin = nullptr;
      h->out_pin_cap = 0;
    }
    const size_t cap = (nb_ptz + nb_rays) + (nb_ptz + nb_rays) / 2 + 4096;
    HIPCHK(hipHostMalloc((void**)&h->out_pin, cap, hipHostMallocDefault));
    h->out_pin_cap = cap;
  }
  if (nb_ptz) HIPCHK(hipMemcpyAsync(h->out_pin, h->ptz.p, nb_ptz, hipMemcpyDeviceToHost, h->st));
  if (nb_rays) HIPCHK(hipMemcpyAsync(h->out_pin + nb_ptz, h->rays.p, nb_rays, hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  if (nb_ptz) std::memcpy(ptz, h->out_pin, nb_ptz);
  if (nb_rays) std::memcpy(rays, h->out_pin + nb_ptz, nb_rays);
  return 0;
}

// ------------------------------------------------------------------------------------------------
// exchanges of a multi-GPU solve (include/ptzba.h PTZBA_X_*): in-place sums on the handle's stream through
// the attached RCCL communicator or the caller's hook
// ------------------------------------------------------------------------------------------------
static int ensure_group_comms(ptzba_ctx* h);
// the tree depth of the group an exchange kind runs over on this rank (0: the whole world)
static int exchange_depth(const ptzba_ctx* h, int kind) {
  if (!h->dist_mode || kind == PTZBA_X_SEP || kind == PTZBA_X_SCAL || kind == PTZBA_X_SYS) return 0;
  for (int q = 0; q < h->n_phase; ++q)
    if (h->ph[q].kind == kind) return h->ph[q].depth;
  return -1;
}
static int exchange_run(ptzba_ctx* h, int kind, double* buf, int64_t n);
// every exchange goes through here: with collective timing on (PTZBA_TIME_COMM) an event pair brackets it on the
// handle's stream (RCCL's kernel, or a hook's stream work), so a multi-rank run reports its collectives' time and
// bytes per kind (ptzba_comm_times) -- alpha and bandwidth measured instead of assumed
static int exchange(ptzba_ctx* h, int kind, double* buf, int64_t n) {
  const bool tm = (h->timing & PTZBA_TIME_COMM) && h->cev_used + 2 <= (int)h->cev.size();
  if (tm) (void)hipEventRecord(h->cev[h->cev_used], h->st);
  const int rc = exchange_run(h, kind, buf, n);
  if (tm) {
    (void)hipEventRecord(h->cev[h->cev_used + 1], h->st);
    h->cev_used += 2;
    h->clog.emplace_back(kind, n);
  }
  return rc;
}
static int exchange_run(ptzba_ctx* h, int kind, double* buf, int64_t n) {
  if (h->hook) {
    if (h->hook(h->hook_ctx, kind, buf, n, (void*)h->st)) return fail("exchange hook failed (kind %d)", kind);
    return 0;
  }
  if (h->comm) {
    // ncclCommSplit is collective over comm: done before this rank's first exchange of the problem, where every
    // rank of a sharded solve arrives in the same order
    if (ensure_group_comms(h)) return fail("group communicator split failed");
    const int d = exchange_depth(h, kind);
    if (d < 0 || d >= 4) return fail("no rank group for exchange kind %d", kind);
    ptzba_comm c = d == 0 ? h->comm : h->group_comms[d];
    if (!c) return fail("part-owned exchange kind %d has no group communicator (ptzba_attach_comm)", kind);
    return ptzba_comm_allreduce(c, buf, n, (void*)h->st);
  }
  return 0;
}
static int64_t scal_count(const ptzba_ctx* h) { return h->dist_mode ? 2 * PTZBA_NSCALARS : PTZBA_NSCALARS; }

// the rank tree's group communicators, one split per tree depth 1..depth (collective over ALL ranks of comm, in the
// same order everywhere: a rank whose path does not reach that depth, or whose node there holds it alone, joins a
// one-rank communicator it never uses)
static int ensure_group_comms(ptzba_ctx* h) {
  if (!h->comm || !h->have_problem || !h->dist_mode || h->groups_split) return 0;
  for (int d = 1; d <= h->tree_depth && d < 4; ++d) {
    int color = 1 << 20 | h->dist_rank;
    for (int q = 0; q < h->n_phase; ++q)
      if (h->ph[q].depth == d && h->ph[q].nr >= 2) color = h->ph[q].node;
    h->group_comms[d] = ptzba_comm_split(h->comm, color, h->dist_rank);
    if (!h->group_comms[d]) return -1;
  }
  h->groups_split = true;
  return 0;
}

int ptzba_linearize(ptzba_handle h) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  // the scalar block is zeroed by the tables launch (one launch less than a memset)
  tables(h, h->ptz.as<double>(), h->rays.as<double>(), nullptr, h->scal.as<double>(), (int)(h->scal.bytes / 8));
  linearize_into(h, h->cur);
  launch_reduce_cols(h->lm_out[h->cur].as<double>() + 5, h->n_lm, 8, 1, 0, h->scal.as<double>(),
                     h->red_scratch.as<double>(), h->st);
  HIPCHK(hipGetLastError());
  if (h->has_exchange()) return exchange(h, PTZBA_X_SCAL, h->scal.as<double>(), scal_count(h));
  return 0;
}

// reduced camera system at the current linearisation (slot h->cur, or in the device-driven LM slot *sel);
// lambda from the argument or, in the device-driven LM (lam_dev != nullptr), from device memory
static int build_impl(ptzba_ctx* h, double lambda, const double* lam_dev, const int* skip_if = nullptr,
                      const int* sel = nullptr) {
  const int c = sel ? 0 : h->cur;
  FusedPrep fp{};
  // fused only in the device-driven LM (sel != nullptr): the host-step API (ptzba_build_reduced) leaves the
  // system raw for callers that sum it between build and solve (include/ptzba.h, the round-2 protocol)
  if (sel && h->fused_prep())
    fp = FusedPrep{h->row_pad.as<uint8_t>(), h->n_aug, h->info.as<int>(), h->D_pose.as<double>(), lambda, lam_dev};
  launch_build_prologue(h->S(), h->ld, h->ztiles.as<int2>(), h->n_ztiles, h->bvec(), 3 * h->ld,
                        h->lm_out[c].as<double>(), h->lm_seg_begin.as<int32_t>(), h->D_ray.as<double>(),
                        h->lm_aux.as<double>(), h->n_lm, lambda, lam_dev, skip_if, h->st, h->lm_out[1].as<double>(),
                        sel, fp);
  SchurArgs a;
  a.items = h->s2_items.as<int4>();
  a.groups = h->s2_groups.as<int4>();
  a.part = h->s2_part.as<double>();
  a.part_diag = h->part_diag.as<double>();
  a.item_lm = h->s2_lm.as<int4>();
  a.frame_win_hi = h->frame_win_hi.as<int32_t>();
  a.ug_slot = h->ug_slot[c].p;
  a.w_slot = h->w_slot[c].p;
  a.lm_aux = h->lm_aux.as<double>();
  a.frame_pos = h->frame_pos.as<int32_t>();
  a.S = h->S();
  a.b = h->bvec();
  a.g_pose = h->gpose();
  a.dU = h->dU();
  a.ld = h->ld;
  a.n_pose = h->n_pose;
  a.skip_if = skip_if;
  a.ug_slot1 = h->ug_slot[1].p;
  a.w_slot1 = h->w_slot[1].p;
  a.sel = sel;
  a.prep = fp;
  tm_begin(h, TM_SCHUR);
  if (h->precision == PTZBA_FP32)
    launch_schur<float>(a, h->n_s2_items, h->n_s2_groups, h->n_fixed, h->st);
  else
    launch_schur<double>(a, h->n_s2_items, h->n_s2_groups, h->n_fixed, h->st);
  tm_end(h, TM_SCHUR);
  HIPCHK(hipGetLastError());
  if (h->dist_mode) {
    if (!h->has_exchange()) return fail("a part-owned handle needs an exchange (ptzba_attach_comm / ptzba_set_exchange_hook)");
    const auto& p0 = h->ph[0];
    if (p0.nr > 1) {  // a shared leaf: its columns (and b | g | dU over its rows) summed inside the leaf's group
      launch_pack_region(h->S(), h->ld, h->ph_tiles[0].as<int2>(), p0.n_tiles, h->bvec(), p0.vr, h->ph_buf[0].as<double>(), 0, h->st);
      if (exchange(h, PTZBA_X_PART, h->ph_buf[0].as<double>(), p0.n_buf)) return -1;
      launch_pack_region(h->S(), h->ld, h->ph_tiles[0].as<int2>(), p0.n_tiles, h->bvec(), p0.vr, h->ph_buf[0].as<double>(), 1, h->st);
      HIPCHK(hipGetLastError());
    }
  } else if (h->has_exchange()) {  // replicated: the packed reduced system summed over all ranks
    if (ptzba_exchange_packed(h, nullptr, nullptr)) return -1;
    const int64_t n = (int64_t)h->n_xtiles * CHOL_NB * CHOL_NB + 3 * h->ld;
    launch_pack_exchange(h->S(), h->ld, h->xtiles.as<int2>(), h->n_xtiles, h->bvec(), h->xbuf.as<double>(), 0, h->st);
    if (exchange(h, PTZBA_X_SYS, h->xbuf.as<double>(), n)) return -1;
    launch_pack_exchange(h->S(), h->ld, h->xtiles.as<int2>(), h->n_xtiles, h->bvec(), h->xbuf.as<double>(), 1, h->st);
    HIPCHK(hipGetLastError());
  }
  return 0;
}

int ptzba_build_reduced(ptzba_handle h, double lambda) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!(lambda >= 0) || !std::isfinite(lambda)) return fail("bad lambda");
  HIPCHK(hipSetDevice(h->device));
  h->lambda = lambda;
  return build_impl(h, lambda, nullptr);
}

// damped solve, trial state, trial linearisation into slot `nx` and the trial scalars (device-driven LM:
// current slot *sel, trial slot *sel ^ 1, chosen on the device)
static int solve_impl(ptzba_ctx* h, const double* lam_dev, int nx, const int* sel = nullptr) {
  const int c = sel ? 0 : h->cur;
  if (sel) nx = 1;  // the trial's slot, with the other slot as the selector's alternative
  tm_begin(h, TM_CHOL);
  const int4* th = reinterpret_cast<const int4*>(h->chol_tasks_host.data());
  if (h->dist_mode) {
    // the rank's phases (make_plan_tree): before each later phase its columns are summed over its node's group
    for (int q = 0; q < h->n_phase; ++q) {
      const auto& d = h->ph[q];
      if (q > 0) {
        launch_pack_region(h->S(), h->ld, h->ph_tiles[q].as<int2>(), d.n_tiles, h->bvec(), d.vr, h->ph_buf[q].as<double>(), 0, h->st);
        HIPCHK(hipGetLastError());
        if (exchange(h, d.kind, h->ph_buf[q].as<double>(), d.n_buf)) return -1;
        launch_pack_region(h->S(), h->ld, h->ph_tiles[q].as<int2>(), d.n_tiles, h->bvec(), d.vr, h->ph_buf[q].as<double>(), 1, h->st);
      }
      launch_chol_prepare_damped(h->S(), h->ld, h->n_aug, h->bvec(), h->row_pad.as<uint8_t>(), h->info.as<int>(),
                                 h->dU(), h->D_pose.as<double>(), h->frame_pos.as<int32_t>(), h->n_pose, h->n_fixed,
                                 h->lambda, lam_dev, h->st, h->row_phase.as<uint8_t>(), q + 1);
      launch_cholesky(h->S(), h->ld, h->chol_tasks.as<int4>(), h->chol_task_off.data(), d.lv1, h->Ldiag.as<double>(),
                      h->info.as<int>(), h->st, nullptr, th, h->Minv.as<double>(), d.lv0, h->chol_delayed);
      HIPCHK(hipGetLastError());
    }
  } else {
    if (!(sel && h->fused_prep()))  // device-driven single-GPU builds wrote the augmented row, padding, damping
      launch_chol_prepare_damped(h->S(), h->ld, h->n_aug, h->bvec(), h->row_pad.as<uint8_t>(), h->info.as<int>(),
                                 h->dU(), h->D_pose.as<double>(), h->frame_pos.as<int32_t>(), h->n_pose, h->n_fixed,
                                 h->lambda, lam_dev, h->st);
    launch_cholesky(h->S(), h->ld, h->chol_tasks.as<int4>(), h->chol_task_off.data(), h->chol_levels,
                      h->Ldiag.as<double>(), h->info.as<int>(), h->st, nullptr, th, h->Minv.as<double>(), 0,
                      h->chol_delayed);
  }
  if (h->bs_pst)
    launch_chol_backsolve_pst(h->S(), h->ld, h->n_aug, h->bsb_tasks.as<int4>(), h->bsp_expect.as<int4>(),
                              h->bsb_step_off.back(), h->Ldiag.as<double>(), h->Minv.as<double>(), h->bsb_r.as<double>(),
                              h->dpose.as<double>(), h->bsp_cnt.as<unsigned>(), h->bsp_tot.as<int>(), h->bsp_epoch++,
                              h->bsp_err, h->st, h->tinv_tail.as<int>(), h->n_tinv_tail);
  else if (h->bs_blk)
    launch_chol_backsolve_blk(h->S(), h->ld, h->n_aug, h->bsb_tasks.as<int4>(), h->bsb_step_off.data(), (int)h->bsb_step_off.size() - 1, h->Ldiag.as<double>(),
                              h->Minv.as<double>(), h->bsb_r.as<double>(), h->dpose.as<double>(), h->st,
                              h->tinv_tail.as<int>(), h->n_tinv_tail);
  else
    launch_chol_backsolve(h->S(), h->ld, h->n_aug, h->n_chain, h->bs_npos, h->bs_chain_off.as<int>(),
                          h->bs_chain_cols.as<int>(), h->bs_upd_off.as<int>(), h->bs_upd_tiles.as<int>(), h->bs_nupd,
                          h->bs_la_tasks.as<int>(), h->bs_ntasks,
                          h->Ldiag.as<double>(), h->Minv.as<double>(), h->dpose.as<double>(),
                          h->bs_ll ? h->bs_lo_off.as<int>() : nullptr, h->bs_lo_tiles.as<int>(), h->st,
                          h->tinv_tail.as<int>(), h->n_tinv_tail);
  tm_end(h, TM_CHOL);
  HIPCHK(hipGetLastError());
  tm_begin(h, TM_BACK);
  BacksubArgs b;
  b.lm_seg_begin = h->lm_seg_begin.as<int32_t>();
  b.seg_frame = h->seg_frame.as<int32_t>();
  b.w_slot = h->w_slot[c].p;
  b.lm_meta = h->lm_meta.as<int4>();
  b.lm_out = h->lm_out[c].as<double>();
  b.lm_aux = h->lm_aux.as<double>();
  b.D_ray = h->D_ray.as<double>();
  b.dpose = h->dpose.as<double>();
  b.frame_pos = h->frame_pos.as<int32_t>();
  b.rays = h->rays.as<double>();
  b.rays_trial = h->rays_trial.as<double>();
  b.lm_red = h->lm_red.as<double>();
  b.n_lm = h->n_lm;
  b.n_fixed = h->n_fixed;
  b.lambda = h->lambda;
  b.lam_dev = lam_dev;
  b.w_slot1 = h->w_slot[1].p;
  b.lm_out1 = h->lm_out[1].as<double>();
  b.sel = sel;
  b.state_xor = h->state_base;
  // ray back-substitution, trial poses and the trial's frame / ray tables: one launch
  const uint8_t* fm = h->dist_mode ? h->fmask.as<uint8_t>() : nullptr;
  const int* finfo = h->dist_mode ? h->info.as<int>() : nullptr;
  if (h->precision == PTZBA_FP32)
    launch_trial<float>(b, h->ptz.as<double>(), h->gpose(), h->D_pose.as<double>(), h->ptz_trial.as<double>(),
                        h->locp(), h->n_pose, h->ft64.p, h->rt64.p, h->ft.p, h->rt.p, h->st, fm, finfo);
  else
    launch_trial<double>(b, h->ptz.as<double>(), h->gpose(), h->D_pose.as<double>(), h->ptz_trial.as<double>(),
                         h->locp(), h->n_pose, h->ft64.p, h->rt64.p, h->ft64.p, h->rt64.p, h->st, fm, finfo);
  tm_end(h, TM_BACK);
  // trial linearisation (its cost decides acceptance; kept as the next linearisation if accepted).  Device-driven LM
  // with the huber curvature switch pending: single GPU (relin_mode 0), the trial's predicted reduction is reduced
  // first and picks the curvature of this linearisation (LMDev::hc_trial); ranks (relin_mode 1) use LMDev::hc
  const double* hc_dev = nullptr;
  if (sel) {
    LMDev* st = h->lmdev.as<LMDev>();
    hc_dev = h->lm_relin_mode ? &st->hc : &st->hc_trial;
    if (!h->lm_relin_mode && h->lm_curv_pending) {
      const DecideArgs cd{st, h->locp(), nullptr, nullptr, 0, 1};
      launch_reduce_cols(h->lm_red.as<double>(), h->n_lm, 4, 1, 0, h->curv_pred.as<double>(), h->red_scratch.as<double>(),
                         h->st, nullptr, 0, 0, nullptr, nullptr, nullptr, 0, &cd);
    }
  }
  linearize_into(h, nx, sel, 1, nullptr, hc_dev);
  // scal[1] (trial cost) and scal[2..4] are overwritten below, loc[0..3] by the trial kernel: no memsets
  if (sel && !h->has_exchange() && !h->ext_exchange && !h->scal_exported && !h->dist_mode) {
    // launched by ptzba_lm_decide with the decision fused into it (nothing runs between the two calls)
    h->scal_deferred = true;
    return 0;
  }
  launch_reduce_cols(h->lm_out[sel ? 0 : nx].as<double>() + 5, h->n_lm, 8, 1, 0, h->scal.as<double>() + 1,
                     h->red_scratch.as<double>(), h->st, h->lm_red.as<double>(), 4, 3, h->scal.as<double>() + 2,
                     h->lm_out[1].as<double>() + 5, sel, 1);
  HIPCHK(hipGetLastError());
  // partial scalars (replicated: the landmark sums; part-owned: also the pose partials, each frame counted
  // by one rank -- the gradient max then sums the ranks' maxima, an upper bound: gtol can only stop later)
  if (h->has_exchange()) return exchange(h, PTZBA_X_SCAL, h->scal.as<double>(), scal_count(h));
  return 0;
}

int ptzba_solve_reduced(ptzba_handle h) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  return solve_impl(h, nullptr, 1 - h->cur);
}

// ------------------------------------------------------------------------------------------------
// device-driven Levenberg-Marquardt (the decisions of ptzba.LMSolver on the device): the host only
// enqueues trials and polls a pinned record ring, so no trial waits for a host round trip.  The two
// linearisation slots are selected on the device (LMDev::cur): a trial linearises into the other slot, an
// accepted trial flips cur, a rejected one leaves the current linearisation in place (no re-linearisation).
// ------------------------------------------------------------------------------------------------
static int lm_check(ptzba_ctx* h) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!h->lmdev.p) return fail("call ptzba_lm_start first");
  return 0;
}

int ptzba_lm_start(ptzba_handle h) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  if (!h->lmdev.p && h->lmdev.alloc(sizeof(LMDev))) return -1;
  if (!h->curv_pred.p && h->curv_pred.alloc(64)) return -1;
  h->hcurv = 1.0;  // the initial linearisation: IRLS (the host-driven LM's setting does not carry over)
  if (!h->lm_host) {
    HIPCHK(hipHostMalloc((void**)&h->lm_host, LM_RING * sizeof(LMDev), hipHostMallocCoherent));
  }
  h->cur = 0;
  return ptzba_linearize(h);
}

int ptzba_lm_init(ptzba_handle h, const ptzba_lm_opts* o) {
  if (lm_check(h)) return -1;
  if (!o) return fail("null options");
  if (!(o->lambda0 >= 0) || !(o->min_lambda > 0) || !(o->max_lambda > 0) || o->max_iter < 0 || o->max_retries < 1)
    return fail("bad LM options");
  HIPCHK(hipSetDevice(h->device));
  // the two curvature fields (added in version 5 of the options struct) matter for the Huber loss only; a caller that
  // zero-fills them gets the default curvature (0.1) and no switch (curvature_switch 0)
  const double hcv = o->huber_curvature == 0.0 ? 0.1 : o->huber_curvature;
  if (h->loss == PTZBA_LOSS_HUBER && (!(hcv > 0.0 && hcv <= 1.0) || !(o->curvature_switch >= 0.0)))
    return fail("bad LM options (huber_curvature in (0, 1], curvature_switch >= 0)");
  const bool sw = h->loss == PTZBA_LOSS_HUBER && o->curvature_switch > 0.0 && hcv < 1.0;
  LMParams p{o->ftol, o->xtol, o->gtol, o->lambda0, o->min_lambda, o->max_lambda,
             sw ? hcv : 1.0, sw ? o->curvature_switch : 0.0, o->max_iter, o->max_retries,
             o->gauss_newton ? 1 : 0, 0};
  // the switch's launches (relin_mode 1: the conditional re-linearisation in lm_build; 0: the predicted-reduction
  // reduce in front of the trial K1) are queued until the host sees the switch in a decision record
  h->lm_curv_pending = sw;
  h->lm_relin_mode = h->has_exchange() || h->ext_exchange || h->scal_exported || h->dist_mode;
  p.relin_mode = h->lm_relin_mode ? 1 : 0;
  // no decision of an earlier run is in flight (its lm_wait returned): clear the ring's sequence tags
  for (int k = 0; k < LM_RING; ++k) __atomic_store_n(&h->lm_host[k].seq, 0, __ATOMIC_RELAXED);
  launch_lm_init(h->lmdev.as<LMDev>(), h->scal.as<double>(), p, h->cur, h->st);
  h->state_base = h->cur;  // (ptz, rays) hold the current state now
  if (h->bsp_err) *h->bsp_err = 0;  // a run starts without an earlier run's gave-up flag (nothing of it is in flight)
  h->scal_deferred = false;
  HIPCHK(hipGetLastError());
  return 0;
}

int ptzba_lm_build(ptzba_handle h) {
  if (lm_check(h)) return -1;
  HIPCHK(hipSetDevice(h->device));
  // the curvature switch of the last decision (LMDev::relin): re-linearise the current point into its slot first.
  // Queued only until the host has seen the switch in a decision record; the launch reads the flag on the device
  if (h->lm_curv_pending && h->lm_relin_mode)
    linearize_into(h, 0, &h->lmdev.as<LMDev>()->cur, 0, &h->lmdev.as<LMDev>()->relin, &h->lmdev.as<LMDev>()->hc);
  // a build queued after the final decision (the host pipelines one trial ahead) exits at once
  return build_impl(h, 0.0, &h->lmdev.as<LMDev>()->lam, &h->lmdev.as<LMDev>()->done, &h->lmdev.as<LMDev>()->cur);
}

int ptzba_lm_solve(ptzba_handle h) {
  if (lm_check(h)) return -1;
  HIPCHK(hipSetDevice(h->device));
  return solve_impl(h, &h->lmdev.as<LMDev>()->lam, 1 - h->cur, &h->lmdev.as<LMDev>()->cur);
}

int ptzba_lm_decide(ptzba_handle h, int trial) {
  if (lm_check(h)) return -1;
  if (trial < 0) return fail("bad trial index");
  HIPCHK(hipSetDevice(h->device));
  LMDev* st = h->lmdev.as<LMDev>();
  const int k = trial % LM_RING;
  // the record is written by the decision straight into pinned host memory.  No commit copy: an accepted trial
  // flips LMDev::cur, which selects the state pair as it selects the linearisation slot (BacksubArgs::state_xor)
  if (h->scal_deferred) {
    // single GPU: the trial-cost reduction (deferred by lm_solve) with the decision in its last workgroup
    h->scal_deferred = false;
    const int* sel = &h->lmdev.as<LMDev>()->cur;
    const DecideArgs dec{st, h->locp(), h->info.as<int>(), h->lm_host + k, trial + 1};
    launch_reduce_cols(h->lm_out[0].as<double>() + 5, h->n_lm, 8, 1, 0, h->scal.as<double>() + 1,
                       h->red_scratch.as<double>(), h->st, h->lm_red.as<double>(), 4, 3, h->scal.as<double>() + 2,
                       h->lm_out[1].as<double>() + 5, sel, 1, &dec);
  } else {
    launch_lm_decide(st, h->scal.as<double>(), h->locp(), h->info.as<int>(), h->lm_host + k, trial + 1,
                     h->st, h->dist_mode);
  }
  HIPCHK(hipGetLastError());
  return 0;
}

int ptzba_lm_wait(ptzba_handle h, int trial, ptzba_lm_record* out) {
  if (lm_check(h)) return -1;
  if (trial < 0 || !out) return fail("bad arguments");
  HIPCHK(hipSetDevice(h->device));
  const int k = trial % LM_RING;
  // the decision kernel tags its record last; poll the tag (an event record per trial would add a
  // ~6 us gap to the stream).  Every 4096 polls check that the stream is still alive.
  for (int64_t n = 0; __atomic_load_n(&h->lm_host[k].seq, __ATOMIC_ACQUIRE) != trial + 1; ++n) {
    if ((n & 4095) == 4095) {
      const hipError_t q = hipStreamQuery(h->st);
      if (q != hipSuccess && q != hipErrorNotReady) return fail("lm_wait: stream error %s", hipGetErrorString(q));
      if (q == hipSuccess && __atomic_load_n(&h->lm_host[k].seq, __ATOMIC_ACQUIRE) != trial + 1)
        return fail("lm_wait: no decision record for trial %d (was ptzba_lm_decide called?)", trial);
    }
    __builtin_ia32_pause();
  }
  if (h->bs_pst && __atomic_load_n(h->bsp_err, __ATOMIC_ACQUIRE))
    return fail("lm_wait: a persistent factorisation / back-substitution kernel gave up waiting (workgroups not "
                "co-resident?); PTZBA_BS_PERSIST=0 selects the per-step form");
  const LMDev& r = h->lm_host[k];
  out->cost = r.cost;
  out->initial_cost = r.initial_cost;
  out->lambda = r.lam;
  out->iterations = r.it;
  out->nfev = r.nfev;
  out->trials = r.trials;
  out->retries = r.retries;
  out->status = r.status;
  out->done = r.done;
  out->accepted = r.accepted;
  if (r.hc != 1.0) h->lm_curv_pending = false;  // switched: the launches already queued behind it suffice
  h->cur = r.cur;  // the host's view of the current slot follows the device (ptzba_accept / linearize)
  if ((r.cur ^ h->state_base) & 1) {
    // the device's decisions moved the current state to the other pair: swap the pointers and the base together,
    // so that kernels already queued (old pair, old base) and later ones (new pair, new base) select the same buffer
    std::swap(h->ptz.p, h->ptz_trial.p);
    std::swap(h->ptz.bytes, h->ptz_trial.bytes);
    std::swap(h->ptz.cap, h->ptz_trial.cap);
    std::swap(h->rays.p, h->rays_trial.p);
    std::swap(h->rays.bytes, h->rays_trial.bytes);
    std::swap(h->rays.cap, h->rays_trial.cap);
    h->state_base ^= 1;
  }
  return 0;
}

// One-shot solve: the device-driven LM run to termination in C (the sequence ptzba.LMSolver drives from
// Python, single process).  Replaces the optimizer call least_squares(_compute_residual, x0, x_scale='jac',
// ftol=1e-4, method='trf') of bundle_adjustment.py:200-202 and the empty C stub bundle_adjustment_opt
// (rf_map/python_package/backup/bundle_adjustment_python.hpp:21-24): the state goes in and the optimum
// comes out through the caller's buffers (rf_map.cpp:77, 113-116 in/out convention).
// the device-driven LM from the handle's current device state to termination (shared by the one-shot entries)
static int lm_run(ptzba_ctx* h, const ptzba_lm_opts& o, ptzba_lm_record& rec) {
  if (ptzba_lm_start(h) || ptzba_lm_init(h, &o)) return -1;
  rec = ptzba_lm_record{};
  if (o.max_iter > 0) {
    const int64_t limit = (int64_t)o.max_iter * (o.max_retries + 1);
    if (ptzba_lm_build(h)) return -1;
    for (int k = 0;; ) {
      if (ptzba_lm_solve(h) || ptzba_lm_decide(h, k)) return -1;
      if (k + 1 < limit && ptzba_lm_build(h)) return -1;  // next trial queued behind this decision
      if (ptzba_lm_wait(h, k, &rec)) return -1;
      ++k;
      if (rec.done || k >= limit) break;
    }
  } else {
    double s[PTZBA_NSCALARS];
    if (ptzba_read_scalars(h, s)) return -1;
    rec.cost = rec.initial_cost = s[0];
    rec.nfev = 1;
  }
  return 0;
}
static const ptzba_lm_opts k_default_opts{1e-4, 1e-8, 0.0, 1e-12, 1e-12, 1e16, 100, 30, 0, 0.1, 0.25};

int ptzba_solve_resident(ptzba_handle h, int restore, const ptzba_lm_opts* opts, ptzba_report* report) {
  if (!h || !h->have_problem) return fail("no problem set");
  const ptzba_lm_opts o = opts ? *opts : k_default_opts;
  const auto t0 = std::chrono::steady_clock::now();
  if (restore && ptzba_restore_state(h)) return -1;
  ptzba_lm_record rec{};
  if (lm_run(h, o, rec)) return -1;
  if (report) {
    report->cost = rec.cost;
    report->initial_cost = rec.initial_cost;
    report->time_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    report->iterations = rec.iterations;
    report->nfev = rec.nfev;
    report->trials = rec.trials;
    report->status = rec.status;
  }
  return 0;
}

int ptzba_solve(ptzba_handle h, double* ptz_inout, double* rays_inout, const ptzba_lm_opts* opts,
                ptzba_report* report) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!ptz_inout || (h->n_lm > 0 && !rays_inout)) return fail("null state buffer");
  const ptzba_lm_opts o = opts ? *opts : k_default_opts;
  const auto t0 = std::chrono::steady_clock::now();
  if (ptzba_set_state(h, ptz_inout, rays_inout)) return -1;
  ptzba_lm_record rec{};
  if (lm_run(h, o, rec)) return -1;
  std::vector<double> ptz(3 * (size_t)h->n_pose), rays(2 * (size_t)h->n_lm);
  if (ptzba_get_state(h, ptz.data(), rays.data())) return -1;
  std::copy(ptz.begin(), ptz.end(), ptz_inout);
  if (h->n_lm) std::copy(rays.begin(), rays.end(), rays_inout);
  if (report) {
    report->cost = rec.cost;
    report->initial_cost = rec.initial_cost;
    report->time_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    report->iterations = rec.iterations;
    report->nfev = rec.nfev;
    report->trials = rec.trials;
    report->status = rec.status;
  }
  return 0;
}

int ptzba_step(ptzba_handle h, double lambda) {
  int rc = ptzba_build_reduced(h, lambda);
  if (rc) return rc;
  return ptzba_solve_reduced(h);
}

int ptzba_read_scalars(ptzba_handle h, double* out) {
  if (!h || !h->have_problem) return fail("no problem set");
  HIPCHK(hipSetDevice(h->device));
  // one kernel packs scal | loc | info, one copy brings the block to pinned host memory
  launch_pack_scalars(h->scal.as<double>(), h->locp(), h->info.as<int>(), h->scal_pack.as<double>(), h->st);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(h->scal_host, h->scal_pack.p, 17 * sizeof(double), hipMemcpyDeviceToHost, h->st));
  HIPCHK(hipStreamSynchronize(h->st));
  if (h->bs_pst && __atomic_load_n(h->bsp_err, __ATOMIC_ACQUIRE))
    return fail("the persistent back-substitution kernel gave up waiting (PTZBA_BS_PERSIST=0 selects the per-step form)");
  const double* s = h->scal_host;
  const double* l = h->scal_host + 8;
  out[0] = s[0];
  out[1] = s[1];
  out[2] = s[2] + l[0];
  out[3] = s[3] + l[1];
  out[4] = s[4] + l[2];
  out[5] = h->dist_mode ? l[4] : h->scal_host[16];  // part-owned: the status summed over ranks
  out[6] = l[3];
  out[7] = 0;
  return 0;
}

int ptzba_accept(ptzba_handle h, int accept) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (accept) {
    h->cur = 1 - h->cur;
    std::swap(h->ptz.p, h->ptz_trial.p);
    std::swap(h->ptz.bytes, h->ptz_trial.bytes);
    std::swap(h->ptz.cap, h->ptz_trial.cap);
    std::swap(h->rays.p, h->rays_trial.p);
    std::swap(h->rays.bytes, h->rays_trial.bytes);
    std::swap(h->rays.cap, h->rays_trial.cap);
  }
  return 0;
}

int ptzba_exchange(ptzba_handle h, void** sys_ptr, int64_t* sys_count, void** scal_ptr) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (sys_ptr) h->ext_exchange = true;  // the caller may sum the system between build and solve: prepare after it
  if (sys_ptr) *sys_ptr = h->sys.p;
  if (sys_count) *sys_count = h->sys_count();
  if (scal_ptr) {
    *scal_ptr = h->scal.p;
    h->scal_exported = true;  // the caller may sum the scalars between lm_solve and lm_decide: no fused decision
  }
  return 0;
}

int ptzba_exchange_packed(ptzba_handle h, void** buf, int64_t* count) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (buf && !h->has_exchange()) h->ext_exchange = true;  // the caller's own protocol (see ptzba_exchange)
  const int64_t n = (int64_t)h->n_xtiles * CHOL_NB * CHOL_NB + 3 * h->ld;
  if (!h->xbuf.p && h->xbuf.alloc((size_t)n * 8)) return -1;
  if (buf) *buf = h->xbuf.p;
  if (count) *count = n;
  return 0;
}

static int pack_impl(ptzba_handle h, int unpack) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!h->xbuf.p) return fail("call ptzba_exchange_packed first");
  HIPCHK(hipSetDevice(h->device));
  launch_pack_exchange(h->S(), h->ld, h->xtiles.as<int2>(), h->n_xtiles, h->bvec(), h->xbuf.as<double>(), unpack, h->st);
  HIPCHK(hipGetLastError());
  return 0;
}
int ptzba_pack(ptzba_handle h) { return pack_impl(h, 0); }
int ptzba_unpack(ptzba_handle h) { return pack_impl(h, 1); }

int ptzba_set_exchange_hook(ptzba_handle h, ptzba_exchange_fn fn, void* ctx) {
  if (!h) return fail("null handle");
  h->hook = fn;
  h->hook_ctx = ctx;
  return 0;
}

int ptzba_attach_comm(ptzba_handle h, ptzba_comm comm) {
  if (!h) return fail("null handle");
  h->drop_groups();
  h->comm = comm;
  return 0;  // the group communicator is split lazily by the first exchange (collective, every rank reaches it)
}

int ptzba_dist_info(ptzba_handle h, int64_t* info8) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!info8) return fail("null output");
  info8[0] = h->dist_mode;
  info8[1] = h->dist_mode ? h->base_node : -1;
  info8[2] = h->dist_mode ? h->ph[0].nr : 1;
  info8[3] = h->dist_mode ? (h->dist_rank == h->ph[0].r0) : 1;
  int64_t sep = 0, sub = 0;
  for (int q = 1; q < h->n_phase; ++q) (h->ph[q].kind == PTZBA_X_SEP ? sep : sub) += h->ph[q].n_buf;
  info8[4] = sep;
  info8[5] = h->dist_mode && h->ph[0].nr > 1 ? h->ph[0].n_buf : 0;
  info8[6] = h->dist_mode || h->dist_world < 2 ? 0 : (int64_t)h->n_xtiles * CHOL_NB * CHOL_NB + 3 * h->ld;
  info8[7] = scal_count(h);
  return 0;
}

int ptzba_dist_exchanges(ptzba_handle h, int64_t* out, int32_t cap, int32_t* n_out) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!n_out) return fail("null output");
  std::vector<int64_t> v;
  if (h->dist_mode) {
    if (h->ph[0].nr > 1) v.insert(v.end(), {PTZBA_X_PART, h->ph[0].r0, h->ph[0].nr, h->ph[0].n_buf});
    for (int q = 1; q < h->n_phase; ++q) v.insert(v.end(), {h->ph[q].kind, h->ph[q].r0, h->ph[q].nr, h->ph[q].n_buf});
    v.insert(v.end(), {PTZBA_X_SCAL, 0, h->dist_world, scal_count(h)});
  } else if (h->dist_world >= 2) {
    v.insert(v.end(), {PTZBA_X_SYS, 0, h->dist_world, (int64_t)h->n_xtiles * CHOL_NB * CHOL_NB + 3 * h->ld});
    v.insert(v.end(), {PTZBA_X_SCAL, 0, h->dist_world, scal_count(h)});
  }
  *n_out = (int32_t)(v.size() / 4);
  if (out) {
    if (cap < *n_out) return fail("output holds %d exchanges, %d needed", cap, *n_out);
    std::copy(v.begin(), v.end(), out);
  }
  return 0;
}
int ptzba_dist_groups(ptzba_handle h, int32_t* out, int32_t cap, int32_t* n_out) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!n_out) return fail("null output");
  *n_out = (int32_t)(h->tree_groups.size() / 3);
  if (out) {
    if (cap < *n_out) return fail("output holds %d groups, %d needed", cap, *n_out);
    std::copy(h->tree_groups.begin(), h->tree_groups.end(), out);
  }
  return 0;
}
int ptzba_exchange_group(ptzba_handle h, int32_t kind, int32_t* r0_nr) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!r0_nr) return fail("null output");
  r0_nr[0] = 0;
  r0_nr[1] = h->dist_world;
  if (h->dist_mode && kind != PTZBA_X_SEP && kind != PTZBA_X_SCAL) {
    for (int q = 0; q < h->n_phase; ++q)
      if (h->ph[q].kind == kind && (q > 0 || h->ph[0].nr > 1)) {
        r0_nr[0] = h->ph[q].r0;
        r0_nr[1] = h->ph[q].nr;
        return 0;
      }
    return fail("this rank runs no exchange of kind %d", kind);
  }
  return 0;
}
int ptzba_owned_frames(ptzba_handle h, uint8_t* mask_out) {
  if (!h || !h->have_problem) return fail("no problem set");
  if (!mask_out) return fail("null output");
  std::copy(h->owned_host.begin(), h->owned_host.end(), mask_out);
  return 0;
}

int ptzba_sync(ptzba_handle h) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  return 0;
}

int ptzba_reset_kernel_times(ptzba_handle h, int enable) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  for (int k = 0; k < TM_N; ++k) {
    if (((enable >> k) & 1) && h->ev[k].empty()) {
      h->ev[k].resize(TM_POOL);
      for (auto& e : h->ev[k]) HIPCHK(hipEventCreate(&e));
    }
    h->ev_used[k] = 0;
    h->tm_seen[k] = 0;
    h->tm_sampled[k] = false;
  }
  h->timing = enable & (((1 << TM_N) - 1) | PTZBA_TIME_COMM);
  if ((enable & PTZBA_TIME_COMM) && h->cev.empty()) {
    h->cev.resize(2 * COMM_POOL);
    for (auto& e : h->cev) HIPCHK(hipEventCreate(&e));
  }
  h->cev_used = 0;
  h->clog.clear();
  h->tm_stride = std::max(1, (enable >> 8) & 0xff);
  h->tm_flush = (enable & PTZBA_TIME_FLUSH) != 0;
  h->tm_flush_read = h->tm_flush && (enable & PTZBA_TIME_FLUSH_READ) != 0;
  if (h->tm_flush && !h->flush_buf.p) {
    if (h->flush_buf.alloc(FLUSH_BYTES)) return -1;
    k_flush_caches<<<4096, 256, 0, h->st>>>(h->flush_buf.as<float4>(), (int64_t)(FLUSH_BYTES / 16), 1.0f);
    HIPCHK(hipGetLastError());
  }
  if (!h->tm_flush) h->flush_buf.release();
  return 0;
}

int ptzba_kernel_times(ptzba_handle h, double* ms_out, int64_t* count_out) {
  if (!h) return fail("null handle");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  for (int k = 0; k < TM_N; ++k) {
    double tot = 0;
    int n = h->ev_used[k] / 2;
    for (int i = 0; i < n; ++i) {
      float ms = 0;
      HIPCHK(hipEventElapsedTime(&ms, h->ev[k][2 * i], h->ev[k][2 * i + 1]));
      tot += ms;
    }
    ms_out[k] = n ? tot / n : 0.0;
    count_out[k] = n;
  }
  return 0;
}

int ptzba_comm_times(ptzba_handle h, int32_t cap, int32_t* kinds, int64_t* doubles, double* ms, int32_t* n_out) {
  if (!h || !n_out || cap < 0 || (cap > 0 && (!kinds || !doubles || !ms))) return fail("ptzba_comm_times: bad arguments");
  HIPCHK(hipSetDevice(h->device));
  HIPCHK(hipStreamSynchronize(h->st));
  const int32_t n = (int32_t)h->clog.size();
  for (int32_t i = 0; i < std::min(n, cap); ++i) {
    float t = 0;
    HIPCHK(hipEventElapsedTime(&t, h->cev[2 * i], h->cev[2 * i + 1]));
    kinds[i] = h->clog[i].first;
    doubles[i] = h->clog[i].second;
    ms[i] = t;
  }
  *n_out = n;
  return 0;
}

// ------------------------------------------------------------------------------------------------
// camera model batch API
// ------------------------------------------------------------------------------------------------
struct Tmp {
  std::vector<DBuf*> bufs;
  ~Tmp() {
    for (auto* b : bufs) delete b;
  }
  double* in(const double* h, size_t n) {
    auto* b = new DBuf();
    bufs.push_back(b);
    if (b->alloc(n * 8)) return nullptr;
    if (hipMemcpy(b->p, h, n * 8, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
    return b->as<double>();
  }
  double* out(size_t n) {
    auto* b = new DBuf();
    bufs.push_back(b);
    if (b->alloc(n * 8)) return nullptr;
    return b->as<double>();
  }
};

#define NEED(p)                                   \
  do {                                            \
    if (!(p)) return fail("device allocation/copy failed"); \
  } while (0)

int ptz_ray_to_image(int device, int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                     const double* th, const double* ph, double* x_out, double* y_out) {
  if (n < 0) return fail("n < 0");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(device));
  Tmp t;
  double *df = t.in(f, n), *dcp = t.in(cp, n), *dct = t.in(ct, n), *dth = t.in(th, n), *dph = t.in(ph, n);
  double *dx = t.out(n), *dy = t.out(n);
  NEED(df && dcp && dct && dth && dph && dx && dy);
  launch_ray_to_image(n, u, v, df, dcp, dct, dth, dph, dx, dy, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(x_out, dx, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(y_out, dy, n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptz_image_to_ray(int device, int64_t n, double u, double v, const double* f, const double* cp, const double* ct,
                     const double* x, const double* y, double* th_out, double* ph_out) {
  if (n < 0) return fail("n < 0");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(device));
  Tmp t;
  double *df = t.in(f, n), *dcp = t.in(cp, n), *dct = t.in(ct, n), *dx = t.in(x, n), *dy = t.in(y, n);
  double *dth = t.out(n), *dph = t.out(n);
  NEED(df && dcp && dct && dx && dy && dth && dph);
  launch_image_to_ray(n, u, v, df, dcp, dct, dx, dy, dth, dph, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(th_out, dth, n * 8, hipMemcpyDeviceToHost));
  HIPCHK(hipMemcpy(ph_out, dph, n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptz_project_rays(int device, int64_t n, double u, double v, double f, double pan, double tilt, const double* d6,
                     const double* rays, double* xy_out) {
  if (n < 0) return fail("n < 0");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(device));
  Tmp t;
  double *dr = t.in(rays, 2 * n), *dxy = t.out(2 * n);
  NEED(dr && dxy);
  launch_project_rays(n, u, v, f, pan, tilt, d6, dr, dxy, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(xy_out, dxy, 2 * n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptz_back_project_rays(int device, int64_t n, double u, double v, double f, double pan, double tilt,
                          const double* d6, const double* xy, double* rays_out) {
  if (n < 0) return fail("n < 0");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(device));
  Tmp t;
  double *dxy = t.in(xy, 2 * n), *dr = t.out(2 * n);
  NEED(dxy && dr);
  launch_back_project(n, u, v, f, pan, tilt, d6, dxy, dr, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(rays_out, dr, 2 * n * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptz_h_jacobian(int device, int64_t n, double u, double v, double f, double pan, double tilt, const double* d6,
                   const double* rays, double* H_out) {
  if (n < 0) return fail("n < 0");
  if (n == 0) return 0;
  HIPCHK(hipSetDevice(device));
  Tmp t;
  const size_t nh = (size_t)(2 * n) * (size_t)(3 + 2 * n);
  double *dr = t.in(rays, 2 * n), *dH = t.out(nh);
  NEED(dr && dH);
  HIPCHK(hipMemset(dH, 0, nh * 8));
  launch_h_jacobian(n, u, v, f, pan, tilt, d6, dr, dH, nullptr);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpy(H_out, dH, nh * 8, hipMemcpyDeviceToHost));
  return 0;
}

int ptzba_coupling_window(int32_t n_pose, int32_t n_landmark, int64_t n_obs, const int32_t* obs_frame,
                          const int32_t* obs_landmark, int32_t* win_out) {
  if (n_pose < 1 || n_landmark < 0 || n_obs < 0 || !win_out || (n_obs > 0 && (!obs_frame || !obs_landmark)))
    return fail("bad arguments");
  std::vector<int32_t> hi(std::max(n_landmark, 1), -1);
  for (int64_t r = 0; r < n_obs; ++r) {
    const int32_t f = obs_frame[r], l = obs_landmark[r];
    if (f < 0 || f >= n_pose || l < 0 || l >= n_landmark) return fail("record %lld out of range", (long long)r);
    hi[l] = std::max(hi[l], f);
  }
  for (int f = 0; f < n_pose; ++f) win_out[f] = f;
  for (int64_t r = 0; r < n_obs; ++r) win_out[obs_frame[r]] = std::max(win_out[obs_frame[r]], hi[obs_landmark[r]]);
  return 0;
}

// Landmark -> rank assignment of a sharded solve (include/ptzba.h): the part-owned split when the frame
// chain has one (landmarks seeing A to rank group 0, B to group 1, C-only landmarks to the group whose part
// their first frame is nearer; equal-record contiguous blocks inside a group), else contiguous landmark
// blocks of equal record counts over all ranks (replicated solve).
// host only (no device): the order and plan set_problem would choose for a coupling window -- for tests and
// tools (include/ptzba.h)
int ptzba_plan_summary(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t ordering, int64_t* out8) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !out8) return fail("bad arguments");
  if (ordering < PTZBA_ORDER_NATURAL || ordering > PTZBA_ORDER_NESTED_FORCE) return fail("bad ordering %d", ordering);
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  SysOrder so;
  CholPlan plan;
  if (choose_order_plan(n_pose, n_fixed, win, ordering, so, plan)) return fail("no factorisation plan");
  int max_tasks = 0;
  for (int L = 0; L < plan.n_levels; ++L) max_tasks = std::max(max_tasks, plan.level_off[L + 1] - plan.level_off[L]);
  int max_chain = 0;
  for (size_t c = 0; c + 1 < plan.chain_off.size(); ++c) max_chain = std::max(max_chain, plan.chain_off[c + 1] - plan.chain_off[c]);
  out8[0] = so.n_aug;
  out8[1] = pad_tile(so.n_aug + 1);
  out8[2] = plan.n_levels;
  out8[3] = so.nd_depth;
  out8[4] = (int64_t)plan.chain_off.size() - 1;
  out8[5] = max_chain;
  out8[6] = (int64_t)plan.bsb_step_off.size() - 1;  // blocked back-solve steps (0: no valid schedule)
  out8[7] = max_tasks | ((int64_t)plan.delayed << 32);
  return 0;
}

// host only: the chosen order's frame positions and the factorisation task list (int4 records, as the level
// launches receive them) with the level offsets -- the plan a CPU executor of the tile tasks can replay
int ptzba_plan_export(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t ordering, int32_t* pos_out,
                      int32_t* tasks_out, int64_t tasks_cap, int32_t* level_off_out, int64_t levels_cap, int64_t* counts) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !counts) return fail("bad arguments");
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  SysOrder so;
  CholPlan plan;
  if (choose_order_plan(n_pose, n_fixed, win, ordering, so, plan)) return fail("no factorisation plan");
  const int64_t nt = (int64_t)plan.tasks.size() / 4, nl = plan.n_levels;
  counts[0] = nt;
  counts[1] = nl;
  counts[2] = so.n_aug;
  counts[3] = plan.delayed ? 1 : 0;
  // a null output buffer only queries the counts; a non-null one that is too small is an error (no partial copy)
  if (tasks_out && tasks_cap < nt) return fail("tasks buffer holds %lld tasks, the plan has %lld", (long long)tasks_cap, (long long)nt);
  if (level_off_out && levels_cap < nl + 1)
    return fail("level offset buffer holds %lld entries, the plan needs %lld", (long long)levels_cap, (long long)(nl + 1));
  if (pos_out) std::copy(so.pos.begin(), so.pos.end(), pos_out);
  if (tasks_out) std::copy(plan.tasks.begin(), plan.tasks.end(), tasks_out);
  if (level_off_out) std::copy(plan.level_off.begin(), plan.level_off.end(), level_off_out);
  return 0;
}

// host only (round 6): which form of an N-rank solve the planner predicts faster -- the rank tree (each rank factors
// its subtree + its ancestors' separators, separator blocks summed per group) or the replicated solve (one all-reduce
// of the packed system, every rank factors all of it).  Both shard the landmarks over all ranks, so K1 / K2 / trial
// cancel out; compared are the slowest rank's factorisation estimate (plan_est_us, the planner's own figure) plus its
// collectives per trial as ring all-reduces, alpha + 2 (p - 1) / p * bytes / B.  At config 3 the tree
// does not shorten the chain (separators ~110 frames), so its extra exchanges lose from 4 ranks on; at config 4 the
// tree's factorisation is 1.5-2x shorter.  out8: [0] tree estimate us (0: no tree), [1] replicated us, [2] the tree's
// slowest-rank factorisation us, [3] the full plan's factorisation us, [4] tree collectives per trial on that rank,
// [5] tree doubles on that rank, [6] replicated doubles (packed system), [7] chosen form (1 tree, 0 replicated).
int ptzba_dist_form_estimate(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world,
                             double alpha_us, double link_gbs, double* out8) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !out8 || world < 1 || !(alpha_us >= 0) ||
      !(link_gbs > 0))
    return fail("bad arguments");
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  std::fill(out8, out8 + 8, 0.0);
  auto ring_us = [&](double doubles, int p) {
    return p < 2 ? 0.0 : alpha_us + 2.0 * (p - 1) / p * 8.0 * doubles / (link_gbs * 1e3);
  };
  SysOrder so;
  CholPlan plan;
  if (choose_order_plan(n_pose, n_fixed, win, PTZBA_ORDER_NESTED, so, plan)) return fail("no factorisation plan");
  const double sys_doubles = (double)(plan.xtiles.size() / 2) * CHOL_NB * CHOL_NB + 3.0 * (double)pad_tile(so.n_aug + 1);
  const double full_us = plan_est_us(plan);
  const double scal = 2.0 * PTZBA_NSCALARS;
  out8[1] = full_us + ring_us(sys_doubles, world) + ring_us(scal, world);
  out8[3] = full_us;
  out8[6] = sys_doubles;
  SysOrder o;
  DistTree DT;
  if (world >= 2 && dist_order(n_pose, n_fixed, win, world, o) && dist_tree(o, world, DT)) {
    const int64_t ld = pad_tile(o.n_aug + 1);
    double worst = 0;
    for (int r = 0; r < world; ++r) {
      CholPlan P;
      TreePlan Q;
      if (!make_plan_tree(o, DT, r, n_pose, n_fixed, win, ld, P, Q)) return fail("no rank-tree plan for rank %d", r);
      double comm = ring_us(scal, world), nd = 0;
      int nx = 1;
      for (size_t q = 0; q < Q.ph.size(); ++q) {
        const auto& t = Q.ph[q];
        if (q == 0 && t.nr < 2) continue;
        const double n = (double)(t.xt.size() / 2) * CHOL_NB * CHOL_NB + t.vr.count[0] + t.vr.count[1] + t.vr.count[2];
        comm += ring_us(n, t.nr);
        nd += n;
        ++nx;
      }
      const double est = plan_est_us(P);
      if (est + comm > worst) {
        worst = est + comm;
        out8[2] = est;
        out8[4] = nx;
        out8[5] = nd;
      }
    }
    out8[0] = worst;
  }
  out8[7] = (out8[0] > 0 && out8[0] <= out8[1]) ? 1.0 : 0.0;
  return 0;
}

// host only: the rank-tree plan set_problem builds for rank `rank` of `world` (tools/dist_predict.py, tests)
int ptzba_dist_plan_summary(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world, int32_t rank,
                            int64_t* out16) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !out16 || world < 1 || rank < 0 || rank >= world)
    return fail("bad arguments");
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  std::fill(out16, out16 + 16, 0);
  SysOrder o;
  DistTree DT;
  if (world < 2 || !dist_order(n_pose, n_fixed, win, world, o) || !dist_tree(o, world, DT)) return 0;
  CholPlan P;
  TreePlan Q;
  const int64_t ld = pad_tile(o.n_aug + 1);
  if (!make_plan_tree(o, DT, rank, n_pose, n_fixed, win, ld, P, Q)) return fail("no rank-tree plan");
  out16[0] = 1;
  out16[1] = o.nd_depth;
  out16[2] = Q.base;
  out16[3] = (int64_t)Q.ph.size();
  out16[4] = P.n_levels;
  out16[5] = (int64_t)plan_est_us(P);
  out16[6] = P.level_off[P.n_levels];
  int mx = 0;
  for (int L = 0; L < P.n_levels; ++L) mx = std::max(mx, P.level_off[L + 1] - P.level_off[L]);
  out16[7] = mx;
  for (size_t q = 0; q < Q.ph.size(); ++q) {
    const auto& t = Q.ph[q];
    if (q == 0 && t.nr < 2) continue;
    const int64_t n = (int64_t)(t.xt.size() / 2) * CHOL_NB * CHOL_NB + t.vr.count[0] + t.vr.count[1] + t.vr.count[2];
    out16[t.kind == PTZBA_X_PART ? 8 : (t.kind == PTZBA_X_SUB ? 9 : 10)] += n;
    out16[t.kind == PTZBA_X_PART ? 11 : (t.kind == PTZBA_X_SUB ? 12 : 13)] = t.nr;
  }
  out16[14] = o.n_aug;
  out16[15] = (int64_t)P.bsb_step_off.size() - 1;
  return 0;
}

// host only: rank `rank`'s whole rank-tree plan for a CPU replay (tests/test_plan_replay.py): frame positions, tasks,
// level offsets, per phase {lv0, lv1, exchange kind, group first rank, group size, exchanged tiles}, and the tiles
// (ti, tj) of every phase's exchange concatenated.  counts: [0] tasks, [1] levels, [2] n_aug, [3] phases,
// [4] exchanged tiles.  Null outputs only query the counts.
int ptzba_dist_plan_export(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world, int32_t rank,
                           int32_t* pos_out, int32_t* tasks_out, int64_t tasks_cap, int32_t* level_off_out,
                           int64_t levels_cap, int32_t* phases_out, int32_t phases_cap, int32_t* xt_out, int64_t xt_cap,
                           int64_t* counts) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !counts || world < 2 || rank < 0 || rank >= world)
    return fail("bad arguments");
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  SysOrder o;
  DistTree DT;
  if (!dist_order(n_pose, n_fixed, win, world, o) || !dist_tree(o, world, DT)) return fail("no rank-tree split");
  CholPlan P;
  TreePlan Q;
  if (!make_plan_tree(o, DT, rank, n_pose, n_fixed, win, pad_tile(o.n_aug + 1), P, Q)) return fail("no rank-tree plan");
  int64_t nxt = 0;
  for (const auto& t : Q.ph) nxt += (int64_t)t.xt.size() / 2;
  counts[0] = (int64_t)P.tasks.size() / 4;
  counts[1] = P.n_levels;
  counts[2] = o.n_aug;
  counts[3] = (int64_t)Q.ph.size();
  counts[4] = nxt;
  if ((tasks_out && tasks_cap < counts[0]) || (level_off_out && levels_cap < counts[1] + 1) ||
      (phases_out && phases_cap < counts[3]) || (xt_out && xt_cap < nxt))
    return fail("an output buffer is too small");
  if (pos_out) std::copy(o.pos.begin(), o.pos.end(), pos_out);
  if (tasks_out) std::copy(P.tasks.begin(), P.tasks.end(), tasks_out);
  if (level_off_out) std::copy(P.level_off.begin(), P.level_off.end(), level_off_out);
  for (size_t q = 0; q < Q.ph.size(); ++q) {
    const auto& t = Q.ph[q];
    if (phases_out) {
      int32_t* r = phases_out + 6 * q;
      r[0] = t.lv0; r[1] = t.lv1; r[2] = t.kind; r[3] = t.r0; r[4] = t.nr; r[5] = (int32_t)(t.xt.size() / 2);
    }
    if (xt_out) {
      std::copy(t.xt.begin(), t.xt.end(), xt_out);
      xt_out += t.xt.size();
    }
  }
  return 0;
}

// host only: the phases of rank `rank` (tests/numpy_handle.py NumpyTreeHandle emulates the protocol from them):
// per phase {exchange kind before it, group first rank, group size, first frame, end frame}
int ptzba_dist_rank_phases(int32_t n_pose, int32_t n_fixed, const int32_t* frame_win_hi, int32_t world, int32_t rank,
                           int32_t* out, int32_t cap, int32_t* n_out) {
  if (n_pose < 1 || n_fixed < 0 || n_fixed > n_pose || !frame_win_hi || !n_out || world < 2 || rank < 0 || rank >= world)
    return fail("bad arguments");
  std::vector<int32_t> win(frame_win_hi, frame_win_hi + n_pose);
  for (int f = 0; f < n_pose; ++f)
    if (win[f] < f || win[f] >= n_pose) return fail("frame_win_hi[%d] = %d out of range", f, win[f]);
  SysOrder o;
  DistTree DT;
  *n_out = 0;
  if (!dist_order(n_pose, n_fixed, win, world, o) || !dist_tree(o, world, DT)) return 0;
  std::vector<int> anc;
  const int base = dist_base(DT, rank, &anc);
  const auto& bn = DT.n[base];
  std::vector<int32_t> v;
  if (bn.nr >= 2) v.insert(v.end(), {PTZBA_X_PART, bn.r0, bn.nr, bn.f0, bn.f1});
  else v.insert(v.end(), {PTZBA_X_PART, rank, 1, bn.sf0, bn.sf1});
  for (int u : anc)
    v.insert(v.end(), {DT.n[u].parent < 0 ? PTZBA_X_SEP : PTZBA_X_SUB, DT.n[u].r0, DT.n[u].nr, DT.n[u].f0, DT.n[u].f1});
  *n_out = (int32_t)(v.size() / 5);
  if (out) {
    if (cap < *n_out) return fail("output holds %d phases, %d needed", cap, *n_out);
    std::copy(v.begin(), v.end(), out);
  }
  return 0;
}

int ptzba_partition_landmarks(int32_t n_pose, int32_t n_landmark, int64_t n_obs, const int32_t* obs_frame,
                              const int32_t* obs_landmark, int32_t n_fixed, int32_t world, int32_t* rank_of_landmark,
                              int32_t* mode_out, int32_t* split_out) {
  if (n_pose < 1 || n_landmark < 0 || n_obs < 0 || world < 1 || n_fixed < 0 || n_fixed > n_pose || !rank_of_landmark ||
      (n_obs > 0 && (!obs_frame || !obs_landmark)))
    return fail("bad arguments");
  std::vector<int32_t> win(n_pose);
  if (ptzba_coupling_window(n_pose, n_landmark, n_obs, obs_frame, obs_landmark, win.data())) return -1;
  std::vector<int64_t> cnt(std::max(n_landmark, 1), 0);
  std::vector<int32_t> lo(std::max(n_landmark, 1), INT32_MAX), hi(std::max(n_landmark, 1), -1);
  for (int64_t r = 0; r < n_obs; ++r) {
    const int l = obs_landmark[r], f = obs_frame[r];
    cnt[l]++;
    if (f >= n_fixed) {
      lo[l] = std::min(lo[l], f);
      hi[l] = std::max(hi[l], f);
    }
  }
  // equal-record contiguous blocks of the landmarks in `ids` over ranks [r0, r0 + nr)
  auto blocks = [&](const std::vector<int32_t>& ids, int r0, int nr) {
    int64_t tot = 0;
    for (int l : ids) tot += cnt[l];
    int64_t acc = 0;
    for (int l : ids) {
      const int k = tot > 0 ? (int)std::min<int64_t>(nr - 1, (acc * nr) / std::max<int64_t>(tot, 1)) : 0;
      rank_of_landmark[l] = r0 + k;
      acc += cnt[l];
    }
  };
  for (int l = 0; l < n_landmark; ++l) rank_of_landmark[l] = -1;
  SysOrder o;
  DistTree DT;
  const bool part = world >= 2 && dist_order(n_pose, n_fixed, win, world, o) && dist_tree(o, world, DT);
  if (mode_out) *mode_out = part ? 1 : 0;
  if (split_out) {
    split_out[0] = part ? o.split_m : 0;
    split_out[1] = part ? o.split_cend : 0;
    split_out[2] = n_pose;
  }
  if (!part) {
    std::vector<int32_t> ids;
    for (int l = 0; l < n_landmark; ++l)
      if (cnt[l] > 0) ids.push_back(l);
    blocks(ids, 0, world);
    return 0;
  }
  // rank tree (make_plan_tree): from the root, a landmark goes to the child whose subtree frames it sees (no landmark
  // sees both: the node's separator); one that sees only separator frames goes to the child nearer to it; a node
  // with one rank keeps it; a shared leaf deals its landmarks out in equal-record contiguous blocks
  // the tree nodes each landmark's (non-fixed) frames lie in, as a bit mask; per node the mask of its subtree
  const int nn = (int)DT.n.size();
  if (nn > 32) return fail("rank tree too large");
  std::vector<int32_t> node_of(n_pose, -1);
  for (int v = 0; v < nn; ++v)
    for (int f = DT.n[v].f0; f < DT.n[v].f1; ++f) node_of[f] = v;
  std::vector<uint32_t> lmask(std::max(n_landmark, 1), 0u), smask(nn, 0u);
  for (int64_t r = 0; r < n_obs; ++r)
    if (obs_frame[r] >= n_fixed && node_of[obs_frame[r]] >= 0) lmask[obs_landmark[r]] |= 1u << node_of[obs_frame[r]];
  for (int v = 0; v < nn; ++v)
    for (int u = v; u >= 0; u = DT.n[u].parent) smask[u] |= 1u << v;
  std::vector<std::vector<int32_t>> leaf_ids(DT.n.size());
  for (int l = 0; l < n_landmark; ++l) {
    if (cnt[l] == 0) continue;
    int v = 0;
    for (;;) {
      const auto& x = DT.n[v];
      if (x.nr == 1) {
        rank_of_landmark[l] = x.r0;
        break;
      }
      if (x.nch != 2) {
        leaf_ids[v].push_back(l);
        break;
      }
      int go;
      if (hi[l] < 0) {
        go = 0;  // fixed frames only
      } else {
        const bool in0 = (lmask[l] & smask[x.child[0]]) != 0, in1 = (lmask[l] & smask[x.child[1]]) != 0;
        if (in0 && in1) return fail("landmark %d couples both parts (bad split)", l);
        if (in0) go = 0;
        else if (in1) go = 1;
        else go = (lo[l] - x.f0) < (x.f1 - 1 - hi[l]) ? 0 : 1;  // separator frames only: the nearer part
      }
      v = x.child[go];
    }
  }
  for (size_t v = 0; v < DT.n.size(); ++v)
    if (!leaf_ids[v].empty()) blocks(leaf_ids[v], DT.n[v].r0, DT.n[v].nr);
  return 0;
}

// ------------------------------------------------------------------------------------------------
// matching-graph landmark ids: first-seen rule of image_process.py:611-639 (bit-exact)
// ------------------------------------------------------------------------------------------------
int ptzba_build_landmarks(int32_t n_frames, const int64_t* kp_count, int64_t n_pairs, const int32_t* pair_i,
                          const int32_t* pair_j, const int64_t* pair_count, const int64_t* idx_a, const int64_t* idx_b,
                          int64_t* landmark_out, int64_t* n_landmark, int64_t* n_inconsistent) {
  if (n_frames < 0 || n_pairs < 0) return fail("bad sizes");
  std::vector<std::vector<int64_t>> map(n_frames);
  for (int f = 0; f < n_frames; ++f) {
    if (kp_count[f] < 0) return fail("bad kp_count");
    map[f].assign((size_t)kp_count[f], -1);
  }
  int64_t g = 0, warn = 0, off = 0;
  for (int64_t p = 0; p < n_pairs; ++p) {
    const int i = pair_i[p], j = pair_j[p];
    if (i < 0 || i >= n_frames || j < 0 || j >= n_frames) return fail("pair %lld: frame out of range", (long long)p);
    for (int64_t k = 0; k < pair_count[p]; ++k) {
      const int64_t a = idx_a[off + k], b = idx_b[off + k];
      if (a < 0 || a >= kp_count[i] || b < 0 || b >= kp_count[j]) return fail("pair %lld: keypoint index out of range", (long long)p);
      int64_t& ma = map[i][a];
      int64_t& mb = map[j][b];
      if (ma >= 0 && mb >= 0) {
        if (ma != mb) ++warn;
      } else if (ma >= 0) {
        mb = ma;
      } else if (mb >= 0) {
        ma = mb;
      } else {
        ma = g;
        mb = g;
        ++g;
      }
    }
    off += pair_count[p];
  }
  // landmark of each match = landmark_index_map[i][idx1] after all pairs (image_process.py:652-653)
  off = 0;
  for (int64_t p = 0; p < n_pairs; ++p) {
    for (int64_t k = 0; k < pair_count[p]; ++k) landmark_out[off + k] = map[pair_i[p]][idx_a[off + k]];
    off += pair_count[p];
  }
  *n_landmark = g;
  if (n_inconsistent) *n_inconsistent = warn;
  return 0;
}



// host-driven LM (ptzba.LMSolver._run_host, ptzba_linearize / ptzba_step): the huber curvature weight of the
// following linearisations (the device-driven LM keeps its own in LMDev::hc)
int ptzba_set_huber_curvature(ptzba_handle h, double hc) {
  if (!h) return fail("null handle");
  if (!(hc > 0.0 && hc <= 1.0)) return fail("huber curvature must lie in (0, 1]");
  h->hcurv = hc;
  return 0;
}

// which front the following set_problem calls use (round 6): the device front from min_records records on
// (0: always, INT64_MAX: never, -1: the default GPU_SETUP_MIN_REC = 64K).  Both fronts build the same arrays bit for bit
// (tests/test_gpu_ba.py compares them); the knob is the test hook and a per-handle tuning point.
int ptzba_set_setup_front(ptzba_handle h, int64_t min_records) {
  if (!h) return fail("null handle");
  h->gpu_setup_min = min_records < 0 ? -1 : min_records;
  return 0;
}

// host phase times of the last ptzba_set_problem: names[k] (static strings) and ms[k], k < *n_out (<= cap)
int ptzba_setup_timing(ptzba_handle h, int32_t cap, const char** names, double* ms, int32_t* n_out) {
  if (!h || !n_out || cap < 0 || (cap > 0 && (!names || !ms))) return fail("ptzba_setup_timing: bad arguments");
  const int32_t n = (int32_t)std::min<size_t>(h->setup_phases.size(), (size_t)cap);
  for (int32_t k = 0; k < n; ++k) {
    names[k] = h->setup_phases[k].first;
    ms[k] = h->setup_phases[k].second;
  }
  *n_out = (int32_t)h->setup_phases.size();
  return 0;
}
