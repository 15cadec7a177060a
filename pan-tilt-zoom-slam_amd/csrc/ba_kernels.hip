// Bundle-adjustment kernels for gfx950 (CDNA4, wave64).
//
// Hot path: one Levenberg-Marquardt iteration over the reference's
// pair-form reprojection residual (bundle_adjustment.py:25-106), solved exactly through the
// Schur complement on the keyframe poses instead of scipy's dense FD-Jacobian + SVD trf
// (bundle_adjustment.py:200-202).
//
// Data layout in HBM (all built once by ptzba_set_problem, see api.hip):
//   records   sorted by (landmark, frame, original index); SoA  rec_xy[2R] (real), rec_seg[R] (int32)
//             and optional rec_w[R] (multiplicity of de-duplicated records)
//   segments  one per unique (landmark, frame): seg_frame, seg_rec_begin (CSR into records);
//             landmark CSR lm_seg_begin; frame CSR frame_seg_begin/frame_seg_list
//   tables    FrameTab[n_pose] (cos/sin pan, cos/sin tilt, f), RayTab[n_lm] (ray direction + derivs)
//   lin       w_slot[n_slot][W_STRIDE] = W(3x2) (real) in the dense landmark x frame slot table:
//                                 slot = toff_l + frame - first_l; slots of unobserved frames stay 0
//             ug_slot[n_slot][UG_STRIDE] = U(3x3 sym, 6) | g_pose(3) (real, same slots; summed per frame by K2)
//             lm_out[n_lm][8]    = V(2x2 sym, 3) | g_ray(2) | cost | pad      (fp64)
//
// K1 `k_linearize` is the HBM-streaming kernel: one wave per landmark walks the landmark's records
// (coalesced 8/16-B loads), forms residuals against per-segment projections staged in LDS, and
// segment-reduces the sufficient statistics (sum w, sum w r per image axis) with a wave64 segmented
// scan.  All observations of one (frame, landmark) segment share the projection and the 2x5
// Jacobian (they depend on pose and ray only), so the Jacobian and the 3x3/3x2/2x2 normal-equation
// blocks are formed once per segment.
#include "../../include/ptzba.h"
#include "ptzba_common.h"
#include <hip/hip_ext.h>

#include "ptzba_kernels.h"

namespace ptzba {

// ------------------------------------------------------------------------------------------------
// tables
// ------------------------------------------------------------------------------------------------
template <typename real>
__global__ void k_tables(const double* __restrict__ ptz, const double* __restrict__ rays, int n_pose,
                         int n_lm, FrameTab<double>* __restrict__ ft64, RayTab<double>* __restrict__ rt64,
                         FrameTab<real>* __restrict__ ft, RayTab<real>* __restrict__ rt,
                         const int* __restrict__ run_if, double* __restrict__ zero, int n_zero) {
  if (run_if && !*run_if) return;
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n_zero) zero[i] = 0.0;  // (ptzba_linearize: the scalar block, instead of a memset launch)
  if (i < n_pose) {
    FrameTab<double> t = make_frame_tab<double>(ptz[3 * i], ptz[3 * i + 1], ptz[3 * i + 2]);
    ft64[i] = t;
    if constexpr (sizeof(real) != sizeof(double)) {
      FrameTab<real> r;
      r.ca = (real)t.ca; r.sa = (real)t.sa; r.cb = (real)t.cb; r.sb = (real)t.sb; r.f = (real)t.f;
      r.pad0 = r.pad1 = r.pad2 = (real)0;
      ft[i] = r;
    }
  } else if (i < n_pose + n_lm) {
    int l = i - n_pose;
    RayTab<double> t = make_ray_tab<double>(rays[2 * l], rays[2 * l + 1]);
    rt64[l] = t;
    if constexpr (sizeof(real) != sizeof(double)) {
      RayTab<real> r;
      r.p0 = (real)t.p0; r.p1 = (real)t.p1; r.d0t = (real)t.d0t; r.d1t = (real)t.d1t; r.d1p = (real)t.d1p;
      r.pad0 = r.pad1 = r.pad2 = (real)0;
      rt[l] = r;
    }
  }
}

template <typename real>
void launch_tables(const double* ptz, const double* rays, int n_pose, int n_lm, void* ft64, void* rt64, void* ft,
                   void* rt, const int* run_if, hipStream_t st, double* zero, int n_zero) {
  int n = std::max(n_pose + n_lm, n_zero);
  hipLaunchKernelGGL(k_tables<real>, dim3((n + 255) / 256), dim3(256), 0, st, ptz, rays, n_pose, n_lm,
                     (FrameTab<double>*)ft64, (RayTab<double>*)rt64, (FrameTab<real>*)ft, (RayTab<real>*)rt, run_if,
                     zero, n_zero);
}

// ------------------------------------------------------------------------------------------------
// K1: linearize (residual + Jacobian + per-segment / per-landmark normal-equation blocks + cost)
// ------------------------------------------------------------------------------------------------
constexpr int SEGW = K1_SEGW;  // segments per LDS window per wave
#ifndef K1_FTL_ALWAYS
#define K1_FTL_ALWAYS 1
#endif
#ifndef K1_RPL
#define K1_RPL 4  // phase B: records per lane (one segmented scan per 64 K1_RPL records; 8 measured 62.0 vs 60.4 us, r06j)
#endif
// (Round 5 removed the measured-slower build variants: one record per lane (K1_COARSE 0), three record groups in
// flight (K1_DEPTH 3), LDS-atomic tail runs, issue-order tails and phase C's own table loads (K1_FTV_LATE))
#ifndef K1_WPB
#define K1_WPB 4  // waves (landmarks) per workgroup: the frame tables are staged once per workgroup
#endif
#ifndef K1_MIN_WAVES
#define K1_MIN_WAVES 4  // waves per SIMD the register budget must allow (occupancy)
#endif
#ifndef K1_MIN_WAVES64
#define K1_MIN_WAVES64 3  // fp64: 4 waves/SIMD spill 128-196 B/lane; 3 fit (fp64 K1 193 -> 138 us, r02 A/B)
#endif

// ---- DPP lane shuffles (VALU, no LDS round trip).  Lanes whose source is out of range or whose row
// is masked off read 0 (bound_ctrl), which the segmented scan treats as "different segment".
template <int CTRL, int ROWMASK>
__device__ __forceinline__ int dpp_i(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, ROWMASK, 0xf, true);
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ float dpp_r(float x) {
  return __int_as_float(dpp_i<CTRL, ROWMASK>(__float_as_int(x)));
}
template <int CTRL, int ROWMASK>
__device__ __forceinline__ double dpp_r(double x) {
  const int lo = dpp_i<CTRL, ROWMASK>(__double2loint(x)), hi = dpp_i<CTRL, ROWMASK>(__double2hiint(x));
  return __hiloint2double(hi, lo);
}
constexpr int DPP_ROW_SHR1 = 0x111, DPP_ROW_SHR2 = 0x112, DPP_ROW_SHR4 = 0x114, DPP_ROW_SHR8 = 0x118;
constexpr int DPP_ROW_BCAST15 = 0x142, DPP_ROW_BCAST31 = 0x143, DPP_WAVE_SHL1 = 0x130;

// Wave total by a DPP inclusive scan (VALU only): the sum is valid in lane 63.  Needs every lane active.
// The butterfly of wave_sum costs one LDS round trip (ds_bpermute) per step and value: at the end of K1
// six fp64 butterflies took ~5K cycles per wave, 15 % of the wave's time (K1_TIMING build).
template <typename T>
__device__ __forceinline__ T wave_total(T v) {
  v += dpp_r<DPP_ROW_SHR1, 0xf>(v);
  v += dpp_r<DPP_ROW_SHR2, 0xf>(v);
  v += dpp_r<DPP_ROW_SHR4, 0xf>(v);
  v += dpp_r<DPP_ROW_SHR8, 0xf>(v);
  v += dpp_r<DPP_ROW_BCAST15, 0xa>(v);
  v += dpp_r<DPP_ROW_BCAST31, 0xc>(v);
  return v;
}

// Six wave totals at once, step by step across the values (round 6): each DPP step's six reads of the previous step's
// results are independent, so the DPP read-after-write wait states of one value are covered by the others' work
// instead of s_nop padding (six back-to-back wave_total calls serialised).  Same additions, same order per value.
template <int CTRL, int ROWMASK>
__device__ __forceinline__ void wave_total_step6(double (&v)[6]) {
  double t[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) t[k] = dpp_r<CTRL, ROWMASK>(v[k]);
#pragma unroll
  for (int k = 0; k < 6; ++k) v[k] += t[k];
}
__device__ __forceinline__ void wave_total6(double (&v)[6]) {
  wave_total_step6<DPP_ROW_SHR1, 0xf>(v);
  wave_total_step6<DPP_ROW_SHR2, 0xf>(v);
  wave_total_step6<DPP_ROW_SHR4, 0xf>(v);
  wave_total_step6<DPP_ROW_SHR8, 0xf>(v);
  wave_total_step6<DPP_ROW_BCAST15, 0xa>(v);
  wave_total_step6<DPP_ROW_BCAST31, 0xc>(v);
}

// one Kogge-Stone step of the segmented inclusive scan (keys sorted within the wave; kenc >= 1)
template <int CTRL, int ROWMASK, typename real>
__device__ __forceinline__ void seg_scan_step(int kenc, real& v0, real& v1, real& v2, real& v3) {
  const int kk = dpp_i<CTRL, ROWMASK>(kenc);
  const real t0 = dpp_r<CTRL, ROWMASK>(v0), t1 = dpp_r<CTRL, ROWMASK>(v1);
  const real t2 = dpp_r<CTRL, ROWMASK>(v2), t3 = dpp_r<CTRL, ROWMASK>(v3);
  if (kk == kenc) {
    v0 += t0; v1 += t1; v2 += t2; v3 += t3;
  }
}

__device__ __forceinline__ void store4(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<float4*>(p) = make_float4(a, b, c, d);
}
__device__ __forceinline__ void store4(double* p, double a, double b, double c, double d) {
  reinterpret_cast<double2*>(p)[0] = make_double2(a, b);
  reinterpret_cast<double2*>(p)[1] = make_double2(c, d);
}

#ifdef K1_TIMING
// phase timing build (tools/k1_timing.py): per task (plain stores, no shared counters: same-address atomics
// from every wave would serialise the launch) start / end stamps (s_memrealtime) and clock64 phase sums
__device__ long long g_k1_items[32768][8];  // start, end, A, B, C, final, segments, -
#define K1_NOW(t) do { t = clock64(); } while (0)
#define K1_ACC(k, t0, t1) do { k1acc[k] += (t1) - (t0); } while (0)
#else
#define K1_NOW(t) do { } while (0)
#define K1_ACC(k, t0, t1) do { } while (0)
#endif
// FTL: the frame tables are staged in LDS (n_pose <= K1_FT_LDS): phase A's chain is descriptor -> segment frame id
// -> LDS instead of descriptor -> frame id -> global frame table (one dependent memory latency less per wave)
// WT: records carry multiplicities (rec_w; the dedup form) -- unweighted problems keep no weight registers
template <typename real, int LOSS, bool FTL, bool WT = true>
__global__ __launch_bounds__(64 * K1_WPB, sizeof(real) == 4 ? K1_MIN_WAVES : K1_MIN_WAVES64) void k_linearize(LinArgs a) {
  __shared__ real s_x[K1_WPB][SEGW], s_y[K1_WPB][SEGW], s_acc[K1_WPB][4][SEGW];
  __shared__ double s_ft[5][FTL ? K1_FT_LDS : 1];  // ca, sa, cb, sb, f per frame (fp64)
  const int lane = lane_id();
  // wave-uniform by construction: with readfirstlane the compiler sees it, so the descriptor, the ray table, the
  // window and record bounds and the slot offsets are scalar loads / SGPRs (SALU address math, fewer VGPRs)
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int task = blockIdx.x * K1_WPB + wv;
  if (a.run_if && !*a.run_if) return;  // conditional re-linearisation (device-driven LM): the whole grid leaves
  if constexpr (!FTL) {
    if (task >= a.n_work) return;  // whole wave leaves; no block-level barriers in this variant
  }
  long long kt0 = 0, kt1 = 0, kt2 = 0, kt3 = 0, kt4 = 0, k1acc[4] = {0, 0, 0, 0};
  (void)kt0; (void)kt1; (void)kt2; (void)kt3; (void)kt4; (void)k1acc;
  K1_NOW(kt0);
#ifdef K1_TIMING
  if (lane == 0 && task < 32768) g_k1_items[task][0] = __builtin_amdgcn_s_memrealtime();
#endif
  // one 32-B work descriptor {landmark, first segment, end segment, first record | first frame, last
  // frame, slot offset, end record of the first window}: no dependent lm_order -> lm_seg_begin -> seg_rec_begin -> lm_meta chain before
  // the records and the frame tables can be requested
  const int tq = FTL ? min(task, a.n_work - 1) : task;
  const int4 wd = a.lm_work[2 * tq];
  const int4 wm = a.lm_work[2 * tq + 1];
  int fbase = 0;  // FTL: the first staged frame (s_ft[k][fs - fbase])
  bool ftl_ok = FTL;  // FTL: this workgroup's frame range fits the LDS table
  if constexpr (FTL) {
    // the frames the workgroup's landmarks see, [min first frame, max last frame] over its K1_WPB descriptors (scalar
    // loads; the work order keeps a workgroup's landmarks close in frame order, so this is ~a coupling window, not the
    // whole table); the barrier below is the block's only one
    int fmax = -1;
    fbase = a.n_pose;
#pragma unroll
    for (int q = 0; q < K1_WPB; ++q) {
      const int4 m = a.lm_work[2 * min((int)blockIdx.x * K1_WPB + q, a.n_work - 1) + 1];
      fbase = min(fbase, m.x);
      fmax = max(fmax, m.y);
    }
    ftl_ok = fmax - fbase < K1_FT_LDS;  // (else this workgroup reads the tables from global memory)
    const double4* src = reinterpret_cast<const double4*>(a.ft64);
    if (ftl_ok)
    for (int e = fbase + (int)threadIdx.x; e <= fmax; e += blockDim.x) {
      const double4 t0 = src[2 * e];
      const double f = reinterpret_cast<const double*>(a.ft64)[8 * e + 4];
      const int el = e - fbase;
      s_ft[0][el] = t0.x; s_ft[1][el] = t0.y; s_ft[2][el] = t0.z; s_ft[3][el] = t0.w; s_ft[4][el] = f;
    }
    __syncthreads();
    if (task >= a.n_work) return;  // whole wave leaves after the barrier
  }
  auto ft_lds = [&](int fs) {
    if (!ftl_ok) return ((const FrameTab<double>*)a.ft64)[fs];
    FrameTab<double> F;
    fs -= fbase;
    F.ca = s_ft[0][fs]; F.sa = s_ft[1][fs]; F.cb = s_ft[2][fs]; F.sb = s_ft[3][fs]; F.f = s_ft[4][fs];
    F.pad0 = F.pad1 = F.pad2 = 0.0;
    return F;
  };
  const int l = wd.x, s0 = wd.y, s1 = wd.z;
  const FrameTab<double>* __restrict__ ft64 = (const FrameTab<double>*)a.ft64;
  const RayTab<double> R64 = ((const RayTab<double>*)a.rt64)[l];
  RayTab<real> R;  // the record-precision table is the rounded fp64 one (k_tables)
  R.p0 = (real)R64.p0; R.p1 = (real)R64.p1; R.d0t = (real)R64.d0t; R.d1t = (real)R64.d1t; R.d1p = (real)R64.d1p;
  const FrameTab<real>* __restrict__ ft = (const FrameTab<real>*)a.ft;
  const double2* __restrict__ seg_base = a.seg_base;
  const real* __restrict__ rec_xy = (const real*)a.rec_xy;
  const real* __restrict__ rec_w = (const real*)a.rec_w;
  const bool alt = a.sel && ((*a.sel ^ a.sel_xor) & 1);  // device-chosen linearisation slot
  real* __restrict__ ug_slot = (real*)(alt ? a.ug_slot1 : a.ug_slot);
  real* __restrict__ w_slot = (real*)(alt ? a.w_slot1 : a.w_slot);
  const int64_t slot0 = (int64_t)wm.z - wm.x;
  const real u = (real)a.u, v = (real)a.v;
  const real fs2 = (real)a.fs2, ifs2 = (real)a.inv_fs2;
  const real hc = (real)(a.hcurv_dev ? *a.hcurv_dev : a.hcurv);
  real* sx = s_x[wv];
  real* sy = s_y[wv];
  real* acc0 = s_acc[wv][0];
  real* acc1 = s_acc[wv][1];
  real* acc2 = s_acc[wv][2];
  real* acc3 = s_acc[wv][3];

  double V00 = 0, V01 = 0, V11 = 0, g0 = 0, g1 = 0, cost = 0;

  // phase B, thread-coarsened: a lane owns RPL consecutive records of a 64 RPL-record batch (RPL-aligned: RPL / 4
  // 4-B key words and RPL / 2 16-B delta loads per lane), reduces its own runs, and only its tail run enters the wave's
  // segmented scan (one scan per 64 RPL records); records before r0 / after r1 of the aligned batch are masked (the
  // record arrays are padded by 8 records).  Round 6 measured RPL 8 (one scan per 512 records): slower (62.0 vs 60.4 us).
  constexpr int RPL = sizeof(real) == 4 ? K1_RPL : 4;  // (fp64: 3 waves / SIMD already at 4)
  static_assert(RPL == 4 || RPL == 8, "records per lane");
  struct CGrp {
    uint32_t keyw[RPL / 4];
    real ox[RPL], oy[RPL], wt[WT ? RPL : 1];
  };
  auto load_cgrp = [&](CGrp& g, int64_t rb, int64_t r1) {
    const int64_t q = min(rb + RPL * lane, (r1 - 1) & ~(int64_t)(RPL - 1));
#pragma unroll
    for (int k = 0; k < RPL / 4; ++k) g.keyw[k] = reinterpret_cast<const uint32_t*>(a.rec_key + q)[k];
    if constexpr (sizeof(real) == 4) {
#pragma unroll
      for (int k = 0; k < RPL / 2; ++k) {
        const float4 p = reinterpret_cast<const float4*>(rec_xy)[q / 2 + k];
        g.ox[2 * k] = p.x; g.oy[2 * k] = p.y; g.ox[2 * k + 1] = p.z; g.oy[2 * k + 1] = p.w;
      }
    } else {
#pragma unroll
      for (int j = 0; j < RPL; ++j) {
        const double2 o = reinterpret_cast<const double2*>(rec_xy)[q + j];
        g.ox[j] = o.x; g.oy[j] = o.y;
      }
    }
    if constexpr (WT) {
#pragma unroll
      for (int j = 0; j < RPL; ++j) g.wt[j] = rec_w[min(q + j, r1 - 1)];
    }
  };
  auto consume_c = [&](const CGrp& g, int64_t rb, int64_t r0, int64_t r1) {
    int key[RPL];
    real cb = 0;  // the batch's cost terms, summed in the record precision, then added in fp64
    // branch-free (round 6): the validity test on a 32-bit offset from r0, and the records' projection reads issued
    // unconditionally (key clamped into the window; an invalid record's values are masked below), so one LDS wait
    // serves the lane's records instead of one exec-masked branch with its own wait per record
    const int rel0 = (int)(rb - r0) + RPL * lane, nrec = (int)(r1 - r0);
    real px[RPL], py[RPL];
    bool vld[RPL];
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const int kb = (int)((g.keyw[j >> 2] >> (8 * (j & 3))) & 0xffu);
      vld[j] = (unsigned)(rel0 + j) < (unsigned)nrec;
      key[j] = vld[j] ? kb : (rel0 + j < 0 ? -1 : 255);
      px[j] = sx[kb & (SEGW - 1)];
      py[j] = sy[kb & (SEGW - 1)];
    }
    real t0 = 0, t1 = 0, t2 = 0, t3 = 0;  // the open run's sums
#pragma unroll
    for (int j = 0; j < RPL; ++j) {
      const bool valid = vld[j];
      const real rx = valid ? px[j] - g.ox[j] : (real)0;
      const real ry = valid ? py[j] - g.oy[j] : (real)0;
      real wt;
      if constexpr (WT) wt = valid ? g.wt[j] : (real)0;
      else wt = valid ? (real)1 : (real)0;
      real wx, wy, c, hx, hy;
      if constexpr (LOSS == 0) {
        wx = wt; wy = wt;
        hx = wt; hy = wt;
        c = wt * (rx * rx + ry * ry);
      } else {
        real zx = rx * rx * ifs2, zy = ry * ry * ifs2;
        bool ix = zx <= (real)1, iy = zy <= (real)1;
        real sqx, sqy;
        if constexpr (sizeof(real) == 4) {
          const real rsx = __builtin_amdgcn_rsqf(ix ? (real)1 : zx), rsy = __builtin_amdgcn_rsqf(iy ? (real)1 : zy);
          sqx = zx * rsx; sqy = zy * rsy;
          wx = ix ? wt : wt * rsx;
          wy = iy ? wt : wt * rsy;
        } else {
          sqx = sqrt(zx); sqy = sqrt(zy);
          wx = ix ? wt : wt / sqx;
          wy = iy ? wt : wt / sqy;
        }
        c = wt * fs2 * ((ix ? zx : (real)2 * sqx - (real)1) + (iy ? zy : (real)2 * sqy - (real)1));
        hx = ix ? wx : wx * hc;
        hy = iy ? wy : wy * hc;
      }
      cb += c;
      // runs merged forward as the records are formed (round 6: only the open run is live, not all RPL records'
      // terms): a run that ends inside the lane is the lane's alone unless it continues the previous lane's tail --
      // one set of LDS atomic adds per such run; the lane's tail run (key of its last record) joins the scan
      const real e0 = hx, e1 = hy, e2 = wx * rx, e3 = wy * ry;
      if (j == 0) {
        t0 = e0; t1 = e1; t2 = e2; t3 = e3;
      } else if (key[j] == key[j - 1]) {
        t0 += e0; t1 += e1; t2 += e2; t3 += e3;
      } else {
        if (key[j - 1] >= 0) {
          atomicAdd(acc0 + key[j - 1], t0); atomicAdd(acc1 + key[j - 1], t1);
          atomicAdd(acc2 + key[j - 1], t2); atomicAdd(acc3 + key[j - 1], t3);
        }
        t0 = e0; t1 = e1; t2 = e2; t3 = e3;
      }
    }
    cost += (double)cb;
    const int kt = key[RPL - 1];
    const int kenc = kt + 2;
    seg_scan_step<DPP_ROW_SHR1, 0xf>(kenc, t0, t1, t2, t3);
    seg_scan_step<DPP_ROW_SHR2, 0xf>(kenc, t0, t1, t2, t3);
    seg_scan_step<DPP_ROW_SHR4, 0xf>(kenc, t0, t1, t2, t3);
    seg_scan_step<DPP_ROW_SHR8, 0xf>(kenc, t0, t1, t2, t3);
    seg_scan_step<DPP_ROW_BCAST15, 0xa>(kenc, t0, t1, t2, t3);
    seg_scan_step<DPP_ROW_BCAST31, 0xc>(kenc, t0, t1, t2, t3);
    const int knext = dpp_i<DPP_WAVE_SHL1, 0xf>(kenc);
    // The next lane's head run may have added into the same slot above (ds_add).  A plain read-modify-write
    // after those adds have completed (lgkmcnt(0)) sees them; the compiler must not hoist the read above the
    // wait (per lane it can prove key[j] != kt, but the adds of OTHER lanes alias), hence the compiler
    // barrier.
    if (knext != kenc && kt >= 0 && kt < SEGW) {
      // the read below must see the ds_adds issued above by the other lanes of this wave: wait until they have
      // completed (lgkmcnt(0)) instead of relying on the LDS executing a wave's operations in issue order
      __builtin_amdgcn_s_waitcnt(0xc07f);
      asm volatile("" ::: "memory");
      acc0[kt] += t0; acc1[kt] += t1; acc2[kt] += t2; acc3[kt] += t3;
    }
  };

  for (int w0 = s0; w0 < s1; w0 += SEGW) {
    const int w1 = min(s1, w0 + SEGW);
    // the first window's record range comes with the descriptor (no dependent load before the records)
    const int64_t r0 = (w0 == s0) ? (int64_t)(uint32_t)wd.w : a.seg_rec_begin[w0];
    const int64_t r1 = (w0 == s0) ? (int64_t)(uint32_t)wm.w : a.seg_rec_begin[w1];
    // the window's first record group is requested before phase A: its latency overlaps the projections
    CGrp ca, cb;
    const int64_t rb0 = r0 & ~(int64_t)(RPL - 1);
    load_cgrp(ca, rb0, r1);
    // phase A: fp64 projection of every segment of the window (lanes over segments), kept as the
    // offset from the segment's base observation so phase B works on O(residual) magnitudes.  The
    // frame ids and the phase-C frame tables stay in registers.
    int fsv[SEGW / WAVE];
    FrameTab<real> ftv[SEGW / WAVE];  // phase C's frame tables, loaded here (off phase C's path)
#pragma unroll
    for (int i = 0; i < SEGW / WAVE; ++i) {
      const int s = w0 + lane + i * WAVE;
      fsv[i] = 0;
      if (s < w1) {
        const int sl = s - w0;
        const int fs = a.seg_frame[s];
        fsv[i] = fs;
        double x, y;
        if constexpr (FTL) ptz_project<double>(ft_lds(fs), R64, a.u, a.v, x, y);
        else ptz_project<double>(ft64[fs], R64, a.u, a.v, x, y);
        const double2 bs = seg_base[s];
        sx[sl] = (real)(x - bs.x);
        sy[sl] = (real)(y - bs.y);
        acc0[sl] = 0; acc1[sl] = 0; acc2[sl] = 0; acc3[sl] = 0;
      }
      if constexpr (!FTL) {  // (FTL: phase C reads its tables from LDS)
        // the five used fields only (not the 32-B struct)
        const FrameTab<real>* fp = ft + fsv[i];
        ftv[i].ca = fp->ca; ftv[i].sa = fp->sa; ftv[i].cb = fp->cb; ftv[i].sb = fp->sb; ftv[i].f = fp->f;
      }
    }
    wave_lds_fence();
    K1_NOW(kt1);
    K1_ACC(0, kt0, kt1);
    // phase B: stream the window's records (coalesced), segmented reduction into LDS.  Two register
    // groups alternate: the next group's loads are in flight while the current one is consumed.
    // (An LDS-DMA ring of 3 batches per wave, global_load_lds, was measured slower: hipcc puts a
    // vmcnt(0) -- every pending DMA -- in front of each LDS write of the reduction)
    for (int64_t rb = r0 & ~(int64_t)(RPL - 1); rb < r1; rb += 2 * RPL * WAVE) {
      load_cgrp(cb, rb + RPL * WAVE, r1);
      consume_c(ca, rb, r0, r1);
      if (rb + RPL * WAVE >= r1) break;
      load_cgrp(ca, rb + 2 * RPL * WAVE, r1);
      consume_c(cb, rb + RPL * WAVE, r0, r1);
    }
    wave_lds_fence();
    K1_NOW(kt2);
    K1_ACC(1, kt1, kt2);
    // phase C: per-segment Jacobian and normal-equation blocks
#pragma unroll
    for (int i = 0; i < SEGW / WAVE; ++i) {
      const int s = w0 + lane + i * WAVE;
      if (s >= w1) break;
      const int sl = s - w0;
      real x, y, J[2][5];
      const int fs = fsv[i];
      if (FTL && !ftl_ok) {
        ptz_project_jac<real>(ft[fs], R, u, v, x, y, J);
      } else if constexpr (FTL) {
        // the record-precision table is the rounded fp64 one (k_tables): the same values as ft[fs]
        FrameTab<real> F;
        const int fl = fs - fbase;
        F.ca = (real)s_ft[0][fl]; F.sa = (real)s_ft[1][fl]; F.cb = (real)s_ft[2][fl]; F.sb = (real)s_ft[3][fl];
        F.f = (real)s_ft[4][fl];
        F.pad0 = F.pad1 = F.pad2 = (real)0;
        ptz_project_jac<real>(F, R, u, v, x, y, J);
      } else {
        ptz_project_jac<real>(ftv[i], R, u, v, x, y, J);
      }
      const real Sx = acc0[sl], Sy = acc1[sl], Srx = acc2[sl], Sry = acc3[sl];
      // W = Jp^T diag(Sx,Sy) Jr (3x2), U = Jp^T diag Jp (upper: 00 01 02 11 12 22), g_pose = Jp^T (w r)
      real W[6];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        W[2 * p + 0] = Sx * J[0][p] * J[0][3] + Sy * J[1][p] * J[1][3];
        W[2 * p + 1] = Sx * J[0][p] * J[0][4] + Sy * J[1][p] * J[1][4];
      }
      // W into the landmark's dense frame slot: the Schur kernel's inner-loop operand and the
      // back-substitution's W
      slot_store6(w_slot + (slot0 + fs) * W_STRIDE, W);
      // U (6) | g_pose (3) into the same dense slot: summed per frame by the Schur kernel
      const real UG[9] = {Sx * J[0][0] * J[0][0] + Sy * J[1][0] * J[1][0], Sx * J[0][0] * J[0][1] + Sy * J[1][0] * J[1][1],
                          Sx * J[0][0] * J[0][2] + Sy * J[1][0] * J[1][2], Sx * J[0][1] * J[0][1] + Sy * J[1][1] * J[1][1],
                          Sx * J[0][1] * J[0][2] + Sy * J[1][1] * J[1][2], Sx * J[0][2] * J[0][2] + Sy * J[1][2] * J[1][2],
                          J[0][0] * Srx + J[1][0] * Sry, J[0][1] * Srx + J[1][1] * Sry, J[0][2] * Srx + J[1][2] * Sry};
      slot_store9(ug_slot + (slot0 + fs) * UG_STRIDE, UG);
      V00 += (double)(Sx * J[0][3] * J[0][3] + Sy * J[1][3] * J[1][3]);
      V01 += (double)(Sx * J[0][3] * J[0][4] + Sy * J[1][3] * J[1][4]);
      V11 += (double)(Sx * J[0][4] * J[0][4] + Sy * J[1][4] * J[1][4]);
      g0 += (double)(J[0][3] * Srx + J[1][3] * Sry);
      g1 += (double)(J[0][4] * Srx + J[1][4] * Sry);
    }
    wave_lds_fence();
    K1_NOW(kt3);
    K1_ACC(2, kt2, kt3);
    kt0 = kt3;
  }
  double tot[6] = {V00, V01, V11, g0, g1, cost};
  wave_total6(tot);
  V00 = tot[0]; V01 = tot[1]; V11 = tot[2]; g0 = tot[3]; g1 = tot[4]; cost = tot[5];
  if (lane == WAVE - 1) {
    double* o = (alt ? a.lm_out1 : a.lm_out) + (int64_t)l * 8;
    o[0] = V00; o[1] = V01; o[2] = V11; o[3] = g0; o[4] = g1; o[5] = 0.5 * cost; o[6] = 0; o[7] = 0;
  }
#ifdef K1_TIMING
  K1_NOW(kt4);
  K1_ACC(3, kt3, kt4);
  if (lane == 0 && task < 32768) {
    g_k1_items[task][1] = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < 4; ++k) g_k1_items[task][2 + k] = k1acc[k];
    g_k1_items[task][6] = s1 - s0;
  }
#endif
}

template <typename real>
void launch_linearize(const LinArgs& a, int loss, hipStream_t st, hipEvent_t ev0, hipEvent_t ev1) {
  if (a.n_work <= 0) return;
  dim3 grid((a.n_work + K1_WPB - 1) / K1_WPB);
  // frame tables staged in LDS per workgroup frame range (round 6: any n_pose; a workgroup whose range exceeds K1_FT_LDS
  // frames reads them from global memory -- config 4's multi-row landmarks); the global-table form stays for A/B builds
  const bool ftl = K1_FTL_ALWAYS ? true : a.n_pose <= K1_FT_LDS;
  auto go = [&](auto kern) {
    if (ev0) hipExtLaunchKernelGGL(kern, grid, dim3(64 * K1_WPB), 0, st, ev0, ev1, 0, a);
    else hipLaunchKernelGGL(kern, grid, dim3(64 * K1_WPB), 0, st, a);
  };
  const bool wt = a.rec_w != nullptr;
  if (ftl) {
    if (loss == 0) wt ? go(k_linearize<real, 0, true, true>) : go(k_linearize<real, 0, true, false>);
    else wt ? go(k_linearize<real, 1, true, true>) : go(k_linearize<real, 1, true, false>);
  } else {
    if (loss == 0) wt ? go(k_linearize<real, 0, false, true>) : go(k_linearize<real, 0, false, false>);
    else wt ? go(k_linearize<real, 1, false, true>) : go(k_linearize<real, 1, false, false>);
  }
}

// ------------------------------------------------------------------------------------------------
// landmark damping: V~ = V + lambda diag(D), D = max(D, diag V) (Marquardt scaling with the
// monotone column-norm memory of scipy's x_scale='jac', common.py:598-612); Vinv and Vinv g.
// lm_aux[l][8] = Vinv00 Vinv01 Vinv11 (Vinv g)0 (Vinv g)1 . . .
// ------------------------------------------------------------------------------------------------
// Build prologue in one launch: blocks [0, n_tiles) zero the factor pattern's tiles of S, block n_tiles the
// b | g_pose | dU vectors, the rest damp the landmark blocks as above.
__global__ __launch_bounds__(256) void k_build_prologue(double* __restrict__ S, int64_t ld, const int2* __restrict__ zt,
                                                        int n_tiles, double* __restrict__ vec, int64_t n_vec,
                                                        const double* __restrict__ lm_out,
                                                        const int32_t* __restrict__ lm_seg_begin,
                                                        double* __restrict__ D_ray, double* __restrict__ lm_aux, int n_lm,
                                                        double lambda_arg, const double* __restrict__ lam_dev,
                                                        const int* __restrict__ skip_if,
                                                        const double* __restrict__ lm_out1, const int* __restrict__ sel,
                                                        FusedPrep fp) {
  const int b = blockIdx.x;
  if (b < n_tiles) {
    const int2 tij = zt[b];
    double* T = S + (int64_t)tij.x * CHOL_NB * ld + (int64_t)tij.y * CHOL_NB;
    const bool diag_tile = fp.pad && tij.x == tij.y;
    for (int e = threadIdx.x; e < CHOL_NB * CHOL_NB / 2; e += blockDim.x) {
      const int row = e >> 4, c0 = 2 * (e & 15);
      double2 v = make_double2(0.0, 0.0);
      if (diag_tile && (row == c0 || row == c0 + 1)) {
        // single-GPU build: the constant diagonal entries of k_chol_prepare (identity on padding rows, the
        // augmented diagonal, identity below it).  The thread that zeroes the double2 holding (row, row)
        // stores the value itself, so no other thread's zero store can land after it.
        const int64_t r = (int64_t)tij.x * CHOL_NB + row;
        double dv;
        if (r < fp.n_aug) dv = fp.pad[r] ? 1.0 : 0.0;
        else dv = r == fp.n_aug ? 1e300 : 1.0;
        if (row == c0) v.x = dv; else v.y = dv;
      }
      *reinterpret_cast<double2*>(T + (int64_t)row * ld + c0) = v;
    }
    return;
  }
  if (b == n_tiles) {
    for (int64_t e = threadIdx.x; e < n_vec; e += blockDim.x) vec[e] = 0.0;
    if (fp.pad && threadIdx.x == 0) fp.info[0] = 0;
    return;
  }
  if (skip_if && *skip_if) return;
  const double lambda = lam_dev ? *lam_dev : lambda_arg;
  const int l = (b - n_tiles - 1) * blockDim.x + threadIdx.x;
  if (l >= n_lm) return;
  double* o = lm_aux + (int64_t)l * 8;
  if (lm_seg_begin[l + 1] == lm_seg_begin[l]) {
    for (int k = 0; k < 8; ++k) o[k] = 0;
    return;
  }
  const double* in = ((sel && *sel) ? lm_out1 : lm_out) + (int64_t)l * 8;
  double d0 = fmax(D_ray[2 * l], fmax(in[0], 1e-12));
  double d1 = fmax(D_ray[2 * l + 1], fmax(in[2], 1e-12));
  D_ray[2 * l] = d0;
  D_ray[2 * l + 1] = d1;
  double a = in[0] + lambda * d0, bb = in[1], c = in[2] + lambda * d1;
  double det = a * c - bb * bb;
  double i00 = 0, i01 = 0, i11 = 0;
  if (det > 0 && isfinite(det)) {
    double id = 1.0 / det;
    i00 = c * id; i01 = -bb * id; i11 = a * id;
  }
  o[0] = i00; o[1] = i01; o[2] = i11;
  o[3] = i00 * in[3] + i01 * in[4];
  o[4] = i01 * in[3] + i11 * in[4];
  o[5] = 0; o[6] = 0; o[7] = det > 0 ? 0.0 : 1.0;
}

void launch_build_prologue(double* S, int64_t ld, const int2* zt, int n_tiles, double* vec, int64_t n_vec,
                           const double* lm_out, const int32_t* lm_seg_begin, double* D_ray, double* lm_aux, int n_lm,
                           double lambda, const double* lam_dev, const int* skip_if, hipStream_t st,
                           const double* lm_out1, const int* sel, const FusedPrep& fp) {
  const unsigned nb = (unsigned)(n_tiles + 1 + (n_lm + 255) / 256);
  hipLaunchKernelGGL(k_build_prologue, dim3(nb), dim3(256), 0, st, S, ld, zt, n_tiles, vec, n_vec, lm_out, lm_seg_begin,
                     D_ray, lm_aux, n_lm, lambda, lam_dev, skip_if, lm_out1, sel, fp);
}

// (pose damping of the exchanged reduced system: k_chol_prepare, chol_kernels.hip)
// ------------------------------------------------------------------------------------------------
// K5: back-substitution of the rays + trial state + predicted-reduction partials
//   delta_l = -Vinv (g_l + sum_s W_s^T delta_p(f_s));  trial ray = ray + delta_l
//   pred_l  = -1/2 g_l.delta_l + 1/2 lambda delta_l^T D delta_l
// one wave per landmark (lanes over segments)
// ------------------------------------------------------------------------------------------------
// Trial state in one launch (with the trial's frame / ray tables, which the trial linearisation reads):
// blocks [0, nb) back-substitute 4 landmarks each as above, the last block forms the trial poses, their
// tables and the pose partials (one thread per frame, fixed-order reduction: identical on every rank).
struct PoseTrialArgs {
  const double* ptz;
  const double* g_pose;
  const double* D_pose;
  double* ptz_trial;
  double* out4;
  int n_pose;
  const uint8_t* fmask;  // part-owned solve: bit 0 pose updated here, bit 1 counted here (nullptr: all)
  const int* info;       // part-owned solve: this rank's factorisation status -> out4[4] (summed over ranks)
};
// (Round 4 tried staging the pose steps in LDS and walking a landmark's DENSE slot range instead of its segments:
// 35.9 vs 27.9 us per trial, and it sums t0 / t1 in another lane order -- not bitwise the same trial.  Removed in
// round 5.)
template <typename real>
__global__ __launch_bounds__(256) void k_trial(BacksubArgs a, PoseTrialArgs pa, FrameTab<double>* __restrict__ ft64,
                                               RayTab<double>* __restrict__ rt64, FrameTab<real>* __restrict__ ft,
                                               RayTab<real>* __restrict__ rt) {
  const int nb = (a.n_lm + 3) / 4;
  // device-driven LM: current state and trial output by the decision's slot (BacksubArgs::state_xor)
  const bool sflip = a.sel && (((*a.sel) ^ a.state_xor) & 1);
  if (sflip) {
    const double* t = pa.ptz;
    pa.ptz = pa.ptz_trial;
    pa.ptz_trial = const_cast<double*>(t);
    const double* u = a.rays;
    a.rays = a.rays_trial;
    a.rays_trial = const_cast<double*>(u);
  }
  if ((int)blockIdx.x == nb) {
    const double lambda = a.lam_dev ? *a.lam_dev : a.lambda;
    __shared__ double red[4][256 / WAVE];
    double pr = 0, dx = 0, xx = 0, gm = 0;
    for (int f = threadIdx.x; f < pa.n_pose; f += blockDim.x) {
      double x3[3];
      const int fm = pa.fmask ? pa.fmask[f] : 3;
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const double x = pa.ptz[3 * f + q];
        if (fm & 2) xx += x * x;
        double y = x;
        if (f >= a.n_fixed && (fm & 1)) {
          const int k = a.frame_pos[f] + q;  // system row
          const double d = a.dpose[k];
          y = x + d;
          if (fm & 2) {
            pr += -0.5 * pa.g_pose[k] * d + 0.5 * lambda * pa.D_pose[3 * f + q] * d * d;
            dx += d * d;
            gm = fmax(gm, fabs(pa.g_pose[k]));
          }
        }
        pa.ptz_trial[3 * f + q] = y;
        x3[q] = y;
      }
      const FrameTab<double> t = make_frame_tab<double>(x3[0], x3[1], x3[2]);
      ft64[f] = t;
      if constexpr (sizeof(real) != sizeof(double)) {
        FrameTab<real> r;
        r.ca = (real)t.ca; r.sa = (real)t.sa; r.cb = (real)t.cb; r.sb = (real)t.sb; r.f = (real)t.f;
        r.pad0 = r.pad1 = r.pad2 = (real)0;
        ft[f] = r;
      }
    }
    pr = wave_sum(pr); dx = wave_sum(dx); xx = wave_sum(xx);
    for (int o = 32; o > 0; o >>= 1) gm = fmax(gm, __shfl_xor(gm, o, WAVE));
    const int w = threadIdx.x >> 6;
    if (lane_id() == 0) { red[0][w] = pr; red[1][w] = dx; red[2][w] = xx; red[3][w] = gm; }
    __syncthreads();
    if (threadIdx.x == 0) {
      double s0 = 0, s1 = 0, s2 = 0, s3 = 0;
      for (int k = 0; k < (int)(blockDim.x / WAVE); ++k) {
        s0 += red[0][k]; s1 += red[1][k]; s2 += red[2][k]; s3 = fmax(s3, red[3][k]);
      }
      pa.out4[0] = s0; pa.out4[1] = s1; pa.out4[2] = s2; pa.out4[3] = s3;
      if (pa.info) pa.out4[4] = (double)pa.info[0];
    }
    return;
  }
  const int lane = lane_id();
  const int l = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (l >= a.n_lm) return;
  const int s0 = a.lm_seg_begin[l], s1 = a.lm_seg_begin[l + 1];
  const bool alt = a.sel && *a.sel;  // device-chosen linearisation slot
  const real* __restrict__ w_slot = (const real*)(alt ? a.w_slot1 : a.w_slot);
  const int4 lmeta = a.lm_meta[l];
  // the landmark's own operands (independent of the segment walk) requested up front: the wave's dependent
  // chain is segment list -> frame -> W slot / system row -> dpose, then the reduction and the stores
  const double* lo = (alt ? a.lm_out1 : a.lm_out) + (int64_t)l * 8;
  const double* vi = a.lm_aux + (int64_t)l * 8;
  const double g0 = lo[3], g1 = lo[4], v0 = vi[0], v1 = vi[1], v2 = vi[2];
  const double th = a.rays[2 * l], ph = a.rays[2 * l + 1];
  const double D0 = a.D_ray[2 * l], D1 = a.D_ray[2 * l + 1];
  double t0 = 0, t1 = 0;
  for (int s = s0 + lane; s < s1; s += WAVE) {
    const int f = a.seg_frame[s];
    if (f < a.n_fixed) continue;
    const double* dp = a.dpose + a.frame_pos[f];
    real w[6];
    slot_load6(w, w_slot + ((int64_t)lmeta.z + f - lmeta.x) * W_STRIDE);
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      t0 += (double)w[2 * q] * dp[q];
      t1 += (double)w[2 * q + 1] * dp[q];
    }
  }
  t0 = wave_total(t0);
  t1 = wave_total(t1);
  if (lane == WAVE - 1) {
    double* red = a.lm_red + (int64_t)l * 4;
    double nth = th, nph = ph;
    if (s1 == s0) {
      red[0] = 0; red[1] = 0; red[2] = 0; red[3] = 0;
    } else {
      const double r0 = g0 + t0, r1 = g1 + t1;
      const double d0 = -(v0 * r0 + v1 * r1);
      const double d1 = -(v1 * r0 + v2 * r1);
      nth = th + d0;
      nph = ph + d1;
      const double lam = a.lam_dev ? *a.lam_dev : a.lambda;
      red[0] = -0.5 * (g0 * d0 + g1 * d1) + 0.5 * lam * (D0 * d0 * d0 + D1 * d1 * d1);
      red[1] = d0 * d0 + d1 * d1;
      red[2] = th * th + ph * ph;
      red[3] = fmax(fabs(g0), fabs(g1));
    }
    a.rays_trial[2 * l] = nth;
    a.rays_trial[2 * l + 1] = nph;
    const RayTab<double> t = make_ray_tab<double>(nth, nph);
    rt64[l] = t;
    if constexpr (sizeof(real) != sizeof(double)) {
      RayTab<real> r;
      r.p0 = (real)t.p0; r.p1 = (real)t.p1; r.d0t = (real)t.d0t; r.d1t = (real)t.d1t; r.d1p = (real)t.d1p;
      r.pad0 = r.pad1 = r.pad2 = (real)0;
      rt[l] = r;
    }
  }
}

template <typename real>
void launch_trial(const BacksubArgs& a, const double* ptz, const double* g_pose, const double* D_pose, double* ptz_trial,
                  double* out4, int n_pose, void* ft64, void* rt64, void* ft, void* rt, hipStream_t st,
                  const uint8_t* fmask, const int* info) {
  PoseTrialArgs pa{ptz, g_pose, D_pose, ptz_trial, out4, n_pose, fmask, info};
  hipLaunchKernelGGL((k_trial<real>), dim3((unsigned)((a.n_lm + 3) / 4 + 1)), dim3(256), 0, st, a, pa,
                       (FrameTab<double>*)ft64, (RayTab<double>*)rt64, (FrameTab<real>*)ft, (RayTab<real>*)rt);
}

__device__ void lm_decide_body(LMDev* st, const double* scal, const double* __restrict__ loc,
                               const int* __restrict__ info, LMDev* __restrict__ rec, int seq, int info_in_loc);

// deterministic strided reduction: out[k] = sum_i src[i*stride + k] (fixed order), k < nk;
// mode bit k set -> max(|.|) instead of sum for column k.  RED_BLOCKS workgroups reduce contiguous row
// ranges into scratch partials; the last workgroup to finish (agent-scope counter) combines them in
// block order and re-arms the counter, so the result is bitwise reproducible in one launch.
constexpr int RED_BLOCKS = 64;
// (src2, stride2, nk2, out2): an optional second set of columns over the same n rows, reduced in the same
// launch into out2 (columns nk .. nk + nk2 - 1 of the internal accumulators; nk + nk2 <= 8)
__global__ __launch_bounds__(256) void k_reduce_cols(const double* __restrict__ src, int64_t n, int stride, int nk,
                                                     int maxmask, double* __restrict__ out,
                                                     double* __restrict__ partial, unsigned* __restrict__ counter,
                                                     const double* __restrict__ src2, int stride2, int nk2,
                                                     double* __restrict__ out2, const double* __restrict__ src1,
                                                     const int* __restrict__ sel, int sel_xor, DecideArgs dec) {
  if (sel && ((*sel ^ sel_xor) & 1)) src = src1;
  __shared__ double red[8][256 / WAVE];
  __shared__ bool last;
  const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
  const int64_t i0 = blockIdx.x * chunk, i1 = min(n, i0 + chunk);
  double acc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) acc[k] = 0;
  // every column of a row is requested before any is used (clamped column index, branch-free), so a row costs
  // one memory latency instead of one per column
  const int nkt = nk + nk2;
  for (int64_t i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int kc = min(k, nkt - 1);
      x[k] = kc < nk ? src[i * stride + kc] : src2[i * stride2 + (kc - nk)];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < nkt) acc[k] = (maxmask & (1 << k)) ? fmax(acc[k], fabs(x[k])) : acc[k] + x[k];
  }
  nk += nk2;  // from here on: all accumulated columns
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k >= nk) break;
    if (maxmask & (1 << k)) {
      for (int o = 32; o > 0; o >>= 1) acc[k] = fmax(acc[k], __shfl_xor(acc[k], o, WAVE));
    } else {
      acc[k] = wave_sum(acc[k]);
    }
  }
  const int w = threadIdx.x >> 6;
  if (lane_id() == 0)
    for (int k = 0; k < nk; ++k) red[k][w] = acc[k];
  __syncthreads();
  // the partials go out write-through (sc1 stores: L2 bypassed to memory) and the storing wave waits for them
  // before its counter add, so the add needs no agent-scope release -- which would write back every dirty line
  // of this XCD's L2 (K1 just stored ~90 MB of slots) -- and the last workgroup reads them with sc1 loads
  // (MI355X_MICROARCH.md, inter-workgroup visibility, Valid forms: one lane's agent atomic add per storing
  // workgroup, the last adder told by the returned value, stores and loads all sc1, one workgroup per CU).
  // The partial stores and the add are issued by the same wave (wave 0: nk <= 8 lanes).
  if (threadIdx.x < WAVE) {
    if (threadIdx.x < nk) {
      const int k = threadIdx.x;
      double s = 0;
      for (int j = 0; j < (int)(blockDim.x / WAVE); ++j) s = (maxmask & (1 << k)) ? fmax(s, red[k][j]) : s + red[k][j];
      __hip_atomic_store(partial + blockIdx.x * 8 + k, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (threadIdx.x == 0) {
      const unsigned done = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = (done == gridDim.x - 1);
    }
  }
  __syncthreads();
  if (!last) return;
  // reader-side acquire at agent scope (invalidates this CU's vector cache; the L2 is not written back), so the
  // partial loads below cannot be satisfied from lines older than the counter observation
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // all partials in parallel (agent-scope loads: other workgroups wrote them), then a fixed-order sum
  __shared__ double fin[RED_BLOCKS][8];
  for (int e = threadIdx.x; e < (int)gridDim.x * 8; e += blockDim.x)
    fin[e >> 3][e & 7] = __hip_atomic_load(partial + e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  __shared__ double tot[8];
  if (threadIdx.x < nk) {
    const int k = threadIdx.x;
    double s = 0;
    for (int b = 0; b < (int)gridDim.x; ++b) s = (maxmask & (1 << k)) ? fmax(s, fin[b][k]) : s + fin[b][k];
    if (k < nk - nk2) out[k] = s;
    else out2[k - (nk - nk2)] = s;
    tot[k] = s;
  }
  if (threadIdx.x == 0) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (dec.st && dec.curv) {
    // curvature mode (relin_mode 0): out = the trial's landmark part of the predicted reduction; with the pose part
    // (loc[0]) the whole predicted reduction of the trial, known before the trial point is linearised -- the trial
    // linearisation uses the floored Newton curvature from the step that is predicted to change the cost by less
    // than curvature_switch of it (k_lm_decide's relin_mode 1 rule, decided one launch earlier)
    __syncthreads();
    if (threadIdx.x == 0) {
      LMDev* st = dec.st;
      const double pred = tot[0] + dec.loc[0];
      const LMParams& p = st->p;
      st->hc_trial = (st->hc != 1.0 || pred < p.curvature_switch * st->cost) ? p.huber_curvature : 1.0;
    }
  } else if (dec.st) {
    // fused decision (trial-cost reduction of a single-GPU device-driven LM): out = scal + 1 (trial cost), out2 =
    // scal + 2 (pred, |dx|^2, |x|^2 landmark partials); the sums come from LDS, not from the stores above
    __syncthreads();
    if (threadIdx.x == 0) {
      double sc[5];
      sc[0] = 0.0;  // (the current cost lives in LMDev)
      sc[1] = tot[0]; sc[2] = tot[1]; sc[3] = tot[2]; sc[4] = tot[3];
      lm_decide_body(dec.st, sc, dec.loc, dec.info, dec.rec, dec.seq, 0);
    }
  }
}

__global__ void k_pack_scalars(const double* __restrict__ scal, const double* __restrict__ loc,
                               const int* __restrict__ info, double* __restrict__ host) {
  const int t = threadIdx.x;
  if (t < 8) host[t] = scal[t];
  else if (t < 16) host[t] = loc[t - 8];
  else if (t == 16) host[16] = (double)info[0];
}

void launch_pack_scalars(const double* scal, const double* loc, const int* info, double* host_dev, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_scalars, dim3(1), dim3(64), 0, st, scal, loc, info, host_dev);
}

void launch_reduce_cols(const double* src, int64_t n, int stride, int nk, int maxmask, double* out, double* scratch,
                        hipStream_t st, const double* src2, int stride2, int nk2, double* out2, const double* src1,
                        const int* sel, int sel_xor, const DecideArgs* decide) {
  unsigned* counter = reinterpret_cast<unsigned*>(scratch + RED_BLOCKS * 8);
  const DecideArgs dec = decide ? *decide : DecideArgs{nullptr, nullptr, nullptr, nullptr, 0, 0};
  const int nb = RED_BLOCKS;
  hipLaunchKernelGGL(k_reduce_cols, dim3(nb), dim3(256), 0, st, src, n, stride, nk, maxmask, out, scratch,
                     counter, src2, stride2, src2 ? nk2 : 0, out2, src1, sel, sel_xor, dec);
}

// ------------------------------------------------------------------------------------------------
// record-order residual (parity API for bundle_adjustment._compute_residual)
// ------------------------------------------------------------------------------------------------
template <typename real>
__global__ void k_residual(const int32_t* __restrict__ rec_seg, const int32_t* __restrict__ seg_frame,
                           const int32_t* __restrict__ seg_lm, const double2* __restrict__ seg_base,
                           const real* __restrict__ rec_xy, const int64_t* __restrict__ perm,
                           const FrameTab<double>* __restrict__ ft64, const RayTab<double>* __restrict__ rt64,
                           double u, double v, int64_t n_rec, double* __restrict__ r_out) {
  int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= n_rec) return;
  const int s = rec_seg[r];
  double x, y;
  ptz_project<double>(ft64[seg_frame[s]], rt64[seg_lm[s]], u, v, x, y);
  const double2 bs = seg_base[s];
  const real ex = (real)(x - bs.x), ey = (real)(y - bs.y);
  const int64_t o = perm[r];
  r_out[2 * o] = (double)(ex - rec_xy[2 * r]);
  r_out[2 * o + 1] = (double)(ey - rec_xy[2 * r + 1]);
}

template <typename real>
void launch_residual(const int32_t* rec_seg, const int32_t* seg_frame, const int32_t* seg_lm, const double2* seg_base,
                     const void* rec_xy, const int64_t* perm, const void* ft64, const void* rt64, double u, double v,
                     int64_t n_rec, double* r_out, hipStream_t st) {
  if (n_rec <= 0) return;
  hipLaunchKernelGGL(k_residual<real>, dim3((unsigned)((n_rec + 255) / 256)), dim3(256), 0, st, rec_seg, seg_frame,
                     seg_lm, seg_base, (const real*)rec_xy, perm, (const FrameTab<double>*)ft64,
                     (const RayTab<double>*)rt64, u, v, n_rec, r_out);
}

// ------------------------------------------------------------------------------------------------
// device-resident Levenberg-Marquardt control (the decision logic of ptzba.LMSolver, which follows
// scipy's trf acceptance / termination rules, common.py:705-718): one thread per call.
// ------------------------------------------------------------------------------------------------
__global__ void k_lm_init(LMDev* st, const double* __restrict__ scal, LMParams p, int cur0) {
  st->p = p;
  st->cur = cur0;
  st->cost = scal[0];
  st->initial_cost = scal[0];
  st->lam = p.lambda0;
  st->nu = 2.0;
  st->hc = 1.0;
  st->hc_trial = 1.0;
  st->it = 0;
  st->nfev = 1;
  st->trials = 0;
  st->retries = 0;
  st->status = 0;
  st->done = 0;
  st->accepted = 0;
  st->relin = 0;
}

// scipy trf decision rules (one thread): scal = {cost, trial cost, pred, |dx|^2, |x|^2} partial sums
__device__ void lm_decide_body(LMDev* st, const double* scal, const double* __restrict__ loc,
                               const int* __restrict__ info, LMDev* __restrict__ rec, int seq, int info_in_loc) {
  LMDev s = *st;
  s.accepted = 0;
  s.relin = 0;
  if (!s.done) {
    const LMParams& p = s.p;
    const double new_cost = scal[1], pred = scal[2] + loc[0], dx2 = scal[3] + loc[1], x2 = scal[4] + loc[2];
    const double gmax = loc[3];
    s.nfev += 1;
    s.trials += 1;
    // part-owned solve: the factorisation status summed over ranks (loc[4]), so every rank decides alike
    const bool fact_ok = info_in_loc ? loc[4] == 0.0 : info[0] == 0;
    const bool ok = fact_ok && isfinite(new_cost) && isfinite(pred);
    const double actual = s.cost - new_cost;
    const double rho = (ok && pred > 0) ? actual / pred : -1.0;
    const bool gn0 = p.gauss_newton && s.lam == 0.0;
    if (ok && (rho > 0 || (gn0 && actual >= 0))) {
      s.accepted = 1;
      s.cur ^= 1;  // the trial's linearisation (other slot) becomes current
      if (!gn0) {
        const double t = 2.0 * rho - 1.0;
        s.lam = fmax(p.min_lambda, s.lam * fmax(1.0 / 3.0, 1.0 - t * t * t));
      }
      s.nu = 2.0;
      s.retries = 0;
      s.it += 1;
      const double old = s.cost;
      s.cost = new_cost;
      s.last_actual = actual;
      s.last_rho = rho;
      if (actual < p.ftol * old && rho > 0.25) {
        s.status = 2;
        s.done = 1;
      } else if (sqrt(dx2) < p.xtol * (p.xtol + sqrt(x2))) {
        s.status = 3;
        s.done = 1;
      } else if (p.gtol > 0 && gmax < p.gtol) {
        s.status = 1;
        s.done = 1;
      } else if (s.it >= p.max_iter) {
        s.status = 0;
        s.done = 1;
      } else if (p.relin_mode && s.hc == 1.0 && p.curvature_switch > 0 && pred < p.curvature_switch * old) {
        // in the final basin (the step was predicted to change the cost by < curvature_switch of it): the residuals
        // move little against the huber scale, so the loss's own (floored Newton) curvature replaces IRLS's
        // majoriser from the current point on, which the next build re-linearises first (LMSolver._run_host: the
        // same rule).  relin_mode 0 reaches the same linearisations without the re-linearisation: see hc_trial
        s.hc = p.huber_curvature;
        s.relin = 1;
      }
      if (!p.relin_mode) s.hc = s.hc_trial;  // the accepted trial's linearisation is the current one
    } else {
      s.lam = s.lam > 0 ? fmax(s.lam * s.nu, 1e-9) : 1e-9;
      s.nu *= 2.0;
      s.retries += 1;
      if (s.lam > p.max_lambda) {
        // no decrease at any damping up to max_lambda: the step is below the cost's resolution (scipy's trf
        // ends such a run through xtol once its radius collapses); its own status, not "max iterations"
        s.status = PTZBA_STATUS_DAMPING;
        s.done = 1;
      } else if (s.retries >= p.max_retries) {
        s.status = -1;
        s.done = 1;
      }  // rejected: the current linearisation is intact in its slot (the trial wrote the other one)
    }
  }
  *st = s;
  s.seq = 0;
  *rec = s;
  // the host polls rec->seq (pinned memory): the record's fields must be visible before it
  __threadfence_system();
  __hip_atomic_store(&rec->seq, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__global__ void k_lm_decide(LMDev* st, const double* __restrict__ scal, const double* __restrict__ loc,
                            const int* __restrict__ info, LMDev* __restrict__ rec, int seq, int info_in_loc) {
  lm_decide_body(st, scal, loc, info, rec, seq, info_in_loc);
}

// accepted trial -> current state (the trial's linearisation is already in place)
__global__ void k_lm_commit(const LMDev* __restrict__ st, double* __restrict__ ptz, const double* __restrict__ ptz_trial,
                            int n3, double* __restrict__ rays, const double* __restrict__ rays_trial, int64_t n2) {
  if (!st->accepted) return;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n3 + n2; i += (int64_t)gridDim.x * blockDim.x) {
    if (i < n3) ptz[i] = ptz_trial[i];
    else rays[i - n3] = rays_trial[i - n3];
  }
}

void launch_lm_init(LMDev* st, const double* scal, const LMParams& p, int cur0, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_init, dim3(1), dim3(1), 0, s, st, scal, p, cur0);
}
void launch_lm_decide(LMDev* st, const double* scal, const double* loc, const int* info, LMDev* rec, int seq,
                      hipStream_t s, int info_in_loc) {
  hipLaunchKernelGGL(k_lm_decide, dim3(1), dim3(1), 0, s, st, scal, loc, info, rec, seq, info_in_loc);
}
void launch_lm_commit(const LMDev* st, double* ptz, const double* ptz_trial, int n3, double* rays,
                      const double* rays_trial, int64_t n2, hipStream_t s) {
  hipLaunchKernelGGL(k_lm_commit, dim3(64), dim3(256), 0, s, st, ptz, ptz_trial, n3, rays, rays_trial, n2);
}

// explicit instantiations
template void launch_tables<float>(const double*, const double*, int, int, void*, void*, void*, void*, const int*,
                                   hipStream_t, double*, int);
template void launch_tables<double>(const double*, const double*, int, int, void*, void*, void*, void*, const int*,
                                    hipStream_t, double*, int);
template void launch_linearize<float>(const LinArgs&, int, hipStream_t, hipEvent_t, hipEvent_t);
template void launch_linearize<double>(const LinArgs&, int, hipStream_t, hipEvent_t, hipEvent_t);
template void launch_trial<float>(const BacksubArgs&, const double*, const double*, const double*, double*, double*, int,
                                  void*, void*, void*, void*, hipStream_t, const uint8_t*, const int*);
template void launch_trial<double>(const BacksubArgs&, const double*, const double*, const double*, double*, double*,
                                   int, void*, void*, void*, void*, hipStream_t, const uint8_t*, const int*);
template void launch_residual<float>(const int32_t*, const int32_t*, const int32_t*, const double2*, const void*,
                                     const int64_t*, const void*, const void*, double, double, int64_t, double*,
                                     hipStream_t);
template void launch_residual<double>(const int32_t*, const int32_t*, const int32_t*, const double2*, const void*,
                                      const int64_t*, const void*, const void*, double, double, int64_t, double*,
                                      hipStream_t);

}  // namespace ptzba

#ifdef K1_TIMING
// the first n tasks' records of the last launch: [start, end (s_memrealtime, 100 MHz), cycles in phase A
// (incl. the descriptor), B, C, final, segments, -]
extern "C" int ptzba_debug_k1(long long* items, int n) {
  if (hipMemcpyFromSymbol(items, HIP_SYMBOL(ptzba::g_k1_items), (size_t)(n < 32768 ? n : 32768) * 64) != hipSuccess)
    return -1;
  return 0;
}
#endif
