// lompc_plan.hip — the PATH engine: a fixed EV batch (one price loop / one time step) solved
// at new prices by ONE fused kernel per price iteration plus a per-set reduction.
//
// Hot path replaced: LoMPC.solve_lompc (chargingstation/lompc.py:137-156) called once per EV
// from PriceSolver._get_w_err (price_solver.py:203-209) and PriceSolver.get_w0_price0
// (price_solver.py:280-283).  Within one parameter set (an (EV type, partition) price vector)
// every EV solves the same QP except gamma_i = y_max - y0_i (price_solver.py:202, :281), so
// w*(gamma) is a continuous piecewise-affine path.
//
// Plan (once per batch, lompc_plan_create): each set's gamma window [lo, hi] is cut into G
// cells; every EV is keyed by (set, cell) — cell G of a set collects invalid gamma — and the
// keys are radix-sorted (stable, rocPRIM) so each cell's EVs are contiguous: perm[j] is the
// caller index of sorted position j, gs[j] its gamma.
//
// Run (every price iteration, lompc_plan_run):
//   k_solve   one 64-lane wave per (set, cell), lane t = horizon stage t:
//             (1) exact solve at the cell start (wave-parallel PDAS, KKT-certified),
//             (2) parametric active-set tracking of w*(gamma) across the cell: pieces
//                 w = a + b gamma, each KKT-certified at its end (the residual is convex along
//                 an affine piece, so both ends certify the whole piece), kept in LDS with the
//                 cost / squared A_bar error as quadratics in gamma,
//             (3) the cell's EVs: lane = EV for the scalar outputs (cost, w0, status, price0,
//                 A_bar error) and the per-piece moments (count, sum gamma); lane = stage for
//                 the w rows (16-B write-through stores to the caller's row perm[j]); EVs no
//                 certified piece covers are re-solved individually by the whole wave,
//             (4) the cell's partial reduction record (sum w from the piece moments).
//   k_reduce  one workgroup per set: deterministic sum / max of its cells' records.
// No path table, no dependent kernel between the path and the per-EV outputs.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <rocprim/device/device_radix_sort.hpp>

#include "lompc_ctx.hpp"
#include "lompc_wave.hpp"

#ifdef LOMPC_STAMPS
// diagnostic build only (scripts/kstamps.py): per-wave s_memtime at k_solve's phase boundaries
__device__ long long g_stamps[65536 * 8];
#define LQ_STAMP(k)                                                                         \
  do {                                                                                      \
    const long long t__ = __builtin_amdgcn_s_memtime();                                     \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_stamps[blockIdx.x * 8 + (k)] = t__;      \
  } while (0)
#else
#define LQ_STAMP(k)
#endif

namespace {

typedef unsigned int lq_v4u __attribute__((ext_vector_type(4)));
typedef unsigned int lq_v2u __attribute__((ext_vector_type(2)));

// write-through (sc1) stores: the outputs leave no dirty lines in the XCD's L2, so the kernel
// boundary behind k_solve has no L2 writeback to wait for (MI355X_MICROARCH.md, price list)
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t rs, int off, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lq_v4u, make_double2(x, y)), rs, off, 0, 16);
}
__device__ __forceinline__ void st_wt8b(__amdgpu_buffer_rsrc_t rs, int off, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(lq_v2u, x), rs, off, 0, 16);
}
__device__ __forceinline__ void st_wt8(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double clampw(double x, double wmax) { return fmin(fmax(x, 0.0), wmax); }

struct PlanArgs {
  int S, G, nbk, pad;
  int64_t B;
  const QPConst* qd;
  const uint8_t* set_ctx;
  const int64_t* set_off;
  double* window;
  const double* gamma;
  uint32_t* keys;
  uint32_t* vals;
  uint32_t* keys_out;
  uint32_t* vals_out;
  int* bucket_off;
  double* gs;
};

// ---------------------------------------------------------------- plan kernels
// per set: [lo, hi] = range of its valid gamma, widened by 1e-7 y_max (a zero-width set still
// gets cells of positive width), clipped to [0, y_max]; no valid EV -> [0, y_max]
__global__ __launch_bounds__(256) void k_plan_window(PlanArgs a) {
  __shared__ double smin[256], smax[256];
  const int s = blockIdx.x;
  const QPConst& q = a.qd[a.set_ctx[s]];
  const double ym = q.y_max;
  double lo = INFINITY, hi = -INFINITY;
  for (int64_t i = a.set_off[s] + threadIdx.x; i < a.set_off[s + 1]; i += 256) {
    const double g = a.gamma[i];
    if (g >= 0.0 && g <= ym) {
      lo = fmin(lo, g);
      hi = fmax(hi, g);
    }
  }
  smin[threadIdx.x] = lo;
  smax[threadIdx.x] = hi;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if ((int)threadIdx.x < k) {
      smin[threadIdx.x] = fmin(smin[threadIdx.x], smin[threadIdx.x + k]);
      smax[threadIdx.x] = fmax(smax[threadIdx.x], smax[threadIdx.x + k]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double mg = 1e-7 * ym;
    double wlo = 0.0, whi = ym;
    if (smin[0] <= smax[0]) {
      wlo = fmin(fmax(smin[0] - mg, 0.0), ym);
      whi = fmin(fmax(smax[0] + mg, wlo + mg), ym);
      if (!(whi > wlo)) {
        wlo = fmax(whi - 2.0 * mg, 0.0);
      }
    }
    a.window[2 * s] = wlo;
    a.window[2 * s + 1] = whi;
  }
}

__device__ __forceinline__ int set_of(const int64_t* off, int S, int64_t i) {  // off[s] <= i < off[s+1]
  int lo = 0, hi = S - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= i) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// cell of gamma in set s (the same arithmetic as k_solve's cell bounds; G = invalid)
__device__ __forceinline__ int cell_of(double g, double ym, double lo, double hi, int G) {
  if (!(g >= 0.0 && g <= ym)) return G;
  const double x = (g - lo) * ((double)G / (hi - lo));
  return x <= 0.0 ? 0 : (x >= (double)(G - 1) ? G - 1 : (int)x);
}

__global__ __launch_bounds__(256) void k_plan_keys(PlanArgs a) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.B) return;
  const int s = set_of(a.set_off, a.S, i);
  const double ym = a.qd[a.set_ctx[s]].y_max;
  const int c = cell_of(a.gamma[i], ym, a.window[2 * s], a.window[2 * s + 1], a.G);
  a.keys[i] = (uint32_t)s * (uint32_t)(a.G + 1) + (uint32_t)c;
  a.vals[i] = (uint32_t)i;
}

// bucket offsets from the sorted keys (every bucket's start written exactly once) and the
// gamma of each sorted position
__global__ __launch_bounds__(256) void k_plan_finish(PlanArgs a) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= a.B) return;
  const int64_t kj = a.keys_out[j];
  const int64_t kp = j ? (int64_t)a.keys_out[j - 1] : -1;
  for (int64_t k = kp + 1; k <= kj; ++k) a.bucket_off[k] = (int)j;
  if (j == a.B - 1)
    for (int64_t k = kj + 1; k <= a.nbk; ++k) a.bucket_off[k] = (int)a.B;
  a.gs[j] = a.gamma[a.vals_out[j]];
}

// ---------------------------------------------------------------- k_solve
// k_solve<SOLVE_WAVES, SOLVE_PATHS>: SOLVE_WAVES waves per (set, cell) workgroup all evaluate the
// cell's EVs; the first SOLVE_PATHS of them compute the path of one sub-cell each
#ifndef LQ_SOLVE_WAVES
#define LQ_SOLVE_WAVES 2
#endif
#ifndef LQ_SOLVE_PATHS
#define LQ_SOLVE_PATHS 1
#endif
#define LQ_PPLX 8  // max certified pieces per sub-cell
#define LQ_WS_MAX 8  // warm-start buffer: working sets per cell

struct SolveArgs {
  int S, G, flags, want_err, N, pad;
  int64_t B;
  const QPConst* qd;
  const uint8_t* set_ctx;
  const double* window;
  const int* bucket_off;
  const double* gs;
  const uint32_t* perm;
  const double* lmbd;    // [S][3N]
  const double* lmbd_r;  // [S]
  const double* w_ref;   // [S][N] or null
  uint8_t* ws;           // [nbk][64] warm-start working sets or null
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* partial;       // [nbk][N + NPX]
  int* errflag;
  int w_rsrc_ok;         // B*N*8 fits a buffer descriptor's 31-bit offsets
  // per-set reduction by the set's last-arriving workgroup (null arrive: k_reduce does it)
  unsigned* arrive;      // [S] arrival counters, 0 between launches
  const int64_t* set_off;
  double* set_sum_w;
  double* set_stats;
  double* stats;
};

struct SetData {  // per-set scalars every lane holds (uniform)
  double c0, kappa, l10, l20, l30, lr;
};

// cost / A_bar error / price0 of a QP solved by the whole wave (lane t = w_t), valid on every lane
__device__ __forceinline__ void wave_ev_outputs(const QPConst& q, const lqw::WaveSet& ws, const SetData& sd,
                                                double wr, double gamma, double w, double& cost, double& err,
                                                double& price0) {
  const int N = ws.N, lane = ws.lane;
  const bool act = lane < N;
  lqw::Aff<2> h = lqw::Aff<2>::identity();
  if (act) {
    h.B[0] = w;
    h.B[1] = w - wr;
  }
  const lqw::Aff<2> Y = lqw::wave_scan(h, N);
  double t[3] = {0.0, 0.0, 0.0};
  double pwl = 0.0;
  if (act) {
    const double y = Y.B[0], ey = Y.B[1];
    t[0] = 0.5 * q.c * y * y - q.c * gamma * y + w * fma(0.5 * ws.d_nat, w, ws.e_nat);
    if (!q.ev_small) pwl = lq_pwl(w * q.inv_wmax);
    t[1] = ey * ey;
    t[2] = (w - wr) * (w - wr);
  }
  const double tw = q.theta * q.w_max;
  double v[4] = {t[0], t[1], t[2], q.ev_small ? 0.0 : pwl};
  lqw::wave_totals(v, N);
  cost = v[0] + sd.c0 + tw * tw * v[3];
  err = sqrt(fmax(v[1] + sd.kappa * v[2], 0.0));
  const double w0 = __shfl(w, 0, 64);
  price0 = q.theta * (w0 * sd.l10 + (q.w_max - w0) * sd.l20) + q.q_scale * w0 * w0 * sd.l30 +
           q.theta * q.theta * w0 * w0 * sd.lr;
}

__device__ __forceinline__ double ld_wt8(const double* p) {  // global_load ... sc1 (L2-served, not L1)
  return __builtin_bit_cast(double, __hip_atomic_load(reinterpret_cast<const unsigned long long*>(p),
                                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Called by ONE wave per workgroup after it wrote the workgroup's record write-through (sc1).
// Hand-off of the G+1 cell records of set s to the set's last-arriving workgroup
// (MI355X_MICROARCH.md, "Valid forms": sc1 stores drained by s_waitcnt vmcnt(0) before one
// agent-scope add per workgroup; the adder that sees G + 1 arrivals reads every record with sc1
// loads after its add returned): sum / max in a fixed order -> set_sum_w, set_stats.
__device__ __forceinline__ void arrive_reduce(const SolveArgs& a, int s, int lane, int N) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned old = 0;
  if (lane == 0) old = __hip_atomic_fetch_add(a.arrive + s, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = (unsigned)__shfl((int)old, 0, 64);
  if (old != (unsigned)a.G) return;  // G + 1 workgroups per set; the last one reduces
  const int W = N + NPX, G1 = a.G + 1;
  const double* base = a.partial + (size_t)s * G1 * W;
  double col[2] = {0.0, 0.0};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = lane + 64 * h;
    if (c < W) {
      const bool is_max = c == N + PX_MAX_ERR;
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      constexpr int U = 32;  // all records of a set in one or two memory rounds
      for (int b = 0; b < G1; b += U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = b + u < G1 ? ld_wt8(base + (size_t)(b + u) * W + c) : 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u & 3] = is_max ? fmax(acc[u & 3], v[u]) : acc[u & 3] + v[u];
      }
      col[h] = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
    }
  }
  if (lane < N && a.set_sum_w) a.set_sum_w[(size_t)s * N + lane] = col[0];
  // stats row: lane t < 8 takes its column's total
  int src = 0;
  switch (lane) {
    case LOMPC_STAT_SUM_W0: src = 0; break;
    case LOMPC_STAT_SUM_PRICE0: src = N + PX_PRICE0; break;
    case LOMPC_STAT_MAX_ERR: src = N + PX_MAX_ERR; break;
    case LOMPC_STAT_SUM_COST: src = N + PX_COST; break;
    case LOMPC_STAT_N_REPAIRED: src = N + PX_N_REPAIRED; break;
    case LOMPC_STAT_N_FAILED: src = N + PX_N_FAILED; break;
    case LOMPC_STAT_N_INVALID: src = N + PX_N_INVALID; break;
    default: src = 0; break;
  }
  const double v0 = __shfl(col[0], src & 63, 64), v1 = __shfl(col[1], src & 63, 64);
  double v = src < 64 ? v0 : v1;
  if (lane == LOMPC_STAT_COUNT) v = (double)(a.set_off[s + 1] - a.set_off[s]);
  if (lane < LOMPC_SET_STATS) {
    if (a.set_stats) a.set_stats[(size_t)s * LOMPC_SET_STATS + lane] = v;
    a.stats[(size_t)s * LOMPC_SET_STATS + lane] = v;
  }
  if (lane == 0) __hip_atomic_store(a.arrive + s, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One workgroup of SOLVE_WAVES waves per (set, gamma cell).  The cell is split into
// SOLVE_PATHS sub-cells: waves 0..SOLVE_PATHS-1 (one per SIMD) each compute one sub-cell's
// certified path pieces into LDS (latency-bound wave-parallel scans; the other waves wait at the
// barrier and cost no issue slots), then all waves split the cell's EVs in 64-EV chunks.
template <int SOLVE_WAVES, int SOLVE_PATHS>
__global__ __launch_bounds__(64 * SOLVE_WAVES) void k_solve(SolveArgs a) {
  constexpr int NSLOT = SOLVE_PATHS * LQ_PPLX;  // piece slots: sub-cell k owns [k PPL, (k+1) PPL)
  __shared__ double2 s_ab[NSLOT][64];                              // piece rows (a_t, b_t), lane t
  __shared__ __attribute__((aligned(16))) double s_cf[NSLOT][8];  // K0 K1 K2 (cost) F0 F1 F2 (err^2) a_0 b_0
  __shared__ double s_ge[NSLOT];                                   // gamma at each piece's end
  __shared__ double s_g[SOLVE_WAVES][64];                          // chunk: gamma, piece slot (-1 re-solved,
  __shared__ int s_p[SOLVE_WAVES][64];                             //   -2 invalid), caller row
  __shared__ int s_o[SOLVE_WAVES][64];
  __shared__ double s_mom[SOLVE_WAVES][NSLOT][2];                  // per wave and piece: count, sum gamma
  __shared__ double s_red[SOLVE_WAVES][8];                         // per wave: cost, price0, max err, counts
  __shared__ double s_repw[SOLVE_WAVES][64];                       // per wave: sum of re-solved rows (lane t)
  __shared__ double s_cov[SOLVE_PATHS][2];                         // sub-cell coverage [glo, gcov]
  __shared__ int s_npc[SOLVE_PATHS];
  __shared__ uint8_t s_sl0[SOLVE_PATHS][64];                       // working set at each sub-cell start
  const int blk = (int)blockIdx.x;
  const int G = a.G, G1 = a.G + 1;
  const int s = blk / G1;
  const int cell = blk - s * G1;
  const int lane = (int)threadIdx.x & 63, wv = (int)threadIdx.x >> 6;
  const int N = a.N;  // every context of a plan has the same horizon
  const int W = N + NPX;
  const int b0 = a.bucket_off[blk], b1 = a.bucket_off[blk + 1];
  // the first chunk of this wave: issued before anything waits on memory
  const int j0 = b0 + 64 * wv + lane;
  const double g_pre = j0 < b1 ? a.gs[j0] : 0.0;
  const int o_pre = j0 < b1 ? (int)a.perm[j0] : 0;
  const QPConst& q = a.qd[a.set_ctx[s]];  // uniform: scalar loads, no register copy
  LQ_STAMP(0);
  lq_tab_init(q);
  double* part = a.partial + (size_t)blk * W;
  if (b1 <= b0) {  // empty cell (workgroup-uniform)
    if (wv == 0) {
      for (int c = lane; c < W; c += 64) st_wt8(part + c, 0.0);
      if (a.arrive) arrive_reduce(a, s, lane, N);
    }
    return;
  }
  const double tt = q.theta * q.theta;
  // ---- per-set data (lompc.py:92-135 in standard form); every wave holds it
  const double* __restrict__ L = a.lmbd + (size_t)s * 3 * N;
  const double lr = a.lmbd_r[s];
  lqw::WaveSet ws;
  ws.N = N;
  ws.lane = lane;
  ws.rsrc = lane < N ? N - 1 - lane : lane;
  double l2 = 0.0;
  if (lane < N) {
    const double l1 = L[lane], l3 = L[2 * N + lane];
    l2 = L[N + lane];
    if (wv == 0 && !(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0)) atomicOr(a.errflag, 1);
    ws.d_nat = 2.0 * lr * tt + 2.0 * q.q_scale * l3 + q.dsmall;
    ws.e_nat = q.theta * (l1 - l2);
    const int tr = ws.rsrc;
    ws.d_rev = 2.0 * lr * tt + 2.0 * q.q_scale * L[2 * N + tr] + q.dsmall;
    ws.e_rev = q.theta * (L[tr] - L[N + tr]);
  } else {
    ws.d_nat = ws.e_nat = ws.d_rev = ws.e_rev = 0.0;
  }
  if (wv == 0 && lane == 0 && !(lr >= 0.0)) atomicOr(a.errflag, 1);
  const double wr_nat = (a.w_ref && lane < N) ? a.w_ref[(size_t)s * N + lane] : 0.0;
  SetData sd;
  sd.c0 = q.theta * q.w_max * lqw::wave_sum(l2, N);  // lompc.py:128
  sd.kappa = lr / q.delta;                            // price_solver.py:191
  sd.l10 = L[0];
  sd.l20 = L[N];
  sd.l30 = L[2 * N];
  sd.lr = lr;
  const int want_err = a.want_err;
  const bool invalid_cell = cell == G;
  // the cell [clo, chi] of the set's window and its SOLVE_PATHS sub-cells
  const double wlo = a.window[2 * s], whi = a.window[2 * s + 1];
  const double h = (whi - wlo) / (double)G;
  const double clo = cell == 0 ? wlo : fma((double)cell, h, wlo);
  const double chi = cell >= G - 1 ? whi : fma((double)(cell + 1), h, wlo);
  const double hs = (chi - clo) / (double)SOLVE_PATHS;
  LQ_STAMP(1);
  // ---- waves 0..SOLVE_PATHS-1: sub-cell wv's path pieces
  if (wv < SOLVE_PATHS) {
    const int k = wv;
    int npc = 0;
    double glo = 0.0, gcov = -INFINITY;  // certified coverage [glo, gcov]
    int sl0 = lane < N ? 1 : 0;
    if (!invalid_cell && !(a.flags & LOMPC_PLAN_DIAG_REPAIR)) {
      const double mg = 1e-13 * q.y_max;  // sub-cells overlap by a rounding margin
      glo = fmax((k == 0 ? clo : fma((double)k, hs, clo)) - mg, 0.0);
      const double ghi = fmin((k == SOLVE_PATHS - 1 ? chi : fma((double)(k + 1), hs, clo)) + mg, q.y_max);
      double Ywr;
      {
        lqw::Sums<1> y;
        y.v[0] = wr_nat;
        Ywr = lqw::wave_scan(y, N).v[0];
      }
      const size_t wso = ((size_t)blk * LQ_WS_MAX + k) * 64 + lane;
      int sl = sl0;
      if (a.ws) {
        const int v = a.ws[wso];
        sl = (lane < N && v >= 0 && v <= 2 * q.m) ? v : sl0;
      }
      double w = 0.0, r = 0.0;
      const bool solved = lqw::wave_solve(q, ws, glo, sl, w, r);
      LQ_STAMP(2);
      if (solved) {
        sl0 = sl;
        if (a.ws) a.ws[wso] = (uint8_t)sl;
        // ---- parametric active-set tracking of w*(gamma) on [glo, ghi]
        double gcur = glo;
        int last = -1;
        const int max_iter = 4 * LQ_PPLX + 16;
        const double ee = ws.e_nat;
        for (int it = 0; it < max_iter && npc < LQ_PPLX; ++it) {
          const lqw::StageSol<2> sol = lqw::solve_stage<2>(q, ws, 0.0, sl);
          const double av = sol.w[0], bv = sol.w[1], r0 = sol.r[0], r1 = sol.r[1];
          double gc = INFINITY;
          int ns = sl;
          if (lane < N) {
            const Box bx = lq_box(sl);
            if (sl & 1) {  // free: w(gamma) = a + b gamma leaves [lo, hi]
              if (bv > 0.0) { gc = (bx.hi - av) / bv; ns = sl + 1; }
              else if (bv < 0.0) { gc = (bx.lo - av) / bv; ns = sl - 1; }
            } else {       // fixed: v(gamma) = -r0 - r1 gamma leaves [slo, shi]
              if (r1 < 0.0) { gc = -(bx.shi + r0) / r1; ns = sl + 1; }
              else if (r1 > 0.0) { gc = -(bx.slo + r0) / r1; ns = sl - 1; }
            }
            if (!(gc == gc)) gc = INFINITY;  // NaN guard
            if (lane == last && gc <= gcur) gc = INFINITY;
            gc = fmax(gc, gcur);
          }
          double best = gc;
          int bj = lane;
          lqw::wave_argmin(best, bj, N);
          if (!(best < ghi)) {
            best = ghi;
            bj = -1;
          }
          const bool final_piece = (bj < 0) || (npc == LQ_PPLX - 1);
          if (best > gcur || final_piece) {
            // KKT certificate at the piece's end; its start is the previous certified end (same
            // w and r, only the switched coordinate's box changed and it contains the value)
            const Box bx = lq_box(lane < N ? sl : 0);
            const double wz = fmin(fmax(fma(bv, best, av), bx.lo), bx.hi);
            const double res = lqw::wave_kkt_point(q, ws, best, sl, wz);
            if (!(res <= q.tol_cert)) break;  // coverage ends at gcur
            // cost and err^2 are quadratics in gamma on the piece
            const bool act = lane < N;
            lqw::Sums<2> pf;
            pf.v[0] = act ? av : 0.0;
            pf.v[1] = act ? bv : 0.0;
            pf = lqw::wave_scan(pf, N);
            const double Ya = pf.v[0], Yb = pf.v[1];
            const double Ea = Ya - Ywr, da = av - wr_nat;
            const double dd = ws.d_nat, cc = q.c;
            const double sg = (sl & 1) ? bx.slo : 0.0;  // PWL slope of a free coordinate
            double icpt = 0.0;                          // PWL value at w = 0 of its linear piece
            if (!q.ev_small) {
              const double wm = fma(bv, 0.5 * (gcur + best), av);
              const double tw = q.theta * q.w_max;
              icpt = fma(-sg, wm, tw * tw * lq_pwl(wm * q.inv_wmax));
            }
            double t[6];
            t[0] = fma(0.5 * cc, Ya * Ya, fma(av, fma(0.5 * dd, av, ee + sg), icpt));
            t[1] = fma(cc, fma(Ya, Yb, -Ya), bv * fma(dd, av, ee + sg));
            t[2] = fma(0.5 * cc, Yb * Yb, fma(-cc, Yb, 0.5 * dd * bv * bv));
            t[3] = fma(Ea, Ea, sd.kappa * da * da);
            t[4] = 2.0 * fma(Ea, Yb, sd.kappa * da * bv);
            t[5] = fma(Yb, Yb, sd.kappa * bv * bv);
#pragma unroll
            for (int kk = 0; kk < 6; ++kk) t[kk] = act ? t[kk] : 0.0;
            lqw::wave_totals(t, N);
            const int slot = k * LQ_PPLX + npc;
            s_ab[slot][lane] = make_double2(act ? av : 0.0, act ? bv : 0.0);
            const double a0 = __shfl(av, 0, 64), b0v = __shfl(bv, 0, 64);
            if (lane < 8) {
              double v = t[0] + sd.c0;
#pragma unroll
              for (int kk = 1; kk < 6; ++kk) v = lane == kk ? t[kk] : v;
              v = lane == 6 ? a0 : (lane == 7 ? b0v : v);
              s_cf[slot][lane] = v;
            }
            if (lane == 0) s_ge[slot] = best;
            gcov = best;
            ++npc;
          }
          if (bj < 0) break;
          const int bns = __shfl(ns, bj, 64);
          if (lane == bj) sl = bns;
          gcur = best;
          last = bj;
        }
      }
    }
    s_sl0[k][lane] = (uint8_t)sl0;
    if (lane == 0) {
      s_npc[k] = npc;
      s_cov[k][0] = glo;
      s_cov[k][1] = gcov;
    }
  }
  __syncthreads();  // pieces published to every wave (no global stores outstanding here)
  LQ_STAMP(3);
  // ---- the cell's EVs: wave wv takes chunks wv, wv + SOLVE_WAVES, ...
  double acc_cost = 0.0, acc_p0 = 0.0, acc_err = 0.0;
  int n_ok = 0, n_rep = 0, n_fail = 0, n_inv = 0;
  double rep_w = 0.0;  // lane = stage: sum of individually re-solved rows
  if (lane < NSLOT) {
    s_mom[wv][lane][0] = 0.0;
    s_mom[wv][lane][1] = 0.0;
  }
  const int V = (N & 1) ? 1 : 2;  // stages per lane in the row stores (16-B stores for even N)
  const int Lr = N / V;           // lanes per row
  const int R = 64 / Lr;          // rows per store instruction
  const int rr = lane / Lr, col = lane - rr * Lr;
  const bool rlane = rr < R;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(a.w, (short)0, 0x7fffffff, 0x00020000);
  const double wm = q.w_max;
  const double ksc = (double)SOLVE_PATHS / (chi - clo);
  for (int i0 = b0 + 64 * wv; i0 < b1; i0 += 64 * SOLVE_WAVES) {
    const int j = i0 + lane;
    const bool act = j < b1;
    const bool first = i0 == b0 + 64 * wv;
    const double g = first ? g_pre : (act ? a.gs[j] : 0.0);
    const int o = first ? o_pre : (act ? (int)a.perm[j] : 0);
    // sub-cell, then piece within it (s_ge of a sub-cell ascends)
    const double kf = (g - clo) * ksc;
    const int k = kf <= 0.0 ? 0 : (kf >= (double)(SOLVE_PATHS - 1) ? SOLVE_PATHS - 1 : (int)kf);
    const int npk = s_npc[k];
    int p = 0;
    for (int pp = 0; pp < LQ_PPLX - 1; ++pp) p += (pp < npk - 1 && g > s_ge[k * LQ_PPLX + pp]) ? 1 : 0;
    const int slot = k * LQ_PPLX + p;
    const bool cov = act && !invalid_cell && npk > 0 && g >= s_cov[k][0] && g <= s_cov[k][1];
    int tag = -1;
    if (act && invalid_cell) {
      tag = -2;
      ++n_inv;
      if (a.cost) st_wt8(a.cost + o, NAN);
      if (a.w0) st_wt8(a.w0 + o, NAN);
      if (a.status) a.status[o] = LOMPC_QP_INVALID;
    } else if (cov) {
      tag = slot;
      const double4 c0 = *reinterpret_cast<const double4*>(&s_cf[slot][0]);
      const double4 c1 = *reinterpret_cast<const double4*>(&s_cf[slot][4]);
      const double cst = fma(fma(c0.z, g, c0.y), g, c0.x);
      const double e2 = fma(fma(c1.y, g, c1.x), g, c0.w);
      const double er = want_err ? sqrt(fmax(e2, 0.0)) : 0.0;
      const double w0v = clampw(fma(c1.w, g, c1.z), wm);
      const double p0 = q.theta * (w0v * sd.l10 + (wm - w0v) * sd.l20) + q.q_scale * w0v * w0v * sd.l30 +
                        tt * w0v * w0v * sd.lr;  // lompc.py:164-170
      acc_cost += cst;
      acc_p0 += p0;
      acc_err = fmax(acc_err, er);
      ++n_ok;
      if (a.cost) st_wt8(a.cost + o, cst);
      if (a.w0) st_wt8(a.w0 + o, w0v);
      if (a.status) a.status[o] = LOMPC_QP_OK;
    }
    // per-piece moments of the covered EVs (sum w = sum over pieces of count a + b sum gamma):
    // one masked wave total per distinct piece in the chunk, in lane order (deterministic)
    unsigned long long rem = __ballot(cov);
    while (rem) {
      const int key = __builtin_amdgcn_readlane(tag, (int)__builtin_ctzll(rem));
      const bool m = cov && tag == key;
      rem &= ~__ballot(m);
      double v[2] = {m ? 1.0 : 0.0, m ? g : 0.0};
      lqw::wave_totals(v, 64);
      if (lane == 0) {
        s_mom[wv][key][0] += v[0];
        s_mom[wv][key][1] += v[1];
      }
    }
    s_g[wv][lane] = g;
    s_p[wv][lane] = tag;
    s_o[wv][lane] = o;
    // ---- EVs no certified piece covers: whole-wave certified re-solve, row written here
    unsigned long long need = __ballot(act && !invalid_cell && !cov);
    while (need) {
      const int l = (int)__builtin_ctzll(need);
      need &= need - 1ull;
      const double gl = lqw::readlane_d(g, l);
      const int ol = __builtin_amdgcn_readlane(o, l);
      const int kl = __builtin_amdgcn_readlane(k, l);
      int sl = lane < N ? (int)s_sl0[kl][lane] : 0;
      double wl = 0.0, rl = 0.0;
      const bool okk = lqw::wave_solve(q, ws, gl, sl, wl, rl);
      double cl, el, pl;
      wave_ev_outputs(q, ws, sd, wr_nat, gl, wl, cl, el, pl);
      if (!want_err) el = 0.0;
      if (a.w && lane < N) st_wt8(a.w + (size_t)ol * N + lane, wl);
      rep_w += lane < N ? wl : 0.0;
      const double w0l = __shfl(wl, 0, 64);
      if (lane == l) {
        acc_cost += cl;
        acc_p0 += pl;
        acc_err = fmax(acc_err, el);
        n_rep += okk ? 1 : 0;
        n_fail += okk ? 0 : 1;
        if (a.cost) st_wt8(a.cost + ol, cl);
        if (a.w0) st_wt8(a.w0 + ol, w0l);
        if (a.status) a.status[ol] = okk ? LOMPC_QP_REPAIRED : LOMPC_QP_FAILED;
      }
    }
    __builtin_amdgcn_wave_barrier();  // one wave's own LDS rows: in order, no vmcnt drain
    // ---- rows (lane = stage): w_t = a_t + b_t gamma of the EV's piece -> caller row perm[j]
    if (a.w) {
      const int nrow = min(64, b1 - i0);
      for (int r0 = 0; r0 < nrow; r0 += R) {
        const int row = r0 + rr;
        if (rlane && row < nrow) {
          const int pp = s_p[wv][row];
          if (pp != -1) {
            const double gr = s_g[wv][row];
            const int orow = s_o[wv][row];
            const int t0 = V * col;
            double x0, x1 = 0.0;
            if (pp >= 0) {
              const double2 u = s_ab[pp][t0];
              x0 = clampw(fma(u.y, gr, u.x), wm);
              if (V == 2) {
                const double2 u1 = s_ab[pp][t0 + 1];
                x1 = clampw(fma(u1.y, gr, u1.x), wm);
              }
            } else {
              x0 = x1 = NAN;  // invalid gamma
            }
            if (a.w_rsrc_ok) {
              const int off = (orow * N + t0) * 8;
              if (V == 2) st_wt16(rs, off, x0, x1);
              else st_wt8b(rs, off, x0);
            } else {
              double* dst = a.w + (size_t)orow * N + t0;
              st_wt8(dst, x0);
              if (V == 2) st_wt8(dst + 1, x1);
            }
          }
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
  }
  LQ_STAMP(4);
  // ---- per-wave totals, then wave 0 combines the waves in a fixed order
  {
    double tot[4] = {acc_cost, acc_p0, (double)(n_ok + n_rep), (double)n_rep};
    lqw::wave_totals(tot, 64);
    const double mx = lqw::wave_max(acc_err, 64);
    double cnt[2] = {(double)n_fail, (double)n_inv};
    lqw::wave_totals(cnt, 64);
    if (lane == 0) {
      s_red[wv][0] = tot[0];
      s_red[wv][1] = tot[1];
      s_red[wv][2] = mx;
      s_red[wv][3] = tot[2];
      s_red[wv][4] = tot[3];
      s_red[wv][5] = cnt[0];
      s_red[wv][6] = cnt[1];
    }
    s_repw[wv][lane] = rep_w;
  }
  __syncthreads();
  if (wv == 0) {
    double sw = 0.0;
    for (int kk = 0; kk < SOLVE_WAVES; ++kk) sw += s_repw[kk][lane];
    for (int k = 0; k < SOLVE_PATHS; ++k) {
      const int npk = s_npc[k];  // uniform
      for (int pp = 0; pp < npk; ++pp) {
        const int slot = k * LQ_PPLX + pp;
        double cnt = 0.0, sg = 0.0;
        for (int kk = 0; kk < SOLVE_WAVES; ++kk) {
          cnt += s_mom[kk][slot][0];
          sg += s_mom[kk][slot][1];
        }
        const double2 u = s_ab[slot][lane];
        sw += (lane < N) ? fma(u.x, cnt, u.y * sg) : 0.0;
      }
    }
    if (lane < N) st_wt8(part + lane, sw);
    if (lane < NPX) {
      double v = 0.0;
      for (int kk = 0; kk < SOLVE_WAVES; ++kk) v = lane == PX_MAX_ERR ? fmax(v, s_red[kk][lane]) : v + s_red[kk][lane];
      st_wt8(part + N + lane, v);
    }
    if (a.arrive) arrive_reduce(a, s, lane, N);
  }
  LQ_STAMP(5);
#ifdef LOMPC_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 65536) {
    int np = 0;
    for (int k = 0; k < SOLVE_PATHS; ++k) np += s_npc[k];
    g_stamps[blockIdx.x * 8 + 6] = np;
    g_stamps[blockIdx.x * 8 + 7] = b1 - b0;
  }
#endif
}

// ---------------------------------------------------------------- k_reduce
struct ReduceArgs {
  int G, N;
  const int64_t* set_off;
  const double* partial;
  double* set_sum_w;
  double* set_stats;
  double* stats;
};

// One 256-thread workgroup per set: wave wv sums the cell records wv, wv+4, ... (lane =
// column, 4 accumulators), then the 4 waves combine in a fixed order: deterministic.
__global__ __launch_bounds__(256) void k_reduce(ReduceArgs r) {
  __shared__ double red[4][LOMPC_MAX_N + NPX + 1];
  const int s = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = r.N, W = N + NPX, G1 = r.G + 1;
  const double* base = r.partial + (size_t)s * G1 * W;
  for (int c = lane; c < W; c += 64) {
    const bool is_max = c == N + PX_MAX_ERR;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    constexpr int U = 8;
    for (int b = wv; b < G1; b += 4 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int bb = b + 4 * u;
        v[u] = bb < G1 ? base[(size_t)bb * W + c] : 0.0;  // 0: neutral for sums and max of errors >= 0
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u & 3] = is_max ? fmax(acc[u & 3], v[u]) : acc[u & 3] + v[u];
    }
    red[wv][c] = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  if (tid < W) {
    const bool is_max = tid == N + PX_MAX_ERR;
    double v = red[0][tid];
    for (int k = 1; k < 4; ++k) v = is_max ? fmax(v, red[k][tid]) : v + red[k][tid];
    red[0][tid] = v;
  }
  __syncthreads();
  if (tid < N && r.set_sum_w) r.set_sum_w[(size_t)s * N + tid] = red[0][tid];
  if (tid < LOMPC_SET_STATS) {
    double v = 0.0;
    switch (tid) {
      case LOMPC_STAT_COUNT: v = (double)(r.set_off[s + 1] - r.set_off[s]); break;
      case LOMPC_STAT_SUM_W0: v = red[0][0]; break;
      case LOMPC_STAT_SUM_PRICE0: v = red[0][N + PX_PRICE0]; break;
      case LOMPC_STAT_MAX_ERR: v = red[0][N + PX_MAX_ERR]; break;
      case LOMPC_STAT_SUM_COST: v = red[0][N + PX_COST]; break;
      case LOMPC_STAT_N_REPAIRED: v = red[0][N + PX_N_REPAIRED]; break;
      case LOMPC_STAT_N_FAILED: v = red[0][N + PX_N_FAILED]; break;
      default: v = red[0][N + PX_N_INVALID]; break;
    }
    if (r.set_stats) r.set_stats[(size_t)s * LOMPC_SET_STATS + tid] = v;
    r.stats[(size_t)s * LOMPC_SET_STATS + tid] = v;
  }
}

int pick_cells(int64_t max_set, int flags) {
  const char* env = getenv("LOMPC_CELLS");  // diagnostics (cell-count sweeps)
  if (env) {
    const int g = atoi(env);
    if (g >= 1 && g <= 4096) return g;
  }
  (void)flags;
  // cells per set: the path has only a handful of breakpoints over a set's gamma window, so a
  // cell is sized by its EVs: ~3 chunks of 64 per wave of the cell's workgroup
  int G = 8;
  while (G < 1024 && max_set > (int64_t)G * 64 * 3 * LQ_SOLVE_WAVES) G *= 2;
  return G;
}

}  // namespace

// ============================================================== host
int lq_plan_prepare(lompc_plan* p, int nctx, lompc_ctx* const* ctxs, const int64_t* sets_per_ctx, int64_t B,
                    const double* gamma, const int64_t* set_offsets, const double* w_ref, int flags,
                    hipStream_t st) {
  if (nctx < 1 || nctx > LQ_PLAN_MAX_CTX || !ctxs || !sets_per_ctx || !set_offsets)
    return fail_arg(p, "plan: 1 <= n_ctx <= LOMPC_PLAN_MAX_CTX contexts and their set counts required");
  int64_t S = 0;
  for (int k = 0; k < nctx; ++k) {
    if (!ctxs[k]) return fail_arg(p, "plan: null context");
    if (ctxs[k]->N != ctxs[0]->N || ctxs[k]->device != ctxs[0]->device)
      return fail_arg(p, "plan: every context must have the same horizon N and device");
    if (sets_per_ctx[k] < 0) return fail_arg(p, "plan: negative set count");
    S += sets_per_ctx[k];
  }
  if (S < 1) return fail_arg(p, "plan: at least one parameter set required");
  if (S > (1 << 20)) return fail_arg(p, "plan: too many parameter sets");
  if (B < 0 || B >= (1ll << 31) - 64) return fail_arg(p, "plan: 0 <= B < 2^31 required");
  if (set_offsets[0] != 0 || set_offsets[S] != B) return fail_arg(p, "plan: set_offsets must run from 0 to B");
  int64_t max_set = 0;
  for (int64_t s = 0; s < S; ++s) {
    const int64_t m = set_offsets[s + 1] - set_offsets[s];
    if (m < 0) return fail_arg(p, "plan: set_offsets must be non-decreasing");
    max_set = std::max(max_set, m);
  }
  if (B > 0 && !gamma) return fail_arg(p, "plan: gamma required");
  const int N = ctxs[0]->N;
  HIPCHK(p, hipSetDevice(ctxs[0]->device));
  const int G = pick_cells(max_set, flags);
  const int64_t nbk = S * (G + 1);
  if (nbk >= (1ll << 31)) return fail_arg(p, "plan: too many cells");
  p->device = ctxs[0]->device;
  p->N = N;
  p->nctx = nctx;
  for (int k = 0; k < nctx; ++k) p->ctx[k] = ctxs[k];
  p->flags = flags;
  p->w_ref = w_ref;
  int rc;
  if (!p->d_q && (rc = grow(p, &p->d_q, LQ_PLAN_MAX_CTX))) return rc;
  if (!p->d_errflag) {
    if ((rc = grow(p, &p->d_errflag, 1))) return rc;
    HIPCHK(p, hipMemset(p->d_errflag, 0, sizeof(int)));
  }
  if (!p->ev_stage) HIPCHK(p, hipEventCreateWithFlags(&p->ev_stage, hipEventDisableTiming));
  if (S > p->cap_S) {
    if ((rc = grow(p, &p->d_set_ctx, S)) || (rc = grow(p, &p->d_set_off, S + 1)) || (rc = grow(p, &p->d_arrive, S)) ||
        (rc = grow(p, &p->d_window, 2 * S)) || (rc = grow(p, &p->d_stats_own, S * LOMPC_SET_STATS)))
      return rc;
    p->cap_S = S;
  }
  if (B > p->cap_B) {
    if ((rc = grow(p, &p->d_keys, 2 * B)) || (rc = grow(p, &p->d_vals, 2 * B)) || (rc = grow(p, &p->d_gs, B)))
      return rc;
    p->cap_B = B;
  }
  const bool warm = (flags & LOMPC_PLAN_WARM_START) != 0;
  bool fresh_ws = false;
  if (nbk > p->cap_bk || (warm && !p->d_ws)) {
    if ((rc = grow(p, &p->d_bucket_off, nbk + 1)) || (rc = grow(p, &p->d_partial, (size_t)nbk * (N + NPX))))
      return rc;
    if (warm && (rc = grow(p, &p->d_ws, (size_t)nbk * LQ_WS_MAX * 64))) return rc;
    p->cap_bk = nbk;
    fresh_ws = true;
  }
  if (warm && (fresh_ws || p->G != G || p->S != S))
    HIPCHK(p, hipMemsetAsync(p->d_ws, 1, (size_t)nbk * LQ_WS_MAX * 64, st));
  HIPCHK(p, hipMemsetAsync(p->d_arrive, 0, S * sizeof(unsigned), st));
  p->B = B;
  p->S = S;
  p->G = G;
  p->d_stats = p->d_stats_own;
  p->d_perm = p->d_vals + B;
  // radix-sort temporary storage
  const unsigned end_bit = std::max(1u, (unsigned)(64 - __builtin_clzll((unsigned long long)nbk)));
  size_t tmp = 0;
  if (B > 0) {
    HIPCHK(p, rocprim::radix_sort_pairs(nullptr, tmp, p->d_keys, p->d_keys + B, p->d_vals, p->d_vals + B,
                                        (size_t)B, 0u, end_bit, st));
    if (tmp > p->cap_tmp) {
      if (p->d_tmp) HIPCHK(p, hipFree(p->d_tmp));
      p->d_tmp = nullptr;
      HIPCHK(p, hipMalloc(&p->d_tmp, tmp));
      p->cap_tmp = tmp;
    }
  }
  // host arrays -> pinned staging -> device (the staging may still feed the previous prepare)
  const size_t need_h = (size_t)(S + 1) * sizeof(int64_t) + S + LQ_PLAN_MAX_CTX * sizeof(QPConst) + 64;
  if ((int64_t)need_h > p->cap_h) {
    HIPCHK(p, hipEventSynchronize(p->ev_stage));
    if (p->h_off) HIPCHK(p, hipHostFree(p->h_off));
    p->h_off = nullptr;
    HIPCHK(p, hipHostMalloc((void**)&p->h_off, need_h, hipHostMallocDefault));
    p->cap_h = (int64_t)need_h;
  }
  HIPCHK(p, hipEventSynchronize(p->ev_stage));
  QPConst* hq = reinterpret_cast<QPConst*>(p->h_off);
  for (int k = 0; k < nctx; ++k) hq[k] = ctxs[k]->q;
  int64_t* hoff = reinterpret_cast<int64_t*>(hq + LQ_PLAN_MAX_CTX);
  memcpy(hoff, set_offsets, (S + 1) * sizeof(int64_t));
  uint8_t* hctx = reinterpret_cast<uint8_t*>(hoff + S + 1);
  for (int k = 0, s = 0; k < nctx; ++k)
    for (int64_t u = 0; u < sets_per_ctx[k]; ++u) hctx[s++] = (uint8_t)k;
  HIPCHK(p, hipMemcpyAsync(p->d_q, hq, nctx * sizeof(QPConst), hipMemcpyHostToDevice, st));
  HIPCHK(p, hipMemcpyAsync(p->d_set_off, hoff, (S + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
  HIPCHK(p, hipMemcpyAsync(p->d_set_ctx, hctx, S, hipMemcpyHostToDevice, st));
  HIPCHK(p, hipEventRecord(p->ev_stage, st));
  PlanArgs a{};
  a.S = (int)S;
  a.G = G;
  a.nbk = (int)nbk;
  a.B = B;
  a.qd = p->d_q;
  a.set_ctx = p->d_set_ctx;
  a.set_off = p->d_set_off;
  a.window = p->d_window;
  a.gamma = gamma;
  a.keys = p->d_keys;
  a.vals = p->d_vals;
  a.keys_out = p->d_keys + B;
  a.vals_out = p->d_vals + B;
  a.bucket_off = p->d_bucket_off;
  a.gs = p->d_gs;
  hipLaunchKernelGGL(k_plan_window, dim3((unsigned)S), dim3(256), 0, st, a);
  HIPCHK(p, hipGetLastError());
  if (B > 0) {
    const unsigned nb = (unsigned)((B + 255) / 256);
    hipLaunchKernelGGL(k_plan_keys, dim3(nb), dim3(256), 0, st, a);
    HIPCHK(p, hipGetLastError());
    size_t t2 = p->cap_tmp;
    HIPCHK(p, rocprim::radix_sort_pairs(p->d_tmp, t2, p->d_keys, p->d_keys + B, p->d_vals, p->d_vals + B,
                                        (size_t)B, 0u, end_bit, st));
    hipLaunchKernelGGL(k_plan_finish, dim3(nb), dim3(256), 0, st, a);
    HIPCHK(p, hipGetLastError());
  } else {
    HIPCHK(p, hipMemsetAsync(p->d_bucket_off, 0, (nbk + 1) * sizeof(int), st));
  }
  return LOMPC_OK;
}

static int take_events(std::vector<hipEvent_t>& pool, hipEvent_t* e0, hipEvent_t* e1) {
  for (hipEvent_t* e : {e0, e1}) {
    if (!pool.empty()) {
      *e = pool.back();
      pool.pop_back();
    } else if (hipEventCreateWithFlags(e, hipEventDisableSystemFence) != hipSuccess) {
      return LOMPC_ERR_HIP;
    }
  }
  return LOMPC_OK;
}

int lq_plan_launch(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, hipStream_t st, lompc_ctx* prof_ctx) {
  if (!lmbd || !lmbd_r) return fail_arg(p, "run: lmbd and lmbd_r required");
  const int N = p->N;
  const int64_t nbk = p->S * (p->G + 1);
  SolveArgs a{};
  a.S = (int)p->S;
  a.G = p->G;
  a.flags = p->flags;
  a.want_err = 1;
  a.N = N;
  a.B = p->B;
  a.qd = p->d_q;
  a.set_ctx = p->d_set_ctx;
  a.window = p->d_window;
  a.bucket_off = p->d_bucket_off;
  a.gs = p->d_gs;
  a.perm = p->d_perm;
  a.lmbd = lmbd;
  a.lmbd_r = lmbd_r;
  a.w_ref = p->w_ref;
  a.ws = (p->flags & LOMPC_PLAN_WARM_START) ? p->d_ws : nullptr;
  a.w = w;
  a.cost = cost;
  a.w0 = w0;
  a.status = status;
  a.partial = p->d_partial;
  a.errflag = p->d_errflag;
  a.w_rsrc_ok = (p->B * (int64_t)N * 8) < (1ll << 31) ? 1 : 0;
  // the in-kernel per-set reduction (last-arriving workgroup) measured 4-5 us slower on the
  // config-3 step than k_reduce (rejected designs): diagnostics only
  static const bool fused = getenv("LOMPC_REDUCE_FUSED") != nullptr;
  const bool separate = !fused;
  a.arrive = separate ? nullptr : p->d_arrive;
  a.set_off = p->d_set_off;
  a.set_sum_w = set_sum_w;
  a.set_stats = set_stats;
  a.stats = p->d_stats;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  const bool prof = p->prof || (prof_ctx && prof_ctx->prof);
  if (prof) {
    std::vector<hipEvent_t>& pool = p->prof ? p->prof_pool : prof_ctx->prof_pool;
    if (take_events(pool, &e0, &e1)) return fail_arg(p, "profiling events");
  }
  hipExtLaunchKernelGGL((k_solve<LQ_SOLVE_WAVES, LQ_SOLVE_PATHS>), dim3((unsigned)nbk), dim3(64 * LQ_SOLVE_WAVES), 0,
                        st, e0, e1, 0, a);
  HIPCHK(p, hipGetLastError());
  if (prof) {
    std::vector<hipEvent_t>& ev = p->prof ? p->prof_ev : prof_ctx->prof_ev;
    ev.push_back(e0);
    ev.push_back(e1);
  }
  if (!separate) return LOMPC_OK;
  ReduceArgs r{};
  r.G = p->G;
  r.N = N;
  r.set_off = p->d_set_off;
  r.partial = p->d_partial;
  r.set_sum_w = set_sum_w;
  r.set_stats = set_stats;
  r.stats = p->d_stats;
  hipLaunchKernelGGL(k_reduce, dim3((unsigned)p->S), dim3(256), 0, st, r);
  HIPCHK(p, hipGetLastError());
  return LOMPC_OK;
}

void lq_plan_free(lompc_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  (void)hipDeviceSynchronize();
  void* ptrs[] = {p->d_q, p->d_stats_own, p->d_set_ctx, p->d_set_off, p->d_window, p->d_keys, p->d_vals,
                  p->d_bucket_off, p->d_gs, p->d_partial, p->d_ws, p->d_tmp, p->d_errflag, p->d_arrive};
  for (void* x : ptrs)
    if (x) (void)hipFree(x);
  if (p->h_off) (void)hipHostFree(p->h_off);
  if (p->ev_stage) (void)hipEventDestroy(p->ev_stage);
  for (hipEvent_t e : p->prof_ev) (void)hipEventDestroy(e);
  for (hipEvent_t e : p->prof_pool) (void)hipEventDestroy(e);
  delete p;
}

static int plan_events_read(std::vector<hipEvent_t>& ev, std::vector<hipEvent_t>& pool, double& ms_acc,
                            int64_t& n_acc) {
  for (size_t k = 0; k + 1 < ev.size(); k += 2) {
    if (hipEventSynchronize(ev[k + 1]) != hipSuccess) return LOMPC_ERR_HIP;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev[k], ev[k + 1]) != hipSuccess) return LOMPC_ERR_HIP;
    ms_acc += ms;
    n_acc += 1;
  }
  pool.insert(pool.end(), ev.begin(), ev.end());
  ev.clear();
  return LOMPC_OK;
}

extern "C" {

#ifdef LOMPC_STAMPS
int lompc_debug_stamps(long long* host, int n) {
  if (n > 65536 * 8) n = 65536 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(long long) * n, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? LOMPC_OK
             : LOMPC_ERR_HIP;
}
#endif

int lompc_plan_create(int n_ctx, lompc_ctx* const* ctxs, const int64_t* sets_per_ctx, int64_t B,
                      const double* gamma, const int64_t* set_offsets, const double* w_ref, int flags, void* stream,
                      lompc_plan** out) {
  if (!out) return LOMPC_ERR_INVALID_ARG;
  *out = nullptr;
  lompc_plan* p = new lompc_plan();
  const int rc = lq_plan_prepare(p, n_ctx, ctxs, sets_per_ctx, B, gamma, set_offsets, w_ref, flags,
                                 (hipStream_t)stream);
  if (rc) {
    if (n_ctx >= 1 && ctxs && ctxs[0]) ctxs[0]->err = p->err;
    lq_plan_free(p);
    return rc;
  }
  *out = p;
  return LOMPC_OK;
}

int lompc_plan_run(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, void* stream) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  return lq_plan_launch(p, lmbd, lmbd_r, w, cost, w0, status, set_sum_w, set_stats, (hipStream_t)stream, nullptr);
}

int lompc_plan_status(lompc_plan* p, void* stream, int64_t* n_repaired, int64_t* n_failed, int64_t* n_invalid) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  std::vector<double> h((size_t)p->S * LOMPC_SET_STATS, 0.0);
  int ef = 0;
  HIPCHK(p, hipMemcpyAsync(h.data(), p->d_stats, h.size() * sizeof(double), hipMemcpyDeviceToHost,
                           (hipStream_t)stream));
  HIPCHK(p, hipMemcpyAsync(&ef, p->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(p, hipStreamSynchronize((hipStream_t)stream));
  double rep = 0, fail = 0, inv = 0;
  for (int64_t s = 0; s < p->S; ++s) {
    rep += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_REPAIRED];
    fail += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_FAILED];
    inv += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_INVALID];
  }
  if (n_repaired) *n_repaired = (int64_t)rep;
  if (n_failed) *n_failed = (int64_t)fail;
  if (n_invalid) *n_invalid = (int64_t)inv;
  if (ef) {
    HIPCHK(p, hipMemsetAsync(p->d_errflag, 0, sizeof(int), (hipStream_t)stream));
    return fail_arg(p, "negative or NaN price parameter (lmbd >= 0, lmbd_r >= 0 required)");
  }
  return LOMPC_OK;
}

int lompc_plan_get_info(const lompc_plan* p, int64_t* B, int64_t* S, int* cells) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  if (B) *B = p->B;
  if (S) *S = p->S;
  if (cells) *cells = p->G;
  return LOMPC_OK;
}

int lompc_plan_profile_enable(lompc_plan* p, int enable) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  p->prof = enable != 0;
  while (p->prof && p->prof_pool.size() < 512) {
    hipEvent_t e;
    HIPCHK(p, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    p->prof_pool.push_back(e);
  }
  return LOMPC_OK;
}

int lompc_plan_profile_read(lompc_plan* p, double* total_ms, int64_t* launches, int reset) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  if (plan_events_read(p->prof_ev, p->prof_pool, p->prof_ms, p->prof_n)) return LOMPC_ERR_HIP;
  if (total_ms) *total_ms = p->prof_ms;
  if (launches) *launches = p->prof_n;
  if (reset) {
    p->prof_ms = 0.0;
    p->prof_n = 0;
  }
  return LOMPC_OK;
}

const char* lompc_plan_last_error(const lompc_plan* p) { return p ? p->err.c_str() : ""; }

int lompc_plan_destroy(lompc_plan* p) {
  lq_plan_free(p);
  return LOMPC_OK;
}

}  // extern "C"
