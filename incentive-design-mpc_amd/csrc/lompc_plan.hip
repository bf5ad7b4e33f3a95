// lompc_plan.hip — the PATH engine: a fixed EV batch (one price loop / one time step) solved
// at new prices every price iteration.
//
// Hot path replaced: LoMPC.solve_lompc (chargingstation/lompc.py:137-156) called once per EV
// from PriceSolver._get_w_err (price_solver.py:203-209) and PriceSolver.get_w0_price0
// (price_solver.py:280-283).  Within one parameter set (an (EV type, partition) price vector)
// every EV solves the same QP except gamma_i = y_max - y0_i (price_solver.py:202, :281), so
// w*(gamma) is a continuous piecewise-affine path with a handful of breakpoints over the
// set's gamma range.
//
// Plan (once per batch, lompc_plan_create): per-set gamma window [lo, hi] (range of the set's
// valid gamma, k_plan_window) cut into G cells; the block map of k_eval (256 consecutive EVs of
// one set per workgroup).
//
// Run (every price iteration, lompc_plan_run), three launches for ALL EV types of the plan:
//   k_path    one 64-lane wave per (set, cell), lane t = horizon stage t: exact solve at the
//             cell start (fp32 working-set search + fp64 PDAS, KKT-certified), then parametric
//             active-set tracking of w*(gamma) across the cell; every piece w = a + b gamma is
//             KKT-certified at its end (the residual is convex along an affine piece, so both
//             ends certify the whole piece) and stored with the cost and the squared A_bar
//             error as quadratics in gamma.  Latency-bound: wave-parallel DPP scans.
//   k_eval    256 EVs of one set per workgroup in the caller's order: the set's pieces staged
//             in LDS (a few KB), per EV (lane = EV) its piece, cost, w0, status, price0, A_bar
//             error; the w rows (lane = stage) as contiguous 16-B write-through stores; EVs no
//             certified piece covers listed for k_finalize; per-workgroup sums in a fixed
//             order.  HBM-bound: 8(N+2) B per EV.
//   k_finalize one workgroup per set: deterministic sum / max of its workgroups' records, and the
//             individual certified re-solve of any EV k_eval listed (no certified piece covers it).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "lompc_ctx.hpp"
#include "lompc_loopstep.hpp"
#include "lompc_wave.hpp"

#ifdef LOMPC_STAMPS
// diagnostic build only (scripts/kstamps.py): per-wave s_memtime at k_path's and k_eval's phase
// boundaries (k_eval: workgroup b at g_stamps[(32768 + b) * 8 + k]); LOMPC_STAMPS_RT: the
// device-wide 100 MHz s_memrealtime instead (comparable across XCDs: launch timelines)
#ifdef LOMPC_STAMPS_RT
#define __builtin_amdgcn_s_memtime __builtin_amdgcn_s_memrealtime
#endif
__device__ long long g_stamps[65536 * 8];
__device__ long long g_wstart[32768 * 8];          // k_eval: start of wave w of workgroup b at [b * 8 + w]
__device__ unsigned long long g_lstamps[64 * 16];  // k_loop_iter's phase sums (LQ_LSTAMP)
#define LQ_WSTART()                                                                              \
  do {                                                                                           \
    const long long t__ = __builtin_amdgcn_s_memtime();                                          \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 32768) g_wstart[blockIdx.x * 8 + (threadIdx.x >> 6)] = t__; \
  } while (0)
#define LQ_STAMPE(k)                                                                        \
  do {                                                                                      \
    const long long t__ = __builtin_amdgcn_s_memtime();                                     \
    if (threadIdx.x == 0 && blockIdx.x < 32768) g_stamps[(32768 + blockIdx.x) * 8 + (k)] = t__; \
  } while (0)
#define LQ_STAMPW(k)                                                                        \
  do {                                                                                      \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                        \
    LQ_STAMPE(k);                                                                           \
  } while (0)
#define LQ_STAMP(k)                                                                         \
  do {                                                                                      \
    const long long t__ = __builtin_amdgcn_s_memtime();                                     \
    if ((threadIdx.x & 63) == 0 && blk < 65536) g_stamps[blk * 8 + (k)] = t__;              \
  } while (0)
#else
#define LQ_STAMP(k)
#define LQ_STAMPE(k)
#define LQ_STAMPW(k)
#define LQ_WSTART()
#endif

#ifndef EVAL_WAVES
#define EVAL_WAVES 8  // k_eval: waves per workgroup (16: 16.1 us, 8: 14.8 us, 4: 16.2 us at config 3)
#endif
#ifndef EVAL_RU
#define EVAL_RU 2  // k_eval: row store instructions per software-pipelined batch (2: k_evals 11.17 vs 11.70 us
                   // per run with 4, 11.68 with 3 — the same rows in the same order, so the same bits)
#endif
#ifndef EVAL_MIN_WAVES
#define EVAL_MIN_WAVES ((2 * EVAL_WAVES + 3) / 4)  // k_eval: waves per SIMD for two workgroups per CU
#endif
#define EVAL_EVS (64 * EVAL_WAVES)         // k_eval: threads per workgroup
#ifndef EVAL_PASSES
#define EVAL_PASSES 2                      // k_eval: EVs per thread, at most
#endif
#define EVAL_MAXB (EVAL_EVS * EVAL_PASSES)  // k_eval: EVs per workgroup, at most
#ifndef LQ_PIECE_CAP
#define LQ_PIECE_CAP 128                   // k_eval: piece slots of one set staged in LDS (more: re-solved)
#endif
#define LQ_GMAX 1024                       // max cells per set
#ifndef LQ_EVAL_OUT_AFTER_ROWS
#define LQ_EVAL_OUT_AFTER_ROWS 1  // k_eval / k_step / k_evals: a pass's scalar outputs after its rows
#endif
#ifndef LQ_DIAG_NOLOOKUP
#define LQ_DIAG_NOLOOKUP 0  // diagnostic timing builds: every valid EV takes its cell's first piece (wrong results)
#endif
#ifndef LQ_DIAG_NOROWLDS
#define LQ_DIAG_NOROWLDS 0  // diagnostic timing builds: the rows' values without their LDS reads (wrong results)
#endif
#ifndef LQ_STEP_CELLS
#define LQ_STEP_CELLS 4                    // k_step: path cells per workgroup, one per wave (<= EVAL_WAVES; 4: one per
                                           // SIMD — 19.2 us per step vs 22.4 with 8, 19.9 with 2, profiles/r03_v5)
#endif
#ifndef LQ_STEP_PRIO
#define LQ_STEP_PRIO 1                     // k_step: path waves at raised issue priority
#endif
#ifndef LQ_WARM_FP64
#define LQ_WARM_FP64 1                     // k_path with a warm start: fp64 PDAS straight from the stored set
#endif
#define LQ_DROP_OFF 0x7fff0000             // k_eval: a store offset past any w descriptor's range (dropped)

namespace {

typedef unsigned int lq_v4u __attribute__((ext_vector_type(4)));
typedef unsigned int lq_v2u __attribute__((ext_vector_type(2)));

// write-through (sc1) stores: the outputs leave no dirty lines in the XCD's L2, so the kernel
// boundary behind k_eval has no L2 writeback to wait for (MI355X_MICROARCH.md, price list)
#ifndef LQ_ROW_AUX
#define LQ_ROW_AUX 16  // the row stores' cache policy bits (16: sc1, write-through); diagnostic builds vary it
#endif
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t rs, int off, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lq_v4u, make_double2(x, y)), rs, off, 0, LQ_ROW_AUX);
}
__device__ __forceinline__ void st_wt8b(__amdgpu_buffer_rsrc_t rs, int off, double x) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(lq_v2u, x), rs, off, 0, LQ_ROW_AUX);
}
__device__ __forceinline__ void st_wt8(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// per-EV scalar outputs (cost, w0): 8-B write-through stores are one fabric write each (2.7x the
// per-byte time of 16-B ones, MI355X_MICROARCH.md); EV_PLAIN (diagnostic builds) stores them plain
#ifndef LQ_EV_PLAIN
#define LQ_EV_PLAIN 0
#endif
__device__ __forceinline__ void st_ev8(double* p, double v) {
  if (LQ_EV_PLAIN) *p = v;
  else st_wt8(p, v);
}

__device__ __forceinline__ void st_wt4(int* p, int v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// k_eval: double2 per LDS piece row (padding shifts consecutive rows across the banks)
__host__ __device__ constexpr int eval_row_stride(int N) { return N + 1; }
// k_eval: LDS double of coefficient j of piece k; the record's four 16-B quarters are permuted
// by bits 2..3 of k, so lanes reading quarter q of different pieces spread over all 64 banks
// (records are 64 B: unswizzled, quarter q of every piece falls on one of 4 bank slots)
__device__ __forceinline__ int cfx(const int k, const int j) {
  return k * 8 + ((((j >> 1) ^ (k >> 2)) & 3) << 1) + (j & 1);
}
static_assert((LQ_PPL & (LQ_PPL - 1)) == 0, "k_eval's piece-end transpose needs a power-of-two LQ_PPL");

// ---- k_evals' staged form: wave LQ_EVALS_RW of every workgroup stages the NEXT run's piece table
// while waves 0 .. LQ_EVALS_RW - 1 evaluate the current run from the other of two LDS tables, so no
// workgroup stops its row stores to wait for table loads (a wave's loads wait for every store it
// issued before them — vmcnt counts both, in order — and the stager issues no stores).  Its tables
// are compact: only the set's used pieces, cell c's at slots pre[c] .. pre[c] + cnt[c] - 1 (cells past
// the capacity left to the re-solve, as cells past the plain table's `cap` are).
#ifndef LQ_EVALS_STAGER
#define LQ_EVALS_STAGER 0  // 1: the wide form's evaluation through k_evals_st (diagnostic builds: measured slower,
                           // 12.5 vs 11.8 us per run at config 3 — DESIGN.md section 10)
#endif
#ifndef LQ_EVALS_CAP
#define LQ_EVALS_CAP 64                                 // compact table: pieces of a set staged at most
#endif
#ifndef LQ_STG_CHUNK
#define LQ_STG_CHUNK 8                                  // the stager's pieces per load round
#endif
#define LQ_EVALS_RW 7                                   // row waves (the eighth stages)
#define LQ_EVALS_MAXB (LQ_EVALS_RW * 64 * EVAL_PASSES)  // EVs per block at most (each wave's re-solve list)

struct CTab {
  double2* ab;  // [capc + 2][eval_row_stride(N)] piece rows (abx order); rows capc, capc + 1 all zero
  double* cf;   // [capc][8] coefficient records (cfx)
  double* ge;   // [capc + 8] piece ends (a lookup reads up to 8 past a cell's first slot)
  double* lo;   // [G] coverage starts
  int* cnt;     // [G] staged pieces per cell (0: none, or past the capacity)
  int* pre;     // [G] the cell's first slot
  int* meta;    // [0] the largest cnt, [1] the staged pieces
};
__host__ __device__ inline size_t ctab_bytes(int N, int G, int capc) {
  const size_t b = (size_t)(capc + 2) * eval_row_stride(N) * 16 + (size_t)capc * 64 + (size_t)(capc + 8) * 8 +
                   (size_t)G * 16 + 16;
  return (b + 15) & ~(size_t)15;
}
__device__ __forceinline__ CTab ctab_at(char* base, int N, int G, int capc) {
  CTab t;
  t.ab = reinterpret_cast<double2*>(base);
  t.cf = reinterpret_cast<double*>(base + (size_t)(capc + 2) * eval_row_stride(N) * 16);
  t.ge = t.cf + (size_t)capc * 8;
  t.lo = t.ge + capc + 8;
  t.cnt = reinterpret_cast<int*>(t.lo + G);
  t.pre = t.cnt + G;
  t.meta = t.pre + G;
  return t;
}
// k_evals_st dynamic LDS: two tables | row sums [2][EVAL_WAVES][N] | wave records [2][EVAL_WAVES][8]
inline size_t evals_st_lds(int N, int G, int capc) {
  return 2 * ctab_bytes(N, G, capc) + (size_t)2 * EVAL_WAVES * (N + 8) * sizeof(double);
}

__device__ __forceinline__ double clampw(double x, double wmax) { return fmin(fmax(x, 0.0), wmax); }

// ---------------------------------------------------------------- plan kernel
// the constants of set s's EV type: the context index from the kernel arguments and wave-uniform,
// so every field is a scalar (constant-cache) load instead of a vector load with a full memory
// round trip
// (the table is read-only for the whole launch: the constant address space lets the compiler use
// scalar loads although the kernels store to other global memory)
typedef const __attribute__((address_space(4))) QPConst QPConstK;
__device__ __forceinline__ const QPConst& set_consts(const QPConst* qd, const CtxEnds& ce, int s) {
  s = __builtin_amdgcn_readfirstlane(s);
  int k = 0;
#pragma unroll
  for (int j = 0; j + 1 < LQ_PLAN_MAX_CTX; ++j) k += s >= ce.end[j] ? 1 : 0;
  QPConstK* p = (QPConstK*)(uintptr_t)qd + k;
  return *(const QPConst*)p;
}

struct WindowArgs {
  const QPConst* qd;
  CtxEnds ce;
  const int4* blk;         // k_eval's block map: (set, begin, end)
  const int* blk_prefix;   // [S+1] first block of each set
  const double* gamma;
  unsigned long long* acc; // [S][3], zero on entry and on exit
  double* window;
  int S, nblk;
};

// per set: [lo, hi] = range of its valid gamma, widened by 1e-7 y_max (a zero-width set still
// gets cells of positive width), clipped to [0, y_max]; no valid EV -> [0, y_max].
// One workgroup per k_eval block (>= one per CU): a block folds its EVs, then merges into its
// set's accumulators with integer atomics (the bits of a non-negative double order like the
// double, so min/max are exact and the result does not depend on the order); the set's last
// block writes the window and zeroes the accumulators for the next launch.  One extra workgroup
// (the last) writes the windows of the empty sets, which have no blocks.
// the window from the set's smallest / largest valid gamma (any: there is one)
__device__ __forceinline__ void window_store(double* window, int s, double ym, bool any, double lo, double hi) {
  const double mg = 1e-7 * ym;
  double wlo = 0.0, whi = ym;
  if (any) {
    wlo = fmin(fmax(lo - mg, 0.0), ym);
    whi = fmin(fmax(hi + mg, wlo + mg), ym);
    if (!(whi > wlo)) wlo = fmax(whi - 2.0 * mg, 0.0);
  }
  window[2 * s] = wlo;
  window[2 * s + 1] = whi;
}

__global__ __launch_bounds__(256) void k_plan_window(WindowArgs a) {
  __shared__ double smin[4], smax[4];
  __shared__ int last;
  if ((int)blockIdx.x == a.nblk) {
    for (int s = threadIdx.x; s < a.S; s += 256)
      if (a.blk_prefix[s + 1] == a.blk_prefix[s]) {
        int k = 0;  // (s differs per lane: no scalar set_consts)
        for (int j = 0; j + 1 < LQ_PLAN_MAX_CTX; ++j) k += s >= a.ce.end[j] ? 1 : 0;
        a.window[2 * s] = 0.0;
        a.window[2 * s + 1] = a.qd[k].y_max;
      }
    return;
  }
  const int4 bk = a.blk[blockIdx.x];
  const int s = bk.x;
  const double ym = set_consts(a.qd, a.ce, s).y_max;
  double lo = INFINITY, hi = -INFINITY;
  for (int i = bk.y + (int)threadIdx.x; i < bk.z; i += 256) {
    const double g = a.gamma[i];
    if (g >= 0.0 && g <= ym) {
      lo = fmin(lo, g);
      hi = fmax(hi, g);
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, o));
    hi = fmax(hi, __shfl_xor(hi, o));
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    smin[wv] = lo;
    smax[wv] = hi;
  }
  __syncthreads();
  unsigned long long* acc = a.acc + 3 * s;
  if (threadIdx.x == 0) {
    lo = fmin(fmin(smin[0], smin[1]), fmin(smin[2], smin[3]));
    hi = fmax(fmax(smax[0], smax[1]), fmax(smax[2], smax[3]));
    if (lo <= hi) {  // + 0.0: -0.0 -> +0.0, whose bits order with the positive doubles
      atomicMax(&acc[0], ~(unsigned long long)__double_as_longlong(lo + 0.0));
      atomicMax(&acc[1], (unsigned long long)__double_as_longlong(hi + 0.0));
    }
    __threadfence();
    const unsigned long long nb = (unsigned long long)(a.blk_prefix[s + 1] - a.blk_prefix[s]);
    last = atomicAdd(&acc[2], 1ull) == nb - 1;
  }
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const unsigned long long blo = atomicExch(&acc[0], 0ull), bhi = atomicExch(&acc[1], 0ull);
  atomicExch(&acc[2], 0ull);
  window_store(a.window, s, ym, blo != 0, __longlong_as_double((long long)~blo), __longlong_as_double((long long)bhi));
}

// gamma-sorted plans (LOMPC_PLAN_SORTED_GAMMA): one wave per set.  An ascending set whose first and
// last gamma are valid has its valid range at its ends — the same window as k_plan_window's in one
// load round instead of a pass over the set and one atomic per block (a set whose ends are not both
// valid is folded by the wave, as k_plan_window does; an unsorted set is reported failed by k_agg).
__global__ __launch_bounds__(64) void k_plan_window_sorted(WindowArgs a, const int64_t* __restrict__ set_off) {
  const int s = (int)blockIdx.x, lane = (int)threadIdx.x;
  const double ym = set_consts(a.qd, a.ce, s).y_max;
  const int64_t s0 = set_off[s], s1 = set_off[s + 1];
  if (s1 == s0) {
    if (lane == 0) window_store(a.window, s, ym, false, 0.0, 0.0);
    return;
  }
  const double g0 = a.gamma[s0], g1 = a.gamma[s1 - 1];
  const bool v0 = g0 >= 0.0 && g0 <= ym, v1 = g1 >= 0.0 && g1 <= ym;
  double lo = g0, hi = g1;
  if (!(v0 && v1)) {
    lo = INFINITY;
    hi = -INFINITY;
    for (int64_t i = s0 + lane; i < s1; i += 64) {
      const double g = a.gamma[i];
      if (g >= 0.0 && g <= ym) {
        lo = fmin(lo, g);
        hi = fmax(hi, g);
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      lo = fmin(lo, __shfl_xor(lo, o));
      hi = fmax(hi, __shfl_xor(hi, o));
    }
  }
  if (lane == 0) window_store(a.window, s, ym, lo <= hi, lo + 0.0, hi + 0.0);
}

// cell of a valid gamma in a set's window (k_eval), the same arithmetic as k_path's cell bounds
__device__ __forceinline__ int cell_of(double g, double lo, double inv_h, int G) {
  const double x = (g - lo) * inv_h;
  return x <= 0.0 ? 0 : (x >= (double)(G - 1) ? G - 1 : (int)x);
}

// ---------------------------------------------------------------- k_path
struct PathArgs {
  int S, G, N, flags;
  const QPConst* qd;
  CtxEnds ce;
  const double* window;
  const double* lmbd;    // [S][3N]
  const double* lmbd_r;  // [S]
  const double* w_ref;   // [S][N] or null
  uint8_t* ws;           // [S*G][64] warm-start working sets or null
  // per cell
  int* t_cnt;            // [S*G]             certified pieces of the cell (0: none)
  double* t_lo;          // [S*G]             coverage start
  uint8_t* t_sl;         // [S*G][64]         working set at the cell start (repairs)
  // per cell LQ_PPL piece slots, the first t_cnt used (ascending gamma)
  double* t_ge;          // [S][G*PPL]        gamma at each piece's end
  double* t_cf;          // [S][G*PPL][8]     K0 K1 K2 (cost) F0 F1 F2 (err^2) a_0 b_0
  double2* t_ab;         // [S][G*PPL][N]     (a_t, b_t)
  int* errflag;
  const int* skip;       // device-resident price loop: nonzero = the loop has finished, run nothing
};

// price loads: plain, or (COH) device-coherent sc1 loads past this CU's L1 — the persistent price
// loop (k_loop_run) re-reads prices that another workgroup of the same launch wrote through (sc1)
template <bool COH>
__device__ __forceinline__ double ld_price(const double* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// per-stage data of set s from its prices (lompc.py:92-135 in standard form)
// (bad: a negative or NaN price on this lane's stage)
template <bool COH = false>
__device__ __forceinline__ void load_set(const QPConst& q, const double* __restrict__ L, double lr, int N,
                                         int lane, lqw::WaveSet& ws, double& l2, bool& bad) {
  const double tt = q.theta * q.theta;
  ws.N = N;
  ws.lane = lane;
  l2 = 0.0;
  bad = false;
  if (lane < N) {
    const double l1 = ld_price<COH>(L + lane), l3 = ld_price<COH>(L + 2 * N + lane);
    l2 = ld_price<COH>(L + N + lane);
    bad = !(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0);
    ws.d_nat = 2.0 * lr * tt + 2.0 * q.q_scale * l3 + q.dsmall;
    ws.e_nat = q.theta * (l1 - l2);
  } else {
    ws.d_nat = ws.e_nat = 0.0;
  }
}

// load_set with the set's prices already in registers (lane t < N: prices t, N + t, 2N + t)
__device__ __forceinline__ void load_set_regs(const QPConst& q, double l1, double l2v, double l3, double lr, int N,
                                              int lane, lqw::WaveSet& ws, double& l2, bool& bad) {
  const double tt = q.theta * q.theta;
  ws.N = N;
  ws.lane = lane;
  l2 = 0.0;
  bad = false;
  if (lane < N) {
    l2 = l2v;
    bad = !(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0);
    ws.d_nat = 2.0 * lr * tt + 2.0 * q.q_scale * l3 + q.dsmall;
    ws.e_nat = q.theta * (l1 - l2);
  } else {
    ws.d_nat = ws.e_nat = 0.0;
  }
}

// One (set, gamma cell) path by one wave (blk = s * G + cell); the wave's workgroup has
// initialised the box table for the set's constants (lq_tab_init).  Every piece goes straight
// to the cell's fixed slots with write-through stores (visible to any XCD once they complete).
// NT: the horizon as a compile-time constant (0: a.N at run time) — the scans' row / bank steps
// become straight-line code, so independent chains can be interleaved
template <int NT = 0, bool INIT_TAB = false, bool COH = false, bool PREG = false>
__device__ __forceinline__ void path_cell(const PathArgs& a, const int blk, double p1 = 0.0, double p2 = 0.0,
                                          double p3 = 0.0, double wr_in = 0.0, int* ws_io = nullptr) {
  // (PREG: the set's prices p1..p3, the lane's w_ref wr_in and the cell's stored working set *ws_io
  // in registers — k_loop_run2's later calls; the working set still stored for the next loop)
  const int G = a.G;
  const int s = __builtin_amdgcn_readfirstlane(blk / G);
  const int cell = blk - s * G;
  const int lane = (int)threadIdx.x & 63;
  const int N = NT ? NT : a.N;
  const double* __restrict__ L = a.lmbd + (size_t)s * 3 * N;
  const double lr = a.lmbd_r[s];
  const double wr_nat = PREG ? wr_in : (a.w_ref && lane < N) ? a.w_ref[(size_t)s * N + lane] : 0.0;
  const double wlo = a.window[2 * s], whi = a.window[2 * s + 1];
  const QPConst& q = set_consts(a.qd, a.ce, s);  // scalar loads, no register copy
  LQ_STAMP(0);
  lqw::WaveSet ws;
  double l2;
  bool bad;
  if constexpr (PREG) load_set_regs(q, p1, p2, p3, lr, N, lane, ws, l2, bad);
  else load_set<COH>(q, L, lr, N, lane, ws, l2, bad);
  if (INIT_TAB) lq_tab_init(q);  // (after the price loads are issued: the barrier overlaps them)
  if (bad || (lane == 0 && !(lr >= 0.0))) atomicOr(a.errflag, 1);
  const double c0 = q.theta * q.w_max * lqw::wave_sum(l2, N);  // lompc.py:128
  const double kappa = lr / q.delta;                            // price_solver.py:191
  double Ywr;
  {
    lqw::Sums<1> y;
    y.v[0] = wr_nat;
    Ywr = lqw::wave_scan(y, N).v[0];
  }
  const double h = (whi - wlo) / (double)G;
  const double mg = 1e-13 * q.y_max;  // cells overlap by a rounding margin
  const double glo = fmax((cell == 0 ? wlo : fma((double)cell, h, wlo)) - mg, 0.0);
  const double ghi = fmin((cell == G - 1 ? whi : fma((double)(cell + 1), h, wlo)) + mg, q.y_max);
  LQ_STAMP(1);
  int npc = 0;
  int sl0 = lane < N ? 1 : 0;
  if (!(a.flags & LOMPC_PLAN_DIAG_REPAIR)) {
    int sl = sl0;
    bool warm = false;
    if (a.ws) {
      const int v = (PREG && ws_io) ? *ws_io : a.ws[(size_t)blk * 64 + lane];
      sl = (lane < N && v >= 0 && v <= 2 * q.m) ? v : sl0;
      warm = LQ_WARM_FP64 && __all(lane >= N || v <= 2 * q.m);  // (a stored set on every stage: wave-uniform)
    }
    lqw::StageSol<2> sol;
    bool has_sol = false;
#ifdef LOMPC_STAMPS
    int nit = 0;
    const bool solved = lqw::wave_solve_path(q, ws, glo, sl, sol, has_sol, &nit, warm);
    if (lane == 0 && blk < 32768) g_stamps[blk * 8 + 4] = nit;
#else
    const bool solved = lqw::wave_solve_path(q, ws, glo, sl, sol, has_sol, nullptr, warm);
#endif
    LQ_STAMP(2);
    if (solved) {
      sl0 = sl;
      if (a.ws) a.ws[(size_t)blk * 64 + lane] = (uint8_t)sl;
      if (ws_io) *ws_io = (int)(uint8_t)sl;
      const size_t sb = (size_t)blk * LQ_PPL;  // the cell's fixed piece slots
      // ---- parametric active-set tracking of w*(gamma) on [glo, ghi]
      double gcur = glo;
      int last = -1;
      const int max_iter = 4 * LQ_PPL + 16;
      const double ee = ws.e_nat;
      if (!has_sol) sol = lqw::solve_stage<2>(q, ws, 0.0, sl);  // (else the start's solve is reused)
      Box bxn = lq_box(lane < N ? sl : 0);  // the working set's boxes (carried: read with its solve)
      for (int it = 0; it < max_iter && npc < LQ_PPL; ++it) {
#ifdef LOMPC_STAMPS
        if (lane == 0 && blk < 32768) g_stamps[blk * 8 + 5] = it + 1;
#endif
        const double av = sol.w[0], bv = sol.w[1], r0 = sol.r[0], r1 = sol.r[1];
        double gc = INFINITY;
        int ns = sl;
        const bool act = lane < N;
        const Box bx = bxn;
        if (act) {
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
        const bool final_piece = (bj < 0) || (npc == LQ_PPL - 1);
        const bool emit = best > gcur || final_piece;  // (wave-uniform)
        // The next working set (the switch at the breakpoint) and its sub-problem solve do not
        // depend on this piece's certificate and quadratics: all of them in one basic block, so
        // the scheduler interleaves the independent DPP-scan chains (the next solve is wasted
        // work, not latency, when this piece is the last).
        const int bns = lqw::readlane_i(ns, bj < 0 ? 0 : bj);  // (bj wave-uniform: from a ballot)
        const int sln = lane == bj ? bns : sl;
        lqw::StageSol<2> nsol;
        double res;
        double t[6];
        auto piece = [&]() {
          // KKT certificate at the piece's end; its start is the previous certified end (same w
          // and r, only the switched coordinate's box changed and it contains the value)
          // (the gradient from the prefix sums of a and b, which the cost quadratics need anyway:
          // y = Ya + gamma Yb, Z = sum_{i<=t} y_i = Za + gamma Zb — two 2-value scans instead of
          // wave_kkt_point's two affine scans over w; the same point up to rounding)
          const double wz = fmin(fmax(fma(bv, best, av), bx.lo), bx.hi);
          lqw::Sums<2> pf;
          pf.v[0] = act ? av : 0.0;
          pf.v[1] = act ? bv : 0.0;
          pf = lqw::wave_scan(pf, N);
          const double Ya = pf.v[0], Yb = pf.v[1];
          {
            lqw::Sums<2> zf;
            zf.v[0] = act ? Ya : 0.0;
            zf.v[1] = act ? Yb : 0.0;
            zf = lqw::wave_scan(zf, N);
            const double y = fma(best, Yb, Ya), Z = fma(best, zf.v[1], zf.v[0]);
            const double Zt = lqw::readlane_d(Z, N - 1);
            const double rr = q.c * (Zt - Z + y - (double)(N - lane) * best) + ws.d_nat * wz + ws.e_nat;
            res = lqw::wave_max(act ? lq_resid(q, bx, wz, rr) : 0.0, N);
          }
          const double Ea = Ya - Ywr, da = av - wr_nat;
          const double dd = ws.d_nat, cc = q.c;
          const double sg = (sl & 1) ? bx.slo : 0.0;  // PWL slope of a free coordinate
          const double wmid = fma(bv, 0.5 * (gcur + best), av);
          const double tw = q.theta * q.w_max;
          // PWL value at w = 0 of its linear piece (large EVs; small EVs have no PWL term)
          const double icpt = q.ev_small ? 0.0 : fma(-sg, wmid, tw * tw * lq_pwl(wmid * q.inv_wmax));
          t[0] = fma(0.5 * cc, Ya * Ya, fma(av, fma(0.5 * dd, av, ee + sg), icpt));
          t[1] = fma(cc, fma(Ya, Yb, -Ya), bv * fma(dd, av, ee + sg));
          t[2] = fma(0.5 * cc, Yb * Yb, fma(-cc, Yb, 0.5 * dd * bv * bv));
          t[3] = fma(Ea, Ea, kappa * da * da);
          t[4] = 2.0 * fma(Ea, Yb, kappa * da * bv);
          t[5] = fma(Yb, Yb, kappa * bv * bv);
#pragma unroll
          for (int k = 0; k < 6; ++k) t[k] = act ? t[k] : 0.0;
          lqw::wave_totals(t, N);
        };
        if (bj >= 0) {  // (wave-uniform) the next solve beside this piece's certificate
          bxn = lq_box(act ? sln : 0);
          nsol = lqw::solve_stage<2>(q, ws, bxn, 0.0, sln);
          piece();
        } else {
          piece();
        }
        if (emit) {
          if (!(res <= q.tol_cert)) break;  // coverage ends at gcur
          if (lane < N) {
            double* dst = reinterpret_cast<double*>(a.t_ab + (sb + npc) * N + lane);
            st_wt8(dst, av);
            st_wt8(dst + 1, bv);
          }
          const double a0 = lqw::readlane_d(av, 0), b0v = lqw::readlane_d(bv, 0);
          if (lane < 8) {
            double v = t[0] + c0;
#pragma unroll
            for (int k = 1; k < 6; ++k) v = lane == k ? t[k] : v;
            v = lane == 6 ? a0 : (lane == 7 ? b0v : v);
            st_wt8(a.t_cf + (sb + npc) * 8 + lane, v);
          }
          if (lane == 0) st_wt8(a.t_ge + sb + npc, best);
          ++npc;
        }
        if (bj < 0) break;
        sl = sln;
        sol = nsol;
        gcur = best;
        last = bj;
      }
    }
  }
  a.t_sl[(size_t)blk * 64 + lane] = (uint8_t)sl0;
  if (lane == 0) {
    __hip_atomic_store(a.t_cnt + blk, npc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    st_wt8(a.t_lo + blk, glo);
  }
  LQ_STAMP(3);
#ifdef LOMPC_STAMPS
  if (lane == 0 && blk < 65536) g_stamps[blk * 8 + 6] = npc;
#endif
}

template <int NT>
__global__ __launch_bounds__(64) void k_path(PathArgs a) {
  if (a.skip && *a.skip) return;
  path_cell<NT, true>(a, (int)blockIdx.x);
}

// forward (defined with k_finalize below)
struct FinalArgs;
template <int NT>
__global__ __launch_bounds__(64) void k_path_fin(PathArgs a, FinalArgs r);

typedef void (*PathKernel)(PathArgs);
typedef void (*PathKernel2)(PathArgs, FinalArgs);
PathKernel path_kernel(int N) {
  switch (N) {
    case 12: return k_path<12>;
    case 16: return k_path<16>;
    case 24: return k_path<24>;
    case 48: return k_path<48>;
    default: return k_path<0>;
  }
}

// ---------------------------------------------------------------- k_eval
struct EvalArgs {
  int S, G, N, want_err;
  const QPConst* qd;
  CtxEnds ce;
  const int4* blk;        // [nblk] (set, first EV, end EV, -): <= EVAL_MAXB EVs of one set
  const int64_t* set_off; // [S+1]
  const double* window;
  const double* gamma;    // caller's [B]
  const double* lmbd;
  const double* lmbd_r;
  const double* w_ref;
  const int* t_cnt;
  const double* t_lo;
  const uint8_t* t_sl;
  const double* t_ge;
  const double* t_cf;
  const double2* t_ab;
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* partial;        // [nblk][N + NPX]
  int* fail_cnt;          // [nblk][EVAL_WAVES]  EVs left for the individual re-solve (k_finalize)
  int* fail_idx;          // [nblk][EVAL_MAXB]   their indices, per wave in row order
  int w_rsrc_ok;          // B*N*8 <= LQ_DROP_OFF: w through a buffer descriptor (offsets from 0)
  int w_bytes;            // B*N*8 when w_rsrc_ok (the descriptor's range)
  int cap;                // pieces staged in LDS (a set with more re-solves the rest individually)
  int nblk;               // workgroups of EVs (close mode: workgroup nblk closes the empty sets)
  const int* skip;        // device-resident price loop: nonzero = the loop has finished, run nothing
  int piece_sums;         // (k_evals, no w output) per-stage sums from per-piece aggregates, no rows
};

// cost / A_bar error / price0 of a QP solved by the whole wave (lane t = w_t), valid on every lane
__device__ __forceinline__ void wave_ev_outputs(const QPConst& q, const lqw::WaveSet& ws, double c0, double kappa,
                                                const double* l0, double lr, double wr, double gamma, double w,
                                                double& cost, double& err, double& price0) {
  const int N = ws.N, lane = ws.lane;
  const bool act = lane < N;
  lqw::Aff<2> h = lqw::Aff<2>::identity();
  if (act) {
    h.B[0] = w;
    h.B[1] = w - wr;
  }
  const lqw::Aff<2> Y = lqw::wave_scan(h, N);
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  if (act) {
    const double y = Y.B[0], ey = Y.B[1];
    v[0] = 0.5 * q.c * y * y - q.c * gamma * y + w * fma(0.5 * ws.d_nat, w, ws.e_nat);
    v[1] = ey * ey;
    v[2] = (w - wr) * (w - wr);
    v[3] = q.ev_small ? 0.0 : lq_pwl(w * q.inv_wmax);
  }
  lqw::wave_totals(v, N);
  const double tw = q.theta * q.w_max;
  cost = v[0] + c0 + tw * tw * v[3];
  err = sqrt(fmax(v[1] + kappa * v[2], 0.0));
  const double w0 = lqw::readlane_d(w, 0);
  price0 = q.theta * (w0 * l0[0] + (q.w_max - w0) * l0[1]) + q.q_scale * w0 * w0 * l0[2] +
           q.theta * q.theta * w0 * w0 * lr;
}

// loads of k_eval's records: plain after a kernel boundary (k_finalize), device-coherent (sc1, past
// any stale L2 line of this XCD) when other workgroups of the same launch wrote them (close mode)
template <bool COH>
__device__ __forceinline__ double ld_t(const double* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool COH>
__device__ __forceinline__ int ld_t(const int* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}
template <bool COH>
__device__ __forceinline__ double2 ld_t(const double2* p) {
  if constexpr (COH) {
    const double* d = reinterpret_cast<const double*>(p);
    return make_double2(ld_t<true>(d), ld_t<true>(d + 1));
  } else {
    return *p;
  }
}

struct FinalArgs {
  int N, G, want_err;
  unsigned long long* tally;  // [3] plan-wide repaired / failed / invalid since the last status read (or null)
  const int* skip;            // device-resident price loop: nonzero = the loop has finished
  int* arrive;             // [S] k_eval (close mode): arrived workgroups per set, zero between runs
  const QPConst* qd;
  CtxEnds ce;
  const int* blk_prefix;   // [S+1] k_eval workgroups of each set
  const int64_t* set_off;
  const double* window;
  const double* gamma;
  const double* lmbd;
  const double* lmbd_r;
  const double* w_ref;
  const uint8_t* t_sl;
  const int* fail_cnt;
  const int* fail_idx;
  const double* partial;
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* set_sum_w;
  double* set_stats;
  double* stats;
};

constexpr int FIN_W = LOMPC_MAX_N + NPX + 1;

// Closing of set s by one workgroup of NW waves (k_finalize: one 4-wave workgroup per set; k_eval
// in close mode and k_step: 8 waves; k_path_fin: one wave; COH = records read with sc1 loads when
// other workgroups of the same launch wrote them).  The summation order does not depend on NW, so
// every form of a run gives the same bits: records (and re-solve lists) fall into LQ_FIN_CLASSES
// classes by their index mod 4, each class summed in increasing index by one wave, the classes
// combined as ((c0 + c1) + c2) + c3.
// (1) reduction of the set's k_eval records (lane = column);
// (2) if k_eval listed EVs no certified piece covers: the lists of waves (workgroup, wave) are
//     re-solved individually (wave_solve from the working set at their cell's start: fp32 search,
//     fp64 PDAS, primal active set; KKT-certified), their outputs written and added by class.
#define LQ_FIN_CLASSES 4
template <int NW, bool COH>
__device__ __forceinline__ void finalize_set(const FinalArgs& r, const int s, double (*red)[FIN_W], double (*rep)[FIN_W]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int N = r.N, W = N + NPX;
  const int b0 = r.blk_prefix[s], b1 = r.blk_prefix[s + 1];
  constexpr int NC = LQ_FIN_CLASSES;
  for (int cl = wv; cl < NC; cl += NW) {
    for (int c = lane; c < W; c += 64) {
      const bool is_max = c == N + PX_MAX_ERR;
      double acc = 0.0;
      constexpr int U = 8;
      for (int b = b0 + cl; b < b1; b += NC * U) {
        double v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int bb = b + NC * u;
          v[u] = bb < b1 ? ld_t<COH>(r.partial + (size_t)bb * W + c) : 0.0;  // 0: neutral for sums and max of errors >= 0
        }
#pragma unroll
        for (int u = 0; u < U; ++u) acc = is_max ? fmax(acc, v[u]) : acc + v[u];
      }
      red[cl][c] = acc;
    }
  }
  __syncthreads();
  for (int c = tid; c < W; c += 64 * NW) {
    const bool is_max = c == N + PX_MAX_ERR;
    double v = red[0][c];
#pragma unroll
    for (int k = 1; k < NC; ++k) v = is_max ? fmax(v, red[k][c]) : v + red[k][c];
    red[0][c] = v;
  }
  __syncthreads();
  if (red[0][N + PX_N_FAILED] > 0.0) {  // block-uniform: individual re-solves pending
    const QPConst& q = set_consts(r.qd, r.ce, s);
    lq_tab_init(q);
    const double* __restrict__ L = r.lmbd + (size_t)s * 3 * N;
    const double lr = r.lmbd_r[s];
    lqw::WaveSet ws;
    double l2;
    bool bad;  // (checked by k_path)
    load_set(q, L, lr, N, lane, ws, l2, bad);
    const double c0 = q.theta * q.w_max * lqw::wave_sum(l2, N);
    const double kappa = lr / q.delta;
    const double l0[3] = {L[0], L[N], L[2 * N]};
    const double wr = (r.w_ref && lane < N) ? r.w_ref[(size_t)s * N + lane] : 0.0;
    const double wlo = r.window[2 * s], whi = r.window[2 * s + 1];
    const int G = r.G;
    for (int cl = wv; cl < NC; cl += NW) {
      double acc_w = 0.0, acc_cost = 0.0, acc_p0 = 0.0, acc_err = 0.0;
      int nrep = 0, nfail = 0;
      for (int j = b0 * EVAL_WAVES + cl; j < b1 * EVAL_WAVES; j += NC) {  // (workgroup, wave) lists of class cl
        const int nf = ld_t<COH>(r.fail_cnt + j);
        for (int k = 0; k < nf; ++k) {
          const int i = ld_t<COH>(r.fail_idx + (size_t)(j / EVAL_WAVES) * EVAL_MAXB + 64 * EVAL_PASSES * (j % EVAL_WAVES) + k);
          const double g = r.gamma[i];
          const int c = cell_of(g, wlo, (double)G / (whi - wlo), G);
          int sl = lane < N ? (int)r.t_sl[((size_t)s * G + c) * 64 + lane] : 0;
          double wl = 0.0, rl = 0.0;
          const bool okk = lqw::wave_solve(q, ws, g, sl, wl, rl);
          double co, eo, po;
          wave_ev_outputs(q, ws, c0, kappa, l0, lr, wr, g, wl, co, eo, po);
          if (!r.want_err) eo = 0.0;
          if (r.w && lane < N) r.w[(size_t)i * N + lane] = wl;
          if (lane == 0) {
            if (r.cost) r.cost[i] = co;
            if (r.w0) r.w0[i] = wl;
            if (r.status) r.status[i] = okk ? LOMPC_QP_REPAIRED : LOMPC_QP_FAILED;
          }
          acc_w += lane < N ? wl : 0.0;
          acc_cost += co;
          acc_p0 += po;
          acc_err = fmax(acc_err, eo);
          nrep += okk ? 1 : 0;
          nfail += okk ? 0 : 1;
        }
      }
      if (lane < N) rep[cl][lane] = acc_w;
      if (lane == 0) {
        rep[cl][N + PX_COST] = acc_cost;
        rep[cl][N + PX_PRICE0] = acc_p0;
        rep[cl][N + PX_MAX_ERR] = acc_err;
        rep[cl][N + PX_N_OK] = (double)nrep;
        rep[cl][N + PX_N_REPAIRED] = (double)nrep;
        rep[cl][N + PX_N_FAILED] = (double)nfail;
        rep[cl][N + PX_N_INVALID] = 0.0;
      }
    }
    __syncthreads();
    for (int c = tid; c < W; c += 64 * NW) {
      const bool is_max = c == N + PX_MAX_ERR;
      double v = (c == N + PX_N_FAILED) ? 0.0 : red[0][c];  // pending -> the outcome
#pragma unroll
      for (int k = 0; k < NC; ++k) v = is_max ? fmax(v, rep[k][c]) : v + rep[k][c];
      red[0][c] = v;
    }
    __syncthreads();
  }
  if (tid == 0 && r.tally) {  // sticky plan-wide counters (lompc_plan_status): one atomic per nonzero count
    const double nr = red[0][N + PX_N_REPAIRED], nf = red[0][N + PX_N_FAILED], ni = red[0][N + PX_N_INVALID];
    if (nr > 0.0) __hip_atomic_fetch_add(r.tally + 0, (unsigned long long)nr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (nf > 0.0) __hip_atomic_fetch_add(r.tally + 1, (unsigned long long)nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ni > 0.0) __hip_atomic_fetch_add(r.tally + 2, (unsigned long long)ni, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
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
    if (r.stats) r.stats[(size_t)s * LOMPC_SET_STATS + tid] = v;
  }
}


__global__ __launch_bounds__(256) void k_finalize(FinalArgs r) {
  __shared__ double red[LQ_FIN_CLASSES][FIN_W];
  __shared__ double rep[LQ_FIN_CLASSES][FIN_W];
  if (r.skip && *r.skip) return;
  finalize_set<4, false>(r, (int)blockIdx.x, red, rep);
}

// lompc_plan_run_steps: run k's path (workgroups [0, S G)) and run k - 1's closing (one one-wave
// workgroup per set after them) in ONE launch — the two are independent (run k - 1's records
// are complete at the kernel boundary behind its k_eval; run k's path writes the other half of
// the cell-start working sets the closing's individual re-solves read), so every run after the
// first costs two launches instead of three.
template <int NT>
__global__ __launch_bounds__(64) void k_path_fin(PathArgs a, FinalArgs r) {
  const int b = (int)blockIdx.x, nc = a.S * a.G;
  if (b < nc) {
    path_cell<NT, true>(a, b);
  } else {
    __shared__ double red[LQ_FIN_CLASSES][FIN_W];
    __shared__ double rep[LQ_FIN_CLASSES][FIN_W];
    finalize_set<1, false>(r, b - nc, red, rep);
  }
}

PathKernel2 path_fin_kernel(int N) {
  switch (N) {
    case 12: return k_path_fin<12>;
    case 16: return k_path_fin<16>;
    case 24: return k_path_fin<24>;
    case 48: return k_path_fin<48>;
    default: return k_path_fin<0>;
  }
}

// Plans with a communicator: the all-gathered records recv[rank][S (N + 8)] of every rank combined
// in rank order — sums, max for LOMPC_STAT_MAX_ERR — into the caller's set outputs (either may be
// null).  Every rank runs the same arithmetic on the same bytes: the results are bitwise equal.
__global__ __launch_bounds__(256) void k_combine(const double* __restrict__ recv, int nranks, int S, int N,
                                                 double* set_sum_w, double* set_stats) {
  const int SN = S * N, L = S * (N + LOMPC_SET_STATS);
  for (int c = (int)(blockIdx.x * 256 + threadIdx.x); c < L; c += (int)(gridDim.x * 256)) {
    const bool is_max = c >= SN && (c - SN) % LOMPC_SET_STATS == LOMPC_STAT_MAX_ERR;
    double v = recv[c];
    for (int k = 1; k < nranks; ++k) {
      const double x = recv[(size_t)k * L + c];
      v = is_max ? fmax(v, x) : v + x;
    }
    if (c < SN) {
      if (set_sum_w) set_sum_w[c] = v;
    } else if (set_stats) {
      set_stats[c - SN] = v;
    }
  }
}

// The wide form's exchange for a group of n runs (one all-gather of the n runs' packed records):
// recv[rank][n][S (N + 8)]; run r's records combined in rank order as k_combine does, into the run's
// set outputs at (run0 + r) * stride (stride 0: shared outputs, only run `last` writes them)
struct CombineRunsArgs {
  const double* recv;
  int nranks, n, S, N, run0, last;
  double* set_sum_w;
  double* set_stats;
  int64_t sw_stride, st_stride;
};
__global__ __launch_bounds__(256) void k_combine_runs(CombineRunsArgs a) {
  const int SN = a.S * a.N, L = a.S * (a.N + LOMPC_SET_STATS);
  const int64_t tot = (int64_t)a.n * L;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (int64_t)gridDim.x * 256) {
    const int r = (int)(e / L), c = (int)(e - (int64_t)r * L), j = a.run0 + r;
    const bool is_max = c >= SN && (c - SN) % LOMPC_SET_STATS == LOMPC_STAT_MAX_ERR;
    double v = a.recv[(size_t)r * L + c];
    for (int k = 1; k < a.nranks; ++k) {
      const double x = a.recv[((size_t)k * a.n + r) * L + c];
      v = is_max ? fmax(v, x) : v + x;
    }
    if (c < SN) {
      if (a.set_sum_w && (a.sw_stride || j == a.last)) a.set_sum_w[(size_t)j * a.sw_stride + c] = v;
    } else if (a.set_stats && (a.st_stride || j == a.last)) {
      a.set_stats[(size_t)j * a.st_stride + c - SN] = v;
    }
  }
}

// lompc_plan_run_chain: run k's prices from run k - 1's closed set reductions (the dependence of the
// reference's price iterations, price_solver.py:111-140): one workgroup per set, lane = price
// coordinate i = seg N + t,
//   lmbd_k[i] = max(0, lmbd_{k-1}[i] + step (phi(wbar)[i] - phi(w_target)[i])),  wbar = sum_w / count
// with phi = (theta w, theta (w_max - w), q_s w^2) (lompc.py:172-177) of the set's EV type.  A set
// without EVs keeps its prices.
__global__ __launch_bounds__(256) void k_chain_price(const QPConst* __restrict__ q, CtxEnds ce, int nctx, int N,
                                                     const double* __restrict__ prev, const double* __restrict__ sum_w,
                                                     const double* __restrict__ stats,
                                                     const double* __restrict__ target, double step,
                                                     double* __restrict__ next) {
  const int s = blockIdx.x;
  int k = 0;
  while (k + 1 < nctx && s >= ce.end[k]) ++k;
  const double th = q[k].theta, wm = q[k].w_max, qs = q[k].q_scale;
  const double n = stats[(size_t)s * LOMPC_SET_STATS + LOMPC_STAT_COUNT];
  for (int i = threadIdx.x; i < 3 * N; i += blockDim.x) {
    const int seg = i / N, t = i - seg * N;
    const double x = prev[(size_t)s * 3 * N + i];
    double v = x;
    if (n > 0) {
      const double wb = sum_w[(size_t)s * N + t] / n, wr = target[(size_t)s * N + t];
      const double g = seg == 0 ? th * (wb - wr) : (seg == 1 ? th * ((wm - wb) - (wm - wr)) : qs * (wb * wb - wr * wr));
      v = fmax(0.0, x + step * g);
    }
    next[(size_t)s * 3 * N + i] = v;
  }
}

// One k_eval block (EVs [start, end) of one set, <= EVAL_MAXB) by the whole workgroup.
// NT: the horizon as a compile-time constant (0: a.N at run time) — the row loop's lane map
// (stages per lane, rows per store instruction) and its address arithmetic become constants.
// CLOSE: the set is closed inside the launch (no k_finalize).  The workgroup record is built
// BEFORE the rows: the per-stage sums come from per-piece aggregates (EV count and gamma sum of
// each piece, fixed-point integer LDS atomics: exact and order-free), so wave 0 publishes the
// record and arrives on the set's counter while no row store is in flight, and the other waves
// write all the rows; the set's last arriver closes it (finalize_set) after its rows.  Rows of
// EVs left to the individual re-solve are not written here (key ZD), the closing workgroup writes
// them, so no two writes of a row race.
// k_evals: where one run's tables, records, per-EV outputs and prices sit (offsets from the
// EvalArgs pointers, so a loop over runs keeps one base per array instead of one pointer per run)
struct RunOff {
  int64_t tab = 0;  // cells: the run's path-table ring slot
  int rec = 0;      // blocks: the run's record slot
  int64_t ev = 0;   // EVs: per-run per-EV outputs
  const double* lmbd = nullptr;    // (null: a.lmbd / a.lmbd_r)
  const double* lmbd_r = nullptr;
  bool launder = false;
  bool gamma_lds = false;  // the block's gamma from the previous run's s_g (k_evals: the same EVs every run)
  bool nostage = false;  // (diagnostic builds, LQ_EVALS_NOSTAGE: keep the previous run's staged table)
  bool pipelined = false;  // (k_evals) staging loads before a barrier, the record by the block's last wave
  bool first = false;      // (k_evals) the launch's first run
  int buf = 0;           // (k_evals_st) the compact table and the record scratch of this run: parity
};

// k_evals_st's stager: set s's path table of ring offset `tab` into the compact table T, by ONE wave
// (lane c: cell c, G <= 64).  The cells' counts and coverage starts in one memory round, their prefix
// by a wave scan (cells from the first whose pieces pass `capc` on: none staged), then the pieces LQ_STG_CHUNK at
// a time: one load per piece (lanes t < N its row, lanes N .. N + 3 its coefficient record in 16-B
// quarters) and one for the 8 pieces' ends, each piece's cell from a ballot over the cells' ends.
__device__ __forceinline__ void stage_compact(const EvalArgs& a, const int s, const int64_t tab, const CTab T,
                                           const int N, const int G, const int capc, const int lane) {
  const int64_t cb = tab + (int64_t)s * G;
  int cn = 0;
  double cl = 0.0;
  if (lane < G) {
    cn = min(max(ld_t<false>(a.t_cnt + cb + lane), 0), LQ_PPL);
    cl = ld_t<false>(a.t_lo + cb + lane);
  }
  int incl = cn;  // inclusive prefix of the counts over the cells
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int y = __shfl_up(incl, d, 64);
    if (lane >= d) incl += y;
  }
  const bool fit = incl <= capc;
  const int ends = fit ? incl : 0x7fffffff;  // (an unstaged cell ends past every staged piece)
  const int pre = incl - cn;
  int np = fit ? incl : 0, mx = fit ? cn : 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    np = max(np, __shfl_xor(np, d, 64));
    mx = max(mx, __shfl_xor(mx, d, 64));
  }
  if (lane < G) {
    T.cnt[lane] = fit ? cn : 0;
    T.pre[lane] = pre;
    T.lo[lane] = cl;
  }
  if (lane == 0) {
    T.meta[0] = mx;
    T.meta[1] = np;
  }
  const int NS = eval_row_stride(N);
  const size_t sb = (size_t)cb * LQ_PPL;
  for (int p0 = 0; p0 < np; p0 += LQ_STG_CHUNK) {
    double2 v[LQ_STG_CHUNK];
    int sl = 0;  // lane u < LQ_STG_CHUNK: the slot of piece p0 + u
#pragma unroll
    for (int u = 0; u < LQ_STG_CHUNK; ++u) {
      const int p = p0 + u;
      const int c = __popcll(__ballot(lane < G && ends <= p));  // cells wholly before piece p
      const int slot = c * LQ_PPL + p - __builtin_amdgcn_readlane(pre, min(c, 63));
      if (lane == u) sl = slot;
      const double2* src = lane < N ? a.t_ab + (sb + slot) * N + lane
                                    : reinterpret_cast<const double2*>(a.t_cf + (sb + slot) * 8) + (lane - N);
      v[u] = p < np && lane < N + 4 ? ld_t<false>(src) : make_double2(0.0, 0.0);
    }
    const double vg = lane < LQ_STG_CHUNK && p0 + lane < np ? ld_t<false>(a.t_ge + sb + sl) : 0.0;
#pragma unroll
    for (int u = 0; u < LQ_STG_CHUNK; ++u) {
      const int p = p0 + u;
      if (p < np) {
        if (lane < N) T.ab[p * NS + ((N & 1) ? lane : (lane & 1) * (N >> 1) + (lane >> 1))] = v[u];
        else if (lane < N + 4) *reinterpret_cast<double2*>(T.cf + cfx(p, 2 * (lane - N))) = v[u];
      }
    }
    if (lane < LQ_STG_CHUNK && p0 + lane < np) T.ge[p0 + lane] = vg;
  }
}

// STG (k_evals_st): waves 0 .. LQ_EVALS_RW - 1 only, the table already staged (compact, LDS table
// ro.buf), EVs in one contiguous segment per wave (its passes: 64 rows each), the row sums and wave
// records into the run's scratch parity — no barrier inside: the caller's one barrier per run orders
// the table, the rows and the record.
template <int NT = 0, bool CLOSE = false, bool STG = false>
__device__ __forceinline__ void eval_block(const EvalArgs& a, const int blk, const FinalArgs* fr = nullptr,
                                           const RunOff ro = RunOff{}) {
  static_assert(!(STG && CLOSE), "the staged form has no in-launch closing");
  // dynamic LDS: [cap + 2][NS] piece rows (rows cap, cap + 1: zero pieces) | [cap][8]
  // coefficients (cfx) | [LQ_PPL][Gs] piece ends | cells: coverage start | piece count | (CLOSE) per
  // piece: gamma sum, EV count.  Laid out for the banks (64 dwords for ds_read_b64 / b128): a
  // piece row holds its even stages, then its odd ones (even N: the row phase's two 16-B reads
  // per lane are contiguous across a row's lanes, not 32 B apart), and rows, coefficient records
  // and piece ends are padded / swizzled / transposed so that lanes reading different pieces or cells
  // spread over the banks instead of landing on the same few
  extern __shared__ __attribute__((aligned(16))) double2 s_dyn[];
  __shared__ double s_g[EVAL_MAXB];  // block row r = EV start + r: gamma
  __shared__ int s_k[EVAL_MAXB];     //   its piece (ZK / ZD: zero pieces)
  __shared__ double s_accw[EVAL_WAVES][LOMPC_MAX_N];  // per-wave row sums per stage
  __shared__ double s_red[EVAL_WAVES][8];
  __shared__ int s_fc[EVAL_WAVES];  // (CLOSE) re-solve list lengths
  __shared__ int s_last;            // (CLOSE) this workgroup closes the set
  __shared__ int s_mx;              // the set's largest piece count of a cell
  __shared__ int s_done;            // (pipelined) waves past their rows, this run
  int tid_ = (int)threadIdx.x;
  if (ro.launder) asm volatile("" : "+v"(tid_));  // (k_evals: lane-derived indices recomputed every run, not
                                                  // hoisted out of its loop and spilled)
  const int tid = tid_, lane = tid & 63, wv = tid >> 6;
  const int4 info = a.blk[blk];
  const int rb = ro.rec + blk;  // this block's record (k_evals: in its run's record slot)
  // per-EV outputs (k_evals with per-run outputs: at the run's offset)
  double* const aw = a.w ? a.w + ro.ev * (NT ? NT : a.N) : nullptr;
  double* const acost = a.cost ? a.cost + ro.ev : nullptr;
  double* const aw0 = a.w0 ? a.w0 + ro.ev : nullptr;
  int8_t* const astatus = a.status ? a.status + ro.ev : nullptr;
  const int s = info.x, start = info.y, end = info.z;  // thread: EVs start + tid + EVAL_EVS h
  // (STG: wave wv's EVs are block rows sg0 .. sg0 + sgn - 1, lane + 64 h in pass h)
  const int sg_per = STG ? (end - start + LQ_EVALS_RW - 1) / LQ_EVALS_RW : 0;
  const int sg0 = STG ? wv * sg_per : 0;
  const int sgn = STG ? max(0, min(sg_per, end - start - sg0)) : 0;
  auto brow = [&](const int h) { return STG ? sg0 + 64 * h + lane : tid + EVAL_EVS * h; };  // block row of pass h
  auto bact = [&](const int h) { return STG ? 64 * h + lane < sgn : start + tid + EVAL_EVS * h < end; };
  LQ_STAMPW(6);  // (diagnostic build: the block map's load round)
  int G_ = a.G, cap_ = a.cap;
  if (ro.launder) asm volatile("" : "+s"(G_), "+s"(cap_));  // (k_evals: the LDS layout per run, as tid)
  const int N = NT ? NT : a.N, G = G_;
  const int cap = cap_;
  const int ZK = cap;      // the zero piece (a = b = 0): rows of invalid (and, without CLOSE,
                           // re-solved) EVs, which then add exactly 0 to the row sums and need no
                           // branch in the row loop
  const int ZD = cap + 1;  // (CLOSE) zero piece whose row is not written: re-solved EVs
  // (k_evals of a run with no w output: the set's per-stage sums from per-piece EV counts and
  // fixed-point gamma sums — sum_p n_p a_p + Gamma_p b_p, unclamped, as the close mode and k_agg —
  // instead of evaluating and summing every EV's N rows that are never stored)
  const bool psum = !CLOSE && !STG && ro.pipelined && a.piece_sums && !aw;
  LQ_STAMPE(0);
  LQ_WSTART();
  const int NS = eval_row_stride(N);
  // LDS index of stage t of piece row k
  auto abx = [&](const int k, const int t) { return k * NS + ((N & 1) ? t : (t & 1) * (N >> 1) + (t >> 1)); };
  double2* s_ab = s_dyn;
  double* s_cf = reinterpret_cast<double*>(s_ab + (size_t)(cap + 2) * NS);
  double* s_ge = s_cf + (size_t)cap * 8;
  double* s_lo = s_ge + cap;
  int* s_cnt = reinterpret_cast<int*>(s_lo + G);
  int* s_pre = nullptr;  // (STG: a cell's first slot)
  int stg_meta[2] = {0, 0};
  if constexpr (STG) {
    const CTab T = ctab_at(reinterpret_cast<char*>(s_dyn) + (size_t)ro.buf * ctab_bytes(N, G, cap), N, G, cap);
    s_ab = T.ab;
    s_cf = T.cf;
    s_ge = T.ge;
    s_lo = T.lo;
    s_cnt = T.cnt;
    s_pre = T.pre;
    stg_meta[0] = T.meta[0];
    stg_meta[1] = T.meta[1];
  }
  unsigned long long* s_pf = reinterpret_cast<unsigned long long*>(s_cnt + ((G + 1) & ~1));
  int* s_pn = reinterpret_cast<int*>(s_pf + cap + 2);
  const int np = STG ? stg_meta[1] : min(G * LQ_PPL, cap);
  const int Gs = STG ? G : np / LQ_PPL;  // cells with staged pieces (the rest are re-solved)
  // staged cells per wave (wv, wv + W, ...) and piece-row loads per lane and cell
  constexpr int CPW = (LQ_PIECE_CAP / LQ_PPL + EVAL_WAVES - 1) / EVAL_WAVES;
  constexpr int UA = ((NT ? NT : LOMPC_MAX_N) * LQ_PPL + 63) / 64;
  int wc = 0;  // lane j < CPW: piece count of cell wv + W j
  if (!STG && lane < CPW && wv + EVAL_WAVES * lane < Gs)
    wc = ld_t<false>(a.t_cnt + ro.tab + (size_t)s * G + wv + EVAL_WAVES * lane);
  // this thread's EVs (caller order)
  double gh[EVAL_PASSES];
#pragma unroll
  for (int h = 0; h < EVAL_PASSES; ++h) {  // (k_evals after its first run: from LDS, no memory round
    const int i = start + brow(h);            //  queued behind the previous run's row stores)
    gh[h] = ro.gamma_lds ? s_g[brow(h)] : bact(h) ? a.gamma[i] : 0.0;
  }
  const QPConst& q = set_consts(a.qd, a.ce, s);
  double wlo = a.window[2 * s], whi = a.window[2 * s + 1];
  const double* __restrict__ L = (ro.lmbd ? ro.lmbd : a.lmbd) + (size_t)s * 3 * N;
  double l0[3] = {L[0], L[N], L[2 * N]};  // price0 (lompc.py:164-170)
  double lr = (ro.lmbd_r ? ro.lmbd_r : a.lmbd_r)[s];
  const int64_t cb = ro.tab + (int64_t)s * G;  // the set's first cell in the table
  // the set's USED piece slots (a cell's first t_cnt of its LQ_PPL; cells past the first `cap`
  // slots are re-solved individually) and the cells' counts / coverage starts.  Two memory rounds,
  // both wave-local (no barrier): each wave reads the counts of the cells whose pieces it stages
  // (issued before the gamma loads, above), then only those cells' used rows, coefficient records
  // and piece ends — cells hold 1-2 pieces on average, so this moves a fraction of the 8 slots
  const size_t sb = (size_t)cb * LQ_PPL;
  if (ro.pipelined && ro.first && tid == 0) s_done = 0;  // (published by the staging barriers)
  if constexpr (!STG) if (!ro.nostage) {  // (STG: staged by the stager wave)
    int vn = 0;
    double vl = 0.0;
    if (tid < G) {
      vn = ld_t<false>(a.t_cnt + cb + tid);
      vl = ld_t<false>(a.t_lo + cb + tid);
    }
    // the set's constants and this workgroup's scalars land with this round, not after the
    // staging (scalar loads are otherwise issued at first use, each a memory round of its own)
    lq_tab_fill(q);  // (published by the barrier below)
    lq_pin(wlo);
    lq_pin(whi);
    lq_pin(l0[0]);
    lq_pin(l0[1]);
    lq_pin(l0[2]);
    lq_pin(lr);
    LQ_STAMPW(2);  // (diagnostic build: counts, gamma and the cells' loads)
    double2 v[CPW][UA];
    double vc[CPW], vg[CPW];
    int nc[CPW];
#pragma unroll
    for (int j = 0; j < CPW; ++j)  // (every count read before any piece load is issued; a lane of
      nc[j] = min(max(lqw::readlane_i(wc, j), 0), LQ_PPL);  //  a cell past Gs loaded 0)
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c = wv + EVAL_WAVES * j;
      const size_t so = sb + (size_t)c * LQ_PPL;  // the cell's first slot
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int it = lane + 64 * u;
        v[j][u] = it < nc[j] * N ? ld_t<false>(a.t_ab + so * N + it) : make_double2(0.0, 0.0);
      }
      vc[j] = lane < nc[j] * 8 ? ld_t<false>(a.t_cf + so * 8 + lane) : 0.0;
      vg[j] = lane < nc[j] ? ld_t<false>(a.t_ge + so + lane) : 0.0;
    }
    LQ_STAMPW(3);  // (diagnostic build: the pieces' load round)
    // (k_evals: the loads above were issued while other waves may still write the previous run's rows
    // from the table; the LDS writes below wait until every wave is past them)
    if (ro.pipelined) __syncthreads();
#pragma unroll
    for (int j = 0; j < CPW; ++j) {
      const int c = wv + EVAL_WAVES * j;
#pragma unroll
      for (int u = 0; u < UA; ++u) {
        const int it = lane + 64 * u;
        if (it < nc[j] * N) {
          const int k = it / N;
          s_ab[abx(c * LQ_PPL + k, it - k * N)] = v[j][u];
        }
      }
      if (lane < nc[j] * 8) s_cf[cfx(c * LQ_PPL + (lane >> 3), lane & 7)] = vc[j];
      if (lane < nc[j]) s_ge[lane * Gs + c] = vg[j];
    }
    if (tid < G) {
      s_cnt[tid] = vn;
      s_lo[tid] = vl;
    }
    if (wv == 0) {  // the set's largest cell piece count: the lookup reads no piece end past it
      const double m = lqw::wave_max(tid < G ? (double)vn : 0.0, 64);
      if (lane == 0) s_mx = G <= 64 ? (int)m : LQ_PPL;
    }
    if (tid < 2 * NS) s_ab[ZK * NS + tid] = make_double2(0.0, 0.0);  // both zero pieces
    if ((CLOSE || psum) && tid < cap + 2) {
      s_pf[tid] = 0ull;
      s_pn[tid] = 0;
    }
    for (int c = tid + EVAL_EVS; c < G; c += EVAL_EVS) {
      s_cnt[c] = ld_t<false>(a.t_cnt + cb + c);
      s_lo[c] = ld_t<false>(a.t_lo + cb + c);
    }
  }
  if constexpr (!STG) __syncthreads();  // the staged table and the box table (lq_tab_fill) published
  LQ_STAMPE(1);
  // ---- lane = EV: piece, scalar outputs; EVs no certified piece covers listed for the
  //      individual re-solve (counted as pending failures until then)
  const double ym = q.y_max, wm = q.w_max;
  const double tt = q.theta * q.theta;
  const double cscale = (double)G / (whi - wlo);
  const double fxs = 0x1p40 / (whi - wlo);  // (CLOSE) gamma - wlo in units of the window / 2^40
  double acc_cost = 0.0, acc_p0 = 0.0, acc_err = 0.0;
  int n_ok = 0, n_fail = 0, n_inv = 0, nlist = 0;
  bool inv_rows = false;  // (wave-uniform) some row of this wave has an invalid gamma
  const int mxc = STG ? stg_meta[0] : s_mx;  // (block-uniform) the set's largest cell piece count: no piece end past it is read
  // one pass of the lookup: this thread's EV h
  // the lookup in two halves: lookup_key (the piece: the rows need only it) and lookup_out (the piece's
  // coefficients -> the scalar outputs), which the row passes run after their rows (its LDS round and
  // stores then follow the row stores instead of holding them back); per pass the piece and flags
  int pk[EVAL_PASSES];
  unsigned pf[EVAL_PASSES];  // bit 0: cov, bit 1: act && !valid
  auto lookup_key = [&](const int h) {
    const int i = start + brow(h);
    const bool act = bact(h);
    const double g = gh[h];
    const bool valid = act && g >= 0.0 && g <= ym;
    const int c = valid ? cell_of(g, wlo, cscale, G) : 0;
    const int nc = s_cnt[c];
    const int kb = STG ? s_pre[c] : c * LQ_PPL, ke = kb + nc;  // the cell's pieces [kb, ke), ascending gamma
    double ge[LQ_PPL];
#pragma unroll
    for (int k = 0; k < LQ_PPL; ++k)
      ge[k] = (k < mxc && !LQ_DIAG_NOLOOKUP) ? s_ge[STG ? kb + k : k * Gs + min(c, Gs - 1)] : 0.0;
    const double glo_c = s_lo[c];
    int key = kb;  // piece = number of piece ends below g (every end read at once, no loop)
    double gend = ge[0];
#pragma unroll
    for (int k = 0; k + 1 < LQ_PPL; ++k) key += (k + 1 < nc && g > ge[k]) ? 1 : 0;
#pragma unroll
    for (int k = 1; k < LQ_PPL; ++k) gend = nc == k + 1 ? ge[k] : gend;  // the last piece's end
    const bool cov = LQ_DIAG_NOLOOKUP ? valid && ke > kb  // (diagnostic timing builds: the cell's first piece)
                                      : valid && ke > kb && (STG || ke <= np) && g >= glo_c && g <= gend;
    pk[h] = key;
    pf[h] = (cov ? 1u : 0u) | ((act && !valid) ? 2u : 0u);
    if (!STG || act) {  // (STG: a pass's lanes past the wave's segment are the next wave's rows)
      s_g[brow(h)] = g;
      s_k[brow(h)] = cov ? key : ((CLOSE && valid) ? ZD : ZK);
    }
    inv_rows |= __ballot(act && !valid) != 0ull;
    const unsigned long long need = __ballot(valid && !cov);
    if (valid && !cov) {
      st_wt4(a.fail_idx + (size_t)rb * EVAL_MAXB + 64 * EVAL_PASSES * wv + nlist +
                 __popcll(need & ((1ull << lane) - 1ull)), i);
      ++n_fail;
    }
    nlist += __popcll(need);
  };
  auto lookup_out = [&](const int h) {
    const int i = start + brow(h);
    const double g = gh[h];
    const int key = pk[h];
    const bool cov = (pf[h] & 1u) != 0u;
    if ((pf[h] & 2u) != 0u) {
      ++n_inv;
      if (acost) st_ev8(acost + i, NAN);
      if (aw0) st_ev8(aw0 + i, NAN);
      if (astatus) astatus[i] = LOMPC_QP_INVALID;
    } else if (cov) {
      const double2 q0 = *reinterpret_cast<const double2*>(s_cf + cfx(key, 0));
      const double2 q1 = *reinterpret_cast<const double2*>(s_cf + cfx(key, 2));
      const double2 q2 = *reinterpret_cast<const double2*>(s_cf + cfx(key, 4));
      const double2 q3 = *reinterpret_cast<const double2*>(s_cf + cfx(key, 6));
      const double4 c0 = make_double4(q0.x, q0.y, q1.x, q1.y), c1 = make_double4(q2.x, q2.y, q3.x, q3.y);
      const double cst = fma(fma(c0.z, g, c0.y), g, c0.x);
      const double e2 = fma(fma(c1.y, g, c1.x), g, c0.w);
      const double er = a.want_err ? fmax(e2, 0.0) : 0.0;  // squared: sqrt of the max at the record
      const double w0v = clampw(fma(c1.w, g, c1.z), wm);
      const double p0 = q.theta * (w0v * l0[0] + (wm - w0v) * l0[1]) + q.q_scale * w0v * w0v * l0[2] +
                        tt * w0v * w0v * lr;  // lompc.py:164-170
      acc_cost += cst;
      acc_p0 += p0;
      acc_err = fmax(acc_err, er);
      ++n_ok;
      if (acost) st_ev8(acost + i, cst);
      if (aw0) st_ev8(aw0 + i, w0v);
      if (astatus) astatus[i] = LOMPC_QP_OK;
      if (CLOSE || psum) {
        atomicAdd(s_pn + key, 1);
        atomicAdd(s_pf + key, (unsigned long long)rint(fmax(g - wlo, 0.0) * fxs));
      }
    }
  };
  auto lookup = [&](const int h) {
    lookup_key(h);
    lookup_out(h);
  };
  // a wave without EVs in a pass skips it (wave-uniform; its rows are never read)
  auto pass_live = [&](const int h) { return STG ? 64 * h < sgn : h == 0 || start + EVAL_EVS * h + 64 * wv < end; };
  if constexpr (CLOSE) {  // (the record is built before the rows: every lookup first)
#pragma unroll
    for (int h = 0; h < EVAL_PASSES; ++h)
      if (pass_live(h)) lookup(h);
  }
  LQ_STAMPE(7);
  // this wave's record and row sums (STG: in the run's parity of the scratch after the two tables)
  double* accw_all;  // [EVAL_WAVES][astr] row sums
  double* red_all;   // [EVAL_WAVES][8] wave records
  int astr;
  if constexpr (STG) {
    double* scr = reinterpret_cast<double*>(reinterpret_cast<char*>(s_dyn) + 2 * ctab_bytes(N, G, cap));
    accw_all = scr + (size_t)ro.buf * EVAL_WAVES * N;
    red_all = scr + (size_t)2 * EVAL_WAVES * N + (size_t)ro.buf * EVAL_WAVES * 8;
    astr = N;
  } else {
    accw_all = &s_accw[0][0];
    red_all = &s_red[0][0];
    astr = LOMPC_MAX_N;
  }
  double* const red_w = red_all + wv * 8;
  double* const accw_w = accw_all + wv * astr;
  // per-wave totals of the scalar outputs
  auto wave_record = [&]() {
    double tot[4] = {acc_cost, acc_p0, (double)n_ok, 0.0};
    lqw::wave_totals(tot, 64);
    const double mx = sqrt(lqw::wave_max(acc_err, 64));  // (sqrt is monotone: max of the roots)
    double cnt[2] = {(double)n_fail, (double)n_inv};
    lqw::wave_totals(cnt, 64);
    if (lane == 0) {
      red_w[PX_COST] = tot[0];
      red_w[PX_PRICE0] = tot[1];
      red_w[PX_MAX_ERR] = mx;
      red_w[PX_N_OK] = tot[2];
      red_w[PX_N_REPAIRED] = tot[3];
      red_w[PX_N_FAILED] = cnt[0];
      red_w[PX_N_INVALID] = cnt[1];
    }
  };
  // the workgroup record (fixed-order combination of the waves'), by the threads of `lanes`
  auto store_record = [&](int t, int nthreads) {
    double* part = a.partial + (size_t)rb * (N + NPX);
    for (int c = t; c < N + NPX; c += nthreads) {
      double v = 0.0;
      if (c < N) {
        for (int k = 0; k < EVAL_WAVES; ++k) v += accw_all[k * astr + c];
      } else {
        const int x = c - N;
        for (int k = 0; k < EVAL_WAVES; ++k) v = x == PX_MAX_ERR ? fmax(v, red_all[k * 8 + x]) : v + red_all[k * 8 + x];
      }
      st_wt8(part + c, v);
    }
  };
  bool any_inv = inv_rows;  // (CLOSE: the block's; else this wave's own rows)
  if constexpr (CLOSE) {
    if (lane == 0) s_fc[wv] = nlist;
    if (nlist > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's re-solve list has landed
    __syncthreads();  // every row's key, the piece aggregates and the list lengths complete
    // per-stage sums of the block's rows: sum over pieces p of n_p a_t + Gamma_p b_t, pieces
    // p = wv, wv + W, ... by wave wv (lane = stage), the waves combined in a fixed order
    const double fxi = (whi - wlo) * 0x1p-40;
    double accs = 0.0;
    constexpr int PU = (LQ_PIECE_CAP + EVAL_WAVES - 1) / EVAL_WAVES;
    for (int p0 = wv; p0 < np; p0 += EVAL_WAVES * PU) {  // (one iteration for np <= LQ_PIECE_CAP)
      int n[PU];
      unsigned long long f[PU];
      double2 ab[PU];
#pragma unroll
      for (int k = 0; k < PU; ++k) {  // every read of the batch in flight together
        const int p = p0 + EVAL_WAVES * k;
        const int pc = min(p, np - 1);
        n[k] = p < np ? s_pn[pc] : 0;
        f[k] = s_pf[pc];
        ab[k] = s_ab[abx(pc, min(lane, N - 1))];
      }
#pragma unroll
      for (int k = 0; k < PU; ++k) {
        // (n = 0: an unused slot, whose row is not read into the sum)
        const double gsum = fma((double)f[k], fxi, (double)n[k] * wlo);
        accs = fma((double)n[k], n[k] ? ab[k].x : 0.0, accs);
        accs = fma(n[k] ? gsum : 0.0, n[k] ? ab[k].y : 0.0, accs);
      }
    }
    if (lane < N) s_accw[wv][lane] = accs;
    wave_record();
    __syncthreads();
    any_inv = false;
    for (int k = 0; k < EVAL_WAVES; ++k) any_inv |= s_red[k][PX_N_INVALID] > 0.0;
    if (wv == 0) {  // publish the record, then arrive (nothing but the lookup's stores in flight)
      store_record(lane, 64);
      if (lane < EVAL_WAVES) st_wt4(a.fail_cnt + (size_t)rb * EVAL_WAVES + lane, s_fc[lane]);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) {
        const int nb = fr->blk_prefix[s + 1] - fr->blk_prefix[s];
        const int old = __hip_atomic_fetch_add(fr->arrive + s, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_last = old == nb - 1;
        if (old == nb - 1) __hip_atomic_store(fr->arrive + s, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  // ---- rows (lane = stage pair): w_t = a_t + b_t gamma of the EV's piece -> contiguous rows
  const int V = (N & 1) ? 1 : 2;  // stages per lane (16-B stores for even N)
  const int Lr = N / V;           // lanes per row
  const int R = 64 / Lr;          // rows per store instruction
  const int rr = lane / Lr, col = lane - rr * Lr;
  const bool rlane = rr < R;
  const int t0 = V * col;
  constexpr int RU = EVAL_RU;  // row instructions per batch: their LDS reads in flight together
  double acc0 = 0.0, acc1 = 0.0;
  // a segment of the block's rows r0b .. r0b + nrows - 1 (EVs start + r, contiguous in w): every
  // row is a plain piece lookup (re-solved and invalid EVs read a zero piece), so the loop has
  // no per-row branch: the stores of a full batch use one address register and immediate
  // offsets; lanes past the row width (rlane false) store out of the descriptor's range, which
  // drops them
  const bool fast = aw && a.w_rsrc_ok;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(aw, (short)0, aw ? a.w_bytes : 0, 0x00020000);
  auto row_segment = [&](const int r0b, const int nrows) {
    const int* sk = s_k + r0b;
    const double* sg = s_g + r0b;
    const int rbase = start + r0b;
    const int vb = rlane ? ((rbase + rr) * N + t0) * 8 : LQ_DROP_OFF;  // row rr of the segment
    int kk[RU];
    double gg[RU];
#pragma unroll
    for (int j = 0; j < RU; ++j) {
      const int rc = min(j * R + rr, nrows - 1);
      kk[j] = sk[rc];
      gg[j] = sg[rc];
    }
    for (int r0 = 0; r0 < nrows; r0 += RU * R) {
      double2 u0[RU], u1[RU];
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        if (LQ_DIAG_NOROWLDS) {  // (diagnostic timing builds: no LDS reads in the rows)
          u0[j] = make_double2(1e-3 * kk[j], 1e-3);
          u1[j] = make_double2(2e-3 * kk[j], 1e-3);
        } else {
          u0[j] = s_ab[kk[j] * NS + col];  // stages t0, t0 + 1 (abx)
          u1[j] = V == 2 ? s_ab[kk[j] * NS + (N >> 1) + col] : make_double2(0.0, 0.0);
        }
      }
      int kn[RU];  // the next batch's keys and gammas (software pipeline: one LDS round per batch)
      double gn[RU];
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        const int rc = min(r0 + (RU + j) * R + rr, nrows - 1);
        kn[j] = sk[rc];
        gn[j] = sg[rc];
      }
      // a batch's row math and stores; FULL (every row of the batch exists and is written: no
      // per-row masks) and FAST (w through the descriptor: one address register, immediate
      // offsets) are wave-uniform and specialised so the common case has no exec-mask change
      auto rows = [&](auto full_t, auto fast_t) {
        constexpr bool FULL = decltype(full_t)::value, FAST = decltype(fast_t)::value;
#pragma unroll
        for (int j = 0; j < RU; ++j) {
          const double x0 = clampw(fma(u0[j].y, gg[j], u0[j].x), wm);
          const double x1 = V == 2 ? clampw(fma(u1[j].y, gg[j], u1[j].x), wm) : 0.0;
          if (FULL || (rlane && r0 + j * R + rr < nrows && (!CLOSE || kk[j] != ZD))) {
            if (!CLOSE) {  // (FULL: lanes past the row width add 0 below)
              acc0 += x0;
              acc1 += x1;
            }
            if (FAST) {
              const int off = vb + (r0 + j * R) * N * 8;
              if (V == 2) st_wt16(rs, off, x0, x1);
              else st_wt8b(rs, off, x0);
            } else if (aw) {
              double* dst = aw + (size_t)(rbase + r0 + j * R + rr) * N + t0;
              st_wt8(dst, x0);
              if (V == 2) st_wt8(dst + 1, x1);
            }
          }
        }
      };
      using T_ = std::true_type;
      using F_ = std::false_type;
      bool full = r0 + RU * R <= nrows;  // wave-uniform
      if constexpr (CLOSE) {  // a batch with a row left to the re-solve takes the masked path
        bool drop = false;
#pragma unroll
        for (int j = 0; j < RU; ++j) drop |= kk[j] == ZD;
        full = full && !__any(drop);
      }
      if (full) {
        if (fast) rows(T_{}, T_{});
        else rows(T_{}, F_{});
      } else {
        if (fast) rows(F_{}, T_{});
        else rows(F_{}, F_{});
      }
#pragma unroll
      for (int j = 0; j < RU; ++j) {
        kk[j] = kn[j];
        gg[j] = gn[j];
      }
    }
    // rows of invalid EVs (gamma outside [0, y_max] or NaN): NaN, written after the loop's
    // zeros of the same rows (rare; ordered by the wait)
    if (any_inv && aw) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      for (int r = 0; r < nrows; ++r) {
        const double g = sg[r];
        if (!(g >= 0.0 && g <= ym) && lane < N) st_wt8(aw + (size_t)(rbase + r) * N + lane, NAN);
      }
    }
  };
  if constexpr (CLOSE) {  // waves 1.. split the block's rows evenly (wave 0 published the record)
    if (wv > 0 && aw) {  // (no w output: nothing to write, the sums are in the record)
      const int tot = end - start;
      const int lo = (wv - 1) * tot / (EVAL_WAVES - 1), hi = wv * tot / (EVAL_WAVES - 1);
      if (hi > lo) row_segment(lo, hi - lo);
    }
  } else {  // each wave: the lookup of a pass, then that pass's rows (the first row stores leave
            // half a lookup earlier and the second lookup overlaps their drain)
#pragma unroll
    for (int h = 0; h < EVAL_PASSES; ++h) {
      if (!pass_live(h)) break;
      if (LQ_EVAL_OUT_AFTER_ROWS) lookup_key(h);
      else lookup(h);
      __builtin_amdgcn_wave_barrier();  // this wave's own rows in LDS: in order
      any_inv = inv_rows;
      const int r0b = STG ? sg0 + 64 * h : EVAL_EVS * h + 64 * wv;
      const int nh = STG ? min(64, sgn - 64 * h) : max(0, min(64, end - start - r0b));  // wave-uniform
      if (nh > 0 && !psum) row_segment(r0b, nh);
      if (LQ_EVAL_OUT_AFTER_ROWS) lookup_out(h);
    }
    if (lane == 0) st_wt4(a.fail_cnt + (size_t)rb * EVAL_WAVES + wv, nlist);
    wave_record();
  }
  LQ_STAMPE(4);
  if constexpr (CLOSE) {
    __syncthreads();  // every row written; the staged table is free (finalize_set's scratch)
    if (s_last) {
      double (*red)[FIN_W] = reinterpret_cast<double (*)[FIN_W]>(s_dyn);
      finalize_set<EVAL_WAVES, true>(*fr, s, red, red + EVAL_WAVES);
    }
  } else {
    if (!rlane) acc0 = acc1 = 0.0;  // (lanes past the row width read real rows in full batches)
    // this wave's row sums per stage: lanes col, col + Lr, ... (fixed order)
    {
      double s0 = acc0, s1 = acc1;
      for (int k = 1; k < R; ++k) {
        s0 += __shfl(acc0, lane + k * Lr, 64);
        s1 += __shfl(acc1, lane + k * Lr, 64);
      }
      if (lane < Lr) {
        accw_w[V * lane] = s0;
        if (V == 2) accw_w[V * lane + 1] = s1;
      }
    }
    if constexpr (!STG) {
      if (ro.pipelined) {
        // the block's last wave to finish its rows writes the record (the others go on to the next run's
        // staging loads); the acquire-release LDS counter orders every wave's row sums before its read
        // Every lane of the wave takes part in the ordering: a workgroup-scope release fence (LDS only:
        // the row stores to HBM stay in flight) before lane 0's increment orders all lanes' row-sum
        // writes, and the acquire fence after the broadcast orders the last wave's reads of every
        // wave's sums, per the HIP memory model rather than per-wave LDS issue order
        int old = 0;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
        if (lane == 0) old = __hip_atomic_fetch_add(&s_done, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_WORKGROUP);
        old = __shfl(old, 0, 64);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
        if (old == EVAL_WAVES - 1) {
          if (psum) {
            // every wave's lookups (and their LDS piece aggregates) are complete: the per-stage sums
            // over the set's piece slots in slot order (lane = stage) into this wave's row sums (the
            // other waves' are zero: they evaluated no rows)
            const double fxi = (whi - wlo) * 0x1p-40;
            double accs = 0.0;
            for (int p = 0; p < np; ++p) {
              const int n = s_pn[p];
              if (n == 0) continue;  // (block-uniform)
              const double2 ab = s_ab[abx(p, min(lane, N - 1))];
              const double gsum = fma((double)s_pf[p], fxi, (double)n * wlo);
              accs = fma((double)n, ab.x, accs);
              accs = fma(gsum, ab.y, accs);
            }
            if (lane < N) accw_w[lane] = accs;  // (its own row: zero, no rows were evaluated)
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          }
          store_record(lane, 64);
          if (lane == 0) __hip_atomic_store(&s_done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
      } else {
        __syncthreads();
        if (tid < 64) store_record(tid, 64);
      }
    }
  }
  LQ_STAMPE(5);
}

// k_eval.  CLOSE: the set's closing (finalize_set) runs inside the launch, by the workgroup of the
// set that arrives last (eval_block<..., CLOSE>), so no k_finalize launch and no kernel boundary
// follow; workgroup nblk closes the sets that have no EVs.
template <bool CLOSE, int NT>
__global__ __launch_bounds__(EVAL_EVS, EVAL_MIN_WAVES) void k_eval(EvalArgs a, FinalArgs r) {  // (4 waves per SIMD: two workgroups per CU)
  extern __shared__ __attribute__((aligned(16))) double2 s_dyn[];
  const int b = (int)blockIdx.x;
  if (a.skip && *a.skip) return;  // (every workgroup: the arrival counters stay at zero)
  if constexpr (CLOSE) {
    if (b == a.nblk) {
      double (*red)[FIN_W] = reinterpret_cast<double (*)[FIN_W]>(s_dyn);
      for (int s = 0; s < a.S; ++s)
        if (r.blk_prefix[s + 1] == r.blk_prefix[s]) {
          finalize_set<EVAL_WAVES, true>(r, s, red, red + EVAL_WAVES);
          __syncthreads();  // (red / rep are rewritten for the next set)
        }
      return;
    }
  }
  eval_block<NT, CLOSE>(a, b, &r);
}

// k_eval for horizon N: exact-N instantiations for the shipped horizons, run-time N otherwise
typedef void (*EvalKernel)(EvalArgs, FinalArgs);
template <bool CLOSE>
EvalKernel eval_kernel(int N) {
  switch (N) {
    case 12: return k_eval<CLOSE, 12>;
    case 16: return k_eval<CLOSE, 16>;
    case 24: return k_eval<CLOSE, 24>;
    case 48: return k_eval<CLOSE, 48>;
    default: return k_eval<CLOSE, 0>;
  }
}

// lompc_plan_run_steps, stepped form: ONE launch carries run k + 1's path (workgroups [0, np_wg):
// LQ_STEP_CELLS cells of one set each, one per wave), run k's evaluation (the next ne workgroups,
// k_eval's block; the block map sized for the slots the path leaves) and run k - 1's closing (nf
// workgroups, one per set).  The three are independent (separate path tables, records and cell-start
// working sets per run in flight), so the latency-bound path chain runs beside the bandwidth-bound
// evaluation instead of before it.  (The arguments stay kernel arguments: preloaded, where a record in
// memory would add a dependent load round at the start of every workgroup.)
template <int NT>
__global__ __launch_bounds__(EVAL_EVS, EVAL_MIN_WAVES) void k_step(PathArgs pa, EvalArgs ea, FinalArgs ff, int np_wg,
                                                                    int ne, int nf) {
  extern __shared__ __attribute__((aligned(16))) double2 s_dyn[];
  int b = (int)blockIdx.x;
  if (b < np_wg) {
    // (G % LQ_STEP_CELLS == 0: every cell of the workgroup in one set).  The waves without a cell exit
    // here; the path waves initialise the set's box table inside path_cell, after their price loads
    // are issued (the barrier overlaps them, as in k_path)
    const int wv = (int)(threadIdx.x >> 6), cell = b * LQ_STEP_CELLS + wv;
    if (wv >= LQ_STEP_CELLS || cell >= pa.S * pa.G) return;
    // the path chain is the launch's critical path: its waves issue first on a SIMD they share
    // with evaluation waves (which mostly wait on memory)
    if (LQ_STEP_PRIO) __builtin_amdgcn_s_setprio(3);
    path_cell<NT, true>(pa, cell);
    return;
  }
  b -= np_wg;
  if (b < ne) {
    eval_block<NT, false>(ea, b);
    return;
  }
  b -= ne;
  if (b < nf) {
    double (*red)[FIN_W] = reinterpret_cast<double (*)[FIN_W]>(s_dyn);
    finalize_set<EVAL_WAVES, false>(ff, b, red, red + EVAL_WAVES);
  }
}

typedef void (*StepKernel)(PathArgs, EvalArgs, FinalArgs, int, int, int);
StepKernel step_kernel(int N) {
  switch (N) {
    case 12: return k_step<12>;
    case 16: return k_step<16>;
    case 24: return k_step<24>;
    case 48: return k_step<48>;
    default: return k_step<0>;
  }
}

// The wide form's path launch (lompc_plan_run_steps without warm starts): the paths of runs run0 ..
// run0 + nruns - 1 in ONE launch, one wave per (run, set, cell) — thousands of independent
// latency-bound chains at once instead of one run's 384 beside an evaluation; run j's prices at
// lmbd + j lm_stride, its tables in ring slot j % slots
#ifndef LQ_PATHS_WAVES
#define LQ_PATHS_WAVES 1  // k_paths: min waves per SIMD the compiler must fit (registers)
#endif
template <int NT>
__global__ __launch_bounds__(64, LQ_PATHS_WAVES) void k_paths(PathArgs a, int64_t lm_stride, int64_t lr_stride, int run0,
                                                               int slots) {
  const int SG = a.S * a.G;
  const int r = (int)blockIdx.x / SG, cell = (int)blockIdx.x - r * SG;
  const int j = run0 + r;
  const int64_t o = (int64_t)(j % slots) * SG;
  PathArgs b = a;
  b.lmbd = a.lmbd + (size_t)j * lm_stride;
  b.lmbd_r = a.lmbd_r + (size_t)j * lr_stride;
  b.t_cnt = a.t_cnt + o;
  b.t_lo = a.t_lo + o;
  b.t_sl = a.t_sl + o * 64;
  b.t_ge = a.t_ge + o * LQ_PPL;
  b.t_cf = a.t_cf + o * LQ_PPL * 8;
  b.t_ab = a.t_ab + o * LQ_PPL * a.N;
  path_cell<NT, true>(b, cell);
}

typedef void (*PathsKernel)(PathArgs, int64_t, int64_t, int, int);
PathsKernel paths_kernel(int N) {
  switch (N) {
    case 12: return k_paths<12>;
    case 16: return k_paths<16>;
    case 24: return k_paths<24>;
    case 48: return k_paths<48>;
    default: return k_paths<0>;
  }
}

// The wide form's evaluations (lompc_plan_run_steps without warm starts, one part per kind): the
// evaluations of runs run0 .. run0 + nruns - 1 in ONE launch.  Workgroup b evaluates its block of
// every run in turn (k_eval's block map and arithmetic: eval_block), run j from ring slot j % slots
// of the path tables and into record slot j - run0, so the launch holds no kernel boundary between
// runs: while one workgroup stages run j + 1's pieces (its own loads wait for its row stores to be
// acknowledged: vmcnt counts both in order), the other workgroups of the CU keep their rows streaming,
// and no workgroup tail idles the chip between two runs.  Per-EV outputs at j ev_stride (0: every
// run rewrites the same rows, each row by the same wave and lane in every run, so in run order).
struct EvalsArgs {
  int run0, nruns, slots, nblk;
  int64_t lm_stride, lr_stride, ev_stride, SG;
};

#ifndef LQ_EVALS_PIPELINED
#define LQ_EVALS_PIPELINED 1  // k_evals: staging loads issued before the table's barrier, records by the last wave
#endif
#ifndef LQ_EVALS_RUN_BARRIER
#define LQ_EVALS_RUN_BARRIER 0  // 1: k_evals' former barrier at the end of every run (diagnostic builds)
#endif
#ifndef LQ_EVALS_SKEW
#define LQ_EVALS_SKEW 0  // k_evals: start delay (100 MHz ticks) of the grid's second half (diagnostic builds)
#endif

template <int NT>
__global__ __launch_bounds__(EVAL_EVS, EVAL_MIN_WAVES) void k_evals(EvalArgs a, EvalsArgs x) {
  const int b = (int)blockIdx.x;
  if (LQ_EVALS_SKEW > 0 && 2 * b >= x.nblk) {  // (the two workgroups of a CU out of phase)
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < LQ_EVALS_SKEW) __builtin_amdgcn_s_sleep(8);
  }
  for (int r = 0; r < x.nruns; ++r) {
    const int j = x.run0 + r;
    RunOff ro;
    ro.tab = (int64_t)(j % x.slots) * x.SG;
    ro.rec = r * x.nblk;
    ro.ev = (int64_t)j * x.ev_stride;
    ro.lmbd = a.lmbd + (size_t)j * x.lm_stride;
    ro.lmbd_r = a.lmbd_r + (size_t)j * x.lr_stride;
    ro.launder = true;
    ro.gamma_lds = r > 0;
    ro.pipelined = LQ_EVALS_PIPELINED;
    ro.first = r == 0;
#ifdef LQ_EVALS_NOSTAGE
    ro.nostage = r > 0;  // (timing only: every run after the first evaluates run 0's table)
#endif
    // (the block index laundered per run: nothing derived from it — the block's EVs and gamma, the set's
    // constants — is hoisted out of the loop and kept live across runs, which made the loop spill)
    int bl = b;
    asm volatile("" : "+s"(bl));
#ifdef LOMPC_STAMPS
    // diagnostic build (scripts/evals_stamps.py): per (workgroup, run < 32) the run's start, the end
    // of its staging phases, the end of its rows and its end, at g_stamps[((b * 32 + r) * 8 + k]
    const long long t0__ = __builtin_amdgcn_s_memtime();
#endif
    eval_block<NT, false>(a, bl, nullptr, ro);
    // (no barrier here: every wave has passed the block's record barrier, so every row of the run is
    // written and its table no longer read; wave 0 reads only the row sums while the others stage the
    // next run, and no wave writes row sums again before the next run's staging barrier, which wave 0
    // reaches after its record)
#if LQ_EVALS_RUN_BARRIER
    __syncthreads();
#endif
#ifdef LOMPC_STAMPS
    if (threadIdx.x == 0 && r < 32 && b < 512) {  // start, block map, scalars, counts, pieces, staged, rows, end
      long long* q = g_stamps + ((size_t)b * 32 + r) * 8;
      const long long* e = g_stamps + (32768 + b) * 8;
      q[0] = t0__;
      q[1] = e[6];
      q[2] = e[0];
      q[3] = e[2];
      q[4] = e[3];
      q[5] = e[1];
      q[6] = e[4];
      q[7] = __builtin_amdgcn_s_memtime();
    }
#endif
  }
}

// k_evals with the stager (LQ_EVALS_STAGER; compact tables, a.cap = their capacity, a.G <= 64, N + 4
// <= 64, blocks of <= LQ_EVALS_MAXB EVs): wave LQ_EVALS_RW stages run 0's table, then during run r the
// table of run r + 1 into the other LDS table while waves 0 .. LQ_EVALS_RW - 1 evaluate run r (eval_block
// STG); ONE barrier per run, after which wave 0 stores run r's workgroup record from the run's scratch
// parity (the stager's row sums and record are zero) while the other waves start run r + 1.
template <int NT>
__global__ __launch_bounds__(EVAL_EVS, EVAL_MIN_WAVES) void k_evals_st(EvalArgs a, EvalsArgs x) {
  extern __shared__ __attribute__((aligned(16))) double2 s_dyn[];
  const int b = (int)blockIdx.x, tid = (int)threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);  // (wave-uniform: the roles' branches are scalar)
  const int N = NT ? NT : a.N, G = a.G, capc = a.cap;
  const size_t tb = ctab_bytes(N, G, capc);
  char* const base = reinterpret_cast<char*>(s_dyn);
  double* const accw = reinterpret_cast<double*>(base + 2 * tb);  // [2][EVAL_WAVES][N]
  double* const red = accw + (size_t)2 * EVAL_WAVES * N;         // [2][EVAL_WAVES][8]
  const int s = a.blk[b].x;
  if (wv == LQ_EVALS_RW) {
    const int NS = eval_row_stride(N);
    for (int k = 0; k < 2; ++k) {
      const CTab T = ctab_at(base + k * tb, N, G, capc);
      for (int i = lane; i < 2 * NS; i += 64) T.ab[(size_t)capc * NS + i] = make_double2(0.0, 0.0);  // zero pieces
      for (int i = lane; i < N; i += 64) accw[((size_t)k * EVAL_WAVES + LQ_EVALS_RW) * N + i] = 0.0;
      if (lane < 8) red[((size_t)k * EVAL_WAVES + LQ_EVALS_RW) * 8 + lane] = 0.0;
    }
    stage_compact(a, s, (int64_t)(x.run0 % x.slots) * x.SG, ctab_at(base, N, G, capc), N, G, capc, lane);
  }
  __syncthreads();
  for (int r = 0; r < x.nruns; ++r) {
    const int j = x.run0 + r;
    if (wv < LQ_EVALS_RW) {
      RunOff ro;
      ro.tab = (int64_t)(j % x.slots) * x.SG;
      ro.rec = r * x.nblk;
      ro.ev = (int64_t)j * x.ev_stride;
      ro.lmbd = a.lmbd + (size_t)j * x.lm_stride;
      ro.lmbd_r = a.lmbd_r + (size_t)j * x.lr_stride;
      ro.launder = true;
      ro.gamma_lds = r > 0;
      ro.buf = r & 1;
      int bl = b;
      asm volatile("" : "+s"(bl));
      eval_block<NT, false, true>(a, bl, nullptr, ro);
    } else if (r + 1 < x.nruns) {
      stage_compact(a, s, (int64_t)((j + 1) % x.slots) * x.SG, ctab_at(base + ((r + 1) & 1) * tb, N, G, capc), N, G,
                    capc, lane);
    }
    __syncthreads();  // run r's rows, row sums and wave records done; run r + 1's table staged
    if (wv == 0) {    // run r's workgroup record (the waves combined in a fixed order, as store_record)
      const int rb = r * x.nblk + b;
      const int par = r & 1;
      double* part = a.partial + (size_t)rb * (N + NPX);
      for (int c = lane; c < N + NPX; c += 64) {
        double v = 0.0;
        if (c < N) {
          for (int k = 0; k < EVAL_WAVES; ++k) v += accw[((size_t)par * EVAL_WAVES + k) * N + c];
        } else {
          const int xx = c - N;
          for (int k = 0; k < EVAL_WAVES; ++k) {
            const double u = red[((size_t)par * EVAL_WAVES + k) * 8 + xx];
            v = xx == PX_MAX_ERR ? fmax(v, u) : v + u;
          }
        }
        st_wt8(part + c, v);
      }
      if (lane == 0) st_wt4(a.fail_cnt + (size_t)rb * EVAL_WAVES + LQ_EVALS_RW, 0);  // (the stager's list)
    }
  }
}

typedef void (*EvalsKernel)(EvalArgs, EvalsArgs);
EvalsKernel evals_st_kernel(int N) {
  switch (N) {
    case 12: return k_evals_st<12>;
    case 16: return k_evals_st<16>;
    case 24: return k_evals_st<24>;
    case 48: return k_evals_st<48>;
    default: return k_evals_st<0>;
  }
}
EvalsKernel evals_kernel(int N) {
  switch (N) {
    case 12: return k_evals<12>;
    case 16: return k_evals<16>;
    case 24: return k_evals<24>;
    case 48: return k_evals<48>;
    default: return k_evals<0>;
  }
}

// ... and their closings in ONE launch: workgroup (r, s) closes set s of run run0 + r (finalize_set: the
// same summation order as every other closing form).  Set outputs at j sw_stride / st_stride; with
// shared set outputs (stride 0) or shared per-EV outputs (ev_stride 0) only the call's last run writes
// them (the closings of one launch are unordered); the plan's status rows likewise.
struct ClosesArgs {
  int run0, nruns, slots, nblk, S, last;
  int rel;  // set outputs indexed by the run's place in the launch (a communicator's send slots), not j
  int64_t lm_stride, lr_stride, ev_stride, sw_stride, st_stride, SG;
};

__global__ __launch_bounds__(256) void k_closes(FinalArgs f, ClosesArgs x) {
  __shared__ double red[LQ_FIN_CLASSES][FIN_W];
  __shared__ double rep[LQ_FIN_CLASSES][FIN_W];
  const int r = (int)blockIdx.x / x.S, s = (int)blockIdx.x - r * x.S, j = x.run0 + r, N = f.N;
  FinalArgs c = f;
  c.lmbd = f.lmbd + (size_t)j * x.lm_stride;
  c.lmbd_r = f.lmbd_r + (size_t)j * x.lr_stride;
  c.t_sl = f.t_sl + (int64_t)(j % x.slots) * x.SG * 64;
  c.partial = f.partial + (size_t)r * x.nblk * (N + NPX);
  c.fail_cnt = f.fail_cnt + (size_t)r * x.nblk * EVAL_WAVES;
  c.fail_idx = f.fail_idx + (size_t)r * x.nblk * EVAL_MAXB;
  const bool last = j == x.last;
  if (x.ev_stride) {
    const size_t eo = (size_t)j * x.ev_stride;
    if (f.w) c.w = f.w + eo * N;
    if (f.cost) c.cost = f.cost + eo;
    if (f.w0) c.w0 = f.w0 + eo;
    if (f.status) c.status = f.status + eo;
  } else if (!last) {
    c.w = c.cost = c.w0 = nullptr;
    c.status = nullptr;
  }
  const int js = x.rel ? r : j;
  if (f.set_sum_w) c.set_sum_w = (x.sw_stride || last) ? f.set_sum_w + (size_t)js * x.sw_stride : nullptr;
  if (f.set_stats) c.set_stats = (x.st_stride || last) ? f.set_stats + (size_t)js * x.st_stride : nullptr;
  if (!last) c.stats = nullptr;
  finalize_set<4, false>(c, s, red, rep);
}

#include "lompc_agg.hpp"

// ---------------------------------------------------------------- k_loop_iter
// One iteration of the device-resident price loop over gamma-sorted sets (lompc_loop.hip) in ONE
// launch, one wave per (set, cell) as k_path: the wave tracks its cell's path (path_cell), then
// aggregates the same cell from the tables it has just written (agg_cell, coherent loads) into a
// cell record (write-through).  The last of the S * G cells to arrive closes both sets from their
// records in cell order (agg_finish: k_agg's arithmetic — the same bits for G <= LQ_AGG_W, where
// k_agg's wave c holds cell c; G <= LQ_LOOP_G) and runs the loop step (lompc_loopstep.hpp) on the
// closed outputs in its registers.  The unfused form's three launches (k_path, k_agg, k_loop_step) and two kernel
// boundaries become one launch and one arrival counter (ctl[1]).
constexpr int LQ_LOOP_G = 16;  // k_loop_iter: at most this many cells per set (its closing's records in registers)
constexpr int LQ_LOOP_G2 = 32;  // k_loop_run2: at most this many (its closing reads the records 16 at a time)

#ifdef LOMPC_STAMPS
// diagnostic build: per k_loop_iter wave (blk < 64) the phases' s_memrealtime ticks summed over the
// launches: [0] path, [1] aggregation, [2] record + arrival, [3] both sets' closing, [4] loop step,
// [5] launches, [6] closings, [7] steps; sub-phases of [3] and [4]: [10] the records' load round,
// [8] the step's inputs and error metric, [9] the price QP (scripts/loop_stamps.py)
#define LQ_LSTAMP(k)                                                                                 \
  do {                                                                                               \
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");                                                 \
    const long long t__ = __builtin_amdgcn_s_memrealtime();                                          \
    if (lane == 0 && blk < 64) {                                                                     \
      __hip_atomic_fetch_add(g_lstamps + blk * 16 + (k), (unsigned long long)(t__ - tl__), __ATOMIC_RELAXED, \
                             __HIP_MEMORY_SCOPE_AGENT);                                              \
      if ((k) == 0 || (k) == 3 || (k) == 4)                                                          \
        __hip_atomic_fetch_add(g_lstamps + blk * 16 + 5 + ((k) >= 3 ? (k) - 2 : 0), 1ull, __ATOMIC_RELAXED, \
                               __HIP_MEMORY_SCOPE_AGENT);                                            \
    }                                                                                                \
    tl__ = t__;                                                                                      \
  } while (0)
#else
#define LQ_LSTAMP(k)
#endif

template <int NT>
__global__ __launch_bounds__(64) void k_loop_iter(PathArgs pa, AggArgs ga, StepArgs sa, double* rec, int m) {
  constexpr int S = 2;  // (lq_loop_fusable: the loop's two sets)
  if (sa.ctl[0]) return;  // finished: a call enqueued ahead of the convergence (every workgroup)
  const int blk = (int)blockIdx.x, lane = (int)threadIdx.x, G = pa.G;
  const int s = blk / G, c = blk - s * G;
#ifdef LOMPC_STAMPS
  long long tl__ = __builtin_amdgcn_s_memrealtime();
#endif
  StepIn in;
  step_prices(sa, lane, in);  // (every wave: the one that runs the step has them when it arrives last)
  // the sets' sizes and order flags for the closing, loaded now (scalar loads are otherwise issued
  // at their first use: a memory round on the closing's critical path)
  int cl_n[S], cl_v[S], cl_ok[S];
#pragma unroll
  for (int t = 0; t < S; ++t) {
    const int4 si = ga.sinfo[t];
    cl_n[t] = (int)(ga.set_off[t + 1] - ga.set_off[t]);
    cl_v[t] = si.x;
    cl_ok[t] = si.y;
    asm volatile("" : "+v"(cl_n[t]), "+v"(cl_v[t]), "+v"(cl_ok[t]));  // (held in VGPRs: SGPRs are scarce here)
  }
  path_cell<NT, true>(pa, blk);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the cell's tables have reached L2
  LQ_LSTAMP(0);
  {
    const AggSet z = agg_set_init<NT>(ga, s);
    AggPart ap;
    if (z.order_ok) agg_cell<NT, true>(ga, z, s, c, agg_cell_range(z, c), lane, ap);
    LQ_LSTAMP(1);
    const AggRec x = agg_wave_record(ap);
    double* rc = rec + (size_t)blk * LQ_AGG_REC;
    if (lane < z.N) st_wt8(rc + lane, ap.accw);
    if (lane < 5) st_wt8(rc + LOMPC_MAX_N + lane, x.pick(lane));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int old = 0;
  if (lane == 0) {
    old = __hip_atomic_fetch_add(sa.ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (old == S * G - 1) __hip_atomic_store(sa.ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  LQ_LSTAMP(2);
  if (lqw::readlane_i(old, 0) != S * G - 1) return;
  // the last arriver: every record of both sets in flight at once (one memory round), each set
  // closed in cell order, then the loop step on the closed outputs
  AggSet zs[S];  // (agg_finish reads N and the sizes / order flags loaded at the start)
#pragma unroll
  for (int t = 0; t < S; ++t) {
    zs[t].N = NT ? NT : ga.N;
    zs[t].n_s = cl_n[t];
    zs[t].si = make_int4(cl_v[t], cl_ok[t], 0, 0);
    zs[t].order_ok = cl_ok[t] != 0;
  }
  const int N = zs[0].N;
  // (records k >= G read the zero record past the S * G real ones: no per-load branch or mask)
  double rw[S][LQ_LOOP_G], rx[S][LQ_LOOP_G];
  const int tl = min(lane, N - 1), xl = min(lane, 4);
#pragma unroll
  for (int t = 0; t < S; ++t)
#pragma unroll
    for (int k = 0; k < LQ_LOOP_G; ++k) {
      const double* rk = rec + (size_t)(k < G ? t * G + k : S * G) * LQ_AGG_REC;
      rw[t][k] = ld_t<true>(rk + tl);
      rx[t][k] = ld_t<true>(rk + LOMPC_MAX_N + xl);
    }
  LQ_LSTAMP(10);
  AggSetOut o[S];
#pragma unroll
  for (int t = 0; t < S; ++t)
    o[t] = agg_finish<false, true, LQ_LOOP_G>(ga, zs[t], t, lane, G, [&](int k) { return rw[t][k]; },
                             [&](int k) { return rx[t][k]; });
  LQ_LSTAMP(3);
  in.s0 = o[0].sumw;
  in.wk = o[1].sumw;
  in.emax = lqw::readlane_d(o[0].stat, LOMPC_STAT_MAX_ERR);
  in.cost_c = lqw::readlane_d(o[1].stat, LOMPC_STAT_SUM_COST);
  in.n_inv = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_INVALID) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_INVALID);
  in.n_fail = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_FAILED) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_FAILED);
#ifdef LOMPC_STAMPS
  loop_step_core(sa, m, lane, in, [&](int k) { LQ_LSTAMP(k); });
#else
  loop_step_core(sa, m, lane, in);
#endif
  LQ_LSTAMP(4);
}

// ---------------------------------------------------------------- k_loop_run
// The WHOLE device-resident price loop as ONE launch (persistent): the S * G waves of k_loop_iter
// run call after call.  Call m is k_loop_iter's body; the last arriver's step writes the next prices,
// the loop state and (m = 0) the A_bar factor write-through (sc1), drains them, and publishes the
// generation word ctl[2] = m + 1; every other wave polls ctl[2] (lane 0, sc1 loads, s_sleep backoff)
// and then re-reads everything the step wrote with sc1 loads (prices in the path, the aggregation and
// the step; the loop state and factor in step_prices) — MI355X_MICROARCH.md's valid hand-off form:
// sc1 payload drained before an sc1 flag, sc1 polls, sc1 payload loads.  The finishing step sets
// ctl[0] before its generation, so every wave leaves at the next call's top.  No launch boundary and
// no per-launch setup between calls (k_loop_iter: one launch per call, 1.5-1.7 us apart).  Bounded
// spins: a wave that waits LQ_RUN_SPINS polls without a new generation sets ctl[3] and ctl[0] and
// leaves (the host reports the timeout).  Same arithmetic as k_loop_iter: the same bits.
#ifndef LQ_RUN_SPINS
#define LQ_RUN_SPINS (1 << 22)  // ~ seconds of polls (a call takes ~15 us)
#endif
template <int NT>
__global__ __launch_bounds__(64) void k_loop_run(PathArgs pa, AggArgs ga, StepArgs sa, double* rec) {
  constexpr int S = 2;  // (lq_loop_fusable: the loop's two sets)
  const int blk = (int)blockIdx.x, lane = (int)threadIdx.x, G = pa.G;
  const int s = blk / G, c = blk - s * G;
  int cl_n[S], cl_v[S], cl_ok[S];  // (the sets' sizes and order flags: constant over the loop)
#pragma unroll
  for (int t = 0; t < S; ++t) {
    const int4 si = ga.sinfo[t];
    cl_n[t] = (int)(ga.set_off[t + 1] - ga.set_off[t]);
    cl_v[t] = si.x;
    cl_ok[t] = si.y;
    asm volatile("" : "+v"(cl_n[t]), "+v"(cl_v[t]), "+v"(cl_ok[t]));
  }
  for (int m = 0; m <= sa.max_iter; ++m) {
    if (m > 0) {  // call m - 1's step has published the prices of call m
      int ok = 1;
      if (lane == 0) {
        int spins = 0;
        while (__hip_atomic_load(sa.ctl + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < m) {
          __builtin_amdgcn_s_sleep(2);
          if (++spins >= LQ_RUN_SPINS) {
            ok = 0;
            break;
          }
        }
        if (!ok) {
          __hip_atomic_store(sa.ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(sa.ctl + 0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (!lqw::readlane_i(ok, 0)) return;
    }
    if (__hip_atomic_load(sa.ctl + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;  // finished
    StepIn in;
    step_prices<true>(sa, lane, in);
    path_cell<NT, true, true>(pa, blk);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the cell's tables have reached L2
    {
      const AggSet z = agg_set_init<NT, true>(ga, s);
      AggPart ap;
      if (z.order_ok) agg_cell<NT, true, true>(ga, z, s, c, agg_cell_range(z, c), lane, ap);
      const AggRec x = agg_wave_record(ap);
      double* rc = rec + (size_t)blk * LQ_AGG_REC;
      if (lane < z.N) st_wt8(rc + lane, ap.accw);
      if (lane < 5) st_wt8(rc + LOMPC_MAX_N + lane, x.pick(lane));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int old = 0;
    if (lane == 0) {
      old = __hip_atomic_fetch_add(sa.ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old == S * G - 1) __hip_atomic_store(sa.ctl + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lqw::readlane_i(old, 0) != S * G - 1) continue;
    // the last arriver: both sets closed from the records (one memory round), then the loop step
    AggSet zs[S];
#pragma unroll
    for (int t = 0; t < S; ++t) {
      zs[t].N = NT ? NT : ga.N;
      zs[t].n_s = cl_n[t];
      zs[t].si = make_int4(cl_v[t], cl_ok[t], 0, 0);
      zs[t].order_ok = cl_ok[t] != 0;
    }
    const int N = zs[0].N;
    double rw[S][LQ_LOOP_G], rx[S][LQ_LOOP_G];
    const int tl = min(lane, N - 1), xl = min(lane, 4);
#pragma unroll
    for (int t = 0; t < S; ++t)
#pragma unroll
      for (int k = 0; k < LQ_LOOP_G; ++k) {
        const double* rk = rec + (size_t)(k < G ? t * G + k : S * G) * LQ_AGG_REC;
        rw[t][k] = ld_t<true>(rk + tl);
        rx[t][k] = ld_t<true>(rk + LOMPC_MAX_N + xl);
      }
    AggSetOut o[S];
#pragma unroll
    for (int t = 0; t < S; ++t)
      o[t] = agg_finish<false, true, LQ_LOOP_G>(ga, zs[t], t, lane, G, [&](int k) { return rw[t][k]; },
                                               [&](int k) { return rx[t][k]; });
    in.s0 = o[0].sumw;
    in.wk = o[1].sumw;
    in.emax = lqw::readlane_d(o[0].stat, LOMPC_STAT_MAX_ERR);
    in.cost_c = lqw::readlane_d(o[1].stat, LOMPC_STAT_SUM_COST);
    in.n_inv = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_INVALID) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_INVALID);
    in.n_fail = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_FAILED) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_FAILED);
    // the step releases call m + 1 as soon as its prices and loop state (sc1) have left this wave —
    // before its host-memory writes, which then overlap call m + 1 (a finishing step releases nothing:
    // its ctl[0] and `done` end the loop, and the waves leave at the next call's top)
    bool released = false;
    const auto release = [&]() {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(sa.ctl + 2, m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      released = true;
    };
    loop_step_core(sa, m, lane, in, NoStamp{}, release);
    if (!released) {  // (finished: the waiting waves find ctl[0] behind this generation)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(sa.ctl + 2, m + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// k_loop_run, redundant form (LQ_LOOP_REDUNDANT): no hand-off of the step's results.  Every wave
// arrives on a monotonic counter (ctl[1]) after writing its cell record (write-through, drained),
// waits until all S * G waves of the call have arrived, loads every record (sc1) and runs the SAME
// closing and loop step as every other wave — the same instructions on the same records in the same
// order, so the same bits in every wave — and goes straight on to the next call with the prices, the
// loop state and the A_bar factor in its registers (the path and the aggregation take the prices from
// registers: no memory round between the step and the next path).  Wave 0 alone writes: the set
// outputs, the stats and tallies, the prices / state / factor to memory and the host results.  The
// records alternate between two buffers by call parity (a wave may write call m + 1's record while a
// slower wave still reads call m's: never call m + 2's, which needs every wave's call m + 1 arrival).
// The same arithmetic as k_loop_run and k_loop_iter: the same bits.
#ifndef LQ_LOOP_REDUNDANT
#define LQ_LOOP_REDUNDANT 1
#endif
template <int NT>
__global__ __launch_bounds__(64) void k_loop_run2(PathArgs pa, AggArgs ga, StepArgs sa, double* rec) {
  constexpr int S = 2;
  const int blk = (int)blockIdx.x, lane = (int)threadIdx.x, G = pa.G;
  const int s = blk / G, c = blk - s * G;
  const bool writer = blk == 0;
  int cl_n[S], cl_v[S], cl_ok[S];
#pragma unroll
  for (int t = 0; t < S; ++t) {
    const int4 si = ga.sinfo[t];
    cl_n[t] = (int)(ga.set_off[t + 1] - ga.set_off[t]);
    cl_v[t] = si.x;
    cl_ok[t] = si.y;
    asm volatile("" : "+v"(cl_n[t]), "+v"(cl_v[t]), "+v"(cl_ok[t]));
  }
  AggArgs gw = ga;  // (the closing's outputs: wave 0's only)
  if (!writer) {
    gw.set_sum_w = nullptr;
    gw.set_stats = nullptr;
    gw.stats = nullptr;
    gw.tally = nullptr;
  }
  const int nsg = S * G;
  StepIn in;
  step_prices<false>(sa, lane, in);  // (the first call's prices, w_ref, the zeroed loop state)
  double pv[3] = {in.lm[0], in.lm[1], in.lm[2]};
  // the cell's stored working set, kept in a register from call to call (as each call stores it);
  // w_ref from the price buffer (the plan's w_ref of both sets, constant over the loop)
  const int N_ = NT ? NT : pa.N;
  const double wr_c = (pa.w_ref && lane < N_) ? pa.w_ref[(size_t)s * N_ + lane] : 0.0;
  int wsr = pa.ws ? (int)pa.ws[(size_t)blk * 64 + lane] : 0;
  for (int m = 0; m <= sa.max_iter; ++m) {
    // (the box table in LDS: written by the first call; the one-wave workgroup keeps its LDS)
    if (m == 0) path_cell<NT, true, true, true>(pa, blk, pv[0], pv[1], pv[2], wr_c, &wsr);
    else path_cell<NT, false, true, true>(pa, blk, pv[0], pv[1], pv[2], wr_c, &wsr);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the cell's tables have reached L2
    double* rb = rec + (size_t)(m & 1) * (nsg + 1) * LQ_AGG_REC;  // this call's record buffer
    {
      AggSet z = agg_set_init<NT, true>(ga, s);
      if (m > 0) {  // (the prices of this call: registers)
        z.preg = true;
        z.p1 = pv[0];
        z.p2 = pv[1];
        z.p3 = pv[2];
        z.l1 = lqw::readlane_d(pv[0], 0);
        z.l2 = lqw::readlane_d(pv[1], 0);
        z.l3 = lqw::readlane_d(pv[2], 0);
      }
      AggPart ap;
      if (z.order_ok) agg_cell<NT, true, true>(ga, z, s, c, agg_cell_range(z, c), lane, ap);
      const AggRec x = agg_wave_record(ap);
      double* rc = rb + (size_t)blk * LQ_AGG_REC;
      if (lane < z.N) st_wt8(rc + lane, ap.accw);
      if (lane < 5) st_wt8(rc + LOMPC_MAX_N + lane, x.pick(lane));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int ok = 1;
    if (lane == 0) {
      __hip_atomic_fetch_add(sa.ctl + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int target = (m + 1) * nsg;
      int spins = 0;
      while (__hip_atomic_load(sa.ctl + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins >= LQ_RUN_SPINS) {
          ok = 0;
          break;
        }
      }
      if (!ok) {
        __hip_atomic_store(sa.ctl + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(sa.ctl + 0, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    if (!lqw::readlane_i(ok, 0)) return;
    AggSet zs[S];
#pragma unroll
    for (int t = 0; t < S; ++t) {
      zs[t].N = NT ? NT : ga.N;
      zs[t].n_s = cl_n[t];
      zs[t].si = make_int4(cl_v[t], cl_ok[t], 0, 0);
      zs[t].order_ok = cl_ok[t] != 0;
    }
    const int N = zs[0].N;
    const int tl = min(lane, N - 1), xl = min(lane, 4);
    // the records in cell order, 16 of each set per memory round (records k >= G: the zero record
    // after buffer 0; with G <= 16 one round, the sums of k_loop_run's padded 16)
    double v[S] = {0.0, 0.0}, xs[S] = {0.0, 0.0}, xm[S] = {0.0, 0.0};
    for (int k0 = 0; k0 < G; k0 += LQ_LOOP_G) {  // (wave-uniform)
      double rw[S][LQ_LOOP_G], rx[S][LQ_LOOP_G];
#pragma unroll
      for (int t = 0; t < S; ++t)
#pragma unroll
        for (int k = 0; k < LQ_LOOP_G; ++k) {
          const double* rk =
              k0 + k < G ? rb + (size_t)(t * G + k0 + k) * LQ_AGG_REC : rec + (size_t)nsg * LQ_AGG_REC;
          rw[t][k] = ld_t<true>(rk + tl);
          rx[t][k] = ld_t<true>(rk + LOMPC_MAX_N + xl);
        }
#pragma unroll
      for (int t = 0; t < S; ++t)
#pragma unroll
        for (int k = 0; k < LQ_LOOP_G; ++k) {
          v[t] += rw[t][k];
          xs[t] += rx[t][k];
          xm[t] = fmax(xm[t], rx[t][k]);
        }
    }
    AggSetOut o[S];
#pragma unroll
    for (int t = 0; t < S; ++t) o[t] = agg_finish_tail<false>(gw, zs[t], t, lane, v[t], xs[t], xm[t]);
    in.s0 = o[0].sumw;
    in.wk = o[1].sumw;
    in.emax = lqw::readlane_d(o[0].stat, LOMPC_STAT_MAX_ERR);
    in.cost_c = lqw::readlane_d(o[1].stat, LOMPC_STAT_SUM_COST);
    in.n_inv = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_INVALID) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_INVALID);
    in.n_fail = lqw::readlane_d(o[0].stat, LOMPC_STAT_N_FAILED) + lqw::readlane_d(o[1].stat, LOMPC_STAT_N_FAILED);
    StepOut so;
    if (writer) loop_step_core<NoStamp, NoRelease, true>(sa, m, lane, in, NoStamp{}, NoRelease{}, &so);
    else loop_step_core<NoStamp, NoRelease, false>(sa, m, lane, in, NoStamp{}, NoRelease{}, &so);
    if (so.fin) return;
    // the next call's inputs: what the step stored, kept in registers
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pv[k] = so.v[k];
      in.lm[k] = so.v[k];
    }
    in.dc = so.cost_c;
    in.dterm = so.dterm;
    in.ab = so.ab;
  }
}

typedef void (*LoopRunKernel)(PathArgs, AggArgs, StepArgs, double*);
LoopRunKernel loop_run_kernel(int N) {
  if (LQ_LOOP_REDUNDANT) switch (N) {
      case 12: return k_loop_run2<12>;
      case 16: return k_loop_run2<16>;
      case 24: return k_loop_run2<24>;
      case 48: return k_loop_run2<48>;
      default: return k_loop_run2<0>;
    }
  switch (N) {
    case 12: return k_loop_run<12>;
    case 16: return k_loop_run<16>;
    case 24: return k_loop_run<24>;
    case 48: return k_loop_run<48>;
    default: return k_loop_run<0>;
  }
}

typedef void (*LoopIterKernel)(PathArgs, AggArgs, StepArgs, double*, int);
LoopIterKernel loop_iter_kernel(int N) {
  switch (N) {
    case 12: return k_loop_iter<12>;
    case 16: return k_loop_iter<16>;
    case 24: return k_loop_iter<24>;
    case 48: return k_loop_iter<48>;
    default: return k_loop_iter<0>;
  }
}

// ---------------------------------------------------------------- host helpers

// capacities of the buffers a re-targeted plan (lompc_plan_update) may outgrow: 1/4 headroom, and at
// least double the previous capacity, so a batch whose size wanders from call to call (a station's
// partitions, step to step: EVs move between charge-level partitions) reallocates O(log) times, not
// at every new high (hipMalloc / hipHostMalloc took 50-470 us per re-targeted plan in the station's
// staging, scripts/stage_profile.py)
int64_t with_slack(int64_t n, int64_t cap) { return std::max(n + n / 4 + 16, 2 * cap); }
constexpr int LQ_RESERVE_CELLS = 16;  // lompc_plan_reserve: cell-indexed buffers sized for this many cells per set (pick_cells' most)

#ifndef LQ_WIDE_ALPHA
#define LQ_WIDE_ALPHA 0.85  // EVs of a second-dispatch-round k_eval / k_evals block relative to a first-round one
#endif
// The k_eval block map of a batch: every set in near-equal blocks of <= maxb EVs (at least 256),
// `target` blocks in all, set-major (blocks[b] = (set, first EV, end EV); pre[s] = set s's first block).
// weighted (one dispatch round of persistent or single launches, more blocks than CUs): the blocks of
// the later dispatch round (index >= n_cu) get LQ_WIDE_ALPHA of the EVs of the first round's — a CU's
// second-dispatched workgroup runs ~13 % slower than its first (younger waves: the SIMDs' issue
// arbitration favours the older workgroup; scripts/evals_stamps.py), and a launch ends
// with its slowest workgroup.  Each set takes the blocks whose weights cover its share of the batch,
// and inside a set the EVs split in proportion to the weights.  A map only: the same QPs and per-EV
// arithmetic, the per-set sums combine per-block records in block order.
void block_map(const int64_t* off, int64_t S, int64_t B, int64_t maxb, int64_t target, int n_cu, bool weighted,
               std::vector<int4>& blks, std::vector<int>& pre) {
  blks.clear();
  pre.assign((size_t)S + 1, 0);
  auto blocks_of = [&](int64_t m) -> int64_t {
    if (m <= 0) return 0;
    const int64_t lo = (m + maxb - 1) / maxb, hi = (m + 255) / 256;
    return std::max<int64_t>(lo, std::min<int64_t>(hi, m * target / std::max<int64_t>(B, 1)));
  };
  int64_t nblk = 0;
  for (int64_t s = 0; s < S; ++s) nblk += blocks_of(off[s + 1] - off[s]);
  if (weighted && LQ_WIDE_ALPHA < 1.0 && nblk > (int64_t)n_cu && B > 0) {
    std::vector<double> wc((size_t)nblk + 1, 0.0);
    for (int64_t k = 0; k < nblk; ++k) wc[k + 1] = wc[k] + (k < (int64_t)n_cu ? 1.0 : LQ_WIDE_ALPHA);
    std::vector<int64_t> lo_of((size_t)S);
    int64_t need_after = 0;  // blocks the later non-empty sets need at least
    for (int64_t t = 0; t < S; ++t) {
      const int64_t m = off[t + 1] - off[t];
      lo_of[t] = m > 0 ? (m + maxb - 1) / maxb : 0;
      need_after += lo_of[t];
    }
    auto wt = [&](int64_t k) { return k < nblk ? wc[k] : wc[nblk] + (double)(k - nblk) * LQ_WIDE_ALPHA; };
    int64_t b = 0;
    for (int64_t s = 0; s < S; ++s) {
      const int64_t o = off[s], m = off[s + 1] - o;
      need_after -= lo_of[s];
      int64_t nb = lo_of[s];
      if (m > 0) {
        const double tgt = wc[nblk] * (double)off[s + 1] / (double)B;  // the set's cumulative weight
        const int64_t hi = std::min<int64_t>((m + 255) / 256, nblk - b - need_after);
        while (nb < hi && b + nb < nblk && wc[b + nb] + 0.5 * (wc[b + nb + 1] - wc[b + nb]) < tgt) ++nb;
      }
      auto fits = [&](int64_t n) {  // every block of the set within maxb EVs (the kernels' LDS rows)
        const double ws_ = wt(b + n) - wt(b);
        for (int64_t k = 0; k < n; ++k)
          if ((double)m * (wt(b + k + 1) - wt(b + k)) / ws_ > (double)(maxb - 2)) return false;
        return true;
      };
      while (m > 0 && nb < m && !fits(nb)) ++nb;
      const double w0 = wt(b), ws = wt(b + nb) - w0;
      for (int64_t k = 0; k < nb; ++k) {
        const int64_t e0 = o + (int64_t)((double)m * (wt(b + k) - w0) / ws);
        const int64_t e1 = k + 1 == nb ? o + m : o + (int64_t)((double)m * (wt(b + k + 1) - w0) / ws);
        blks.push_back(make_int4((int)s, (int)e0, (int)e1, 0));
      }
      b += nb;
      pre[s + 1] = (int)b;
    }
    return;
  }
  for (int64_t s = 0; s < S; ++s) {
    const int64_t o = off[s], m = off[s + 1] - o, nb = blocks_of(m);
    for (int64_t k = 0; k < nb; ++k) blks.push_back(make_int4((int)s, (int)(o + m * k / nb), (int)(o + m * (k + 1) / nb), 0));
    pre[s + 1] = (int)blks.size();
  }
}

int pick_cells(int64_t max_set, int flags) {
  const int g = (flags >> LOMPC_PLAN_CELLS_SHIFT) & 2047;  // the caller's choice (LOMPC_PLAN_CELLS)
  if (g >= 1 && g <= LQ_GMAX) return g;
  // the path of a set has a handful of breakpoints over its gamma window: the cell count trades
  // per-wave tracking latency against more cold starts; one cell for tiny sets
  if (max_set <= 64) return 1;
  if (max_set <= 1024) return 8;
  return 16;  // measured flat over 12..24 at config 3 (42.1-42.4 us/step), 8 and 48+ slower
}

int take_events(std::vector<hipEvent_t>& pool, hipEvent_t* e0, hipEvent_t* e1) {
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

// every recorded pair (a pair may span `mult` launches: read as that many launches)
int plan_events_read(std::vector<hipEvent_t>& ev, std::vector<int>& mult, std::vector<hipEvent_t>& pool, double& ms_acc,
                     int64_t& n_acc) {
  for (size_t k = 0; k + 1 < ev.size(); k += 2) {
    if (hipEventSynchronize(ev[k + 1]) != hipSuccess) return LOMPC_ERR_HIP;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ev[k], ev[k + 1]) != hipSuccess) return LOMPC_ERR_HIP;
    ms_acc += ms;
    n_acc += k / 2 < mult.size() ? mult[k / 2] : 1;
  }
  pool.insert(pool.end(), ev.begin(), ev.end());
  ev.clear();
  mult.clear();
  return LOMPC_OK;
}

}  // namespace

// ============================================================== host
// k_eval's dynamic LDS: up to cap pieces of one set (NS double2 + 8 + 1 doubles each) + the cells
size_t eval_lds(int N, int G, int cap) {
  const size_t stage = (size_t)cap * (eval_row_stride(N) * sizeof(double2) + 9 * sizeof(double)) +
                       (size_t)2 * eval_row_stride(N) * sizeof(double2) +
                       (size_t)G * sizeof(double) + (size_t)((G + 1) & ~1) * sizeof(int) +
                       (size_t)(cap + 2) * (sizeof(unsigned long long) + sizeof(int));
  return std::max(stage, (size_t)2 * EVAL_WAVES * FIN_W * sizeof(double));  // (close mode: red / rep)
}

// events of one profiled dispatch (null events when kernel k is not profiled)
int plan_prof_begin(lompc_plan* p, int k, hipEvent_t* e0, hipEvent_t* e1) {
  *e0 = *e1 = nullptr;
  return (p->prof >> k) & 1 ? take_events(p->prof_pool, e0, e1) : LOMPC_OK;
}
void plan_prof_end(lompc_plan* p, int k, hipEvent_t e0, hipEvent_t e1, int launches = 1) {
  if (!e0) return;
  p->prof_ev[k].push_back(e0);
  p->prof_ev[k].push_back(e1);
  p->prof_mult[k].push_back(launches);
}

#ifdef LQ_PREP_PROF  // diagnostic builds: lq_plan_prepare's phases on stderr (host microseconds)
#define LQ_PREP_MARK(k) prep_t[k] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count()
#else
#define LQ_PREP_MARK(k)
#endif
int lq_plan_prepare(lompc_plan* p, int nctx, lompc_ctx* const* ctxs, const int64_t* sets_per_ctx, int64_t B,
                    const double* gamma, const int64_t* set_offsets, const double* w_ref, int flags,
                    hipStream_t st) {
#ifdef LQ_PREP_PROF
  double prep_t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  struct PrepPrint {
    double* t;
    ~PrepPrint() {
      fprintf(stderr, "prep us: checks %.1f occ %.1f grow %.1f evsync %.1f host %.1f copy %.1f kernels %.1f\n", t[1] - t[0],
              t[2] - t[1], t[3] - t[2], t[4] - t[3], t[5] - t[4], t[6] - t[5], t[7] - t[6]);
    }
  } prep_print{prep_t};
#endif
  LQ_PREP_MARK(0);
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
  if (B < 0 || B >= (1ll << 31) - EVAL_MAXB) return fail_arg(p, "plan: 0 <= B < 2^31 required");
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
  if (((flags >> LOMPC_PLAN_CELLS_SHIFT) & 2047) > LQ_GMAX) return fail_arg(p, "plan: at most 1024 cells per set");
  const int G = pick_cells(max_set, flags);
  const int64_t ncell = S * G;
  // k_eval work split: every set in nb near-equal blocks of <= EVAL_MAXB EVs, the block count
  // chosen so the workgroups fill the CUs a whole number of times (r rounds of n_cu, at most 90%
  // of EVAL_MAXB per block) rather than spilling a few blocks into an extra round
  if (!p->n_cu) {
    HIPCHK(p, hipDeviceGetAttribute(&p->n_cu, hipDeviceAttributeMultiprocessorCount, ctxs[0]->device));
    if (p->n_cu < 1) p->n_cu = 1;
  }
  LQ_PREP_MARK(1);
  const int cap = std::min(LQ_PIECE_CAP, G * LQ_PPL);
  const int64_t occ_key = (int64_t)N * 4096 + cap;
  if (p->eval_occ_key != occ_key) {  // k_eval workgroups resident per CU (either variant may run)
    int occ0 = 0, occ1 = 0;
    HIPCHK(p, hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ0, eval_kernel<false>(N), EVAL_EVS, eval_lds(N, G, cap)));
    HIPCHK(p, hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ1, eval_kernel<true>(N), EVAL_EVS, eval_lds(N, G, cap)));
    p->eval_occ = std::max(std::min(occ0, occ1), 1);
    p->eval_occ_key = occ_key;
  }
  LQ_PREP_MARK(2);
  const int64_t slots = (int64_t)p->n_cu * p->eval_occ;
  const int64_t rounds = std::max<int64_t>(1, (10 * B + 9ll * slots * EVAL_MAXB - 1) / (9ll * slots * EVAL_MAXB));
  const int64_t target = rounds * slots;
  // the k_eval block map (weighted by dispatch round when the blocks take one round: block_map)
  std::vector<int4> bmap;
  std::vector<int> bpre;
  block_map(set_offsets, S, B, EVAL_MAXB, target, p->n_cu, rounds == 1, bmap, bpre);
  const int64_t nblk = (int64_t)bmap.size();
  int64_t n_empty = 0;
  // lompc_plan_reserve: a buffer that must grow is sized at once for the reserved batch size (upper
  // bounds: blocks_of(m) <= ceil(m / 256), sorted blocks ceil(m / LQ_AGG_SB) per set)
  const int64_t RB = std::max(B, p->reserve_B);
  const int64_t nblk_r = p->reserve_B ? RB / 256 + S + 1 : 0, nsblk_r = p->reserve_B ? RB / LQ_AGG_SB + S + 1 : 0;
  for (int64_t s = 0; s < S; ++s) n_empty += bpre[s + 1] == bpre[s] ? 1 : 0;
  p->device = ctxs[0]->device;
  p->N = N;
  p->nctx = nctx;
  for (int k = 0; k < nctx; ++k) p->ctx[k] = ctxs[k];
  p->flags = flags;
  p->w_ref = w_ref;
  p->gamma = gamma;
  int rc;
  if (!p->d_errflag) {
    if ((rc = grow(p, &p->d_errflag, 1))) return rc;
    HIPCHK(p, hipMemset(p->d_errflag, 0, sizeof(int)));
  }
  if (!p->ev_stage) HIPCHK(p, hipEventCreateWithFlags(&p->ev_stage, hipEventDisableTiming));
  if (S > p->cap_S) {
    if ((rc = grow(p, &p->d_window, 2 * S)) || (rc = grow(p, &p->d_wacc, 3 * S)) ||
        (rc = grow(p, &p->d_stats_own, S * LOMPC_SET_STATS)) || (rc = grow(p, &p->d_arrive, S)))
      return rc;
    HIPCHK(p, hipMemsetAsync(p->d_wacc, 0, 3 * S * sizeof(unsigned long long), st));
    HIPCHK(p, hipMemsetAsync(p->d_arrive, 0, S * sizeof(int), st));
    p->cap_S = S;
  }
  if (nblk > p->cap_blk) {
    const int64_t c = std::max(with_slack(nblk, p->cap_blk), nblk_r);
    if ((rc = grow(p, &p->d_partial, (size_t)c * (N + NPX))) ||
        (rc = grow(p, &p->d_fail_cnt, (size_t)c * EVAL_WAVES)) || (rc = grow(p, &p->d_fail_idx, (size_t)c * EVAL_MAXB)))
      return rc;
    p->cap_blk = c;
  }
  const bool warm = (flags & LOMPC_PLAN_WARM_START) != 0;
  bool fresh_ws = false;
  if (ncell > p->cap_cells || (warm && !p->d_ws)) {
    // (a reserved plan: sized for the most cells the plan's choice gives a set, LQ_RESERVE_CELLS)
    const int64_t cn = std::max(ncell, p->reserve_B ? S * (int64_t)std::max(G, LQ_RESERVE_CELLS) : 0);
    if ((rc = grow(p, &p->t_cnt, cn)) || (rc = grow(p, &p->t_lo, cn)) ||
        (rc = grow(p, &p->t_ge, cn * LQ_PPL)) || (rc = grow(p, &p->t_cf, cn * LQ_PPL * 8)) ||
        (rc = grow(p, &p->t_ab, cn * LQ_PPL * N)) || (rc = grow(p, &p->t_sl, 2 * cn * 64)))
      return rc;
    if (warm && (rc = grow(p, &p->d_ws, (size_t)cn * 64))) return rc;
    p->cap_cells = cn;
    fresh_ws = true;
  }
  // (0xff: no stored set — a cell's first run starts cold, from "all free", and its later runs warm)
  if (warm && (fresh_ws || p->G != G || p->S != S)) HIPCHK(p, hipMemsetAsync(p->d_ws, 0xff, (size_t)ncell * 64, st));
  if (!p->d_tally) {
    if ((rc = grow(p, &p->d_tally, 3))) return rc;
    HIPCHK(p, hipMemsetAsync(p->d_tally, 0, 3 * sizeof(unsigned long long), st));
  }
  // the sets close inside k_eval when the plan asks for it, and by default in single runs that
  // write no w rows (a price loop's reductions-only runs): nothing then makes the arriving
  // workgroups wait for row stores, and the k_finalize launch and its boundary go
  p->close = (flags & LOMPC_PLAN_CLOSE_IN_EVAL) != 0;
  p->close_no_w = (flags & LOMPC_PLAN_CLOSE_IN_FINALIZE) == 0;
  p->B = B;
  p->S = S;
  p->G = G;
  p->nblk = (int)nblk;
  p->n_empty = (int)n_empty;
  p->d_stats = p->d_stats_own;
  p->stp.ok = false;
  // host arrays -> pinned staging -> device (the staging may still feed the previous prepare)
  // the plan's host-built metadata, one block in pinned memory and one copy to its device
  // mirror: [QPConst x LQ_PLAN_MAX_CTX | int4 blocks | int64 set offsets | int block prefix]
  auto up16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
  const size_t o_blk = up16(LQ_PLAN_MAX_CTX * sizeof(QPConst));
  const size_t o_off = o_blk + up16((size_t)nblk * sizeof(int4));
  const size_t o_pre = o_off + up16((size_t)(S + 1) * sizeof(int64_t));
  // gamma-sorted sets: blocks of <= LQ_AGG_SB positions of one set for the prepare kernels
  // (the exact prefix sums hold 2^40-scaled gamma in 64 bits: a set of 2^24 EVs or more would wrap,
  // so such a plan evaluates every EV instead)
  const bool sorted = (flags & LOMPC_PLAN_SORTED_GAMMA) != 0 && max_set < (1ll << 24);
  int64_t nsblk = 0;
  if (sorted)
    for (int64_t s = 0; s < S; ++s) nsblk += (set_offsets[s + 1] - set_offsets[s] + LQ_AGG_SB - 1) / LQ_AGG_SB;
  const size_t o_sblk = o_pre + up16((size_t)(S + 1) * sizeof(int));
  const size_t o_spre = o_sblk + up16((size_t)nsblk * sizeof(int4));
  const size_t need_h = sorted ? o_spre + up16((size_t)(S + 1) * sizeof(int)) : o_sblk;
  const size_t need_h_r = p->reserve_B ? up16(LQ_PLAN_MAX_CTX * sizeof(QPConst)) + up16((size_t)nblk_r * sizeof(int4)) +
                                             2 * up16((size_t)(S + 1) * sizeof(int64_t)) + up16((size_t)nsblk_r * sizeof(int4)) +
                                             up16((size_t)(S + 1) * sizeof(int))
                                       : 0;
  LQ_PREP_MARK(3);
  HIPCHK(p, hipEventSynchronize(p->ev_stage));  // (the staging may still feed the previous copy)
  LQ_PREP_MARK(4);
  if ((int64_t)need_h > p->cap_h) {
    const int64_t c = std::max(with_slack((int64_t)need_h, p->cap_h), (int64_t)need_h_r);
    if (p->h_buf) HIPCHK(p, hipHostFree(p->h_buf));
    p->h_buf = nullptr;
    HIPCHK(p, hipHostMalloc((void**)&p->h_buf, (size_t)c, hipHostMallocDefault));
    if ((rc = grow(p, &p->d_meta, (size_t)c))) return rc;
    p->cap_h = c;
  }
  QPConst* hq = reinterpret_cast<QPConst*>(p->h_buf);
  for (int k = 0; k < nctx; ++k) hq[k] = ctxs[k]->q;
  int4* hblk = reinterpret_cast<int4*>(p->h_buf + o_blk);
  int64_t* hoff = reinterpret_cast<int64_t*>(p->h_buf + o_off);
  p->h_off_at = (int64_t)o_off;
  int* hpre = reinterpret_cast<int*>(p->h_buf + o_pre);
  memcpy(hoff, set_offsets, (S + 1) * sizeof(int64_t));
  if (nblk > 0) memcpy(hblk, bmap.data(), (size_t)nblk * sizeof(int4));
  memcpy(hpre, bpre.data(), (size_t)(S + 1) * sizeof(int));
  for (int k = 0, e = 0; k < LQ_PLAN_MAX_CTX; ++k) {
    e += k < nctx ? (int)sets_per_ctx[k] : 0;
    p->ce.end[k] = k + 1 < nctx ? e : (int)S;  // contexts past the last: never selected
  }
  p->d_q = reinterpret_cast<QPConst*>(p->d_meta);
  p->d_blk = reinterpret_cast<int4*>(p->d_meta + o_blk);
  p->d_set_off = reinterpret_cast<int64_t*>(p->d_meta + o_off);
  p->d_blk_prefix = reinterpret_cast<int*>(p->d_meta + o_pre);
  p->sorted = sorted;
  p->nsblk = (int)nsblk;
  if (sorted) {
    int4* hs = reinterpret_cast<int4*>(p->h_buf + o_sblk);
    int* hsp = reinterpret_cast<int*>(p->h_buf + o_spre);
    int64_t k = 0;
    hsp[0] = 0;
    for (int64_t s = 0; s < S; ++s) {
      for (int64_t i = set_offsets[s]; i < set_offsets[s + 1]; i += LQ_AGG_SB)
        hs[k++] = make_int4((int)s, (int)i, (int)std::min<int64_t>(i + LQ_AGG_SB, set_offsets[s + 1]), 0);
      hsp[s + 1] = (int)k;
    }
    p->d_sblk = reinterpret_cast<int4*>(p->d_meta + o_sblk);
    p->d_sblk_prefix = reinterpret_cast<int*>(p->d_meta + o_spre);
    p->aggF = G * LQ_AGG_KF;
    const int64_t nP = 3 * (B + S), npos = S * (int64_t)(p->aggF + 1);
    if (nsblk > p->cap_sblk) {
      const int64_t c = std::max(with_slack(nsblk, p->cap_sblk), nsblk_r);
      if ((rc = grow(p, &p->d_bsum, (size_t)c * 4))) return rc;
      p->cap_sblk = c;
    }
    if (nP > p->cap_P) {
      const int64_t c = std::max(with_slack(nP, p->cap_P), p->reserve_B ? 3 * (RB + S) : 0);
      if ((rc = grow(p, &p->d_P, c))) return rc;
      p->cap_P = c;
    }
    if (npos > p->cap_pos) {
      const int64_t pr = std::max(npos, p->reserve_B ? S * (int64_t)(std::max(G, LQ_RESERVE_CELLS) * LQ_AGG_KF + 1) : 0);
      if ((rc = grow(p, &p->d_pos, pr))) return rc;
      p->cap_pos = pr;
    }
    if (S > p->cap_sinfo) {
      if ((rc = grow(p, &p->d_sinfo, S))) return rc;
      p->cap_sinfo = S;
    }
  }
  LQ_PREP_MARK(5);
  HIPCHK(p, hipMemcpyAsync(p->d_meta, p->h_buf, need_h, hipMemcpyHostToDevice, st));
  HIPCHK(p, hipEventRecord(p->ev_stage, st));
  LQ_PREP_MARK(6);
  WindowArgs wa{p->d_q, p->ce, p->d_blk, p->d_blk_prefix, gamma, p->d_wacc, p->d_window, (int)S, (int)nblk};
  if (sorted) hipLaunchKernelGGL(k_plan_window_sorted, dim3((unsigned)S), dim3(64), 0, st, wa, p->d_set_off);
  else hipLaunchKernelGGL(k_plan_window, dim3((unsigned)nblk + 1), dim3(256), 0, st, wa);
  HIPCHK(p, hipGetLastError());
  if (sorted) {  // order check, prefix sums and fine index of the sorted sets (lompc_agg.hpp)
    SortArgs sa{p->d_q, p->ce, p->d_sblk, p->d_sblk_prefix, p->d_set_off, gamma, p->d_window, p->d_bsum, p->d_P,
                p->d_pos, p->d_sinfo, (int)S, G, p->aggF, B + S};
    if (nsblk > 0) hipLaunchKernelGGL(k_sorted_sum, dim3((unsigned)nsblk), dim3(256), 0, st, sa);
    hipLaunchKernelGGL(k_sorted_scan, dim3((unsigned)S), dim3(256), 0, st, sa);
    if (nsblk > 0) hipLaunchKernelGGL(k_sorted_fill, dim3((unsigned)nsblk), dim3(256), 0, st, sa);
    HIPCHK(p, hipGetLastError());
  }
  LQ_PREP_MARK(7);
  return LOMPC_OK;
}

// the plan's path table; `half` selects one of the two halves of the cell-start working sets
// (run_steps alternates them: a run's closing may re-solve from its own while the next run's path
// writes the other)
PathTab own_tab(const lompc_plan* p, int half = 0) {
  PathTab t;
  t.cnt = p->t_cnt;
  t.lo = p->t_lo;
  t.ge = p->t_ge;
  t.cf = p->t_cf;
  t.ab = p->t_ab;
  t.sl = p->t_sl + (size_t)half * p->S * p->G * 64;
  return t;
}

PathArgs path_args(lompc_plan* p, const double* lmbd, const double* lmbd_r, const PathTab& tb) {
  PathArgs pa{};
  const int N = p->N;
  pa.S = (int)p->S;
  pa.G = p->G;
  pa.N = N;
  pa.flags = p->flags;
  pa.qd = p->d_q;
  pa.ce = p->ce;
  pa.window = p->d_window;
  pa.lmbd = lmbd;
  pa.lmbd_r = lmbd_r;
  pa.w_ref = p->w_ref;
  pa.ws = (p->flags & LOMPC_PLAN_WARM_START) ? p->d_ws : nullptr;
  pa.t_cnt = tb.cnt;
  pa.t_lo = tb.lo;
  pa.t_sl = tb.sl;
  pa.t_ge = tb.ge;
  pa.t_cf = tb.cf;
  pa.t_ab = tb.ab;
  pa.errflag = p->d_errflag;
  pa.skip = p->skip;
  return pa;
}

// k_path of one run into the path table `tb`; with `fin` (run_steps) the previous run's closing
// rides in the same launch (k_path_fin)
int lq_launch_path(lompc_plan* p, const double* lmbd, const double* lmbd_r, const PathTab& tb, hipStream_t st,
                   const FinalArgs* fin = nullptr) {
  if (!lmbd || !lmbd_r) return fail_arg(p, "run: lmbd and lmbd_r required");
  const PathArgs pa = path_args(p, lmbd, lmbd_r, tb);
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (plan_prof_begin(p, LOMPC_PLAN_K_PATH, &e0, &e1)) return fail_arg(p, "profiling events");
  const unsigned ncell = (unsigned)(p->S * p->G);
  if (fin)
    hipExtLaunchKernelGGL(path_fin_kernel(p->N), dim3(ncell + (unsigned)p->S), dim3(64), 0, st, e0, e1, 0, pa, *fin);
  else
    hipExtLaunchKernelGGL(path_kernel(p->N), dim3(ncell), dim3(64), 0, st, e0, e1, 0, pa);
  HIPCHK(p, hipGetLastError());
  plan_prof_end(p, LOMPC_PLAN_K_PATH, e0, e1);
  return LOMPC_OK;
}

// the rest of one run from the path table `tb`: k_eval (or k_agg) and k_finalize, then with a
// communicator the all-gather and the combine
// defer (run_steps, no communicator): a k_finalize launch is not issued but its arguments are
// returned in *defer (defer->N = 0 when this run needs none) for the next run's k_path_fin
// the arguments of k_eval and of the set closing for one run from path table `tb`
void eval_args(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
               int8_t* status, const PathTab& tb, EvalArgs& a, FinalArgs& r) {
  const int N = p->N;
  a = EvalArgs{};
  a.S = (int)p->S;
  a.G = p->G;
  a.N = N;
  a.want_err = 1;
  a.qd = p->d_q;
  a.ce = p->ce;
  a.blk = p->d_blk;
  a.set_off = p->d_set_off;
  a.window = p->d_window;
  a.gamma = p->gamma;
  a.lmbd = lmbd;
  a.lmbd_r = lmbd_r;
  a.w_ref = p->w_ref;
  a.t_cnt = tb.cnt;
  a.t_lo = tb.lo;
  a.t_sl = tb.sl;
  a.t_ge = tb.ge;
  a.t_cf = tb.cf;
  a.t_ab = tb.ab;
  a.w = w;
  a.cost = cost;
  a.w0 = w0;
  a.status = status;
  a.partial = p->d_partial;
  a.fail_cnt = p->d_fail_cnt;
  a.fail_idx = p->d_fail_idx;
  a.w_rsrc_ok = (p->B * (int64_t)N * 8) <= LQ_DROP_OFF ? 1 : 0;
  a.w_bytes = a.w_rsrc_ok ? (int)(p->B * (int64_t)N * 8) : 0;
  a.cap = std::min(LQ_PIECE_CAP, p->G * LQ_PPL);
  a.nblk = p->nblk;
  a.skip = p->skip;
  r = FinalArgs{};
  r.N = N;
  r.G = p->G;
  r.want_err = 1;
  r.qd = p->d_q;
  r.ce = p->ce;
  r.blk_prefix = p->d_blk_prefix;
  r.set_off = p->d_set_off;
  r.window = p->d_window;
  r.gamma = p->gamma;
  r.lmbd = lmbd;
  r.lmbd_r = lmbd_r;
  r.w_ref = p->w_ref;
  r.t_sl = tb.sl;
  r.fail_cnt = p->d_fail_cnt;
  r.fail_idx = p->d_fail_idx;
  r.partial = p->d_partial;
  r.w = w;
  r.cost = cost;
  r.w0 = w0;
  r.status = status;
  r.stats = p->d_stats;
  r.tally = p->d_tally;
  r.skip = p->skip;
  r.arrive = p->d_arrive;
}

// with a communicator: `slots` packed send records [S][N] sums | [S][8] stats and the all-gather's
// receive buffer [nranks][S (N + 8)] (grown when the plan or the communicator outgrows them)
int lq_xbufs(lompc_plan* p, int slots, int recv_runs = 1) {
  const int64_t L = p->S * (p->N + LOMPC_SET_STATS);
  int rc;
  if (L * slots > p->cap_xsend) {
    if ((rc = grow(p, &p->d_xsend, L * slots))) return rc;
    p->cap_xsend = L * slots;
  }
  if (L * p->comm->nranks * recv_runs > p->cap_xrecv) {
    if ((rc = grow(p, &p->d_xrecv, L * p->comm->nranks * recv_runs))) return rc;
    p->cap_xrecv = L * p->comm->nranks * recv_runs;
  }
  return LOMPC_OK;
}

void lq_combine(const double* recv, int nranks, int64_t S, int N, double* set_sum_w, double* set_stats, hipStream_t st) {
  const int64_t L = S * (N + LOMPC_SET_STATS);
  const unsigned nb = (unsigned)std::max<int64_t>(1, std::min<int64_t>((L + 255) / 256, 1024));
  hipLaunchKernelGGL(k_combine, dim3(nb), dim3(256), 0, st, recv, nranks, (int)S, N, set_sum_w, set_stats);
}

// a run's send record (closed on this rank) -> every rank's record -> the rank-ordered combine into
// the caller's set outputs (all ranks bitwise equal)
int lq_exchange(lompc_plan* p, const double* send, double* set_sum_w, double* set_stats, hipStream_t st) {
  const int64_t L = p->S * (p->N + LOMPC_SET_STATS);
  int rc = lq_comm_allgather(p->comm, send, p->d_xrecv, (size_t)L, st);
  if (rc) {
    p->err = p->comm->err;
    return rc;
  }
  if (set_sum_w || set_stats) {
    lq_combine(p->d_xrecv, p->comm->nranks, p->S, p->N, set_sum_w, set_stats, st);
    HIPCHK(p, hipGetLastError());
  }
  return LOMPC_OK;
}

int lq_launch_eval(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, const PathTab& tb, hipStream_t st,
                   lompc_ctx* prof_ctx, FinalArgs* defer = nullptr) {
  if (defer) defer->N = 0;
  const int N = p->N;
  EvalArgs a;
  FinalArgs r;
  eval_args(p, lmbd, lmbd_r, w, cost, w0, status, tb, a, r);
  const size_t lds = eval_lds(N, p->G, a.cap);
  // with a communicator the sets close into the packed send record [S][N] | [S][8]
  const bool xr = p->comm != nullptr;
  if (xr) {
    const int rc = lq_xbufs(p, 1);
    if (rc) return rc;
  }
  r.set_sum_w = xr ? p->d_xsend : set_sum_w;
  r.set_stats = xr ? p->d_xsend + p->S * N : set_stats;
  // gamma-sorted sets and no per-EV output: per-piece aggregation (k_agg) instead of k_eval
  const bool agg = p->sorted && !w && !cost && !w0 && !status && p->nblk > 0;
  const bool close = !agg && (p->close || (p->close_no_w && !w)) && p->nblk > 0;
  const bool cprof = prof_ctx && prof_ctx->prof;  // lompc_solve_batch: the context's k_eval timing
  if (agg) {  // timed as k_eval
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &e0, &e1)) return fail_arg(p, "profiling events");
    AggArgs ga{(int)p->S, p->G, N, p->aggF, p->d_q, p->ce, p->d_set_off, p->d_window, p->gamma, lmbd, lmbd_r,
               p->w_ref, tb.cnt, tb.lo, tb.sl, tb.ge, tb.cf, tb.ab, p->d_P, p->B + p->S, p->d_pos,
               p->d_sinfo, r.set_sum_w, r.set_stats, p->d_stats, p->d_tally, p->skip};
    const int nw = std::min(p->G, (int)LQ_AGG_W);
    hipExtLaunchKernelGGL(agg_kernel(N), dim3((unsigned)p->S), dim3(64 * nw), 0, st, e0, e1, 0, ga);
    HIPCHK(p, hipGetLastError());
    plan_prof_end(p, LOMPC_PLAN_K_EVAL, e0, e1);
  } else if (p->nblk > 0) {
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (cprof ? take_events(prof_ctx->prof_pool, &e0, &e1) : plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &e0, &e1))
      return fail_arg(p, "profiling events");
    if (close) {  // + one workgroup for the sets without EVs
      hipExtLaunchKernelGGL(eval_kernel<true>(N), dim3((unsigned)(p->nblk + (p->n_empty > 0 ? 1 : 0))), dim3(EVAL_EVS), lds, st,
                            e0, e1, 0, a, r);
    } else {
      hipExtLaunchKernelGGL(eval_kernel<false>(N), dim3((unsigned)p->nblk), dim3(EVAL_EVS), lds, st, e0, e1, 0, a, r);
    }
    HIPCHK(p, hipGetLastError());
    if (cprof) {
      prof_ctx->prof_ev.push_back(e0);
      prof_ctx->prof_ev.push_back(e1);
    } else {
      plan_prof_end(p, LOMPC_PLAN_K_EVAL, e0, e1);
    }
  }
  if (!close && !agg && defer && !xr && N + NPX <= 64) {  // (one-wave closing: a record fits the wave)
    *defer = r;
    return LOMPC_OK;
  }
  if (!close && !agg) {  // (else the sets were closed inside k_eval / k_agg)
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (plan_prof_begin(p, LOMPC_PLAN_K_FINAL, &e0, &e1)) return fail_arg(p, "profiling events");
    hipExtLaunchKernelGGL(k_finalize, dim3((unsigned)p->S), dim3(256), 0, st, e0, e1, 0, r);
    HIPCHK(p, hipGetLastError());
    plan_prof_end(p, LOMPC_PLAN_K_FINAL, e0, e1);
  }
  if (!xr) return LOMPC_OK;
  return lq_exchange(p, p->d_xsend, set_sum_w, set_stats, st);
}

int lq_plan_launch(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, hipStream_t st, lompc_ctx* prof_ctx) {
  const PathTab tb = own_tab(p);
  int rc = lq_launch_path(p, lmbd, lmbd_r, tb, st);
  if (rc) return rc;
  return lq_launch_eval(p, lmbd, lmbd_r, w, cost, w0, status, set_sum_w, set_stats, tb, st, prof_ctx);
}

bool lq_loop_fusable(const lompc_plan* p, bool persistent) {  // (S = 2: the loop's sets; ctl holds 2 set counters)
  const int gmax = (persistent && LQ_LOOP_REDUNDANT) ? LQ_LOOP_G2 : LQ_LOOP_G;  // (k_loop_run2: chunked closing)
  return p->sorted && !p->comm && p->nblk > 0 && p->S == 2 && p->G >= 1 && p->G <= gmax;
}

int lq_launch_loop_iter(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                        const StepArgs& sa, int m, hipStream_t st) {
  return lq_launch_loop(p, lmbd, lmbd_r, set_sum_w, set_stats, sa, m, st, false);
}

// the whole loop as one persistent launch (k_loop_run)
int lq_launch_loop_run(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                       const StepArgs& sa, hipStream_t st) {
  return lq_launch_loop(p, lmbd, lmbd_r, set_sum_w, set_stats, sa, 0, st, true);
}

int lq_launch_loop(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                   const StepArgs& sa, int m, hipStream_t st, bool persistent) {
  if (!lq_loop_fusable(p, persistent)) return fail_arg(p, "k_loop_iter: plan not fusable");
  const int N = p->N;
  // [cell records | the zero record (k_loop_iter's padding) | (k_loop_run2) the second record buffer]
  const int64_t zoff = p->S * p->G * (int64_t)LQ_AGG_REC;
  const int64_t nrec = (2 * p->S * p->G + 1) * (int64_t)LQ_AGG_REC;
  if (nrec > p->cap_aggrec) {
    const int64_t c = std::max(nrec, p->reserve_B ? (2 * p->S * LQ_RESERVE_CELLS + 1) * (int64_t)LQ_AGG_REC : 0);
    const int rc = grow(p, &p->d_aggrec, c);
    if (rc) return rc;
    p->cap_aggrec = c;
    p->aggrec_zero = -1;
  }
  if (p->aggrec_zero != zoff) {  // (the cell records never reach it: zeroed once per layout)
    HIPCHK(p, hipMemsetAsync(p->d_aggrec + zoff, 0, LQ_AGG_REC * sizeof(double), st));
    p->aggrec_zero = zoff;
  }
  const PathTab tb = own_tab(p);
  const PathArgs pa = path_args(p, lmbd, lmbd_r, tb);
  AggArgs ga{(int)p->S, p->G, N, p->aggF, p->d_q, p->ce, p->d_set_off, p->d_window, p->gamma, lmbd, lmbd_r,
             p->w_ref, tb.cnt, tb.lo, tb.sl, tb.ge, tb.cf, tb.ab, p->d_P, p->B + p->S, p->d_pos,
             p->d_sinfo, set_sum_w, set_stats, p->d_stats, p->d_tally, p->skip};
  hipEvent_t e0 = nullptr, e1 = nullptr;  // (timed as k_path)
  if (plan_prof_begin(p, LOMPC_PLAN_K_PATH, &e0, &e1)) return fail_arg(p, "profiling events");
  if (persistent)  // (S * G one-wave workgroups: all resident at once, whatever else runs)
    hipExtLaunchKernelGGL(loop_run_kernel(N), dim3((unsigned)(p->S * p->G)), dim3(64), 0, st, e0, e1, 0, pa, ga, sa,
                          p->d_aggrec);
  else
    hipExtLaunchKernelGGL(loop_iter_kernel(N), dim3((unsigned)(p->S * p->G)), dim3(64), 0, st, e0, e1, 0, pa, ga, sa,
                          p->d_aggrec, m);
  HIPCHK(p, hipGetLastError());
  plan_prof_end(p, LOMPC_PLAN_K_PATH, e0, e1);
  return LOMPC_OK;
}

void lq_plan_free(lompc_plan* p) {
  if (!p) return;
  (void)hipSetDevice(p->device);
  (void)hipDeviceSynchronize();
  void* ptrs[] = {p->d_meta,  p->d_stats_own, p->d_window, p->d_partial, p->t_cnt,     p->t_lo,      p->t_ge,         p->t_cf,
                  p->t_ab,    p->t_sl,        p->d_ws,      p->d_errflag,
                  p->d_fail_cnt, p->d_fail_idx, p->d_tally, p->d_wacc, p->d_arrive, p->d_xsend, p->d_xrecv, p->d_loop, p->d_aggrec,
                  p->d_bsum, p->d_P, p->d_pos, p->d_sinfo};
  for (void* x : ptrs)
    if (x) (void)hipFree(x);
  {
    auto& z = p->stp;
    for (int k = 0; k < 2; ++k) {
      void* zs[] = {z.tab[k].cnt, z.tab[k].lo, z.tab[k].ge, z.tab[k].cf, z.tab[k].ab, z.part[k], z.fcnt[k], z.fidx[k]};
      for (void* x : zs)
        if (x) (void)hipFree(x);
    }
    for (void* x : {(void*)z.d_map, (void*)z.sl3, (void*)z.wt.cnt, (void*)z.wt.lo, (void*)z.wt.ge, (void*)z.wt.cf,
                    (void*)z.wt.ab, (void*)z.wt.sl, (void*)z.rpart, (void*)z.rfcnt, (void*)z.rfidx})
      if (x) (void)hipFree(x);
    if (z.h_map) (void)hipHostFree(z.h_map);
  }
  if (p->h_buf) (void)hipHostFree(p->h_buf);

  if (p->h_loop) (void)hipHostFree(p->h_loop);
  if (p->h_dec) (void)hipHostFree(p->h_dec);
  if (p->ev_stage) (void)hipEventDestroy(p->ev_stage);
  for (auto& v : p->prof_ev)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  for (hipEvent_t e : p->prof_pool) (void)hipEventDestroy(e);
  delete p;
}

extern "C" {

#ifdef LOMPC_STAMPS
int lompc_debug_wstart(long long* host, int n) {
  if (n > 32768 * 8) n = 32768 * 8;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_wstart), sizeof(long long) * n, 0, hipMemcpyDeviceToHost) == hipSuccess
             ? LOMPC_OK
             : LOMPC_ERR_HIP;
}
int lompc_debug_loopstamps(unsigned long long* host, int reset) {  // [64][16] (g_lstamps)
  if (hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lstamps), sizeof(g_lstamps), 0, hipMemcpyDeviceToHost) != hipSuccess)
    return LOMPC_ERR_HIP;
  if (reset) {
    static const unsigned long long z[64 * 16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lstamps), z, sizeof(z), 0, hipMemcpyHostToDevice) != hipSuccess)
      return LOMPC_ERR_HIP;
  }
  return LOMPC_OK;
}
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

int lompc_plan_update(lompc_plan* p, int64_t B, const double* gamma, const int64_t* set_offsets,
                      const double* w_ref, void* stream) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  int64_t spc[LQ_PLAN_MAX_CTX];
  for (int k = 0, prev = 0; k < p->nctx; ++k) {  // the plan's set counts per context
    const int e = k + 1 < p->nctx ? p->ce.end[k] : (int)p->S;
    spc[k] = e - prev;
    prev = e;
  }
  return lq_plan_prepare(p, p->nctx, p->ctx, spc, B, gamma, set_offsets, w_ref, p->flags, (hipStream_t)stream);
}

int lompc_plan_reserve(lompc_plan* p, int64_t max_B) {
  if (!p || max_B < 0 || max_B >= (1ll << 31) - EVAL_MAXB) return LOMPC_ERR_INVALID_ARG;
  p->reserve_B = max_B;
  return LOMPC_OK;
}

}  // extern "C"

// the message for QPs reported failed by a gamma-sorted plan: a set whose gamma is not ascending
// (k_agg reports all its EVs failed) says so instead of "no certified optimum" (synchronises `st`)
const char* lq_failed_text(lompc_plan* p, hipStream_t st) {
  const char* none = "LoMPC QPs without a certified optimum";
  if (!p->sorted || !p->d_sinfo || p->S < 1) return none;
  std::vector<int4> si((size_t)p->S);
  if (hipMemcpyAsync(si.data(), p->d_sinfo, si.size() * sizeof(int4), hipMemcpyDeviceToHost, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return none;
  for (const int4& x : si)
    if (x.y == 0) return "LOMPC_PLAN_SORTED_GAMMA: a set's valid gamma is not ascending (all its EVs reported failed)";
  return none;
}

// The host form of lompc_price_loop (device_loop = 0): per iteration one plan run, one D2H copy and a
// stream sync, the convergence test and lompc_price_step on the host.  Arguments checked by the caller.
int lq_price_loop_host(lompc_plan* p, const lompc_price_loop_args* a, double* lmbd, double* w_k, double* dual_cost,
                       double* dec_actual, double* dec_pred, int* iterations, double* errs, hipStream_t st) {
  const int N = a->N, r = a->r, N3 = 3 * N;
  const size_t n_in = (size_t)6 * N + 2 + 2 * N;
  // per-part timing (args->prof): host clock for issue / wait / price step, HIP events for the
  // GPU span of every engine call (H2D copy .. D2H copy)
  double* prof = a->prof;
  hipEvent_t pe[2] = {nullptr, nullptr};
  if (prof) {
    for (hipEvent_t& x : pe) HIPCHK(p, hipEventCreateWithFlags(&x, hipEventDefault));
  }
  struct EvGuard {
    hipEvent_t* e;
    ~EvGuard() {
      for (int k = 0; k < 2; ++k)
        if (e[k]) (void)hipEventDestroy(e[k]);
    }
  } ev_guard{pe};
  auto now_us = []() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t_start = prof ? now_us() : 0.0;
  // one engine call at prices x: the batch errors and the central solve (price_solver.py:106/:132)
  double e[3] = {0.0, 0.0, 0.0};
  double cost_c = 0.0;
  auto iterate = [&](const double* x) -> int {
    const double t0 = prof ? now_us() : 0.0;
    if (prof) HIPCHK(p, hipEventRecord(pe[0], st));
    double* h = a->host_in;
    memcpy(h, x, N3 * sizeof(double));
    memcpy(h + N3, x, N3 * sizeof(double));
    h[2 * N3] = h[2 * N3 + 1] = a->lmbd_r;
    memcpy(h + 2 * N3 + 2, a->w_ref, N * sizeof(double));
    memcpy(h + 2 * N3 + 2 + N, a->w_ref, N * sizeof(double));
    HIPCHK(p, hipMemcpyAsync(a->dev_in, h, n_in * sizeof(double), hipMemcpyHostToDevice, st));
    const int rc = lq_plan_launch(p, a->dev_in, a->dev_in + 2 * N3, nullptr, nullptr, nullptr, nullptr,
                                  const_cast<double*>(a->dev_sw), const_cast<double*>(a->dev_st), st, nullptr);
    if (rc) return rc;
    if (a->dev_sw != a->host_sw)  // (pinned outputs written by the kernel itself need no copy)
      HIPCHK(p, hipMemcpyAsync(a->host_sw, a->dev_sw, 2 * N * sizeof(double), hipMemcpyDeviceToHost, st));
    if (a->dev_st != a->host_st)
      HIPCHK(p, hipMemcpyAsync(a->host_st, a->dev_st, 2 * LOMPC_SET_STATS * sizeof(double), hipMemcpyDeviceToHost,
                               st));
    double t1 = 0.0;
    if (prof) {
      HIPCHK(p, hipEventRecord(pe[1], st));
      t1 = now_us();
    }
    HIPCHK(p, hipStreamSynchronize(st));
    if (prof) {
      const double t2 = now_us();
      float ms = 0.f;
      HIPCHK(p, hipEventElapsedTime(&ms, pe[0], pe[1]));
      prof[LOMPC_LOOP_PROF_ITERS] += 1.0;
      prof[LOMPC_LOOP_PROF_ISSUE] += t1 - t0;
      prof[LOMPC_LOOP_PROF_WAIT] += t2 - t1;
      prof[LOMPC_LOOP_PROF_GPU] += 1e3 * ms;
    }
    const double* sw = a->host_sw;
    const double* sst = a->host_st;
    for (int s = 0; s < 2; ++s) {
      if (sst[s * LOMPC_SET_STATS + LOMPC_STAT_N_INVALID] > 0) return fail_arg(p, "gamma outside [0, y_max]");
      if (sst[s * LOMPC_SET_STATS + LOMPC_STAT_N_FAILED] > 0) {
        p->err = lq_failed_text(p, st);
        return LOMPC_ERR_NOT_CONVERGED;
      }
    }
    double qf = 0.0;  // (w_avg - w_ref)' A_bar (w_avg - w_ref)  (price_solver.py:210-214)
    for (int i = 0; i < N; ++i) {
      const double di = sw[i] / a->n_evs - a->w_ref[i];
      double acc = 0.0;
      for (int j = 0; j < N; ++j) acc += a->A_bar[(size_t)i * N + j] * (sw[j] / a->n_evs - a->w_ref[j]);
      qf += di * acc;
    }
    e[0] = sst[LOMPC_STAT_MAX_ERR];
    e[1] = std::fabs(sw[0] / a->n_evs - a->w_ref[0]);
    e[2] = std::sqrt(qf);
    memcpy(w_k, sw + N, N * sizeof(double));
    cost_c = sst[LOMPC_SET_STATS + LOMPC_STAT_SUM_COST];
    return LOMPC_OK;
  };
  // phi(w_ref) (lompc.py:172-177)
  std::vector<double> phi_ref(N3), lm(lmbd, lmbd + N3), lm_new(N3, 0.0);
  const double q_s = 3.0 * a->theta / (4.0 * a->w_max);
  for (int t = 0; t < N; ++t) {
    phi_ref[t] = a->theta * a->w_ref[t];
    phi_ref[N + t] = a->theta * (a->w_max - a->w_ref[t]);
    phi_ref[2 * N + t] = q_s * a->w_ref[t] * a->w_ref[t];
  }
  int rc = iterate(lm.data());
  if (rc) return rc;
  double dc = cost_c;
  int it = 0;
  for (it = 0; it < a->max_iter; ++it) {
    if ((a->tol_avg ? e[2] : e[0]) <= a->tol) break;
    double dec = 0.0;
    int qit = 0;
    const double ts = prof ? now_us() : 0.0;
    rc = lompc_price_step(N, r, a->theta, a->w_max, a->m, a->kappa, a->eps_reg, a->w_ref, w_k, lm.data(),
                          lm_new.data(), &dec, &qit);
    if (prof) prof[LOMPC_LOOP_PROF_STEP] += now_us() - ts;
    if (rc) {
      p->err = "price-gradient QP: no certified optimum";
      return rc;
    }
    rc = iterate(lm_new.data());
    if (rc) return rc;
    double dterm = 0.0;  // (lmbd_k - lmbd_k_new) @ phi(w_ref): the reference's two arrays alias
    if (it == 0)         // after the first iteration (lmbd_k = lmbd_k_new), so the term is 0 then
      for (int i = 0; i < N3; ++i) dterm += (lm[i] - lm_new[i]) * phi_ref[i];
    if (dec_actual) dec_actual[it] = cost_c - dc + dterm;
    if (dec_pred) dec_pred[it] = dec;
    dc = cost_c;
    lm = lm_new;
  }
  *iterations = it;  // steps taken (= the reference's `iter` unless the cap was hit: then max_iter)
  if (prof) {
    const double wall = now_us() - t_start;
    prof[LOMPC_LOOP_PROF_WALL] += wall;
    // the rest of the loop's host time: convergence test, A_bar metric, copies into the staging
    prof[LOMPC_LOOP_PROF_HOST] = prof[LOMPC_LOOP_PROF_WALL] - prof[LOMPC_LOOP_PROF_ISSUE] -
                                 prof[LOMPC_LOOP_PROF_WAIT] - prof[LOMPC_LOOP_PROF_STEP];
  }
  memcpy(lmbd, lm.data(), N3 * sizeof(double));
  if (dual_cost) *dual_cost = dc;
  if (errs) memcpy(errs, e, sizeof(e));
  return LOMPC_OK;
}

// The stepped form's block map, tables and records (once per prepare).  The path takes np_wg of the
// k_step workgroup slots for the whole launch, so the evaluation blocks are sized to fill the rest once
// (or a whole number of times for big batches).
// the wide form's evaluation takes k_evals_st (the stager wave) when its compact table and lane maps fit
bool evals_stg_ok(const lompc_plan* p) { return LQ_EVALS_STAGER && p->G <= 64 && p->N + 4 <= 64; }

int stepped_setup(lompc_plan* p, hipStream_t st, bool wide) {
  auto& z = p->stp;
  const int N = p->N;
  const int64_t S = p->S, G = p->G, ncell = S * G, B = p->B;
  const bool stg = wide && evals_stg_ok(p);
  const int cap = std::min(stg ? LQ_EVALS_CAP : LQ_PIECE_CAP, p->G * LQ_PPL);
  const int64_t okey = ((int64_t)N * 4096 + G) * 2 + (stg ? 1 : 0);
  if (z.occ_key != okey) {
    if (stg)
      HIPCHK(p, hipOccupancyMaxActiveBlocksPerMultiprocessor(&z.occ, evals_st_kernel(N), EVAL_EVS, evals_st_lds(N, p->G, cap)));
    else
      HIPCHK(p, hipOccupancyMaxActiveBlocksPerMultiprocessor(&z.occ, step_kernel(N), EVAL_EVS, eval_lds(N, p->G, cap)));
    z.occ = std::max(z.occ, 1);
    z.occ_key = okey;
  }
  const int64_t maxb = stg ? LQ_EVALS_MAXB : EVAL_MAXB;  // EVs per block at most
  z.np_wg = wide ? 0 : (int)((ncell + LQ_STEP_CELLS - 1) / LQ_STEP_CELLS);  // (wide: the paths have their own launch)
  const int64_t slots = (int64_t)p->n_cu * z.occ;
  const int64_t free1 = std::max<int64_t>(slots - z.np_wg, slots / 2);  // the first round, beside the path
  const int64_t rounds = std::max<int64_t>(1, (10 * B + 9ll * slots * maxb - 1) / (9ll * slots * maxb));
  const int64_t target = free1 + (rounds - 1) * slots;
  std::vector<int64_t> off(S + 1);
  {  // the set offsets from the prepared map (host copy kept in the pinned metadata)
    const int64_t* hoff = reinterpret_cast<const int64_t*>(p->h_buf + p->h_off_at);
    for (int64_t s = 0; s <= S; ++s) off[s] = hoff[s];
  }
  // the block map: (set, first EV, end EV) per k_evals / k_step workgroup, and each set's first block
  // (the wide form's: one dispatch round, weighted as lq_plan_prepare's — the same map, so the same bits)
  std::vector<int4> blks;
  std::vector<int> pre;
  block_map(off.data(), S, B, maxb, target, p->n_cu, wide && rounds == 1, blks, pre);
  int64_t nblk = (int64_t)blks.size();
  const size_t o_pre = ((size_t)nblk * sizeof(int4) + 15) & ~(size_t)15;
  const size_t bytes = o_pre + (size_t)(S + 1) * sizeof(int);
  int rc;
  if ((int64_t)bytes > z.cap_map) {
    if (z.h_map) HIPCHK(p, hipHostFree(z.h_map));
    z.h_map = nullptr;
    HIPCHK(p, hipHostMalloc((void**)&z.h_map, bytes, hipHostMallocDefault));
    if ((rc = grow(p, &z.d_map, bytes))) return rc;
    z.cap_map = (int64_t)bytes;
  }
  HIPCHK(p, hipStreamSynchronize(st));  // (the pinned map may still feed an earlier copy)
  memcpy(z.h_map, blks.data(), (size_t)nblk * sizeof(int4));
  memcpy(z.h_map + o_pre, pre.data(), (size_t)(S + 1) * sizeof(int));
  HIPCHK(p, hipMemcpyAsync(z.d_map, z.h_map, bytes, hipMemcpyHostToDevice, st));
  z.nblk = (int)nblk;
  if (ncell > z.cap_cells) {
    for (int k = 0; k < 2; ++k) {
      auto& t = z.tab[k];
      if ((rc = grow(p, &t.cnt, ncell)) || (rc = grow(p, &t.lo, ncell)) || (rc = grow(p, &t.ge, ncell * LQ_PPL)) ||
          (rc = grow(p, &t.cf, ncell * LQ_PPL * 8)) || (rc = grow(p, &t.ab, ncell * LQ_PPL * N)))
        return rc;
    }
    if ((rc = grow(p, &z.sl3, 3 * (size_t)ncell * 64))) return rc;
    z.cap_cells = ncell;
  }
  if (nblk > z.cap_blk) {
    for (int k = 0; k < 2; ++k)
      if ((rc = grow(p, &z.part[k], (size_t)nblk * (N + NPX))) || (rc = grow(p, &z.fcnt[k], (size_t)nblk * EVAL_WAVES)) ||
          (rc = grow(p, &z.fidx[k], (size_t)nblk * EVAL_MAXB)))
        return rc;
    z.cap_blk = nblk;
  }
  z.ok = true;
  z.wide = wide;
  z.stg = stg;
  return LOMPC_OK;
}

#ifndef LQ_WIDE_RUNS
#define LQ_WIDE_RUNS 64                 // wide form: runs per path launch (its table ring holds one more; 64: 13.96
                                        // vs 14.32 us per step over 64 steps with 32 — the paths' launch tail amortised)
#endif
#define LQ_WIDE_BYTES (1ll << 30)        // wide form: the table ring's memory at most

// The wide form's runs per path launch for K runs: bounded by the table ring's memory
// (LQ_WIDE_BYTES) and the grid (fit: the most the plan allows; < 1: the plan is too big for two slots)
int64_t wide_fit(const lompc_plan* p) {
  const int64_t ncell = p->S * p->G;
  const int64_t cell_bytes = LQ_PPL * (16 * (int64_t)p->N + 8 * 8 + 8) + 4 + 8 + 64;
  return std::min<int64_t>(LQ_WIDE_BYTES / (ncell * cell_bytes), INT32_MAX / 64 / ncell) - 1;
}

// the wide form's table ring, sized for the largest group the plan allows whatever this call's K (a
// later call with more runs must not reallocate — hipMalloc / hipFree synchronise the device)
int wide_ring(lompc_plan* p, hipStream_t st) {
  auto& z = p->stp;
  int rc;
  const int N = p->N;
  const int64_t ncell = p->S * p->G;
  const int64_t ring = (std::min<int64_t>(LQ_WIDE_RUNS, wide_fit(p)) + 1) * ncell;
  if (ring > z.cap_wt) {
    auto& t = z.wt;
    const int64_t c = ring;
    if ((rc = grow(p, &t.cnt, c)) || (rc = grow(p, &t.lo, c)) || (rc = grow(p, &t.ge, c * LQ_PPL)) ||
        (rc = grow(p, &t.cf, c * LQ_PPL * 8)) || (rc = grow(p, &t.ab, c * LQ_PPL * N)) || (rc = grow(p, &t.sl, c * 64)))
      return rc;
    // every slot written once now, in the call that sizes the ring (a plan's first wide call: the
    // warmup), so a later call's first use of a slot meets no cold page translations
    HIPCHK(p, hipMemsetAsync(t.ge, 0, (size_t)c * LQ_PPL * sizeof(*t.ge), st));
    HIPCHK(p, hipMemsetAsync(t.cf, 0, (size_t)c * LQ_PPL * 8 * sizeof(*t.cf), st));
    HIPCHK(p, hipMemsetAsync(t.ab, 0, (size_t)c * LQ_PPL * N * sizeof(*t.ab), st));
    HIPCHK(p, hipMemsetAsync(t.sl, 0, (size_t)c * 64 * sizeof(*t.sl), st));
    z.cap_wt = c;
  }
  return LOMPC_OK;
}

// K >= 1 independent runs.  Two schedules, one per plan kind:
// * wide (no warm start — every run's path depends on its own prices only): the paths of up to
//   LQ_WIDE_RUNS runs in ONE k_paths launch, then launch k (0 <= k <= K) = k_step(run k's evaluation
//   (k < K), run k - 1's closing (k >= 1)), the next runs' paths launched before the first launch that
//   needs them.  Run j's tables sit in ring slot j % (LQ_WIDE_RUNS + 1) (a slot is rewritten only after
//   its run has closed), records j % 2.  K + 1 evaluation / closing launches + ceil(K / LQ_WIDE_RUNS)
//   path launches.
// * stepped (warm-started plans: run j + 1's path starts from run j's working sets): launch 0 = run
//   0's path; launch k (1 <= k <= K) = k_step(run k's path (k < K), run k - 1's evaluation, run k - 2's
//   closing (k >= 2)); launch K + 1 = run K - 1's closing.  Run j uses path table j % 2, records j % 2
//   and cell-start working sets j % 3.
// Per-EV outputs: run k writes w + k ev_stride N (cost, w0, status + k ev_stride); with ev_stride = 0
// every run writes the same rows and only the LAST run's closing writes per-EV outputs (every earlier
// closing shares its launch with a later run's evaluation, whose rows must win).  Set outputs of run
// k at the per-run strides.  With a communicator, run j's closing fills send slot j % 2 and its
// all-gather + combine follow the launch that carried it, on the same stream (one collective per run).
// split (LOMPC_STEPS_PER_KERNEL): every launch above issued as one launch per part (path / evaluation
// / closing), in that order — the same kernels on the same arguments without the overlap, so the same
// bits (what the bench's verification compares).  span: one event pair from the start of the first
// steady launch's dispatch (the first that carries an evaluation and a closing) to the end of the last
// steady one of the first path group (hipExtLaunchKernel events), read as that many launches.
int lq_run_steps_stepped(lompc_plan* p, const double* lmbd, int64_t lmbd_stride, const double* lmbd_r,
                         int64_t lmbd_r_stride, int n_runs, int profile_every, bool span_events, double* w, double* cost,
                         double* w0, int8_t* status, int64_t ev_stride, double* set_sum_w, int64_t sw_stride,
                         double* set_stats, int64_t st_stride, bool split, hipStream_t st) {
  auto& z = p->stp;
  int rc;
  const int N = p->N;
  const int64_t ncell = p->S * p->G, L = p->S * (N + LOMPC_SET_STATS);
  const int K = n_runs;
  // wide: runs per path launch (wide_fit); a plan too big for two table slots takes the stepped form
  const int64_t fit = wide_fit(p);
  const int Kc = (int)std::min<int64_t>({(int64_t)K, LQ_WIDE_RUNS, fit});
  const bool wide = (p->flags & LOMPC_PLAN_WARM_START) == 0 && Kc >= 1;
  const int slots = Kc + 1;
  if ((!z.ok || z.wide != wide || z.stg != (wide && evals_stg_ok(p))) && (rc = stepped_setup(p, st, wide))) return rc;
  const bool xr = p->comm != nullptr;
  if (xr && (rc = lq_xbufs(p, 2))) return rc;
  if (wide && (rc = wide_ring(p, st))) return rc;
  auto tab = [&](int j) {
    if (wide) {  // ring slot j % slots
      const int64_t o = (int64_t)(j % slots) * ncell;
      PathTab t;
      t.cnt = z.wt.cnt + o;
      t.lo = z.wt.lo + o;
      t.ge = z.wt.ge + o * LQ_PPL;
      t.cf = z.wt.cf + o * LQ_PPL * 8;
      t.ab = z.wt.ab + o * LQ_PPL * N;
      t.sl = z.wt.sl + o * 64;
      return t;
    }
    PathTab t = z.tab[j & 1];
    t.sl = z.sl3 + (size_t)(j % 3) * ncell * 64;
    return t;
  };
  auto lm = [&](int j) { return lmbd + (size_t)j * lmbd_stride; };
  auto lr = [&](int j) { return lmbd_r + (size_t)j * lmbd_r_stride; };
  auto sw_of = [&](int j) { return set_sum_w ? set_sum_w + (size_t)j * sw_stride : nullptr; };
  auto st_of = [&](int j) { return set_stats ? set_stats + (size_t)j * st_stride : nullptr; };
  auto xsend = [&](int j) { return p->d_xsend + (size_t)(j & 1) * L; };
  auto args = [&](int j, EvalArgs& a, FinalArgs& r) {
    const size_t eo = (size_t)j * ev_stride;
    eval_args(p, lm(j), lr(j), w ? w + eo * N : nullptr, cost ? cost + eo : nullptr, w0 ? w0 + eo : nullptr,
              status ? status + eo : nullptr, tab(j), a, r);
    a.blk = reinterpret_cast<const int4*>(z.d_map);
    a.nblk = z.nblk;
    a.partial = z.part[j & 1];
    r.partial = z.part[j & 1];
    a.fail_cnt = z.fcnt[j & 1];
    r.fail_cnt = z.fcnt[j & 1];
    a.fail_idx = z.fidx[j & 1];
    r.fail_idx = z.fidx[j & 1];
    r.blk_prefix = reinterpret_cast<const int*>(z.d_map + (((size_t)z.nblk * sizeof(int4) + 15) & ~(size_t)15));
    r.set_sum_w = xr ? xsend(j) : sw_of(j);
    r.set_stats = xr ? xsend(j) + p->S * N : st_of(j);
    if (ev_stride == 0 && j != K - 1) {  // (its re-solved rows would race a later evaluation's)
      r.w = r.cost = r.w0 = nullptr;
      r.status = nullptr;
    }
  };
  const int cap = std::min(LQ_PIECE_CAP, p->G * LQ_PPL);
  const size_t lds = eval_lds(N, p->G, cap);
  const StepKernel kern = step_kernel(N);
  // (split runs without w output take the batched launches one run per group too: their evaluation
  // sums the certified pieces instead of rows, so only these kernels give the wide form's bits)
  if (wide && (!split || z.stg || !w)) {
    // batched: per path group of n <= Kc runs THREE launches — k_paths (the n paths), k_evals (the n
    // evaluations, each workgroup through its block of every run) and k_closes (the n x S closings);
    // the same kernels' arithmetic as the split form below, so the same bits
    // record slots x blocks, bounded like the table ring: a run's slot holds every block's record, its
    // re-solve counts and its re-solve list (EVAL_MAXB indices per block), so a batch of many blocks
    // takes smaller groups instead of gigabytes of mostly empty lists (the runs are independent: the
    // group size changes no bits)
    const int64_t rec_run = (int64_t)z.nblk * ((N + NPX) * 8 + EVAL_WAVES * 4 + EVAL_MAXB * 4);
    const int64_t kr = std::max<int64_t>(1, std::min<int64_t>(std::min<int64_t>(LQ_WIDE_RUNS, fit), LQ_WIDE_BYTES / rec_run));
    const int64_t need = kr * z.nblk;
    if (need > z.cap_rrec) {
      if ((rc = grow(p, &z.rpart, need * (N + NPX))) || (rc = grow(p, &z.rfcnt, need * EVAL_WAVES)) ||
          (rc = grow(p, &z.rfidx, need * EVAL_MAXB)))
        return rc;
      // (touched once here, as the table ring)
      HIPCHK(p, hipMemsetAsync(z.rpart, 0, (size_t)need * (N + NPX) * sizeof(*z.rpart), st));
      HIPCHK(p, hipMemsetAsync(z.rfcnt, 0, (size_t)need * EVAL_WAVES * sizeof(*z.rfcnt), st));
      HIPCHK(p, hipMemsetAsync(z.rfidx, 0, (size_t)need * EVAL_MAXB * sizeof(*z.rfidx), st));
      z.cap_rrec = need;
    }
    if (xr && (rc = lq_xbufs(p, Kc, Kc))) return rc;
    EvalArgs ea;
    FinalArgs ff;
    eval_args(p, lmbd, lmbd_r, w, cost, w0, status, tab(0), ea, ff);
    ea.piece_sums = w ? 0 : 1;  // (no rows to store: the per-stage sums from the piece aggregates)
    ea.blk = reinterpret_cast<const int4*>(z.d_map);
    ea.nblk = z.nblk;
    ea.partial = z.rpart;
    ff.partial = z.rpart;
    ea.fail_cnt = z.rfcnt;
    ff.fail_cnt = z.rfcnt;
    ea.fail_idx = z.rfidx;
    ff.fail_idx = z.rfidx;
    ff.blk_prefix = reinterpret_cast<const int*>(z.d_map + (((size_t)z.nblk * sizeof(int4) + 15) & ~(size_t)15));
    ff.set_sum_w = xr ? p->d_xsend : set_sum_w;
    ff.set_stats = xr ? p->d_xsend + p->S * N : set_stats;
    // (k_evals_st's split form: the same three kernels, one run per group — its arithmetic is not
    // k_step's: the stager leaves seven waves to the rows, so the row sums group differently)
    const int grp = split ? 1 : (int)std::min<int64_t>(Kc, kr);
    if (z.stg) ea.cap = std::min(LQ_EVALS_CAP, p->G * LQ_PPL);
    const size_t lds_e = z.stg ? evals_st_lds(N, p->G, ea.cap) : lds;
    for (int g0 = 0; g0 < K; g0 += grp) {
      const int n = std::min(grp, K - g0);
      {
        PathArgs pw = path_args(p, lmbd, lmbd_r, z.wt);
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (plan_prof_begin(p, LOMPC_PLAN_K_PATH, &e0, &e1)) return fail_arg(p, "profiling events");
        hipExtLaunchKernelGGL(paths_kernel(N), dim3((unsigned)(n * ncell)), dim3(64), 0, st, e0, e1, 0, pw, lmbd_stride,
                              lmbd_r_stride, g0, slots);
        HIPCHK(p, hipGetLastError());
        plan_prof_end(p, LOMPC_PLAN_K_PATH, e0, e1);
      }
      {  // the evaluation launch carries the K_EVAL timing (span: the first group's only), as n runs
        hipEvent_t e0 = nullptr, e1 = nullptr;
        const bool ev = !span_events || g0 == 0;
        if (ev && plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &e0, &e1)) return fail_arg(p, "profiling events");
        const EvalsArgs x{g0, n, slots, z.nblk, lmbd_stride, lmbd_r_stride, ev_stride, ncell};
        hipExtLaunchKernelGGL(z.stg ? evals_st_kernel(N) : evals_kernel(N), dim3((unsigned)z.nblk), dim3(EVAL_EVS), lds_e, st,
                              e0, e1, 0, ea, x);
        HIPCHK(p, hipGetLastError());
        if (ev) plan_prof_end(p, LOMPC_PLAN_K_EVAL, e0, e1, n);
      }
      {
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (plan_prof_begin(p, LOMPC_PLAN_K_FINAL, &e0, &e1)) return fail_arg(p, "profiling events");
        const ClosesArgs c{g0, n, slots, z.nblk, (int)p->S, K - 1, xr ? 1 : 0, lmbd_stride, lmbd_r_stride, ev_stride,
                           xr ? L : sw_stride, xr ? L : st_stride, ncell};
        hipExtLaunchKernelGGL(k_closes, dim3((unsigned)(n * p->S)), dim3(256), 0, st, e0, e1, 0, ff, c);
        HIPCHK(p, hipGetLastError());
        plan_prof_end(p, LOMPC_PLAN_K_FINAL, e0, e1, n);
      }
      if (xr) {  // ONE collective for the group's n runs (their send records are contiguous), one combine
        if ((rc = lq_comm_allgather(p->comm, p->d_xsend, p->d_xrecv, (size_t)n * L, st))) {
          p->err = p->comm->err;
          return rc;
        }
        if (set_sum_w || set_stats) {
          const CombineRunsArgs ca{p->d_xrecv, p->comm->nranks, n, (int)p->S, N, g0, K - 1, set_sum_w, set_stats,
                                   sw_stride, st_stride};
          const int64_t tot = (int64_t)n * L;
          hipLaunchKernelGGL(k_combine_runs, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((tot + 255) / 256, 1024))),
                             dim3(256), 0, st, ca);
          HIPCHK(p, hipGetLastError());
        }
      }
    }
    return LOMPC_OK;
  }
  // the steady launches 1 .. K - 1 (stepped: path + evaluation + closing; wide: evaluation +
  // closing); the span events cover 1 .. s_last, wide: the first path group's (no path launch inside)
  const int s_first = 1, s_last = wide ? Kc - 1 : K - 1;
  hipEvent_t span0 = nullptr, span1 = nullptr;
  if (span_events && s_last >= s_first && plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &span0, &span1))
    return fail_arg(p, "profiling events");
  // one k_step launch of (npw path, ne evaluation, nf closing workgroups); prof: its own event pair
  auto launch = [&](const PathArgs& pa, const EvalArgs& ea, const FinalArgs& ff, int npw, int ne, int nf, bool prof,
                    hipEvent_t s0, hipEvent_t s1) -> int {
    if (npw + ne + nf == 0) return LOMPC_OK;
    hipEvent_t e0 = s0, e1 = s1;
    if (prof && plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &e0, &e1)) return fail_arg(p, "profiling events");
    hipExtLaunchKernelGGL(kern, dim3((unsigned)(npw + ne + nf)), dim3(EVAL_EVS), lds, st, e0, e1, 0, pa, ea, ff, npw, ne,
                          nf);
    HIPCHK(p, hipGetLastError());
    if (prof) plan_prof_end(p, LOMPC_PLAN_K_EVAL, e0, e1);
    return LOMPC_OK;
  };
  int paths_to = 0;  // wide: runs whose paths are launched
  const int last = wide ? K : K + 1;
  for (int k = 0; k <= last; ++k) {
    PathArgs pa{};
    int npw = 0;
    EvalArgs ea{}, unused_e;
    FinalArgs ff{}, unused_f;
    int ne = 0, nf = 0;
    if (wide) {
      if (k < K && k >= paths_to) {  // the next group's paths, one launch
        const int n = std::min(Kc, K - k);
        PathArgs pw = path_args(p, lmbd, lmbd_r, z.wt);
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (plan_prof_begin(p, LOMPC_PLAN_K_PATH, &e0, &e1)) return fail_arg(p, "profiling events");
        hipExtLaunchKernelGGL(paths_kernel(N), dim3((unsigned)(n * ncell)), dim3(64), 0, st, e0, e1, 0, pw, lmbd_stride,
                              lmbd_r_stride, k, slots);
        HIPCHK(p, hipGetLastError());
        plan_prof_end(p, LOMPC_PLAN_K_PATH, e0, e1);
        paths_to = k + n;
      }
      if (k < K) {
        args(k, ea, unused_f);
        ne = z.nblk;
      }
      if (k >= 1) {
        args(k - 1, unused_e, ff);
        nf = (int)p->S;
      }
    } else {
      if (k < K) {
        pa = path_args(p, lm(k), lr(k), tab(k));
        npw = z.np_wg;
      }
      if (k >= 1 && k - 1 < K) {
        args(k - 1, ea, unused_f);
        ne = z.nblk;
      }
      if (k >= 2) {
        args(k - 2, unused_e, ff);
        nf = (int)p->S;
      }
    }
    int npw_l = npw;
#ifdef LQ_STEP_DIAG
    // diagnostic builds only (-DLQ_STEP_DIAG=1 / 2, timing of the launch's parts): from launch 3 on,
    // 1 drops the path workgroups, 2 the evaluation and closing workgroups; outputs are not the runs'
    if (k >= 3 && k < K) {
      if (LQ_STEP_DIAG == 1) npw_l = 0;
      if (LQ_STEP_DIAG == 2) ne = nf = 0;
    }
#endif
    // the steady launches carry the events: sampled, or one pair around all of them
    const bool steady = k >= 1 && k <= K - 1;
    const bool prof = !span_events && steady && (profile_every <= 0 || (k - 1) % profile_every == 0);
    const hipEvent_t s0 = (span0 && k == s_first) ? span0 : nullptr, s1 = (span0 && k == s_last) ? span1 : nullptr;
    if (split) {  // the same parts, one launch each (no overlap)
      if ((rc = launch(pa, ea, ff, npw_l, 0, 0, false, nullptr, nullptr)) ||
          (rc = launch(pa, ea, ff, 0, ne, 0, prof, s0, s1)) || (rc = launch(pa, ea, ff, 0, 0, nf, false, nullptr, nullptr)))
        return rc;
    } else if ((rc = launch(pa, ea, ff, npw_l, ne, nf, prof, s0, s1))) {
      return rc;
    }
    if (s1) plan_prof_end(p, LOMPC_PLAN_K_EVAL, span0, span1, s_last - s_first + 1);
    const int closed = wide ? k - 1 : k - 2;  // the run closed by this launch
    if (xr && nf && (rc = lq_exchange(p, xsend(closed), sw_of(closed), st_of(closed), st))) return rc;
  }
  return LOMPC_OK;
}

// Reductions-only runs over gamma-sorted sets (k_agg plans), wide: per group of up to Kc runs TWO
// launches — k_paths (the group's paths into the table ring, as the wide form) and k_aggs (one
// workgroup per (run, set): k_agg's per-piece aggregation on run j's tables).  The same kernels'
// arithmetic as one k_path + k_agg per run (the sequential form, LOMPC_STEPS_PER_KERNEL), so the same
// bits.  With a communicator the group's closings fill its contiguous send records: ONE all-gather and
// one combine per group, as the wide form.  K_EVAL events: the k_aggs launch, as n runs.
int lq_run_steps_aggs(lompc_plan* p, const double* lmbd, int64_t lmbd_stride, const double* lmbd_r,
                      int64_t lmbd_r_stride, int K, bool span_events, double* set_sum_w, int64_t sw_stride,
                      double* set_stats, int64_t st_stride, hipStream_t st) {
  int rc;
  const int N = p->N;
  const int64_t ncell = p->S * p->G, L = p->S * (N + LOMPC_SET_STATS);
  const int Kc = (int)std::min<int64_t>({(int64_t)K, LQ_WIDE_RUNS, wide_fit(p)});
  const int slots = Kc + 1;
  if ((rc = wide_ring(p, st))) return rc;
  const bool xr = p->comm != nullptr;
  if (xr && (rc = lq_xbufs(p, Kc, Kc))) return rc;
  const PathTab& wt = p->stp.wt;
  const PathArgs pw = path_args(p, lmbd, lmbd_r, wt);
  const AggArgs ga{(int)p->S, p->G, N, p->aggF, p->d_q, p->ce, p->d_set_off, p->d_window, p->gamma, lmbd, lmbd_r,
                   p->w_ref, wt.cnt, wt.lo, wt.sl, wt.ge, wt.cf, wt.ab, p->d_P, p->B + p->S, p->d_pos,
                   p->d_sinfo, xr ? p->d_xsend : set_sum_w, xr ? p->d_xsend + p->S * N : set_stats, p->d_stats,
                   p->d_tally, nullptr};
  const int nw = std::min(p->G, (int)LQ_AGG_W);
  for (int g0 = 0; g0 < K; g0 += Kc) {
    const int n = std::min(Kc, K - g0);
    {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      if (plan_prof_begin(p, LOMPC_PLAN_K_PATH, &e0, &e1)) return fail_arg(p, "profiling events");
      hipExtLaunchKernelGGL(paths_kernel(N), dim3((unsigned)(n * ncell)), dim3(64), 0, st, e0, e1, 0, pw, lmbd_stride,
                            lmbd_r_stride, g0, slots);
      HIPCHK(p, hipGetLastError());
      plan_prof_end(p, LOMPC_PLAN_K_PATH, e0, e1);
    }
    {
      hipEvent_t e0 = nullptr, e1 = nullptr;
      const bool ev = !span_events || g0 == 0;
      if (ev && plan_prof_begin(p, LOMPC_PLAN_K_EVAL, &e0, &e1)) return fail_arg(p, "profiling events");
      const AggsArgs x{g0, slots, K - 1, xr ? 1 : 0, lmbd_stride, lmbd_r_stride, xr ? L : sw_stride, xr ? L : st_stride};
      hipExtLaunchKernelGGL(aggs_kernel(N), dim3((unsigned)(n * p->S)), dim3(64 * nw), 0, st, e0, e1, 0, ga, x);
      HIPCHK(p, hipGetLastError());
      if (ev) plan_prof_end(p, LOMPC_PLAN_K_EVAL, e0, e1, n);
    }
    if (xr) {
      if ((rc = lq_comm_allgather(p->comm, p->d_xsend, p->d_xrecv, (size_t)n * L, st))) {
        p->err = p->comm->err;
        return rc;
      }
      if (set_sum_w || set_stats) {
        const CombineRunsArgs ca{p->d_xrecv, p->comm->nranks, n, (int)p->S, N, g0, K - 1, set_sum_w, set_stats,
                                 sw_stride, st_stride};
        const int64_t tot = (int64_t)n * L;
        hipLaunchKernelGGL(k_combine_runs, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>((tot + 255) / 256, 1024))),
                           dim3(256), 0, st, ca);
        HIPCHK(p, hipGetLastError());
      }
    }
  }
  return LOMPC_OK;
}

extern "C" {

int lompc_plan_run(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, void* stream) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  return lq_plan_launch(p, lmbd, lmbd_r, w, cost, w0, status, set_sum_w, set_stats, (hipStream_t)stream, nullptr);
}

int lompc_plan_run_steps(lompc_plan* p, const double* lmbd, int64_t lmbd_stride, const double* lmbd_r,
                         int64_t lmbd_r_stride, int n_runs, int profile_every, double* w, double* cost, double* w0,
                         int8_t* status, double* set_sum_w, double* set_stats, int64_t set_sum_w_stride,
                         int64_t set_stats_stride, int64_t ev_stride, int steps_flags, void* stream) {
  constexpr int known = LOMPC_STEPS_PER_KERNEL | LOMPC_STEPS_SPAN_EVENTS;
  if (!p || n_runs < 0 || profile_every < 0 || set_sum_w_stride < 0 || set_stats_stride < 0 || ev_stride < 0 ||
      (steps_flags & ~known))
    return LOMPC_ERR_INVALID_ARG;
  if (ev_stride > 0 && ev_stride < p->B) return fail_arg(p, "run_steps: 0 or ev_stride >= B required");
  HIPCHK(p, hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  // stepped form: the k_eval / k_finalize plans (not k_agg, not closed inside k_eval on request),
  // cells in whole workgroups of one set; runs without w output take it too (their evaluation then
  // sums the rows it does not store)
  const bool per_ev = w || cost || w0 || status;
  const bool agg = p->sorted && !per_ev;
  // gamma-sorted sets without per-EV output: per group of runs one k_paths and one k_aggs launch
  // (the sequential form below on request: LOMPC_STEPS_PER_KERNEL, the same bits)
  if (n_runs >= 1 && !p->skip && agg && p->nblk > 0 && (p->flags & LOMPC_PLAN_WARM_START) == 0 &&
      !(steps_flags & LOMPC_STEPS_PER_KERNEL) && wide_fit(p) >= 1)
    return lq_run_steps_aggs(p, lmbd, lmbd_stride, lmbd_r, lmbd_r_stride, n_runs,
                             (steps_flags & LOMPC_STEPS_SPAN_EVENTS) != 0, set_sum_w, set_sum_w_stride, set_stats,
                             set_stats_stride, st);
  if (n_runs >= 1 && !p->skip && !agg && !p->close && p->nblk > 0 && p->G % LQ_STEP_CELLS == 0)
    return lq_run_steps_stepped(p, lmbd, lmbd_stride, lmbd_r, lmbd_r_stride, n_runs, profile_every,
                                (steps_flags & LOMPC_STEPS_SPAN_EVENTS) != 0, w, cost, w0, status, ev_stride,
                                set_sum_w, set_sum_w_stride, set_stats, set_stats_stride,
                                (steps_flags & LOMPC_STEPS_PER_KERNEL) != 0, st);
  const int mask = p->prof;
  int rc = LOMPC_OK;
  // run k's closing (k_finalize) rides in run k + 1's path launch (k_path_fin); the last run's
  // closes on its own.  The cell-start working sets alternate halves between runs.
  FinalArgs fin{};
  fin.N = 0;
  for (int k = 0; k < n_runs && rc == LOMPC_OK; ++k) {
    if (profile_every > 0) p->prof = (k % profile_every == 0) ? mask : 0;  // sampled runs carry the events
    const double* lm = lmbd + (size_t)k * lmbd_stride;
    const double* lr = lmbd_r + (size_t)k * lmbd_r_stride;
    const PathTab tb = own_tab(p, k & 1);
    if ((rc = lq_launch_path(p, lm, lr, tb, st, fin.N ? &fin : nullptr))) break;
    const size_t eo = (size_t)k * ev_stride;
    rc = lq_launch_eval(p, lm, lr, w ? w + eo * p->N : nullptr, cost ? cost + eo : nullptr, w0 ? w0 + eo : nullptr,
                        status ? status + eo : nullptr, set_sum_w ? set_sum_w + (size_t)k * set_sum_w_stride : nullptr,
                        set_stats ? set_stats + (size_t)k * set_stats_stride : nullptr, tb, st, nullptr, &fin);
  }
  p->prof = mask;
  if (rc == LOMPC_OK && fin.N) {  // the last run's closing
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)p->S), dim3(256), 0, st, fin);
    HIPCHK(p, hipGetLastError());
  }
  return rc;
}

int lompc_plan_run_chain(lompc_plan* p, const double* lmbd0, const double* lmbd_r, const double* w_target, double step,
                         int n_runs, double* lmbd_out, double* w, double* cost, double* w0, int8_t* status,
                         double* set_sum_w, double* set_stats, void* stream) {
  if (!p || n_runs < 0 || !lmbd0 || !lmbd_r || !w_target || !lmbd_out || !set_sum_w || !set_stats ||
      !(step >= 0.0) || !std::isfinite(step))
    return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  const int N = p->N;
  const size_t L = (size_t)p->S * 3 * N, SN = (size_t)p->S * N, SS = (size_t)p->S * LOMPC_SET_STATS;
  for (int k = 0; k < n_runs; ++k) {
    double* lm = lmbd_out + (size_t)k * L;
    if (k == 0) {
      if (lm != lmbd0) HIPCHK(p, hipMemcpyAsync(lm, lmbd0, L * sizeof(double), hipMemcpyDeviceToDevice, st));
    } else {  // run k's prices from run k - 1's (combined) reductions
      hipLaunchKernelGGL(k_chain_price, dim3((unsigned)p->S), dim3(64 * ((3 * N + 63) / 64)), 0, st, p->d_q, p->ce,
                         p->nctx, N, lm - L, set_sum_w + (k - 1) * SN, set_stats + (k - 1) * SS, w_target, step, lm);
      HIPCHK(p, hipGetLastError());
    }
    const int rc = lq_plan_launch(p, lm, lmbd_r, w, cost, w0, status, set_sum_w + k * SN, set_stats + k * SS, st, nullptr);
    if (rc) return rc;
  }
  return LOMPC_OK;
}

int lompc_plan_status(lompc_plan* p, void* stream, int64_t* n_repaired, int64_t* n_failed, int64_t* n_invalid) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  // the sticky tallies of every run since the last call (finalize_set adds each set's counts)
  unsigned long long h[3] = {0, 0, 0};
  int ef = 0;
  HIPCHK(p, hipMemcpyAsync(h, p->d_tally, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(p, hipMemcpyAsync(&ef, p->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(p, hipMemsetAsync(p->d_tally, 0, sizeof(h), (hipStream_t)stream));
  HIPCHK(p, hipStreamSynchronize((hipStream_t)stream));
  if (n_repaired) *n_repaired = (int64_t)h[0];
  if (n_failed) *n_failed = (int64_t)h[1];
  if (n_invalid) *n_invalid = (int64_t)h[2];
  if (h[1]) p->err = lq_failed_text(p, (hipStream_t)stream);  // (the caller's exception text)
  if (ef) {
    HIPCHK(p, hipMemsetAsync(p->d_errflag, 0, sizeof(int), (hipStream_t)stream));
    return fail_arg(p, "negative or NaN price parameter (lmbd >= 0, lmbd_r >= 0 required)");
  }
  return LOMPC_OK;
}

int lompc_plan_get_info(const lompc_plan* p, int64_t* B, int64_t* S, int* cells, int* eval_workgroups,
                        int* steps_group) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  if (steps_group) *steps_group = p->stp.ok ? (p->stp.stg ? 2 : 1) : 0;
  if (B) *B = p->B;
  if (S) *S = p->S;
  if (cells) *cells = p->G;
  if (eval_workgroups) *eval_workgroups = p->nblk;
  return LOMPC_OK;
}

int lompc_plan_profile_enable(lompc_plan* p, int kernel_mask) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipSetDevice(p->device));
  p->prof = kernel_mask & ((1 << LOMPC_PLAN_KERNELS) - 1);
  while (p->prof && p->prof_pool.size() < 512) {
    hipEvent_t e;
    HIPCHK(p, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    p->prof_pool.push_back(e);
  }
  return LOMPC_OK;
}

int lompc_plan_profile_read(lompc_plan* p, int kernel, double* total_ms, int64_t* launches, int reset) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  if (kernel < 0 || kernel >= LOMPC_PLAN_KERNELS) return fail_arg(p, "profile_read: kernel out of range");
  HIPCHK(p, hipSetDevice(p->device));
  for (int k = 0; k < LOMPC_PLAN_KERNELS; ++k)
    if (plan_events_read(p->prof_ev[k], p->prof_mult[k], p->prof_pool, p->prof_ms[k], p->prof_n[k])) return LOMPC_ERR_HIP;
  if (total_ms) *total_ms = p->prof_ms[kernel];
  if (launches) *launches = p->prof_n[kernel];
  if (reset) {
    p->prof_ms[kernel] = 0.0;
    p->prof_n[kernel] = 0;
  }
  return LOMPC_OK;
}

const char* lompc_plan_last_error(const lompc_plan* p) { return p ? p->err.c_str() : ""; }

int lompc_plan_set_comm(lompc_plan* p, lompc_comm* comm) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  if (comm && comm->device != p->device) return fail_arg(p, "set_comm: the communicator's device differs from the plan's");
  p->comm = comm;
  return LOMPC_OK;
}

int lompc_combine_records(const double* recv, int nranks, int64_t S, int N, double* set_sum_w, double* set_stats,
                          int device, void* stream) {
  if (!recv || nranks < 1 || S < 1 || N < 1 || N > LOMPC_MAX_N || S * (N + LOMPC_SET_STATS) >= (1ll << 31))
    return LOMPC_ERR_INVALID_ARG;
  if (hipSetDevice(device) != hipSuccess) return LOMPC_ERR_HIP;
  lq_combine(recv, nranks, S, N, set_sum_w, set_stats, (hipStream_t)stream);
  return hipGetLastError() == hipSuccess ? LOMPC_OK : LOMPC_ERR_HIP;
}

int lompc_plan_destroy(lompc_plan* p) {
  lq_plan_free(p);
  return LOMPC_OK;
}

}  // extern "C"

// diagnostics (scripts/, not in the header): synchronous copies of a plan's path table and sorted index
extern "C" int lompc_debug_plan_tables(lompc_plan* p, int* cnt, double* lo, double* ge, int* pos, int* sinfo,
                                       unsigned long long* P) {
  if (!p) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(p, hipDeviceSynchronize());
  const size_t nc = (size_t)p->S * p->G;
  if (cnt) HIPCHK(p, hipMemcpy(cnt, p->t_cnt, nc * sizeof(int), hipMemcpyDeviceToHost));
  if (lo) HIPCHK(p, hipMemcpy(lo, p->t_lo, nc * sizeof(double), hipMemcpyDeviceToHost));
  if (ge) HIPCHK(p, hipMemcpy(ge, p->t_ge, nc * LQ_PPL * sizeof(double), hipMemcpyDeviceToHost));
  if (pos && p->d_pos) HIPCHK(p, hipMemcpy(pos, p->d_pos, (size_t)p->S * (p->aggF + 1) * sizeof(int), hipMemcpyDeviceToHost));
  if (sinfo && p->d_sinfo) HIPCHK(p, hipMemcpy(sinfo, p->d_sinfo, (size_t)p->S * sizeof(int4), hipMemcpyDeviceToHost));
  if (P && p->d_P) HIPCHK(p, hipMemcpy(P, p->d_P, (size_t)3 * (p->B + p->S) * sizeof(unsigned long long), hipMemcpyDeviceToHost));
  return LOMPC_OK;
}
