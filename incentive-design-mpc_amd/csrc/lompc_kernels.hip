// lompc_kernels.hip — MI355X (gfx950) kernels and the C-ABI of include/lompc_amd.h.
//
// Hot path replaced: LoMPC.solve_lompc (chargingstation/lompc.py:137-156) called once
// per EV from PriceSolver._get_w_err (price_solver.py:203-209) and
// PriceSolver.get_w0_price0 (price_solver.py:280-283).
//
// Kernels (one batched price iteration = lompc_run = K1 -> K2 -> K3 on one stream):
//   K1  k_path      one wave per (parameter set, gamma cell). PATH mode: the exact
//                   piecewise-affine solution path w*(gamma) on the cell [l h, (l+1) h]:
//                   wave-parallel PDAS at the cell start, then parametric active-set
//                   tracking (homotopy) to the cell end.  Pieces w = a + b gamma are
//                   stored with their working sets and the quadratic-in-gamma
//                   coefficients of the cost and of the squared A_bar error.  Every
//                   stored piece is KKT-certified at both ends; the KKT residual is
//                   convex in gamma along an affine piece, so that certifies every gamma
//                   inside it.  DIRECT mode: the central solution.
//   K2  k_eval      one EV per lane, one wave per workgroup (64 EVs of one set):
//                   w = a + b gamma, cost / err / price0 from the EV's piece; EVs no
//                   certified piece covers are re-solved in place by the whole wave
//                   (wave_solve, certified).  LDS-tile epilogue: coalesced w stores and
//                   deterministic per-workgroup column sums.
//   K2d k_direct    DIRECT mode: every EV solved by its own lane (PDAS warm-started
//                   from the central working set) and KKT-certified; same epilogue,
//                   uncertified EVs listed for K3.
//   K3  k_finalize  per set: (DIRECT mode) re-solves the listed EVs with the whole wave,
//                   then the deterministic reduction of the workgroup partials.
// Inter-workgroup handoffs go through kernel boundaries: an in-kernel release/acquire
// handoff costs an L2 writeback / invalidate per wave on the 8-XCD part (a fused
// single-launch variant measured 2-5x slower; DESIGN.md, "Rejected designs").
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "lompc_qp.hpp"
#include "lompc_wave.hpp"
#include "../../include/lompc_amd.h"

#define EVAL_BLOCK 64  // one wave per workgroup
#define NPX 7          // partial record: [0,N) sum_w, then NPX scalars

enum {  // partial columns after the N sums
  PX_COST = 0,
  PX_PRICE0 = 1,
  PX_MAX_ERR = 2,
  PX_N_OK = 3,
  PX_N_REPAIRED = 4,
  PX_N_FAILED = 5,
  PX_N_INVALID = 6
};

struct KArgs {
  int64_t B;
  int S;
  int nblk;
  int want_err;
  int pad;
  const double* gamma;
  const int* blk_prefix;       // [S+1]
  const int64_t* set_off;      // [S+1]
  const longlong4* blk_info;   // [nblk]  (set, first EV, end EV, -)
  const double* setdata;   // [S][SD]
  PathTable tab;
  const uint8_t* central;  // [S][LQ_STB]
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* partial;    // [nblk][N+NPX]
  int* fail_cnt;      // [nblk]      EVs of the workgroup left for the repair pass
  uint8_t* fail_lane; // [nblk][64]  their lanes, ascending
};

// block -> (set, first EV, end of set) for set-contiguous batches: one scalar load
__device__ __forceinline__ void block_set(const KArgs& a, int b, int& s, int64_t& start, int64_t& end) {
  const longlong4 info = a.blk_info[b];
  s = (int)info.x;
  start = info.y;
  end = info.z;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Cost / A_bar error / price0 of the QP solved by the whole wave (lane t = w_t),
// the wave form of lq_outputs.  Result valid on every lane.
__device__ __forceinline__ EVOut wave_outputs(const QPConst& q, const double* __restrict__ sd, double gamma,
                                              int lane, double w, bool want_err) {
  const int N = q.N;
  const bool act = lane < N;
  lqw::Aff<2> h = lqw::Aff<2>::identity();  // prefix sums of w and of (w - w_ref)
  const double wr = act ? sd[2 * N + lane] : 0.0;
  if (act) {
    h.B[0] = w;
    h.B[1] = w - wr;
  }
  const lqw::Aff<2> Y = lqw::wave_scan(h);
  const double y = Y.B[0], ey = Y.B[1];
  double term = 0.0, eyy = 0.0, edd = 0.0, pwl = 0.0;
  if (act) {
    const double d = sd[lane], e = sd[N + lane];
    term = 0.5 * q.c * y * y - q.c * gamma * y + w * fma(0.5 * d, w, e);
    if (!q.ev_small) pwl = lq_pwl(w * q.inv_wmax);
    eyy = ey * ey;
    edd = (w - wr) * (w - wr);
  }
  const double tw = q.theta * q.w_max;
  EVOut o;
  o.cost = wave_sum(term) + sd[3 * N + 0] + (q.ev_small ? 0.0 : tw * tw * wave_sum(pwl));
  o.err = want_err ? sqrt(wave_sum(eyy) + sd[3 * N + 5] * wave_sum(edd)) : 0.0;
  const double w0 = __shfl(w, 0, 64);
  o.price0 = lq_price0(q, sd, w0);
  return o;
}

// write-through (sc1) stores: 16 B through a buffer descriptor (aux 16 = sc1), 8 B as a relaxed
// agent-scope atomic store (global_store_dwordx2 ... sc1)
typedef unsigned int lq_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t rs, int off, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lq_v4u, make_double2(x, y)), rs, off, 0, 16);
}
__device__ __forceinline__ void st_wt8(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Shared epilogue of the per-EV kernels for one wave of EVs [start, start+64) of set s.
// !INPLACE (K2d): ok lanes carry a certified w[] and outputs; valid-but-not-ok lanes
//   are listed for the repair pass in k_finalize (their rows are rewritten there).
// INPLACE (fused path kernel): repairs already happened in the block; every valid
//   lane carries its final w[] (rep = repaired, ok = certified) and is summed.
template <int NMAX, bool INPLACE = false>
__device__ __forceinline__ void ev_epilogue(const QPConst& q, const int N, const KArgs& a, int b, int64_t start,
                                            int64_t end, bool valid, bool ok, const double (&w)[NMAX],
                                            const EVOut& o, bool rep = false) {
  __shared__ double tile[EVAL_BLOCK * (NMAX + 3)];
  const int TS = N + 3;  // odd for even N: conflict-free row-per-lane ds_write_b64
  const int lane = threadIdx.x;
  const int64_t i = start + lane;
  const bool active = i < end;
  const double fill = valid ? 0.0 : NAN;
  const bool row = INPLACE ? valid : ok;  // rows that carry a result
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < N) tile[lane * TS + t] = row ? w[t] : fill;
  tile[lane * TS + N] = row ? o.cost : fill;
  tile[lane * TS + N + 1] = row ? o.price0 : 0.0;
  tile[lane * TS + N + 2] = row ? o.err : 0.0;
  const unsigned long long okm = __ballot(row);
  const unsigned long long fm = __ballot(valid && !ok);
  const unsigned long long im = __ballot(active && !valid);
  const unsigned long long rm = INPLACE ? __ballot(valid && ok && rep) : 0ull;
  if (!INPLACE) {
    if (valid && !ok) a.fail_lane[(size_t)b * EVAL_BLOCK + __popcll(fm & ((1ull << lane) - 1ull))] = (uint8_t)lane;
    if (lane == 0) a.fail_cnt[b] = __popcll(fm);
  }
  __syncthreads();
  // coalesced WRITE-THROUGH stores (row-major w[B][N]): sc1 stores leave no dirty lines in the
  // XCD's L2, so the kernel boundary behind this launch has no L2 writeback of the outputs to
  // wait for (MI355X_MICROARCH.md: boundary + B / 6 TB/s for B dirty bytes; 16-B sc1 ~ plain)
  const int nrow = (int)min((int64_t)EVAL_BLOCK, end - start);
  if (a.w && nrow > 0) {
    double* wo = a.w + (size_t)start * N;
    if (nrow == EVAL_BLOCK && (N % 2) == 0) {  // full tile, 16 B per lane (start*N*8 is 16-B aligned)
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(wo, (short)0, EVAL_BLOCK * N * (int)sizeof(double), 0x00020000);
#pragma unroll
      for (int r = 0; r < NMAX / 2; ++r) {
        if (r < N / 2) {
          const int e = 2 * (lane + EVAL_BLOCK * r);  // even element index
          const int row = e / N, col = e - row * N;
          st_wt16(rs, (lane + EVAL_BLOCK * r) * 16, tile[row * TS + col], tile[row * TS + col + 1]);
        }
      }
    } else {
      const int tot = nrow * N;
      const int q64 = EVAL_BLOCK / N, r64 = EVAL_BLOCK % N;
      int row = lane / N, col = lane % N;
      for (int e = lane; e < tot; e += EVAL_BLOCK) {
        st_wt8(wo + e, tile[row * TS + col]);
        row += q64;
        col += r64;
        if (col >= N) {
          col -= N;
          row += 1;
        }
      }
    }
  }
  if (active) {
    if (a.cost) st_wt8(a.cost + i, tile[lane * TS + N]);
    if (a.w0) st_wt8(a.w0 + i, tile[lane * TS + 0]);
    if (a.status)
      a.status[i] = !valid ? LOMPC_QP_INVALID : (ok ? ((INPLACE && rep) ? LOMPC_QP_REPAIRED : LOMPC_QP_OK) : LOMPC_QP_FAILED);
  }
  // per-workgroup partials: column sums over the certified rows (max for the error);
  // lanes l and l+32 each sum half of the rows of column l, then combine
  double* part = a.partial + (size_t)b * (N + NPX);
  const int half = lane >> 5;
  for (int c0 = 0; c0 < TS; c0 += 32) {
    const int c = c0 + (lane & 31);
    const bool is_max = (c == N + PX_MAX_ERR);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < TS) {
#pragma unroll
      for (int rr = 0; rr < EVAL_BLOCK / 2; ++rr) {
        const int r = half * (EVAL_BLOCK / 2) + rr;
        const double v = ((okm >> r) & 1ull) ? tile[r * TS + c] : 0.0;
        acc[rr & 3] = is_max ? fmax(acc[rr & 3], v) : acc[rr & 3] + v;
      }
    }
    double v = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const double o2 = __shfl_xor(v, 32, 64);
    v = is_max ? fmax(v, o2) : v + o2;
    if (half == 0 && c < TS) part[c] = v;
  }
  if (lane == 0) {
    part[N + PX_N_OK] = (double)__popcll(INPLACE ? (okm & ~fm) : okm);
    part[N + PX_N_REPAIRED] = (double)__popcll(rm);
    part[N + PX_N_FAILED] = (double)__popcll(fm);  // !INPLACE: pending, re-solved in k_finalize
    part[N + PX_N_INVALID] = (double)__popcll(im);
  }
}

// ------------------------------------------------------------------- K1
#ifdef LOMPC_K1_STATS
__device__ long long g_k1_stats[8192 * 4];  // per cell: PDAS iterations, pieces, cycles solve, cycles tracking
#endif

// A cell's count is tagged with the parameter epoch (set_params call) that wrote it:
// tab.cnt[cell] = epoch << 4 | pieces.  K2 treats a cell of another epoch as unsolved.
__device__ __forceinline__ void publish_cell(int* cnt, int epoch, int npc) {
  if (threadIdx.x == 0) *cnt = (epoch << 4) | npc;
}
__device__ __forceinline__ int cell_epoch(int v) { return v >> 4; }
__device__ __forceinline__ int cell_pieces(int v) { return v & 15; }

struct PathArgs {
  int S, mode, epoch, pad;
  const double* lmbd;
  const double* lmbd_r;
  const double* w_ref;
  const double* gamma_ref;
  const double* window;  // [S][2] gamma window of the path, or null = [0, y_max]
  double* setdata;
  uint8_t* central;
  int* errflag;
};

__device__ __forceinline__ void path_cell(const QPConst& q, const PathArgs& pa, const PathTable& tab, int blk) {
  const double* __restrict__ lmbd = pa.lmbd;
  const double* __restrict__ lmbd_r = pa.lmbd_r;
  const double* __restrict__ w_ref = pa.w_ref;
  const double* __restrict__ gamma_ref = pa.gamma_ref;
  double* __restrict__ setdata = pa.setdata;
  uint8_t* __restrict__ central = pa.central;
  int* __restrict__ errflag = pa.errflag;
  const int mode = pa.mode;
  const int lane = threadIdx.x;
  const int N = q.N;
  const bool path = mode != LOMPC_MODE_DIRECT;
  const int s = path ? blk / LQ_G : blk;
  const int cell = path ? blk % LQ_G : 0;
  const double* L = lmbd + (size_t)s * 3 * N;
  const double lr = lmbd_r[s];
  const double tt = q.theta * q.theta;
  // per-stage data, natural (stage = lane) and reversed (stage = N-1-lane) layouts
  lqw::WaveSet ws;
  ws.N = N;
  ws.lane = lane;
  ws.rsrc = lane < N ? N - 1 - lane : lane;
  double l2 = 0.0;
  if (lane < N) {
    const double l1 = L[lane], l3 = L[2 * N + lane];
    l2 = L[N + lane];
    if (!(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0)) atomicOr(errflag, 1);
    ws.d_nat = 2.0 * lr * tt + 2.0 * q.q_scale * l3 + q.dsmall;
    ws.e_nat = q.theta * (l1 - l2);
    const int tr = ws.rsrc;
    ws.d_rev = 2.0 * lr * tt + 2.0 * q.q_scale * L[2 * N + tr] + q.dsmall;
    ws.e_rev = q.theta * (L[tr] - L[N + tr]);
  } else {
    ws.d_nat = ws.e_nat = ws.d_rev = ws.e_rev = 0.0;
  }
  const double wr_nat = (w_ref && lane < N) ? w_ref[(size_t)s * N + lane] : 0.0;
  const double c0 = q.theta * q.w_max * lqw::wave_sum(l2, N);  // lompc.py:128
  const double kappa = lr / q.delta;                    // price_solver.py:191
  const double ee = ws.e_nat;
  double Ywr;  // prefix sums of w_ref
  {
    lqw::Sums<1> y;
    y.v[0] = wr_nat;
    Ywr = lqw::wave_scan(y, N).v[0];
  }
  // gamma window of this set's path (lompc_set_gamma_window), widened by a margin
  double wlo = 0.0, whi = q.y_max;
  if (pa.window) {
    const double mg = 1e-7 * q.y_max;
    wlo = fmin(fmax(pa.window[2 * s] - mg, 0.0), q.y_max);
    whi = fmin(fmax(pa.window[2 * s + 1] + mg, wlo + mg), q.y_max);
    if (!(whi > wlo)) {  // window at y_max (or NaN input): full range
      wlo = 0.0;
      whi = q.y_max;
    }
  }
  if (cell == 0) {  // one block per set writes the derived set record
    const int SD = lq_sd(N);
    double* out = setdata + (size_t)s * SD;
    if (lane < N) {
      out[lane] = ws.d_nat;
      out[N + lane] = ws.e_nat;
      out[2 * N + lane] = wr_nat;
    }
    const double s2 = c0 / (q.theta * q.w_max);
    if (lane == 0) {
      if (!(lr >= 0.0)) atomicOr(errflag, 1);
      out[3 * N + 0] = q.theta * q.w_max * s2;  // c0, lompc.py:128
      out[3 * N + 1] = L[0];
      out[3 * N + 2] = L[N];
      out[3 * N + 3] = L[2 * N];
      out[3 * N + 4] = lr;
      out[3 * N + 5] = lr / q.delta;  // kappa, price_solver.py:191
      out[3 * N + 6] = gamma_ref ? gamma_ref[s] : 0.5 * q.y_max;
      out[3 * N + 7] = w_ref ? 1.0 : 0.0;
      out[3 * N + 8] = wlo;                         // path window start
      out[3 * N + 9] = (double)LQ_G / (whi - wlo);  // cells per unit gamma
    }
  }
  if (mode == LOMPC_MODE_PATH_REPAIR) {  // diagnostics: no table, every EV re-solved
    publish_cell(tab.cnt + (size_t)s * LQ_G + cell, pa.epoch, 0);
    return;
  }
  if (!path) {
    const double g = gamma_ref ? gamma_ref[s] : 0.5 * q.y_max;
    int sl = lane < N ? 1 : 0;
    double w = 0.0, r = 0.0;
    if (!lqw::wave_solve(q, ws, g, sl, w, r)) sl = lane < N ? 1 : 0;
    central[(size_t)s * LQ_STB + lane] = (uint8_t)(lane < N ? sl : 0);
    return;
  }
  const double h = (whi - wlo) / (double)LQ_G;
  const double glo = cell == 0 ? wlo : fma((double)cell, h, wlo);
  const double ghi = (cell == LQ_G - 1) ? whi : fma((double)(cell + 1), h, wlo);
  const size_t cb = (size_t)s * LQ_G + cell;
  int sl = lane < N ? 1 : 0;
  double w = 0.0, r = 0.0;
#ifdef LOMPC_K1_STATS
  const long long t0 = clock64();
  int nit = 0;
  const bool solved = lqw::wave_solve(q, ws, glo, sl, w, r, &nit);
  const long long t1 = clock64();
#else
  const bool solved = lqw::wave_solve(q, ws, glo, sl, w, r);
#endif
  if (!solved) {
    publish_cell(tab.cnt + cb, pa.epoch, 0);  // EVs of this cell are re-solved by wave_solve
    return;
  }
  // parametric active-set tracking of w*(gamma) on [glo, ghi]
  double gcur = glo;
  int last = -1, npc = 0;
  const int max_iter = 4 * LQ_PPL + 16;
  for (int it = 0; it < max_iter && npc < LQ_PPL; ++it) {
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
    const bool final_piece = (bj < 0) || (npc == LQ_PPL - 1);
    if (best > gcur || final_piece) {
      // KKT certificate at the piece's end.  Its start is certified too: the first
      // piece starts at the wave_solve point; a later one at the previous piece's
      // certified end with the same w and r, where only the switched coordinate's
      // box changed and it contains that coordinate's value.  The residual is
      // convex in gamma along an affine piece => the whole piece is certified.
      const Box bx = lq_box(lane < N ? sl : 0);
      const double wz = fmin(fmax(fma(bv, best, av), bx.lo), bx.hi);
      const double res = lqw::wave_kkt_point(q, ws, best, sl, wz);
      if (!(res <= q.tol_cert)) break;  // coverage of the cell ends at gcur
      // cost and err^2 are quadratics in gamma on the piece (w = a + b gamma):
      // per-lane terms, two prefix sums (Ya, Yb) and six wave totals
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
      t[1] = fma(cc, fma(Ya, Yb, -Ya), fma(bv, fma(dd, av, ee + sg), 0.0));
      t[2] = fma(0.5 * cc, Yb * Yb, fma(-cc, Yb, 0.5 * dd * bv * bv));
      t[3] = fma(Ea, Ea, kappa * da * da);
      t[4] = 2.0 * fma(Ea, Yb, kappa * da * bv);
      t[5] = fma(Yb, Yb, kappa * bv * bv);
#pragma unroll
      for (int k = 0; k < 6; ++k) t[k] = act ? t[k] : 0.0;
      lqw::wave_totals(t, N);
      const size_t pidx = cb * LQ_PPL + npc;
      if (lane < N) {
        reinterpret_cast<double2*>(tab.ab + pidx * (size_t)N * 2)[lane] = make_double2(av, bv);
        tab.st[pidx * LQ_STB + lane] = (uint8_t)sl;
      }
      if (lane < 6) {  // row: K0, K1, K2 (cost), F0, F1, F2 (err^2), -, -
        double v = t[0];
#pragma unroll
        for (int k = 1; k < 6; ++k) v = lane == k ? t[k] : v;
        tab.coef[pidx * 8 + lane] = lane == 0 ? v + c0 : v;
      }
      if (lane == 0) tab.gend[pidx] = best;
      ++npc;
    }
    if (bj < 0) break;
    const int bns = __shfl(ns, bj, 64);
    if (lane == bj) sl = bns;
    gcur = best;
    last = bj;
  }
  publish_cell(tab.cnt + cb, pa.epoch, npc);
#ifdef LOMPC_K1_STATS
  const long long t2 = clock64();
  if (lane == 0 && cb < 8192) {
    g_k1_stats[cb * 4 + 0] = nit;
    g_k1_stats[cb * 4 + 1] = npc;
    g_k1_stats[cb * 4 + 2] = t1 - t0;
    g_k1_stats[cb * 4 + 3] = t2 - t1;
  }
#endif
}

__global__ __launch_bounds__(64) void k_path(QPConst q, PathArgs pa, PathTable tab) {
  lq_tab_init(q);
  path_cell(q, pa, tab, (int)blockIdx.x);
}

// ------------------------------------------------------------------- K2
template <int NMAX, int NT>
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval(QPConst q, KArgs a, int epoch) {
  const int b = (int)blockIdx.x;
  int s;
  int64_t start, end;
  block_set(a, b, s, start, end);
  const int N = NT ? NT : q.N;
  const int lane = threadIdx.x;
  const int64_t i = start + lane;
  const bool active = i < end;
  const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
  const double g = active ? a.gamma[i] : 0.0;
  const bool valid = active && (g >= 0.0) && (g <= q.y_max);
  const double wlo = sd[3 * N + 8], invh = sd[3 * N + 9];  // path window (uniform loads)
  const bool inwin = g >= wlo;                             // below the window: re-solved
  const int cell = valid ? max(0, min(LQ_G - 1, (int)((g - wlo) * invh))) : 0;
  const size_t cb = (size_t)s * LQ_G + cell;
  // the cell count and the piece ends are loaded together (cb is always a valid cell: one
  // dependent memory round less than loading the ends behind the count test)
  const int raw = a.tab.cnt[cb];
  double ge[LQ_PPL];
  {
    const double2* g2 = reinterpret_cast<const double2*>(a.tab.gend + cb * LQ_PPL);
#pragma unroll
    for (int pp = 0; pp < LQ_PPL / 2; ++pp) {
      const double2 v = g2[pp];
      ge[2 * pp] = v.x;
      ge[2 * pp + 1] = v.y;
    }
  }
  const bool ready = cell_epoch(raw) == epoch;  // written by this parameter epoch
  const int cnt = (valid && ready && inwin) ? cell_pieces(raw) : 0;
  double w[NMAX];
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  bool ok = false;
  EVOut o{0.0, 0.0, 0.0};
  if (cnt > 0) {
    int p = cnt - 1;
    double glast = -1.0;
#pragma unroll
    for (int pp = LQ_PPL - 1; pp >= 0; --pp) {
      if (pp < cnt && g <= ge[pp]) p = pp;
      if (pp == cnt - 1) glast = ge[pp];
    }
    ok = g <= glast;  // inside a certified piece
    if (ok) {
      const size_t pidx = cb * LQ_PPL + p;
      const double2* row = reinterpret_cast<const double2*>(a.tab.ab + pidx * (size_t)N * 2);
      const double4 cf0 = *reinterpret_cast<const double4*>(a.tab.coef + pidx * 8);
      const double2 cf1 = *reinterpret_cast<const double2*>(a.tab.coef + pidx * 8 + 4);
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) {
          const double2 ab = row[t];
          w[t] = fmin(fmax(fma(ab.y, g, ab.x), 0.0), q.w_max);
        }
      o.cost = fma(fma(cf0.z, g, cf0.y), g, cf0.x);
      o.err = a.want_err ? sqrt(fmax(fma(fma(cf1.y, g, cf1.x), g, cf0.w), 0.0)) : 0.0;
      o.price0 = lq_price0(q, sd, w[0]);
    }
  }
  // ---- in-place repair: EVs no certified piece covers are solved by the whole wave
  bool rep = false;
  unsigned long long need = __ballot(valid && !ok);
  if (need) {  // wave-uniform (one wave per workgroup)
    lq_tab_init(q);
    __shared__ double stage[64];
    lqw::WaveSet ws;
    ws.load(sd, N);
    while (need) {
      const int l = (int)__builtin_ctzll(need);
      need &= need - 1ull;
      const double gl = lqw::readlane_d(g, l);
      const int rawl = __builtin_amdgcn_readlane(raw, l);
      const int celll = __builtin_amdgcn_readlane(cell, l);
      int sl = 1;
      if (cell_epoch(rawl) == epoch && cell_pieces(rawl) > 0)
        sl = a.tab.st[((size_t)s * LQ_G + celll) * LQ_PPL * LQ_STB + lane];
      if (lane >= N) sl = 0;
      double wl = 0.0, rl = 0.0;
      const bool okk = lqw::wave_solve(q, ws, gl, sl, wl, rl);
      const EVOut ol = wave_outputs(q, sd, gl, lane, wl, a.want_err != 0);
      stage[lane] = wl;
      __syncthreads();
      if (lane == l) {
#pragma unroll
        for (int t = 0; t < NMAX; ++t)
          if (t < N) w[t] = stage[t];
        o = ol;
        ok = okk;
        rep = true;
      }
      __syncthreads();
    }
  }
  ev_epilogue<NMAX, true>(q, N, a, b, start, end, valid, ok, w, o, rep);
}

// ------------------------------------------------------------------- K2d
template <int NMAX, int NT>
__global__ __launch_bounds__(EVAL_BLOCK) void k_direct(QPConst q, KArgs a) {
  lq_tab_init(q);
  const int b = blockIdx.x;
  int s;
  int64_t start, end;
  block_set(a, b, s, start, end);
  const int N = NT ? NT : q.N;
  const int lane = threadIdx.x;
  const int64_t i = start + lane;
  const bool active = i < end;
  const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
  const double g = active ? a.gamma[i] : 0.0;
  const bool valid = active && (g >= 0.0) && (g <= q.y_max);
  double w[NMAX];
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  bool ok = false;
  const uint8_t* cst = a.central + (size_t)s * LQ_STB;
  if (valid) {
    States<NMAX> st;
    st.load_bytes(cst);
    ok = lq_pdas<NMAX>(q, N, sd, sd + N, g, st, w, 4 * N + 8);
    if (ok) {
      lq_snap<NMAX>(N, st, w);
      ok = lq_kkt<NMAX>(q, N, sd, sd + N, g, st, w) <= q.tol_cert;
    }
  }
  EVOut o{0.0, 0.0, 0.0};
  if (ok) o = lq_outputs<NMAX>(q, N, sd, g, w, a.want_err != 0);
  ev_epilogue<NMAX>(q, N, a, b, start, end, valid, ok, w, o);
}

// ------------------------------------------------------------------- K3
// One workgroup of 1024 threads (16 waves) per set.
// (1) repair: wave wv re-solves the listed EVs of workgroups b0+wv, b0+wv+16, ...
//     (wave_solve: PDAS from the cell's / central working set, primal active set
//     if needed, KKT-certified) and writes their outputs;
// (2) reduction: wave wv sums partial rows wv, wv+16, ... (lane = column), the 16
//     waves and the repair accumulators combine in LDS in a fixed order.
__global__ __launch_bounds__(1024) void k_finalize(QPConst q, KArgs a, int mode, double* __restrict__ set_sum_w,
                                                   double* __restrict__ set_stats, double* __restrict__ stats_int) {
  __shared__ double red[16][LOMPC_MAX_N + NPX + 1];
  __shared__ double rep[16][LOMPC_MAX_N + NPX + 1];
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int N = q.N;
  const int W = N + NPX;
  const int b0 = a.blk_prefix[s], b1 = a.blk_prefix[s + 1];
  // ---- (1) reduction of the workgroup partials (their N_FAILED column = pending repairs)
  for (int c = lane; c < W; c += 64) {
    const bool is_max = (c == N + PX_MAX_ERR);
    // 16 independent (predicated) loads per round: one memory round trip per 256 partial
    // rows of the set instead of one per row of the tail
    constexpr int U = 16;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = b0 + wv; b < b1; b += 16 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int bb = b + 16 * u;
        v[u] = bb < b1 ? a.partial[(size_t)bb * W + c] : 0.0;  // 0: neutral for sums and for max of errors >= 0
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u & 3] = is_max ? fmax(acc[u & 3], v[u]) : acc[u & 3] + v[u];
    }
    red[wv][c] = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  if (tid < W) {
    const int c = tid;
    const bool is_max = (c == N + PX_MAX_ERR);
    double acc = red[0][c];
    for (int k = 1; k < 16; ++k) acc = is_max ? fmax(acc, red[k][c]) : acc + red[k][c];
    red[0][c] = acc;
  }
  __syncthreads();
  // DIRECT mode: N_FAILED counts EVs listed for repair; PATH partials hold final counts
  // (k_eval repairs in place)
  const bool pending = mode == LOMPC_MODE_DIRECT && red[0][N + PX_N_FAILED] > 0.0;  // block-uniform
  // ---- (2) repair: wave wv re-solves the listed EVs of workgroups b0+wv, b0+wv+16, ...
  if (pending) {
    lq_tab_init(q);
    double acc_w = 0.0, acc_cost = 0.0, acc_p0 = 0.0, acc_err = 0.0;
    int nrep = 0, nfail = 0;
    const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
    lqw::WaveSet ws;
    ws.load(sd, N);
    for (int b = b0 + wv; b < b1; b += 16) {
      const int nf = a.fail_cnt[b];
      for (int k = 0; k < nf; ++k) {
        const int l = a.fail_lane[(size_t)b * EVAL_BLOCK + k];
        const int64_t i = a.set_off[s] + (int64_t)(b - b0) * EVAL_BLOCK + l;
        const double g = a.gamma[i];
        int sl = a.central[(size_t)s * LQ_STB + lane];  // DIRECT mode only
        if (lane >= N) sl = 0;
        double wl = 0.0, rl = 0.0;
        const bool okk = lqw::wave_solve(q, ws, g, sl, wl, rl);
        const EVOut o = wave_outputs(q, sd, g, lane, wl, a.want_err != 0);
        if (a.w && lane < N) a.w[(size_t)i * N + lane] = wl;
        if (lane == 0) {
          if (a.cost) a.cost[i] = o.cost;
          if (a.w0) a.w0[i] = wl;
          if (a.status) a.status[i] = okk ? LOMPC_QP_REPAIRED : LOMPC_QP_FAILED;
        }
        acc_w += lane < N ? wl : 0.0;
        acc_cost += o.cost;
        acc_p0 += o.price0;
        acc_err = fmax(acc_err, o.err);
        nrep += okk ? 1 : 0;
        nfail += okk ? 0 : 1;
      }
    }
    if (lane < N) rep[wv][lane] = acc_w;
    if (lane == 0) {
      rep[wv][N + PX_COST] = acc_cost;
      rep[wv][N + PX_PRICE0] = acc_p0;
      rep[wv][N + PX_MAX_ERR] = acc_err;
      rep[wv][N + PX_N_OK] = (double)nrep;
      rep[wv][N + PX_N_REPAIRED] = (double)nrep;
      rep[wv][N + PX_N_FAILED] = (double)nfail;
      rep[wv][N + PX_N_INVALID] = 0.0;
    }
    __syncthreads();
    if (tid < W) {
      const int c = tid;
      const bool is_max = (c == N + PX_MAX_ERR);
      double acc = (c == N + PX_N_FAILED) ? 0.0 : red[0][c];  // pending -> replaced by real failures
      for (int k = 0; k < 16; ++k) acc = is_max ? fmax(acc, rep[k][c]) : acc + rep[k][c];
      red[0][c] = acc;
    }
    __syncthreads();
  }
  if (tid < N && set_sum_w) set_sum_w[(size_t)s * N + tid] = red[0][tid];
  if (tid == 0) {
    double row[LOMPC_SET_STATS];
    row[LOMPC_STAT_COUNT] = (double)(a.set_off[s + 1] - a.set_off[s]);
    row[LOMPC_STAT_SUM_W0] = red[0][0];
    row[LOMPC_STAT_SUM_PRICE0] = red[0][N + PX_PRICE0];
    row[LOMPC_STAT_MAX_ERR] = red[0][N + PX_MAX_ERR];
    row[LOMPC_STAT_SUM_COST] = red[0][N + PX_COST];
    row[LOMPC_STAT_N_REPAIRED] = red[0][N + PX_N_REPAIRED];
    row[LOMPC_STAT_N_FAILED] = red[0][N + PX_N_FAILED];
    row[LOMPC_STAT_N_INVALID] = red[0][N + PX_N_INVALID];
    for (int k = 0; k < LOMPC_SET_STATS; ++k) {
      if (set_stats) set_stats[(size_t)s * LOMPC_SET_STATS + k] = row[k];
      stats_int[(size_t)s * LOMPC_SET_STATS + k] = row[k];
    }
  }
}

// ===================================================================== host
struct lompc_ctx {
  int device = 0;
  int N = 0;
  int ev_type = 0;
  int mode = LOMPC_MODE_PATH;
  int nmax = 0;
  QPConst q{};
  // parameter sets
  int64_t S = 0, S_cap = 0;
  double* d_setdata = nullptr;
  PathTable tab{nullptr, nullptr, nullptr, nullptr, nullptr};
  uint8_t* d_central = nullptr;
  int* d_errflag = nullptr;
  const double* d_window = nullptr;  // lompc_set_gamma_window (caller-owned, sticky)
  int params_mode = -1;
  // batch workspaces
  int64_t nblk_cap = 0, soff_cap = 0, stats_cap = 0;
  double* d_partial = nullptr;
  int* d_fail_cnt = nullptr;
  uint8_t* d_fail_lane = nullptr;
  int* d_blk_prefix = nullptr;
  int64_t* d_set_off = nullptr;
  longlong4* d_blk_info = nullptr;
  longlong4* h_pin_info = nullptr;
  int64_t info_cap = 0;
  double* d_stats = nullptr;  // [S][LOMPC_SET_STATS], always written by the set reduction
  int epoch = 0;  // parameter epoch of the path table (tags tab.cnt)
  int64_t stats_S = 0;
  int* h_pin_prefix = nullptr;
  int64_t* h_pin_off = nullptr;
  hipEvent_t ev_map = nullptr;
  std::vector<int64_t> last_off;
  void* last_off_stream = nullptr;
  // single-solve scratch (3N + N + 8 doubles)
  double* d_single = nullptr;
  int8_t* d_single_status = nullptr;
  // profiling
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;    // pairs recorded since the last read
  std::vector<hipEvent_t> prof_pool;  // recycled events (no creation inside timed loops)
  double prof_ms = 0.0;
  int64_t prof_n = 0;
  std::string err;
};

#define HIPCHK(ctx, call)                                                        \
  do {                                                                           \
    hipError_t e__ = (call);                                                     \
    if (e__ != hipSuccess) {                                                     \
      if (ctx) (ctx)->err = std::string(#call) + ": " + hipGetErrorString(e__); \
      return LOMPC_ERR_HIP;                                                      \
    }                                                                            \
  } while (0)

static int fail_arg(lompc_ctx* ctx, const char* msg) {
  if (ctx) ctx->err = msg;
  return LOMPC_ERR_INVALID_ARG;
}

template <typename T>
static int grow(lompc_ctx* ctx, T** p, size_t n_elems) {
  if (*p) {
    hipError_t e = hipFree(*p);
    if (e != hipSuccess) {
      ctx->err = std::string("hipFree: ") + hipGetErrorString(e);
      return LOMPC_ERR_HIP;
    }
  }
  *p = nullptr;
  hipError_t e = hipMalloc((void**)p, std::max<size_t>(n_elems, 1) * sizeof(T));
  if (e != hipSuccess) {
    ctx->err = std::string("hipMalloc: ") + hipGetErrorString(e);
    return LOMPC_ERR_HIP;
  }
  return LOMPC_OK;
}

static int pick_nmax(int N) {
  if (N <= 16) return 16;
  if (N <= 24) return 24;
  if (N <= 32) return 32;
  if (N <= 48) return 48;
  if (N <= 64) return 64;
  return 0;
}

// (NM, NT): exact-horizon kernels for the common N, NMAX buckets with runtime N otherwise
#define DISPATCH_N(N, nmax, ...)                                                    \
  switch (N) {                                                                      \
    case 12: { constexpr int NM = 12, NT = 12; __VA_ARGS__; } break;                \
    case 16: { constexpr int NM = 16, NT = 16; __VA_ARGS__; } break;                \
    case 24: { constexpr int NM = 24, NT = 24; __VA_ARGS__; } break;                \
    case 32: { constexpr int NM = 32, NT = 32; __VA_ARGS__; } break;                \
    case 48: { constexpr int NM = 48, NT = 48; __VA_ARGS__; } break;                \
    case 64: { constexpr int NM = 64, NT = 64; __VA_ARGS__; } break;                \
    default:                                                                        \
      switch (nmax) {                                                               \
        case 16: { constexpr int NM = 16, NT = 0; __VA_ARGS__; } break;             \
        case 24: { constexpr int NM = 24, NT = 0; __VA_ARGS__; } break;             \
        case 32: { constexpr int NM = 32, NT = 0; __VA_ARGS__; } break;             \
        case 48: { constexpr int NM = 48, NT = 0; __VA_ARGS__; } break;             \
        case 64: { constexpr int NM = 64, NT = 0; __VA_ARGS__; } break;             \
        default: break;                                                             \
      }                                                                             \
  }

extern "C" {

int lompc_abi_version(void) { return 1; }

#ifdef LOMPC_K1_STATS
// diagnostic build only (scripts/k1_stats.py): per-cell K1 counters of the last launch
int lompc_debug_k1_stats(long long* host, int n) {
  if (n > 8192 * 4) n = 8192 * 4;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_k1_stats), sizeof(long long) * n, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? LOMPC_OK
             : LOMPC_ERR_HIP;
}
#endif

const char* lompc_status_string(int status) {
  switch (status) {
    case LOMPC_OK: return "ok";
    case LOMPC_ERR_INVALID_ARG: return "invalid argument";
    case LOMPC_ERR_NOT_CONVERGED: return "solver did not produce a certified optimum";
    case LOMPC_ERR_HIP: return "HIP runtime error";
    case LOMPC_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return "unknown status";
  }
}

const char* lompc_last_error(const lompc_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

int lompc_create(int N, double delta, double theta, double y_max, double w_max, int ev_type, int device,
                 lompc_ctx** out) {
  if (!out) return LOMPC_ERR_INVALID_ARG;
  *out = nullptr;
  // lompc.py:36-38 (settings.py:7-9); delta > 0 keeps the QP strictly convex
  if (!(y_max >= 0.75 && y_max <= 0.9)) return LOMPC_ERR_INVALID_ARG;
  if (!(w_max > 0.0 && w_max <= 0.25)) return LOMPC_ERR_INVALID_ARG;
  if (ev_type != LOMPC_EV_SMALL && ev_type != LOMPC_EV_LARGE) return LOMPC_ERR_INVALID_ARG;
  if (!(delta > 0.0) || !(theta > 0.0) || N < 1) return LOMPC_ERR_INVALID_ARG;
  const int nmax = pick_nmax(N);
  if (!nmax) return LOMPC_ERR_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LOMPC_ERR_HIP;
  if (hipSetDevice(device) != hipSuccess) return LOMPC_ERR_HIP;
  lompc_ctx* c = new lompc_ctx();
  c->device = device;
  c->N = N;
  c->ev_type = ev_type;
  c->nmax = nmax;
  QPConst& q = c->q;
  q.N = N;
  q.ev_small = ev_type == LOMPC_EV_SMALL;
  q.delta = delta;
  q.theta = theta;
  q.y_max = y_max;
  q.w_max = w_max;
  q.inv_wmax = 1.0 / w_max;
  q.c = 2.0 * delta * theta * theta;        // lompc.py:71
  q.q_scale = 3.0 * theta / (4.0 * w_max);  // lompc.py:67
  q.dsmall = q.ev_small ? 2.0 * theta * theta / (0.9 * 0.9) : 0.0;  // lompc.py:105
  if (q.ev_small) {
    q.m = 1;
    q.knots[0] = 0.0;
    for (int k = 1; k <= LQ_MAXSEG; ++k) q.knots[k] = w_max;
    for (int k = 0; k < LQ_MAXSEG; ++k) q.slopes[k] = 0.0;
  } else {  // lompc.py:108-114
    q.m = 4;
    const double kr[5] = {0.0, 0.125, 0.5, 0.75, 1.0};
    const double sr[4] = {0.0, 1.0, 1.5, 2.0};
    const double sc = (theta * w_max) * (theta * w_max) / w_max;
    for (int k = 0; k < 5; ++k) q.knots[k] = w_max * kr[k];
    q.knots[4] = w_max;
    for (int k = 0; k < 4; ++k) q.slopes[k] = sc * sr[k];
  }
  // gradient magnitude: charging term c N^2 w_max, PWL slopes, prices ~ theta * lambda ~ theta^2
  q.scale = 1.0 + q.c * (double)N * (double)N * w_max + q.slopes[q.m - 1] + theta * theta;
  q.tol_switch = 1e-13 * q.scale;
  q.tol_cert = 1e-11 * q.scale;
  q.ktol = 1e-13 * w_max;
  hipError_t e;
  if ((e = hipMalloc((void**)&c->d_errflag, sizeof(int))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single, (4 * N + 8) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single_status, 8)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev_map, hipEventDisableTiming)) != hipSuccess) {
    delete c;
    return LOMPC_ERR_HIP;
  }
  (void)hipMemset(c->d_errflag, 0, sizeof(int));
  *out = c;
  return LOMPC_OK;
}

int lompc_destroy(lompc_ctx* c) {
  if (!c) return LOMPC_OK;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  void* ptrs[] = {c->d_setdata, c->tab.cnt, c->tab.gend, c->tab.ab, c->tab.coef, c->tab.st, c->d_central, c->d_errflag,
                  c->d_partial, c->d_fail_cnt, c->d_fail_lane, c->d_blk_prefix, c->d_set_off, c->d_blk_info, c->d_stats,
                  c->d_single, c->d_single_status};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_pin_prefix) (void)hipHostFree(c->h_pin_prefix);
  if (c->h_pin_off) (void)hipHostFree(c->h_pin_off);
  if (c->h_pin_info) (void)hipHostFree(c->h_pin_info);
  if (c->ev_map) (void)hipEventDestroy(c->ev_map);
  for (hipEvent_t ev : c->prof_ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->prof_pool) (void)hipEventDestroy(ev);
  delete c;
  return LOMPC_OK;
}

int lompc_set_mode(lompc_ctx* c, int mode) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (mode != LOMPC_MODE_PATH && mode != LOMPC_MODE_DIRECT && mode != LOMPC_MODE_PATH_REPAIR)
    return fail_arg(c, "mode must be PATH, DIRECT or PATH_REPAIR");
  c->mode = mode;
  return LOMPC_OK;
}

int lompc_get_info(const lompc_ctx* c, int* N, int* ev_type) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (N) *N = c->N;
  if (ev_type) *ev_type = c->ev_type;
  return LOMPC_OK;
}

// Validate / size the parameter-set buffers and open a new cell epoch.
static int prepare_params(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, PathArgs* pa,
                          const double* w_ref, const double* gamma_ref) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (S < 1 || !lmbd || !lmbd_r) return fail_arg(c, "set_params: S >= 1 and lmbd, lmbd_r required");
  if (S > (1 << 20)) return fail_arg(c, "set_params: too many parameter sets");
  HIPCHK(c, hipSetDevice(c->device));
  const int N = c->N;
  if (S > c->S_cap) {
    int rc;
    const size_t cells = (size_t)S * LQ_G;
    if ((rc = grow(c, &c->d_setdata, (size_t)S * lq_sd(N))) || (rc = grow(c, &c->tab.cnt, cells)) ||
        (rc = grow(c, &c->tab.gend, cells * LQ_PPL)) || (rc = grow(c, &c->tab.ab, cells * LQ_PPL * (size_t)N * 2)) ||
        (rc = grow(c, &c->tab.coef, cells * LQ_PPL * 8)) ||
        (rc = grow(c, &c->tab.st, cells * LQ_PPL * LQ_STB)) || (rc = grow(c, &c->d_central, (size_t)S * LQ_STB)))
      return rc;
    HIPCHK(c, hipMemset(c->tab.cnt, 0, cells * sizeof(int)));  // epoch 0 = never published
    c->S_cap = S;
  }
  c->S = S;
  c->params_mode = c->mode;
  c->epoch = (c->epoch + 1) & 0x7ffffff;
  if (c->epoch == 0) c->epoch = 1;
  pa->S = (int)S;
  pa->mode = c->mode;
  pa->epoch = c->epoch;
  pa->pad = 0;
  pa->lmbd = lmbd;
  pa->lmbd_r = lmbd_r;
  pa->w_ref = w_ref;
  pa->gamma_ref = gamma_ref;
  pa->window = c->mode != LOMPC_MODE_DIRECT ? c->d_window : nullptr;
  pa->setdata = c->d_setdata;
  pa->central = c->d_central;
  pa->errflag = c->d_errflag;
  return LOMPC_OK;
}

int lompc_set_gamma_window(lompc_ctx* c, const double* window) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  c->d_window = window;
  return LOMPC_OK;
}

int lompc_set_params(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, const double* w_ref,
                     const double* gamma_ref, void* stream) {
  PathArgs pa{};
  const int rc = prepare_params(c, S, lmbd, lmbd_r, &pa, w_ref, gamma_ref);
  if (rc) return rc;
  const unsigned grid = (unsigned)(c->mode != LOMPC_MODE_DIRECT ? S * LQ_G : S);
  hipLaunchKernelGGL(k_path, dim3(grid), dim3(64), 0, (hipStream_t)stream, c->q, pa, c->tab);
  HIPCHK(c, hipGetLastError());
  return LOMPC_OK;
}

static int upload_block_map(lompc_ctx* c, const int64_t* set_off, int64_t S, int* nblk_out, hipStream_t st) {
  std::vector<int> pre(S + 1);
  int64_t nb = 0;
  pre[0] = 0;
  for (int64_t s = 0; s < S; ++s) {
    const int64_t m = set_off[s + 1] - set_off[s];
    if (m < 0) return fail_arg(c, "solve_batch: set_offsets must be non-decreasing");
    nb += (m + EVAL_BLOCK - 1) / EVAL_BLOCK;
    if (nb > (1ll << 30)) return fail_arg(c, "solve_batch: batch too large");
    pre[s + 1] = (int)nb;
  }
  *nblk_out = (int)nb;
  if (nb > c->nblk_cap) {
    int rc;
    if ((rc = grow(c, &c->d_partial, (size_t)nb * (c->N + NPX))) || (rc = grow(c, &c->d_fail_cnt, (size_t)nb)) ||
        (rc = grow(c, &c->d_fail_lane, (size_t)nb * EVAL_BLOCK)))
      return rc;
    c->nblk_cap = nb;
  }
  if (S > c->stats_cap) {
    int rc;
    if ((rc = grow(c, &c->d_stats, (size_t)S * LOMPC_SET_STATS))) return rc;
    c->stats_cap = S;
  }
  const bool same = (int64_t)c->last_off.size() == S + 1 && c->last_off_stream == (void*)st &&
                    memcmp(c->last_off.data(), set_off, (S + 1) * sizeof(int64_t)) == 0;
  if (same && c->d_blk_prefix) return LOMPC_OK;
  if (S + 1 > c->soff_cap) {
    int rc;
    if ((rc = grow(c, &c->d_blk_prefix, (size_t)(S + 1))) || (rc = grow(c, &c->d_set_off, (size_t)(S + 1))))
      return rc;
    if (c->h_pin_prefix) (void)hipHostFree(c->h_pin_prefix);
    if (c->h_pin_off) (void)hipHostFree(c->h_pin_off);
    c->h_pin_prefix = nullptr;
    c->h_pin_off = nullptr;
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_prefix, (S + 1) * sizeof(int), hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_off, (S + 1) * sizeof(int64_t), hipHostMallocDefault));
    c->soff_cap = S + 1;
  }
  if (nb > c->info_cap) {
    int rc;
    if ((rc = grow(c, &c->d_blk_info, (size_t)nb))) return rc;
    if (c->h_pin_info) (void)hipHostFree(c->h_pin_info);
    c->h_pin_info = nullptr;
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_info, nb * sizeof(longlong4), hipHostMallocDefault));
    c->info_cap = nb;
  }
  // the pinned staging buffers may still be read by the previous upload
  HIPCHK(c, hipEventSynchronize(c->ev_map));
  memcpy(c->h_pin_prefix, pre.data(), (S + 1) * sizeof(int));
  memcpy(c->h_pin_off, set_off, (S + 1) * sizeof(int64_t));
  for (int64_t s = 0; s < S; ++s)
    for (int b = pre[s]; b < pre[s + 1]; ++b)  // (set, first EV, end EV, -)
      c->h_pin_info[b] = make_longlong4(s, set_off[s] + (int64_t)(b - pre[s]) * EVAL_BLOCK, set_off[s + 1], 0);
  HIPCHK(c, hipMemcpyAsync(c->d_blk_prefix, c->h_pin_prefix, (S + 1) * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->d_set_off, c->h_pin_off, (S + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
  if (nb > 0)
    HIPCHK(c, hipMemcpyAsync(c->d_blk_info, c->h_pin_info, nb * sizeof(longlong4), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipEventRecord(c->ev_map, st));
  c->last_off.assign(set_off, set_off + S + 1);
  c->last_off_stream = (void*)st;
  return LOMPC_OK;
}

// Per-EV work of one batch: k_eval (PATH) or k_direct (DIRECT), then k_finalize.
static int launch_batch(lompc_ctx* c, int64_t B, const double* gamma,
                        const int64_t* set_offsets, double* w, double* cost, double* w0, int8_t* status,
                        double* set_sum_w, double* set_stats, hipStream_t st) {
  if (B < 0 || !set_offsets) return fail_arg(c, "solve_batch: invalid batch");
  if (set_offsets[0] != 0 || set_offsets[c->S] != B)
    return fail_arg(c, "solve_batch: set_offsets must start at 0 and end at B");
  if (B > 0 && !gamma) return fail_arg(c, "solve_batch: gamma required");
  int nblk = 0;
  int rc = upload_block_map(c, set_offsets, c->S, &nblk, st);
  if (rc) return rc;
  KArgs a{};
  a.B = B;
  a.S = (int)c->S;
  a.nblk = nblk;
  a.want_err = 1;
  a.gamma = gamma;
  a.blk_prefix = c->d_blk_prefix;
  a.set_off = c->d_set_off;
  a.blk_info = c->d_blk_info;
  a.setdata = c->d_setdata;
  a.tab = c->tab;
  a.central = c->d_central;
  a.w = w;
  a.cost = cost;
  a.w0 = w0;
  a.status = status;
  a.partial = c->d_partial;
  a.fail_cnt = c->d_fail_cnt;
  a.fail_lane = c->d_fail_lane;
  // profiling: start/stop timestamps ride on the per-EV kernel's own dispatch
  // (hipExtLaunchKernel), no marker packets between the kernels
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof && nblk > 0) {
    for (hipEvent_t* e : {&e0, &e1}) {
      if (!c->prof_pool.empty()) {
        *e = c->prof_pool.back();
        c->prof_pool.pop_back();
      } else {
        HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableSystemFence));
      }
    }
  }
  if (nblk > 0) {
    dim3 grid((unsigned)nblk), block(EVAL_BLOCK);
    if (c->params_mode != LOMPC_MODE_DIRECT) {
      const int ep = c->epoch;
      DISPATCH_N(c->N, c->nmax,
                 hipExtLaunchKernelGGL((k_eval<NM, NT>), grid, block, 0, st, e0, e1, 0, c->q, a, ep));
    } else {
      DISPATCH_N(c->N, c->nmax, hipExtLaunchKernelGGL((k_direct<NM, NT>), grid, block, 0, st, e0, e1, 0, c->q, a));
    }
    HIPCHK(c, hipGetLastError());
    if (e0) {
      c->prof_ev.push_back(e0);
      c->prof_ev.push_back(e1);
    }
  }
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)c->S), dim3(1024), 0, st, c->q, a, c->params_mode, set_sum_w,
                     set_stats, c->d_stats);
  HIPCHK(c, hipGetLastError());
  c->stats_S = c->S;
  return LOMPC_OK;
}

int lompc_solve_batch(lompc_ctx* c, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
                      double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats,
                      void* stream) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (c->S < 1) return fail_arg(c, "solve_batch: call lompc_set_params first");
  HIPCHK(c, hipSetDevice(c->device));
  return launch_batch(c, B, gamma, set_offsets, w, cost, w0, status, set_sum_w, set_stats, (hipStream_t)stream);
}

int lompc_run(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, const double* w_ref,
              const double* gamma_ref, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
              double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats, void* stream) {
  const int rc = lompc_set_params(c, S, lmbd, lmbd_r, w_ref, gamma_ref, stream);
  if (rc) return rc;
  return lompc_solve_batch(c, B, gamma, set_offsets, w, cost, w0, status, set_sum_w, set_stats, stream);
}

int lompc_last_status(lompc_ctx* c, void* stream, int64_t* n_repaired, int64_t* n_failed, int64_t* n_invalid) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<double> h((size_t)std::max<int64_t>(c->stats_S, 1) * LOMPC_SET_STATS, 0.0);
  int ef = 0;
  if (c->stats_S > 0)
    HIPCHK(c, hipMemcpyAsync(h.data(), c->d_stats, c->stats_S * LOMPC_SET_STATS * sizeof(double),
                             hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipMemcpyAsync(&ef, c->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  double rep = 0, fail = 0, inv = 0;
  for (int64_t s = 0; s < c->stats_S; ++s) {
    rep += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_REPAIRED];
    fail += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_FAILED];
    inv += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_INVALID];
  }
  if (n_repaired) *n_repaired = (int64_t)rep;
  if (n_failed) *n_failed = (int64_t)fail;
  if (n_invalid) *n_invalid = (int64_t)inv;
  if (ef) {
    HIPCHK(c, hipMemsetAsync(c->d_errflag, 0, sizeof(int), (hipStream_t)stream));
    return fail_arg(c, "negative or NaN price parameter (lmbd >= 0, lmbd_r >= 0 required)");
  }
  return LOMPC_OK;
}

int lompc_solve_host(lompc_ctx* c, const double* lmbd, double lmbd_r, double gamma, double* w, double* cost) {
  if (!c || !lmbd) return LOMPC_ERR_INVALID_ARG;
  const int N = c->N;
  if (!(gamma <= c->q.y_max)) return fail_arg(c, "gamma <= y_max required (lompc.py:87)");
  if (!(gamma >= 0.0) || !(lmbd_r >= 0.0)) return fail_arg(c, "Parameter value must be nonnegative.");
  for (int i = 0; i < 3 * N; ++i)
    if (!(lmbd[i] >= 0.0)) return fail_arg(c, "Parameter value must be nonnegative.");
  HIPCHK(c, hipSetDevice(c->device));
  // scratch layout: [0,3N) lmbd | 3N lmbd_r | 3N+1 gamma | [3N+2, 4N+2) w | 4N+2 cost
  std::vector<double> h(4 * N + 8, 0.0);
  memcpy(h.data(), lmbd, 3 * N * sizeof(double));
  h[3 * N] = lmbd_r;
  h[3 * N + 1] = gamma;
  double* d = c->d_single;
  HIPCHK(c, hipMemcpy(d, h.data(), (3 * N + 2) * sizeof(double), hipMemcpyHostToDevice));
  const int saved = c->mode;
  c->mode = LOMPC_MODE_DIRECT;
  int rc = lompc_set_params(c, 1, d, d + 3 * N, nullptr, d + 3 * N + 1, nullptr);
  c->mode = saved;
  if (rc) return rc;
  const int64_t off[2] = {0, 1};
  rc = lompc_solve_batch(c, 1, d + 3 * N + 1, off, d + 3 * N + 2, d + 4 * N + 2, nullptr, c->d_single_status,
                         nullptr, nullptr, nullptr);
  if (rc) return rc;
  int8_t stt = 0;
  HIPCHK(c, hipMemcpy(h.data() + 3 * N + 2, d + 3 * N + 2, (N + 1) * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&stt, c->d_single_status, 1, hipMemcpyDeviceToHost));
  if (w) memcpy(w, h.data() + 3 * N + 2, N * sizeof(double));
  if (cost) *cost = h[4 * N + 2];
  if (stt == LOMPC_QP_INVALID) return fail_arg(c, "invalid gamma");
  if (stt == LOMPC_QP_FAILED) {
    c->err = "no certified optimum";
    return LOMPC_ERR_NOT_CONVERGED;
  }
  return LOMPC_OK;
}

int lompc_profile_enable(lompc_ctx* c, int enable) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  c->prof = enable != 0;
  HIPCHK(c, hipSetDevice(c->device));
  while (c->prof && c->prof_pool.size() < 512) {  // recorded pairs are recycled by lompc_profile_read
    hipEvent_t e;  // timing only: no system-scope fence (an L2 writeback) per record
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    c->prof_pool.push_back(e);
  }
  return LOMPC_OK;
}

int lompc_profile_read(lompc_ctx* c, double* total_ms, int64_t* launches, int reset) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  for (size_t k = 0; k + 1 < c->prof_ev.size(); k += 2) {
    HIPCHK(c, hipEventSynchronize(c->prof_ev[k + 1]));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->prof_ev[k], c->prof_ev[k + 1]));
    c->prof_ms += ms;
    c->prof_n += 1;
  }
  c->prof_pool.insert(c->prof_pool.end(), c->prof_ev.begin(), c->prof_ev.end());
  c->prof_ev.clear();
  if (total_ms) *total_ms = c->prof_ms;
  if (launches) *launches = c->prof_n;
  if (reset) {
    c->prof_ms = 0.0;
    c->prof_n = 0;
  }
  return LOMPC_OK;
}

}  // extern "C"
