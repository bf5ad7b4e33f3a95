// lompc_kernels.hip — MI355X (gfx950) kernels and the C-ABI of include/lompc_amd.h.
//
// Hot path replaced: LoMPC.solve_lompc (chargingstation/lompc.py:137-156) called once
// per EV from PriceSolver._get_w_err (price_solver.py:203-209) and
// PriceSolver.get_w0_price0 (price_solver.py:280-283).
//
// Kernels (one batched call = K1 at set_params time, K2 -> K2b -> K3 per solve):
//   K1 k_prepare   one wave per parameter set. Derived data (d, e, c0, ...) and, in
//                  PATH mode, the exact piecewise-affine solution path w*(gamma) over
//                  [0, y_max]: lane l solves the QP at gamma_l = l*y_max/64 (PDAS with
//                  primal active-set fallback) and tracks the active-set changes up to
//                  gamma_{l+1} (parametric-QP homotopy). In DIRECT mode: the central
//                  solution's working set.
//   K2 k_eval      one EV per lane, 256 EVs of one set per workgroup. Looks up its
//                  piece, w = a + b*gamma, certifies it by the KKT residual, computes
//                  cost / w0 / price0 / A_bar error, writes outputs and per-workgroup
//                  partial reductions. Uncertified EVs go to a per-workgroup list.
//   K2b k_direct   per-EV active-set solve (PDAS from a warm start, primal active set
//                  as last resort), certified; repairs K2's list (PATH) or solves every
//                  EV (DIRECT).
//   K3 k_finalize  deterministic per-set reduction of the workgroup partials.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "lompc_qp.hpp"
#include "../../include/lompc_amd.h"

#define EVAL_BLOCK 256
#define NPART_EXTRA 8  // partial record: [0,N) sum_w, then 8 scalars

enum {
  PT_SUM_W0 = 0,
  PT_SUM_PRICE0 = 1,
  PT_MAX_ERR = 2,
  PT_SUM_COST = 3,
  PT_N_OK = 4,
  PT_N_REPAIRED = 5,
  PT_N_FAILED = 6,
  PT_N_INVALID = 7
};

struct KArgs {
  int64_t B;
  int S;
  int nblk;
  int want_err;
  int pad;
  const double* gamma;
  const int* blk_prefix;   // [S+1]
  const int64_t* set_off;  // [S+1]
  const double* setdata;   // [S][SD]
  PathTable tab;
  const uint32_t* central; // [S][LQ_NW_MAX]
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* partial;  // [nblk][N+8]
  int* fail_cnt;    // [nblk]
  int* fail_idx;    // [nblk][EVAL_BLOCK]
};

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off, 64));
  return v;
}

// block -> (set, first EV) for set-contiguous batches
__device__ __forceinline__ void block_set(const KArgs& a, int b, int& s, int64_t& start, int64_t& end) {
  int lo = 0, hi = a.S - 1;
  while (lo < hi) {  // largest s with blk_prefix[s] <= b
    const int mid = (lo + hi + 1) >> 1;
    if (a.blk_prefix[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  s = lo;
  start = a.set_off[s] + (int64_t)(b - a.blk_prefix[s]) * EVAL_BLOCK;
  end = a.set_off[s + 1];
}

// Block reduction of the per-EV contributions into partial[b] (deterministic).
// mode_add = 1: add into the existing record (repair pass).
template <int NMAX>
__device__ __forceinline__ void block_partials(const QPConst& q, const double (&w)[NMAX], bool ok, const EVOut& o,
                               int n_rep, int n_fail, int n_inv, double* __restrict__ part, bool mode_add) {
  __shared__ double red[EVAL_BLOCK / 64][NMAX + NPART_EXTRA];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = q.N;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      const double v = wave_sum(ok ? w[t] : 0.0);
      if (lane == 0) red[wv][t] = v;
    }
  }
  double s0 = wave_sum(ok ? w[0] : 0.0);
  double s1 = wave_sum(ok ? o.price0 : 0.0);
  double s2 = wave_max(ok ? o.err : 0.0);
  double s3 = wave_sum(ok ? o.cost : 0.0);
  double s4 = wave_sum(ok ? 1.0 : 0.0);
  double s5 = wave_sum((double)n_rep);
  double s6 = wave_sum((double)n_fail);
  double s7 = wave_sum((double)n_inv);
  if (lane == 0) {
    red[wv][NMAX + 0] = s0;
    red[wv][NMAX + 1] = s1;
    red[wv][NMAX + 2] = s2;
    red[wv][NMAX + 3] = s3;
    red[wv][NMAX + 4] = s4;
    red[wv][NMAX + 5] = s5;
    red[wv][NMAX + 6] = s6;
    red[wv][NMAX + 7] = s7;
  }
  __syncthreads();
  const int tid = threadIdx.x;
  if (tid < N + NPART_EXTRA) {
    const int src = tid < N ? tid : NMAX + (tid - N);
    const bool is_max = (tid == N + PT_MAX_ERR);
    double acc = red[0][src];
#pragma unroll
    for (int k = 1; k < EVAL_BLOCK / 64; ++k) acc = is_max ? fmax(acc, red[k][src]) : acc + red[k][src];
    if (mode_add) {
      const double old = part[tid];
      acc = is_max ? fmax(old, acc) : old + acc;
    }
    part[tid] = acc;
  }
}

template <int NMAX>
__device__ __forceinline__ void load_states(States<NMAX>& st, const uint32_t* __restrict__ src) {
#pragma unroll
  for (int i = 0; i < States<NMAX>::NW; ++i) st.w[i] = src[i];
}

// ------------------------------------------------------------------- K1
// Piecewise-affine tracking of w*(gamma) from (st optimal at g_lo) up to g_hi.
template <int NMAX>
__device__ __forceinline__ int lq_track(const QPConst& q, const double* __restrict__ d, const double* __restrict__ e,
                        States<NMAX>& st, double g_lo, double g_hi, const PathTable& tab, size_t cb) {
  const int N = q.N;
  double gcur = g_lo;
  int last = -1, npc = 0;
  const int max_iter = 4 * LQ_PPL + 16;
  for (int it = 0; it < max_iter && npc < LQ_PPL; ++it) {
    double K[NMAX], a[NMAX], b[NMAX];
    {
      double P = 0.0, p0 = 0.0, p1 = 0.0;
#pragma unroll
      for (int t = NMAX - 1; t >= 0; --t) {
        if (t < N) {
          const double Q = q.c + P;
          const double q0 = p0, q1 = p1 - q.c;
          const int s = st.get(t);
          const bool fr = (s & 1) != 0;
          const double dt = d[t];
          const double et = e[t] + lq_slope(q, (s - 1) >> 1);
          const double inv = 1.0 / (Q + dt);
          const double wb = lq_knot(q, s >> 1);
          K[t] = fr ? -Q * inv : 0.0;
          a[t] = fr ? -(q0 + et) * inv : wb;
          b[t] = fr ? -q1 * inv : 0.0;
          P = fr ? Q * dt * inv : Q;
          p0 = fr ? (q0 * dt - et * Q) * inv : fma(Q, wb, q0);
          p1 = fr ? q1 * dt * inv : q1;
        }
      }
      double y0 = 0.0, y1 = 0.0;
#pragma unroll
      for (int t = 0; t < NMAX; ++t) {
        if (t < N) {
          a[t] = fma(K[t], y0, a[t]);
          b[t] = fma(K[t], y1, b[t]);
          y0 += a[t];
          y1 += b[t];
        }
      }
    }
    // totals of the cumulative sums (gradient r = r0 + gamma r1 by the prefix trick)
    double Z0t = 0.0, Z1t = 0.0;
    {
      double y0 = 0.0, y1 = 0.0;
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) {
          y0 += a[t];
          y1 += b[t];
          Z0t += y0;
          Z1t += y1;
        }
    }
    double best = g_hi;
    int bj = -1, bns = 0;
    {
      double y0 = 0.0, y1 = 0.0, Z0 = 0.0, Z1 = 0.0;
#pragma unroll
      for (int t = 0; t < NMAX; ++t) {
        if (t < N) {
          y0 += a[t];
          y1 += b[t];
          const double r0 = q.c * (Z0t - Z0) + d[t] * a[t] + e[t];
          const double r1 = q.c * (Z1t - Z1 - (double)(N - t)) + d[t] * b[t];
          Z0 += y0;
          Z1 += y1;
          const int s = st.get(t);
          double gc = INFINITY;
          int ns = s;
          if (s & 1) {
            const int kk = (s - 1) >> 1;
            if (b[t] > 0.0) {
              gc = (lq_knot(q, kk + 1) - a[t]) / b[t];
              ns = 2 * (kk + 1);
            } else if (b[t] < 0.0) {
              gc = (lq_knot(q, kk) - a[t]) / b[t];
              ns = 2 * kk;
            }
          } else {
            const int kk = s >> 1;
            if (r1 < 0.0 && kk < q.m) {
              gc = -(lq_slope(q, kk) + r0) / r1;
              ns = 2 * kk + 1;
            } else if (r1 > 0.0 && kk > 0) {
              gc = -(lq_slope(q, kk - 1) + r0) / r1;
              ns = 2 * kk - 1;
            }
          }
          if (t == last && gc <= gcur) gc = INFINITY;
          gc = fmax(gc, gcur);
          if (gc < best) {
            best = gc;
            bj = t;
            bns = ns;
          }
        }
      }
    }
    // record piece [gcur, best] unless it has zero length (simultaneous events)
    const bool final_piece = (bj < 0) || (npc == LQ_PPL - 1);
    if (best > gcur || bj < 0 || final_piece) {
      const size_t pidx = cb * LQ_PPL + npc;
      tab.gend[pidx] = (bj < 0) ? g_hi : best;
      double2* row = reinterpret_cast<double2*>(tab.ab + pidx * (size_t)N * 2);
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) row[t] = make_double2(a[t], b[t]);
#pragma unroll
      for (int i = 0; i < States<NMAX>::NW; ++i) tab.st[pidx * LQ_NW_MAX + i] = st.w[i];
      ++npc;
    }
    if (bj < 0) break;
    st.set_rt(bj, bns);
    gcur = best;
    last = bj;
  }
  tab.cnt[cb] = npc;
  return npc;
}

template <int NMAX>
__global__ __launch_bounds__(64) void k_prepare(QPConst q, int S, const double* __restrict__ lmbd,
                                                const double* __restrict__ lmbd_r,
                                                const double* __restrict__ w_ref,
                                                const double* __restrict__ gamma_ref,
                                                double* __restrict__ setdata, int mode, PathTable tab,
                                                uint32_t* __restrict__ central, int* __restrict__ errflag) {
  lq_tab_init(q);
  const int s = blockIdx.x;
  const int lane = threadIdx.x;
  const int N = q.N;
  const int SD = lq_sd(N);
  __shared__ double sd[3 * NMAX + 8];
  const double* L = lmbd + (size_t)s * 3 * N;
  const double lr = lmbd_r[s];
  for (int t = lane; t < N; t += 64) {
    const double l1 = L[t], l2 = L[N + t], l3 = L[2 * N + t];
    if (!(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0)) atomicOr(errflag, 1);
    sd[t] = 2.0 * lr * q.theta * q.theta + 2.0 * q.q_scale * l3 + q.dsmall;
    sd[N + t] = q.theta * (l1 - l2);
    sd[2 * N + t] = w_ref ? w_ref[(size_t)s * N + t] : 0.0;
  }
  if (lane == 0) {
    double s2 = 0.0;
    for (int t = 0; t < N; ++t) s2 += L[N + t];
    if (!(lr >= 0.0)) atomicOr(errflag, 1);
    sd[3 * N + 0] = q.theta * q.w_max * s2;
    sd[3 * N + 1] = L[0];
    sd[3 * N + 2] = L[N];
    sd[3 * N + 3] = L[2 * N];
    sd[3 * N + 4] = lr;
    sd[3 * N + 5] = lr / q.delta;
    sd[3 * N + 6] = gamma_ref ? gamma_ref[s] : 0.5 * q.y_max;
    sd[3 * N + 7] = w_ref ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int i = lane; i < SD; i += 64) setdata[(size_t)s * SD + i] = sd[i];
  const double* d = sd;
  const double* e = sd + N;
  if (mode == LOMPC_MODE_PATH) {
    const double h = q.y_max / (double)LQ_G;
    const double glo = (double)lane * h;
    const double ghi = (lane == LQ_G - 1) ? q.y_max : (double)(lane + 1) * h;
    States<NMAX> st;
    st.fill(1);
    double w[NMAX];
    bool ok = lq_pdas<NMAX>(q, d, e, glo, st, w, 4 * N + 8);
    if (!ok) ok = lq_primal_as<NMAX>(q, d, e, glo, st, w, 16 * N + 16);
    const size_t cb = (size_t)s * LQ_G + lane;
    if (ok) lq_track<NMAX>(q, d, e, st, glo, ghi, tab, cb);
    else tab.cnt[cb] = 0;
  } else if (lane == 0) {
    const double g = sd[3 * N + 6];
    States<NMAX> st;
    st.fill(1);
    double w[NMAX];
    bool ok = lq_pdas<NMAX>(q, d, e, g, st, w, 4 * N + 8);
    if (!ok) ok = lq_primal_as<NMAX>(q, d, e, g, st, w, 16 * N + 16);
    if (!ok) st.fill(1);
#pragma unroll
    for (int i = 0; i < LQ_NW_MAX; ++i) central[(size_t)s * LQ_NW_MAX + i] = (i < States<NMAX>::NW) ? st.w[i] : 0u;
  }
}

// ------------------------------------------------------------------- K2
template <int NMAX>
__global__ __launch_bounds__(EVAL_BLOCK) void k_eval(QPConst q, KArgs a) {
  lq_tab_init(q);
  const int b = blockIdx.x;
  int s;
  int64_t start, end;
  block_set(a, b, s, start, end);
  const int N = q.N;
  const int tid = threadIdx.x;
  const int64_t i = start + tid;
  const bool active = i < end;
  const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
  const double* d = sd;
  const double* e = sd + N;
  const double g = active ? a.gamma[i] : 0.0;
  const bool valid = active && (g >= 0.0) && (g <= q.y_max);
  double w[NMAX];
  States<NMAX> st;
  bool ok = false;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  if (valid) {
    const double invh = (double)LQ_G / q.y_max;
    const int cell = min(LQ_G - 1, (int)(g * invh));
    const size_t cb = (size_t)s * LQ_G + cell;
    const int cnt = a.tab.cnt[cb];
    if (cnt > 0) {
      int p = cnt - 1;
#pragma unroll
      for (int pp = LQ_PPL - 1; pp >= 0; --pp)
        if (pp < cnt && g <= a.tab.gend[cb * LQ_PPL + pp]) p = pp;
      const size_t pidx = cb * LQ_PPL + p;
      const double2* row = reinterpret_cast<const double2*>(a.tab.ab + pidx * (size_t)N * 2);
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) {
          const double2 ab = row[t];
          w[t] = fma(ab.y, g, ab.x);
        }
      load_states<NMAX>(st, a.tab.st + pidx * LQ_NW_MAX);
      lq_snap<NMAX>(q, st, w);
      ok = lq_kkt<NMAX>(q, d, e, g, st, w) <= q.tol_cert;
    }
  }
  const bool fail = valid && !ok;
  EVOut o{0.0, 0.0, 0.0};
  if (ok) {
    o = lq_outputs<NMAX>(q, sd, g, w, a.want_err != 0);
    if (a.w) {
      double* wo = a.w + (size_t)i * N;
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) wo[t] = w[t];
    }
    if (a.cost) a.cost[i] = o.cost;
    if (a.w0) a.w0[i] = w[0];
  } else if (active && !valid) {
    if (a.w) {
      double* wo = a.w + (size_t)i * N;
      for (int t = 0; t < N; ++t) wo[t] = NAN;
    }
    if (a.cost) a.cost[i] = NAN;
    if (a.w0) a.w0[i] = NAN;
  }
  if (a.status && active) a.status[i] = valid ? (ok ? LOMPC_QP_OK : LOMPC_QP_FAILED) : LOMPC_QP_INVALID;
  // deterministic compaction of the uncertified EVs (ballot order)
  {
    __shared__ int wcnt[EVAL_BLOCK / 64];
    const int lane = tid & 63, wv = tid >> 6;
    const unsigned long long m = __ballot(fail);
    if (lane == 0) wcnt[wv] = __popcll(m);
    __syncthreads();
    int base = 0;
    for (int k = 0; k < wv; ++k) base += wcnt[k];
    if (fail) {
      const int pos = base + __popcll(m & ((1ull << lane) - 1ull));
      a.fail_idx[(size_t)b * EVAL_BLOCK + pos] = (int)(i - start);
    }
    if (tid == 0) {
      int tot = 0;
      for (int k = 0; k < EVAL_BLOCK / 64; ++k) tot += wcnt[k];
      a.fail_cnt[b] = tot;
    }
  }
  block_partials<NMAX>(q, w, ok, o, 0, 0, (active && !valid) ? 1 : 0,
                       a.partial + (size_t)b * (N + NPART_EXTRA), false);
}

// ------------------------------------------------------------------- K2b
template <int NMAX>
__global__ __launch_bounds__(EVAL_BLOCK) void k_direct(QPConst q, KArgs a, int repair) {
  const int b = blockIdx.x;
  if (repair) {
    const int nf = a.fail_cnt[b];
    if (nf == 0) return;  // uniform exit: nothing to repair in this workgroup
  }
  lq_tab_init(q);
  int s;
  int64_t start, end;
  block_set(a, b, s, start, end);
  const int N = q.N;
  const int tid = threadIdx.x;
  int64_t i;
  bool active;
  if (repair) {
    const int nf = a.fail_cnt[b];
    active = tid < nf;
    i = active ? start + a.fail_idx[(size_t)b * EVAL_BLOCK + tid] : start;
  } else {
    i = start + tid;
    active = i < end;
  }
  const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
  const double* d = sd;
  const double* e = sd + N;
  const double g = active ? a.gamma[i] : 0.0;
  const bool valid = active && (g >= 0.0) && (g <= q.y_max);
  double w[NMAX];
  States<NMAX> st;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  bool ok = false;
  if (valid) {
    if (repair) {
      const double invh = (double)LQ_G / q.y_max;
      const int cell = min(LQ_G - 1, (int)(g * invh));
      const size_t cb = (size_t)s * LQ_G + cell;
      if (a.tab.cnt[cb] > 0) load_states<NMAX>(st, a.tab.st + cb * LQ_PPL * LQ_NW_MAX);
      else st.fill(1);
    } else {
      load_states<NMAX>(st, a.central + (size_t)s * LQ_NW_MAX);
    }
    ok = lq_pdas<NMAX>(q, d, e, g, st, w, 4 * N + 8);
    if (ok) {
      lq_snap<NMAX>(q, st, w);
      ok = lq_kkt<NMAX>(q, d, e, g, st, w) <= q.tol_cert;
    }
    if (!ok) {
      ok = lq_primal_as<NMAX>(q, d, e, g, st, w, 16 * N + 16);
      if (ok) {
        lq_snap<NMAX>(q, st, w);
        ok = lq_kkt<NMAX>(q, d, e, g, st, w) <= q.tol_cert;
      }
    }
  }
  EVOut o{0.0, 0.0, 0.0};
  if (valid) {
    o = lq_outputs<NMAX>(q, sd, g, w, a.want_err != 0);
    if (a.w) {
      double* wo = a.w + (size_t)i * N;
#pragma unroll
      for (int t = 0; t < NMAX; ++t)
        if (t < N) wo[t] = w[t];
    }
    if (a.cost) a.cost[i] = o.cost;
    if (a.w0) a.w0[i] = w[0];
  } else if (active) {
    if (a.w) {
      double* wo = a.w + (size_t)i * N;
      for (int t = 0; t < N; ++t) wo[t] = NAN;
    }
    if (a.cost) a.cost[i] = NAN;
    if (a.w0) a.w0[i] = NAN;
  }
  if (a.status && active)
    a.status[i] = !valid ? LOMPC_QP_INVALID : (ok ? (repair ? LOMPC_QP_REPAIRED : LOMPC_QP_OK) : LOMPC_QP_FAILED);
  // failed EVs still contribute their best-effort w (the status says so)
  const bool contrib = valid;
  block_partials<NMAX>(q, w, contrib, o, (repair && valid && ok) ? 1 : 0, (valid && !ok) ? 1 : 0,
                       (!repair && active && !valid) ? 1 : 0, a.partial + (size_t)b * (N + NPART_EXTRA),
                       repair != 0);
}

// ------------------------------------------------------------------- K3
__global__ __launch_bounds__(128) void k_finalize(int N, int S, const int* __restrict__ blk_prefix,
                                                  const int64_t* __restrict__ set_off,
                                                  const double* __restrict__ partial,
                                                  double* __restrict__ set_sum_w, double* __restrict__ set_stats,
                                                  unsigned long long* __restrict__ counters) {
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int W = N + NPART_EXTRA;
  const int b0 = blk_prefix[s], b1 = blk_prefix[s + 1];
  for (int col = tid; col < W; col += blockDim.x) {
    const bool is_max = (col == N + PT_MAX_ERR);
    double acc = 0.0;
    for (int b = b0; b < b1; ++b) {
      const double v = partial[(size_t)b * W + col];
      acc = is_max ? fmax(acc, v) : acc + v;
    }
    if (col < N) {
      if (set_sum_w) set_sum_w[(size_t)s * N + col] = acc;
    } else {
      const int k = col - N;
      if (set_stats) {
        double* row = set_stats + (size_t)s * LOMPC_SET_STATS;
        switch (k) {
          case PT_SUM_W0: row[LOMPC_STAT_SUM_W0] = acc; break;
          case PT_SUM_PRICE0: row[LOMPC_STAT_SUM_PRICE0] = acc; break;
          case PT_MAX_ERR: row[LOMPC_STAT_MAX_ERR] = acc; break;
          case PT_SUM_COST: row[LOMPC_STAT_SUM_COST] = acc; break;
          case PT_N_OK: row[LOMPC_STAT_COUNT] = (double)(set_off[s + 1] - set_off[s]); break;
          case PT_N_REPAIRED: row[LOMPC_STAT_N_REPAIRED] = acc; break;
          case PT_N_FAILED: row[LOMPC_STAT_N_FAILED] = acc; break;
          case PT_N_INVALID: row[LOMPC_STAT_N_INVALID] = acc; break;
        }
      }
      if (k == PT_N_REPAIRED && acc > 0) atomicAdd(&counters[0], (unsigned long long)acc);
      if (k == PT_N_FAILED && acc > 0) atomicAdd(&counters[1], (unsigned long long)acc);
      if (k == PT_N_INVALID && acc > 0) atomicAdd(&counters[2], (unsigned long long)acc);
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
  PathTable tab{nullptr, nullptr, nullptr, nullptr};
  uint32_t* d_central = nullptr;
  int* d_errflag = nullptr;
  int params_mode = -1;
  // batch workspaces
  int64_t nblk_cap = 0, soff_cap = 0;
  double* d_partial = nullptr;
  int* d_fail_cnt = nullptr;
  int* d_fail_idx = nullptr;
  int* d_blk_prefix = nullptr;
  int64_t* d_set_off = nullptr;
  unsigned long long* d_counters = nullptr;
  int* h_pin_prefix = nullptr;
  int64_t* h_pin_off = nullptr;
  hipEvent_t ev_map = nullptr;
  std::vector<int64_t> last_off;
  void* last_off_stream = nullptr;
  // single-solve scratch (3N + N + 4 doubles)
  double* d_single = nullptr;
  int8_t* d_single_status = nullptr;
  // profiling
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;  // pairs
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

#define DISPATCH_NMAX(nmax, ...) \
  switch (nmax) {                 \
    case 16: { constexpr int NM = 16; __VA_ARGS__; } break; \
    case 24: { constexpr int NM = 24; __VA_ARGS__; } break; \
    case 32: { constexpr int NM = 32; __VA_ARGS__; } break; \
    case 48: { constexpr int NM = 48; __VA_ARGS__; } break; \
    case 64: { constexpr int NM = 64; __VA_ARGS__; } break; \
    default: break;               \
  }

extern "C" {

int lompc_abi_version(void) { return 1; }

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
  q.c = 2.0 * delta * theta * theta;          // lompc.py:71
  q.q_scale = 3.0 * theta / (4.0 * w_max);    // lompc.py:67
  q.dsmall = q.ev_small ? 2.0 * theta * theta / (0.9 * 0.9) : 0.0;  // lompc.py:105
  if (q.ev_small) {
    q.m = 1;
    q.knots[0] = 0.0;
    q.knots[1] = w_max;
    for (int k = 2; k <= LQ_MAXSEG; ++k) q.knots[k] = w_max;
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
      (e = hipMalloc((void**)&c->d_counters, 4 * sizeof(unsigned long long))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single, (4 * N + 8) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single_status, 8)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev_map, hipEventDisableTiming)) != hipSuccess) {
    delete c;
    return LOMPC_ERR_HIP;
  }
  (void)hipMemset(c->d_errflag, 0, sizeof(int));
  (void)hipMemset(c->d_counters, 0, 4 * sizeof(unsigned long long));
  *out = c;
  return LOMPC_OK;
}

int lompc_destroy(lompc_ctx* c) {
  if (!c) return LOMPC_OK;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  void* ptrs[] = {c->d_setdata, c->tab.cnt, c->tab.gend, c->tab.ab, c->tab.st, c->d_central, c->d_errflag,
                  c->d_partial, c->d_fail_cnt, c->d_fail_idx, c->d_blk_prefix, c->d_set_off, c->d_counters,
                  c->d_single, c->d_single_status};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_pin_prefix) (void)hipHostFree(c->h_pin_prefix);
  if (c->h_pin_off) (void)hipHostFree(c->h_pin_off);
  if (c->ev_map) (void)hipEventDestroy(c->ev_map);
  for (hipEvent_t ev : c->prof_ev) (void)hipEventDestroy(ev);
  delete c;
  return LOMPC_OK;
}

int lompc_set_mode(lompc_ctx* c, int mode) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (mode != LOMPC_MODE_PATH && mode != LOMPC_MODE_DIRECT) return fail_arg(c, "mode must be PATH or DIRECT");
  c->mode = mode;
  return LOMPC_OK;
}

int lompc_get_info(const lompc_ctx* c, int* N, int* ev_type) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (N) *N = c->N;
  if (ev_type) *ev_type = c->ev_type;
  return LOMPC_OK;
}

int lompc_set_params(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, const double* w_ref,
                     const double* gamma_ref, void* stream) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (S < 1 || !lmbd || !lmbd_r) return fail_arg(c, "set_params: S >= 1 and lmbd, lmbd_r required");
  if (S > (1 << 24)) return fail_arg(c, "set_params: too many parameter sets");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  const int N = c->N;
  if (S > c->S_cap) {
    int rc;
    const size_t cells = (size_t)S * LQ_G;
    if ((rc = grow(c, &c->d_setdata, (size_t)S * lq_sd(N))) ||
        (rc = grow(c, &c->tab.cnt, cells)) || (rc = grow(c, &c->tab.gend, cells * LQ_PPL)) ||
        (rc = grow(c, &c->tab.ab, cells * LQ_PPL * (size_t)N * 2)) ||
        (rc = grow(c, &c->tab.st, cells * LQ_PPL * LQ_NW_MAX)) ||
        (rc = grow(c, &c->d_central, (size_t)S * LQ_NW_MAX)))
      return rc;
    c->S_cap = S;
  }
  c->S = S;
  c->params_mode = c->mode;
  dim3 grid((unsigned)S), block(64);
  DISPATCH_NMAX(c->nmax, hipLaunchKernelGGL(k_prepare<NM>, grid, block, 0, st, c->q, (int)S, lmbd, lmbd_r, w_ref,
                                             gamma_ref, c->d_setdata, c->mode, c->tab, c->d_central,
                                             c->d_errflag));
  HIPCHK(c, hipGetLastError());
  return LOMPC_OK;
}

static int upload_block_map(lompc_ctx* c, const int64_t* set_off, int64_t S, int* nblk_out, hipStream_t st) {
  // host prefix of workgroups per set
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
  const bool same = (int64_t)c->last_off.size() == S + 1 && c->last_off_stream == (void*)st &&
                    memcmp(c->last_off.data(), set_off, (S + 1) * sizeof(int64_t)) == 0;
  if (nb > c->nblk_cap) {
    int rc;
    if ((rc = grow(c, &c->d_partial, (size_t)nb * (c->N + NPART_EXTRA))) ||
        (rc = grow(c, &c->d_fail_cnt, (size_t)nb)) || (rc = grow(c, &c->d_fail_idx, (size_t)nb * EVAL_BLOCK)))
      return rc;
    c->nblk_cap = nb;
  }
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
  // the pinned staging buffer may still be read by the previous upload
  HIPCHK(c, hipEventSynchronize(c->ev_map));
  memcpy(c->h_pin_prefix, pre.data(), (S + 1) * sizeof(int));
  memcpy(c->h_pin_off, set_off, (S + 1) * sizeof(int64_t));
  HIPCHK(c, hipMemcpyAsync(c->d_blk_prefix, c->h_pin_prefix, (S + 1) * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->d_set_off, c->h_pin_off, (S + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipEventRecord(c->ev_map, st));
  c->last_off.assign(set_off, set_off + S + 1);
  c->last_off_stream = (void*)st;
  return LOMPC_OK;
}

int lompc_solve_batch(lompc_ctx* c, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
                      double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats,
                      void* stream) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (c->S < 1) return fail_arg(c, "solve_batch: call lompc_set_params first");
  if (B < 0 || !set_offsets) return fail_arg(c, "solve_batch: invalid batch");
  if (set_offsets[0] != 0 || set_offsets[c->S] != B)
    return fail_arg(c, "solve_batch: set_offsets must start at 0 and end at B");
  if (B > 0 && !gamma) return fail_arg(c, "solve_batch: gamma required");
  HIPCHK(c, hipSetDevice(c->device));
  hipStream_t st = (hipStream_t)stream;
  int nblk = 0;
  int rc = upload_block_map(c, set_offsets, c->S, &nblk, st);
  if (rc) return rc;
  HIPCHK(c, hipMemsetAsync(c->d_counters, 0, 4 * sizeof(unsigned long long), st));
  KArgs a{};
  a.B = B;
  a.S = (int)c->S;
  a.nblk = nblk;
  a.want_err = 1;
  a.gamma = gamma;
  a.blk_prefix = c->d_blk_prefix;
  a.set_off = c->d_set_off;
  a.setdata = c->d_setdata;
  a.tab = c->tab;
  a.central = c->d_central;
  a.w = w;
  a.cost = cost;
  a.w0 = w0;
  a.status = status;
  a.partial = c->d_partial;
  a.fail_cnt = c->d_fail_cnt;
  a.fail_idx = c->d_fail_idx;
  if (nblk > 0) {
    dim3 grid((unsigned)nblk), block(EVAL_BLOCK);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (c->prof) {
      HIPCHK(c, hipEventCreate(&e0));
      HIPCHK(c, hipEventCreate(&e1));
      HIPCHK(c, hipEventRecord(e0, st));
    }
    if (c->params_mode == LOMPC_MODE_PATH) {
      DISPATCH_NMAX(c->nmax, hipLaunchKernelGGL(k_eval<NM>, grid, block, 0, st, c->q, a));
    } else {
      DISPATCH_NMAX(c->nmax, hipLaunchKernelGGL(k_direct<NM>, grid, block, 0, st, c->q, a, 0));
    }
    if (c->prof) {
      HIPCHK(c, hipEventRecord(e1, st));
      c->prof_ev.push_back(e0);
      c->prof_ev.push_back(e1);
    }
    HIPCHK(c, hipGetLastError());
    if (c->params_mode == LOMPC_MODE_PATH) {
      DISPATCH_NMAX(c->nmax, hipLaunchKernelGGL(k_direct<NM>, grid, block, 0, st, c->q, a, 1));
      HIPCHK(c, hipGetLastError());
    }
  }
  if (set_sum_w || set_stats || nblk > 0) {
    hipLaunchKernelGGL(k_finalize, dim3((unsigned)c->S), dim3(128), 0, st, c->N, (int)c->S, c->d_blk_prefix,
                       c->d_set_off, c->d_partial, set_sum_w, set_stats, c->d_counters);
    HIPCHK(c, hipGetLastError());
  }
  return LOMPC_OK;
}

int lompc_last_status(lompc_ctx* c, void* stream, int64_t* n_repaired, int64_t* n_failed, int64_t* n_invalid) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  unsigned long long h[4] = {0, 0, 0, 0};
  int ef = 0;
  HIPCHK(c, hipMemcpyAsync(h, c->d_counters, sizeof(h), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipMemcpyAsync(&ef, c->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  if (n_repaired) *n_repaired = (int64_t)h[0];
  if (n_failed) *n_failed = (int64_t)h[1];
  if (n_invalid) *n_invalid = (int64_t)h[2];
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
    (void)hipEventDestroy(c->prof_ev[k]);
    (void)hipEventDestroy(c->prof_ev[k + 1]);
  }
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
