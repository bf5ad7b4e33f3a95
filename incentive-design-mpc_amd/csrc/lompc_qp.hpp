// lompc_qp.hpp — device-side building blocks of the batched LoMPC QP engine.
//
// The per-EV program is LoMPC.solve_lompc (reference chargingstation/lompc.py:137-156):
//
//   minimize  0.5 c ||A w||^2 - c*gamma*1'A w + sum_t (0.5 d_t w_t^2 + e_t w_t)
//             + [large EVs] sum_t pwl(w_t) + c0
//   s.t.      0 <= w <= w_max                                    (lompc.py:74, :93)
//
// with A = tril(ones) (lompc.py:69), c = 2 delta theta^2 (lompc.py:71, :117-122),
// d_t = 2 lmbd_r theta^2 + 2 q_scale lmbd3_t [+ 2 theta^2/0.81 small]   (:105, :131, :133)
// e_t = theta (lmbd1_t - lmbd2_t), c0 = theta w_max sum(lmbd2)          (:126-129)
// pwl = (theta w_max)^2 max(0, u-0.125, 1.5u-0.375, 2u-0.75), u = w/w_max (:108-114).
//
// y = A w is the cumulative charge, so the program is a scalar-state chain:
// for any working set (each coordinate either fixed at a "knot" — a box bound
// or a PWL kink — or free inside one PWL segment) the equality-constrained
// sub-problem is solved EXACTLY by a backward scalar Riccati recursion plus a
// forward pass: O(N) flops and N divisions, no N x N matrix anywhere.
//
// State encoding per coordinate (4 bits): even s = 2k  -> fixed at knot k,
//                                          odd  s = 2k+1 -> free in segment k.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LQ_MAXSEG 4     // large EVs: 4 PWL segments (lompc.py:111)
#define LQ_G 64         // path cells per parameter set (one lane each)
#define LQ_PPL 8        // max affine pieces stored per cell
#define LQ_NW_MAX 8     // packed state words per stored piece (64 coords / 8)

struct QPConst {
  int N;             // horizon
  int m;             // number of separable segments (1 small, 4 large)
  int ev_small;      // 1 for "small"
  int pad0;
  double c;          // 2 delta theta^2
  double delta, theta, y_max, w_max, q_scale;
  double dsmall;     // 2 theta^2 / 0.9^2 for small EVs, 0 otherwise
  double knots[LQ_MAXSEG + 1];
  double slopes[LQ_MAXSEG];
  double scale;      // magnitude of the gradient, for relative tolerances
  double tol_switch; // active-set switching tolerance (absolute, gradient units)
  double tol_cert;   // KKT certificate tolerance (absolute, gradient units)
  double ktol;       // knot tolerance on w (absolute)
};

// Per-set data record (doubles), stride SD(N) = 3N + 8:
//   [0,N) d   [N,2N) e   [2N,3N) w_ref
//   3N+0 c0, +1 lmbd1_0, +2 lmbd2_0, +3 lmbd3_0, +4 lmbd_r, +5 kappa, +6 gamma_ref, +7 has_wref
__host__ __device__ inline int lq_sd(int N) { return 3 * N + 8; }

// Path table (device pointers). Cell l of set s covers gamma in [l h, (l+1) h], h = y_max / LQ_G.
struct PathTable {
  int* cnt;          // [S][G]          pieces stored in the cell (0 = cell unsolved)
  double* gend;      // [S][G][PPL]     upper gamma of each piece
  double* ab;        // [S][G][PPL][N][2]  w_j(gamma) = a_j + b_j gamma
  uint32_t* st;      // [S][G][PPL][LQ_NW_MAX] packed working set of the piece
};

// Knot / slope tables live in LDS: indexed by a per-lane state, a register
// select chain is turned into an indexed load by the compiler, and indexing the
// by-value kernel argument would force a scratch copy of QPConst.
__device__ __forceinline__ double* lq_tab() {
  __shared__ double tab[LQ_MAXSEG * 2 + 2];
  return tab;
}
// Every kernel calls this (all threads) before the first lq_knot / lq_slope.
__device__ __forceinline__ void lq_tab_init(const QPConst& q) {
  double* tb = lq_tab();
  const int t = threadIdx.x;
  if (t <= LQ_MAXSEG) tb[t] = q.knots[t];
  if (t < LQ_MAXSEG) tb[LQ_MAXSEG + 1 + t] = q.slopes[t];
  __syncthreads();
}
__device__ __forceinline__ double lq_knot(const QPConst&, int k) { return lq_tab()[k]; }
// k = -1 is read only on paths whose value is discarded (fixed coordinates).
__device__ __forceinline__ double lq_slope(const QPConst&, int k) { return lq_tab()[LQ_MAXSEG + 1 + k]; }

// Packed working set: 4 bits per coordinate, 8 coordinates per word.
template <int NMAX>
struct States {
  static constexpr int NW = (NMAX + 7) / 8;
  uint32_t w[NW];
  __device__ __forceinline__ int get(int t) const {  // t must be compile-time in hot loops
    return (int)((w[t >> 3] >> ((t & 7) * 4)) & 15u);
  }
  __device__ __forceinline__ void set(int t, int v) {
    const int sh = (t & 7) * 4;
    w[t >> 3] = (w[t >> 3] & ~(15u << sh)) | ((uint32_t)v << sh);
  }
  // runtime-index set without dynamic register indexing
  __device__ __forceinline__ void set_rt(int t, int v) {
    const int wi = t >> 3;
    const int sh = (t & 7) * 4;
#pragma unroll
    for (int i = 0; i < NW; ++i)
      if (i == wi) w[i] = (w[i] & ~(15u << sh)) | ((uint32_t)v << sh);
  }
  __device__ __forceinline__ void fill(int v) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x |= ((uint32_t)v) << (4 * i);
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = x;
  }
};

// ---------------------------------------------------------------------------
// Exact sub-problem solve for a working set (single right-hand side).
// Backward:  V_{t+1}(y) = 0.5 P y^2 + p y;  Q = c + P, q = p - c gamma
//   free  : w_t = K y_{t-1} + k,  K = -Q/(Q+d), k = -(q+e~)/(Q+d),
//           P' = Q d/(Q+d),  p' = (q d - e~ Q)/(Q+d)       (e~ = e_t + slope)
//   fixed : w_t = wbar,  P' = Q,  p' = Q wbar + q
// Q >= c > 0, so every division is well defined.
// ---------------------------------------------------------------------------
template <int NMAX>
__device__ __forceinline__ void lq_riccati(const QPConst& q, const double* __restrict__ d,
                                           const double* __restrict__ e, double gamma,
                                           const States<NMAX>& st, double (&w)[NMAX]) {
  double K[NMAX], k[NMAX];
  double P = 0.0, p = 0.0;
  const double cg = q.c * gamma;
#pragma unroll
  for (int t = NMAX - 1; t >= 0; --t) {
    if (t < q.N) {
      const double Q = q.c + P;
      const double qq = p - cg;
      const int s = st.get(t);
      const double dt = d[t];
      const bool fr = (s & 1) != 0;
      const double et = e[t] + lq_slope(q, (s - 1) >> 1);
      const double inv = 1.0 / (Q + dt);
      const double wb = lq_knot(q, s >> 1);
      K[t] = fr ? -Q * inv : 0.0;
      k[t] = fr ? -(qq + et) * inv : wb;
      P = fr ? Q * dt * inv : Q;
      p = fr ? (qq * dt - et * Q) * inv : fma(Q, wb, qq);
    }
  }
  double y = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < q.N) {
      w[t] = fma(K[t], y, k[t]);
      y += w[t];
    }
  }
}

// Gradient of the smooth part: r_j = c (sum_{i>=j} y_i - (N-j) gamma) + d_j w_j + e_j.
// Computed on the fly by callers with the prefix trick (two forward passes).
template <int NMAX>
__device__ __forceinline__ double lq_sum_y(const QPConst& q, const double (&w)[NMAX]) {
  double y = 0.0, Z = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < q.N) {
      y += w[t];
      Z += y;
    }
  return Z;
}

// One PDAS (semismooth-Newton active-set) state update from the current
// sub-problem solution w.  Returns true if any coordinate changed state.
template <int NMAX>
__device__ __forceinline__ bool lq_pdas_update(const QPConst& q, const double* __restrict__ d,
                                               const double* __restrict__ e, double gamma,
                                               const double (&w)[NMAX], States<NMAX>& st) {
  const double Zt = lq_sum_y<NMAX>(q, w);
  double y = 0.0, Z = 0.0;
  bool changed = false;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < q.N) {
      y += w[t];
      const double r = q.c * (Zt - Z - (double)(q.N - t) * gamma) + d[t] * w[t] + e[t];
      Z += y;
      const int s = st.get(t);
      int ns = s;
      if (s & 1) {
        const int kk = (s - 1) >> 1;
        if (w[t] > lq_knot(q, kk + 1) + q.ktol) ns = 2 * (kk + 1);
        else if (w[t] < lq_knot(q, kk) - q.ktol) ns = 2 * kk;
      } else {
        const int kk = s >> 1;
        const double v = -r;
        if (kk < q.m && v > lq_slope(q, kk) + q.tol_switch) ns = 2 * kk + 1;
        else if (kk > 0 && v < lq_slope(q, kk - 1) - q.tol_switch) ns = 2 * kk - 1;
      }
      if (ns != s) {
        st.set(t, ns);
        changed = true;
      }
    }
  }
  return changed;
}

// PDAS from the given working set. Returns true on convergence (w then solves
// the sub-problem of the final working set, which satisfies KKT within tol).
template <int NMAX>
__device__ __forceinline__ bool lq_pdas(const QPConst& q, const double* __restrict__ d, const double* __restrict__ e,
                        double gamma, States<NMAX>& st, double (&w)[NMAX], int max_it) {
  bool done = false;
  for (int it = 0; it < max_it && !done; ++it) {
    lq_riccati<NMAX>(q, d, e, gamma, st, w);
    done = !lq_pdas_update<NMAX>(q, d, e, gamma, w, st);
  }
  return done;
}

// Clamp a free coordinate into its segment; fixed coordinates sit exactly on their knot.
template <int NMAX>
__device__ __forceinline__ void lq_snap(const QPConst& q, const States<NMAX>& st, double (&w)[NMAX]) {
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < q.N) {
      const int s = st.get(t);
      if (s & 1) {
        const int kk = (s - 1) >> 1;
        w[t] = fmin(fmax(w[t], lq_knot(q, kk)), lq_knot(q, kk + 1));
      } else {
        w[t] = lq_knot(q, s >> 1);
      }
    }
}

// Primal active-set method (Nocedal & Wright Alg. 16.3 with PWL kinks as
// knots) from w = 0 with every coordinate fixed at knot 0.  Slow but
// monotone; used only when PDAS does not converge.
template <int NMAX>
__device__ __forceinline__ bool lq_primal_as(const QPConst& q, const double* __restrict__ d, const double* __restrict__ e,
                             double gamma, States<NMAX>& st, double (&w)[NMAX], int max_it) {
  st.fill(0);
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  bool done = false;
  for (int it = 0; it < max_it && !done; ++it) {
    double wh[NMAX];
    lq_riccati<NMAX>(q, d, e, gamma, st, wh);
    double alpha = 1.0;
    int blk = -1, bknot = 0;
#pragma unroll
    for (int t = 0; t < NMAX; ++t) {
      if (t < q.N) {
        const int s = st.get(t);
        const double pj = wh[t] - w[t];
        if (s & 1) {
          const int kk = (s - 1) >> 1;
          if (pj > 0.0) {
            const double a = (lq_knot(q, kk + 1) - w[t]) / pj;
            if (a < alpha) { alpha = a; blk = t; bknot = kk + 1; }
          } else if (pj < 0.0) {
            const double a = (lq_knot(q, kk) - w[t]) / pj;
            if (a < alpha) { alpha = a; blk = t; bknot = kk; }
          }
        }
      }
    }
    if (blk < 0) {
#pragma unroll
      for (int t = 0; t < NMAX; ++t) w[t] = wh[t];
      // most violated fixed coordinate
      const double Zt = lq_sum_y<NMAX>(q, w);
      double y = 0.0, Z = 0.0, best = q.tol_switch;
      int bj = -1, bs = 0;
#pragma unroll
      for (int t = 0; t < NMAX; ++t) {
        if (t < q.N) {
          y += w[t];
          const double r = q.c * (Zt - Z - (double)(q.N - t) * gamma) + d[t] * w[t] + e[t];
          Z += y;
          const int s = st.get(t);
          if (!(s & 1)) {
            const int kk = s >> 1;
            if (kk < q.m) {
              const double v = -r - lq_slope(q, kk);
              if (v > best) { best = v; bj = t; bs = 2 * kk + 1; }
            }
            if (kk > 0) {
              const double v = r + lq_slope(q, kk - 1);
              if (v > best) { best = v; bj = t; bs = 2 * kk - 1; }
            }
          }
        }
      }
      if (bj < 0) done = true;
      else st.set_rt(bj, bs);
    } else {
      alpha = fmax(alpha, 0.0);
      const double kv = lq_knot(q, bknot);
#pragma unroll
      for (int t = 0; t < NMAX; ++t) {
        w[t] = fma(alpha, wh[t] - w[t], w[t]);
        if (t == blk) w[t] = kv;
      }
      st.set_rt(blk, 2 * bknot);
    }
  }
  return done;
}

// KKT certificate of (w, working set): returns the max violation in gradient
// units (stationarity of free coordinates, multiplier range of fixed ones) or
// +inf when a free coordinate left its segment by more than ktol.
template <int NMAX>
__device__ __forceinline__ double lq_kkt(const QPConst& q, const double* __restrict__ d,
                                         const double* __restrict__ e, double gamma,
                                         const States<NMAX>& st, const double (&w)[NMAX]) {
  const double Zt = lq_sum_y<NMAX>(q, w);
  double y = 0.0, Z = 0.0, res = 0.0;
  bool outside = false;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < q.N) {
      y += w[t];
      const double r = q.c * (Zt - Z - (double)(q.N - t) * gamma) + d[t] * w[t] + e[t];
      Z += y;
      const int s = st.get(t);
      const double v = -r;
      if (s & 1) {
        const int kk = (s - 1) >> 1;
        res = fmax(res, fabs(v - lq_slope(q, kk)));
        outside |= (w[t] < lq_knot(q, kk) - q.ktol) || (w[t] > lq_knot(q, kk + 1) + q.ktol);
      } else {
        const int kk = s >> 1;
        if (kk > 0) res = fmax(res, lq_slope(q, kk - 1) - v);
        if (kk < q.m) res = fmax(res, v - lq_slope(q, kk));
      }
    }
  }
  return outside ? INFINITY : res;
}

// Per-EV scalar outputs from an optimal w:
//   cost  (lompc.py:155: the full objective incl. c0)
//   err   = sqrt((w-w_ref)' A_bar (w-w_ref)), A_bar = A'A + kappa I (price_solver.py:191-192, :207)
//   price0 (lompc.py:164-170)
struct EVOut {
  double cost, err, price0;
};

template <int NMAX>
__device__ __forceinline__ EVOut lq_outputs(const QPConst& q, const double* __restrict__ sd, double gamma,
                                            const double (&w)[NMAX], bool want_err) {
  const int N = q.N;
  const double* d = sd;
  const double* e = sd + N;
  const double* wr = sd + 2 * N;
  const double kappa = sd[3 * N + 5];
  double y = 0.0, sy = 0.0, syy = 0.0, quad = 0.0, pwl = 0.0;
  double ey = 0.0, eyy = 0.0, edd = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      const double wt = w[t];
      y += wt;
      sy += y;
      syy = fma(y, y, syy);
      quad += wt * fma(0.5 * d[t], wt, e[t]);
      if (!q.ev_small) {
        const double u = wt / q.w_max;
        const double v = fmax(fmax(0.0 * u, u - 0.125), fmax(1.5 * u - 0.375, 2.0 * u - 0.75));
        pwl += v;
      }
      if (want_err) {
        const double dv = wt - wr[t];
        ey += dv;
        eyy = fma(ey, ey, eyy);
        edd = fma(dv, dv, edd);
      }
    }
  }
  EVOut o;
  const double tw = q.theta * q.w_max;
  o.cost = 0.5 * q.c * syy - q.c * gamma * sy + quad + sd[3 * N + 0] + (q.ev_small ? 0.0 : tw * tw * pwl);
  o.err = want_err ? sqrt(eyy + kappa * edd) : 0.0;
  const double w0 = w[0];
  o.price0 = q.theta * (w0 * sd[3 * N + 1] + (q.w_max - w0) * sd[3 * N + 2]) +
             q.q_scale * w0 * w0 * sd[3 * N + 3] + q.theta * q.theta * w0 * w0 * sd[3 * N + 4];
  return o;
}
