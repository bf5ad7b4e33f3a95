// lompc_pricewave.hpp — the price-gradient step of PriceSolver (price_solver.py:216-246, its CVXPY
// problem :257-270) on ONE 64-lane wave, lane t = horizon stage t: the device form of
// lompc_price_step (lompc_price.cpp), used by the device-resident price loop (lompc_loop.hip).
//
//   lmbd_next = argmin_{x >= 0} 1/2 x'Qx + q'x,   Q = 2P = 2 eps I + U A_bar^-1 U' / m,
//   q = -Q lmbd - (phi(w) - phi(w_ref)),           A_bar = A'A + kappa I   (price_solver.py:188-194)
//
// Every row of U = Dphi(w) (lompc.py:179-187) touches one stage, so lane t owns the price rows
// t, N + t and 2N + t (theta, -theta, 2 q_s w_t).  Each reduced solve of the active-set method is
// ONE solve with a A_bar + diag(E) = a A'A + diag(a kappa + E) (lompc_price.cpp's TriSolve); here it
// is the stage (Riccati) recursion of the LoMPC kernels — a Moebius-map prefix scan with
// nonnegative entries and two affine prefix scans — so a solve is a few DPP scans instead of 4N
// dependent host steps.  Same method as the host: primal-dual active set from the previous prices' free set,
// primal active set from x = 0 as the fallback (ties broken in the host's row order), KKT-certified.
#pragma once
#include "lompc_wave.hpp"

namespace lqp {

using lqw::Aff;
using lqw::Mob;

// Solves with c A'A + diag(E) (c > 0, E >= 0) as the stage recursion of
//   min 1/2 x'(c A'A + diag(E)) x - b'x,   y_t = y_{t-1} + x_t  (A = tril(1): y = A x)
// — the cost-to-go V_t(y) = 1/2 P_t y^2 + p_t y of the LoMPC kernels' Riccati form
// (lompc_wave.hpp solve_stage, all coordinates free):
//   P_t = E_t (c + P_{t+1}) / (E_t + c + P_{t+1})      Moebius map with entries >= 0 (no cancellation;
//                                                      the pivot form a_t - E_t^2 / d_{t-1} loses ~1e-11)
//   p_t = E_t iv_t p_{t+1} + b_t Q_t iv_t,  Q_t = c + P_{t+1},  iv_t = 1 / (Q_t + E_t)
//   x_t = K_t y_{t-1} + k_t,  K_t = -Q_t iv_t,  k_t = (b_t - p_{t+1}) iv_t
// All in the natural layout (lane t = stage t): P and p are suffix scans (lqw::wave_scan_rev: DPP
// inside the 16-lane rows, row totals by v_readlane), y a prefix scan — no lane reversal through LDS.
struct Tri {
  double Q, iv, d;  // Q_t, iv_t, E_t
  double K;         // K_t
};

__device__ __forceinline__ Tri tri_factor(double c, double E, int N, int lane) {
  const bool act = lane < N;
  const double d = act ? E : 0.0;
  Mob f = Mob::identity();
  if (act) {  // P -> d (c + P) / (c + P + d), scaled to d-entry 1
    const double u = 1.0 / (c + d);
    f = {d * u, d * c * u, u, 1.0};
  }
  const Mob T = lqw::wave_scan_rev(f, N);
  const double Pn = lqw::shl1(0.0, T.b / T.d);  // P_{t+1} (P_N = 0: lane N holds the identity, or lane 63's old)
  Tri t;
  t.Q = c + Pn;
  t.iv = 1.0 / (t.Q + d);
  t.d = d;
  t.K = act ? -t.Q * t.iv : 0.0;
  return t;
}

// x = (c A'A + diag(E))^-1 b
__device__ __forceinline__ double tri_solve(const Tri& T, double b, int N, int lane) {
  const bool act = lane < N;
  Aff<1> g = Aff<1>::identity();
  if (act) {
    g.A = T.d * T.iv;
    g.B[0] = b * T.Q * T.iv;
  }
  const double pn = lqw::shl1(0.0, lqw::wave_scan_rev(g, N).B[0]);  // p_{t+1}
  const double k = act ? (b - pn) * T.iv : 0.0;
  Aff<1> h = Aff<1>::identity();
  if (act) {
    h.A = 1.0 + T.K;
    h.B[0] = k;
  }
  const double y = lqw::wave_scan(h, N).B[0];
  return act ? fma(T.K, lqw::shr1(0.0, y), k) : 0.0;
}

// the price QP of one step: rows k = 0, 1, 2 of lane t are price rows kN + t (k < nb = r / N)
struct PriceQPW {
  int N, nb, lane;
  double u[3];
  double eps, m, kappa;
  Tri Ab;  // factor of A_bar = A'A + kappa I

  // ab: the factor of A_bar = A'A + kappa I when known (it depends on kappa and N only: the device
  // loop computes it at its first step and keeps it), else null
  __device__ __forceinline__ void init(int N_, int r, double theta, double w_max, double m_, double kappa_,
                                       double eps_, double w, const Tri* ab = nullptr) {
    N = N_;
    nb = r / N_;
    lane = (int)threadIdx.x & 63;
    eps = eps_;
    m = m_;
    kappa = kappa_;
    const double q_s = 3.0 * theta / (4.0 * w_max);  // lompc.py:67
    const bool act = lane < N;
    u[0] = act ? theta : 0.0;   // Dphi rows, lompc.py:179-187
    u[1] = act ? -theta : 0.0;
    u[2] = (act && nb > 2) ? 2.0 * q_s * w : 0.0;
    Ab = ab ? *ab : tri_factor(1.0, kappa, N, lane);
  }
  __device__ __forceinline__ bool has(int k) const { return lane < N && k < nb; }

  __device__ __forceinline__ void mulQ(const double (&x)[3], double (&y)[3]) const {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) v = has(k) ? fma(u[k], x[k], v) : v;
    v = tri_solve(Ab, v, N, lane);
    const double im = 1.0 / m;
#pragma unroll
    for (int k = 0; k < 3; ++k) y[k] = has(k) ? fma(u[k] * v, im, 2.0 * eps * x[k]) : 0.0;
  }

  // z = argmin 1/2 z'Qz + q'z over {z_i = 0, i not free}: Woodbury in the free rows,
  // (a A_bar + D_F) s = U_F' q with a = 2 eps m
  __device__ __forceinline__ void solveF(const bool (&F)[3], const double (&q)[3], double (&z)[3]) const {
    const double a = 2.0 * eps * m;
    double E = a * kappa, s = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (F[k]) {
        E = fma(u[k], u[k], E);
        s = fma(u[k], q[k], s);
      }
    const Tri G = tri_factor(a, E, N, lane);
    s = tri_solve(G, s, N, lane);
    const double h = -0.5 / eps;
#pragma unroll
    for (int k = 0; k < 3; ++k) z[k] = F[k] ? h * fma(-u[k], s, q[k]) : 0.0;
  }

  __device__ __forceinline__ double kkt(const double (&x)[3], const double (&mu)[3]) const {
    double res = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k)
      if (has(k)) {
        if (x[k] < 0.0) res = fmax(res, -x[k]);
        res = fmax(res, x[k] > 0.0 ? fabs(mu[k]) : fmax(0.0, -mu[k]));
      }
    return lqw::wave_max(res, 64);
  }
};

// lowest row (host order: block k first, then stage) holding the minimum of v over rows with
// sel; returns false if none.  Strict-less updates in row order as the host's scans.
__device__ __forceinline__ bool row_argmin(const PriceQPW& P, const double (&v)[3], const bool (&sel)[3], double& best,
                                           int& bk, int& bl) {
  bool found = false;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    double x = sel[k] ? v[k] : INFINITY;
    int l = P.lane;
    lqw::wave_argmin(x, l, 64);
    if (x < best) {
      best = x;
      bk = k;
      bl = l;
      found = true;
    }
  }
  return found;
}

// exact non-negative QP (lompc_price.cpp nnqp): PDAS from the warm free set, primal active set
// from x = 0 as the fallback.  Returns false when neither certifies (LOMPC_ERR_NOT_CONVERGED);
// on success mu = Q x + q (the certificate's multipliers).
__device__ __forceinline__ bool nnqp_wave(const PriceQPW& P, const double (&q)[3], const double (&xw)[3], double (&x)[3],
                                          double tol, double (&mu)[3]) {
  bool F[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) F[k] = P.has(k) && xw[k] > 0.0;
  double z[3];
  for (int it = 0; it < 64; ++it) {
    P.solveF(F, q, z);
    P.mulQ(z, mu);
    bool Fn[3], diff = false;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      mu[k] += q[k];
      Fn[k] = P.has(k) && (F[k] ? (z[k] > 0.0) : (mu[k] < 0.0));
      diff |= Fn[k] != F[k];
    }
    if (!__any(diff)) {
      if (P.kkt(z, mu) <= tol) {
#pragma unroll
        for (int k = 0; k < 3; ++k) x[k] = z[k];
        return true;
      }
      break;
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) F[k] = Fn[k];
  }
  // primal active set from x = 0 (feasible): finite for a strictly convex QP
  const int r = P.nb * P.N;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    F[k] = false;
    x[k] = 0.0;
  }
  for (int it = 0; it < 64 * r + 64; ++it) {
    P.solveF(F, q, z);
    double ratio[3];
    bool blocking[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      blocking[k] = F[k] && z[k] <= 0.0;
      ratio[k] = blocking[k] ? x[k] / (x[k] - z[k]) : INFINITY;
    }
    double alpha = 1.0;
    int bk = -1, bl = -1;
    const bool blk = row_argmin(P, ratio, blocking, alpha, bk, bl);
    if (!blk) {
#pragma unroll
      for (int k = 0; k < 3; ++k) x[k] = z[k];
      P.mulQ(x, mu);
      bool cand[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        mu[k] += q[k];
        cand[k] = P.has(k) && !F[k];
      }
      double best = -tol;
      int jk = -1, jl = -1;
      if (!row_argmin(P, mu, cand, best, jk, jl)) return P.kkt(x, mu) <= tol;
      if (P.lane == jl) {
#pragma unroll
        for (int k = 0; k < 3; ++k) F[k] = F[k] || k == jk;
      }
    } else {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        if (F[k]) x[k] = fma(alpha, z[k] - x[k], x[k]);
        if (P.lane == bl && k == bk) {
          x[k] = 0.0;
          F[k] = false;
        }
        if (F[k] && x[k] <= 0.0) {
          x[k] = 0.0;
          F[k] = false;
        }
      }
    }
  }
  return false;
}

}  // namespace lqp
