// lompc_price.cpp — host solvers of the per-partition price step (C-ABI in include/lompc_amd.h).
//
// Around the batched LoMPC solve, every price iteration of PriceSolver.compute_optimal_prices
// (price_solver.py:79-174) runs two small r-variable problems that are NOT per EV:
//   * the price-gradient step (price_solver.py:216-246): min_{x>=0} x'Px + q'x with
//       P = Dphi(w) A_bar^-1 Dphi(w)' / (2m) + eps_reg I,  q = -2 P lmbd - (phi(w) - phi(w_ref)),
//     which the reference hands to CVXPY/Clarabel as sum_squares(chol(P)' x) + q'x (:257-270);
//   * the price regularization LP (price_regularizer.py:68-85, called at price_solver.py:248-255):
//       min c'x  s.t.  A x = b,  x >= 0   with A = Dphi(w)', b = Dphi(w)' lmbd, c = phi(w).
// Both are solved exactly here on the host core that runs the convergence test, with no
// modelling layer:
//   * Dphi = [theta I; -theta I; 2 q_s diag(w)] (lompc.py:179-187): every row of Dphi touches ONE
//     time step, so for any free set F the reduced Hessian 2P_FF = 2 eps I + U_F A_bar^-1 U_F' / m
//     has U_F'U_F diagonal.  Woodbury turns each reduced solve into one solve with
//     G = 2 eps m A_bar + diag(d_F), and A_bar = A'A + kappa I makes every such matrix
//     A' (tridiagonal) A: O(N) per solve (TriSolve) instead of an N x N Cholesky.  Primal-dual active-set
//     (PDAS) iterations from the previous free set, a finite primal active-set method as the
//     fallback; the result is KKT-certified (LOMPC_ERR_NOT_CONVERGED otherwise).
//   * an LP whose every column touches one row separates into one-row LPs; the optimum of each is
//     the column with the smallest cost per unit of right-hand side (lompc_lp_separable).
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <vector>

#include "lompc_dense.hpp"
#include "../../include/lompc_amd.h"

namespace {

// Solves with c A'A + diag(E) (A = tril(ones), c > 0, E >= 0) in O(N): since A^-1 is the
// difference operator, c A'A + E = A' T A with T = c I + A^-T E A^-1 TRIDIAGONAL (diagonal
// c + E_t + E_{t+1}, off-diagonal -E_{t+1}); x = A^-1 T^-1 A^-T b by two differences and one
// tridiagonal LDL' solve (SPD: c > 0).
struct TriSolve {
  int N = 0;
  std::vector<double> d, l;  // LDL' of T: inverse pivots, sub-diagonal multipliers
  bool factor(int N_, double c, const double* E) {
    N = N_;
    d.resize(N);
    l.resize(N);
    for (int t = 0; t < N; ++t) {
      const double En = t + 1 < N ? E[t + 1] : 0.0;
      double a = c + E[t] + En;
      if (t > 0) a += l[t - 1] * E[t];  // - l_{t-1}^2 p_{t-1} with l_{t-1} = -E_t / p_{t-1}
      if (!(a > 0.0)) return false;
      d[t] = 1.0 / a;
      l[t] = -En * d[t];
    }
    return true;
  }
  void solve(double* x) const {  // in place: x <- (c A'A + E)^-1 x
    for (int t = 0; t + 1 < N; ++t) x[t] -= x[t + 1];   // A^-T
    for (int t = 1; t < N; ++t) x[t] -= l[t - 1] * x[t - 1];
    for (int t = 0; t < N; ++t) x[t] *= d[t];
    for (int t = N - 2; t >= 0; --t) x[t] -= l[t] * x[t + 1];
    for (int t = N - 1; t > 0; --t) x[t] -= x[t - 1];    // A^-1
  }
};

// Q = 2P = 2 eps I + U A_bar^-1 U' / m ;  row i of U is u[i] e_{i mod N}'.
// A_bar = A'A + kappa I (price_solver.py:191-192).
struct PriceQP {
  int N = 0, r = 0;
  double eps = 0.0, m = 0.0, kappa = 0.0;
  std::vector<double> u, E, s, v;
  std::vector<int> st;  // stage of row i (i mod N, precomputed: integer division dominated the loops)
  TriSolve Ab, Gf;

  bool init(int N_, int r_, double theta, double w_max, double m_, double kappa_, double eps_, const double* w) {
    N = N_;
    r = r_;
    eps = eps_;
    m = m_;
    kappa = kappa_;
    const double q_s = 3.0 * theta / (4.0 * w_max);  // lompc.py:67
    u.assign(r, 0.0);
    st.resize(r);
    for (int i = 0; i < r; ++i) {
      const int b = i / N, j = i % N;
      st[i] = j;
      u[i] = b == 0 ? theta : (b == 1 ? -theta : 2.0 * q_s * w[j]);  // Dphi rows, lompc.py:179-187
    }
    E.assign(N, kappa);
    s.assign(N, 0.0);
    v.assign(N, 0.0);
    return Ab.factor(N, 1.0, E.data());
  }

  void mulQ(const double* x, double* y) {
    std::fill(v.begin(), v.end(), 0.0);
    for (int i = 0; i < r; ++i) v[st[i]] += u[i] * x[i];
    Ab.solve(v.data());
    const double im = 1.0 / m;
    for (int i = 0; i < r; ++i) y[i] = 2.0 * eps * x[i] + u[i] * v[st[i]] * im;
  }

  // z = argmin 1/2 z'Qz + q'z over {z : z_i = 0 for i not in F}:  Woodbury in the free rows,
  // (a A_bar + D_F) s = U_F'q with a = 2 eps m, D_F = sum of u_i^2 over the free rows of a stage
  bool solveF(const std::vector<char>& F, const double* q, double* z) {
    const double a = 2.0 * eps * m;
    std::fill(s.begin(), s.end(), 0.0);
    for (int j = 0; j < N; ++j) E[j] = a * kappa;
    for (int i = 0; i < r; ++i)
      if (F[i]) {
        const int j = st[i];
        E[j] += u[i] * u[i];
        s[j] += u[i] * q[i];
      }
    if (!Gf.factor(N, a, E.data())) return false;
    Gf.solve(s.data());
    const double h = -0.5 / eps;
    for (int i = 0; i < r; ++i) z[i] = F[i] ? h * (q[i] - u[i] * s[st[i]]) : 0.0;
    return true;
  }
};

// KKT residual of x for min 1/2 x'Qx + q'x, x >= 0 (mu = Qx + q).
double kkt_res(const std::vector<double>& x, const std::vector<double>& mu) {
  double res = 0.0;
  for (size_t i = 0; i < x.size(); ++i) {
    if (x[i] < 0.0) res = std::max(res, -x[i]);
    res = std::max(res, x[i] > 0.0 ? std::fabs(mu[i]) : std::max(0.0, -mu[i]));
  }
  return res;
}

// Exact non-negative QP: PDAS from the warm free set, primal active set as fallback.
int nnqp(PriceQP& P, const double* q, const double* x_warm, double* x_out, double tol, int* iters) {
  const int r = P.r;
  std::vector<char> F(r, 0), Fn(r, 0);
  std::vector<double> z(r), mu(r), x(r, 0.0);
  for (int i = 0; i < r; ++i) F[i] = x_warm && x_warm[i] > 0.0;
  int it = 0;
  // primal-dual active set (Hintermueller-Ito-Kunisch)
  for (int k = 0; k < 64; ++k, ++it) {
    if (!P.solveF(F, q, z.data())) return LOMPC_ERR_NOT_CONVERGED;
    P.mulQ(z.data(), mu.data());
    bool same = true;
    for (int i = 0; i < r; ++i) {
      mu[i] += q[i];
      Fn[i] = F[i] ? (z[i] > 0.0) : (mu[i] < 0.0);
      same = same && (Fn[i] == F[i]);
    }
    if (same) {
      if (kkt_res(z, mu) <= tol) {
        std::copy(z.begin(), z.end(), x_out);
        if (iters) *iters = it + 1;
        return LOMPC_OK;
      }
      break;
    }
    F.swap(Fn);
  }
  // primal active set from x = 0 (feasible): finite for a strictly convex QP
  std::fill(F.begin(), F.end(), 0);
  std::fill(x.begin(), x.end(), 0.0);
  for (int k = 0; k < 64 * r + 64; ++k, ++it) {
    if (!P.solveF(F, q, z.data())) return LOMPC_ERR_NOT_CONVERGED;
    double alpha = 1.0;
    int blk = -1;
    for (int i = 0; i < r; ++i)
      if (F[i] && z[i] <= 0.0) {
        const double a = x[i] / (x[i] - z[i]);
        if (a < alpha) {
          alpha = a;
          blk = i;
        }
      }
    if (blk < 0) {
      x = z;
      P.mulQ(x.data(), mu.data());
      int jmin = -1;
      double best = -tol;
      for (int i = 0; i < r; ++i) {
        mu[i] += q[i];
        if (!F[i] && mu[i] < best) {
          best = mu[i];
          jmin = i;
        }
      }
      if (jmin < 0) {
        if (kkt_res(x, mu) > tol) return LOMPC_ERR_NOT_CONVERGED;
        std::copy(x.begin(), x.end(), x_out);
        if (iters) *iters = it + 1;
        return LOMPC_OK;
      }
      F[jmin] = 1;
    } else {
      for (int i = 0; i < r; ++i)
        if (F[i]) x[i] += alpha * (z[i] - x[i]);
      x[blk] = 0.0;
      F[blk] = 0;
      for (int i = 0; i < r; ++i)
        if (F[i] && x[i] <= 0.0) {
          x[i] = 0.0;
          F[i] = 0;
        }
    }
  }
  return LOMPC_ERR_NOT_CONVERGED;
}

}  // namespace

extern "C" {

int lompc_price_step(int N, int r, double theta, double w_max, double m, double kappa, double eps_reg,
                     const double* w_ref, const double* w, const double* lmbd, double* lmbd_next,
                     double* dual_cost_decrease, int* iterations) {
  if (N < 1 || N > 4096 || (r != 2 * N && r != 3 * N) || !w_ref || !w || !lmbd || !lmbd_next)
    return LOMPC_ERR_INVALID_ARG;
  if (!(theta > 0.0) || !(w_max > 0.0) || !(m > 0.0) || !(kappa >= 0.0) || !(eps_reg > 0.0))
    return LOMPC_ERR_INVALID_ARG;
  PriceQP P;
  if (!P.init(N, r, theta, w_max, m, kappa, eps_reg, w)) return LOMPC_ERR_NOT_CONVERGED;
  const double q_s = 3.0 * theta / (4.0 * w_max);
  // q = -2 P lmbd - (phi(w) - phi(w_ref))[:r]     (price_solver.py:229-235; phi: lompc.py:172-177)
  std::vector<double> q(r), Ql(r);
  P.mulQ(lmbd, Ql.data());
  double qmax = 0.0;
  for (int i = 0; i < r; ++i) {
    const int b = i / N, j = i % N;
    const double dphi = b == 0 ? theta * (w[j] - w_ref[j])
                               : (b == 1 ? -theta * (w[j] - w_ref[j]) : q_s * (w[j] * w[j] - w_ref[j] * w_ref[j]));
    q[i] = -Ql[i] - dphi;
    qmax = std::max(qmax, std::fabs(q[i]));
  }
  // dual_cost = lmbd'P lmbd + q'lmbd  (price_solver.py:236)
  double dual_cost = 0.0;
  for (int i = 0; i < r; ++i) dual_cost += lmbd[i] * (0.5 * Ql[i] + q[i]);
  const double tol = 1e-11 * (1.0 + qmax);
  std::vector<double> x(r);
  const int rc = nnqp(P, q.data(), lmbd, x.data(), tol, iterations);
  if (rc) return rc;
  std::vector<double> Qx(r);
  P.mulQ(x.data(), Qx.data());
  double cost_new = 0.0;  // sum_squares(P_chol x) + q'x  (price_solver.py:270, :244)
  for (int i = 0; i < r; ++i) cost_new += x[i] * (0.5 * Qx[i] + q[i]);
  memcpy(lmbd_next, x.data(), r * sizeof(double));
  if (dual_cost_decrease) *dual_cost_decrease = dual_cost - cost_new;  // price_solver.py:245
  return LOMPC_OK;
}

int lompc_lp_separable(int n_rows, int n_cols, const double* A, const double* b, const double* c, double* x) {
  if (n_rows < 0 || n_cols < 0) return LOMPC_ERR_INVALID_ARG;
  if ((n_cols > 0 && (!c || !x)) || (n_rows > 0 && !b) || ((int64_t)n_rows * n_cols > 0 && !A))
    return LOMPC_ERR_INVALID_ARG;
  // every column must touch at most one row and cost >= 0 (otherwise the LP is not of the
  // separable kind solved here, or is unbounded)
  std::vector<int> row(n_cols, -1);
  for (int i = 0; i < n_cols; ++i) {
    if (!(c[i] >= 0.0)) return LOMPC_ERR_UNSUPPORTED;
    for (int j = 0; j < n_rows; ++j) {
      if (A[(size_t)j * n_cols + i] != 0.0) {
        if (row[i] >= 0) return LOMPC_ERR_UNSUPPORTED;
        row[i] = j;
      }
    }
    x[i] = 0.0;
  }
  for (int j = 0; j < n_rows; ++j) {
    if (b[j] == 0.0) continue;
    // one-row LP: the cheapest column per unit of b_j among those whose coefficient has b_j's
    // sign; ties keep the lowest column index
    int best = -1;
    double best_ratio = INFINITY;
    for (int i = 0; i < n_cols; ++i) {
      if (row[i] != j) continue;
      const double a = A[(size_t)j * n_cols + i];
      if ((a > 0.0) != (b[j] > 0.0)) continue;
      const double ratio = c[i] / std::fabs(a);
      if (ratio < best_ratio) {
        best_ratio = ratio;
        best = i;
      }
    }
    if (best < 0) return LOMPC_ERR_NOT_CONVERGED;  // row j infeasible
    x[best] = b[j] / A[(size_t)j * n_cols + best];
  }
  return LOMPC_OK;
}

// General LP  min c'x  s.t.  A x = b, x >= 0  (the reference's PriceRegularizer accepts any
// such LP, price_regularizer.py:62-85): dense two-phase tableau simplex with Bland's rule (no
// cycling), artificial basis for phase 1, redundant rows dropped.  Sizes here are the price
// vector's (r <= 3N columns, N rows), so a dense tableau is the simple exact choice.
int lompc_lp_solve(int n_rows, int n_cols, const double* A, const double* b, const double* c, double* x,
                   double* objective) {
  if (n_rows < 0 || n_cols < 0) return LOMPC_ERR_INVALID_ARG;
  if ((n_cols > 0 && (!c || !x)) || (n_rows > 0 && !b) || ((int64_t)n_rows * n_cols > 0 && !A))
    return LOMPC_ERR_INVALID_ARG;
  const int m = n_rows, n = n_cols, W = n + m + 1;  // columns: x | artificials | rhs
  std::vector<double> T((size_t)(m + 1) * W, 0.0);
  std::vector<int> basis(m);
  double scale = 1.0;
  for (int i = 0; i < m; ++i) {
    const double sg = b[i] < 0.0 ? -1.0 : 1.0;  // rows with b >= 0
    for (int j = 0; j < n; ++j) {
      T[(size_t)i * W + j] = sg * A[(size_t)i * n + j];
      scale = std::max(scale, std::fabs(A[(size_t)i * n + j]));
    }
    T[(size_t)i * W + n + i] = 1.0;
    T[(size_t)i * W + W - 1] = sg * b[i];
    scale = std::max(scale, std::fabs(b[i]));
    basis[i] = n + i;
  }
  const double eps = 1e-11 * scale;
  std::vector<char> live(m, 1);  // rows not removed as redundant
  double* obj = &T[(size_t)m * W];
  auto pivot = [&](int pr, int pc) {
    double* rp = &T[(size_t)pr * W];
    const double inv = 1.0 / rp[pc];
    for (int j = 0; j < W; ++j) rp[j] *= inv;
    rp[pc] = 1.0;
    for (int i = 0; i <= m; ++i) {
      if (i == pr) continue;
      double* ri = &T[(size_t)i * W];
      const double f = ri[pc];
      if (f == 0.0) continue;
      for (int j = 0; j < W; ++j) ri[j] -= f * rp[j];
      ri[pc] = 0.0;
    }
    basis[pr] = pc;
  };
  // simplex on the objective row `obj` over columns [0, ncol): Bland's rule
  auto run = [&](int ncol) -> int {
    for (int it = 0; it < 50 * (m + n) + 100; ++it) {
      int pc = -1;
      for (int j = 0; j < ncol; ++j)
        if (obj[j] < -eps) {
          pc = j;
          break;
        }
      if (pc < 0) return LOMPC_OK;
      int pr = -1;
      double best = INFINITY;
      for (int i = 0; i < m; ++i) {
        if (!live[i]) continue;
        const double a = T[(size_t)i * W + pc];
        if (a > eps) {
          const double ratio = T[(size_t)i * W + W - 1] / a;
          if (pr < 0 || ratio < best - 1e-15 * best || (ratio <= best && basis[i] < basis[pr])) {
            best = ratio;
            pr = i;
          }
        }
      }
      if (pr < 0) return LOMPC_ERR_UNSUPPORTED;  // unbounded
      pivot(pr, pc);
    }
    return LOMPC_ERR_NOT_CONVERGED;
  };
  // phase 1: minimise the sum of the artificials (objective row = -sum of the rows)
  for (int j = 0; j < W; ++j) {
    double sacc = 0.0;
    for (int i = 0; i < m; ++i) sacc += T[(size_t)i * W + j];
    obj[j] = (j >= n && j < n + m) ? 0.0 : -sacc;
  }
  int rc = run(n + m);
  if (rc == LOMPC_ERR_NOT_CONVERGED) return rc;
  if (-obj[W - 1] > 1e-9 * scale) return LOMPC_ERR_NOT_CONVERGED;  // infeasible
  for (int i = 0; i < m; ++i) {  // drive the artificials out of the basis
    if (basis[i] < n) continue;
    int pc = -1;
    for (int j = 0; j < n; ++j)
      if (std::fabs(T[(size_t)i * W + j]) > eps) {
        pc = j;
        break;
      }
    if (pc >= 0) pivot(i, pc);
    else live[i] = 0;  // redundant row
  }
  // phase 2: the original costs, reduced by the basis
  for (int j = 0; j < W; ++j) obj[j] = j < n ? c[j] : 0.0;
  for (int i = 0; i < m; ++i) {
    if (!live[i]) continue;
    const int k = basis[i];
    const double f = obj[k];
    if (f == 0.0) continue;
    for (int j = 0; j < W; ++j) obj[j] -= f * T[(size_t)i * W + j];
  }
  rc = run(n);
  if (rc != LOMPC_OK) return rc;
  for (int j = 0; j < n; ++j) x[j] = 0.0;
  for (int i = 0; i < m; ++i)
    if (live[i] && basis[i] < n) x[basis[i]] = std::max(0.0, T[(size_t)i * W + W - 1]);
  if (objective) {
    double f = 0.0;
    for (int j = 0; j < n; ++j) f += c[j] * x[j];
    *objective = f;
  }
  return LOMPC_OK;
}

}  // extern "C"
