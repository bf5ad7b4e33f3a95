// lompc_bimpc.cpp — host interior-point solver of the BiMPC team-optimal planner
// (C-ABI in include/lompc_amd.h).
//
// Replaces the CVXPY/Clarabel conic solve of BiMPC.solve_bimpc (bimpc.py:267-292): ONE problem
// per time step over P partitions (not per EV):
//   variables  W_s, W_l in R^{P x N}, 0 <= W <= w_max            (bimpc.py:143-144, :182-183)
//              u_g in R^N, 0 <= u_g <= u_g_max                     (:145, :185-186)
//   cost       c_g sum_t u_g,t^1.7                                  (:220-221)
//            + delta sum_{k, t} omega_kt ((A W_k)_t - g_k)^2        (:223-265; k = (type, partition))
//   coupling   v = u_g - demand - theta_s Mp_s'W_s - theta_l Mp_l'W_l          (:189-194)
//              -u_b_max + d_e e1 <= v <= u_b_max - d_e e1                       (:195-203)
//              d_e <= x0 1 + A v <= x_max - d_e,  d_e = theta_s Mp_s'beta_s + theta_l Mp_l'beta_l  (:205-218)
// The problem is smooth and strictly convex (u^1.7 and A'Omega A > 0 for every cost type with
// omega > 0), so its optimum is unique; Clarabel's answer is that optimum up to its tolerance.
//
// Method: primal-dual interior point (Mehrotra predictor-corrector).  Box rows stay primal
// feasible (slack = distance to the bound), the 4N coupling rows carry explicit slacks.  The
// Newton matrix is
//     M = blockdiag(H_k + D_k, D_u) + L'QL,   H_k = 2 delta A'Omega_k A,  Q = E'D_g E (N x N),
// with L z = u_g + sum_k c_k W_k the aggregate storage input.  It is solved by Woodbury in the
// coupling rows (Newton::factor): tridiagonal block factors (O(N) each, O(N^2) for the explicit
// inverses) and one 2N x 2N Cholesky, O(2P N^2 + N^3) per iteration instead of
// O(((2P+1) N)^3).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <cmath>
#include <vector>

#include "lompc_dense.hpp"
#include "../../include/lompc_amd.h"

namespace {

struct Bimpc {
  int N = 0, P = 0, nb = 0, n = 0, mg = 0;
  int cost_type = 0;
  double delta = 0, c_g = 0, u_g_max = 0, u_b_max = 0, x_max = 0, exp_rate = 1;
  double theta_s = 0, theta_l = 0, w_max_s = 0, w_max_l = 0;
  // per-solve data
  std::vector<double> omega;  // [nb][N] charging weights
  std::vector<double> gk;     // [nb]    charging target
  std::vector<double> ck;     // [nb]    coefficient of W_k in L z
  std::vector<double> ub;     // [n]     upper bounds (lower bounds are 0)
  std::vector<double> h;      // [4N]    coupling right-hand sides
};

// grad / Hessian pieces of f at z
double f_value(const Bimpc& B, const double* z) {
  const int N = B.N;
  double f = 0.0;
  for (int t = 0; t < N; ++t) f += B.c_g * std::pow(z[B.nb * N + t], 1.7);
  double ch = 0.0;
  for (int k = 0; k < B.nb; ++k) {
    double y = 0.0;
    for (int t = 0; t < N; ++t) {
      y += z[k * N + t];
      const double d = y - B.gk[k];
      ch += B.omega[k * N + t] * d * d;
    }
  }
  return f + B.delta * ch;
}

void f_grad(const Bimpc& B, const double* z, double* g) {
  const int N = B.N;
  std::vector<double> r(N);
  for (int k = 0; k < B.nb; ++k) {
    double y = 0.0;
    for (int t = 0; t < N; ++t) {
      y += z[k * N + t];
      r[t] = 2.0 * B.delta * B.omega[k * N + t] * (y - B.gk[k]);
    }
    double s = 0.0;  // A' r = suffix sums
    for (int t = N - 1; t >= 0; --t) {
      s += r[t];
      g[k * N + t] = s;
    }
  }
  for (int t = 0; t < N; ++t) {
    const double u = z[B.nb * N + t];
    g[B.nb * N + t] = 1.7 * B.c_g * std::pow(u, 0.7);
  }
}

// L z (N) and L' y (n)
void mulL(const Bimpc& B, const double* z, double* y) {
  const int N = B.N;
  for (int t = 0; t < N; ++t) y[t] = z[B.nb * N + t];
  for (int k = 0; k < B.nb; ++k)
    if (B.ck[k] != 0.0)
      for (int t = 0; t < N; ++t) y[t] += B.ck[k] * z[k * N + t];
}
void mulLt(const Bimpc& B, const double* y, double* z) {
  const int N = B.N;
  for (int k = 0; k < B.nb; ++k)
    for (int t = 0; t < N; ++t) z[k * N + t] = B.ck[k] * y[t];
  for (int t = 0; t < N; ++t) z[B.nb * N + t] = y[t];
}
// E y (4N) with E = [-I; I; -A; A];  E' v (N)
void mulE(int N, const double* y, double* out) {
  double c = 0.0;
  for (int t = 0; t < N; ++t) {
    c += y[t];
    out[t] = -y[t];
    out[N + t] = y[t];
    out[2 * N + t] = -c;
    out[3 * N + t] = c;
  }
}
void mulEt(int N, const double* v, double* out) {
  double s = 0.0;
  for (int t = N - 1; t >= 0; --t) {
    s += v[3 * N + t] - v[2 * N + t];
    out[t] = v[N + t] - v[t] + s;
  }
}

// Persistent host worker pool for the independent per-block work of the Newton system
// (2P blocks of N x N factorizations / solves).  Each block writes only its own buffers and
// block results are combined afterwards in block order, so results do not depend on the
// thread count.  LOMPC_HOST_THREADS caps the workers (default min(16, cores)).
class BlockPool {
 public:
  static BlockPool& get() {
    static BlockPool p;
    return p;
  }
  void run(int n, const std::function<void(int)>& fn) {
    if (workers_.empty() || n <= 1) {
      for (int i = 0; i < n; ++i) fn(i);
      return;
    }
    std::lock_guard<std::mutex> call(call_mu_);  // one parallel region at a time
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      next_.store(0);
      busy_.store((int)workers_.size());
      gen_.fetch_add(1, std::memory_order_release);
    }
    cv_.notify_all();
    drain();
    while (busy_.load(std::memory_order_acquire) != 0) std::this_thread::yield();
    fn_ = nullptr;
  }
  ~BlockPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_.store(true);
      gen_.fetch_add(1);
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  BlockPool() {
    int nt = (int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()));
    if (const char* e = getenv("LOMPC_HOST_THREADS")) nt = std::max(1, atoi(e));
    for (int i = 1; i < nt; ++i) workers_.emplace_back([this] { loop(); });
  }
  void drain() {
    for (int i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
  }
  // workers spin briefly on the generation counter (a region follows the previous one within
  // microseconds inside a solve) and sleep on the condition variable otherwise
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      bool got = false;
      for (int spin = 0; spin < 20000 && !got; ++spin) {
        got = gen_.load(std::memory_order_acquire) != seen;
        if (!got) std::this_thread::yield();
      }
      if (!got) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load() != seen; });
      }
      seen = gen_.load(std::memory_order_acquire);
      if (stop_.load()) return;
      drain();
      busy_.fetch_sub(1, std::memory_order_acq_rel);
    }
  }
  std::vector<std::thread> workers_;
  std::mutex mu_, call_mu_;
  std::condition_variable cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0;
  std::atomic<int> next_{0}, busy_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<bool> stop_{false};
};

// In-place Cholesky W = U'U of the 2N x 2N coupling matrix (row-major; U in the upper triangle,
// the lower one not read), right-looking in panels of 4 rows: row j of U is contiguous, so the
// panel's rows are scaled and updated along rows, and every trailing row then takes ONE rank-4
// update from the panel — four FMAs per element loaded and stored instead of one, every loop
// contiguous (AVX2 / FMA along the row), n^3 / 6 FMAs in all.
static bool chol_upper(double* a, int m) {
  for (int j0 = 0; j0 < m; j0 += 4) {
    const int je = std::min(m, j0 + 4);
    for (int j = j0; j < je; ++j) {  // the panel's rows: U_j = a_j / sqrt(a_jj); later panel rows updated
      double* aj = a + (size_t)j * m;
      const double s = aj[j];
      if (!(s > 0.0)) return false;
      const double d = std::sqrt(s), inv = 1.0 / d;
      aj[j] = d;
      for (int k = j + 1; k < m; ++k) aj[k] *= inv;
      for (int i = j + 1; i < je; ++i) {
        double* ai = a + (size_t)i * m;
        const double u = aj[i];
        for (int k = i; k < m; ++k) ai[k] -= u * aj[k];
      }
    }
    const int jb = je - j0;
    if (je >= m) break;
    const double* p0 = a + (size_t)j0 * m;  // the panel's rows of U
    for (int i = je; i < m; ++i) {  // trailing rows: a_ik -= sum_q U_qi U_qk, k >= i
      double* ai = a + (size_t)i * m;
      if (jb == 4) {
        const double* p1 = p0 + m;
        const double* p2 = p1 + m;
        const double* p3 = p2 + m;
        const double u0 = p0[i], u1 = p1[i], u2 = p2[i], u3 = p3[i];
        for (int k = i; k < m; ++k) ai[k] -= (u0 * p0[k] + u1 * p1[k]) + (u2 * p2[k] + u3 * p3[k]);
      } else {
        for (int q = 0; q < jb; ++q) {
          const double* pq = p0 + (size_t)q * m;
          const double u = pq[i];
          for (int k = i; k < m; ++k) ai[k] -= u * pq[k];
        }
      }
    }
  }
  return true;
}

// U'U x = b in place with the factor of chol_upper: U'y = b by row updates (row k of U scatters
// y_k into the later entries), then U x = y by row dots — every access contiguous
static void chol_upper_solve(const double* U, int m, double* b) {
  for (int k = 0; k < m; ++k) {
    const double* uk = U + (size_t)k * m;
    const double y = b[k] / uk[k];
    b[k] = y;
    for (int i = k + 1; i < m; ++i) b[i] -= uk[i] * y;
  }
  for (int i = m - 1; i >= 0; --i) {
    const double* ui = U + (size_t)i * m;
    b[i] = (b[i] - lqd::dot(ui + i + 1, b + i + 1, m - i - 1)) / ui[i];
  }
}

// iterative refinement of a Newton solve runs while its residual exceeds this fraction of the
// right-hand side (1e-12 before round 6: the passes between 1e-12 and 1e-10 changed no iteration count)
#ifndef LQ_BIMPC_REFINE_TOL
#define LQ_BIMPC_REFINE_TOL 1e-10
#endif

struct Newton {
  int N = 0, nb = 0, n = 0;
  std::vector<double> Du;   // [N]
  std::vector<double> Q;    // [N*N]
  std::vector<double> W;    // [2N*2N] D2^-1 + F T F' = U'U (U upper, row-major)
  std::vector<double> ck;
  std::vector<double> S;    // [N*N] sum_k c_k^2 T_k^-1 (H_k^-1 = A^-1 T_k^-1 A^-T)
  std::vector<double> Lf, Df, Di;  // [N][nb] LDL' factors of the T_k (Di = 1 / Df), stage-major (hb_solve)
  std::vector<double> row, dd, rho, pl, pd;  // factor() scratch
  mutable std::vector<double> hb_tmp;
  mutable std::vector<double> sv_r, sv_c, sv_trial;                                  // solve()
  mutable std::vector<double> sr_t1, sr_y, sr_fy, sr_g, sr_tmp;                      // solve_reg()
  mutable std::vector<double> ap_Lx, ap_Qy, ap_tmp, ap_acc, ap_rk;                  // apply()

  // factor M for the current iterate; dbox: [n] box barrier diagonal, dg: [4N] coupling D_g.
  //
  // Block k: H_k = 2 delta A'Omega_k A + D_k = A' (Omega'_k + A^-T D_k A^-1) A with A^-1 the
  // difference operator, so the middle factor T_k is TRIDIAGONAL (diagonal Omega'_t + D_t +
  // D_{t+1}, off-diagonal -D_{t+1}): an O(N) LDL' and H_k^-1 = A^-1 T_k^-1 A^-T in O(N^2),
  // instead of a dense Cholesky and inverse (O(N^3)) per block.
  //
  // Coupling rows: the 4N rows come in +/- pairs on the same linear forms (v_t and (A v)_t), so
  // E'D_g E = F'D_2 F with F = [I; A] and D_2 = the pairwise sums of D_g: the Woodbury matrix
  // is W = D_2^-1 + F T F' (2N x 2N) — the same Newton step as the 4N form at 1/8 of its
  // Cholesky.  An active row (D_g -> inf) keeps F T F'; inactive rows become a large diagonal.
  bool factor(const Bimpc& B, const double* z, const double* dbox, const double* dg) {
#ifdef LQ_BIMPC_PROF
    const double tf_start = nowus();
#endif
    N = B.N;
    nb = B.nb;
    n = B.n;
    ck = B.ck;
    Lf.resize((size_t)nb * N);
    Df.resize((size_t)nb * N);
    Di.resize((size_t)nb * N);
    S.assign((size_t)N * N, 0.0);
    row.resize(N);
    dd.resize(N);
    // LDL' of every block's tridiagonal T_k at once, stage-major (stage t of all blocks is one
    // vector operation: the blocks' independent recurrences overlap instead of 2P latency chains):
    // diag a_t, sub-diagonal c_t = -D_{t+1} (rows t+1, t).  Static regularisation rho_k (the EXP
    // weights 5^(t-N+1) leave early steps with almost no curvature; iterative refinement against the
    // exact matrix removes its bias)
    rho.resize(nb);
    pl.assign(nb, 0.0);
    pd.assign(nb, 0.0);
    for (int k = 0; k < nb; ++k) {
      double s = 0.0;
      for (int t = 0; t < N; ++t) s += B.omega[k * N + t];
      rho[k] = 1e-11 * (1.0 + 2.0 * B.delta * s);  // relative to the charging curvature
    }
    bool okk = true;
    for (int t = 0; t < N; ++t) {
      double* dft = &Df[(size_t)t * nb];
      double* dit = &Di[(size_t)t * nb];
      double* lft = &Lf[(size_t)t * nb];
      for (int k = 0; k < nb; ++k) {
        const double Dt = dbox[k * N + t] + rho[k];
        const double Dn = t + 1 < N ? dbox[k * N + t + 1] + rho[k] : 0.0;
        const double a = 2.0 * B.delta * B.omega[k * N + t] + Dt + Dn - pl[k] * pl[k] * pd[k];  // (t = 0: pl = 0)
        okk = okk && a > 0.0;
        const double ia = 1.0 / a;  // (one division per stage)
        const double l = t + 1 < N ? -Dn * ia : 0.0;  // L_{t+1,t}
        dft[k] = a;
        dit[k] = ia;
        lft[k] = l;
        pl[k] = l;
        pd[k] = a;
      }
    }
    if (!okk) return false;
    // S = sum_k c_k^2 T_k^-1 (upper triangle), block by block in block order; T_k^-1 row by row from
    // the LDL' factors: X_jj = 1/d_j + l_j^2 X_{j+1,j+1} and, right of the diagonal, row i = -l_i x
    // row i+1 (L'X = D^-1 L^-1 is lower triangular) — ONE row buffer per block, scaled in place and
    // added into S (no N x N inverse per block is stored)
    for (int k = 0; k < nb; ++k) {
      if (ck[k] == 0.0) continue;
      const double c2 = ck[k] * ck[k];
      double* r = row.data();
      r[N - 1] = Di[(size_t)(N - 1) * nb + k];
      S[(size_t)(N - 1) * N + N - 1] += c2 * r[N - 1];
      for (int i = N - 2; i >= 0; --i) {
        const double li = Lf[(size_t)i * nb + k];
        const double diag = Di[(size_t)i * nb + k] + li * li * r[i + 1];  // (Di: 1 / d)
        for (int j = i + 1; j < N; ++j) r[j] *= -li;
        r[i] = diag;
        double* si = &S[(size_t)i * N];
        for (int j = i; j < N; ++j) si[j] += c2 * r[j];
      }
    }
#ifdef LQ_BIMPC_PROF
    double tq = nowus();
    t_fx += tq - tf_start;
#endif
    for (int i = 1; i < N; ++i)  // lower triangle by symmetry
      for (int j = 0; j < i; ++j) S[(size_t)i * N + j] = S[(size_t)j * N + i];
    Du.assign(N, 0.0);
    for (int t = 0; t < N; ++t) {
      const double u = z[nb * N + t];
      Du[t] = 1.19 * B.c_g * std::pow(u, -0.3) + dbox[nb * N + t];  // f'' of c_g u^1.7
      if (!(Du[t] > 0.0)) return false;
    }
    // Q = E' D_g E = diag(d0 + d1) + A' diag(d2 + d3) A  (apply() uses the exact matrix)
    Q.assign((size_t)N * N, 0.0);
    {
      double s = 0.0;
      std::vector<double>& suf = row;
      for (int t = N - 1; t >= 0; --t) {
        s += dg[2 * N + t] + dg[3 * N + t];
        suf[t] = s;
      }
      for (int i = 0; i < N; ++i) {
        double* qi = &Q[(size_t)i * N];
        for (int j = 0; j < i; ++j) qi[j] = suf[i];
        for (int j = i; j < N; ++j) qi[j] = suf[j];
        qi[i] += dg[i] + dg[N + i];
      }
    }
    // W = D_2^-1 + F T F' with F = [I; A] and T = A^-1 S A^-T + D^-1 (D = Du, the u_g block):
    //   T A'   = A^-1 S + D^-1 A'     (A^-1: differences down the columns; (D^-1 A')_ij = 1/Du_i, j >= i)
    //   A T A' = S + A D^-1 A'       ((A D^-1 A')_ij = sum_{u <= min(i, j)} 1/Du_u)
    // straight from S: no prefix sums of differences (the same matrix, fewer roundings)
    const int m = 2 * N;
    W.assign((size_t)m * m, 0.0);
    std::vector<double>& cum = dd;  // cumulative 1/Du
    {
      double c = 0.0;
      for (int t = 0; t < N; ++t) cum[t] = (c += 1.0 / Du[t]);
    }
    for (int i = 0; i < N; ++i) {
      const double* si = &S[(size_t)i * N];
      const double* sp = i ? si - N : nullptr;
      double* w1 = &W[(size_t)i * m];       // row i:     [T | T A']
      double* w2 = &W[(size_t)(N + i) * m];  // row N + i: [A T | A T A']
      const double du = 1.0 / Du[i];
      for (int j = 0; j < N; ++j) {
        const double m0 = si[j] - (sp ? sp[j] : 0.0);  // (A^-1 S)_ij
        w1[N + j] = m0 + (j >= i ? du : 0.0);
        w2[N + j] = si[j] + cum[std::min(i, j)];
      }
      for (int j = 0; j < N; ++j) {  // T_ij = (A^-1 S)_ij - (A^-1 S)_i(j-1), + 1/Du on the diagonal
        const double m0 = si[j] - (sp ? sp[j] : 0.0);
        const double m1 = j ? si[j - 1] - (sp ? sp[j - 1] : 0.0) : 0.0;
        w1[j] = m0 - m1 + (j == i ? du : 0.0);
      }
    }
    for (int i = 0; i < N; ++i)  // A T = (T A')'
      for (int j = 0; j < N; ++j) W[(size_t)(N + i) * m + j] = W[(size_t)j * m + N + i];
    for (int t = 0; t < N; ++t) {
      W[(size_t)t * m + t] += 1.0 / (dg[t] + dg[N + t]);
      W[(size_t)(N + t) * m + N + t] += 1.0 / (dg[2 * N + t] + dg[3 * N + t]);
    }
#ifdef LQ_BIMPC_PROF
    const double tc = nowus();
    t_fasm += tc - tq;
    const bool okc = chol_upper(W.data(), m);
    t_fch += nowus() - tc;
    return okc;
#else
    return chol_upper(W.data(), m);
#endif
  }

  void hb_solve(double* x) const {  // Hb^-1 in place
    // H_k^-1 x = A^-1 T_k^-1 A^-T x with the tridiagonal LDL' factors: differences and
    // bidiagonal substitutions, O(N) per block; the blocks are interleaved (stage-major) so
    // their independent recurrences overlap instead of running as one long chain
    hb_tmp.resize((size_t)N * nb);
    double* v = hb_tmp.data();  // [t][k]
    for (int k = 0; k < nb; ++k) {
      const double* xk = x + (size_t)k * N;
      for (int t = 0; t < N; ++t) v[(size_t)t * nb + k] = xk[t] - (t + 1 < N ? xk[t + 1] : 0.0);  // A^-T
    }
    for (int t = 1; t < N; ++t) {  // L w = v
      double* vt = v + (size_t)t * nb;
      const double* vp = vt - nb;
      const double* lp = &Lf[(size_t)(t - 1) * nb];
      for (int k = 0; k < nb; ++k) vt[k] -= lp[k] * vp[k];
    }
    for (size_t e = 0; e < (size_t)N * nb; ++e) v[e] *= Di[e];
    for (int t = N - 2; t >= 0; --t) {  // L' u = D^-1 w
      double* vt = v + (size_t)t * nb;
      const double* vn = vt + nb;
      const double* lt = &Lf[(size_t)t * nb];
      for (int k = 0; k < nb; ++k) vt[k] -= lt[k] * vn[k];
    }
    for (int k = 0; k < nb; ++k) {
      double* xk = x + (size_t)k * N;
      for (int t = 0; t < N; ++t) xk[t] = v[(size_t)t * nb + k] - (t ? v[(size_t)(t - 1) * nb + k] : 0.0);  // A^-1
    }
    for (int t = 0; t < N; ++t) x[nb * N + t] /= Du[t];
  }

  // y = M x with the exact (unregularised) Newton matrix
  void apply(const Bimpc& B, const double* dbox, const double* x, double* y) const {
    ap_Lx.resize(N);
    ap_Qy.resize(N);
    ap_tmp.resize(n);
    double* Lx = ap_Lx.data();
    double* Qy = ap_Qy.data();
    double* tmp = ap_tmp.data();
    // 2 delta A'Omega A x_k for every block: prefix sums then suffix sums, stage-major (stage t of all
    // blocks together: the blocks' independent recurrences overlap instead of 2P latency chains)
    ap_acc.assign(nb, 0.0);
    ap_rk.resize((size_t)N * nb);
    double* acc = ap_acc.data();
    double* rk = ap_rk.data();  // [t][k]
    const double d2 = 2.0 * B.delta;
    for (int t = 0; t < N; ++t)
      for (int k = 0; k < nb; ++k) {
        acc[k] += x[k * N + t];
        rk[(size_t)t * nb + k] = d2 * B.omega[k * N + t] * acc[k];
      }
    std::fill(acc, acc + nb, 0.0);
    for (int t = N - 1; t >= 0; --t)
      for (int k = 0; k < nb; ++k) {
        acc[k] += rk[(size_t)t * nb + k];
        y[k * N + t] = acc[k] + dbox[k * N + t] * x[k * N + t];
      }
    for (int t = 0; t < N; ++t) y[nb * N + t] = Du[t] * x[nb * N + t];
    mulL(B, x, Lx);
    for (int i = 0; i < N; ++i) Qy[i] = lqd::dot(&Q[(size_t)i * N], Lx, N);
    mulLt(B, Qy, tmp);
    for (int i = 0; i < n; ++i) y[i] += tmp[i];
  }

#ifdef LQ_BIMPC_PROF
  mutable int n_solve = 0, n_reg = 0, n_apply = 0;
  mutable double t_hb = 0, t_chs = 0, t_app = 0, t_fx = 0, t_fasm = 0, t_fch = 0;
  static double nowus() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
#endif
  // M dz = rhs: regularised Schur solve + iterative refinement against apply()
  void solve(const Bimpc& B, const double* dbox, const double* rhs, double* dz, bool refine = true) const {
    // refinement stops as soon as it stops reducing the residual: in the nearly flat directions
    // of the EXP weights it would diverge, and the regularised (proximal) step is kept there
    solve_reg(B, rhs, dz);
    if (!refine) return;
    std::vector<double>& r = sv_r;
    std::vector<double>& c = sv_c;
    std::vector<double>& trial = sv_trial;
    r.resize(n);
    c.resize(n);
    trial.resize(n);
#ifdef LQ_BIMPC_PROF
    ++n_solve;
#endif
    auto resid = [&](const double* x) {
#ifdef LQ_BIMPC_PROF
      ++n_apply;
#endif
#ifdef LQ_BIMPC_PROF
      const double ta = nowus();
#endif
      apply(B, dbox, x, r.data());
#ifdef LQ_BIMPC_PROF
      t_app += nowus() - ta;
#endif
      double nr = 0.0;
      for (int i = 0; i < n; ++i) {
        r[i] = rhs[i] - r[i];
        nr = std::max(nr, std::fabs(r[i]));
      }
      return nr;
    };
    double rn = 0.0;
    for (int i = 0; i < n; ++i) rn = std::max(rn, std::fabs(rhs[i]));
    double best = resid(dz);
#ifdef LQ_BIMPC_PROF
    if (getenv("LQ_BIMPC_RES")) fprintf(stderr, "solve %d: initial residual %.2e of rhs\n", n_solve, best / rn);
#endif
    // a residual 1e-10 of the right-hand side is far below what a Newton direction needs (the
    // early iterations' regularised solves land there: no pass then); the passes matter late, where
    // the exp weights' flat directions leave the regularised solve 1e-9 .. 1e-2 off
    for (int pass = 0; pass < 4 && best > LQ_BIMPC_REFINE_TOL * rn; ++pass) {
      solve_reg(B, r.data(), c.data());
      for (int i = 0; i < n; ++i) trial[i] = dz[i] + c[i];
      const double nr = resid(trial.data());
#ifdef LQ_BIMPC_PROF
      if (getenv("LQ_BIMPC_RES")) fprintf(stderr, "   pass %d: %.2e\n", pass, nr / rn);
#endif
      if (!(nr < 0.5 * best)) break;
      best = nr;
      std::copy(trial.begin(), trial.end(), dz);
    }
  }

  void solve_reg(const Bimpc& B, const double* rhs, double* dz) const {
#ifdef LQ_BIMPC_PROF
    ++n_reg;
#endif
    sr_t1.assign(rhs, rhs + n);
    sr_y.resize(N);
    sr_fy.resize(2 * N);
    sr_g.resize(N);
    sr_tmp.resize(n);
    std::vector<double>&t1 = sr_t1, &y = sr_y, &fy = sr_fy, &g = sr_g, &tmp = sr_tmp;
#ifdef LQ_BIMPC_PROF
    double t0 = nowus();
#endif
    hb_solve(t1.data());
#ifdef LQ_BIMPC_PROF
    t_hb += nowus() - t0;
    t0 = nowus();
#endif
    mulL(B, t1.data(), y.data());
    double acc = 0.0;
    for (int t = 0; t < N; ++t) {  // F y = [y; A y]
      fy[t] = y[t];
      fy[N + t] = (acc += y[t]);
    }
    chol_upper_solve(W.data(), 2 * N, fy.data());
#ifdef LQ_BIMPC_PROF
    t_chs += nowus() - t0;
#endif
    acc = 0.0;
    for (int t = N - 1; t >= 0; --t) {  // F' v = v_0 + A' v_1
      acc += fy[N + t];
      g[t] = fy[t] + acc;
    }
    mulLt(B, g.data(), tmp.data());
#ifdef LQ_BIMPC_PROF
    t0 = nowus();
#endif
    hb_solve(tmp.data());
#ifdef LQ_BIMPC_PROF
    t_hb += nowus() - t0;
#endif
    for (int i = 0; i < n; ++i) dz[i] = t1[i] - tmp[i];
  }
};

double max_step(const std::vector<double>& s, const std::vector<double>& ds) {
  double a = 1.0;
  for (size_t i = 0; i < s.size(); ++i)
    if (ds[i] < 0.0) a = std::min(a, -s[i] / ds[i]);
  return a;
}

// Active-set polish of the interior-point solution (cf. OSQP's solution polishing): the
// constraints whose multiplier exceeds their slack are fixed as equalities, the resulting
// equality-constrained problem is solved by Newton steps (only c_g u^1.7 is nonlinear) through
// the |J| x |J| Schur complement of the per-block reduced Hessians, and the result replaces the
// IPM point only if it is primal feasible and every multiplier has the right sign — then it is
// the exact optimum up to round-off.
static bool g_trace_polish = false;

// Cholesky of the symmetric PSD matrix S (nJ x nJ) in row order; the rows whose pivot is below
// 1e-12 of the largest diagonal are linearly dependent on earlier rows: remove them from J.
// Returns true when J changed.
static bool prune_dependent(const std::vector<double>& S, int nJ, std::vector<int>& J) {
  std::vector<double> L(S);
  std::vector<char> drop(nJ, 0);
  double dmax = 0.0;
  for (int a = 0; a < nJ; ++a) dmax = std::max(dmax, S[(size_t)a * nJ + a]);
  const double tol = 1e-12 * dmax;
  bool any = false;
  for (int j = 0; j < nJ; ++j) {
    double d = L[(size_t)j * nJ + j];
    for (int k = 0; k < j; ++k)
      if (!drop[k]) d -= L[(size_t)j * nJ + k] * L[(size_t)j * nJ + k];
    if (!(d > tol)) {
      drop[j] = 1;
      any = true;
      continue;
    }
    const double r = std::sqrt(d);
    L[(size_t)j * nJ + j] = r;
    for (int i = j + 1; i < nJ; ++i) {
      double t = L[(size_t)i * nJ + j];
      for (int k = 0; k < j; ++k)
        if (!drop[k]) t -= L[(size_t)i * nJ + k] * L[(size_t)j * nJ + k];
      L[(size_t)i * nJ + j] = t / r;
    }
  }
  if (!any) return false;
  std::vector<int> Jn;
  for (int a = 0; a < nJ; ++a)
    if (!drop[a]) Jn.push_back(J[a]);
  J.swap(Jn);
  return true;
}
#define PFAIL(msg) do { if (g_trace_polish) fprintf(stderr, "polish: %s\n", msg); return false; } while (0)
bool polish(const Bimpc& B, std::vector<double>& z, std::vector<double>& llo, std::vector<double>& lhi,
            std::vector<double>& lg, const std::vector<double>& sg) {
  const int N = B.N, nb = B.nb, n = B.n, mg = B.mg;
  std::vector<int> fix(n, 0);  // -1 at the lower bound, +1 at the upper bound, 0 free
  for (int i = 0; i < n; ++i) {
    if (llo[i] > z[i])
      fix[i] = -1;
    else if (lhi[i] > B.ub[i] - z[i])
      fix[i] = +1;
  }
  std::vector<int> J;
  for (int j = 0; j < mg; ++j)
    if (lg[j] > sg[j]) J.push_back(j);
  std::vector<double> zp(z);
  std::vector<double> Ej, nu, g(n), Lz(N), ELz(mg), S, rhs;
  std::vector<int> piv;
  int nJ = 0;
  std::vector<double> lgn, tN(N), tn(n), llon, lhin;
  for (int outer = 0;; ++outer) {
  if (outer >= 8) PFAIL("active set");
  bool feasible = false;
  // rounds: a free variable that leaves its box is fixed at that bound, a violated coupling row
  // joins the active set, and the equality-constrained problem is solved again
  for (int round = 0, prunes = 0; round < 6 && !feasible; ++round) {
    bool pruned = false;
    nJ = (int)J.size();
    Ej.assign((size_t)nJ * N, 0.0);  // active rows of E = [-I; I; -A; A]
    for (int a = 0; a < nJ; ++a) {
      const int j = J[a], blk = j / N, t = j % N;
      double* e = &Ej[(size_t)a * N];
      if (blk == 0 || blk == 1)
        e[t] = blk == 0 ? -1.0 : 1.0;
      else
        for (int u = 0; u <= t; ++u) e[u] = blk == 2 ? -1.0 : 1.0;
    }
    nu.assign(nJ, 0.0);
    rhs.assign(nJ, 0.0);
    piv.assign(std::max(nJ, 1), 0);
    for (int i = 0; i < n; ++i) zp[i] = fix[i] < 0 ? 0.0 : (fix[i] > 0 ? B.ub[i] : zp[i]);
    double step = INFINITY;
    for (int newton = 0; newton < 8 && step > 1e-15; ++newton) {
      f_grad(B, zp.data(), g.data());
      mulL(B, zp.data(), Lz.data());
      mulE(N, Lz.data(), ELz.data());
      S.assign((size_t)nJ * nJ, 0.0);
      std::fill(rhs.begin(), rhs.end(), 0.0);
      // per block k (independent, on the host pool): reduced Hessian on the free set F_k,
      // hg = H^-1 g_F, YT = (H^-1 c_k E_F')' and the block's Schur term c_k E_F H^-1 c_k E_F'
      std::vector<std::vector<double>> YT(nb + 1), hg(nb + 1), Sk(nb + 1), rk(nb + 1);
      std::vector<std::vector<int>> F(nb + 1);
      std::vector<int> bad(nb + 1, 0);  // 1: u <= 0, 2: chol
      BlockPool::get().run(nb + 1, [&](int k) {
        for (int t = 0; t < N; ++t)
          if (!fix[k * N + t]) F[k].push_back(t);
        const int m = (int)F[k].size();
        if (!m) return;
        const double ck = k < nb ? B.ck[k] : 1.0;
        std::vector<double> H((size_t)m * m, 0.0), EF((size_t)nJ * m);
        if (k < nb) {
          std::vector<double> suf(N);
          double acc = 0.0;
          for (int t = N - 1; t >= 0; --t) {
            acc += B.omega[k * N + t];
            suf[t] = 2.0 * B.delta * acc;
          }
          for (int a = 0; a < m; ++a)
            for (int b = 0; b < m; ++b) H[a * m + b] = suf[std::max(F[k][a], F[k][b])];
        } else {
          for (int a = 0; a < m; ++a) {
            const double u = zp[nb * N + F[k][a]];
            if (!(u > 0.0)) {
              bad[k] = 1;
              return;
            }
            H[a * m + a] = 1.19 * B.c_g * std::pow(u, -0.3);
          }
        }
        if (!lqd::chol(H.data(), m)) {
          bad[k] = 2;
          return;
        }
        hg[k].resize(m);
        for (int a = 0; a < m; ++a) hg[k][a] = g[k * N + F[k][a]];
        lqd::chol_solve(H.data(), m, hg[k].data());
        for (int q = 0; q < nJ; ++q)
          for (int a = 0; a < m; ++a) EF[(size_t)q * m + a] = ck * Ej[(size_t)q * N + F[k][a]];
        YT[k].assign((size_t)nJ * m, 0.0);
        for (int q = 0; q < nJ; ++q) {
          double* y = &YT[k][(size_t)q * m];
          std::copy(&EF[(size_t)q * m], &EF[(size_t)q * m] + m, y);
          lqd::chol_solve(H.data(), m, y);
        }
        Sk[k].assign((size_t)nJ * nJ, 0.0);
        rk[k].assign(nJ, 0.0);
        for (int p = 0; p < nJ; ++p) {
          rk[k][p] = lqd::dot(&EF[(size_t)p * m], hg[k].data(), m);
          for (int q = p; q < nJ; ++q) {  // symmetric
            const double v = lqd::dot(&EF[(size_t)p * m], &YT[k][(size_t)q * m], m);
            Sk[k][(size_t)p * nJ + q] = v;
            Sk[k][(size_t)q * nJ + p] = v;
          }
        }
      });
      for (int k = 0; k <= nb; ++k) {
        if (bad[k] == 1) PFAIL("u <= 0");
        if (bad[k] == 2) PFAIL("chol");
      }
      for (int k = 0; k <= nb; ++k) {  // block order: independent of the thread count
        if (Sk[k].empty()) continue;
        for (size_t e = 0; e < S.size(); ++e) S[e] += Sk[k][e];
        for (int p = 0; p < nJ; ++p) rhs[p] += rk[k][p];
      }
      // degenerate vertex: an active row that is (numerically) a combination of earlier ones —
      // e.g. one touching only fixed variables — gives a zero pivot of the PSD Schur matrix;
      // drop it (its constraint is implied by the others) and solve again
      if (nJ && prune_dependent(S, nJ, J)) {
        pruned = true;
        break;
      }
      // H dz + C' nu = -g, C dz = h_J - C z  =>  S nu = -(C H^-1 g + h_J - C z)
      for (int a = 0; a < nJ; ++a) nu[a] = -(rhs[a] + B.h[J[a]] - ELz[J[a]]);
      if (nJ) {
        if (!lqd::lu(S.data(), nJ, piv.data())) PFAIL("schur singular");
        lqd::lu_solve(S.data(), nJ, piv.data(), nu.data());
      }
      step = 0.0;
      for (int k = 0; k <= nb; ++k)
        for (int a = 0; a < (int)F[k].size(); ++a) {
          const int m = (int)F[k].size();
          double d = -hg[k][a];
          for (int q = 0; q < nJ; ++q) d -= YT[k][(size_t)q * m + a] * nu[q];
          zp[k * N + F[k][a]] += d;
          step = std::max(step, std::fabs(d));
        }
    }
    if (pruned) {
      if (++prunes > B.mg) PFAIL("prune");
      --round;
      continue;
    }
    // primal feasibility (with repairs for the next round)
    const double ptol = 1e-12;
    feasible = true;
    for (int i = 0; i < n; ++i) {
      if (fix[i]) continue;
      if (zp[i] < -ptol * B.ub[i]) {
        fix[i] = -1;
        feasible = false;
      } else if (zp[i] > B.ub[i] * (1.0 + ptol)) {
        fix[i] = +1;
        feasible = false;
      }
    }
    mulL(B, zp.data(), Lz.data());
    mulE(N, Lz.data(), ELz.data());
    for (int j = 0; j < mg; ++j)
      if (ELz[j] > B.h[j] + ptol * (1.0 + std::fabs(B.h[j])) && std::find(J.begin(), J.end(), j) == J.end()) {
        J.push_back(j);
        feasible = false;
      }
  }
  if (!feasible) PFAIL("primal");
  f_grad(B, zp.data(), g.data());
  double gmax = 0.0;
  for (int i = 0; i < n; ++i) gmax = std::max(gmax, std::fabs(g[i]));
  const double dtol = 1e-9 * (1.0 + gmax);
  // dual signs: a fixed variable or an active row with the wrong-sign multiplier is released
  bool changed = false;
  lgn.assign(mg, 0.0);
  std::vector<int> Jn;
  for (int a = 0; a < nJ; ++a) {
    if (nu[a] < -dtol) {
      changed = true;
      continue;
    }
    Jn.push_back(J[a]);
    lgn[J[a]] = std::max(nu[a], 0.0);
  }
  mulEt(N, lgn.data(), tN.data());
  mulLt(B, tN.data(), tn.data());
  llon.assign(n, 0.0);
  lhin.assign(n, 0.0);
  for (int i = 0; i < n; ++i) {
    const double r = g[i] + tn[i];  // = llo - lhi at a KKT point
    if (fix[i] < 0) {
      if (r < -dtol) {
        fix[i] = 0;
        changed = true;
      }
      llon[i] = std::max(r, 0.0);
    } else if (fix[i] > 0) {
      if (r > dtol) {
        fix[i] = 0;
        changed = true;
      }
      lhin[i] = std::max(-r, 0.0);
    } else if (std::fabs(r) > dtol) {
      if (g_trace_polish) fprintf(stderr, "polish: stationarity %d %g tol %g\n", i, r, dtol);
      return false;
    }
  }
  if (!changed) break;
  J = Jn;
  }  // outer
  z = zp;
  llo = llon;
  lhi = lhin;
  lg = lgn;
  return true;
}

}  // namespace

extern "C" {

// the predictor (affine) direction only sets the centring sigma and the corrector's second-order
// term, so it takes the regularised solve alone; the corrector — the step taken — is refined
// (1: both refined, as before round 6 — the same iteration counts, 1.38 vs 1.15 ms per config-5 solve)
#ifndef LQ_BIMPC_REFINE_PRED
#define LQ_BIMPC_REFINE_PRED 0
#endif

int lompc_bimpc_solve(int N, int P, int charging_cost_type, double delta, double c_g, double u_g_max,
                      double u_b_max, double x_max, double exp_rate, double theta_s, double theta_l,
                      double w_max_s, double w_max_l, const double* Mp_s, const double* Mp_l,
                      const double* beta_s, const double* beta_l, const double* gamma_sm,
                      const double* gamma_lm, double x0, const double* demand, double* w_hat_s,
                      double* w_hat_l, double* u_g, double* duals, double* info) {
  if (N < 1 || N > 4096 || P < 1 || !Mp_s || !Mp_l || !beta_s || !beta_l || !gamma_sm || !gamma_lm || !demand ||
      !w_hat_s || !w_hat_l || !u_g)
    return LOMPC_ERR_INVALID_ARG;
  // bimpc.py:79-84
  if (!(delta >= 0) || !(c_g >= 0) || !(u_g_max >= 0) || !(u_b_max >= 0) || !(x_max >= 0) || !(exp_rate >= 1))
    return LOMPC_ERR_INVALID_ARG;
  if (charging_cost_type < 0 || charging_cost_type > 2) return LOMPC_ERR_INVALID_ARG;
  // strict interior of the boxes is required by the barrier
  if (!(u_g_max > 0) || !(w_max_s > 0) || !(w_max_l > 0) || !(c_g > 0)) return LOMPC_ERR_UNSUPPORTED;
  Bimpc B;
  B.N = N;
  B.P = P;
  B.nb = 2 * P;
  B.n = (2 * P + 1) * N;
  B.mg = 4 * N;
  B.cost_type = charging_cost_type;
  B.delta = delta;
  B.c_g = c_g;
  B.u_g_max = u_g_max;
  B.u_b_max = u_b_max;
  B.x_max = x_max;
  B.exp_rate = exp_rate;
  B.theta_s = theta_s;
  B.theta_l = theta_l;
  B.w_max_s = w_max_s;
  B.w_max_l = w_max_l;
  const int nb = B.nb, n = B.n, mg = B.mg;
  B.omega.assign((size_t)nb * N, 0.0);
  B.gk.assign(nb, 0.0);
  B.ck.assign(nb, 0.0);
  B.ub.assign(n, 0.0);
  for (int k = 0; k < nb; ++k) {
    const bool small = k < P;
    const int p = small ? k : k - P;
    const double Mp = small ? Mp_s[p] : Mp_l[p];
    const double th = small ? theta_s : theta_l;
    B.ck[k] = -th * Mp;                      // bimpc.py:192-193
    B.gk[k] = small ? gamma_sm[p] : gamma_lm[p];
    for (int t = 0; t < N; ++t) {
      double om;
      if (charging_cost_type == 0)
        om = th * th * Mp * Mp;  // weighted, :233-242: theta^2 ||Mp (A w - gamma)||^2
      else if (charging_cost_type == 1)
        om = 1.0;  // unweighted, :244-253
      else
        om = std::pow(exp_rate, (double)(t - N + 1));  // exp-unweighted, :255-265
      B.omega[k * N + t] = om;
      B.ub[k * N + t] = small ? w_max_s : w_max_l;
    }
  }
  for (int t = 0; t < N; ++t) B.ub[nb * N + t] = u_g_max;
  double d_e = 0.0;  // bimpc.py:177-178, :197-199
  for (int p = 0; p < P; ++p) d_e += theta_s * Mp_s[p] * beta_s[p] + theta_l * Mp_l[p] * beta_l[p];
  B.h.assign(mg, 0.0);
  {
    double Ad = 0.0;
    for (int t = 0; t < N; ++t) {
      Ad += demand[t];
      const double e1 = t == 0 ? d_e : 0.0;
      B.h[t] = u_b_max - e1 - demand[t];              // -(Lz)_t <= u_b_max - d_e e1 - dem   (:201)
      B.h[N + t] = u_b_max - e1 + demand[t];          //  (Lz)_t <= u_b_max - d_e e1 + dem   (:203)
      B.h[2 * N + t] = x0 - d_e - Ad;                 // -(A L z)_t <= x0 - d_e - (A dem)_t  (:216)
      B.h[3 * N + t] = x_max - d_e - x0 + Ad;         //  (A L z)_t <= x_max - d_e - x0 + (A dem)_t (:218)
    }
  }
  // ---- interior-point iterations
  std::vector<double> z(n), llo(n), lhi(n), sg(mg), lg(mg);
  for (int i = 0; i < n; ++i) z[i] = 0.5 * B.ub[i];
  std::vector<double> grad(n), Lz(N), ELz(mg), rd(n), rg(mg), tmpN(N), tmpn(n), tmpm(mg);
  f_grad(B, z.data(), grad.data());
  double gmax = 0.0, hmax = 0.0;
  for (int i = 0; i < n; ++i) gmax = std::max(gmax, std::fabs(grad[i]));
  for (int i = 0; i < mg; ++i) hmax = std::max(hmax, std::fabs(B.h[i]));
  double ubmax = 0.0;
  for (int i = 0; i < n; ++i) ubmax = std::max(ubmax, B.ub[i]);
  const double mu0 = 1.0 + 0.1 * gmax * ubmax;
  mulL(B, z.data(), Lz.data());
  mulE(N, Lz.data(), ELz.data());
  for (int i = 0; i < n; ++i) {
    llo[i] = mu0 / z[i];
    lhi[i] = mu0 / (B.ub[i] - z[i]);
  }
  for (int i = 0; i < mg; ++i) {
    sg[i] = std::max(B.h[i] - ELz[i], 0.1 * (1.0 + hmax));
    lg[i] = mu0 / sg[i];
  }
  const int m_tot = 2 * n + mg;
  Newton NW;
  std::vector<double> dbox(n), dgv(mg), rhs(n), dz(n), dsg(mg), dlg(mg), dllo(n), dlhi(n);
  std::vector<double> dz_a(n), dsg_a(mg), dlg_a(mg), dllo_a(n), dlhi_a(n);
  std::vector<double> rclo(n), rchi(n), rcg(mg);
  std::vector<double> iz(n), iu(n), isg(mg);  // 1 / z, 1 / (ub - z), 1 / sg at the current iterate
  int it = 0, status = LOMPC_ERR_NOT_CONVERGED;
  // diagnostic builds only (-DLQ_BIMPC_TRACE / -DLQ_BIMPC_PROF): the iterations / the phases' wall
  // times on stderr
#ifdef LQ_BIMPC_TRACE
  constexpr bool trace = true;
#else
  constexpr bool trace = false;
#endif
#ifdef LQ_BIMPC_PROF
  constexpr bool tprof = true;
#else
  constexpr bool tprof = false;
#endif
  auto now = []() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double t_fac = 0.0, t_dir = 0.0, t_pol = 0.0, t_res = 0.0;
  const double t_all = tprof ? now() : 0.0;
  double pres = 0, dres = 0, gap = 0, fval = 0;
  const int max_iter = (info && info[0] >= 1.0 && info[0] <= 1000.0) ? (int)info[0] : 200;  // info[0] in: cap
  auto residuals = [&]() {
    f_grad(B, z.data(), grad.data());
    mulL(B, z.data(), Lz.data());
    mulE(N, Lz.data(), ELz.data());
    mulEt(N, lg.data(), tmpN.data());
    mulLt(B, tmpN.data(), tmpn.data());
    gmax = 0.0;
    for (int i = 0; i < n; ++i) {
      rd[i] = grad[i] - llo[i] + lhi[i] + tmpn[i];
      gmax = std::max(gmax, std::fabs(grad[i]));
    }
    for (int i = 0; i < mg; ++i) rg[i] = ELz[i] + sg[i] - B.h[i];
    double cs = 0.0;
    for (int i = 0; i < n; ++i) cs += z[i] * llo[i] + (B.ub[i] - z[i]) * lhi[i];
    for (int i = 0; i < mg; ++i) cs += sg[i] * lg[i];
    pres = 0.0;
    dres = 0.0;
    for (int i = 0; i < mg; ++i) pres = std::max(pres, std::fabs(rg[i]));
    for (int i = 0; i < n; ++i) dres = std::max(dres, std::fabs(rd[i]));
    fval = f_value(B, z.data());
    gap = cs;
    return cs / m_tot;
  };
  // direction for complementarity targets rc (s dl + l ds = rc per row)
  auto direction = [&](const std::vector<double>& rlo, const std::vector<double>& rhi, const std::vector<double>& rgc,
                       std::vector<double>& dzo, std::vector<double>& dsgo, std::vector<double>& dlgo,
                       std::vector<double>& dlloo, std::vector<double>& dlhio, bool refine) {
    // rhs = -rd + rlo/s_lo - rhi/s_hi - L'E'[(rgc + lg rg)/sg]
    for (int i = 0; i < mg; ++i) tmpm[i] = (rgc[i] + lg[i] * rg[i]) * isg[i];
    mulEt(N, tmpm.data(), tmpN.data());
    mulLt(B, tmpN.data(), tmpn.data());
    for (int i = 0; i < n; ++i) rhs[i] = -rd[i] + rlo[i] * iz[i] - rhi[i] * iu[i] - tmpn[i];
    NW.solve(B, dbox.data(), rhs.data(), dzo.data(), refine);
    mulL(B, dzo.data(), tmpN.data());
    mulE(N, tmpN.data(), tmpm.data());
    for (int i = 0; i < mg; ++i) {
      dsgo[i] = -rg[i] - tmpm[i];
      dlgo[i] = (rgc[i] - lg[i] * dsgo[i]) * isg[i];
    }
    for (int i = 0; i < n; ++i) {
      dlloo[i] = (rlo[i] - llo[i] * dzo[i]) * iz[i];
      dlhio[i] = (rhi[i] + lhi[i] * dzo[i]) * iu[i];
    }
  };
  // largest steps keeping the primal (z in the boxes, coupling slacks) and the dual variables
  // positive; separate primal / dual lengths
  auto step_len = [&](const std::vector<double>& dzv, const std::vector<double>& dsgv, const std::vector<double>& dlgv,
                      const std::vector<double>& dllov, const std::vector<double>& dlhiv, double& ap, double& ad) {
    ap = 1.0;
    for (int i = 0; i < n; ++i) {
      if (dzv[i] < 0.0) ap = std::min(ap, -z[i] / dzv[i]);
      if (dzv[i] > 0.0) ap = std::min(ap, (B.ub[i] - z[i]) / dzv[i]);
    }
    ap = std::min(ap, max_step(sg, dsgv));
    ad = std::min(max_step(lg, dlgv), std::min(max_step(llo, dllov), max_step(lhi, dlhiv)));
  };
  // best iterate by the worst relative KKT measure; returned when the iteration stalls (the
  // reference accepts Clarabel's "optimal_inaccurate" silently, lompc.py / bimpc.py never check status)
  std::vector<double> zb(n), llob(n), lhib(n), lgb(mg), sgb(mg);
  double best_merit = INFINITY, bpres = 0, bdres = 0, bgap = 0, bf = 0;
  int since_best = 0;
  for (it = 0; it < max_iter; ++it) {
    const double tr0 = tprof ? now() : 0.0;
    const double mu = residuals();
    if (tprof) t_res += now() - tr0;
    double merit = std::max({pres / (1.0 + hmax), dres / (1.0 + gmax), gap / (1.0 + std::fabs(fval))});
    for (int i = 0; i < n && std::isfinite(merit); ++i)
      if (!std::isfinite(z[i]) || !std::isfinite(rd[i])) merit = NAN;
    if (!std::isfinite(merit)) break;
    if (merit < best_merit) {
      best_merit = merit;
      zb = z;
      llob = llo;
      lhib = lhi;
      lgb = lg;
      sgb = sg;
      bpres = pres;
      bdres = dres;
      bgap = gap;
      bf = fval;
      since_best = 0;
    } else if (++since_best >= 15) {
      break;
    } else if (best_merit <= 1e-6) {
      // the merit rose from a best iterate that is already accurate: with the exp weights' flat
      // directions this is where the Newton steps start to break down (the following iterations
      // collapse the step length and blow the residuals up) — the best iterate is
      // returned (and polished when the active set allows), as after a breakdown below
      break;
    }
    // Clarabel's default stopping tolerances (the reference's BIMPC_SOLVER, settings.py:24, called with
    // no settings, bimpc.py:287: tol_feas = tol_gap_rel = 1e-8); the polish below then makes the
    // point exact when the active set is identified.  (1e-10 / 1e-9 here before round 6: the extra
    // iterations sit where the exp weights' flat directions break the Newton steps down.)
    if (pres <= 1e-8 * (1.0 + hmax) && dres <= 1e-8 * (1.0 + gmax) && gap <= 1e-8 * (1.0 + std::fabs(fval))) {
      status = LOMPC_OK;
      break;
    }
    for (int i = 0; i < n; ++i) {
      iz[i] = 1.0 / z[i];
      iu[i] = 1.0 / (B.ub[i] - z[i]);
      dbox[i] = llo[i] * iz[i] + lhi[i] * iu[i];
    }
    for (int i = 0; i < mg; ++i) {
      isg[i] = 1.0 / sg[i];
      dgv[i] = lg[i] * isg[i];
    }
    const double tf0 = tprof ? now() : 0.0;
    if (!NW.factor(B, z.data(), dbox.data(), dgv.data())) break;
    const double tf1 = tprof ? now() : 0.0;
    t_fac += tf1 - tf0;
    // predictor
    for (int i = 0; i < n; ++i) {
      rclo[i] = -z[i] * llo[i];
      rchi[i] = -(B.ub[i] - z[i]) * lhi[i];
    }
    for (int i = 0; i < mg; ++i) rcg[i] = -sg[i] * lg[i];
    direction(rclo, rchi, rcg, dz_a, dsg_a, dlg_a, dllo_a, dlhi_a, LQ_BIMPC_REFINE_PRED);
    double ap = 1.0, ad = 1.0;
    step_len(dz_a, dsg_a, dlg_a, dllo_a, dlhi_a, ap, ad);
    double mu_aff = 0.0;
    for (int i = 0; i < n; ++i) {
      mu_aff += (z[i] + ap * dz_a[i]) * (llo[i] + ad * dllo_a[i]);
      mu_aff += (B.ub[i] - z[i] - ap * dz_a[i]) * (lhi[i] + ad * dlhi_a[i]);
    }
    for (int i = 0; i < mg; ++i) mu_aff += (sg[i] + ap * dsg_a[i]) * (lg[i] + ad * dlg_a[i]);
    mu_aff /= m_tot;
    const double sigma = std::pow(std::min(1.0, mu_aff / mu), 3.0);
    // corrector: target sigma mu, second-order term of the affine step
    for (int i = 0; i < n; ++i) {
      rclo[i] = sigma * mu - z[i] * llo[i] - dz_a[i] * dllo_a[i];
      rchi[i] = sigma * mu - (B.ub[i] - z[i]) * lhi[i] + dz_a[i] * dlhi_a[i];
    }
    for (int i = 0; i < mg; ++i) rcg[i] = sigma * mu - sg[i] * lg[i] - dsg_a[i] * dlg_a[i];
    direction(rclo, rchi, rcg, dz, dsg, dlg, dllo, dlhi, true);
    step_len(dz, dsg, dlg, dllo, dlhi, ap, ad);
    if (tprof) t_dir += now() - tf1;
    const double tau = std::max(0.99, 1.0 - mu);  // fraction to the boundary
    ap = ad = std::min(1.0, tau * std::min(ap, ad));  // one step: the objective is nonlinear
    if (trace)
      fprintf(stderr, "it %3d mu %.3e pres %.3e dres %.3e gap %.3e f %.12g sigma %.3e alpha %.3e merit %.3e gmax %.3e\n", it,
              mu, pres, dres, gap, fval, sigma, ap, merit, gmax);
    if (!std::isfinite(ap) || !std::isfinite(ad) || !std::isfinite(sigma)) break;
    for (int i = 0; i < n; ++i) {
      z[i] += ap * dz[i];
      llo[i] += ad * dllo[i];
      lhi[i] += ad * dlhi[i];
    }
    for (int i = 0; i < mg; ++i) {
      sg[i] += ap * dsg[i];
      lg[i] += ad * dlg[i];
    }
  }
  if (status != LOMPC_OK && std::isfinite(best_merit)) {
    z = zb;
    llo = llob;
    lhi = lhib;
    lg = lgb;
    sg = sgb;
    pres = bpres;
    dres = bdres;
    gap = bgap;
    fval = bf;
    if (best_merit <= 5e-5) status = LOMPC_OK;  // Clarabel's reduced tolerances ("almost solved")
  }
  bool polished = false;
  g_trace_polish = trace;
  // the polish certifies its own result (primal feasibility, multiplier signs, stationarity), so
  // it also runs from the best iterate of a stalled IPM: the late iterations of the exp-weighted
  // cost (weights 5^(t-N+1)) lose Newton accuracy before the gap closes, while the active set is
  // already identified
  const double tp0 = tprof ? now() : 0.0;
  const bool pol_ok = std::isfinite(best_merit) && polish(B, z, llo, lhi, lg, sg);
  if (tprof) t_pol = now() - tp0;
  if (pol_ok) {
    polished = true;
    status = LOMPC_OK;
    residuals();  // report the polished point
  }
  for (int p = 0; p < P; ++p)
    for (int t = 0; t < N; ++t) {
      w_hat_s[p * N + t] = z[p * N + t];
      w_hat_l[p * N + t] = z[(P + p) * N + t];
    }
  for (int t = 0; t < N; ++t) u_g[t] = z[nb * N + t];
  if (tprof)
    fprintf(stderr, "bimpc prof: %d it, total %.0f us: factor %.0f, directions %.0f, residuals %.0f, polish %.0f\n", it,
            now() - t_all, t_fac, t_dir, t_res, t_pol);
#ifdef LQ_BIMPC_PROF
  fprintf(stderr, "bimpc prof: solves %d, regularised solves %d, applies %d; hb_solve %.0f us, mulL+chol_solve %.0f us, apply %.0f us\n",
          NW.n_solve, NW.n_reg, NW.n_apply, NW.t_hb, NW.t_chs, NW.t_app);
  fprintf(stderr, "bimpc prof: factor: blocks %.0f us, assembly %.0f us, Cholesky %.0f us\n", NW.t_fx, NW.t_fasm, NW.t_fch);
#endif
  if (duals) {  // [lower-bound duals (n) | upper-bound duals (n) | coupling duals (4N)]
    memcpy(duals, llo.data(), n * sizeof(double));
    memcpy(duals + n, lhi.data(), n * sizeof(double));
    memcpy(duals + 2 * n, lg.data(), mg * sizeof(double));
  }
  if (info) {  // iterations, objective, primal residual, dual residual, complementarity
    info[0] = (double)it;
    info[1] = fval;
    info[2] = pres;
    info[3] = dres;
    info[4] = gap;
    if (trace) fprintf(stderr, "bimpc: %d iterations, polished %d\n", it, (int)polished);
  }
  return status;
}

}  // extern "C"
