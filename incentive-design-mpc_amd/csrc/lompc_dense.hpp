// lompc_dense.hpp — small dense fp64 kernels for the host-side solvers (price step, BiMPC).
// Row-major n x n matrices; n is a horizon length (<= a few hundred), so plain loops.
#pragma once

#include <cmath>
#include <utility>

namespace lqd {

// sum_k a[k] b[k], four independent accumulators (the single-chain form is bound by the
// add latency, ~4x slower on these short dots)
inline double dot(const double* a, const double* b, int n) {
  double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
  int k = 0;
  for (; k + 4 <= n; k += 4) {
    s0 += a[k] * b[k];
    s1 += a[k + 1] * b[k + 1];
    s2 += a[k + 2] * b[k + 2];
    s3 += a[k + 3] * b[k + 3];
  }
  for (; k < n; ++k) s0 += a[k] * b[k];
  return (s0 + s1) + (s2 + s3);
}

// In-place lower Cholesky of a (upper triangle untouched); false if not positive definite.
inline bool chol(double* a, int n) {
  for (int j = 0; j < n; ++j) {
    const double* aj = a + (size_t)j * n;
    const double s = a[j * n + j] - dot(aj, aj, j);
    if (!(s > 0.0)) return false;
    const double d = std::sqrt(s);
    a[j * n + j] = d;
    const double inv = 1.0 / d;
    for (int i = j + 1; i < n; ++i) a[i * n + j] = (a[i * n + j] - dot(a + (size_t)i * n, aj, j)) * inv;
  }
  return true;
}

// Solve (L L') x = b in place with the factor of chol().
inline void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; ++i) b[i] = (b[i] - dot(L + (size_t)i * n, b, i)) / L[i * n + i];
  for (int i = n - 1; i >= 0; --i) {  // L' x = y, row-oriented updates (contiguous rows of L)
    const double x = b[i] / L[i * n + i];
    b[i] = x;
    const double* Li = L + (size_t)i * n;
    for (int k = 0; k < i; ++k) b[k] -= Li[k] * x;
  }
}

// (L L')^-1 from the factor of chol(), full symmetric n x n into out; work: n*n doubles.
// U = L^-T (row j of U = column j of L^-1, zero before j), then inv_ij = sum_{k >= max(i,j)} U_ik U_jk.
inline void chol_inverse(const double* L, int n, double* out, double* work) {
  double* U = work;
  for (int j = 0; j < n; ++j) {
    double* u = U + (size_t)j * n;
    for (int i = 0; i < j; ++i) u[i] = 0.0;
    u[j] = 1.0 / L[j * n + j];
    for (int i = j + 1; i < n; ++i) u[i] = -dot(L + (size_t)i * n + j, u + j, i - j) / L[i * n + i];
  }
  for (int i = 0; i < n; ++i)
    for (int j = i; j < n; ++j) {
      const double v = dot(U + (size_t)i * n + j, U + (size_t)j * n + j, n - j);
      out[i * n + j] = v;
      out[j * n + i] = v;
    }
}

// In-place LU with partial pivoting; false if singular.
inline bool lu(double* a, int n, int* piv) {
  for (int j = 0; j < n; ++j) {
    int p = j;
    double best = std::fabs(a[j * n + j]);
    for (int i = j + 1; i < n; ++i)
      if (std::fabs(a[i * n + j]) > best) {
        best = std::fabs(a[i * n + j]);
        p = i;
      }
    piv[j] = p;
    if (!(best > 0.0)) return false;
    if (p != j)
      for (int k = 0; k < n; ++k) std::swap(a[j * n + k], a[p * n + k]);
    const double inv = 1.0 / a[j * n + j];
    for (int i = j + 1; i < n; ++i) {
      const double f = a[i * n + j] * inv;
      a[i * n + j] = f;
      if (f != 0.0)
        for (int k = j + 1; k < n; ++k) a[i * n + k] -= f * a[j * n + k];
    }
  }
  return true;
}

inline void lu_solve(const double* a, int n, const int* piv, double* b) {
  for (int j = 0; j < n; ++j)
    if (piv[j] != j) std::swap(b[j], b[piv[j]]);
  for (int i = 0; i < n; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= a[i * n + k] * b[k];
    b[i] = t;
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
    for (int k = i + 1; k < n; ++k) t -= a[i * n + k] * b[k];
    b[i] = t / a[i * n + i];
  }
}

}  // namespace lqd
