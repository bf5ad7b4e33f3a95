// lompc_dense.hpp — small dense fp64 kernels for the host-side solvers (price step, BiMPC).
// Row-major n x n matrices; n is a horizon length (<= a few hundred), so plain loops.
#pragma once

#include <cmath>
#include <utility>

namespace lqd {

// In-place lower Cholesky of a (upper triangle untouched); false if not positive definite.
inline bool chol(double* a, int n) {
  for (int j = 0; j < n; ++j) {
    double s = a[j * n + j];
    for (int k = 0; k < j; ++k) s -= a[j * n + k] * a[j * n + k];
    if (!(s > 0.0)) return false;
    const double d = std::sqrt(s);
    a[j * n + j] = d;
    const double inv = 1.0 / d;
    for (int i = j + 1; i < n; ++i) {
      double t = a[i * n + j];
      for (int k = 0; k < j; ++k) t -= a[i * n + k] * a[j * n + k];
      a[i * n + j] = t * inv;
    }
  }
  return true;
}

// Solve (L L') x = b in place with the factor of chol().
inline void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; ++i) {
    double t = b[i];
    for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k];
    b[i] = t / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = b[i];
    for (int k = i + 1; k < n; ++k) t -= L[k * n + i] * b[k];
    b[i] = t / L[i * n + i];
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
