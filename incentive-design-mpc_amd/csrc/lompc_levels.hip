// lompc_levels.hip — the charging station's per-step partition layout on the device.
//
// Reference: ChargingStation._update_indices (chargingstation/charging_station.py:111-116) puts EV i
// in partition p when rng[p] <= y_i <= rng[p+1] (later partitions winning on shared edges), and
// every step each (type, partition) price loop needs its EVs' count / max / min / mean charge level
// (PriceSolver.set_charge_levels, price_solver.py:66-77, via charging_station.py:187-266) and — for
// the batched engine's gamma-sorted loop plans — its EVs in descending charge level.  With every
// level inside [rng[0], rng[P]] (the station's dynamics keep them there: levels only grow, and full
// EVs are redrawn inside the range) partition p is one contiguous run of the levels sorted in
// descending order, so ONE sort gives the layout and the statistics:
//   (1) rocprim's radix sort of (y, index) pairs, descending (stable: ties keep index order);
//   (2) k_lv_bounds: the runs' ends by a 64-way search per boundary (three load rounds for 2^18 EVs);
//   (3) k_lv_partials: per (partition, chunk) partial sums, in a fixed order;
//   (4) k_lv_stats: per partition count / max / min / sum (partials summed in chunk order) and the
//       levels' overall max / min beside rng[0] / rng[P] (the caller's range check: outside it, EVs
//       keep their previous partition and the runs are not the partitions — the caller then takes
//       the index-based path).
// Deterministic: the same levels give the same bits.  lompc_levels_gamma then lays out every
// partition's loop-plan batch (gamma = y_max - y ascending, then its central QP) in one launch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>

#include "../../include/lompc_amd.h"

namespace {

constexpr int LV_CHUNKS = 32;  // partial-sum chunks per partition
constexpr int LV_MAXP = 256;   // partitions at most

// c[p] = #{i : ys[i] >= bounds[p]} for p = 1 .. P-1 in the descending levels (one wave per boundary):
// each round the wave samples 64 evenly spaced positions of the remaining interval and keeps the one
// sub-interval where the predicate flips
__global__ __launch_bounds__(64) void k_lv_bounds(const double* __restrict__ ys, int64_t n,
                                                  const double* __restrict__ bounds, int64_t* __restrict__ cge) {
  const int p = (int)blockIdx.x + 1, lane = (int)threadIdx.x;
  const double v = bounds[p];
  int64_t lo = 0, hi = n;  // answer in [lo, hi]: ys[lo - 1] >= v (or lo = 0), ys[hi] < v (or hi = n)
  while (hi - lo > 64) {
    const int64_t step = (hi - lo + 63) / 64;
    const int64_t i = lo + (int64_t)lane * step;
    const bool ge = i < hi && ys[i] >= v;
    const unsigned long long m = __ballot(ge);
    const int k = __popcll(m);  // samples 0 .. k-1 are >= v (descending)
    const int64_t nlo = k == 0 ? lo : lo + (int64_t)(k - 1) * step + 1;
    const int64_t nhi = lo + (int64_t)k * step < hi ? lo + (int64_t)k * step : hi;
    lo = nlo;
    hi = nhi;
  }
  const int64_t i = lo + lane;
  const bool ge = i < hi && ys[i] >= v;
  const int64_t r = lo + __popcll(__ballot(ge));
  if (lane == 0) cge[p] = r;
}

// partition p = [c[p+1], c[p]) with c[0] = n, c[P] = 0; block (chunk, p) sums its chunk
__global__ __launch_bounds__(256) void k_lv_partials(const double* __restrict__ ys, int64_t n, int P,
                                                     const int64_t* __restrict__ cge, double* __restrict__ part) {
  const int c = (int)blockIdx.x, p = (int)blockIdx.y, t = (int)threadIdx.x;
  const int64_t a = p + 1 < P ? cge[p + 1] : 0, b = p > 0 ? cge[p] : n;
  const int64_t len = b > a ? b - a : 0;
  const int64_t c0 = a + len * c / LV_CHUNKS, c1 = a + len * (c + 1) / LV_CHUNKS;
  double s = 0.0;
  for (int64_t i = c0 + t; i < c1; i += 256) s += ys[i];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  __shared__ double w[4];
  if ((t & 63) == 0) w[t >> 6] = s;
  __syncthreads();
  if (t == 0) part[(size_t)p * LV_CHUNKS + c] = ((w[0] + w[1]) + w[2]) + w[3];
}

// stats [P][4] = (count, max, min, sum) (an empty partition: 0, -inf, +inf, 0), then
// [4] = (ys[0], ys[n-1], bounds[0], bounds[P])
__global__ __launch_bounds__(256) void k_lv_stats(const double* __restrict__ ys, int64_t n, int P,
                                                  const double* __restrict__ bounds, const int64_t* __restrict__ cge,
                                                  const double* __restrict__ part, double* __restrict__ stats) {
  for (int p = (int)threadIdx.x; p < P; p += 256) {
    const int64_t a = p + 1 < P ? cge[p + 1] : 0, b = p > 0 ? cge[p] : n;
    double s = 0.0;
    for (int c = 0; c < LV_CHUNKS; ++c) s += part[(size_t)p * LV_CHUNKS + c];
    const bool any = b > a;
    stats[4 * p + 0] = any ? (double)(b - a) : 0.0;
    stats[4 * p + 1] = any ? ys[a] : -INFINITY;
    stats[4 * p + 2] = any ? ys[b - 1] : INFINITY;
    stats[4 * p + 3] = any ? s : 0.0;
  }
  if (threadIdx.x == 0) {
    stats[4 * P + 0] = ys[0];
    stats[4 * P + 1] = ys[n - 1];
    stats[4 * P + 2] = bounds[0];
    stats[4 * P + 3] = bounds[P];
  }
}

// gam[i + k central] = y_max - ys[i] for element i of storage run k (runs[k] <= i < runs[k + 1]), and with
// `central` each run's central QP gsc[k] right after it, at runs[k + 1] + k
__global__ __launch_bounds__(256) void k_lv_gamma(const double* __restrict__ ys, int64_t n,
                                                  const int64_t* __restrict__ runs, int P, double y_max, int central,
                                                  const double* __restrict__ gsc, double* __restrict__ gam) {
  __shared__ int64_t e[LV_MAXP + 1];
  for (int k = (int)threadIdx.x; k <= P; k += 256) e[k] = runs[k];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    int lo = 0, hi = P;  // the last run with e[lo] <= i (empty runs skipped): e[lo] <= i < e[hi]
    while (hi - lo > 1) {
      const int mid = (lo + hi) >> 1;
      if (e[mid] <= i) lo = mid;
      else hi = mid;
    }
    gam[i + (central ? lo : 0)] = y_max - ys[i];
  }
  if (central && blockIdx.x == 0)
    for (int k = (int)threadIdx.x; k < P; k += 256) gam[e[k + 1] + k] = gsc[k];
}

// The statistics alone, without the sort (lompc_levels_stats, P <= LV_HP): EV i belongs to partition
// p = #{k in 1 .. P-1 : bounds[k] <= y_i} (the sorted runs' rule).  Workgroup b sums its contiguous
// chunk: each thread its strided EVs in registers (one predicated update per partition: no dynamic
// register indexing), then fixed-order wave butterflies and a fixed-order combine of the 4 waves; the
// workgroups' records are then combined by k_lvh_final (one wave per statistic, lane-strided, a fixed
// butterfly).  Deterministic.
constexpr int LV_HP = 16;
constexpr int LV_HBLK = 512;  // workgroups at most

// max / min that propagate NaN (fmax / fmin drop it): the whole-type max y / min y of the statistics
// pass carry a NaN level to the caller, whose range check [rng[0], rng[P]] then fails (a NaN counted
// in partition 0 would otherwise leave the sorted runs and the statistics' counts out of step)
__device__ __forceinline__ double lv_nmax(double a, double b) { return (a != a || b != b) ? NAN : fmax(a, b); }
__device__ __forceinline__ double lv_nmin(double a, double b) { return (a != a || b != b) ? NAN : fmin(a, b); }
__device__ __forceinline__ double lv_comb(int f, double a, double b) {
  return f == 1 ? fmax(a, b) : f == 2 ? fmin(a, b) : f == 4 ? lv_nmax(a, b) : f == 5 ? lv_nmin(a, b) : a + b;
}

__global__ __launch_bounds__(256) void k_lvh_partial(const double* __restrict__ y, int64_t n,
                                                     const double* __restrict__ bounds, int P, int nblk,
                                                     double* __restrict__ part) {
  const int b = (int)blockIdx.x, t = (int)threadIdx.x, lane = t & 63, wv = t >> 6;
  __shared__ double sb[LV_HP];
  if (t < LV_HP) sb[t] = t >= 1 && t < P ? bounds[t] : INFINITY;
  __syncthreads();
  double bd[LV_HP];
#pragma unroll
  for (int k = 0; k < LV_HP; ++k) bd[k] = sb[k];
  double cnt[LV_HP], sum[LV_HP], mx[LV_HP], mn[LV_HP];
#pragma unroll
  for (int k = 0; k < LV_HP; ++k) {
    cnt[k] = 0.0;
    sum[k] = 0.0;
    mx[k] = -INFINITY;
    mn[k] = INFINITY;
  }
  double ymx = -INFINITY, ymn = INFINITY;
  const int64_t c0 = n * b / nblk, c1 = n * (b + 1) / nblk;
  constexpr int U = 4;  // loads in flight per thread: the chunk's memory rounds, not one per element
  for (int64_t i0 = c0 + t; i0 < c1; i0 += 256 * U) {
    double vv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) vv[u] = i0 + 256 * u < c1 ? y[i0 + 256 * u] : NAN;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (!(i0 + 256 * u < c1)) break;
      const double v = vv[u];
      int p = 0;
#pragma unroll
      for (int k = 1; k < LV_HP; ++k) p += bd[k] <= v ? 1 : 0;
#pragma unroll
      for (int k = 0; k < LV_HP; ++k) {
        const bool m = k == p;
        cnt[k] += m ? 1.0 : 0.0;
        sum[k] += m ? v : 0.0;
        mx[k] = m ? fmax(mx[k], v) : mx[k];
        mn[k] = m ? fmin(mn[k], v) : mn[k];
      }
      ymx = lv_nmax(ymx, v);
      ymn = lv_nmin(ymn, v);
    }
  }
  __shared__ double sw[4][4 * LV_HP + 2];
#pragma unroll
  for (int k = 0; k < LV_HP; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      cnt[k] += __shfl_xor(cnt[k], o);
      sum[k] += __shfl_xor(sum[k], o);
      mx[k] = fmax(mx[k], __shfl_xor(mx[k], o));
      mn[k] = fmin(mn[k], __shfl_xor(mn[k], o));
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ymx = lv_nmax(ymx, __shfl_xor(ymx, o));
    ymn = lv_nmin(ymn, __shfl_xor(ymn, o));
  }
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < LV_HP; ++k) {
      sw[wv][4 * k + 0] = cnt[k];
      sw[wv][4 * k + 1] = mx[k];
      sw[wv][4 * k + 2] = mn[k];
      sw[wv][4 * k + 3] = sum[k];
    }
    sw[wv][4 * LV_HP] = ymx;
    sw[wv][4 * LV_HP + 1] = ymn;
  }
  __syncthreads();
  if (t < 4 * LV_HP + 2) {
    // 0 count / 3 sum: add; 1 max; 2 min; 4 / 5: the whole type's max / min (NaN propagated)
    const int f = t < 4 * LV_HP ? (t & 3) : (t == 4 * LV_HP ? 4 : 5);
    double v = sw[0][t];
    for (int w = 1; w < 4; ++w) v = lv_comb(f, v, sw[w][t]);
    part[(size_t)b * (4 * LV_HP + 2) + t] = v;
  }
}

// one wave per statistic t: lane l combines the workgroups' records l, l + 64, ... in order, then a
// fixed butterfly over the lanes (deterministic)
__global__ __launch_bounds__(64) void k_lvh_final(const double* __restrict__ part, int nblk, int P,
                                                  const double* __restrict__ bounds, double* __restrict__ stats) {
  const int t = (int)blockIdx.x, lane = (int)threadIdx.x;
  const int f = t < 4 * LV_HP ? (t & 3) : (t == 4 * LV_HP ? 4 : 5);  // as k_lvh_partial's combine
  const double id = (f == 1 || f == 4) ? -INFINITY : (f == 2 || f == 5) ? INFINITY : 0.0;
  double v = id;
  for (int b = lane; b < nblk; b += 64) v = lv_comb(f, v, part[(size_t)b * (4 * LV_HP + 2) + t]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = lv_comb(f, v, __shfl_xor(v, o));
  if (lane == 0) {
    if (t < 4 * P) stats[t] = v;                                      // per partition (count, max, min, sum)
    else if (t >= 4 * LV_HP) stats[4 * P + (t - 4 * LV_HP)] = v;       // max y, min y
    if (t == 0) {
      stats[4 * P + 2] = bounds[0];
      stats[4 * P + 3] = bounds[P];
    }
  }
}

size_t up256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace

extern "C" int lompc_levels_layout(const double* y, int64_t n, const double* bounds, int P, double* ys, int64_t* perm,
                                   double* stats, void* work, size_t* work_bytes, void* stream) {
  if (!work_bytes || n < 1 || n >= (1ll << 31) || P < 1 || P > LV_MAXP) return LOMPC_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  size_t sort_bytes = 0;
  rocprim::counting_iterator<int64_t> iota(0);
  if (rocprim::radix_sort_pairs_desc(nullptr, sort_bytes, y, ys, iota, perm, (unsigned)n, 0, 64, st) != hipSuccess)
    return LOMPC_ERR_HIP;
  const size_t o_cge = up256(sort_bytes), o_part = o_cge + up256((size_t)(P + 1) * sizeof(int64_t));
  const size_t need = o_part + (size_t)P * LV_CHUNKS * sizeof(double);
  if (!work) {
    *work_bytes = need;
    return LOMPC_OK;
  }
  if (*work_bytes < need || !y || !bounds || !ys || !perm || !stats) return LOMPC_ERR_INVALID_ARG;
  char* wk = static_cast<char*>(work);
  if (rocprim::radix_sort_pairs_desc(wk, sort_bytes, y, ys, iota, perm, (unsigned)n, 0, 64, st) != hipSuccess)
    return LOMPC_ERR_HIP;
  int64_t* cge = reinterpret_cast<int64_t*>(wk + o_cge);
  double* part = reinterpret_cast<double*>(wk + o_part);
  if (P > 1) hipLaunchKernelGGL(k_lv_bounds, dim3((unsigned)(P - 1)), dim3(64), 0, st, ys, n, bounds, cge);
  hipLaunchKernelGGL(k_lv_partials, dim3(LV_CHUNKS, (unsigned)P), dim3(256), 0, st, ys, n, P, cge, part);
  hipLaunchKernelGGL(k_lv_stats, dim3(1), dim3(256), 0, st, ys, n, P, bounds, cge, part, stats);
  return hipGetLastError() == hipSuccess ? LOMPC_OK : LOMPC_ERR_HIP;
}

extern "C" int lompc_levels_gamma(const double* ys, int64_t n, const int64_t* runs, int P, double y_max, int central,
                                  const double* gsc, double* gam, void* stream) {
  if (n < 0 || P < 1 || P > LV_MAXP || !runs || !gam || (n > 0 && !ys) || (central && !gsc)) return LOMPC_ERR_INVALID_ARG;
  const int64_t blocks = std::min<int64_t>(std::max<int64_t>((n + 255) / 256, 1), 2048);
  hipLaunchKernelGGL(k_lv_gamma, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, ys, n, runs, P, y_max,
                     central, gsc, gam);
  return hipGetLastError() == hipSuccess ? LOMPC_OK : LOMPC_ERR_HIP;
}

// The partition statistics of lompc_levels_layout without its sort (P <= 16; more: LOMPC_ERR_UNSUPPORTED).
extern "C" int lompc_levels_stats(const double* y, int64_t n, const double* bounds, int P, double* stats, void* work,
                                  size_t* work_bytes, void* stream) {
  if (!work_bytes || n < 1 || P < 1) return LOMPC_ERR_INVALID_ARG;
  if (P > LV_HP) return LOMPC_ERR_UNSUPPORTED;
  const int nblk = (int)std::min<int64_t>(LV_HBLK, std::max<int64_t>(1, (n + 4095) / 4096));
  const size_t need = (size_t)LV_HBLK * (4 * LV_HP + 2) * sizeof(double);
  if (!work) {
    *work_bytes = need;
    return LOMPC_OK;
  }
  if (*work_bytes < need || !y || !bounds || !stats) return LOMPC_ERR_INVALID_ARG;
  hipStream_t st = (hipStream_t)stream;
  double* part = static_cast<double*>(work);
  hipLaunchKernelGGL(k_lvh_partial, dim3((unsigned)nblk), dim3(256), 0, st, y, n, bounds, P, nblk, part);
  hipLaunchKernelGGL(k_lvh_final, dim3(4 * LV_HP + 2), dim3(64), 0, st, part, nblk, P, bounds, stats);
  return hipGetLastError() == hipSuccess ? LOMPC_OK : LOMPC_ERR_HIP;
}
