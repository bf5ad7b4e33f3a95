// lompc_loop.hip — the price loop of one (EV type, partition), PriceSolver.compute_optimal_prices
// (price_solver.py:106-140), in ONE C-ABI call (lompc_price_loop, include/lompc_amd.h).
//
// Host form (lq_price_loop_host, lompc_plan.hip): per iteration one plan run, one D2H copy, a
// stream sync, the convergence test and the price-gradient QP on the host — a host round trip per
// iteration (~28 us of a ~60 us iteration on the config-5 station, profiles/r03_*).
//
// Device-resident form (here): after every engine call (k_path, k_eval[, RCCL all-gather +
// combine]) one more kernel, k_loop_step — a single wave — runs the convergence test
// (price_solver.py:210-214, 125) and, when not converged, the price-gradient step (:216-246) as a
// wave-parallel exact non-negative QP (lompc_pricewave.hpp), and writes the next prices straight
// into the plan's price buffer.  The host only enqueues engine calls LOMPC_LOOP_AHEAD ahead of
// the device's progress, which k_loop_step publishes in pinned host memory with system-scope
// stores (no copy, no stream sync per iteration); calls enqueued past the convergence find the
// loop's finished flag and return at once.  The enqueue rule depends only on the iteration at
// which the loop finished, so every rank of a sharded plan issues the same collectives.
// Fused form (gamma-sorted sets, one rank, <= LQ_LOOP_G cells per set): the engine call and the
// step are ONE launch, k_loop_iter (lompc_plan.hip) — path, aggregation and step without the two
// kernel boundaries between them.
#include <hip/hip_runtime.h>
#include <string.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "lompc_ctx.hpp"
#include "lompc_loopstep.hpp"

#ifndef LQ_LOOP_PERSIST
#define LQ_LOOP_PERSIST 1  // fused plans: the whole loop as ONE persistent launch (k_loop_run); 0: k_loop_iter per call
#endif

namespace {

// Engine call m of the loop has run: the loop step (lompc_loopstep.hpp) on one wave
__global__ __launch_bounds__(64) void k_loop_step(StepArgs a, int m) {
  if (a.ctl[0]) return;  // finished: a call enqueued ahead of the convergence
  loop_step<false>(a, m, (int)threadIdx.x);
}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

}  // namespace

int lq_price_loop_device(lompc_plan* p, const lompc_price_loop_args* a, double* lmbd, double* w_k, double* dual_cost,
                         double* dec_actual, double* dec_pred, int* iterations, double* errs, hipStream_t st) {
  const int N = a->N, N3 = 3 * N, MI = a->max_iter;
  double* prof = a->prof;
  const double t_start = prof ? now_us() : 0.0;
  double t_issue = 0.0, t_wait = 0.0;
  int rc;
  if (!p->d_loop && (rc = grow(p, reinterpret_cast<char**>(&p->d_loop), LQ_LOOP_BYTES))) return rc;
  if (!p->h_loop)
    HIPCHK(p, hipHostMalloc((void**)&p->h_loop, sizeof(lq_host_loop), hipHostMallocCoherent | hipHostMallocMapped));
  if (MI > p->cap_loop_iter) {
    if (p->h_dec) HIPCHK(p, hipHostFree(p->h_dec));
    p->h_dec = nullptr;
    HIPCHK(p, hipHostMalloc((void**)&p->h_dec, 2 * (size_t)MI * sizeof(double), hipHostMallocCoherent | hipHostMallocMapped));
    p->cap_loop_iter = MI;
  }
  lq_host_loop* d_h = nullptr;
  double* d_dec = nullptr;
  HIPCHK(p, hipHostGetDevicePointer((void**)&d_h, p->h_loop, 0));
  HIPCHK(p, hipHostGetDevicePointer((void**)&d_dec, p->h_dec, 0));
  volatile lq_host_loop* h = p->h_loop;
  // the first prices: staged and copied as in the host loop; the loop state zeroed on the stream
  // (after any call of the previous loop still in flight, which skips)
  double* hin = a->host_in;
  memcpy(hin, lmbd, N3 * sizeof(double));
  memcpy(hin + N3, lmbd, N3 * sizeof(double));
  hin[2 * N3] = hin[2 * N3 + 1] = a->lmbd_r;
  memcpy(hin + 2 * N3 + 2, a->w_ref, N * sizeof(double));
  memcpy(hin + 2 * N3 + 2 + N, a->w_ref, N * sizeof(double));
  const size_t n_in = (size_t)6 * N + 2 + 2 * N;
  HIPCHK(p, hipMemcpyAsync(a->dev_in, hin, n_in * sizeof(double), hipMemcpyHostToDevice, st));
  HIPCHK(p, hipMemsetAsync(p->d_loop, 0, LQ_LOOP_BYTES, st));
  h->progress = 0;
  h->done = 0;
  h->err = 0;
  h->conv_at = -1;
  StepArgs sa{N,        a->r,        MI,       a->tol_avg, a->theta, a->w_max, a->m,
              a->kappa, a->eps_reg,  a->tol,   a->n_evs,   a->dev_sw, a->dev_st, a->dev_in,
              p->d_loop, reinterpret_cast<double*>(reinterpret_cast<char*>(p->d_loop) + 16),
              reinterpret_cast<double*>(reinterpret_cast<char*>(p->d_loop) + LQ_LOOP_TRI), d_h, d_dec};
  const int ahead = LOMPC_LOOP_AHEAD;
  const bool fused = lq_loop_fusable(p, LQ_LOOP_PERSIST);
  auto done = [&]() { return __atomic_load_n(const_cast<long long*>(&h->done), __ATOMIC_ACQUIRE) != 0; };
  auto progress = [&]() { return __atomic_load_n(const_cast<long long*>(&h->progress), __ATOMIC_ACQUIRE); };
  // spin until cond() (the device's progress lives in pinned memory); a generous guard against a hang
  auto wait_for = [&](auto cond) -> int {
    if (cond()) return LOMPC_OK;
    const double t0 = now_us();
    while (!cond()) {
      __builtin_ia32_pause();
      if (now_us() - t0 > 20e6) {
        p->err = "device price loop: no progress for 20 s";
        return LOMPC_ERR_HIP;
      }
    }
    t_wait += now_us() - t0;
    return LOMPC_OK;
  };
  p->skip = p->d_loop;
  rc = LOMPC_OK;
  if (fused && LQ_LOOP_PERSIST) {
    // ONE launch runs every call of the loop (k_loop_run); the host waits for `done` — or for the
    // launch to end without it (a wave's bounded spin expired: ctl[3])
    const double t0 = prof ? now_us() : 0.0;
    rc = lq_launch_loop_run(p, a->dev_in, a->dev_in + 2 * N3, const_cast<double*>(a->dev_sw),
                            const_cast<double*>(a->dev_st), sa, st);
    if (prof) t_issue += now_us() - t0;
    p->skip = nullptr;
    if (rc) return rc;
    bool ended = false;
    rc = wait_for([&]() {
      if (done()) return true;
      ended = hipStreamQuery(st) == hipSuccess;  // (the launch is over: `done` was set before it ended, or never)
      return ended && !done();
    });
    if (rc) return rc;
    if (!done()) {
      p->err = "device price loop: a persistent wave timed out waiting for the next call";
      return LOMPC_ERR_HIP;
    }
  } else {
  for (int j = 0; j <= MI; ++j) {
    // enqueue call j once calls 0 .. j - ahead - 1 have run; never past the finishing call + ahead
    if ((rc = wait_for([&]() { return progress() >= j - ahead || done(); }))) break;
    if (done() && j > h->conv_at + ahead) break;
    const double t0 = prof ? now_us() : 0.0;
    if (fused) {  // path + aggregation + loop step: one launch
      rc = lq_launch_loop_iter(p, a->dev_in, a->dev_in + 2 * N3, const_cast<double*>(a->dev_sw),
                               const_cast<double*>(a->dev_st), sa, j, st);
      if (rc) break;
    } else {
      rc = lq_plan_launch(p, a->dev_in, a->dev_in + 2 * N3, nullptr, nullptr, nullptr, nullptr,
                          const_cast<double*>(a->dev_sw), const_cast<double*>(a->dev_st), st, nullptr);
      if (rc) break;
      hipLaunchKernelGGL(k_loop_step, dim3(1), dim3(64), 0, st, sa, j);
      if (hipGetLastError() != hipSuccess) {
        p->err = "k_loop_step launch";
        rc = LOMPC_ERR_HIP;
        break;
      }
    }
    if (prof) t_issue += now_us() - t0;
  }
  p->skip = nullptr;
  if (rc) return rc;
  if ((rc = wait_for(done))) return rc;
  }
  const long long err = h->err;
  const int it = (int)h->conv_at;
  if (prof) {
    prof[LOMPC_LOOP_PROF_ITERS] += it + 1;
    const double wall = now_us() - t_start;
    prof[LOMPC_LOOP_PROF_WALL] += wall;
    prof[LOMPC_LOOP_PROF_ISSUE] += t_issue;
    prof[LOMPC_LOOP_PROF_WAIT] += t_wait;
    prof[LOMPC_LOOP_PROF_GPU] += wall;  // the device runs the whole loop (host spans included)
    prof[LOMPC_LOOP_PROF_HOST] = prof[LOMPC_LOOP_PROF_WALL] - prof[LOMPC_LOOP_PROF_ISSUE] -
                                 prof[LOMPC_LOOP_PROF_WAIT] - prof[LOMPC_LOOP_PROF_STEP];
  }
  if (err == 1) return fail_arg(p, "gamma outside [0, y_max]");
  if (err == 2) {
    p->err = lq_failed_text(p, st);
    return LOMPC_ERR_NOT_CONVERGED;
  }
  if (err == 3) {
    p->err = "price-gradient QP: no certified optimum";
    return LOMPC_ERR_NOT_CONVERGED;
  }
  *iterations = it;
  for (int i = 0; i < N3; ++i) lmbd[i] = h->lmbd[i];
  for (int i = 0; i < N; ++i) w_k[i] = h->w_k[i];
  if (dual_cost) *dual_cost = h->dual_cost;
  if (errs)
    for (int k = 0; k < 3; ++k) errs[k] = h->errs[k];
  const volatile double* hd = p->h_dec;
  for (int i = 0; i < it; ++i) {
    if (dec_actual) dec_actual[i] = hd[i];
    if (dec_pred) dec_pred[i] = hd[MI + i];
  }
  return LOMPC_OK;
}

extern "C" {

int lompc_price_loop(lompc_plan* p, const lompc_price_loop_args* a, double* lmbd, double* w_k, double* dual_cost,
                     double* dec_actual, double* dec_pred, int* iterations, double* errs, void* stream) {
  if (!p || !a || !lmbd || !w_k || !iterations || !a->A_bar || !a->w_ref || !a->dev_in || !a->host_in ||
      !a->dev_sw || !a->dev_st || !a->host_sw || !a->host_st || a->max_iter < 1 || !(a->n_evs > 0.0))
    return LOMPC_ERR_INVALID_ARG;
  const int N = a->N, r = a->r;
  if (N != p->N || p->S != 2 || (r != 2 * N && r != 3 * N)) return fail_arg(p, "price loop: a plan of 2 sets of horizon N");
  HIPCHK(p, hipSetDevice(p->device));
  hipStream_t st = (hipStream_t)stream;
  bool dev = a->device_loop != 0;
  if (dev) {  // the device form computes the metric as A'A + kappa I: check that A_bar is that
    double worst = 0.0;
    for (int i = 0; i < N; ++i)
      for (int j = 0; j < N; ++j) {
        const double ref = (double)(N - std::max(i, j)) + (i == j ? a->kappa : 0.0);
        worst = std::max(worst, std::fabs(a->A_bar[(size_t)i * N + j] - ref));
      }
    dev = worst <= 1e-12 * (1.0 + N + a->kappa);
  }
  if (dev) return lq_price_loop_device(p, a, lmbd, w_k, dual_cost, dec_actual, dec_pred, iterations, errs, st);
  return lq_price_loop_host(p, a, lmbd, w_k, dual_cost, dec_actual, dec_pred, iterations, errs, st);
}

// The regularisation of price_solver.py:142-147 / 248-255 at the loop's final iterate w: the
// column-separable LP of lompc_lp_separable with A = Dphi(w)'[:, :r], b = Dphi(w)' lmbd, c = phi(w)
// (phi / Dphi of lompc.py:172-187), lmbd[:r] replaced by its solution; *pre / *post = phi(w)' lmbd
// before / after.  One routine for the chain and PriceSolver's per-partition loops, so the two give
// the same bits.
int lompc_price_regularize(int N, int r, double theta, double w_max, const double* w, double* lmbd, double* pre,
                           double* post) {
  if (N < 1 || N > LOMPC_MAX_N || (r != 2 * N && r != 3 * N) || !w || !lmbd || !pre || !post)
    return LOMPC_ERR_INVALID_ARG;
  const int N3 = 3 * N;
  const double th = theta, wm = w_max, qs = 3.0 * th / (4.0 * wm);
  std::vector<double> A((size_t)N * r, 0.0), b(N), phi(N3), x(r);
  for (int t = 0; t < N; ++t) {
    phi[t] = th * w[t];
    phi[N + t] = th * (wm - w[t]);
    phi[2 * N + t] = qs * (w[t] * w[t]);
  }
  double s = 0.0;
  for (int i = 0; i < N3; ++i) s += phi[i] * lmbd[i];
  *pre = s;
  for (int t = 0; t < N; ++t) {  // Dphi(w)'[:r]: row t holds theta (col t), -theta (col N + t), 2 q_s w_t
    A[(size_t)t * r + t] = th;
    A[(size_t)t * r + N + t] = -th;
    if (r == 3 * N) A[(size_t)t * r + 2 * N + t] = 2.0 * qs * w[t];
    double acc = 0.0;
    for (int i = 0; i < r; ++i) acc += A[(size_t)t * r + i] * lmbd[i];
    b[t] = acc;
  }
  int rc = lompc_lp_separable(N, r, A.data(), b.data(), phi.data(), x.data());
  // a cost entry below zero (theta w_t or theta (w_max - w_t) at ~-1e-17 when the loop's w_k, an
  // unclamped piece aggregate, sits a rounding error outside [0, w_max]) leaves the closed form: the
  // general LP then, as PriceRegularizer.solve_price_regularization does (the LP stays bounded:
  // columns t and N + t together cost theta w_max > 0 per unit)
  if (rc == LOMPC_ERR_UNSUPPORTED) rc = lompc_lp_solve(N, r, A.data(), b.data(), phi.data(), x.data(), nullptr);
  if (rc) return rc;
  for (int i = 0; i < r; ++i) lmbd[i] = x[i];
  s = 0.0;
  for (int i = 0; i < N3; ++i) s += phi[i] * lmbd[i];
  *post = s;
  return LOMPC_OK;
}

// One EV type's price loops over its partitions in order (charging_station.py:275-307): each
// partition's loop (lompc_price_loop) starts from the previous partition's regularised prices, then
// its prices are regularised (lompc_price_regularize).
int lompc_price_chain(int n_parts, lompc_price_chain_part* parts, const lompc_price_loop_args* common,
                      double* prev_prices, void* stream) {
  if (n_parts < 0 || (n_parts > 0 && (!parts || !common || !prev_prices))) return LOMPC_ERR_INVALID_ARG;
  if (n_parts == 0) return LOMPC_OK;
  const int N = common->N, r = common->r, N3 = 3 * N;
  if (N < 1 || N > LOMPC_MAX_N || (r != 2 * N && r != 3 * N)) return LOMPC_ERR_INVALID_ARG;
  for (int k = 0; k < n_parts; ++k) {
    lompc_price_chain_part& q = parts[k];
    q.rc = LOMPC_OK;
    if (!q.plan) continue;  // (no EVs: no loop, the prices chain past it)
    lompc_price_loop_args a = *common;
    a.n_evs = q.n_evs;
    a.tol = q.tol;
    a.w_ref = q.w_ref;
    a.dev_sw = q.dev_sw;
    a.dev_st = q.dev_st;
    double* lm = q.lmbd;
    for (int i = 0; i < N3; ++i) lm[i] = i < r ? prev_prices[i] : 0.0;
    int it = 0;
    double dual = 0.0;
    q.rc = lompc_price_loop(q.plan, &a, lm, q.w_k, &dual, q.dec_actual, q.dec_pred, &it, nullptr, stream);
    if (q.rc) return q.rc;
    q.calls = it + 1;
    q.iterations = std::min(it, a.max_iter - 1);  // (the reference's loop variable at its end)
    q.rc = lompc_price_regularize(N, r, common->theta, common->w_max, q.w_k, lm, &q.price_before_reg,
                                  &q.price_after_reg);
    if (q.rc) return q.rc;
    for (int i = 0; i < r; ++i) prev_prices[i] = lm[i];
  }
  return LOMPC_OK;
}

}  // extern "C"
