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
#include <hip/hip_runtime.h>
#include <string.h>

#include <chrono>
#include <cmath>
#include <cstdlib>
#include <vector>

#include "lompc_ctx.hpp"
#include "lompc_pricewave.hpp"

// pinned, written by k_loop_step with system-scope stores, read by the host
struct lq_host_loop {
  long long progress;   // engine calls whose step ran
  long long done;       // 1 once the loop finished (the fields below are then valid)
  long long conv_at;    // the engine call at which it finished (= the reference's iterations)
  long long err;        // 0 ok, 1 invalid gamma, 2 LoMPC QPs without a certified optimum, 3 price QP failed
  double dual_cost;
  double errs[3];
  double lmbd[3 * LOMPC_MAX_N];
  double w_k[LOMPC_MAX_N];
};

namespace {

constexpr int LQ_LOOP_BYTES = 64;  // d_loop: int ctl[4] (ctl[0]: finished = the plan kernels' skip flag) | double state[4]

struct StepArgs {
  int N, r, max_iter, tol_avg;
  double theta, w_max, m, kappa, eps_reg, tol, n_evs;
  const double* sw;  // [2][N]  set sums of the engine call (combined over the ranks)
  const double* st;  // [2][8]  set stats
  double* dev_in;    // [2][3N] prices | [2] lmbd_r | [2][N] w_ref   (the plan's price buffer)
  int* ctl;
  double* state;     // [0] dual cost of the previous call, [1] price term of dec_actual[0]
  lq_host_loop* h;
  double* h_dec;     // [2][max_iter] pinned: dec_actual | dec_pred
};

__device__ __forceinline__ void sys_st(long long* p, long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_st(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void sys_release(long long* p, long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Engine call m of the loop has run (its set sums / stats in a.sw, a.st, at the prices in
// a.dev_in).  The host loop's body for that call (lompc_plan.hip, lq_price_loop_host), on one wave.
__global__ __launch_bounds__(64) void k_loop_step(StepArgs a, int m) {
  if (a.ctl[0]) return;  // finished: a call enqueued ahead of the convergence
  const int lane = (int)threadIdx.x, N = a.N, N3 = 3 * N;
  const bool act = lane < N;
  const double s0 = act ? a.sw[lane] : 0.0;
  const double wk = act ? a.sw[N + lane] : 0.0;  // set 1 = the central QP: its sum of w is its w
  const double wr = act ? a.dev_in[2 * N3 + 2 + lane] : 0.0;
  double lm[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) lm[k] = act ? a.dev_in[k * N + lane] : 0.0;
  const double emax = a.st[LOMPC_STAT_MAX_ERR];
  const double cost_c = a.st[LOMPC_SET_STATS + LOMPC_STAT_SUM_COST];
  const double n_inv = a.st[LOMPC_STAT_N_INVALID] + a.st[LOMPC_SET_STATS + LOMPC_STAT_N_INVALID];
  const double n_fail = a.st[LOMPC_STAT_N_FAILED] + a.st[LOMPC_SET_STATS + LOMPC_STAT_N_FAILED];
  const double dc = a.state[0], dterm = a.state[1];
  long long err = n_inv > 0.0 ? 1 : (n_fail > 0.0 ? 2 : 0);
  // price_solver.py:210-214: w_avg error in the A_bar = A'A + kappa I metric, w0 error, max error
  const double d = act ? s0 / a.n_evs - wr : 0.0;
  lqw::Sums<1> c1;
  c1.v[0] = d;
  const double Ad = lqw::wave_scan(c1, N).v[0];  // (A d)_t = sum_{s <= t} d_s
  const double qf = lqw::wave_sum(act ? fma(Ad, Ad, a.kappa * d * d) : 0.0, N);
  const double e0 = emax, e1 = fabs(lqw::readlane_d(d, 0)), e2 = sqrt(qf);
  // dual cost decrease of the previous step (price_solver.py:133-138; the reference's lmbd_k /
  // lmbd_k_new aliasing keeps the price term only for the first step)
  if (m > 0 && lane == 0) sys_st(a.h_dec + (m - 1), cost_c - dc + dterm);
  const bool conv = (a.tol_avg ? e2 : e0) <= a.tol;
  double x[3] = {0.0, 0.0, 0.0};
  double dec = 0.0;
  if (!err && !conv && m < a.max_iter) {
    // the price-gradient step at (w_k, lmbd) (lompc_price_step)
    lqp::PriceQPW P;
    P.init(N, a.r, a.theta, a.w_max, a.m, a.kappa, a.eps_reg, wk);
    const double q_s = 3.0 * a.theta / (4.0 * a.w_max);
    double Ql[3], q[3];
    P.mulQ(lm, Ql);
    const double dw = wk - wr;
    const double dphi[3] = {a.theta * dw, -a.theta * dw, q_s * (wk * wk - wr * wr)};
    double qmax = 0.0, dual = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      q[k] = P.has(k) ? -Ql[k] - dphi[k] : 0.0;
      qmax = fmax(qmax, fabs(q[k]));
      dual += P.has(k) ? lm[k] * fma(0.5, Ql[k], q[k]) : 0.0;
    }
    qmax = lqw::wave_max(qmax, 64);
    dual = lqw::wave_sum(dual, 64);
    if (lqp::nnqp_wave(P, q, lm, x, 1e-11 * (1.0 + qmax))) {
      double Qx[3], cn = 0.0;
      P.mulQ(x, Qx);
#pragma unroll
      for (int k = 0; k < 3; ++k) cn += P.has(k) ? x[k] * fma(0.5, Qx[k], q[k]) : 0.0;
      dec = dual - lqw::wave_sum(cn, 64);
    } else {
      err = 3;
    }
  }
  if (err || conv || m >= a.max_iter) {  // finished: the results to the host, then the flags
    if (act) {
#pragma unroll
      for (int k = 0; k < 3; ++k) sys_st(&a.h->lmbd[k * N + lane], lm[k]);
      sys_st(&a.h->w_k[lane], wk);
    }
    if (lane == 0) {
      sys_st(&a.h->dual_cost, cost_c);
      sys_st(&a.h->errs[0], e0);
      sys_st(&a.h->errs[1], e1);
      sys_st(&a.h->errs[2], e2);
      sys_st(&a.h->conv_at, (long long)m);
      sys_st(&a.h->err, err);
      __hip_atomic_store(a.ctl, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the later calls skip
      __threadfence_system();
      sys_release(&a.h->done, 1);
      sys_release(&a.h->progress, (long long)m + 1);
    }
    return;
  }
  // the next prices into both sets' rows of the plan's price buffer (rows >= r stay 0)
  const double q_s = 3.0 * a.theta / (4.0 * a.w_max);
  const double phr[3] = {a.theta * wr, a.theta * (a.w_max - wr), q_s * wr * wr};  // phi(w_ref), lompc.py:172-177
  double dt = 0.0;
  if (act) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double v = k * N < a.r ? x[k] : 0.0;
      dt = fma(lm[k] - v, phr[k], dt);
      a.dev_in[k * N + lane] = v;
      a.dev_in[N3 + k * N + lane] = v;
    }
  }
  dt = lqw::wave_sum(dt, N);
  if (lane == 0) {
    sys_st(a.h_dec + a.max_iter + m, dec);
    a.state[0] = cost_c;
    a.state[1] = m == 0 ? dt : 0.0;
    __threadfence_system();
    sys_release(&a.h->progress, (long long)m + 1);
  }
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
              p->d_loop, reinterpret_cast<double*>(reinterpret_cast<char*>(p->d_loop) + 16), d_h, d_dec};
  const int ahead = LOMPC_LOOP_AHEAD;
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
  for (int j = 0; j <= MI; ++j) {
    // enqueue call j once calls 0 .. j - ahead - 1 have run; never past the finishing call + ahead
    if ((rc = wait_for([&]() { return progress() >= j - ahead || done(); }))) break;
    if (done() && j > h->conv_at + ahead) break;
    const double t0 = prof ? now_us() : 0.0;
    rc = lq_plan_launch(p, a->dev_in, a->dev_in + 2 * N3, nullptr, nullptr, nullptr, nullptr,
                        const_cast<double*>(a->dev_sw), const_cast<double*>(a->dev_st), st, nullptr);
    if (rc) break;
    hipLaunchKernelGGL(k_loop_step, dim3(1), dim3(64), 0, st, sa, j);
    if (hipGetLastError() != hipSuccess) {
      p->err = "k_loop_step launch";
      rc = LOMPC_ERR_HIP;
      break;
    }
    if (prof) t_issue += now_us() - t0;
  }
  p->skip = nullptr;
  if (rc) return rc;
  if ((rc = wait_for(done))) return rc;
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

}  // extern "C"
