// lompc_loopstep.hpp — one step of the device-resident price loop (lompc_loop.hip): the host
// loop's body for one engine call (lq_price_loop_host, lompc_plan.hip; price_solver.py:120-140)
// on one wave.  Run by k_loop_step (lompc_loop.hip) after an engine call's launches, or fused
// behind the engine call itself by k_loop_iter (lompc_plan.hip: path + aggregation + this step
// in one launch, run by the workgroup whose set closes last).
#pragma once
#include "lompc_pricewave.hpp"

// pinned, written by the loop step with system-scope stores, read by the host
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

// d_loop: int ctl[4] (ctl[0]: finished = the plan kernels' skip flag; ctl[1]: k_loop_iter's
// arrived workgroups, zero between calls) | double state[4] | pad | the A_bar factor of the loop
// (lqp::Tri per lane: Q[64] iv[64] d[64] K[64], written by the first step)
constexpr int LQ_LOOP_TRI = 64;  // byte offset of the factor
constexpr int LQ_LOOP_BYTES = LQ_LOOP_TRI + 4 * 64 * 8;

struct StepArgs {
  int N, r, max_iter, tol_avg;
  double theta, w_max, m, kappa, eps_reg, tol, n_evs;
  const double* sw;  // [2][N]  set sums of the engine call (combined over the ranks)
  const double* st;  // [2][8]  set stats
  double* dev_in;    // [2][3N] prices | [2] lmbd_r | [2][N] w_ref   (the plan's price buffer)
  int* ctl;
  double* state;     // [0] dual cost of the previous call, [1] price term of dec_actual[0]
  double* tri;       // [4][64] the A_bar factor (valid from the loop's second step)
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

// publish v at p for the host behind every earlier store of the loop (the finishing step: the host
// reads the results once it sees `done`)
__device__ __forceinline__ void lq_publish(long long* p, long long v) {
  __threadfence_system();
  sys_release(p, v);
}

// the step's writes the next call reads (prices, loop state, the A_bar factor): write-through (sc1),
// so a persistent loop's waves on other XCDs read them with sc1 loads after the generation flag
__device__ __forceinline__ void lq_st_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// loads of the engine call's set outputs: plain after a kernel boundary (k_loop_step),
// device-coherent when workgroups of the same launch wrote them (k_loop_iter)
template <bool COH>
__device__ __forceinline__ double lq_ld_set(const double* p) {
  if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else return *p;
}

// the engine call's outputs the step reads (lane t: stage t of the sums of w)
struct StepIn {
  double s0;      // set 0 (the partition's EVs): sum of w_t
  double wk;      // set 1 = the central QP: its sum of w is its w
  double emax;    // set 0's max A_bar error
  double cost_c;  // set 1's cost
  double n_inv, n_fail;
  // the call's own inputs (step_prices: loadable before the engine call has run)
  double lm[3];       // lane t: prices t, N + t, 2N + t
  double wr;          // lane t: w_ref_t
  double dc, dterm;   // state[0], state[1]
  lqp::Tri ab;        // the A_bar factor (the loop's first step computes it)
};

// the step's inputs that do not depend on the engine call's outputs (the prices it ran at, w_ref,
// the loop state): k_loop_iter loads them at its start, before its path.  COH: with sc1 loads (the
// persistent loop, k_loop_run: the previous call's step wrote them in the same launch)
template <bool COH = false>
__device__ __forceinline__ void step_prices(const StepArgs& a, const int lane, StepIn& in) {
  const int N = a.N, N3 = 3 * N;
  const bool act = lane < N;
  in.wr = act ? a.dev_in[2 * N3 + 2 + lane] : 0.0;  // (w_ref: constant over the loop)
#pragma unroll
  for (int k = 0; k < 3; ++k) in.lm[k] = act ? lq_ld_set<COH>(a.dev_in + k * N + lane) : 0.0;
  in.dc = lq_ld_set<COH>(a.state);
  in.dterm = lq_ld_set<COH>(a.state + 1);
  in.ab.Q = lq_ld_set<COH>(a.tri + lane);
  in.ab.iv = lq_ld_set<COH>(a.tri + 64 + lane);
  in.ab.d = lq_ld_set<COH>(a.tri + 128 + lane);
  in.ab.K = lq_ld_set<COH>(a.tri + 192 + lane);
}

// Engine call m of the loop has run (its set sums / stats in `in`, at the prices in a.dev_in);
// one wave, lane = stage.
struct NoStamp {
  __device__ __forceinline__ void operator()(int) const {}
};
struct NoRelease {  // (k_loop_iter / k_loop_step: the kernel's end releases the next call)
  __device__ __forceinline__ void operator()() const {}
};

// what a step leaves for the next call when the caller keeps the loop in registers (k_loop_run's
// redundant form: every wave runs the same step on the same closed outputs)
struct StepOut {
  bool fin = false;      // the loop ended at this call
  double v[3] = {0, 0, 0};  // lane t < N: the next call's prices t, N + t, 2N + t (as stored)
  double cost_c = 0.0, dterm = 0.0;  // the next call's state[0], state[1]
  lqp::Tri ab{};         // the A_bar factor (computed by the first step)
};

// (ST: a diagnostic build's phase stamp, called with 8 after the inputs and the error metric, 9
// after the price QP)
// (REL: called once the next call's prices and loop state are written, before the host-memory writes
// of this step — k_loop_run releases its waiting waves there, so the PCIe writes overlap the next call)
// (WR = false: nothing is written — no prices, state or factor to memory, no host results; the
// outputs only in `out`, for the waves of the redundant form that are not its writer)
template <class ST = NoStamp, class REL = NoRelease, bool WR = true>
__device__ __forceinline__ void loop_step_core(const StepArgs& a, const int m, const int lane, const StepIn& in,
                                               const ST& stamp = ST{}, const REL& release = REL{},
                                               StepOut* out = nullptr) {
  const int N = a.N, N3 = 3 * N;
  const bool act = lane < N;
  const double s0 = act ? in.s0 : 0.0, wk = act ? in.wk : 0.0;
  const double emax = in.emax, cost_c = in.cost_c, n_inv = in.n_inv, n_fail = in.n_fail;
  const double wr = in.wr;
  double lm[3] = {in.lm[0], in.lm[1], in.lm[2]};
  const double dc = in.dc, dterm = in.dterm;
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
  const double dec_prev = cost_c - dc + dterm;  // (stored to the host below, after the release)
  const bool conv = (a.tol_avg ? e2 : e0) <= a.tol;
  stamp(8);
  double x[3] = {0.0, 0.0, 0.0};
  double dec = 0.0;
  if (!err && !conv && m < a.max_iter) {
    // the price-gradient step at (w_k, lmbd) (lompc_price_step)
    lqp::PriceQPW P;
    P.init(N, a.r, a.theta, a.w_max, a.m, a.kappa, a.eps_reg, wk, m > 0 ? &in.ab : nullptr);
    if (out) out->ab = P.Ab;
    if (WR && m == 0) {  // the loop's A_bar factor for its later steps
      lq_st_wt(a.tri + lane, P.Ab.Q);
      lq_st_wt(a.tri + 64 + lane, P.Ab.iv);
      lq_st_wt(a.tri + 128 + lane, P.Ab.d);
      lq_st_wt(a.tri + 192 + lane, P.Ab.K);
    }
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
    double mu[3];
    if (lqp::nnqp_wave(P, q, lm, x, 1e-11 * (1.0 + qmax), mu)) {
      double cn = 0.0;  // 1/2 x'Qx + q'x with Qx = mu - q from the certificate
#pragma unroll
      for (int k = 0; k < 3; ++k) cn += P.has(k) ? x[k] * fma(0.5, mu[k] - q[k], q[k]) : 0.0;
      dec = dual - lqw::wave_sum(cn, 64);
    } else {
      err = 3;
    }
  }
  stamp(9);
  if (err || conv || m >= a.max_iter) {  // finished: the results to the host, then the flags
    if (out) out->fin = true;
    if (!WR) return;
    if (m > 0 && lane == 0) sys_st(a.h_dec + (m - 1), dec_prev);
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
      lq_publish(&a.h->done, 1);
      lq_publish(&a.h->progress, (long long)m + 1);
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
      if (out) out->v[k] = v;
      if (WR) {
        lq_st_wt(a.dev_in + k * N + lane, v);
        lq_st_wt(a.dev_in + N3 + k * N + lane, v);
      }
    }
  }
  dt = lqw::wave_sum(dt, N);
  if (out) {
    out->cost_c = cost_c;
    out->dterm = m == 0 ? dt : 0.0;
  }
  if (!WR) return;
  if (lane == 0) {
    lq_st_wt(a.state, cost_c);
    lq_st_wt(a.state + 1, m == 0 ? dt : 0.0);
  }
  release();
  if (lane == 0) {
    if (m > 0) sys_st(a.h_dec + (m - 1), dec_prev);
    sys_st(a.h_dec + a.max_iter + m, dec);
    // (an unfinished step's progress orders nothing for the host — it only paces the enqueueing;
    // h_dec is read after `done`, which the finishing step publishes behind every earlier store)
    sys_st(&a.h->progress, (long long)m + 1);
  }
}

// the step with the engine call's outputs read from a.sw / a.st
template <bool COH>
__device__ __forceinline__ void loop_step(const StepArgs& a, const int m, const int lane) {
  const int N = a.N;
  const bool act = lane < N;
  StepIn in;
  step_prices(a, lane, in);
  in.s0 = act ? lq_ld_set<COH>(a.sw + lane) : 0.0;
  in.wk = act ? lq_ld_set<COH>(a.sw + N + lane) : 0.0;
  in.emax = lq_ld_set<COH>(a.st + LOMPC_STAT_MAX_ERR);
  in.cost_c = lq_ld_set<COH>(a.st + LOMPC_SET_STATS + LOMPC_STAT_SUM_COST);
  in.n_inv = lq_ld_set<COH>(a.st + LOMPC_STAT_N_INVALID) + lq_ld_set<COH>(a.st + LOMPC_SET_STATS + LOMPC_STAT_N_INVALID);
  in.n_fail = lq_ld_set<COH>(a.st + LOMPC_STAT_N_FAILED) + lq_ld_set<COH>(a.st + LOMPC_SET_STATS + LOMPC_STAT_N_FAILED);
  loop_step_core(a, m, lane, in);
}
