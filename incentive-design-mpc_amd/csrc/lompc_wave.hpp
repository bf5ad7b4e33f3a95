// lompc_wave.hpp — one LoMPC QP per 64-lane wavefront, lane t = horizon stage t.
//
// Used where latency, not throughput, matters: the per-set path kernel (K1) and
// the rare in-kernel repair of an EV whose path value failed its certificate.
// A lane-per-QP Riccati recursion is a ~3N-deep dependent fp64 chain, so here
// the three recursions of one sub-problem solve are wave-parallel scans:
//
//   (1) P_t  = F_t(P_{t+1})          Moebius map   free: d(c+P)/(c+P+d)   fixed: c+P
//   (2) p_t  = al_t p_{t+1} + be_t   affine map    (given P_{t+1})
//   (3) y_t  = (1+K_t) y_{t-1} + k_t affine map    forward, w_t = K_t y_{t-1} + k_t
//
// All three run in the natural layout: (1) and (2) as SUFFIX scans (DPP row_shl 1/2/4/8 inside
// each 16-lane row, then the rows' totals carried down by v_readlane: scalar broadcasts, no LDS
// round trip), (3) as a prefix scan (DPP row_shr 1/2/4/8 + row_bcast 15/31).  The per-stage gains
// of (1)-(2) are then already on the lanes (3) needs.  The multiplier of coordinate t comes from
// the cost-to-go derivative (envelope theorem), so no fourth scan is needed:
//   r_t = c (y_t - gamma) + P_{t+1} y_t + p_{t+1} + d_t w_t + e_t .
#pragma once
#include "lompc_qp.hpp"

#ifndef LQ_JUMP_FREE
#define LQ_JUMP_FREE 0  // fp32 search jumps: 0 = to the knot bounding w's segment, 1 = free inside it
#endif
#ifndef LQ_JUMP_IT
#define LQ_JUMP_IT 3  // PDAS iterations that may jump across segments
#endif
#ifndef LQ_PDAS_CAP
// PDAS iterations before the monotone primal active set takes over (warm-started from the
// projected PDAS iterate).  Random price vectors converge in <= 15 at N = 48; the station's
// structured large-EV prices can make PDAS cycle, which at the old cap of 4N + 8 cost up to
// ~0.2 ms per path cell.
#define LQ_PDAS_CAP 32
#endif

namespace lqw {

// ---- DPP helpers (64-bit values as two 32-bit lanes) -----------------------
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp(double old, double x) {
  const long long xi = __builtin_bit_cast(long long, x);
  const long long oi = __builtin_bit_cast(long long, old);
  const int lo = __builtin_amdgcn_update_dpp((int)oi, (int)xi, CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(oi >> 32), (int)(xi >> 32), CTRL, ROW_MASK, 0xf, false);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
// value of lane l-1 (lane 0 gets `old`): DPP wave_shr:1
__device__ __forceinline__ double shr1(double old, double x) { return dpp<0x138, 0xf>(old, x); }
// value of lane l+1 (lane 63 gets `old`): DPP wave_shl:1
__device__ __forceinline__ double shl1(double old, double x) { return dpp<0x130, 0xf>(old, x); }

// lane `lane`'s value on every lane (lane wave-uniform): v_readlane into scalar registers, no LDS
// round trip (a __shfl is a ds_bpermute)
__device__ __forceinline__ double readlane_d(double x, int lane) {
  const long long xi = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_readlane((int)xi, lane);
  const int hi = __builtin_amdgcn_readlane((int)(xi >> 32), lane);
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ int readlane_i(int x, int lane) { return __builtin_amdgcn_readlane(x, lane); }

struct Mob {  // Moebius map P -> (a P + b) / (c P + d), entries >= 0
  double a, b, c, d;
  __device__ __forceinline__ static Mob identity() { return {1.0, 0.0, 0.0, 1.0}; }
  // R o L (L applied first).  Every per-stage map enters with d = 1 and entries
  // >= 0, so a composition of k maps has d >= 1 and entries <= ~2^k max(c, 1):
  // no cancellation and no rescaling needed for k <= 64.
  __device__ __forceinline__ static Mob combine(const Mob& L, const Mob& R) {
    return {fma(R.a, L.a, R.b * L.c), fma(R.a, L.b, R.b * L.d), fma(R.c, L.a, R.d * L.c),
            fma(R.c, L.b, R.d * L.d)};
  }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ Mob from() const {  // DPP source, identity where no source lane
    return {dpp<CTRL, ROW_MASK>(1.0, a), dpp<CTRL, ROW_MASK>(0.0, b), dpp<CTRL, ROW_MASK>(0.0, c),
            dpp<CTRL, ROW_MASK>(1.0, d)};
  }
  __device__ __forceinline__ Mob rl(int l) const {  // lane l's value, wave-uniform
    return {readlane_d(a, l), readlane_d(b, l), readlane_d(c, l), readlane_d(d, l)};
  }
};

template <int NB>
struct Aff {  // y -> A y + B[k]
  double A;
  double B[NB];
  __device__ __forceinline__ static Aff identity() {
    Aff r;
    r.A = 1.0;
#pragma unroll
    for (int k = 0; k < NB; ++k) r.B[k] = 0.0;
    return r;
  }
  __device__ __forceinline__ static Aff combine(const Aff& L, const Aff& R) {
    Aff r;
    r.A = R.A * L.A;
#pragma unroll
    for (int k = 0; k < NB; ++k) r.B[k] = fma(R.A, L.B[k], R.B[k]);
    return r;
  }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ Aff from() const {
    Aff r;
    r.A = dpp<CTRL, ROW_MASK>(1.0, A);
#pragma unroll
    for (int k = 0; k < NB; ++k) r.B[k] = dpp<CTRL, ROW_MASK>(0.0, B[k]);
    return r;
  }
  __device__ __forceinline__ Aff rl(int l) const {
    Aff r;
    r.A = readlane_d(A, l);
#pragma unroll
    for (int k = 0; k < NB; ++k) r.B[k] = readlane_d(B[k], l);
    return r;
  }
};

// Inclusive prefix scan across the lanes [0, n) (lane order = application order);
// lanes >= n hold identities.  DPP row_shr 1/2/4/8 scans each 16-lane row, row_bcast
// 15 and 31 carry across rows; steps that only serve lanes >= n are skipped (n is
// wave-uniform).
template <typename T>
__device__ __forceinline__ T wave_scan(T x, int n = 64) {
  x = T::combine(x.template from<0x111, 0xf>(), x);  // row_shr:1
  x = T::combine(x.template from<0x112, 0xf>(), x);  // row_shr:2
  x = T::combine(x.template from<0x114, 0xf>(), x);  // row_shr:4
  x = T::combine(x.template from<0x118, 0xf>(), x);  // row_shr:8
  if (n > 16) x = T::combine(x.template from<0x142, 0xa>(), x);  // row_bcast:15 -> rows 1, 3
  if (n > 32) x = T::combine(x.template from<0x143, 0xc>(), x);  // row_bcast:31 -> rows 2, 3
  return x;
}

// Inclusive SUFFIX scan across the lanes [0, n): lane l holds x_l o x_{l+1} o ... (the highest
// lane applied first); lanes >= n hold identities.  DPP row_shl 1/2/4/8 scans each 16-lane row
// backwards, then every row below the last one combines with the totals of the rows above it,
// read from their first lanes with v_readlane (wave-uniform, no LDS).
template <typename T>
__device__ __forceinline__ T wave_scan_rev(T x, int n = 64) {
  x = T::combine(x.template from<0x101, 0xf>(), x);  // row_shl:1
  x = T::combine(x.template from<0x102, 0xf>(), x);  // row_shl:2
  x = T::combine(x.template from<0x104, 0xf>(), x);  // row_shl:4
  x = T::combine(x.template from<0x108, 0xf>(), x);  // row_shl:8
  if (n > 16) {
    const int row = (int)(threadIdx.x & 63) >> 4;
    const T t1 = x.rl(16);
    T c0 = t1, c1 = T::identity(), c2 = T::identity();
    if (n > 32) {
      const T t2 = x.rl(32);
      c1 = t2;
      if (n > 48) {
        c2 = x.rl(48);
        c1 = T::combine(c2, t2);
      }
      c0 = T::combine(c1, t1);
    }
    x = T::combine(row == 0 ? c0 : (row == 1 ? c1 : (row == 2 ? c2 : T::identity())), x);
  }
  return x;
}

template <int K>
struct Sums {  // K independent running sums
  double v[K];
  __device__ __forceinline__ static Sums identity() {
    Sums r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.v[k] = 0.0;
    return r;
  }
  __device__ __forceinline__ Sums rl(int l) const {
    Sums r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.v[k] = readlane_d(v[k], l);
    return r;
  }
  __device__ __forceinline__ static Sums combine(const Sums& L, const Sums& R) {
    Sums r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.v[k] = L.v[k] + R.v[k];
    return r;
  }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ Sums from() const {
    Sums r;
#pragma unroll
    for (int k = 0; k < K; ++k) r.v[k] = dpp<CTRL, ROW_MASK>(0.0, v[k]);
    return r;
  }
};

// totals over lanes [0, n) of K values (lanes >= n must hold 0), broadcast
template <int K>
__device__ __forceinline__ void wave_totals(double (&v)[K], int n) {
  Sums<K> x;
#pragma unroll
  for (int k = 0; k < K; ++k) x.v[k] = v[k];
  x = wave_scan(x, n);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = readlane_d(x.v[k], n - 1);
}

__device__ __forceinline__ double bperm(int src_lane, double x) {
  const long long xi = __builtin_bit_cast(long long, x);
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)xi);
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(xi >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ int bperm_i(int src_lane, int x) { return __builtin_amdgcn_ds_bpermute(src_lane << 2, x); }

struct MinV {
  double v;
  __device__ __forceinline__ static MinV combine(const MinV& L, const MinV& R) { return {fmin(L.v, R.v)}; }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ MinV from() const { return {dpp<CTRL, ROW_MASK>(INFINITY, v)}; }
};
struct MaxV {
  double v;
  __device__ __forceinline__ static MaxV combine(const MaxV& L, const MaxV& R) { return {fmax(L.v, R.v)}; }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ MaxV from() const { return {dpp<CTRL, ROW_MASK>(-INFINITY, v)}; }
};

// min over lanes [0, n) of v and the lowest lane holding it; result on every lane.
// DPP prefix scan (lane n-1 = the min) + ballot, no LDS round trips.
__device__ __forceinline__ void wave_argmin(double& v, int& idx, int n) {
  const double m = readlane_d(wave_scan(MinV{v}, n).v, n - 1);
  const unsigned long long hit = __ballot(v == m) & (n >= 64 ? ~0ull : ((1ull << n) - 1));
  idx = hit ? (int)__builtin_ctzll(hit) : 0;
  v = m;
}
// max over lanes [0, n), on every lane
__device__ __forceinline__ double wave_max(double v, int n) { return readlane_d(wave_scan(MaxV{v}, n).v, n - 1); }
// sum over lanes [0, n), on every lane
__device__ __forceinline__ double wave_sum(double v, int n) {
  Sums<1> x;
  x.v[0] = v;
  return readlane_d(wave_scan(x, n).v[0], n - 1);
}

// Per-set stage data of one wave: lane t holds stage t.
struct WaveSet {
  int N, lane;
  double d_nat, e_nat;
  __device__ __forceinline__ void load(const double* __restrict__ sd, int N_) {
    N = N_;
    lane = threadIdx.x & 63;
    d_nat = lane < N ? sd[lane] : 0.0;
    e_nat = lane < N ? sd[N + lane] : 0.0;
  }
};

// Per-lane (natural layout) results of one sub-problem solve; NB = 1 (value at
// gamma) or 2 (affine in gamma: [0] constant part, [1] gamma coefficient).
template <int NB>
struct StageSol {
  double w[NB];  // w_t
  double r[NB];  // multiplier r_t = gradient of the smooth part
};

// (bx: lq_box(s) on the active lanes, read by the caller — one LDS round per iteration feeds both
// the solve and the caller's move test, and it can be issued an iteration ahead)
template <int NB>
__device__ __forceinline__ StageSol<NB> solve_stage(const QPConst& q, const WaveSet& ws, const Box& bx, double gamma,
                                                    int s) {
  const double c = q.c;
  const int N = ws.N;
  const int lane = ws.lane;
  const bool act = lane < N;
  const double d = ws.d_nat;
  // ---- (1) Moebius suffix scan: lane t = F_t o ... o F_{N-1}
  const bool fr = act && (s & 1);
  Mob f = Mob::identity();
  if (fr) {  // P -> d (c+P) / (c+P+d), scaled to d-entry 1
    const double u = lq_rcp(c + d);
    f = {d * u, d * c * u, u, 1.0};
  } else if (act) {
    f = {1.0, c, 0.0, 1.0};  // P -> c + P
  }
  const Mob T = wave_scan_rev(f, N);
  const double P_here = T.b * lq_rcp(T.d);          // P_t = T_t(0)
  const double P_next = shl1(0.0, P_here);          // P_{t+1}
  // ---- (2) affine suffix scan for p
  const double Q = c + P_next;
  const double iv = lq_rcp(Q + d);
  const double et = ws.e_nat + bx.slo;
  Aff<NB> g = Aff<NB>::identity();
  if (fr) {
    g.A = d * iv;
    if (NB == 1) g.B[0] = -(c * gamma * d + et * Q) * iv;
    else {
      g.B[0] = -et * Q * iv;
      g.B[NB - 1] = -c * d * iv;
    }
  } else if (act) {
    if (NB == 1) g.B[0] = fma(Q, bx.lo, -c * gamma);
    else {
      g.B[0] = Q * bx.lo;
      g.B[NB - 1] = -c;
    }
  }
  const Aff<NB> Gp = wave_scan_rev(g, N);
  double pn[NB];
#pragma unroll
  for (int k = 0; k < NB; ++k) pn[k] = shl1(0.0, Gp.B[k]);  // p_{t+1}
  const double K = fr ? -Q * iv : 0.0;
  double kk[NB];
  if (NB == 1) {
    kk[0] = fr ? -(pn[0] - c * gamma + et) * iv : bx.lo;
  } else {
    kk[0] = fr ? -(pn[0] + et) * iv : bx.lo;
    kk[NB - 1] = fr ? -(pn[NB - 1] - c) * iv : 0.0;
  }
  // ---- (3) forward scan y_t = (1+K_t) y_{t-1} + k_t
  Aff<NB> h = Aff<NB>::identity();
  if (act) {
    h.A = 1.0 + K;
#pragma unroll
    for (int k = 0; k < NB; ++k) h.B[k] = kk[k];
  }
  const Aff<NB> Y = wave_scan(h, N);
  StageSol<NB> out;
#pragma unroll
  for (int k = 0; k < NB; ++k) {
    const double y = Y.B[k];
    const double yp = shr1(0.0, y);
    out.w[k] = fma(K, yp, kk[k]);
    const double base = (NB == 1) ? ws.e_nat - c * gamma : (k == 0 ? ws.e_nat : -c);
    out.r[k] = fma(c + P_next, y, pn[k]) + fma(d, out.w[k], base);
  }
  return out;
}
template <int NB>
__device__ __forceinline__ StageSol<NB> solve_stage(const QPConst& q, const WaveSet& ws, double gamma, int s) {
  return solve_stage<NB>(q, ws, lq_box(ws.lane < ws.N ? s : 0), gamma, s);
}

// Wave-parallel PDAS at gamma from working set s (lane t = stage t).
// Returns true on convergence; s, w, r then hold the final working set,
// solution and multipliers.
__device__ __forceinline__ bool wave_pdas(const QPConst& q, const WaveSet& ws, double gamma, int& s, double& w,
                                          double& r, int max_it, int* nit = nullptr) {
  for (int it = 0; it < max_it; ++it) {
    const Box bx = lq_box(ws.lane < ws.N ? s : 0);
    const StageSol<1> sol = solve_stage<1>(q, ws, bx, gamma, s);
    w = sol.w[0];
    r = sol.r[0];
    const int ns = ws.lane < ws.N ? (it < LQ_JUMP_IT ? lq_move_jump(q, s, bx, w, r) : lq_move(q, s, bx, w, r)) : s;
    const bool changed = __any(ns != s);
    s = ns;
    if (!changed) {
      if (nit) *nit = it + 1;
      return true;
    }
  }
  if (nit) *nit = max_it;
  return false;
}

// Wave-parallel primal active set (monotone).  Cold: from w = 0, all at knot 0.  Warm: from
// the given w projected onto [0, w_max], each coordinate free in the segment that contains it
// (a feasible point consistent with its working set, which is all the method needs).
__device__ __forceinline__ bool wave_primal_as(const QPConst& q, const WaveSet& ws, double gamma, int& s,
                                               double& w, double& r, int max_it, bool warm = false) {
  const bool act = ws.lane < ws.N;
  if (warm && act && w == w) {
    w = fmin(fmax(w, q.knots[0]), q.knots[q.m]);
    if (w <= q.knots[0]) {
      s = 0;
    } else if (w >= q.knots[q.m]) {
      s = 2 * q.m;
    } else {
      int seg = 0;
#pragma unroll
      for (int k = 1; k < LQ_MAXSEG; ++k) seg += (k < q.m && w > q.knots[k]) ? 1 : 0;
      s = 2 * seg + 1;
    }
  } else {
    s = 0;
    w = 0.0;
  }
  for (int it = 0; it < max_it; ++it) {
    const StageSol<1> sol = solve_stage<1>(q, ws, gamma, s);
    const Box b = lq_box(s);
    const double p = sol.w[0] - w;
    double al = INFINITY, bval = 0.0;
    int ns = s;
    if (act && (s & 1)) {
      if (p > 0.0) { al = (b.hi - w) / p; ns = s + 1; bval = b.hi; }
      else if (p < 0.0) { al = (b.lo - w) / p; ns = s - 1; bval = b.lo; }
    }
    double amin = al;
    int j = ws.lane;
    wave_argmin(amin, j, ws.N);
    if (amin >= 1.0) {
      w = sol.w[0];
      r = sol.r[0];
      const double v = -r;
      double viol = -INFINITY;
      int vs = s;
      if (act && !(s & 1)) {
        const double up = v - b.shi, dn = b.slo - v;
        if (up > dn) { viol = up; vs = s + 1; }
        else { viol = dn; vs = s - 1; }
      }
      double nv = -viol;
      int jv = ws.lane;
      wave_argmin(nv, jv, ws.N);
      if (-nv <= q.tol_switch) return true;
      if (ws.lane == jv) s = vs;
    } else {
      const double a = fmax(amin, 0.0);
      w = fma(a, p, w);
      if (ws.lane == j) {
        w = bval;
        s = ns;
      }
    }
  }
  return false;
}

// max KKT residual of (w, r) over the wave for the working set s
__device__ __forceinline__ double wave_kkt(const QPConst& q, const WaveSet& ws, int s, double w, double r) {
  const double res = ws.lane < ws.N ? lq_resid(q, lq_box(s), w, r) : 0.0;
  return wave_max(res, ws.N);
}

// Max KKT residual at gamma of the point w (lane t = w_t) for working set s,
// with the gradient recomputed from w itself (prefix scans), independent of
// the Riccati costate:  r_t = c (sum_{i>=t} y_i - (N-t) gamma) + d_t w_t + e_t.
__device__ __forceinline__ double wave_kkt_point(const QPConst& q, const WaveSet& ws, double gamma, int s,
                                                 double w) {
  const int N = ws.N;
  const bool act = ws.lane < N;
  Aff<1> h = Aff<1>::identity();
  if (act) h.B[0] = w;
  const double y = wave_scan(h, N).B[0];   // y_t = sum_{i<=t} w_i
  Aff<1> z = Aff<1>::identity();
  if (act) z.B[0] = y;
  const double Z = wave_scan(z, N).B[0];   // Z_t = sum_{i<=t} y_i
  const double Zt = readlane_d(Z, N - 1);
  const double r = q.c * (Zt - Z + y - (double)(N - ws.lane) * gamma) + ws.d_nat * w + ws.e_nat;
  const double res = act ? lq_resid(q, lq_box(s), w, r) : 0.0;
  return wave_max(res, N);
}

// ---- fp32 working-set search -------------------------------------------------
// The PDAS iterations that only move the working set toward the optimum's run in fp32: one
// DPP move per value instead of two, v_rcp_f32 without Newton steps.  Their result is only
// a starting working set for the fp64 PDAS + KKT certificate below, so fp32 rounding can
// cost iterations there, never accuracy.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dppf(float old, float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old),
                                                               __builtin_bit_cast(int, x), CTRL, ROW_MASK, 0xf,
                                                               false));
}
struct MobF {
  float a, b, c, d;
  __device__ __forceinline__ static MobF identity() { return {1.f, 0.f, 0.f, 1.f}; }
  __device__ __forceinline__ static MobF combine(const MobF& L, const MobF& R) {
    return {fmaf(R.a, L.a, R.b * L.c), fmaf(R.a, L.b, R.b * L.d), fmaf(R.c, L.a, R.d * L.c),
            fmaf(R.c, L.b, R.d * L.d)};
  }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ MobF from() const {
    return {dppf<CTRL, ROW_MASK>(1.f, a), dppf<CTRL, ROW_MASK>(0.f, b), dppf<CTRL, ROW_MASK>(0.f, c),
            dppf<CTRL, ROW_MASK>(1.f, d)};
  }
  __device__ __forceinline__ MobF rl(int l) const;
};
struct AffF {
  float A, B;
  __device__ __forceinline__ static AffF identity() { return {1.f, 0.f}; }
  __device__ __forceinline__ static AffF combine(const AffF& L, const AffF& R) { return {R.A * L.A, fmaf(R.A, L.B, R.B)}; }
  template <int CTRL, int ROW_MASK>
  __device__ __forceinline__ AffF from() const {
    return {dppf<CTRL, ROW_MASK>(1.f, A), dppf<CTRL, ROW_MASK>(0.f, B)};
  }
  __device__ __forceinline__ AffF rl(int l) const;
};
__device__ __forceinline__ float shr1f(float old, float x) { return dppf<0x138, 0xf>(old, x); }
__device__ __forceinline__ float readlane_f(float x, int l);
__device__ __forceinline__ MobF MobF::rl(int l) const {
  return {readlane_f(a, l), readlane_f(b, l), readlane_f(c, l), readlane_f(d, l)};
}
__device__ __forceinline__ AffF AffF::rl(int l) const { return {readlane_f(A, l), readlane_f(B, l)}; }
__device__ __forceinline__ float shl1f(float old, float x) { return dppf<0x130, 0xf>(old, x); }
__device__ __forceinline__ float readlane_f(float x, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), l));
}

// solve_stage<1> in fp32 (same recursions, see the file header)
// (bx: lq_boxf(s) on the active lanes, from the caller, as solve_stage)
__device__ __forceinline__ void solve_stage_f32(const QPConst& q, const WaveSet& ws, const BoxF& bx, float gamma,
                                                int s, float& w_out, float& r_out) {
  const float c = (float)q.c;
  const int N = ws.N;
  const int lane = ws.lane;
  const bool act = lane < N;
  const float d = (float)ws.d_nat;
  const bool fr = act && (s & 1);
  MobF f = MobF::identity();
  if (fr) {
    const float u = __builtin_amdgcn_rcpf(c + d);
    f = {d * u, d * c * u, u, 1.f};
  } else if (act) {
    f = {1.f, c, 0.f, 1.f};
  }
  const MobF T = wave_scan_rev(f, N);
  const float P_here = T.b * __builtin_amdgcn_rcpf(T.d);
  const float P_next = shl1f(0.f, P_here);
  const float Q = c + P_next;
  const float iv = __builtin_amdgcn_rcpf(Q + d);
  const float et = (float)ws.e_nat + bx.slo;
  AffF g = AffF::identity();
  if (fr) {
    g.A = d * iv;
    g.B = -(c * gamma * d + et * Q) * iv;
  } else if (act) {
    g.B = fmaf(Q, bx.lo, -c * gamma);
  }
  const AffF Gp = wave_scan_rev(g, N);
  const float pn = shl1f(0.f, Gp.B);
  const float K = fr ? -Q * iv : 0.f;
  const float kk = fr ? -(pn - c * gamma + et) * iv : bx.lo;
  AffF h = AffF::identity();
  if (act) {
    h.A = 1.f + K;
    h.B = kk;
  }
  const AffF Y = wave_scan(h, N);
  const float yp = shr1f(0.f, Y.B);
  w_out = fmaf(K, yp, kk);
  r_out = fmaf(c + P_next, Y.B, pn) + fmaf(d, w_out, (float)ws.e_nat - c * gamma);
}

// fp32 PDAS on the working set s (jump moves first, as wave_pdas), relative tolerances at fp32
// resolution.  Returns with s at the fixed point, or after max_it iterations; the iterations run.
__device__ __forceinline__ int wave_pdas_f32(const QPConst& q, const WaveSet& ws, double gamma, int& s,
                                             int max_it) {
  const float gf = (float)gamma;
  const float ktol = (float)(1e-6 * q.w_max), stol = (float)(1e-6 * q.scale);
  int m = q.m;
  asm volatile("" : "+s"(m));  // (read once, before the loop: not re-loaded inside the jump branch)
  for (int it = 0; it < max_it; ++it) {
    float w, r;
    const BoxF bx = lq_boxf(ws.lane < ws.N ? s : 0);
    solve_stage_f32(q, ws, bx, gf, s, w, r);
    int ns = s;
    if (ws.lane < ws.N) {
      const float v = -r;
      const bool freec = (s & 1) != 0;
      const bool up = freec ? (w > bx.hi + ktol) : (v > bx.shi + stol);
      const bool dn = freec ? (w < bx.lo - ktol) : (v < bx.slo - stol);
      if (freec && it < LQ_JUMP_IT && (up || dn)) {  // jump to the knot bounding w's segment
        if (!(w > (float)q.knots[0])) {
          ns = 0;
        } else if (!(w < (float)q.w_max)) {
          ns = 2 * m;
        } else {
          int seg = 0;
#pragma unroll
          for (int k = 1; k < LQ_MAXSEG; ++k) seg += (k < m && w > (float)q.knots[k]) ? 1 : 0;
#if LQ_JUMP_FREE
          ns = 2 * seg + 1;  // free in the segment that contains w
#else
          ns = up ? 2 * seg : 2 * seg + 2;
#endif
        }
      } else {
        ns = s + (up ? 1 : 0) - (dn ? 1 : 0);
      }
    }
    const bool changed = __any(ns != s);
    s = ns;
    if (!changed) return it + 1;
  }
  return max_it;
}

#ifndef LQ_F32_IT
#define LQ_F32_IT 24  // fp32 working-set iterations before the fp64 PDAS (0 = fp64 only)
#endif

// Exact certified solve of one QP by the whole wave: fp32 working-set search, fp64 PDAS from
// its result, primal active set if needed; KKT-certified in fp64.  nit (diagnostics): fp64 PDAS
// iterations + 256 x fp32 iterations + 65536 if the primal active set ran.
__device__ __forceinline__ bool wave_solve(const QPConst& q, const WaveSet& ws, double gamma, int& s, double& w,
                                           double& r, int* nit = nullptr) {
  int n32 = 0, n64 = 0;
  if (LQ_F32_IT > 0) n32 = wave_pdas_f32(q, ws, gamma, s, LQ_F32_IT);
  bool ok = wave_pdas(q, ws, gamma, s, w, r, min(4 * ws.N + 8, LQ_PDAS_CAP), &n64);
  if (nit) *nit = n64 + 256 * n32;
  if (ok) ok = wave_kkt(q, ws, s, w, r) <= q.tol_cert;
  if (!ok) {
    if (nit) *nit += 65536;
    ok = wave_primal_as(q, ws, gamma, s, w, r, 16 * ws.N + 32, true);
    if (ok) ok = wave_kkt(q, ws, s, w, r) <= q.tol_cert;
  }
  const Box b = lq_box(ws.lane < ws.N ? s : 0);
  w = fmin(fmax(w, b.lo), b.hi);
  return ok;
}

// wave_solve for the start of a parametric path: the fp64 PDAS iterations solve the sub-problem
// as an affine function of gamma (solve_stage<2>, evaluated at gamma), so on convergence `sol`
// already holds w(g) = a + b g and r(g) of the final working set for the path tracking (one
// sub-problem solve fewer per path).  has_sol is false when the primal active set had to take
// over (the caller then solves the final working set itself).
// warm: s is the previous run's working set at this point (a price loop's next iteration: at most a
// few coordinates move) — the fp64 PDAS starts from it directly, no fp32 search first
__device__ __forceinline__ bool wave_solve_path(const QPConst& q, const WaveSet& ws, double gamma, int& s,
                                                StageSol<2>& sol, bool& has_sol, int* nit = nullptr, bool warm = false) {
  int n32 = 0, n64 = 0;
  if (LQ_F32_IT > 0 && !warm) n32 = wave_pdas_f32(q, ws, gamma, s, LQ_F32_IT);
  const int max_it = min(4 * ws.N + 8, LQ_PDAS_CAP);
  bool ok = false;
  double w = 0.0, r = 0.0;
  for (int it = 0; it < max_it; ++it) {
    const Box bx = lq_box(ws.lane < ws.N ? s : 0);
    sol = solve_stage<2>(q, ws, bx, 0.0, s);
    w = fma(sol.w[1], gamma, sol.w[0]);
    r = fma(sol.r[1], gamma, sol.r[0]);
    const int ns = ws.lane < ws.N ? (it < LQ_JUMP_IT ? lq_move_jump(q, s, bx, w, r) : lq_move(q, s, bx, w, r)) : s;
    const bool changed = __any(ns != s);
    s = ns;
    n64 = it + 1;
    if (!changed) {
      ok = true;
      break;
    }
  }
  if (nit) *nit = n64 + 256 * n32;
  if (ok) ok = wave_kkt(q, ws, s, w, r) <= q.tol_cert;
  has_sol = ok;
  if (!ok) {
    if (nit) *nit += 65536;
    ok = wave_primal_as(q, ws, gamma, s, w, r, 16 * ws.N + 32, true);
    if (ok) ok = wave_kkt(q, ws, s, w, r) <= q.tol_cert;
  }
  return ok;
}

}  // namespace lqw
