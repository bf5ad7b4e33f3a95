// lompc_qp.hpp — device-side building blocks of the batched LoMPC QP engine.
//
// The per-EV program is LoMPC.solve_lompc (reference chargingstation/lompc.py:137-156):
//
//   minimize  0.5 c ||A w||^2 - c*gamma*1'A w + sum_t (0.5 d_t w_t^2 + e_t w_t)
//             + [large EVs] sum_t pwl(w_t) + c0
//   s.t.      0 <= w <= w_max                                    (lompc.py:74, :93)
//
// with A = tril(ones) (lompc.py:69), c = 2 delta theta^2 (lompc.py:71, :117-122),
// d_t = 2 lmbd_r theta^2 + 2 q_scale lmbd3_t [+ 2 theta^2/0.81 small]   (:105, :131, :133)
// e_t = theta (lmbd1_t - lmbd2_t), c0 = theta w_max sum(lmbd2)          (:126-129)
// pwl = (theta w_max)^2 max(0, u-0.125, 1.5u-0.375, 2u-0.75), u = w/w_max (:108-114).
//
// y = A w is the cumulative charge, so the program is a scalar-state chain:
// for any working set (each coordinate either fixed at a "knot" — a box bound
// or a PWL kink — or free inside one PWL segment) the equality-constrained
// sub-problem is solved EXACTLY by a backward scalar Riccati recursion plus a
// forward pass: O(N) flops, no N x N matrix anywhere.
//
// State encoding per coordinate: even s = 2k -> fixed at knot k, odd s = 2k+1 ->
// free in segment k.  Every state has a "box" (lo, hi, slo, shi):
//   w in [lo, hi]   and   -r in [slo, shi]      (r = gradient of the smooth part)
//   free seg k : [knot_k, knot_k+1] x [sigma_k, sigma_k]
//   knot k     : [knot_k, knot_k]   x [sigma_k-1, sigma_k]   (+-inf at the box ends)
// so projection, KKT residual and the active-set moves (always s -> s +- 1) are
// branch-free: KKT(w) = max over t of dist(-r_t, [slo, shi]) with w_t in [lo, hi].
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LQ_MAXSEG 4                     // large EVs: 4 PWL segments (lompc.py:111)
#define LQ_NSTATE (2 * LQ_MAXSEG + 1)   // 9 states
#ifndef LQ_G
#define LQ_G 64                         // path cells per parameter set (one wave each)
#endif
#ifndef LQ_PPL
#define LQ_PPL 8                        // max affine pieces stored per cell
#endif
#define LQ_STB 64                       // state bytes per stored working set (N <= 64)

struct QPConst {
  int N;             // horizon
  int m;             // number of separable segments (1 small, 4 large)
  int ev_small;      // 1 for "small"
  int pad0;
  double c;          // 2 delta theta^2
  double delta, theta, y_max, w_max, q_scale;
  double inv_wmax;   // 1 / w_max
  double dsmall;     // 2 theta^2 / 0.9^2 for small EVs, 0 otherwise
  double knots[LQ_MAXSEG + 1];
  double slopes[LQ_MAXSEG];
  double scale;      // magnitude of the gradient, for relative tolerances
  double tol_switch; // active-set switching tolerance (absolute, gradient units)
  double tol_cert;   // KKT certificate tolerance (absolute, gradient units)
  double ktol;       // knot tolerance on w (absolute)
};

// Per-set data record (doubles), stride SD(N) = 3N + 8:
//   [0,N) d   [N,2N) e   [2N,3N) w_ref
//   3N+0 c0, +1 lmbd1_0, +2 lmbd2_0, +3 lmbd3_0, +4 lmbd_r, +5 kappa, +6 gamma_ref, +7 has_wref
__host__ __device__ inline int lq_sd(int N) { return 3 * N + 10; }  // + gamma window (lo, G / width)

// Path table (device pointers). Cell l of set s covers gamma in [l h, (l+1) h], h = y_max / LQ_G.
// On a piece (one working set) everything the per-EV outputs need is polynomial in gamma:
//   w_j(gamma)      = a_j + b_j gamma
//   cost(gamma)     = K0 + K1 gamma + K2 gamma^2     (lompc.py:155, incl. c0)
//   err(gamma)^2    = F0 + F1 gamma + F2 gamma^2     (A_bar error vs w_ref, price_solver.py:207)
struct PathTable {
  int* cnt;          // [S][G]              pieces stored in the cell (0 = cell unsolved)
  double* gend;      // [S][G][PPL]         upper gamma of each piece
  double* ab;        // [S][G][PPL][N][2]   (a_j, b_j)
  double* coef;      // [S][G][PPL][8]      K0, K1, K2, F0, F1, F2, -, -
  uint8_t* st;       // [S][G][PPL][STB]    working set of the piece (one byte per stage)
};

struct Box {
  double lo, hi, slo, shi;
};

// Box table in LDS (per-lane state -> one ds_read_b128 pair; a register select
// chain over a by-value kernel argument makes hipcc copy it to scratch).
__device__ __forceinline__ double* lq_tab() {
  __shared__ __attribute__((aligned(16))) double tab[LQ_NSTATE * 4];
  return tab;
}
// fp32 copy of the box table (the fp32 working-set search of lompc_wave.hpp)
__device__ __forceinline__ float* lq_tabf() {
  __shared__ __attribute__((aligned(16))) float tabf[LQ_NSTATE * 4];
  return tabf;
}
// The box table's rows (threads < LQ_NSTATE), without the barrier that publishes them.
__device__ __forceinline__ void lq_tab_fill(const QPConst& q) {
  double* tb = lq_tab();
  const int s = threadIdx.x;
  if (s < LQ_NSTATE) {
    // knots / slopes as opaque uniform values (scalar loads + readfirstlane), selected per lane by
    // compares: a lane-indexed load from q would be a vector memory round at every kernel start
    auto u = [](double x) {
      const long long b = __builtin_bit_cast(long long, x);
      const int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
      return __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
    };
    const double k0 = u(q.knots[0]), k1 = u(q.knots[1]), k2 = u(q.knots[2]), k3 = u(q.knots[3]), k4 = u(q.knots[4]);
    const double s0 = u(q.slopes[0]), s1 = u(q.slopes[1]), s2 = u(q.slopes[2]), s3 = u(q.slopes[3]);
    static_assert(LQ_MAXSEG == 4, "knot selection written for 4 segments");
    auto pick_k = [&](int i) { return i <= 0 ? k0 : i == 1 ? k1 : i == 2 ? k2 : i == 3 ? k3 : k4; };
    auto pick_s = [&](int i) { return i <= 0 ? s0 : i == 1 ? s1 : i == 2 ? s2 : s3; };
    const int k = s >> 1;
    double lo, hi, slo, shi;
    if (s & 1) {
      const int kk = k < q.m ? k : q.m - 1;
      lo = pick_k(kk);
      hi = pick_k(kk + 1);
      slo = shi = pick_s(kk);
    } else {
      const int kk = k <= q.m ? k : q.m;
      lo = hi = pick_k(kk);
      slo = kk > 0 ? pick_s(kk - 1) : -INFINITY;
      shi = kk < q.m ? pick_s(kk) : INFINITY;
    }
    tb[4 * s + 0] = lo;
    tb[4 * s + 1] = hi;
    tb[4 * s + 2] = slo;
    tb[4 * s + 3] = shi;
    float* tf = lq_tabf();
    tf[4 * s + 0] = (float)lo;
    tf[4 * s + 1] = (float)hi;
    tf[4 * s + 2] = (float)slo;
    tf[4 * s + 3] = (float)shi;
  }
}
// Every kernel calls this (all threads, before anything else).
__device__ __forceinline__ void lq_tab_init(const QPConst& q) {
  lq_tab_fill(q);
  __syncthreads();
}
// a wave-uniform value materialised here (its scalar load completes by this point instead of
// being issued at its first use)
__device__ __forceinline__ void lq_pin(double& x) {
  const long long b = __builtin_bit_cast(long long, x);
  int lo = __builtin_amdgcn_readfirstlane((int)b), hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
  asm volatile("" : "+s"(lo), "+s"(hi));
  x = __builtin_bit_cast(double, ((long long)hi << 32) | (long long)(unsigned)lo);
}
__device__ __forceinline__ Box lq_box(int s) {
  const double2* tb = reinterpret_cast<const double2*>(lq_tab());
  const double2 x = tb[2 * s], y = tb[2 * s + 1];
  return {x.x, x.y, y.x, y.y};
}

struct BoxF {
  float lo, hi, slo, shi;
};
__device__ __forceinline__ BoxF lq_boxf(int s) {
  const float4 x = reinterpret_cast<const float4*>(lq_tabf())[s];
  return {x.x, x.y, x.z, x.w};
}

// Active-set move of one coordinate from (w, r): s -> s+1 / s-1 / s.
//   free : w above hi -> fixed at the upper knot (s+1), below lo -> lower knot (s-1)
//   fixed: -r above shi -> free in the segment above (s+1), below slo -> below (s-1)
__device__ __forceinline__ int lq_move(const QPConst& q, int s, const Box& b, double w, double r) {
  const double v = -r;
  const bool fr = (s & 1) != 0;
  const bool up = fr ? (w > b.hi + q.ktol) : (v > b.shi + q.tol_switch);
  const bool dn = fr ? (w < b.lo - q.ktol) : (v < b.slo - q.tol_switch);
  return s + (up ? 1 : 0) - (dn ? 1 : 0);
}
// PDAS move with jumps: a free coordinate whose value left its segment goes straight
// to the knot that bounds the value's segment on the side it came from (the lower
// knot when moving up, the upper knot when moving down); fixed ones move as lq_move.
__device__ __forceinline__ int lq_move_jump(const QPConst& q, int s, const Box& b, double w, double r) {
  if (!(s & 1)) return lq_move(q, s, b, w, r);
  const bool up = w > b.hi + q.ktol, dn = w < b.lo - q.ktol;
  if (!up && !dn) return s;
  if (!(w > q.knots[0])) return 0;
  if (!(w < q.w_max)) return 2 * q.m;
  int seg = 0;
#pragma unroll
  for (int k = 1; k < LQ_MAXSEG; ++k) seg += (k < q.m && w > q.knots[k]) ? 1 : 0;
  return up ? 2 * seg : 2 * seg + 2;
}
// distance of (w, -r) from the state's box, in gradient units (w outside -> +inf)
__device__ __forceinline__ double lq_resid(const QPConst& q, const Box& b, double w, double r) {
  const double v = -r;
  const double res = fmax(fmax(b.slo - v, v - b.shi), 0.0);
  return (w < b.lo - q.ktol || w > b.hi + q.ktol) ? INFINITY : res;
}

// Packed working set for the lane-per-QP solver: 4 bits per coordinate.
template <int NMAX>
struct States {
  static constexpr int NW = (NMAX + 7) / 8;
  uint32_t w[NW];
  __device__ __forceinline__ int get(int t) const {  // t must be compile-time in hot loops
    return (int)((w[t >> 3] >> ((t & 7) * 4)) & 15u);
  }
  __device__ __forceinline__ void set(int t, int v) {
    const int sh = (t & 7) * 4;
    w[t >> 3] = (w[t >> 3] & ~(15u << sh)) | ((uint32_t)v << sh);
  }
  __device__ __forceinline__ void set_rt(int t, int v) {  // runtime index, no dynamic register indexing
    const int wi = t >> 3;
    const int sh = (t & 7) * 4;
#pragma unroll
    for (int i = 0; i < NW; ++i)
      if (i == wi) w[i] = (w[i] & ~(15u << sh)) | ((uint32_t)v << sh);
  }
  __device__ __forceinline__ void fill(int v) {
    uint32_t x = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) x |= ((uint32_t)v) << (4 * i);
#pragma unroll
    for (int i = 0; i < NW; ++i) w[i] = x;
  }
  // from one byte per coordinate (16-byte aligned source)
  __device__ __forceinline__ void load_bytes(const uint8_t* __restrict__ src) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(src);
#pragma unroll
    for (int i = 0; i < NW; ++i) {
      const uint32_t x0 = p[2 * i], x1 = p[2 * i + 1];
      const uint32_t n0 = (x0 & 0xfu) | ((x0 >> 4) & 0xf0u) | ((x0 >> 8) & 0xf00u) | ((x0 >> 12) & 0xf000u);
      const uint32_t n1 = (x1 & 0xfu) | ((x1 >> 4) & 0xf0u) | ((x1 >> 8) & 0xf00u) | ((x1 >> 12) & 0xf000u);
      w[i] = n0 | (n1 << 16);
    }
  }
};

__device__ __forceinline__ double lq_rcp(double x) {  // v_rcp_f64 + two Newton steps (~0.5 ulp)
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// ---------------------------------------------------------------------------
// Exact sub-problem solve for a working set (single right-hand side).
// Backward:  V_{t+1}(y) = 0.5 P y^2 + p y;  Q = c + P, q = p - c gamma
//   free  : w_t = K y_{t-1} + k,  K = -Q/(Q+d), k = -(q+e~)/(Q+d),
//           P' = Q d/(Q+d),  p' = (q d - e~ Q)/(Q+d)       (e~ = e_t + slope)
//   fixed : w_t = wbar,  P' = Q,  p' = Q wbar + q
// Q >= c > 0, so every reciprocal is well defined.
// ---------------------------------------------------------------------------
template <int NMAX>
__device__ __forceinline__ void lq_riccati(const QPConst& q, const int N, const double* __restrict__ d,
                                           const double* __restrict__ e, double gamma,
                                           const States<NMAX>& st, double (&w)[NMAX]) {
  double K[NMAX], k[NMAX];
  double P = 0.0, p = 0.0;
  const double cg = q.c * gamma;
#pragma unroll
  for (int t = NMAX - 1; t >= 0; --t) {
    if (t < N) {
      const double Q = q.c + P;
      const double qq = p - cg;
      const int s = st.get(t);
      const Box b = lq_box(s);
      const double dt = d[t];
      const bool fr = (s & 1) != 0;
      const double et = e[t] + b.slo;
      const double inv = lq_rcp(Q + dt);
      K[t] = fr ? -Q * inv : 0.0;
      k[t] = fr ? -(qq + et) * inv : b.lo;
      P = fr ? Q * dt * inv : Q;
      p = fr ? (qq * dt - et * Q) * inv : fma(Q, b.lo, qq);
    }
  }
  double y = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      w[t] = fma(K[t], y, k[t]);
      y += w[t];
    }
  }
}

// Gradient of the smooth part: r_j = c (sum_{i>=j} y_i - (N-j) gamma) + d_j w_j + e_j,
// computed on the fly with the prefix trick (total of y first, then running prefix).
template <int NMAX>
__device__ __forceinline__ double lq_sum_y(const int N, const double (&w)[NMAX]) {
  double y = 0.0, Z = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < N) {
      y += w[t];
      Z += y;
    }
  return Z;
}

// One PDAS (semismooth-Newton active-set) state update from the sub-problem
// solution w.  Returns true if any coordinate changed state.
template <int NMAX>
__device__ __forceinline__ bool lq_pdas_update(const QPConst& q, const int N, const double* __restrict__ d,
                                               const double* __restrict__ e, double gamma,
                                               const double (&w)[NMAX], States<NMAX>& st) {
  const double Zt = lq_sum_y<NMAX>(N, w);
  double y = 0.0, Z = 0.0;
  bool changed = false;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      y += w[t];
      const double r = q.c * (Zt - Z - (double)(N - t) * gamma) + d[t] * w[t] + e[t];
      Z += y;
      const int s = st.get(t);
      const int ns = lq_move(q, s, lq_box(s), w[t], r);
      changed |= (ns != s);
      st.set(t, ns);
    }
  }
  return changed;
}

template <int NMAX>
__device__ __forceinline__ bool lq_pdas(const QPConst& q, const int N, const double* __restrict__ d,
                                        const double* __restrict__ e, double gamma, States<NMAX>& st,
                                        double (&w)[NMAX], int max_it) {
  bool done = false;
  for (int it = 0; it < max_it && !done; ++it) {
    lq_riccati<NMAX>(q, N, d, e, gamma, st, w);
    done = !lq_pdas_update<NMAX>(q, N, d, e, gamma, w, st);
  }
  return done;
}

// Project onto the working set's box (free: clamp into the segment; fixed: the knot).
template <int NMAX>
__device__ __forceinline__ void lq_snap(const int N, const States<NMAX>& st, double (&w)[NMAX]) {
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < N) {
      const Box b = lq_box(st.get(t));
      w[t] = fmin(fmax(w[t], b.lo), b.hi);
    }
}

// KKT certificate of (w, working set): max distance of -r from the state boxes.
template <int NMAX>
__device__ __forceinline__ double lq_kkt(const QPConst& q, const int N, const double* __restrict__ d,
                                         const double* __restrict__ e, double gamma, const States<NMAX>& st,
                                         const double (&w)[NMAX]) {
  const double Zt = lq_sum_y<NMAX>(N, w);
  double y = 0.0, Z = 0.0, res = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      y += w[t];
      const double r = q.c * (Zt - Z - (double)(N - t) * gamma) + d[t] * w[t] + e[t];
      Z += y;
      res = fmax(res, lq_resid(q, lq_box(st.get(t)), w[t], r));
    }
  }
  return res;
}

// Per-EV scalar outputs from an optimal w:
//   cost   (lompc.py:155: the full objective incl. c0)
//   err    = sqrt((w-w_ref)' A_bar (w-w_ref)), A_bar = A'A + kappa I (price_solver.py:191-192, :207)
//   price0 (lompc.py:164-170)
struct EVOut {
  double cost, err, price0;
};

__device__ __forceinline__ double lq_pwl(double u) {  // lompc.py:111
  return fmax(fmax(0.0 * u, u - 0.125), fmax(1.5 * u - 0.375, 2.0 * u - 0.75));
}

__device__ __forceinline__ double lq_price0(const QPConst& q, const double* __restrict__ sd, double w0) {
  const int N = q.N;
  return q.theta * (w0 * sd[3 * N + 1] + (q.w_max - w0) * sd[3 * N + 2]) + q.q_scale * w0 * w0 * sd[3 * N + 3] +
         q.theta * q.theta * w0 * w0 * sd[3 * N + 4];
}

template <int NMAX>
__device__ __forceinline__ EVOut lq_outputs(const QPConst& q, const int N, const double* __restrict__ sd, double gamma,
                                            const double (&w)[NMAX], bool want_err) {
  const double* d = sd;
  const double* e = sd + N;
  const double* wr = sd + 2 * N;
  const double kappa = sd[3 * N + 5];
  double y = 0.0, sy = 0.0, syy = 0.0, quad = 0.0, pwl = 0.0;
  double ey = 0.0, eyy = 0.0, edd = 0.0;
#pragma unroll
  for (int t = 0; t < NMAX; ++t) {
    if (t < N) {
      const double wt = w[t];
      y += wt;
      sy += y;
      syy = fma(y, y, syy);
      quad = fma(wt, fma(0.5 * d[t], wt, e[t]), quad);
      if (!q.ev_small) pwl += lq_pwl(wt * q.inv_wmax);
      if (want_err) {
        const double dv = wt - wr[t];
        ey += dv;
        eyy = fma(ey, ey, eyy);
        edd = fma(dv, dv, edd);
      }
    }
  }
  EVOut o;
  const double tw = q.theta * q.w_max;
  o.cost = 0.5 * q.c * syy - q.c * gamma * sy + quad + sd[3 * N + 0] + (q.ev_small ? 0.0 : tw * tw * pwl);
  o.err = want_err ? sqrt(eyy + kappa * edd) : 0.0;
  o.price0 = lq_price0(q, sd, w[0]);
  return o;
}
