// lompc_agg.hpp — reductions-only runs over gamma-sorted sets (LOMPC_PLAN_SORTED_GAMMA), included by
// lompc_plan.hip inside its kernel namespace.
//
// A price iteration of PriceSolver._get_w_err (price_solver.py:196-214) needs only per-set sums
// (sum of w, cost, price0, counts) and the max A_bar error — the reference drops the per-EV w
// (:206).  On a certified piece every per-EV output is a polynomial in gamma (w_t = a_t + b_t gamma,
// cost and err^2 quadratics), so the sums over the EVs of a piece need only the
// piece's EV count n, sum of gamma and sum of gamma^2, and the max error sits at the piece's
// smallest or largest gamma (err^2 is a convex quadratic).  When each set's gamma is ascending,
// the EVs of a piece are one contiguous run, so:
//   prepare (once per batch): the order is checked, gamma is quantised to x = round((gamma - lo)
//     2^40 / (hi - lo)) in its set's window and exclusive prefix sums of x and x^2 (as the two
//     40-bit halves) are built in exact integer arithmetic; a fine bucket index (G x KF buckets of
//     the window) maps any gamma to a short run of sorted positions;
//   run (k_agg, one workgroup per set, one wave per gamma cell): the piece ends of the cell become
//     sorted positions (fine index, then one wave-wide compare over <= 64 gammas), the sums come
//     from prefix-sum differences, the per-stage sums of w are sum_p n_p a_p + Gamma_p b_p, and EVs
//     outside the cell's certified coverage are re-solved individually (as k_finalize does).
// The per-iteration work is O(pieces x N), independent of the EV count; the sums are exact up to
// the 2^-41-of-the-window quantisation of gamma (the same one k_eval's close mode uses).
#pragma once

#define LQ_AGG_KF 256  // fine buckets per gamma cell
#define LQ_AGG_SB 1024 // sorted positions per prepare block

struct SortArgs {
  const QPConst* qd;
  CtxEnds ce;
  const int4* sblk;         // [nsblk] (set, first, end) blocks of <= LQ_AGG_SB EVs of one set
  const int* sblk_prefix;   // [S+1]
  const int64_t* set_off;   // [S+1]
  const double* gamma;
  const double* window;
  unsigned long long* bsum; // [nsblk][4] block totals: sum x, sum hi(x^2), sum lo(x^2), valid | bad << 32
  unsigned long long* P;    // [3][B + S] exclusive prefix sums (set s, position j at set_off[s] + s + j)
  int* pos;                 // [S][F + 1] first sorted position of each fine bucket
  int4* sinfo;              // [S] (valid EVs, order ok, -, -)
  int S, G, F;
  int64_t PB;               // B + S (stride of the three prefix arrays)
};

__device__ __forceinline__ bool agg_valid(double g, double ym) { return g >= 0.0 && g <= ym; }
__device__ __forceinline__ unsigned long long agg_fix(double g, double lo, double sc) {  // round((g - lo) sc)
  return (unsigned long long)rint(fmax(g - lo, 0.0) * sc);
}
__device__ __forceinline__ int agg_fine(double g, double lo, double fs, int F) {
  const double x = (g - lo) * fs;
  return x <= 0.0 ? 0 : (x >= (double)(F - 1) ? F - 1 : (int)x);
}
constexpr unsigned long long LQ_M40 = (1ull << 40) - 1ull;

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// (1) per block: the order check and the block totals of x, x^2
__global__ __launch_bounds__(256) void k_sorted_sum(SortArgs a) {
  __shared__ unsigned long long sh[4][4];
  const int4 bk = a.sblk[blockIdx.x];
  const int s = bk.x;
  const double ym = set_consts(a.qd, a.ce, s).y_max;
  const double lo = a.window[2 * s], sc = 0x1p40 / (a.window[2 * s + 1] - lo);
  const int64_t s0 = a.set_off[s];
  unsigned long long t1 = 0, th = 0, tl = 0, nv = 0, bad = 0;
  for (int i = bk.y + (int)threadIdx.x; i < bk.z; i += 256) {
    const double g = a.gamma[i];
    const bool v = agg_valid(g, ym);
    if (i > s0) {  // ascending valid values, invalid ones (NaN, outside [0, y_max]) after them
      const double gp = a.gamma[i - 1];
      const bool vp = agg_valid(gp, ym);
      bad |= (v && (!vp || g < gp)) ? 1ull : 0ull;
    }
    if (v) {
      const unsigned long long x = agg_fix(g, lo, sc);
      const unsigned __int128 x2 = (unsigned __int128)x * x;
      t1 += x;
      th += (unsigned long long)(x2 >> 40);
      tl += (unsigned long long)x2 & LQ_M40;
      ++nv;
    }
  }
  t1 = wave_sum_u64(t1);
  th = wave_sum_u64(th);
  tl = wave_sum_u64(tl);
  nv = wave_sum_u64(nv | (bad << 32));
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[wv][0] = t1;
    sh[wv][1] = th;
    sh[wv][2] = tl;
    sh[wv][3] = nv;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    unsigned long long v = 0;
    for (int w = 0; w < 4; ++w) v += sh[w][threadIdx.x];
    if (threadIdx.x == 3 && (v >> 32)) v = (v & 0xffffffffull) | (1ull << 32);  // any bad element
    a.bsum[(size_t)blockIdx.x * 4 + threadIdx.x] = v;
  }
}

// (2) per set (one workgroup): exclusive scan of the block totals (written back in place as
// offsets), the set's valid count and order flag; an empty index for a set without valid EVs.
// 256 blocks per pass, a workgroup-wide scan each (integer sums: exact, so the same values as a
// sequential scan in any order)
__global__ __launch_bounds__(256) void k_sorted_scan(SortArgs a) {
  __shared__ unsigned long long sh[4][256];
  __shared__ unsigned long long carry[4];  // sum x, sum hi(x^2), sum lo(x^2), valid count so far
  __shared__ int s_bad, s_nv;
  const int s = blockIdx.x, t = threadIdx.x;
  const int b0 = a.sblk_prefix[s], b1 = a.sblk_prefix[s + 1];
  if (t < 4) carry[t] = 0;
  if (t == 0) s_bad = 0;
  __syncthreads();
  for (int base = b0; base < b1; base += 256) {
    const int b = base + t;
    unsigned long long* r = a.bsum + (size_t)b * 4;
    unsigned long long x[4] = {0, 0, 0, 0};
    if (b < b1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = r[k];
      if (x[3] >> 32) s_bad = 1;  // (every writer stores the same value)
      x[3] &= 0xffffffffull;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) sh[k][t] = x[k];
    __syncthreads();
    for (int o = 1; o < 256; o <<= 1) {  // inclusive scan, Hillis-Steele
      unsigned long long y[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = t >= o ? sh[k][t - o] : 0ull;
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 4; ++k) sh[k][t] += y[k];
      __syncthreads();
    }
    if (b < b1) {
#pragma unroll
      for (int k = 0; k < 4; ++k) r[k] = carry[k] + sh[k][t] - x[k];  // exclusive offsets
    }
    __syncthreads();
    if (t < 4) carry[t] += sh[t][255];
    __syncthreads();
  }
  if (t == 0) {
    // the set's totals at position n (valid EVs are the first nv positions)
    const size_t e = (size_t)(a.set_off[s + 1] + s);
    a.P[e] = carry[0];
    a.P[a.PB + e] = carry[1];
    a.P[2 * a.PB + e] = carry[2];
    a.sinfo[s] = make_int4((int)carry[3], s_bad ? 0 : 1, 0, 0);
    s_nv = (int)carry[3];
  }
  __syncthreads();
  if (s_nv == 0) {
    for (int b = threadIdx.x; b <= a.F; b += 256) a.pos[(size_t)s * (a.F + 1) + b] = 0;
  }
}

// (3) per block: exclusive prefix sums at every position and the fine bucket index
__global__ __launch_bounds__(256) void k_sorted_fill(SortArgs a) {
  __shared__ unsigned long long sh[3][256];
  const int4 bk = a.sblk[blockIdx.x];
  const int s = bk.x;
  const double ym = set_consts(a.qd, a.ce, s).y_max;
  const double lo = a.window[2 * s], W = a.window[2 * s + 1] - lo;
  const double sc = 0x1p40 / W, fs = (double)a.F / W;
  const int64_t s0 = a.set_off[s];
  const int4 si = a.sinfo[s];
  const int nv = si.x;
  const unsigned long long* off = a.bsum + (size_t)blockIdx.x * 4;
  // 4 consecutive positions per thread
  const int t = threadIdx.x;
  const int i0 = bk.y + 4 * t;
  unsigned long long x1[4], xh[4], xl[4], c1 = 0, ch = 0, cl = 0;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u;
    const double g = i < bk.z ? a.gamma[i] : -1.0;
    unsigned long long x = 0, h = 0, l = 0;
    if (i < bk.z && agg_valid(g, ym)) {
      x = agg_fix(g, lo, sc);
      const unsigned __int128 x2 = (unsigned __int128)x * x;
      h = (unsigned long long)(x2 >> 40);
      l = (unsigned long long)x2 & LQ_M40;
    }
    x1[u] = c1;
    xh[u] = ch;
    xl[u] = cl;
    c1 += x;
    ch += h;
    cl += l;
  }
  // exclusive scan of the 256 thread totals: a wave-wide inclusive scan (shuffles), the four wave
  // totals combined in LDS (integer sums: exact, so any order gives the sequential scan's values)
  const int lane = t & 63, wv = t >> 6;
  unsigned long long i1 = c1, ih = ch, il = cl;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y1 = __shfl_up(i1, o), yh = __shfl_up(ih, o), yl = __shfl_up(il, o);
    if (lane >= o) {
      i1 += y1;
      ih += yh;
      il += yl;
    }
  }
  __shared__ unsigned long long wt[3][4];
  if (lane == 63) {
    wt[0][wv] = i1;
    wt[1][wv] = ih;
    wt[2][wv] = il;
  }
  __syncthreads();
  unsigned long long b1 = off[0], bh = off[1], bl = off[2];
  for (int w = 0; w < wv; ++w) {
    b1 += wt[0][w];
    bh += wt[1][w];
    bl += wt[2][w];
  }
  sh[0][t] = b1 + i1 - c1;
  sh[1][t] = bh + ih - ch;
  sh[2][t] = bl + il - cl;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u;
    if (i < bk.z) {
      const size_t e = (size_t)(i + s);
      a.P[e] = sh[0][t] + x1[u];
      a.P[a.PB + e] = sh[1][t] + xh[u];
      a.P[2 * a.PB + e] = sh[2][t] + xl[u];
    }
  }
  // fine bucket index: bucket b starts at the first valid position whose bucket is >= b (buckets past
  // the last valid position's: nv).  The block owns the buckets from its first valid position's
  // predecessor's bucket + 1 to its last valid position's (to F when that is the set's last valid
  // position); they are written cooperatively, each by a binary search over the block's buckets in
  // LDS — a set with few EVs has thousands of buckets per EV, which one lane writing its own range
  // serially took tens of microseconds for
  __shared__ int s_fb[LQ_AGG_SB];
  const int jb0 = (int)(bk.y - s0), jb1 = min((int)(bk.z - s0), nv);  // the block's valid positions
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int i = i0 + u, k = i - bk.y;
    if (i < bk.z && (int)(i - s0) < nv) s_fb[k] = agg_fine(a.gamma[i], lo, fs, a.F);
  }
  __syncthreads();
  if (jb0 < jb1) {
    const int m = jb1 - jb0;
    const int b_lo = jb0 == 0 ? 0 : agg_fine(a.gamma[s0 + jb0 - 1], lo, fs, a.F) + 1;
    const int b_hi = jb1 == nv ? a.F : s_fb[m - 1];
    int* ps = a.pos + (size_t)s * (a.F + 1);
    for (int b = b_lo + t; b <= b_hi; b += 256) {
      int l = 0, h = m;  // first block position with bucket >= b
      while (l < h) {
        const int mid = (l + h) >> 1;
        if (s_fb[mid] < b) l = mid + 1;
        else h = mid;
      }
      ps[b] = l < m ? jb0 + l : nv;
    }
  }
}

struct AggArgs {
  int S, G, N, F;
  const QPConst* qd;
  CtxEnds ce;
  const int64_t* set_off;
  const double* window;
  const double* gamma;
  const double* lmbd;
  const double* lmbd_r;
  const double* w_ref;
  const int* t_cnt;
  const double* t_lo;
  const uint8_t* t_sl;
  const double* t_ge;
  const double* t_cf;
  const double2* t_ab;
  const unsigned long long* P;
  int64_t PB;
  const int* pos;
  const int4* sinfo;
  double* set_sum_w;
  double* set_stats;
  double* stats;
  unsigned long long* tally;
  const int* skip;
};

// sorted position of the first gamma >= v (lower) or > v (!lower) within [a, b) of set s,
// b - a <= 64: one load per lane, one ballot; more: binary search (wave-uniform)
__device__ __forceinline__ int agg_search(const double* __restrict__ g, int a, int b, double v, bool lower, int lane) {
  if (b - a <= 64) {
    const double x = a + lane < b ? g[a + lane] : INFINITY;
    const bool before = lower ? (x < v) : (x <= v);
    return a + (int)__popcll(__ballot(before && a + lane < b));
  }
  while (a < b) {
    const int mid = (a + b) >> 1;
    const double x = g[mid];
    if (lower ? (x < v) : (x <= v)) a = mid + 1;
    else b = mid;
  }
  return a;
}

constexpr int LQ_AGG_W = 16;  // k_agg: waves per workgroup (cells per pass)
constexpr int LQ_AGG_REC = LOMPC_MAX_N + 8;  // k_loop_iter: doubles per cell record (sums of w | 5 scalars)

// a set's run-wide values (every wave of the set's cells)
struct AggSet {
  const QPConst* q;
  int N, G, KF, n_s;
  int4 si;
  bool order_ok;
  const double* g;
  const unsigned long long *P1, *PH, *PL;
  const int* ps;
  double wlo, h1, fs;
  const double* L;
  double lr, l1, l2, l3, tt, wm;
  bool preg = false;          // (k_loop_run redundant form) the prices in registers, lane t < N:
  double p1 = 0, p2 = 0, p3 = 0;  // prices t, N + t, 2N + t
};

template <int NT, bool COH = false>  // (COH: the prices re-read with sc1 loads, as load_set<COH>)
__device__ __forceinline__ AggSet agg_set_init(const AggArgs& r, const int s) {
  AggSet z;
  z.N = NT ? NT : r.N;
  z.G = r.G;
  z.KF = r.F / r.G;
  z.q = &set_consts(r.qd, r.ce, s);
  const int64_t so = r.set_off[s];
  z.n_s = (int)(r.set_off[s + 1] - so);
  z.si = r.sinfo[s];
  z.order_ok = z.si.y != 0;
  z.g = r.gamma + so;
  z.P1 = r.P + so + s;
  z.PH = z.P1 + r.PB;
  z.PL = z.P1 + 2 * r.PB;
  z.ps = r.pos + (size_t)s * (r.F + 1);
  z.wlo = r.window[2 * s];
  const double W = r.window[2 * s + 1] - z.wlo;
  z.h1 = W * 0x1p-40;
  z.fs = (double)r.F / W;
  z.L = r.lmbd + (size_t)s * 3 * z.N;
  z.lr = r.lmbd_r[s];
  z.l1 = ld_price<COH>(z.L);
  z.l2 = ld_price<COH>(z.L + z.N);
  z.l3 = ld_price<COH>(z.L + 2 * z.N);
  z.tt = z.q->theta * z.q->theta;
  z.wm = z.q->w_max;
  return z;
}

// a wave's partial sums over its cells (per lane: stage sums of w; lane 0 / wave-reduced: scalars)
struct AggPart {
  double accw = 0.0, acost = 0.0, ap0 = 0.0, aerr = 0.0;
  int nrep = 0, nfail = 0;
};

// Cell c of set s by one wave, into the wave's partials.  COH: the cell's tables were written in
// this launch (by this wave: k_loop_iter) — device-coherent loads (the scalar cache and the L1
// hold no copy of them).
// the cell's sorted positions [cs, ce)
__device__ __forceinline__ int2 agg_cell_range(const AggSet& z, const int c) {
  return make_int2(z.ps[c * z.KF], z.ps[(c + 1) * z.KF]);
}

template <int NT, bool COH, bool PCOH = false>  // (PCOH: the prices with sc1 loads, k_loop_run)
__device__ __forceinline__ void agg_cell(const AggArgs& r, const AggSet& z, const int s, const int c, const int2 rng,
                                         const int lane, AggPart& a) {
  const int N = NT ? NT : z.N, G = z.G, KF = z.KF;
  const QPConst& q = *z.q;
  const double* __restrict__ g = z.g;
  const int* ps = z.ps;
  const double wlo = z.wlo, h1 = z.h1, fs = z.fs;
  const double l1 = z.l1, l2 = z.l2, l3 = z.l3, lr = z.lr, tt = z.tt, wm = z.wm;
  const int cell = s * G + c;
  const size_t sb = (size_t)cell * LQ_PPL;
  // one memory round: the cell's sorted positions, its piece count and coverage start, and
  // every piece slot (whatever the count: no round waits on it) — piece ends and coefficients
  // on lane k, rows on lane t
  const int cs = rng.x, ce = rng.y;
  const int cnt_l = ld_t<COH>(r.t_cnt + cell);
  const double lo = ld_t<COH>(r.t_lo + cell);
  // (every lane loads an in-range slot and the unused ones are masked after: no per-load branch,
  // which the device-coherent loads would otherwise each get)
  const int pl = lane & (LQ_PPL - 1), tl = min(lane, N - 1);
  const double ge_v = ld_t<COH>(r.t_ge + sb + pl);
  const double ge_l = lane < LQ_PPL ? ge_v : INFINITY;
  double cf[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const double v = ld_t<COH>(r.t_cf + (sb + pl) * 8 + k);
    cf[k] = lane < LQ_PPL ? v : 0.0;
  }
  double2 ab[LQ_PPL];
#pragma unroll
  for (int k = 0; k < LQ_PPL; ++k) {
    const double2 v = ld_t<COH>(r.t_ab + (sb + k) * N + tl);
    ab[k] = lane < N ? v : make_double2(0.0, 0.0);
  }
  if (ce <= cs) return;
  const int cnt = min(max(cnt_l, 0), LQ_PPL);
  const double ge = lane < cnt ? ge_l : INFINITY;
#pragma unroll
  for (int k = 0; k < LQ_PPL; ++k) ab[k] = k < cnt ? ab[k] : make_double2(0.0, 0.0);
  // boundary j (lane j <= cnt): j = 0 the coverage start (first gamma >= lo), j >= 1 the end of
  // piece j - 1 (first gamma > ge_{j-1}); its fine bucket clamped to the cell's
  const double gprev = __shfl(ge, max(lane - 1, 0), 64);  // (every lane: no read of an inactive lane)
  const double vb = lane == 0 ? lo : gprev;
  const int fb = min(max(agg_fine(vb, wlo, fs, r.F), c * KF), (c + 1) * KF - 1);
  int qa = lane <= cnt ? ps[fb] : 0, qb = lane <= cnt ? ps[fb + 1] : 0;
  qa = min(max(qa, cs), ce);
  qb = min(max(qb, cs), ce);
  int qpos = cs;
  {
    // every boundary's candidates in flight together (one memory round, not one per boundary);
    // a bucket wider than 64 EVs falls back to agg_search's binary search
    double xg[LQ_PPL + 1];
#pragma unroll
    for (int j = 0; j <= LQ_PPL; ++j) {
      const int a0 = lqw::readlane_i(qa, j), b0 = lqw::readlane_i(qb, j);  // (j wave-uniform)
      xg[j] = (j <= cnt && b0 - a0 <= 64 && a0 + lane < b0) ? g[a0 + lane] : INFINITY;
    }
#pragma unroll
    for (int j = 0; j <= LQ_PPL; ++j) {
      if (j > cnt) continue;  // (wave-uniform)
      const int a0 = lqw::readlane_i(qa, j), b0 = lqw::readlane_i(qb, j);
      const double v = lqw::readlane_d(vb, j);
      int pj;
      if (b0 - a0 <= 64) {
        const bool before = j == 0 ? (xg[j] < v) : (xg[j] <= v);
        pj = a0 + (int)__popcll(__ballot(before && a0 + lane < b0));
      } else {
        pj = agg_search(g, a0, b0, v, j == 0, lane);
      }
      if (lane == j) qpos = pj;
    }
  }
  if (cnt == 0) qpos = ce;
  // per piece k = lane: [qpos_k, qpos_{k+1})
  const int qn = __shfl(qpos, min(lane + 1, 63), 64);
  const bool pk = lane < cnt;
  const int na = pk ? qpos : 0, nb = pk ? max(qn, qpos) : 0;
  const double n = (double)(nb - na);
  unsigned long long d1 = 0, dh = 0, dl = 0;
  double gf = 0.0, gl = 0.0;
  if (pk && nb > na) {
    d1 = z.P1[nb] - z.P1[na];
    dh = z.PH[nb] - z.PH[na];
    dl = z.PL[nb] - z.PL[na];
    gf = g[na];
    gl = g[nb - 1];
  }
  const double X1 = (double)d1;
  const double X2 = fma((double)dh, 0x1p40, (double)dl);
  const double Gm = fma(h1, X1, n * wlo);                                 // sum gamma
  const double G2 = fma(h1 * h1, X2, fma(2.0 * wlo * h1, X1, n * wlo * wlo));  // sum gamma^2
  if (pk && nb > na) {
    a.acost += fma(cf[2], G2, fma(cf[1], Gm, cf[0] * n));
    const double e_f = fma(fma(cf[5], gf, cf[4]), gf, cf[3]), e_l = fma(fma(cf[5], gl, cf[4]), gl, cf[3]);
    a.aerr = fmax(a.aerr, fmax(fmax(e_f, e_l), 0.0));
    const double a0 = cf[6], b0 = cf[7];
    const double sw0 = fma(b0, Gm, a0 * n), sw02 = fma(b0 * b0, G2, fma(2.0 * a0 * b0, Gm, a0 * a0 * n));
    a.ap0 += q.theta * fma(l1, sw0, l2 * fma(wm, n, -sw0)) + fma(q.q_scale, l3, tt * lr) * sw02;  // lompc.py:164-170
  }
  // per-stage sums of w: sum over pieces of n_k a_kt + Gamma_k b_kt (lane t)
#pragma unroll
  for (int k = 0; k < LQ_PPL; ++k) {
    const double nk = lqw::readlane_d(n, k), gk = lqw::readlane_d(Gm, k);
    a.accw = fma(gk, ab[k].y, fma(nk, ab[k].x, a.accw));  // (slots past cnt: n = 0, Gamma = 0)
  }
  // EVs of the cell outside its certified coverage: re-solved one by one (k_finalize's method)
  const int u0 = cs, u1 = lqw::readlane_i(qpos, 0), v0 = lqw::readlane_i(qpos, cnt), v1 = ce;
  if (u1 > u0 || v1 > v0) {
    lqw::WaveSet ws;
    double l2w;
    bool bad;
    if (z.preg) load_set_regs(q, z.p1, z.p2, z.p3, lr, N, lane, ws, l2w, bad);
    else load_set<PCOH>(q, z.L, lr, N, lane, ws, l2w, bad);
    const double c0 = q.theta * q.w_max * lqw::wave_sum(l2w, N);
    const double kappa = lr / q.delta;
    const double l0[3] = {l1, l2, l3};
    const double wr = (r.w_ref && lane < N) ? r.w_ref[(size_t)s * N + lane] : 0.0;
    for (int part = 0; part < 2; ++part) {
      const int e0 = part ? v0 : u0, e1 = part ? v1 : u1;
      for (int j = e0; j < e1; ++j) {
        const double gj = g[j];
        int sl = lane < N ? (int)r.t_sl[(size_t)cell * 64 + lane] : 0;  // (COH: this lane's own store)
        double wl = 0.0, rl = 0.0;
        const bool okk = lqw::wave_solve(q, ws, gj, sl, wl, rl);
        double co, eo, po;
        wave_ev_outputs(q, ws, c0, kappa, l0, lr, wr, gj, wl, co, eo, po);
        a.accw += lane < N ? wl : 0.0;
        if (lane == 0) {
          a.acost += co;
          a.ap0 += po;
          a.aerr = fmax(a.aerr, eo * eo);
          a.nrep += okk ? 1 : 0;
          a.nfail += okk ? 0 : 1;
        }
      }
    }
  }
}

// the wave's record: lane t < N its stage sum; x0..x4 cost, price0, max err^2, repaired, failed
struct AggRec {
  double x0, x1, x2, x3, x4;
  __device__ __forceinline__ double pick(const int j) const {  // (selects: no private array)
    return j == 0 ? x0 : (j == 1 ? x1 : (j == 2 ? x2 : (j == 3 ? x3 : x4)));
  }
};
__device__ __forceinline__ AggRec agg_wave_record(const AggPart& a) {
  double xs[4] = {a.acost, a.ap0, 0.0, 0.0};
  lqw::wave_totals(xs, 64);
  return AggRec{xs[0], xs[1], lqw::wave_max(a.aerr, 64), (double)lqw::readlane_i(a.nrep, 0),
                (double)lqw::readlane_i(a.nfail, 0)};
}

// a set's closed outputs on the closing wave: lane t < N the stage sum of w, lane j < 8 stat j
struct AggSetOut {
  double sumw, stat;
};

// Set s's closing from nrec wave records, combined in record order, by ONE wave (lane = stage):
// wrec(k) lane t's stage sum of record k, xlane(k) on lane j < 5 its scalar j (each lane combines
// one scalar over the records).  WT: set outputs written through to L2, complete when this returns.
// PADDED: records nrec .. MAXREC - 1 exist and are zero (sums and maxima of nonnegative errors
// unchanged: no per-record condition)
template <bool WT>
__device__ __forceinline__ AggSetOut agg_finish_tail(const AggArgs& r, const AggSet& z, const int s, const int lane,
                                                const double v, const double xs, const double xm);

template <bool WT, bool PADDED, int MAXREC, class FW, class FX>
__device__ __forceinline__ AggSetOut agg_finish(const AggArgs& r, const AggSet& z, const int s, const int lane, const int nrec,
                                           FW wrec, FX xlane) {
  // (nrec <= MAXREC: unrolled, so register-held records stay in registers; lanes >= N sum
  // whatever they hold, unread)
  double v = 0.0, xs = 0.0, xm = 0.0;  // lane j < 5: scalar j summed / maximised over the records in order
#pragma unroll
  for (int k = 0; k < MAXREC; ++k) {
    if (PADDED || k < nrec) {  // (no early exit: it would leave the records' registers to a stack array)
      v += wrec(k);
      const double xv = xlane(k);
      xs += xv;
      xm = fmax(xm, xv);
    }
  }
  return agg_finish_tail<WT>(r, z, s, lane, v, xs, xm);
}

// agg_finish's outputs from the records' sums already formed (v: lane t's stage sum; xs / xm: lane
// j < 5's scalar summed / maximised over the records in order)
template <bool WT>
__device__ __forceinline__ AggSetOut agg_finish_tail(const AggArgs& r, const AggSet& z, const int s, const int lane,
                                                const double v, const double xs, const double xm) {
  const int N = z.N, n_s = z.n_s;
  const double xa = lane == 2 ? xm : xs;  // (scalar 2, the max error: a max)
  if (lane < N && r.set_sum_w) {
    if (WT) st_wt8(r.set_sum_w + (size_t)s * N + lane, v);
    else r.set_sum_w[(size_t)s * N + lane] = v;
  }
  const double sw0 = lqw::readlane_d(v, 0);  // (sum of w0)
  const double c = lqw::readlane_d(xa, 0), p0 = lqw::readlane_d(xa, 1), e = lqw::readlane_d(xa, 2);
  const double rr = lqw::readlane_d(xa, 3);
  double ff = lqw::readlane_d(xa, 4);
  if (!z.order_ok) ff = (double)n_s;  // gamma not ascending: every EV reported failed, nothing summed
  const double ni = (double)(n_s - (z.order_ok ? z.si.x : n_s));  // invalid gamma: after the valid ones
  double x = 0.0;
  if (lane < LOMPC_SET_STATS) {
    switch (lane) {
      case LOMPC_STAT_COUNT: x = (double)n_s; break;
      case LOMPC_STAT_SUM_W0: x = sw0; break;
      case LOMPC_STAT_SUM_PRICE0: x = p0; break;
      case LOMPC_STAT_MAX_ERR: x = sqrt(e); break;
      case LOMPC_STAT_SUM_COST: x = c; break;
      case LOMPC_STAT_N_REPAIRED: x = rr; break;
      case LOMPC_STAT_N_FAILED: x = ff; break;
      default: x = ni; break;
    }
    if (r.set_stats) {
      if (WT) st_wt8(r.set_stats + (size_t)s * LOMPC_SET_STATS + lane, x);
      else r.set_stats[(size_t)s * LOMPC_SET_STATS + lane] = x;
    }
    if (r.stats) r.stats[(size_t)s * LOMPC_SET_STATS + lane] = x;
  }
  if (lane == 0 && r.tally) {
    if (rr > 0.0) __hip_atomic_fetch_add(r.tally + 0, (unsigned long long)rr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ff > 0.0) __hip_atomic_fetch_add(r.tally + 1, (unsigned long long)ff, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (ni > 0.0) __hip_atomic_fetch_add(r.tally + 2, (unsigned long long)ni, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (WT) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the set outputs have reached L2
  return AggSetOut{v, x};
}

// set s by one workgroup, wave wv: cells wv, wv + nw, ...; the waves' records combined in wave order
template <int NT>
__device__ __forceinline__ void agg_set_block(const AggArgs& r, const int s, double (*s_w)[LOMPC_MAX_N], double (*s_x)[8]) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
  const AggSet z = agg_set_init<NT>(r, s);
  lq_tab_init(*z.q);  // (the individual re-solves' box table)
  AggPart a;
  for (int c = wv; z.order_ok && c < z.G; c += nw) agg_cell<NT, false>(r, z, s, c, agg_cell_range(z, c), lane, a);
  const AggRec x = agg_wave_record(a);
  if (lane < z.N) s_w[wv][lane] = a.accw;
  if (lane < 5) s_x[wv][lane] = x.pick(lane);
  __syncthreads();
  if (wv == 0)
    agg_finish<false, false, LQ_AGG_W>(r, z, s, lane, nw, [&](int k) { return s_w[k][lane]; }, [&](int k) { return s_x[k][min(lane, 7)]; });
}

// one workgroup per set
template <int NT>
__global__ __launch_bounds__(64 * LQ_AGG_W) void k_agg(AggArgs r) {
  __shared__ double s_w[LQ_AGG_W][LOMPC_MAX_N];
  __shared__ double s_x[LQ_AGG_W][8];  // cost, price0, max err^2, repaired, failed
  if (r.skip && *r.skip) return;
  agg_set_block<NT>(r, (int)blockIdx.x, s_w, s_x);
}

// The wide form over gamma-sorted sets (lompc_plan_run_steps without per-EV outputs): one workgroup
// per (run, set) of a path group, after the group's k_paths launch — run j's prices at lmbd + j
// lm_stride, its tables in ring slot j % slots, its set outputs at out_base + (rel ? j - run0 : j)
// stride (rel: the group's contiguous send records).  k_agg's per-set work with the same cell-to-wave
// map and record order, so the same bits as one k_agg launch per run.  Only the last run writes the
// plan's stats scratch.
struct AggsArgs {
  int run0, slots, last, rel;
  int64_t lm_stride, lr_stride, sw_stride, st_stride;
};

template <int NT>
__global__ __launch_bounds__(64 * LQ_AGG_W) void k_aggs(AggArgs r0, AggsArgs x) {
  __shared__ double s_w[LQ_AGG_W][LOMPC_MAX_N];
  __shared__ double s_x[LQ_AGG_W][8];
  const int rr = (int)blockIdx.x / r0.S, s = (int)blockIdx.x - rr * r0.S;
  const int j = x.run0 + rr, jo = x.rel ? rr : j;
  const int64_t o = (int64_t)(j % x.slots) * r0.S * r0.G;
  const int N = NT ? NT : r0.N;
  AggArgs r = r0;
  r.lmbd = r0.lmbd + (size_t)j * x.lm_stride;
  r.lmbd_r = r0.lmbd_r + (size_t)j * x.lr_stride;
  r.t_cnt = r0.t_cnt + o;
  r.t_lo = r0.t_lo + o;
  r.t_sl = r0.t_sl + o * 64;
  r.t_ge = r0.t_ge + o * LQ_PPL;
  r.t_cf = r0.t_cf + o * LQ_PPL * 8;
  r.t_ab = r0.t_ab + o * LQ_PPL * N;
  r.set_sum_w = r0.set_sum_w ? r0.set_sum_w + (size_t)jo * x.sw_stride : nullptr;
  r.set_stats = r0.set_stats ? r0.set_stats + (size_t)jo * x.st_stride : nullptr;
  if (j != x.last) {  // (a zero stride: every run's outputs at one place, the last run's win)
    r.stats = nullptr;
    if (!x.rel && x.sw_stride == 0) r.set_sum_w = nullptr;
    if (!x.rel && x.st_stride == 0) r.set_stats = nullptr;
  }
  agg_set_block<NT>(r, s, s_w, s_x);
}

typedef void (*AggKernel)(AggArgs);
AggKernel agg_kernel(int N) {
  switch (N) {
    case 12: return k_agg<12>;
    case 16: return k_agg<16>;
    case 24: return k_agg<24>;
    case 48: return k_agg<48>;
    default: return k_agg<0>;
  }
}

typedef void (*AggsKernel)(AggArgs, AggsArgs);
AggsKernel aggs_kernel(int N) {
  switch (N) {
    case 12: return k_aggs<12>;
    case 16: return k_aggs<16>;
    case 24: return k_aggs<24>;
    case 48: return k_aggs<48>;
    default: return k_aggs<0>;
  }
}
