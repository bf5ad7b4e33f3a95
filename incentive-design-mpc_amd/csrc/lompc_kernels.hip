// lompc_kernels.hip — MI355X (gfx950) contexts, the DIRECT-mode kernels and the per-context
// C-ABI of include/lompc_amd.h.
//
// Hot path replaced: LoMPC.solve_lompc (chargingstation/lompc.py:137-156) called once
// per EV from PriceSolver._get_w_err (price_solver.py:203-209) and
// PriceSolver.get_w0_price0 (price_solver.py:280-283).
//
// PATH mode (default) runs through a plan (lompc_plan.hip): lompc_solve_batch prepares the
// context's transient plan for the batch and launches k_solve + k_reduce with the parameter
// sets recorded by lompc_set_params.
// DIRECT mode (this file), one batched solve = K1 -> K2d -> K3 on one stream:
//   K1  k_central   one wave per parameter set: derived set record + the central solution's
//                   working set (wave-parallel PDAS at gamma_ref).
//   K2d k_direct    every EV solved by its own lane (PDAS warm-started from the central
//                   working set) and KKT-certified; LDS-tile epilogue with coalesced w stores
//                   and deterministic per-workgroup column sums; uncertified EVs listed for K3.
//   K3  k_finalize  per set: re-solves the listed EVs with the whole wave, then the
//                   deterministic reduction of the workgroup partials.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <vector>

#include "lompc_ctx.hpp"
#include "lompc_wave.hpp"

#define EVAL_BLOCK 64  // one wave per workgroup
struct KArgs {
  int64_t B;
  int S;
  int nblk;
  int want_err;
  int pad;
  const double* gamma;
  const int* blk_prefix;       // [S+1]
  const int64_t* set_off;      // [S+1]
  const longlong4* blk_info;   // [nblk]  (set, first EV, end EV, -)
  const double* setdata;   // [S][SD]
  const uint8_t* central;  // [S][LQ_STB]
  double* w;
  double* cost;
  double* w0;
  int8_t* status;
  double* partial;    // [nblk][N+NPX]
  int* fail_cnt;      // [nblk]      EVs of the workgroup left for the repair pass
  uint8_t* fail_lane; // [nblk][64]  their lanes, ascending
};

// block -> (set, first EV, end of set) for set-contiguous batches: one scalar load
__device__ __forceinline__ void block_set(const KArgs& a, int b, int& s, int64_t& start, int64_t& end) {
  const longlong4 info = a.blk_info[b];
  s = (int)info.x;
  start = info.y;
  end = info.z;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Cost / A_bar error / price0 of the QP solved by the whole wave (lane t = w_t),
// the wave form of lq_outputs.  Result valid on every lane.
__device__ __forceinline__ EVOut wave_outputs(const QPConst& q, const double* __restrict__ sd, double gamma,
                                              int lane, double w, bool want_err) {
  const int N = q.N;
  const bool act = lane < N;
  lqw::Aff<2> h = lqw::Aff<2>::identity();  // prefix sums of w and of (w - w_ref)
  const double wr = act ? sd[2 * N + lane] : 0.0;
  if (act) {
    h.B[0] = w;
    h.B[1] = w - wr;
  }
  const lqw::Aff<2> Y = lqw::wave_scan(h);
  const double y = Y.B[0], ey = Y.B[1];
  double term = 0.0, eyy = 0.0, edd = 0.0, pwl = 0.0;
  if (act) {
    const double d = sd[lane], e = sd[N + lane];
    term = 0.5 * q.c * y * y - q.c * gamma * y + w * fma(0.5 * d, w, e);
    if (!q.ev_small) pwl = lq_pwl(w * q.inv_wmax);
    eyy = ey * ey;
    edd = (w - wr) * (w - wr);
  }
  const double tw = q.theta * q.w_max;
  EVOut o;
  o.cost = wave_sum(term) + sd[3 * N + 0] + (q.ev_small ? 0.0 : tw * tw * wave_sum(pwl));
  o.err = want_err ? sqrt(wave_sum(eyy) + sd[3 * N + 5] * wave_sum(edd)) : 0.0;
  const double w0 = __shfl(w, 0, 64);
  o.price0 = lq_price0(q, sd, w0);
  return o;
}

// write-through (sc1) stores: 16 B through a buffer descriptor (aux 16 = sc1), 8 B as a relaxed
// agent-scope atomic store (global_store_dwordx2 ... sc1)
typedef unsigned int lq_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_wt16(__amdgpu_buffer_rsrc_t rs, int off, double x, double y) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(lq_v4u, make_double2(x, y)), rs, off, 0, 16);
}
__device__ __forceinline__ void st_wt8(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Epilogue of k_direct for one wave of EVs [start, start+64) of set s: ok lanes carry a
// certified w[] and outputs; valid-but-not-ok lanes are listed for the repair pass in
// k_finalize (their rows are rewritten there).
template <int NMAX>
__device__ __forceinline__ void ev_epilogue(const QPConst& q, const int N, const KArgs& a, int b, int64_t start,
                                            int64_t end, bool valid, bool ok, const double (&w)[NMAX],
                                            const EVOut& o) {
  __shared__ double tile[EVAL_BLOCK * (NMAX + 3)];
  const int TS = N + 3;  // odd for even N: conflict-free row-per-lane ds_write_b64
  const int lane = threadIdx.x;
  const int64_t i = start + lane;
  const bool active = i < end;
  const double fill = valid ? 0.0 : NAN;
#pragma unroll
  for (int t = 0; t < NMAX; ++t)
    if (t < N) tile[lane * TS + t] = ok ? w[t] : fill;
  tile[lane * TS + N] = ok ? o.cost : fill;
  tile[lane * TS + N + 1] = ok ? o.price0 : 0.0;
  tile[lane * TS + N + 2] = ok ? o.err : 0.0;
  const unsigned long long okm = __ballot(ok);
  const unsigned long long fm = __ballot(valid && !ok);
  const unsigned long long im = __ballot(active && !valid);
  if (valid && !ok) a.fail_lane[(size_t)b * EVAL_BLOCK + __popcll(fm & ((1ull << lane) - 1ull))] = (uint8_t)lane;
  if (lane == 0) a.fail_cnt[b] = __popcll(fm);
  __syncthreads();
  // coalesced WRITE-THROUGH stores (row-major w[B][N]): sc1 stores leave no dirty lines in the
  // XCD's L2, so the kernel boundary behind this launch has no L2 writeback of the outputs to
  // wait for (MI355X_MICROARCH.md: boundary + B / 6 TB/s for B dirty bytes; 16-B sc1 ~ plain)
  const int nrow = (int)min((int64_t)EVAL_BLOCK, end - start);
  if (a.w && nrow > 0) {
    double* wo = a.w + (size_t)start * N;
    if (nrow == EVAL_BLOCK && (N % 2) == 0) {  // full tile, 16 B per lane (start*N*8 is 16-B aligned)
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(wo, (short)0, EVAL_BLOCK * N * (int)sizeof(double), 0x00020000);
#pragma unroll
      for (int r = 0; r < NMAX / 2; ++r) {
        if (r < N / 2) {
          const int e = 2 * (lane + EVAL_BLOCK * r);  // even element index
          const int row = e / N, col = e - row * N;
          st_wt16(rs, (lane + EVAL_BLOCK * r) * 16, tile[row * TS + col], tile[row * TS + col + 1]);
        }
      }
    } else {
      const int tot = nrow * N;
      const int q64 = EVAL_BLOCK / N, r64 = EVAL_BLOCK % N;
      int row = lane / N, col = lane % N;
      for (int e = lane; e < tot; e += EVAL_BLOCK) {
        st_wt8(wo + e, tile[row * TS + col]);
        row += q64;
        col += r64;
        if (col >= N) {
          col -= N;
          row += 1;
        }
      }
    }
  }
  if (active) {
    if (a.cost) st_wt8(a.cost + i, tile[lane * TS + N]);
    if (a.w0) st_wt8(a.w0 + i, tile[lane * TS + 0]);
    if (a.status) a.status[i] = !valid ? LOMPC_QP_INVALID : (ok ? LOMPC_QP_OK : LOMPC_QP_FAILED);
  }
  // per-workgroup partials: column sums over the certified rows (max for the error);
  // lanes l and l+32 each sum half of the rows of column l, then combine
  double* part = a.partial + (size_t)b * (N + NPX);
  const int half = lane >> 5;
  for (int c0 = 0; c0 < TS; c0 += 32) {
    const int c = c0 + (lane & 31);
    const bool is_max = (c == N + PX_MAX_ERR);
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    if (c < TS) {
#pragma unroll
      for (int rr = 0; rr < EVAL_BLOCK / 2; ++rr) {
        const int r = half * (EVAL_BLOCK / 2) + rr;
        const double v = ((okm >> r) & 1ull) ? tile[r * TS + c] : 0.0;
        acc[rr & 3] = is_max ? fmax(acc[rr & 3], v) : acc[rr & 3] + v;
      }
    }
    double v = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
    const double o2 = __shfl_xor(v, 32, 64);
    v = is_max ? fmax(v, o2) : v + o2;
    if (half == 0 && c < TS) part[c] = v;
  }
  if (lane == 0) {
    part[N + PX_N_OK] = (double)__popcll(okm);
    part[N + PX_N_REPAIRED] = 0.0;
    part[N + PX_N_FAILED] = (double)__popcll(fm);  // pending, re-solved in k_finalize
    part[N + PX_N_INVALID] = (double)__popcll(im);
  }
}

// ------------------------------------------------------------------- K1 (DIRECT)
struct CentralArgs {
  int S, pad;
  const double* lmbd;
  const double* lmbd_r;
  const double* w_ref;
  const double* gamma_ref;
  double* setdata;
  uint8_t* central;
  int* errflag;
};

// One wave per parameter set: the derived set record (d, e, w_ref, c0, price-0 scalars,
// kappa) and the central solution's working set at gamma_ref (the warm start of k_direct).
__global__ __launch_bounds__(64) void k_central(QPConst q, CentralArgs pa) {
  lq_tab_init(q);
  const int lane = threadIdx.x;
  const int N = q.N;
  const int s = blockIdx.x;
  const double* L = pa.lmbd + (size_t)s * 3 * N;
  const double lr = pa.lmbd_r[s];
  const double tt = q.theta * q.theta;
  lqw::WaveSet ws;
  ws.N = N;
  ws.lane = lane;
  double l2 = 0.0;
  if (lane < N) {
    const double l1 = L[lane], l3 = L[2 * N + lane];
    l2 = L[N + lane];
    if (!(l1 >= 0.0 && l2 >= 0.0 && l3 >= 0.0)) atomicOr(pa.errflag, 1);
    ws.d_nat = 2.0 * lr * tt + 2.0 * q.q_scale * l3 + q.dsmall;
    ws.e_nat = q.theta * (l1 - l2);
  } else {
    ws.d_nat = ws.e_nat = 0.0;
  }
  const double wr_nat = (pa.w_ref && lane < N) ? pa.w_ref[(size_t)s * N + lane] : 0.0;
  const double c0 = q.theta * q.w_max * lqw::wave_sum(l2, N);  // lompc.py:128
  double* out = pa.setdata + (size_t)s * lq_sd(N);
  if (lane < N) {
    out[lane] = ws.d_nat;
    out[N + lane] = ws.e_nat;
    out[2 * N + lane] = wr_nat;
  }
  if (lane == 0) {
    if (!(lr >= 0.0)) atomicOr(pa.errflag, 1);
    out[3 * N + 0] = c0;
    out[3 * N + 1] = L[0];
    out[3 * N + 2] = L[N];
    out[3 * N + 3] = L[2 * N];
    out[3 * N + 4] = lr;
    out[3 * N + 5] = lr / q.delta;  // kappa, price_solver.py:191
    out[3 * N + 6] = pa.gamma_ref ? pa.gamma_ref[s] : 0.5 * q.y_max;
    out[3 * N + 7] = pa.w_ref ? 1.0 : 0.0;
    out[3 * N + 8] = 0.0;
    out[3 * N + 9] = 0.0;
  }
  const double g = pa.gamma_ref ? pa.gamma_ref[s] : 0.5 * q.y_max;
  int sl = lane < N ? 1 : 0;
  double w = 0.0, r = 0.0;
  if (!lqw::wave_solve(q, ws, g, sl, w, r)) sl = lane < N ? 1 : 0;
  pa.central[(size_t)s * LQ_STB + lane] = (uint8_t)(lane < N ? sl : 0);
}

// ------------------------------------------------------------------- K2d
template <int NMAX, int NT>
__global__ __launch_bounds__(EVAL_BLOCK) void k_direct(QPConst q, KArgs a) {
  lq_tab_init(q);
  const int b = blockIdx.x;
  int s;
  int64_t start, end;
  block_set(a, b, s, start, end);
  const int N = NT ? NT : q.N;
  const int lane = threadIdx.x;
  const int64_t i = start + lane;
  const bool active = i < end;
  const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
  const double g = active ? a.gamma[i] : 0.0;
  const bool valid = active && (g >= 0.0) && (g <= q.y_max);
  double w[NMAX];
#pragma unroll
  for (int t = 0; t < NMAX; ++t) w[t] = 0.0;
  bool ok = false;
  const uint8_t* cst = a.central + (size_t)s * LQ_STB;
  if (valid) {
    States<NMAX> st;
    st.load_bytes(cst);
    ok = lq_pdas<NMAX>(q, N, sd, sd + N, g, st, w, 4 * N + 8);
    if (ok) {
      lq_snap<NMAX>(N, st, w);
      ok = lq_kkt<NMAX>(q, N, sd, sd + N, g, st, w) <= q.tol_cert;
    }
  }
  EVOut o{0.0, 0.0, 0.0};
  if (ok) o = lq_outputs<NMAX>(q, N, sd, g, w, a.want_err != 0);
  ev_epilogue<NMAX>(q, N, a, b, start, end, valid, ok, w, o);
}

// ------------------------------------------------------------------- K3
// One workgroup of 1024 threads (16 waves) per set.
// (1) reduction: wave wv sums partial rows wv, wv+16, ... (lane = column), the 16 waves
//     combine in LDS in a fixed order;
// (2) repair: wave wv re-solves the listed EVs of workgroups b0+wv, b0+wv+16, ...
//     (wave_solve: PDAS from the central working set, primal active set if needed,
//     KKT-certified), writes their outputs and adds them to the reduction in a fixed order.
__global__ __launch_bounds__(1024) void k_finalize(QPConst q, KArgs a, double* __restrict__ set_sum_w,
                                                   double* __restrict__ set_stats, double* __restrict__ stats_int) {
  __shared__ double red[16][LOMPC_MAX_N + NPX + 1];
  __shared__ double rep[16][LOMPC_MAX_N + NPX + 1];
  const int s = blockIdx.x;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int N = q.N;
  const int W = N + NPX;
  const int b0 = a.blk_prefix[s], b1 = a.blk_prefix[s + 1];
  for (int c = lane; c < W; c += 64) {
    const bool is_max = (c == N + PX_MAX_ERR);
    // 16 independent (predicated) loads per round: one memory round trip per 256 partial rows
    constexpr int U = 16;
    double acc[4] = {0.0, 0.0, 0.0, 0.0};
    for (int b = b0 + wv; b < b1; b += 16 * U) {
      double v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int bb = b + 16 * u;
        v[u] = bb < b1 ? a.partial[(size_t)bb * W + c] : 0.0;  // 0: neutral for sums and for max of errors >= 0
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc[u & 3] = is_max ? fmax(acc[u & 3], v[u]) : acc[u & 3] + v[u];
    }
    red[wv][c] = is_max ? fmax(fmax(acc[0], acc[1]), fmax(acc[2], acc[3])) : (acc[0] + acc[1]) + (acc[2] + acc[3]);
  }
  __syncthreads();
  if (tid < W) {
    const int c = tid;
    const bool is_max = (c == N + PX_MAX_ERR);
    double acc = red[0][c];
    for (int k = 1; k < 16; ++k) acc = is_max ? fmax(acc, red[k][c]) : acc + red[k][c];
    red[0][c] = acc;
  }
  __syncthreads();
  const bool pending = red[0][N + PX_N_FAILED] > 0.0;  // block-uniform
  if (pending) {
    lq_tab_init(q);
    double acc_w = 0.0, acc_cost = 0.0, acc_p0 = 0.0, acc_err = 0.0;
    int nrep = 0, nfail = 0;
    const double* __restrict__ sd = a.setdata + (size_t)s * lq_sd(N);
    lqw::WaveSet ws;
    ws.load(sd, N);
    for (int b = b0 + wv; b < b1; b += 16) {
      const int nf = a.fail_cnt[b];
      for (int k = 0; k < nf; ++k) {
        const int l = a.fail_lane[(size_t)b * EVAL_BLOCK + k];
        const int64_t i = a.set_off[s] + (int64_t)(b - b0) * EVAL_BLOCK + l;
        const double g = a.gamma[i];
        int sl = a.central[(size_t)s * LQ_STB + lane];
        if (lane >= N) sl = 0;
        double wl = 0.0, rl = 0.0;
        const bool okk = lqw::wave_solve(q, ws, g, sl, wl, rl);
        const EVOut o = wave_outputs(q, sd, g, lane, wl, a.want_err != 0);
        if (a.w && lane < N) a.w[(size_t)i * N + lane] = wl;
        if (lane == 0) {
          if (a.cost) a.cost[i] = o.cost;
          if (a.w0) a.w0[i] = wl;
          if (a.status) a.status[i] = okk ? LOMPC_QP_REPAIRED : LOMPC_QP_FAILED;
        }
        acc_w += lane < N ? wl : 0.0;
        acc_cost += o.cost;
        acc_p0 += o.price0;
        acc_err = fmax(acc_err, o.err);
        nrep += okk ? 1 : 0;
        nfail += okk ? 0 : 1;
      }
    }
    if (lane < N) rep[wv][lane] = acc_w;
    if (lane == 0) {
      rep[wv][N + PX_COST] = acc_cost;
      rep[wv][N + PX_PRICE0] = acc_p0;
      rep[wv][N + PX_MAX_ERR] = acc_err;
      rep[wv][N + PX_N_OK] = (double)nrep;
      rep[wv][N + PX_N_REPAIRED] = (double)nrep;
      rep[wv][N + PX_N_FAILED] = (double)nfail;
      rep[wv][N + PX_N_INVALID] = 0.0;
    }
    __syncthreads();
    if (tid < W) {
      const int c = tid;
      const bool is_max = (c == N + PX_MAX_ERR);
      double acc = (c == N + PX_N_FAILED) ? 0.0 : red[0][c];  // pending -> replaced by real failures
      for (int k = 0; k < 16; ++k) acc = is_max ? fmax(acc, rep[k][c]) : acc + rep[k][c];
      red[0][c] = acc;
    }
    __syncthreads();
  }
  if (tid < N && set_sum_w) set_sum_w[(size_t)s * N + tid] = red[0][tid];
  if (tid == 0) {
    double row[LOMPC_SET_STATS];
    row[LOMPC_STAT_COUNT] = (double)(a.set_off[s + 1] - a.set_off[s]);
    row[LOMPC_STAT_SUM_W0] = red[0][0];
    row[LOMPC_STAT_SUM_PRICE0] = red[0][N + PX_PRICE0];
    row[LOMPC_STAT_MAX_ERR] = red[0][N + PX_MAX_ERR];
    row[LOMPC_STAT_SUM_COST] = red[0][N + PX_COST];
    row[LOMPC_STAT_N_REPAIRED] = red[0][N + PX_N_REPAIRED];
    row[LOMPC_STAT_N_FAILED] = red[0][N + PX_N_FAILED];
    row[LOMPC_STAT_N_INVALID] = red[0][N + PX_N_INVALID];
    for (int k = 0; k < LOMPC_SET_STATS; ++k) {
      if (set_stats) set_stats[(size_t)s * LOMPC_SET_STATS + k] = row[k];
      stats_int[(size_t)s * LOMPC_SET_STATS + k] = row[k];
    }
  }
}

// ===================================================================== host
static int pick_nmax(int N) {
  if (N <= 16) return 16;
  if (N <= 24) return 24;
  if (N <= 32) return 32;
  if (N <= 48) return 48;
  if (N <= 64) return 64;
  return 0;
}

// (NM, NT): exact-horizon kernels for the common N, NMAX buckets with runtime N otherwise
#define DISPATCH_N(N, nmax, ...)                                                    \
  switch (N) {                                                                      \
    case 12: { constexpr int NM = 12, NT = 12; __VA_ARGS__; } break;                \
    case 16: { constexpr int NM = 16, NT = 16; __VA_ARGS__; } break;                \
    case 24: { constexpr int NM = 24, NT = 24; __VA_ARGS__; } break;                \
    case 32: { constexpr int NM = 32, NT = 32; __VA_ARGS__; } break;                \
    case 48: { constexpr int NM = 48, NT = 48; __VA_ARGS__; } break;                \
    case 64: { constexpr int NM = 64, NT = 64; __VA_ARGS__; } break;                \
    default:                                                                        \
      switch (nmax) {                                                               \
        case 16: { constexpr int NM = 16, NT = 0; __VA_ARGS__; } break;             \
        case 24: { constexpr int NM = 24, NT = 0; __VA_ARGS__; } break;             \
        case 32: { constexpr int NM = 32, NT = 0; __VA_ARGS__; } break;             \
        case 48: { constexpr int NM = 48, NT = 0; __VA_ARGS__; } break;             \
        case 64: { constexpr int NM = 64, NT = 0; __VA_ARGS__; } break;             \
        default: break;                                                             \
      }                                                                             \
  }

static int ensure_stats(lompc_ctx* c, int64_t S) {
  if (S > c->stats_cap) {
    int rc;
    if ((rc = grow(c, &c->d_stats, (size_t)S * LOMPC_SET_STATS))) return rc;
    c->stats_cap = S;
  }
  return LOMPC_OK;
}

extern "C" {

int lompc_abi_version(void) { return LOMPC_ABI_VERSION; }

const char* lompc_status_string(int status) {
  switch (status) {
    case LOMPC_OK: return "ok";
    case LOMPC_ERR_INVALID_ARG: return "invalid argument";
    case LOMPC_ERR_NOT_CONVERGED: return "solver did not produce a certified optimum";
    case LOMPC_ERR_HIP: return "HIP runtime error";
    case LOMPC_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return "unknown status";
  }
}

const char* lompc_last_error(const lompc_ctx* ctx) { return ctx ? ctx->err.c_str() : ""; }

int lompc_create(int N, double delta, double theta, double y_max, double w_max, int ev_type, int device,
                 lompc_ctx** out) {
  if (!out) return LOMPC_ERR_INVALID_ARG;
  *out = nullptr;
  // lompc.py:36-38 (settings.py:7-9); delta > 0 keeps the QP strictly convex
  if (!(y_max >= 0.75 && y_max <= 0.9)) return LOMPC_ERR_INVALID_ARG;
  if (!(w_max > 0.0 && w_max <= 0.25)) return LOMPC_ERR_INVALID_ARG;
  if (ev_type != LOMPC_EV_SMALL && ev_type != LOMPC_EV_LARGE) return LOMPC_ERR_INVALID_ARG;
  if (!(delta > 0.0) || !(theta > 0.0) || N < 1) return LOMPC_ERR_INVALID_ARG;
  const int nmax = pick_nmax(N);
  if (!nmax) return LOMPC_ERR_UNSUPPORTED;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LOMPC_ERR_HIP;
  if (hipSetDevice(device) != hipSuccess) return LOMPC_ERR_HIP;
  lompc_ctx* c = new lompc_ctx();
  c->device = device;
  c->N = N;
  c->ev_type = ev_type;
  c->nmax = nmax;
  QPConst& q = c->q;
  q.N = N;
  q.ev_small = ev_type == LOMPC_EV_SMALL;
  q.delta = delta;
  q.theta = theta;
  q.y_max = y_max;
  q.w_max = w_max;
  q.inv_wmax = 1.0 / w_max;
  q.c = 2.0 * delta * theta * theta;        // lompc.py:71
  q.q_scale = 3.0 * theta / (4.0 * w_max);  // lompc.py:67
  q.dsmall = q.ev_small ? 2.0 * theta * theta / (0.9 * 0.9) : 0.0;  // lompc.py:105
  if (q.ev_small) {
    q.m = 1;
    q.knots[0] = 0.0;
    for (int k = 1; k <= LQ_MAXSEG; ++k) q.knots[k] = w_max;
    for (int k = 0; k < LQ_MAXSEG; ++k) q.slopes[k] = 0.0;
  } else {  // lompc.py:108-114
    q.m = 4;
    const double kr[5] = {0.0, 0.125, 0.5, 0.75, 1.0};
    const double sr[4] = {0.0, 1.0, 1.5, 2.0};
    const double sc = (theta * w_max) * (theta * w_max) / w_max;
    for (int k = 0; k < 5; ++k) q.knots[k] = w_max * kr[k];
    q.knots[4] = w_max;
    for (int k = 0; k < 4; ++k) q.slopes[k] = sc * sr[k];
  }
  // gradient magnitude: charging term c N^2 w_max, PWL slopes, prices ~ theta * lambda ~ theta^2
  q.scale = 1.0 + q.c * (double)N * (double)N * w_max + q.slopes[q.m - 1] + theta * theta;
  q.tol_switch = 1e-13 * q.scale;
  q.tol_cert = 1e-11 * q.scale;
  q.ktol = 1e-13 * w_max;
  hipError_t e;
  if ((e = hipMalloc((void**)&c->d_errflag, sizeof(int))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single, (4 * N + 8) * sizeof(double))) != hipSuccess ||
      (e = hipMalloc((void**)&c->d_single_status, 8)) != hipSuccess ||
      (e = hipEventCreateWithFlags(&c->ev_map, hipEventDisableTiming)) != hipSuccess) {
    delete c;
    return LOMPC_ERR_HIP;
  }
  (void)hipMemset(c->d_errflag, 0, sizeof(int));
  *out = c;
  return LOMPC_OK;
}

int lompc_destroy(lompc_ctx* c) {
  if (!c) return LOMPC_OK;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  if (c->tplan) lq_plan_free(c->tplan);
  void* ptrs[] = {c->d_setdata, c->d_central, c->d_errflag, c->d_partial, c->d_fail_cnt, c->d_fail_lane,
                  c->d_blk_prefix, c->d_set_off, c->d_blk_info, c->d_stats, c->d_single, c->d_single_status};
  for (void* p : ptrs)
    if (p) (void)hipFree(p);
  if (c->h_pin_prefix) (void)hipHostFree(c->h_pin_prefix);
  if (c->h_pin_off) (void)hipHostFree(c->h_pin_off);
  if (c->h_pin_info) (void)hipHostFree(c->h_pin_info);
  if (c->ev_map) (void)hipEventDestroy(c->ev_map);
  for (hipEvent_t ev : c->prof_ev) (void)hipEventDestroy(ev);
  for (hipEvent_t ev : c->prof_pool) (void)hipEventDestroy(ev);
  delete c;
  return LOMPC_OK;
}

int lompc_set_mode(lompc_ctx* c, int mode) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (mode != LOMPC_MODE_PATH && mode != LOMPC_MODE_DIRECT)
    return fail_arg(c, "mode must be LOMPC_MODE_PATH or LOMPC_MODE_DIRECT");
  c->mode = mode;
  return LOMPC_OK;
}

int lompc_get_info(const lompc_ctx* c, int* N, int* ev_type) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (N) *N = c->N;
  if (ev_type) *ev_type = c->ev_type;
  return LOMPC_OK;
}

int lompc_set_params(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, const double* w_ref,
                     const double* gamma_ref, void* stream) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (S < 1 || !lmbd || !lmbd_r) return fail_arg(c, "set_params: S >= 1 and lmbd, lmbd_r required");
  if (S > (1 << 20)) return fail_arg(c, "set_params: too many parameter sets");
  HIPCHK(c, hipSetDevice(c->device));
  c->S = S;
  c->params_mode = c->mode;
  c->p_lmbd = lmbd;
  c->p_lmbd_r = lmbd_r;
  c->p_w_ref = w_ref;
  c->p_gamma_ref = gamma_ref;
  if (c->mode != LOMPC_MODE_DIRECT) return LOMPC_OK;  // PATH: read by the solve's k_solve
  const int N = c->N;
  if (S > c->S_cap) {
    int rc;
    if ((rc = grow(c, &c->d_setdata, (size_t)S * lq_sd(N))) || (rc = grow(c, &c->d_central, (size_t)S * LQ_STB)))
      return rc;
    c->S_cap = S;
  }
  CentralArgs pa{};
  pa.S = (int)S;
  pa.lmbd = lmbd;
  pa.lmbd_r = lmbd_r;
  pa.w_ref = w_ref;
  pa.gamma_ref = gamma_ref;
  pa.setdata = c->d_setdata;
  pa.central = c->d_central;
  pa.errflag = c->d_errflag;
  hipLaunchKernelGGL(k_central, dim3((unsigned)S), dim3(64), 0, (hipStream_t)stream, c->q, pa);
  HIPCHK(c, hipGetLastError());
  return LOMPC_OK;
}

static int upload_block_map(lompc_ctx* c, const int64_t* set_off, int64_t S, int* nblk_out, hipStream_t st) {
  std::vector<int> pre(S + 1);
  int64_t nb = 0;
  pre[0] = 0;
  for (int64_t s = 0; s < S; ++s) {
    const int64_t m = set_off[s + 1] - set_off[s];
    if (m < 0) return fail_arg(c, "solve_batch: set_offsets must be non-decreasing");
    nb += (m + EVAL_BLOCK - 1) / EVAL_BLOCK;
    if (nb > (1ll << 30)) return fail_arg(c, "solve_batch: batch too large");
    pre[s + 1] = (int)nb;
  }
  *nblk_out = (int)nb;
  if (nb > c->nblk_cap) {
    int rc;
    if ((rc = grow(c, &c->d_partial, (size_t)nb * (c->N + NPX))) || (rc = grow(c, &c->d_fail_cnt, (size_t)nb)) ||
        (rc = grow(c, &c->d_fail_lane, (size_t)nb * EVAL_BLOCK)))
      return rc;
    c->nblk_cap = nb;
  }
  const bool same = (int64_t)c->last_off.size() == S + 1 && c->last_off_stream == (void*)st &&
                    memcmp(c->last_off.data(), set_off, (S + 1) * sizeof(int64_t)) == 0;
  if (same && c->d_blk_prefix) return LOMPC_OK;
  if (S + 1 > c->soff_cap) {
    int rc;
    if ((rc = grow(c, &c->d_blk_prefix, (size_t)(S + 1))) || (rc = grow(c, &c->d_set_off, (size_t)(S + 1))))
      return rc;
    if (c->h_pin_prefix) (void)hipHostFree(c->h_pin_prefix);
    if (c->h_pin_off) (void)hipHostFree(c->h_pin_off);
    c->h_pin_prefix = nullptr;
    c->h_pin_off = nullptr;
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_prefix, (S + 1) * sizeof(int), hipHostMallocDefault));
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_off, (S + 1) * sizeof(int64_t), hipHostMallocDefault));
    c->soff_cap = S + 1;
  }
  if (nb > c->info_cap) {
    int rc;
    if ((rc = grow(c, &c->d_blk_info, (size_t)nb))) return rc;
    if (c->h_pin_info) (void)hipHostFree(c->h_pin_info);
    c->h_pin_info = nullptr;
    HIPCHK(c, hipHostMalloc((void**)&c->h_pin_info, nb * sizeof(longlong4), hipHostMallocDefault));
    c->info_cap = nb;
  }
  // the pinned staging buffers may still be read by the previous upload
  HIPCHK(c, hipEventSynchronize(c->ev_map));
  memcpy(c->h_pin_prefix, pre.data(), (S + 1) * sizeof(int));
  memcpy(c->h_pin_off, set_off, (S + 1) * sizeof(int64_t));
  for (int64_t s = 0; s < S; ++s)
    for (int b = pre[s]; b < pre[s + 1]; ++b)  // (set, first EV, end EV, -)
      c->h_pin_info[b] = make_longlong4(s, set_off[s] + (int64_t)(b - pre[s]) * EVAL_BLOCK, set_off[s + 1], 0);
  HIPCHK(c, hipMemcpyAsync(c->d_blk_prefix, c->h_pin_prefix, (S + 1) * sizeof(int), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipMemcpyAsync(c->d_set_off, c->h_pin_off, (S + 1) * sizeof(int64_t), hipMemcpyHostToDevice, st));
  if (nb > 0)
    HIPCHK(c, hipMemcpyAsync(c->d_blk_info, c->h_pin_info, nb * sizeof(longlong4), hipMemcpyHostToDevice, st));
  HIPCHK(c, hipEventRecord(c->ev_map, st));
  c->last_off.assign(set_off, set_off + S + 1);
  c->last_off_stream = (void*)st;
  return LOMPC_OK;
}

// DIRECT mode: k_direct then k_finalize
static int launch_direct(lompc_ctx* c, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
                         double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats,
                         hipStream_t st) {
  int nblk = 0;
  int rc = upload_block_map(c, set_offsets, c->S, &nblk, st);
  if (rc) return rc;
  KArgs a{};
  a.B = B;
  a.S = (int)c->S;
  a.nblk = nblk;
  a.want_err = 1;
  a.gamma = gamma;
  a.blk_prefix = c->d_blk_prefix;
  a.set_off = c->d_set_off;
  a.blk_info = c->d_blk_info;
  a.setdata = c->d_setdata;
  a.central = c->d_central;
  a.w = w;
  a.cost = cost;
  a.w0 = w0;
  a.status = status;
  a.partial = c->d_partial;
  a.fail_cnt = c->d_fail_cnt;
  a.fail_lane = c->d_fail_lane;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->prof && nblk > 0) {
    for (hipEvent_t* e : {&e0, &e1}) {
      if (!c->prof_pool.empty()) {
        *e = c->prof_pool.back();
        c->prof_pool.pop_back();
      } else {
        HIPCHK(c, hipEventCreateWithFlags(e, hipEventDisableSystemFence));
      }
    }
  }
  if (nblk > 0) {
    dim3 grid((unsigned)nblk), block(EVAL_BLOCK);
    DISPATCH_N(c->N, c->nmax, hipExtLaunchKernelGGL((k_direct<NM, NT>), grid, block, 0, st, e0, e1, 0, c->q, a));
    HIPCHK(c, hipGetLastError());
    if (e0) {
      c->prof_ev.push_back(e0);
      c->prof_ev.push_back(e1);
    }
  }
  hipLaunchKernelGGL(k_finalize, dim3((unsigned)c->S), dim3(1024), 0, st, c->q, a, set_sum_w, set_stats, c->d_stats);
  HIPCHK(c, hipGetLastError());
  return LOMPC_OK;
}

int lompc_solve_batch(lompc_ctx* c, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
                      double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats,
                      void* stream) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  if (c->S < 1) return fail_arg(c, "solve_batch: call lompc_set_params first");
  if (B < 0 || !set_offsets) return fail_arg(c, "solve_batch: invalid batch");
  if (set_offsets[0] != 0 || set_offsets[c->S] != B)
    return fail_arg(c, "solve_batch: set_offsets must start at 0 and end at B");
  if (B > 0 && !gamma) return fail_arg(c, "solve_batch: gamma required");
  HIPCHK(c, hipSetDevice(c->device));
  const hipStream_t st = (hipStream_t)stream;
  int rc = ensure_stats(c, c->S);
  if (rc) return rc;
  c->stats_S = c->S;
  if (c->params_mode == LOMPC_MODE_DIRECT)
    return launch_direct(c, B, gamma, set_offsets, w, cost, w0, status, set_sum_w, set_stats, st);
  // PATH: the context's transient plan for this batch
  if (!c->tplan) c->tplan = new lompc_plan();
  lompc_plan* p = c->tplan;
  lompc_ctx* cs[1] = {c};
  const int64_t S = c->S;
  rc = lq_plan_prepare(p, 1, cs, &S, B, gamma, set_offsets, c->p_w_ref, 0, st);
  if (rc) {
    c->err = p->err;
    return rc;
  }
  p->d_stats = c->d_stats;
  rc = lq_plan_launch(p, c->p_lmbd, c->p_lmbd_r, w, cost, w0, status, set_sum_w, set_stats, st, c);
  if (rc) c->err = p->err;
  return rc;
}

int lompc_run(lompc_ctx* c, int64_t S, const double* lmbd, const double* lmbd_r, const double* w_ref,
              const double* gamma_ref, int64_t B, const double* gamma, const int64_t* set_offsets, double* w,
              double* cost, double* w0, int8_t* status, double* set_sum_w, double* set_stats, void* stream) {
  const int rc = lompc_set_params(c, S, lmbd, lmbd_r, w_ref, gamma_ref, stream);
  if (rc) return rc;
  return lompc_solve_batch(c, B, gamma, set_offsets, w, cost, w0, status, set_sum_w, set_stats, stream);
}

int lompc_last_status(lompc_ctx* c, void* stream, int64_t* n_repaired, int64_t* n_failed, int64_t* n_invalid) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  std::vector<double> h((size_t)std::max<int64_t>(c->stats_S, 1) * LOMPC_SET_STATS, 0.0);
  int ef = 0, ef2 = 0;
  if (c->stats_S > 0)
    HIPCHK(c, hipMemcpyAsync(h.data(), c->d_stats, c->stats_S * LOMPC_SET_STATS * sizeof(double),
                             hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipMemcpyAsync(&ef, c->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  if (c->tplan && c->tplan->d_errflag)
    HIPCHK(c, hipMemcpyAsync(&ef2, c->tplan->d_errflag, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  HIPCHK(c, hipStreamSynchronize((hipStream_t)stream));
  double rep = 0, fail = 0, inv = 0;
  for (int64_t s = 0; s < c->stats_S; ++s) {
    rep += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_REPAIRED];
    fail += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_FAILED];
    inv += h[s * LOMPC_SET_STATS + LOMPC_STAT_N_INVALID];
  }
  if (n_repaired) *n_repaired = (int64_t)rep;
  if (n_failed) *n_failed = (int64_t)fail;
  if (n_invalid) *n_invalid = (int64_t)inv;
  if (ef || ef2) {
    HIPCHK(c, hipMemsetAsync(c->d_errflag, 0, sizeof(int), (hipStream_t)stream));
    if (ef2) HIPCHK(c, hipMemsetAsync(c->tplan->d_errflag, 0, sizeof(int), (hipStream_t)stream));
    return fail_arg(c, "negative or NaN price parameter (lmbd >= 0, lmbd_r >= 0 required)");
  }
  return LOMPC_OK;
}

int lompc_solve_host(lompc_ctx* c, const double* lmbd, double lmbd_r, double gamma, double* w, double* cost) {
  if (!c || !lmbd) return LOMPC_ERR_INVALID_ARG;
  const int N = c->N;
  if (!(gamma <= c->q.y_max)) return fail_arg(c, "gamma <= y_max required (lompc.py:87)");
  if (!(gamma >= 0.0) || !(lmbd_r >= 0.0)) return fail_arg(c, "Parameter value must be nonnegative.");
  for (int i = 0; i < 3 * N; ++i)
    if (!(lmbd[i] >= 0.0)) return fail_arg(c, "Parameter value must be nonnegative.");
  HIPCHK(c, hipSetDevice(c->device));
  // scratch layout: [0,3N) lmbd | 3N lmbd_r | 3N+1 gamma | [3N+2, 4N+2) w | 4N+2 cost
  std::vector<double> h(4 * N + 8, 0.0);
  memcpy(h.data(), lmbd, 3 * N * sizeof(double));
  h[3 * N] = lmbd_r;
  h[3 * N + 1] = gamma;
  double* d = c->d_single;
  HIPCHK(c, hipMemcpy(d, h.data(), (3 * N + 2) * sizeof(double), hipMemcpyHostToDevice));
  const int saved = c->mode;
  c->mode = LOMPC_MODE_DIRECT;
  int rc = lompc_set_params(c, 1, d, d + 3 * N, nullptr, d + 3 * N + 1, nullptr);
  c->mode = saved;
  if (rc) return rc;
  const int64_t off[2] = {0, 1};
  rc = lompc_solve_batch(c, 1, d + 3 * N + 1, off, d + 3 * N + 2, d + 4 * N + 2, nullptr, c->d_single_status,
                         nullptr, nullptr, nullptr);
  if (rc) return rc;
  int8_t stt = 0;
  HIPCHK(c, hipMemcpy(h.data() + 3 * N + 2, d + 3 * N + 2, (N + 1) * sizeof(double), hipMemcpyDeviceToHost));
  HIPCHK(c, hipMemcpy(&stt, c->d_single_status, 1, hipMemcpyDeviceToHost));
  if (w) memcpy(w, h.data() + 3 * N + 2, N * sizeof(double));
  if (cost) *cost = h[4 * N + 2];
  if (stt == LOMPC_QP_INVALID) return fail_arg(c, "invalid gamma");
  if (stt == LOMPC_QP_FAILED) {
    c->err = "no certified optimum";
    return LOMPC_ERR_NOT_CONVERGED;
  }
  return LOMPC_OK;
}

int lompc_profile_enable(lompc_ctx* c, int enable) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  c->prof = enable != 0;
  HIPCHK(c, hipSetDevice(c->device));
  while (c->prof && c->prof_pool.size() < 512) {  // recorded pairs are recycled by lompc_profile_read
    hipEvent_t e;  // timing only: no system-scope fence (an L2 writeback) per record
    HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    c->prof_pool.push_back(e);
  }
  return LOMPC_OK;
}

int lompc_profile_read(lompc_ctx* c, double* total_ms, int64_t* launches, int reset) {
  if (!c) return LOMPC_ERR_INVALID_ARG;
  HIPCHK(c, hipSetDevice(c->device));
  for (size_t k = 0; k + 1 < c->prof_ev.size(); k += 2) {
    HIPCHK(c, hipEventSynchronize(c->prof_ev[k + 1]));
    float ms = 0.f;
    HIPCHK(c, hipEventElapsedTime(&ms, c->prof_ev[k], c->prof_ev[k + 1]));
    c->prof_ms += ms;
    c->prof_n += 1;
  }
  c->prof_pool.insert(c->prof_pool.end(), c->prof_ev.begin(), c->prof_ev.end());
  c->prof_ev.clear();
  if (total_ms) *total_ms = c->prof_ms;
  if (launches) *launches = c->prof_n;
  if (reset) {
    c->prof_ms = 0.0;
    c->prof_n = 0;
  }
  return LOMPC_OK;
}

}  // extern "C"
