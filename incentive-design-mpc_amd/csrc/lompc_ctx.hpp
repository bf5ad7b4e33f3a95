// lompc_ctx.hpp — host-side state of the C-ABI objects (include/lompc_amd.h):
// lompc_ctx (one EV type on one device, LoMPC.__init__, lompc.py:30-71) and
// lompc_plan (a fixed EV batch solved repeatedly at new prices: the per-EV loops of
// price_solver.py:203-209 / :280-283 over one price loop or one time step).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <string>
#include <vector>

#include "lompc_qp.hpp"
#include "../../include/lompc_amd.h"

#define NPX 7  // partial / reduction record: [0,N) sum_w, then NPX scalars
enum {      // columns after the N sums
  PX_COST = 0,
  PX_PRICE0 = 1,
  PX_MAX_ERR = 2,
  PX_N_OK = 3,
  PX_N_REPAIRED = 4,
  PX_N_FAILED = 5,
  PX_N_INVALID = 6
};

struct lompc_ctx {
  int device = 0;
  int N = 0;
  int ev_type = 0;
  int mode = LOMPC_MODE_PATH;
  int nmax = 0;
  QPConst q{};
  // parameter sets of the last lompc_set_params (PATH mode reads them at solve time)
  int64_t S = 0, S_cap = 0;
  const double* p_lmbd = nullptr;
  const double* p_lmbd_r = nullptr;
  const double* p_w_ref = nullptr;
  const double* p_gamma_ref = nullptr;
  int params_mode = -1;
  // DIRECT mode: derived set records + central working sets (k_central)
  double* d_setdata = nullptr;
  uint8_t* d_central = nullptr;
  int* d_errflag = nullptr;
  // DIRECT mode batch workspaces
  int64_t nblk_cap = 0, soff_cap = 0, stats_cap = 0;
  double* d_partial = nullptr;
  int* d_fail_cnt = nullptr;
  uint8_t* d_fail_lane = nullptr;
  int* d_blk_prefix = nullptr;
  int64_t* d_set_off = nullptr;
  longlong4* d_blk_info = nullptr;
  longlong4* h_pin_info = nullptr;
  int64_t info_cap = 0;
  double* d_stats = nullptr;  // [S][LOMPC_SET_STATS] of the last batch (lompc_last_status)
  int64_t stats_S = 0;
  int* h_pin_prefix = nullptr;
  int64_t* h_pin_off = nullptr;
  hipEvent_t ev_map = nullptr;
  std::vector<int64_t> last_off;
  void* last_off_stream = nullptr;
  // PATH mode: the transient plan behind lompc_solve_batch (re-prepared every call)
  struct lompc_plan* tplan = nullptr;
  // single-solve scratch (3N + N + 8 doubles)
  double* d_single = nullptr;
  int8_t* d_single_status = nullptr;
  // profiling of the per-EV kernel
  bool prof = false;
  std::vector<hipEvent_t> prof_ev;    // pairs recorded since the last read
  std::vector<hipEvent_t> prof_pool;  // recycled events (no creation inside timed loops)
  double prof_ms = 0.0;
  int64_t prof_n = 0;
  std::string err;
};

#define LQ_PLAN_MAX_CTX LOMPC_PLAN_MAX_CTX

struct CtxEnds {  // cumulative set counts of a plan's contexts (a kernel argument: no memory round)
  int end[LQ_PLAN_MAX_CTX];
};

// one copy of the path table (k_path writes it, k_eval / k_agg / k_finalize read it)
struct PathTab {
  int* cnt = nullptr;
  double* lo = nullptr;
  double* ge = nullptr;
  double* cf = nullptr;
  double2* ab = nullptr;
  uint8_t* sl = nullptr;
};

struct lompc_plan {
  int device = 0;
  int N = 0;
  int nctx = 0;
  int flags = 0;
  lompc_ctx* ctx[LQ_PLAN_MAX_CTX] = {};
  char* d_meta = nullptr;       // host-built metadata, one block (the four views below)
  QPConst* d_q = nullptr;       // [nctx]
  int64_t B = 0, S = 0;
  int G = 0;                    // gamma cells per set (k_path waves per set)
  int nblk = 0;                 // k_eval workgroups (blocks of one set's EVs)
  int n_cu = 0;
  bool close = false;           // the sets' closing inside k_eval (no k_finalize launch)
  bool close_no_w = true;       // ... in runs without w output
  int* d_arrive = nullptr;      // [S] k_eval's per-set arrival counters (close mode)
  int n_empty = 0;              // sets without EVs (closed by one extra k_eval workgroup)
  CtxEnds ce{};                 // set s belongs to context #{k : ce.end[k] <= s}
  int eval_occ = 1;             // k_eval workgroups resident per CU (occupancy query)
  int64_t eval_occ_key = -1;    // (N, LDS pieces) it was queried for
  int64_t cap_S = 0, cap_blk = 0, cap_cells = 0;
  const double* gamma = nullptr;  // caller's [B] (read at every run)
  const double* w_ref = nullptr;  // caller's [S][N] (read at every run) or null
  double* d_stats_own = nullptr;  // [S][8] when the plan owns its status rows
  double* d_stats = nullptr;      // where k_finalize writes the status rows
  // device workspaces
  int64_t* d_set_off = nullptr;   // [S+1]                          (view of d_meta)
  int* d_blk_prefix = nullptr;    // [S+1] k_eval workgroups per set (view of d_meta)
  int4* d_blk = nullptr;          // [nblk] (set, first EV, end EV, -) (view of d_meta)
  double* d_window = nullptr;     // [S][2] (lo, hi) of the set's valid gamma, widened
  unsigned long long* d_wacc = nullptr;  // [S][3] k_plan_window accumulators (~lo bits, hi bits,
                                         // blocks done), zero between launches
  double* d_partial = nullptr;    // [nblk][N+NPX] k_eval workgroup records
  int* d_fail_cnt = nullptr;      // [nblk][waves] EVs listed for k_finalize's individual re-solve
  int* d_fail_idx = nullptr;      // [nblk][EVs]
  // path table: per cell piece count / coverage start / working set and LQ_PPL piece slots
  int* t_cnt = nullptr;
  double* t_lo = nullptr;
  double* t_ge = nullptr;
  double* t_cf = nullptr;
  double2* t_ab = nullptr;
  uint8_t* t_sl = nullptr;
  uint8_t* d_ws = nullptr;        // [S*G][64] working set at each cell start (warm start)
  // lompc_plan_run_steps, stepped form (k_step: run k + 1's path, run k's evaluation and run k - 1's
  // closing in one launch): two path tables, three copies of the cell-start working sets, two sets of
  // evaluation records and the evaluation block map sized for the slots the path leaves
  struct Stepped {
    bool ok = false;              // built for the current prepare
    int nblk = 0, np_wg = 0;      // evaluation workgroups, path workgroups of a launch
    char* d_map = nullptr;        // int4 blocks [nblk] | int prefix [S+1]
    char* h_map = nullptr;        // pinned staging of the map
    int64_t cap_map = 0;
    PathTab tab[2]{};
    uint8_t* sl3 = nullptr;       // [3][S*G][64]
    int64_t cap_cells = 0;
    double* part[2] = {nullptr, nullptr};
    int* fcnt[2] = {nullptr, nullptr};
    int* fidx[2] = {nullptr, nullptr};
    int64_t cap_blk = 0;
    int occ = 0;                  // evaluation workgroups per CU (occupancy query)
    int64_t occ_key = -1;         // ... for this horizon, cell count and kernel
    bool wide = false;            // the map is the wide form's (no path workgroups in its launches)
    bool stg = false;             // ... for k_evals_st (compact tables, blocks of <= LQ_EVALS_MAXB EVs)
    PathTab wt{};                 // wide form: a ring of per-run path tables, slot-major
    int64_t cap_wt = 0;           // its capacity in cells (slots x S x G)
    double* rpart = nullptr;      // wide form, batched evaluation (k_evals / k_closes): per-run record
    int* rfcnt = nullptr;         // slots of a path group, [runs][nblk][...]
    int* rfidx = nullptr;
    int64_t cap_rrec = 0;         // their capacity in blocks (runs x nblk)
  } stp;
  int* d_errflag = nullptr;
  unsigned long long* d_tally = nullptr;  // [3] EVs repaired / failed / invalid over every run since
                                          // the last lompc_plan_status (sticky, read and zeroed there)
  // cross-rank combine of the per-set reductions (lompc_plan_set_comm): the sets close into the
  // packed send record [S][N] sums | [S][8] stats, one all-gather, one rank-ordered combine kernel
  struct lompc_comm* comm = nullptr;
  double* d_xsend = nullptr;      // [S (N + 8)]
  double* d_xrecv = nullptr;      // [nranks][S (N + 8)]
  int64_t cap_xsend = 0, cap_xrecv = 0;
  // device-resident price loop (lompc_loop.hip): while it runs every plan kernel first reads
  // *skip and returns when the loop has finished (iterations enqueued ahead of the convergence)
  const int* skip = nullptr;
  int* d_loop = nullptr;          // [LQ_LOOP_CTL] ints | doubles: the loop's device state
  struct lq_host_loop* h_loop = nullptr;  // pinned: progress / done / results, written by k_loop_step
  double* h_dec = nullptr;        // pinned [2][max_iter]: dual cost decreases (actual, predicted)
  int cap_loop_iter = 0;
  double* d_aggrec = nullptr;     // [S * G][LQ_AGG_REC] k_loop_iter's cell records
  int64_t cap_aggrec = 0;
  int64_t aggrec_zero = -1;       // offset of its zeroed padding record (-1: none yet)
  // gamma-sorted sets (LOMPC_PLAN_SORTED_GAMMA, lompc_agg.hpp): runs without per-EV outputs
  // aggregate per piece from prefix sums built at prepare (k_agg) instead of k_eval
  bool sorted = false;
  int nsblk = 0, aggF = 0;
  int4* d_sblk = nullptr;          // [nsblk] (view of d_meta)
  int* d_sblk_prefix = nullptr;    // [S+1]   (view of d_meta)
  unsigned long long* d_bsum = nullptr;  // [nsblk][4]
  unsigned long long* d_P = nullptr;     // [3][B + S]
  int* d_pos = nullptr;                  // [S][F + 1]
  int4* d_sinfo = nullptr;               // [S]
  int64_t cap_sblk = 0, cap_P = 0, cap_pos = 0, cap_sinfo = 0;
  // pinned staging of the host arrays
  char* h_buf = nullptr;
  int64_t cap_h = 0;
  int64_t reserve_B = 0;  // lompc_plan_reserve: batch size the buffers are sized for when they first grow
  int64_t h_off_at = 0;           // byte offset of the set offsets in h_buf
  hipEvent_t ev_stage = nullptr;
  // HIP-event profiling, per kernel (LOMPC_PLAN_K_*): enabled mask, pairs since the last read
  int prof = 0;
  std::vector<hipEvent_t> prof_ev[LOMPC_PLAN_KERNELS], prof_pool;
  std::vector<int> prof_mult[LOMPC_PLAN_KERNELS];  // launches each recorded pair spans (1, or a span)
  double prof_ms[LOMPC_PLAN_KERNELS] = {0.0, 0.0, 0.0};
  int64_t prof_n[LOMPC_PLAN_KERNELS] = {0, 0, 0};
  std::string err;
};

#define HIPCHK(obj, call)                                                        \
  do {                                                                           \
    hipError_t e__ = (call);                                                     \
    if (e__ != hipSuccess) {                                                     \
      if (obj) (obj)->err = std::string(#call) + ": " + hipGetErrorString(e__); \
      return LOMPC_ERR_HIP;                                                      \
    }                                                                            \
  } while (0)

template <typename O>
static inline int fail_arg(O* o, const char* msg) {
  if (o) o->err = msg;
  return LOMPC_ERR_INVALID_ARG;
}

template <typename O, typename T>
static inline int grow(O* o, T** p, size_t n_elems) {
  if (*p) {
    hipError_t e = hipFree(*p);
    if (e != hipSuccess) {
      o->err = std::string("hipFree: ") + hipGetErrorString(e);
      return LOMPC_ERR_HIP;
    }
  }
  *p = nullptr;
  hipError_t e = hipMalloc((void**)p, std::max<size_t>(n_elems, 1) * sizeof(T));
  if (e != hipSuccess) {
    o->err = std::string("hipMalloc: ") + hipGetErrorString(e);
    return LOMPC_ERR_HIP;
  }
  return LOMPC_OK;
}

// Shared by lompc_kernels.hip (transient plan of lompc_solve_batch) and lompc_plan.hip.
int lq_plan_prepare(lompc_plan* p, int nctx, lompc_ctx* const* ctxs, const int64_t* sets_per_ctx, int64_t B,
                    const double* gamma, const int64_t* set_offsets, const double* w_ref, int flags,
                    hipStream_t st);
int lq_plan_launch(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* w, double* cost, double* w0,
                   int8_t* status, double* set_sum_w, double* set_stats, hipStream_t st, lompc_ctx* prof_ctx);
void lq_plan_free(lompc_plan* p);

// RCCL communicator of the extension (lompc_comm.cpp; RCCL resolved at run time)
struct lompc_comm {
  void* nccl = nullptr;  // ncclComm_t
  int nranks = 1, rank = 0, device = 0;
  std::string err;
};
int lq_comm_allgather(lompc_comm* c, const double* send, double* recv, size_t count, hipStream_t st);

// price loops (lompc_plan.hip: host form; lompc_loop.hip: device-resident form and the C-ABI entry)
const char* lq_failed_text(lompc_plan* p, hipStream_t st);
// one device-loop iteration as ONE launch (k_loop_iter: path + aggregation + the loop step) when
// the plan allows it (gamma-sorted sets, no communicator, at most LQ_LOOP_G cells per set)
struct StepArgs;
bool lq_loop_fusable(const lompc_plan* p, bool persistent);
int lq_launch_loop_iter(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                        const StepArgs& sa, int m, hipStream_t st);
int lq_launch_loop_run(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                       const StepArgs& sa, hipStream_t st);
int lq_launch_loop(lompc_plan* p, const double* lmbd, const double* lmbd_r, double* set_sum_w, double* set_stats,
                   const StepArgs& sa, int m, hipStream_t st, bool persistent);
int lq_price_loop_host(lompc_plan* p, const lompc_price_loop_args* a, double* lmbd, double* w_k, double* dual_cost,
                       double* dec_actual, double* dec_pred, int* iterations, double* errs, hipStream_t st);
