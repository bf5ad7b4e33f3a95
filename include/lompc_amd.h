/*
 * lompc_amd.h — C-ABI of the MI355X-native batched LoMPC QP engine.
 *
 * Drop-in boundary for the reference's per-EV LoMPC solve
 * (AkshayThiru/incentive-design-mpc, chargingstation/lompc.py).  The reference
 * has no FFI layer: its boundary is the Python class ``LoMPC``
 * (lompc.py:29-187) whose ``solve_lompc`` (lompc.py:137-156) is called once
 * per EV from the loops in price_solver.py:203-209 and :280-283.  Every
 * entry point below names the reference interface it replaces.
 *
 * Conventions
 *   - Plain C types only (no torch / HIP types in signatures).  ``stream`` is
 *     a ``hipStream_t`` passed as ``void*`` (NULL = the legacy default stream).
 *   - "dev" pointers are device pointers owned by the caller (e.g. the
 *     data_ptr() of a PyTorch-ROCm tensor); "host" pointers are host memory.
 *   - All device work is asynchronous on ``stream`` unless stated otherwise.
 *   - Counts are int64.  Every function returns an int status (LOMPC_OK = 0).
 *   - A context is bound to one device; it is not re-entrant (the reference's
 *     ``LoMPC`` holds mutable cvx.Parameters and is not re-entrant either).
 */
#ifndef LOMPC_AMD_H
#define LOMPC_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes (mapped to the reference's Python exceptions by the shim) */
#define LOMPC_OK                0  /* success                                        */
#define LOMPC_ERR_INVALID_ARG   1  /* AssertionError / ValueError in the reference    */
#define LOMPC_ERR_NOT_CONVERGED 2  /* cvxpy SolverError                               */
#define LOMPC_ERR_HIP           3  /* HIP runtime failure                             */
#define LOMPC_ERR_UNSUPPORTED   4  /* e.g. horizon N > LOMPC_MAX_N                    */

/* ---- EV types (LoMPCConstants.ev_type, lompc.py:26) */
#define LOMPC_EV_SMALL 0
#define LOMPC_EV_LARGE 1

/* ---- solve modes */
#define LOMPC_MODE_PATH   0  /* exact solution path in gamma per (set, gamma cell), fused with the
                                per-EV evaluation; KKT-certified; individual re-solve of any EV a
                                certified piece does not cover (default)                 */
#define LOMPC_MODE_DIRECT 1  /* independent per-EV active-set solve, warm-started from the
                                set's central solution                                  */

/* ---- per-EV status values written to ``status[B]`` */
#define LOMPC_QP_OK        0 /* certified optimal (KKT residual <= tol)                 */
#define LOMPC_QP_REPAIRED  1 /* certified optimal after the per-EV active-set repair    */
#define LOMPC_QP_FAILED    2 /* no certified solution (would be SolverError)            */
#define LOMPC_QP_INVALID   3 /* gamma outside [0, y_max] or NaN (AssertionError)        */

/* ---- layout of one row of ``set_stats[S][LOMPC_SET_STATS]`` */
#define LOMPC_STAT_COUNT      0 /* number of EVs in the set                          */
#define LOMPC_STAT_SUM_W0     1 /* sum_i w_i[0]            (charging_station.py:359) */
#define LOMPC_STAT_SUM_PRICE0 2 /* sum_i get_price0(w_i)   (price_solver.py:283)     */
#define LOMPC_STAT_MAX_ERR    3 /* max_i ||w_i - w_ref||_{A_bar} (price_solver.py:207-209) */
#define LOMPC_STAT_SUM_COST   4 /* sum_i cost_i                                      */
#define LOMPC_STAT_N_REPAIRED 5 /* EVs that needed the active-set repair             */
#define LOMPC_STAT_N_FAILED   6 /* EVs without a certified solution                  */
#define LOMPC_STAT_N_INVALID  7 /* EVs with invalid gamma                            */
#define LOMPC_SET_STATS       8

#define LOMPC_MAX_N 64

typedef struct lompc_ctx lompc_ctx;

/* Create a context for one EV type and horizon on ``device``.
 * Replaces LoMPC.__init__ / _set_constants (lompc.py:30-71): validates
 * y_max in [0.75, 0.9] and w_max in (0, 0.25] (lompc.py:36-37; settings.py:7-9),
 * ev_type (lompc.py:38) and requires delta > 0 (strict convexity). */
int lompc_create(int N, double delta, double theta, double y_max, double w_max,
                 int ev_type, int device, lompc_ctx** out);

/* Release every device/host resource of the context. */
int lompc_destroy(lompc_ctx* ctx);

/* Select LOMPC_MODE_PATH (default) or LOMPC_MODE_DIRECT. */
int lompc_set_mode(lompc_ctx* ctx, int mode);

/* Load S parameter sets.
 * Replaces LoMPC._update_cvx_parameters (lompc.py:84-90) for S sets at once
 * (one set = one (EV type, partition) price vector in price_solver.py).
 * The device buffers are read by the next lompc_solve_batch (PATH mode) or by the
 * preparation kernel this call launches (DIRECT mode); keep them valid until then.
 *   lmbd   dev  [S, 3N]  unit prices lambda >= 0        (lompc.py:78)
 *   lmbd_r dev  [S]      robustness price >= 0           (lompc.py:80)
 *   w_ref  dev  [S, N]   reference w for the A_bar error (price_solver.py:196), or NULL
 *   gamma_ref dev [S]    central gamma per set (gamma_sc, price_solver.py:76), or NULL
 *                        (NULL = y_max / 2); only used by LOMPC_MODE_DIRECT */
int lompc_set_params(lompc_ctx* ctx, int64_t S, const double* lmbd,
                     const double* lmbd_r, const double* w_ref,
                     const double* gamma_ref, void* stream);

/* Solve B LoMPC QPs against the loaded parameter sets.
 * Replaces the per-EV loops of PriceSolver._get_w_err (price_solver.py:196-214)
 * and PriceSolver.get_w0_price0 (price_solver.py:272-285), each iteration of
 * which is one LoMPC.solve_lompc (lompc.py:137-156).
 *   gamma        dev  [B]      gamma_i = y_max - y0_i (price_solver.py:202)
 *   set_offsets  host [S+1]    EVs of set s are [set_offsets[s], set_offsets[s+1])
 *   w            dev  [B, N]   optimal w_i (row-major), or NULL
 *   cost         dev  [B]      optimal cost incl. constant (lompc.py:155), or NULL
 *   w0           dev  [B]      w_i[0] (price_solver.py:282), or NULL
 *   status       dev  [B]      int8 LOMPC_QP_* per EV, or NULL
 *   set_sum_w    dev  [S, N]   sum_i w_i per set (price_solver.py:205), or NULL
 *   set_stats    dev  [S, LOMPC_SET_STATS] fused per-set reductions, or NULL
 * Errors detected on device are reported through ``status``/``set_stats`` and
 * ``lompc_last_status``.  PATH mode prepares a transient plan on every call (gamma windows
 * measured, block map staged); a batch solved at many prices should use a plan
 * (lompc_plan_create) instead. */
int lompc_solve_batch(lompc_ctx* ctx, int64_t B, const double* gamma,
                      const int64_t* set_offsets, double* w, double* cost,
                      double* w0, int8_t* status, double* set_sum_w,
                      double* set_stats, void* stream);

/* lompc_set_params followed by lompc_solve_batch in ONE call (one host round
 * trip; what a batched price iteration issues).  Arguments as in the two calls. */
int lompc_run(lompc_ctx* ctx, int64_t S, const double* lmbd, const double* lmbd_r,
              const double* w_ref, const double* gamma_ref, int64_t B,
              const double* gamma, const int64_t* set_offsets, double* w,
              double* cost, double* w0, int8_t* status, double* set_sum_w,
              double* set_stats, void* stream);

/* Synchronous single-QP convenience entry with host buffers.
 * Replaces LoMPC.solve_lompc (lompc.py:137-156) one-for-one:
 *   lmbd host [3N], lmbd_r, gamma -> w host [N], *cost. */
int lompc_solve_host(lompc_ctx* ctx, const double* lmbd, double lmbd_r,
                     double gamma, double* w, double* cost);

/* Synchronise ``stream`` and report the device-side counters of the last
 * lompc_solve_batch: EVs repaired, failed, invalid (any may be NULL). */
int lompc_last_status(lompc_ctx* ctx, void* stream, int64_t* n_repaired,
                      int64_t* n_failed, int64_t* n_invalid);

/* Profiling: when enabled, every lompc_solve_batch times its per-EV evaluation
 * kernel with HIP events attached to that kernel's own dispatch on ``stream``
 * (hipExtLaunchKernel start/stop events); lompc_profile_read synchronises and
 * returns the summed milliseconds and launch count since the last reset. */
int lompc_profile_enable(lompc_ctx* ctx, int enable);
int lompc_profile_read(lompc_ctx* ctx, double* total_ms, int64_t* launches,
                       int reset);

/* Horizon N and EV type of a context. */
int lompc_get_info(const lompc_ctx* ctx, int* N, int* ev_type);

/* Human-readable text of a status code or of the context's last error. */
const char* lompc_status_string(int status);
const char* lompc_last_error(const lompc_ctx* ctx);

/* ABI version (bumped on any signature change). */
#define LOMPC_ABI_VERSION 5
int lompc_abi_version(void);

/* ---------------------------------------------------------------------------
 * Plans: a fixed EV batch solved at new prices every price iteration.
 * Replaces the per-EV loops of PriceSolver._get_w_err (price_solver.py:203-209) and
 * get_w0_price0 (price_solver.py:280-283) over the iterations of one price loop (gamma_i =
 * y_max - y0_i is fixed between set_charge_levels calls, price_solver.py:66-77), and the
 * charging station's per-type passes over all partitions (charging_station.py:275-329).
 * One plan may span several contexts (EV types) of the same horizon and device: their sets
 * are stacked (sets of ctxs[0] first) and every run is ONE fused launch over all of them.
 * ------------------------------------------------------------------------- */
typedef struct lompc_plan lompc_plan;
#define LOMPC_PLAN_MAX_CTX 4
#define LOMPC_PLAN_WARM_START 1 /* flag: start each gamma cell's exact solve from the working
                                   set the previous run of the plan ended with there (prices
                                   that change little between price iterations) */
#define LOMPC_PLAN_DIAG_REPAIR 2 /* diagnostics: no solution path, every EV takes the individual
                                    whole-wave re-solve (status REPAIRED) */
#define LOMPC_PLAN_CLOSE_IN_EVAL 8 /* the per-set reductions and re-solves inside k_eval, by each
                                      set's last-arriving workgroup, instead of the k_finalize
                                      launch, also in runs that write w rows (slower there, see
                                      DESIGN.md); runs without w output always close this way */
#define LOMPC_PLAN_SORTED_GAMMA 16 /* every set's valid gamma is ascending (invalid values after them)
                                      and gamma is not modified until the next lompc_plan_update:
                                      runs with no per-EV output (w, cost, w0, status all NULL — a
                                      price loop's) aggregate each certified piece's EVs from prefix
                                      sums built at create / update (k_agg: work per run O(pieces),
                                      not O(EVs)); a set found unsorted reports every EV failed
                                      (lompc_plan_last_error then says so) */
#define LOMPC_PLAN_CLOSE_IN_FINALIZE 32 /* runs without w output close their sets in the k_finalize
                                           launch like runs with w (default: inside k_eval); the
                                           A/B form of the close-mode parity tests */
/* gamma cells per set (1 .. 1024) instead of the plan's own choice: flags | LOMPC_PLAN_CELLS(g).
 * The answer does not depend on it (every piece is certified); it trades per-cell tracking
 * latency against cold starts. */
#define LOMPC_PLAN_CELLS_SHIFT 20
#define LOMPC_PLAN_CELLS(g) ((int)(g) << LOMPC_PLAN_CELLS_SHIFT)

/* Build a plan over B EVs grouped by set (S = sum of sets_per_ctx sets):
 *   ctxs         host [n_ctx]   contexts (same N and device), n_ctx <= LOMPC_PLAN_MAX_CTX
 *   sets_per_ctx host [n_ctx]   parameter sets of each context
 *   gamma        dev  [B]       gamma_i = y_max - y0_i, read at every run; each set's gamma
 *                               window is measured here (later values outside it are still
 *                               solved exactly, by the individual re-solve: status REPAIRED)
 *   set_offsets  host [S+1]     EVs of set s are [set_offsets[s], set_offsets[s+1])
 *   w_ref        dev  [S, N]    reference w of the A_bar error, read at every run, or NULL
 * The window measurement runs asynchronously on ``stream``. */
int lompc_plan_create(int n_ctx, lompc_ctx* const* ctxs, const int64_t* sets_per_ctx,
                      int64_t B, const double* gamma, const int64_t* set_offsets,
                      const double* w_ref, int flags, void* stream, lompc_plan** out);

/* Re-target a plan at a new batch of the same contexts and set counts (B, gamma,
 * set_offsets, w_ref as in lompc_plan_create): device workspaces, events and the pinned
 * staging are reused (grown when needed), the gamma windows re-measured on `stream`.  The
 * cheap way to move a price loop from one partition to the next. */
int lompc_plan_update(lompc_plan* plan, int64_t B, const double* gamma, const int64_t* set_offsets,
                      const double* w_ref, void* stream);

/* Size hint for a plan re-targeted at batches of varying size (a station's per-partition loop
 * plans: EVs move between partitions from step to step): when a later lompc_plan_update must
 * grow a workspace, it sizes it for batches of up to max_B EVs at once, so the plan stops
 * reallocating (each hipMalloc / hipHostMalloc costs 50-470 us of host time and synchronises the
 * device).  No allocation happens in this call; 0 clears the hint. */
int lompc_plan_reserve(lompc_plan* plan, int64_t max_B);

/* One price iteration of the whole batch: the exact LoMPC optimum of every EV at the
 * prices of its set plus the fused per-set reductions.  Outputs as lompc_solve_batch, in
 * the caller's EV order (each may be NULL):
 *   lmbd dev [S, 3N], lmbd_r dev [S]; w dev [B, N]; cost, w0 dev [B]; status dev [B];
 *   set_sum_w dev [S, N]; set_stats dev [S, LOMPC_SET_STATS]
 * Three launches on ``stream`` (per-cell solution paths, per-EV evaluation, per-set
 * reduction); no synchronisation.  A plan is not re-entrant: runs are stream-ordered. */
int lompc_plan_run(lompc_plan* plan, const double* lmbd, const double* lmbd_r, double* w,
                   double* cost, double* w0, int8_t* status, double* set_sum_w,
                   double* set_stats, void* stream);

/* n_runs consecutive independent runs (the same optima as n_runs lompc_plan_run calls) at the prices
 * lmbd + k lmbd_stride and lmbd_r + k lmbd_r_stride (k = 0 .. n_runs - 1, strides in doubles).
 * Run k's set reductions go to set_sum_w + k set_sum_w_stride and set_stats + k set_stats_stride,
 * its per-EV outputs to w + k ev_stride N, cost / w0 / status + k ev_stride (strides in elements;
 * 0 = every run writes the same rows and the last run's remain; ev_stride > 0 requires
 * ev_stride >= B), so every run of the call can be observable.  With profile_every > 0 only every
 * E-th launch carries the enabled profiling events.
 * One C-ABI call for a sequence of independent batches (a benchmark's timed steps).  Plans without
 * warm starts take the WIDE form: per group of up to 64 runs three launches — the
 * group's paths, its evaluations (each workgroup through its block of every run) and its closings —
 * and, with a communicator, ONE all-gather + combine per group.  Warm-started plans take the STEPPED
 * form: one launch carries the path of run k + 1, the evaluation of run k and the closing of run
 * k - 1.  In both forms every
 * set is closed by summing its evaluated rows (k_finalize's order), also for runs without w
 * output; lompc_plan_run on a plan without w output closes from the pieces' aggregates inside the
 * evaluation instead: the two agree to the certification tolerance (~1e-12 relative), bit for bit
 * only when the plan closes in k_finalize (tests/test_gpu_pipeline.py).  steps_flags:
 *   LOMPC_STEPS_PER_KERNEL  the same runs issued one part per launch (paths / evaluations /
 *                           closings), with the same evaluation block map, so bit for bit the same
 *                           outputs (verification / A-B)
 *   LOMPC_STEPS_SPAN_EVENTS the enabled K_EVAL timing as ONE event pair (wide form: around the first
 *                           group's evaluation launch, read back as its runs; stepped form: from the
 *                           start of the first full stepped launch to the end of the last, read back
 *                           as that many launches) — no per-launch event boundaries inside the steps */
#define LOMPC_STEPS_PER_KERNEL 1
#define LOMPC_STEPS_SPAN_EVENTS 2
int lompc_plan_run_steps(lompc_plan* plan, const double* lmbd, int64_t lmbd_stride,
                         const double* lmbd_r, int64_t lmbd_r_stride, int n_runs,
                         int profile_every, double* w, double* cost, double* w0, int8_t* status,
                         double* set_sum_w, double* set_stats, int64_t set_sum_w_stride,
                         int64_t set_stats_stride, int64_t ev_stride, int steps_flags, void* stream);

/* n_runs DEPENDENT runs: the call pattern of the reference's price loop (price_solver.py:111-140,
 * where iteration k + 1's prices are computed from iteration k's reductions), so no two runs can
 * overlap.  Run 0 at lmbd0 (dev [S, 3N]); before run k >= 1 one device launch sets, per set s and
 * price coordinate i = seg N + t,
 *   lmbd_k[s][i] = max(0, lmbd_{k-1}[s][i] + step (phi(wbar)[i] - phi(w_target[s])[i])),
 *   wbar = run k-1's set_sum_w[s] / count[s],  phi(w) = (theta w, theta (w_max - w), q_s w^2)
 * (a projected dual-gradient step, phi of lompc.py:172-177; a set without EVs keeps its prices).
 * Every run is one lompc_plan_run (three launches; with a communicator its all-gather + combine, so
 * the next prices come from the combined reductions on every rank).  Outputs: lmbd_out dev
 * [n_runs][S][3N] (every run's prices; lmbd_out == lmbd0 allowed), set_sum_w dev [n_runs][S][N],
 * set_stats dev [n_runs][S][LOMPC_SET_STATS] (required); w / cost / w0 / status as lompc_plan_run
 * (one buffer: the last run's remain).  lmbd_r dev [S], w_target dev [S][N]; step >= 0.
 * No synchronisation. */
int lompc_plan_run_chain(lompc_plan* plan, const double* lmbd0, const double* lmbd_r, const double* w_target,
                         double step, int n_runs, double* lmbd_out, double* w, double* cost, double* w0,
                         int8_t* status, double* set_sum_w, double* set_stats, void* stream);

/* The charging station's partition layout of one EV type's charge levels (replaces
 * ChargingStation._update_indices' masks, charging_station.py:111-116, and the per-partition
 * statistics of PriceSolver.set_charge_levels, price_solver.py:66-77, taken at
 * charging_station.py:196-210).  y dev [n] levels, bounds dev [P+1] the partition boundaries
 * (rng, increasing).  Sorts the levels in descending order (ys dev [n], perm dev [n] int64: ys[k] =
 * y[perm[k]]; stable: ties keep index order), so partition p — levels in [rng[p], rng[p+1]], later
 * partitions winning on shared edges — is the run [c[p+1], c[p]) with c[p] = #{y >= rng[p]}, c[0] = n,
 * c[P] = 0 (partition P-1 first); stats dev [4P + 4] = per partition (count, max, min, sum) (empty:
 * 0, -inf, +inf, 0), then (max y, min y, rng[0], rng[P]): the runs are the reference's partitions only
 * when min y >= rng[0] and max y <= rng[P] (outside it an EV keeps its previous index) — the caller
 * checks.  work: dev scratch of *work_bytes; work == NULL: *work_bytes = the size needed, nothing runs.
 * n < 2^31, 1 <= P <= 256.  Asynchronous on ``stream``. */
int lompc_levels_layout(const double* y, int64_t n, const double* bounds, int P, double* ys, int64_t* perm,
                        double* stats, void* work, size_t* work_bytes, void* stream);

/* Every partition's price-loop batch of one EV type in one launch (PriceSolver.set_charge_levels'
 * gamma = y_max - y0, price_solver.py:66-77, for each partition of charging_station.py:275-307, and
 * the central QP's gamma_sc = y_max - (max + min) / 2, price_solver.py:73-76, the plans' last set):
 * ys dev [n] the levels in storage order (e.g. lompc_levels_layout's), runs dev [P+1] the storage
 * runs' bounds (runs[0] = 0, runs[P] = n, non-decreasing), gsc dev [P] per run (read only with
 * central != 0).  gam dev [n + P central]: run k's gammas at runs[k] + k central .. runs[k+1] + k
 * central - 1 (ascending when ys is descending), its gsc at runs[k+1] + k when central.  Asynchronous. */
int lompc_levels_gamma(const double* ys, int64_t n, const int64_t* runs, int P, double y_max, int central,
                       const double* gsc, double* gam, void* stream);

/* lompc_levels_layout's stats [4P + 4] without its sort (the BiMPC's inputs need only these, so the
 * sort can run later, beside the host interior point): EV i in partition #{k in 1..P-1 : bounds[k] <=
 * y_i}; per partition (count, max, min, sum) — sums in a fixed order of their own, not the sorted
 * runs' —, then (max y, min y, bounds[0], bounds[P]).  P <= 16 (else LOMPC_ERR_UNSUPPORTED).  work /
 * work_bytes as lompc_levels_layout.  Asynchronous, deterministic. */
int lompc_levels_stats(const double* y, int64_t n, const double* bounds, int P, double* stats, void* work,
                       size_t* work_bytes, void* stream);

/* Synchronise ``stream``; EVs repaired / failed / invalid summed over EVERY run since the previous
 * lompc_plan_status call (sticky device tallies, zeroed here), so a failure in any of the runs of a
 * lompc_plan_run_steps call or of a price loop is seen.  These count this rank's EVs only; with a
 * communicator attached the set_stats outputs carry the combined counts. */
int lompc_plan_status(lompc_plan* plan, void* stream, int64_t* n_repaired,
                      int64_t* n_failed, int64_t* n_invalid);

/* Batch size, total parameter sets, gamma cells per set and k_eval workgroups of the plan, and the
 * runs per stepped launch of its lompc_plan_run_steps calls (0 before any; 1 once they have run; 2: in
 * the wide form with the staged evaluation k_evals_st, whose row sums group by seven row waves — its
 * set reductions equal single runs' to rounding, its per-EV outputs bit for bit); any pointer may be
 * null. */
int lompc_plan_get_info(const lompc_plan* plan, int64_t* B, int64_t* S, int* cells, int* eval_workgroups,
                        int* steps_group);

/* HIP-event timing of the plan's kernels (hipExtLaunchKernel start/stop events on their own
 * dispatches): enable takes a mask of (1 << LOMPC_PLAN_K_*) bits (0 = off); read synchronises
 * and returns one kernel's accumulated milliseconds and launch count since the last reset. */
#define LOMPC_PLAN_K_PATH 0  /* per-(set, gamma cell) solution paths */
#define LOMPC_PLAN_K_EVAL 1  /* per-EV evaluation (the HBM-bound kernel) */
#define LOMPC_PLAN_K_FINAL 2 /* per-set reduction + individual re-solves */
#define LOMPC_PLAN_KERNELS 3
int lompc_plan_profile_enable(lompc_plan* plan, int kernel_mask);
int lompc_plan_profile_read(lompc_plan* plan, int kernel, double* total_ms, int64_t* launches, int reset);

const char* lompc_plan_last_error(const lompc_plan* plan);
int lompc_plan_destroy(lompc_plan* plan);

/* ---------------------------------------------------------------------------
 * Sharded batches: one process per GPU, every set's EVs split across the ranks.
 * The only exchange of a price iteration is the per-set reduction record the price step
 * consumes (price_solver.py:205-214: sum of w, max A_bar error; the sums of w0 / price0 / cost
 * and the counts, charging_station.py:356-366).  A communicator attached to a plan makes every
 * run of it combine those records across the ranks on the device: the sets close into one
 * packed record, ONE ncclAllGather over xGMI on the run's stream, then one kernel sums the
 * ranks' records in rank order (max for LOMPC_STAT_MAX_ERR), so every rank holds bitwise the
 * same set_sum_w / set_stats.  Collective calls: every rank must issue the same runs in the same
 * order.  RCCL is loaded at run time (LOMPC_ERR_UNSUPPORTED when it is absent).
 * ------------------------------------------------------------------------- */
typedef struct lompc_comm lompc_comm;
#define LOMPC_COMM_ID_BYTES 128  /* sizeof(ncclUniqueId) */

/* On one rank: a fresh unique id, to be broadcast to the others (e.g. over torch.distributed). */
int lompc_comm_get_unique_id(unsigned char* id);
/* Collective over the nranks ranks: a communicator for this rank on ``device``. */
int lompc_comm_create(const unsigned char* id, int nranks, int rank, int device, lompc_comm** out);
int lompc_comm_destroy(lompc_comm* comm);
/* Attach (NULL: detach) a communicator to a plan: from the next run on, the plan's set outputs
 * are the combined records of all ranks (also inside lompc_plan_run_steps and lompc_price_loop). */
int lompc_plan_set_comm(lompc_plan* plan, lompc_comm* comm);
/* The device combine every run of a plan with a communicator issues after its ncclAllGather,
 * on its own (tests / verification): recv dev [nranks][S (N + 8)] = each rank's packed record
 * (set_sum_w [S][N] | set_stats [S][8]) -> set_sum_w dev [S][N], set_stats dev [S][8] (either may
 * be NULL), summed in rank order with LOMPC_STAT_MAX_ERR taken as the max: bitwise what
 * lompc_amd.dist.combine_set_results computes on the same bytes.  Replaces the aggregate of
 * price_solver.py:205-214 / charging_station.py:356-366 over a sharded batch.  Asynchronous on
 * ``stream`` of ``device``. */
int lompc_combine_records(const double* recv, int nranks, int64_t S, int N, double* set_sum_w,
                          double* set_stats, int device, void* stream);

/* The price loop of one (EV type, partition) on a plan holding [this partition's EVs | the
 * central QP] (PriceSolver.compute_optimal_prices, price_solver.py:106-140): repeated
 * {lompc_plan_run at lmbd_k, one D2H copy + stream sync, convergence test, lompc_price_step}
 * without returning to the caller until convergence.  On a sharded plan (communicator attached:
 * this rank's share of the partition's EVs, the central QP on one rank only, n_evs the global
 * count) every run combines the ranks' records before the copy, and every rank takes the same
 * price steps on bitwise identical inputs.  Buffers:
 *   dev_in / host_in  [2*3N | 2 | 2N] = both sets' prices, lmbd_r, w_ref (the plan reads
 *                     dev_in; host_in is pinned staging), dev_sw [2,N] / dev_st [2,8] the
 *                     plan's set outputs, host_sw / host_st pinned copies (dev_* == host_*:
 *                     the kernels write the pinned buffers directly, no copy).
 * In/out: lmbd [3N] (prev prices in, converged out), w_k [N] (central solve at lmbd).
 * Out: dual_cost (last), dec_actual / dec_pred [max_iter] (price_solver.py:133-138, with the
 * reference's lmbd_k / lmbd_k_new aliasing: the actual decrease drops the price term after
 * the first iteration), *iterations = price steps taken (the reference's `iter` at the break;
 * max_iter when the cap was hit, where the reference's `iter` is max_iter - 1),
 * errs [3] = (w_err_max, w0_err, w_avg_err) at the final prices.
 * device_loop = 1: the DEVICE-RESIDENT loop — the convergence test and the price-gradient QP run on
 * the GPU (one wave, lompc_pricewave.hpp) right after each engine call, the next prices go
 * straight into dev_in, and the host only enqueues engine calls LOMPC_LOOP_AHEAD ahead of the
 * device's progress (read from pinned memory), with no copy and no synchronisation per iteration;
 * engine calls enqueued past the convergence exit at once.  The number of engine calls enqueued
 * depends only on the iteration count, so sharded ranks issue the same collectives.  Requires
 * A_bar = A'A + kappa I (as PriceSolver passes; otherwise the host loop runs).
 * device_loop = 0: the host loop above (one D2H copy + stream sync per iteration).
 * prof (may be NULL): accumulates the loop's time per part, [LOMPC_LOOP_PROF] entries: */
#define LOMPC_LOOP_PROF_ITERS  0 /* engine calls (plan runs)                                     */
#define LOMPC_LOOP_PROF_WALL   1 /* us, host wall time of the whole loop                          */
#define LOMPC_LOOP_PROF_ISSUE  2 /* us, host time issuing copies / launches / the collective       */
#define LOMPC_LOOP_PROF_WAIT   3 /* us, host time blocked in the stream synchronisation           */
#define LOMPC_LOOP_PROF_GPU    4 /* us, GPU span of each engine call (HIP events around H2D .. D2H;
                                    device loop: first enqueue .. convergence, per engine call)   */
#define LOMPC_LOOP_PROF_STEP   5 /* us, host price-gradient QP (lompc_price_step; 0 on the device) */
#define LOMPC_LOOP_PROF_HOST   6 /* us, other host work (convergence test, metric, bookkeeping)   */
#define LOMPC_LOOP_PROF 8
typedef struct lompc_price_loop_args {
  int N, r, max_iter, tol_avg;          /* tol_avg: 1 = PRICE_SOLVER_TOL_TYPE "avg", 0 = "max" */
  double theta, w_max, m, kappa, eps_reg, tol, n_evs, lmbd_r;
  const double* A_bar;                  /* host [N, N] */
  const double* w_ref;                  /* host [N]    */
  double* dev_in; double* host_in;
  const double* dev_sw; const double* dev_st;
  double* host_sw; double* host_st;
  double* prof;                         /* host [LOMPC_LOOP_PROF] or NULL */
  int device_loop;                      /* 1: device-resident loop (see above), 0: host loop */
} lompc_price_loop_args;
#define LOMPC_LOOP_AHEAD 2  /* device loop: engine calls enqueued beyond the device's progress */
int lompc_price_loop(lompc_plan* plan, const lompc_price_loop_args* args, double* lmbd, double* w_k,
                     double* dual_cost, double* dec_actual, double* dec_pred, int* iterations,
                     double* errs, void* stream);

/* One EV type's partitions in order, ONE call (charging_station.py:275-307, whose loop over the
 * partitions chains them through prev_prices): for every part with a plan, lompc_price_loop from
 * the previous part's regularised prices (common args with the part's n_evs, tol, w_ref and set
 * outputs), then the regularisation of price_solver.py:142-147 / 248-255 (lompc_lp_separable on
 * A = Dphi(w)', b = A lmbd, c = phi(w)); a part without a plan (no EVs) is skipped.  prev_prices
 * host [r] in / out.  Per part: lmbd host [3N] (its final prices), w_k host [N], dec_actual /
 * dec_pred host [max_iter] (may be NULL), and on return iterations (the reference's `iter`),
 * calls (engine calls made), price_before_reg / price_after_reg (phi(w)'lmbd before / after), rc.
 * Stops at the first failing part (its rc, also returned; lompc_plan_last_error of its plan). */
typedef struct lompc_price_chain_part {
  lompc_plan* plan;
  double n_evs, tol;
  const double* w_ref;
  const double* dev_sw; const double* dev_st;
  double* lmbd; double* w_k; double* dec_actual; double* dec_pred;
  int iterations, calls, rc, pad;
  double price_before_reg, price_after_reg;
} lompc_price_chain_part;
int lompc_price_chain(int n_parts, lompc_price_chain_part* parts, const lompc_price_loop_args* common,
                      double* prev_prices, void* stream);

/* The regularisation step alone (price_solver.py:142-147 with :248-255; replaces the CVXPY call of
 * price_regularizer.py:68-85 for the station's A = Dphi(w)', b = A lmbd, c = phi(w)): lmbd host [3N]
 * in / out (lmbd[:r] replaced), w host [N] the loop's final iterate, *pre / *post = phi(w)'lmbd
 * before / after.  lompc_price_chain regularises with it, and PriceSolver's per-partition loop too,
 * so the two forms give identical prices. */
int lompc_price_regularize(int N, int r, double theta, double w_max, const double* w, double* lmbd, double* pre,
                           double* post);

/* ---------------------------------------------------------------------------
 * Host-side solvers of the price iteration (no device, no context).  They run
 * once per price iteration / per partition next to the convergence test, like
 * the reference's CVXPY/Clarabel solves they replace.  Host buffers.
 * ------------------------------------------------------------------------- */

/* Price-gradient step.  Replaces PriceSolver._price_gradient_descent_step
 * (price_solver.py:216-246) and its CVXPY problem (:257-270):
 *   lmbd_next = argmin_{x >= 0} x'Px + q'x,
 *   P = Dphi(w) A_bar^-1 Dphi(w)'/(2m) + eps_reg I,  q = -2 P lmbd - (phi(w) - phi(w_ref))
 * with A_bar = A'A + kappa I (kappa = lmbd_r / delta, price_solver.py:188-194),
 * phi/Dphi of lompc.py:172-187 truncated to the first r = 2N or 3N rows.
 *   w_ref, w [N]; lmbd [r]  ->  lmbd_next [r]
 *   *dual_cost_decrease = (lmbd'P lmbd + q'lmbd) - (x'Px + q'x)      (:236, :244-245)
 *   *iterations = active-set iterations used (may be NULL)
 * Exact (finite active-set method), KKT-certified; LOMPC_ERR_NOT_CONVERGED
 * otherwise (cvxpy SolverError). */
int lompc_price_step(int N, int r, double theta, double w_max, double m, double kappa,
                     double eps_reg, const double* w_ref, const double* w, const double* lmbd,
                     double* lmbd_next, double* dual_cost_decrease, int* iterations);

/* Column-separable LP: min c'x s.t. A x = b, x >= 0, where every column of the
 * row-major A [n_rows, n_cols] has at most one nonzero and c >= 0.
 * Replaces PriceRegularizer.solve_price_regularization (price_regularizer.py:68-85),
 * whose only caller passes A = Dphi(w)', b = Dphi(w)' lmbd, c = phi(w)
 * (price_solver.py:248-255) — one nonzero per column (lompc.py:179-187).
 * Each row is a one-row LP solved by its cheapest column per unit of b_j (ties:
 * lowest column index; see DESIGN.md for the degenerate w_j = 0 case).
 * LOMPC_ERR_UNSUPPORTED if A is not column-separable or c has a negative entry,
 * LOMPC_ERR_NOT_CONVERGED if a row is infeasible. */
int lompc_lp_separable(int n_rows, int n_cols, const double* A, const double* b,
                       const double* c, double* x);

/* General LP: min c'x s.t. A x = b, x >= 0 (row-major A [n_rows, n_cols]): the
 * reference's PriceRegularizer accepts any such LP (price_regularizer.py:62-85).  Dense
 * two-phase simplex, Bland's rule; *objective (may be NULL) = c'x.
 * LOMPC_ERR_NOT_CONVERGED if infeasible, LOMPC_ERR_UNSUPPORTED if unbounded. */
int lompc_lp_solve(int n_rows, int n_cols, const double* A, const double* b, const double* c,
                   double* x, double* objective);

/* BiMPC charging cost types (bimpc.py:12-15, BiMPCChargingCostType) */
#define LOMPC_BIMPC_WEIGHTED       0
#define LOMPC_BIMPC_UNWEIGHTED     1
#define LOMPC_BIMPC_EXP_UNWEIGHTED 2
#define LOMPC_BIMPC_INFO           5

/* BiMPC team-optimal planner.  Replaces BiMPC.solve_bimpc (bimpc.py:267-292)
 * and its CVXPY/Clarabel problem (bimpc.py:142-265):
 *   constants  (bimpc.py:18-36, :116-140): N, P, charging_cost_type, delta, c_g,
 *              u_g_max, u_b_max, x_max, exp_rate, theta_s, theta_l, w_max_s, w_max_l
 *   parameters (BiMPCParameters, bimpc.py:39-59): Mp_s, Mp_l, beta_s, beta_l,
 *              gamma_sm, gamma_lm [P]; x0; demand [N]
 *   outputs    w_hat_s, w_hat_l [P, N] row-major, u_g [N]
 *   duals      optional [2 (2P+1) N + 4N]: lower-bound, upper-bound and coupling
 *              multipliers (for certificates), or NULL
 *   info       optional [LOMPC_BIMPC_INFO]: iterations, objective, primal
 *              residual, dual residual, complementarity sum
 * Primal-dual interior point on the smooth strictly convex problem (exact Newton
 * through an N x N Schur complement).  Asserts of bimpc.py:79-84 ->
 * LOMPC_ERR_INVALID_ARG; no convergence in 200 iterations (e.g. infeasible
 * storage bounds) -> LOMPC_ERR_NOT_CONVERGED with the last iterate written;
 * u_g_max, w_max or c_g equal to 0 -> LOMPC_ERR_UNSUPPORTED. */
int lompc_bimpc_solve(int N, int P, int charging_cost_type, double delta, double c_g,
                      double u_g_max, double u_b_max, double x_max, double exp_rate,
                      double theta_s, double theta_l, double w_max_s, double w_max_l,
                      const double* Mp_s, const double* Mp_l, const double* beta_s,
                      const double* beta_l, const double* gamma_sm, const double* gamma_lm,
                      double x0, const double* demand, double* w_hat_s, double* w_hat_l,
                      double* u_g, double* duals, double* info);

#ifdef __cplusplus
}
#endif
#endif /* LOMPC_AMD_H */
