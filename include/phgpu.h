/*
 * phgpu.h -- C-ABI of libphgpu.so, the MI355X (gfx950) progressive-hedging
 * hot path.  Plain pointers and sizes only; every array argument marked
 * "dev" is device memory owned by the caller (PyTorch-ROCm tensors in the
 * Python host), every "host" array is read during the call only.
 *
 * Layout convention ("scenario-fastest"): a per-scenario vector v of length
 * L over S scenarios is stored as v[i*S + s]  (i < L, s < S).
 *
 * Each entry point replaces one reference interface of mpi-sppy
 * (/root/reference, Nov-2020 tree); citations are file:line there.
 *
 * Error model: every int-returning call returns 0 on success, or
 *   PH_EINVAL (-1) invalid argument, PH_EHIP (-2) HIP runtime error,
 *   PH_ENUM (-3) numerical failure, PH_EDEV (-4) a device-side invariant
 *   check failed in an earlier launch (a work list or workspace index out of
 *   range; the offending access was skipped, the batch's results are not to
 *   be trusted; reported by the synchronising calls ph_batch_solve_summary,
 *   ph_loop_status and ph_batch_sync).
 * ph_last_error() returns a thread-local message for the last failure.
 * Calls are stream-ordered on the stream given to ph_batch_create /
 * ph_batch_set_stream and return without synchronising unless stated.
 */
#ifndef PHGPU_H
#define PHGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PH_OK 0
#define PH_EINVAL (-1)
#define PH_EHIP (-2)
#define PH_ENUM (-3)
#define PH_EDEV (-4)

/* per-scenario solve status (phbase.py:959-989 maps 2/3 -> infeasible) */
#define PH_STATUS_OPTIMAL 0
#define PH_STATUS_ITERLIMIT 1
#define PH_STATUS_PRIMAL_INFEASIBLE 2
#define PH_STATUS_DUAL_INFEASIBLE 3

typedef struct ph_batch *ph_batch_t;

typedef struct ph_solve_opts {
  double tol;          /* relative KKT tolerance (default 1e-9)            */
  int32_t max_iters;   /* PDHG iteration cap per scenario (default 200000) */
  int32_t check_every; /* KKT / restart check period (default 64)           */
  int32_t warm_start;  /* 1: start from x,y,omega passed in (default 1)     */
  double reflection;   /* Halpern reflection gamma in [0,1] (default 1.0)  */
  int32_t polish;      /* 1: active-set KKT polish for small scenarios     */
                       /*    (n + m <= 63; default 1)                      */
} ph_solve_opts;

/* doubles per scenario in ph_batch_get_diag's output */
#define PH_DIAG_W 5

/* Library version string. */
const char *ph_version(void);

/* Thread-local message describing the last error. */
const char *ph_last_error(void);

/*
 * Create a batch of S scenario subproblems sharing one sparsity pattern
 *   min 1/2 x'diag(q)x + g'x  s.t.  rl <= A x <= ru,  l <= x <= u,
 * A: m x n with nnz entries, CSR pattern (host arrays, int32).
 * Replaces: per-scenario SolverFactory + set_instance
 *   (mpisppy/phbase.py:1304-1362, _create_solvers).
 * stream: a hipStream_t (may be NULL for the null stream).
 */
int ph_batch_create(ph_batch_t *out, int32_t S, int32_t n, int32_t m,
                    int32_t nnz, const int32_t *row_ptr /*host [m+1]*/,
                    const int32_t *col_idx /*host [nnz]*/, void *stream);

/* Change the stream later calls are ordered on. */
int ph_batch_set_stream(ph_batch_t b, void *stream);

/*
 * Bind the per-scenario data (device, scenario-fastest) and compute the
 * per-scenario Ruiz + Pock-Chambolle scaling and PDHG step size.  Must be
 * called before ph_pdhg_solve; may be called again when data change.
 * c is the objective in MIN form (negate for maximize models).
 * The library copies what it needs; the caller may free the inputs after
 * the stream has passed this call.
 * Replaces: Pyomo model -> solver instance extraction (phbase.py:1327).
 */
int ph_batch_bind(ph_batch_t b, const double *vals /*dev [nnz][S]*/,
                  const double *c /*dev [n][S]*/,
                  const double *l /*dev [n][S]*/, const double *u /*dev [n][S]*/,
                  const double *rl /*dev [m][S]*/, const double *ru /*dev [m][S]*/);

/*
 * Declare the K nonanticipative columns (same for every scenario):
 * nonant_col[k] is the column of nonant slot k, in the reference's
 * nonant order (scenario_tree.py:10-38, spbase.py:272-280).
 */
/*
 * Replace the column bounds of every scenario (dev [n][S] each, copied):
 * nonants fixed at a candidate xhat (l = u) for the inner-bound solves of
 * extensions/xhatbase.py:_try_one (_fix_nonants / _restore_nonants), and
 * back.  The scaling is unchanged (it depends on the matrix only); the
 * active-set cache is invalidated.
 */
int ph_batch_set_bounds(ph_batch_t b, const double *l, const double *u);

int ph_batch_set_nonants(ph_batch_t b, int32_t K,
                         const int32_t *nonant_col /*host [K]*/);

/*
 * Batched PH subproblem solve (restarted, reflected-Halpern PDHG, FP64).
 * The objective of scenario s is the reference's PH-augmented objective
 * (phbase.py:1133-1209) in min form:
 *   g = c + w_on*W - prox_on*rho*xbar   (nonant columns), q = prox_on*rho,
 *   const = prox_on * sum_k rho_k/2 * xbar_k^2.
 * W, rho, xbar: dev [K][S] (xbar already broadcast per scenario).
 * x [n][S], y [m][S], omega [S] are read as the warm start when
 * opts->warm_start and overwritten with the solution (unscaled).
 * Outputs (dev [S]): status, iters, pobj (objective incl. const),
 * dbound (dual objective incl. const = the scenario's outer bound).
 * Replaces: solve_loop -> solve_one -> plugin.solve/load_vars/
 *   results.Problem[0].Lower_bound (phbase.py:864-1095).
 */
int ph_pdhg_solve(ph_batch_t b, const double *W, const double *rho,
                  const double *xbar, double w_on, double prox_on,
                  double *x, double *y, double *omega, int32_t *status,
                  int32_t *iters, double *pobj, double *dbound,
                  const ph_solve_opts *opts);

/*
 * Per-node weighted sums for xbar / xsqbar (phbase.py:144-201, the local
 * half of Compute_Xbar before the Allreduce).
 * G "node slots": slot g covers nonant slot k = slot_k[g] for the scenarios
 * s in [slot_s0[g], slot_s1[g]); out_sums[g] = sum prob_coeff[k][s]*x,
 * out_sums[G+g] = sum prob_coeff[k][s]*x^2, x = x[nonant_col[k]][s].
 * slot_k/slot_s0/slot_s1: dev int32 [G]; prob_coeff: dev [K][S];
 * out_sums: dev [2G].
 */
int ph_xbar_accum(ph_batch_t b, const double *x, const double *prob_coeff,
                  int32_t G, const int32_t *slot_k, const int32_t *slot_s0,
                  const int32_t *slot_s1, double *out_sums);

/*
 * After the Allreduce of out_sums: broadcast xbar/xsqbar to every
 * scenario, update W += rho*(x - xbar) (times w_coeff if not NULL) and
 * return |x - xbar| summed over the nonants of each scenario.
 * (phbase.py:204-217 broadcast, :224-251 Update_W, :266-272 conv local sum)
 * gid: dev int32 [K][S] -> node slot g of (k,s); sums: dev [2G].
 * xbar, xsqbar, W: dev [K][S] (out / out / in-out); absdiff: dev [S] (out).
 * W may be NULL: broadcast and |x - xbar| sums only (Compute_Xbar alone).
 */
int ph_update_w(ph_batch_t b, const double *x, const double *sums, int32_t G,
                const int32_t *gid, const double *rho, const double *w_coeff,
                double *xbar, double *xsqbar, double *W, double *absdiff);

/*
 * Contiguous-segment sums: out[r] = sum_{s in [seg[r], seg[r+1])} v[s],
 * r < R.  Used for convergence_diff's per-rank sums (phbase.py:266-276)
 * and the probability-weighted Ebound/Eobjective partial sums.
 * v: dev [S]; w: dev [S] weights or NULL; seg: dev int32 [R+1]; out: dev [R].
 */
int ph_segment_sum(ph_batch_t b, const double *v, const double *w, int32_t R,
                   const int32_t *seg, double *out);

/*
 * Evaluate each scenario's active objective at x (phbase.py:279-312,
 * Eobjective's per-scenario pyo.value(objfct)), min form incl. const.
 * obj: dev [S].
 */
int ph_eval_objective(ph_batch_t b, const double *x, const double *W,
                      const double *rho, const double *xbar, double w_on,
                      double prox_on, double *obj);

/*
 * Bundles (phbase.py:803-862 FormEF / 1273-1302 subproblem_creation;
 * sputils.py:246-383 _create_EF_from_scen_dict): a bundle is ONE batched
 * subproblem (its scenarios' blocks plus nonanticipativity rows), so the
 * bundle batch's PH terms are gathered from the scenario batch's [K][S]
 * W / rho / xbar with the EF objective's weights p_s / P_b (sputils.py:
 * 314-322), and the bundle solution goes back to the scenarios' [n][S] x
 * (the reference's scenario sub-blocks "naturally get the EF solution",
 * phbase.py:833-838).  One indexed gather on the batch's stream:
 *   dst[e] = wt[e] * src[idx[e]]   (wt NULL: 1;  idx[e] < 0: 0),  e < count.
 * src: dev [src_count]; idx: dev int32 [count]; wt: dev [count] or NULL;
 * dst: dev [count].  An index >= src_count is a device-side check failure
 * (PH_EDEV at the next synchronising call) and reads 0.
 */
int ph_gather(ph_batch_t b, const double *src, int64_t src_count, const int32_t *idx,
              const double *wt, int64_t count, double *dst);

/*
 * Diagnostics of the last ph_pdhg_solve, copied to host out[PH_DIAG_W*S]:
 * per scenario the final relative primal residual, dual residual, duality
 * gap, Halpern fixed-point residual and how the solve ended (0 PDHG reached
 * tol, 1 active-set polish of the warm start, 2 polish of a PDHG iterate,
 * 3 the cached active set's affine map)
 * (synchronises the stream).
 */
int ph_batch_get_diag(ph_batch_t b, double *out /*host [S][PH_DIAG_W]*/);

/*
 * Summary of the last ph_pdhg_solve, copied to host (synchronises the
 * stream): out[0] scenarios not solved to tolerance (status != optimal),
 * out[1] PDHG iterations summed over scenarios, out[2] the largest count,
 * out[3] scenarios finished by an active-set polish (how 1 or 2), out[4]
 * scenarios finished by the active-set cache (how 3).  One small copy
 * replaces reading status[S] after every solve (phbase.py:959-965 checks
 * each scenario's status).
 */
int ph_batch_solve_summary(ph_batch_t b, int64_t *out /*host [5]*/);

/*
 * Device-side PH iteration control (iterk_loop without a host round trip
 * per iteration, phbase.py:1498-1553).  While the loop is enabled, every
 * per-iteration kernel (ph_xbar_accum, ph_update_w, ph_segment_sum,
 * ph_pdhg_solve and the convergence kernels) first reads the batch's stop
 * flag and does nothing once it is set, so the host can queue (or replay as
 * a HIP graph) many iterations and look at the flag only now and then.
 * One iteration, in the reference's order:
 *   [allreduce of the Compute_Xbar sums]       (multi-rank only)
 *   ph_update_w (with W)                       Compute_Xbar broadcast + Update_W
 *   ph_loop_conv_local                         convergence_diff (one rank), or
 *   ph_segment_sum + [allreduce] + ph_loop_conv  (several ranks):
 *       conv = sum_r parts[r]/cnt[r] / nproc (phbase.py:254-276) into
 *       conv_hist[iter-1]; stop (1) when conv < convthresh, BEFORE this
 *       iteration's solve (x stays stale, as in the reference)
 *   ph_pdhg_solve                              solve_loop; its post-solve
 *       kernel also computes the next iteration's Compute_Xbar sums (when
 *       ph_loop_set_xbar gave them) and begins the next iteration
 *       (counter += 1, or stop (2) past iter_limit)
 * ph_loop_reset sets iter = start_iter, clears the flag and the solve
 * counters and begins iteration start_iter + 1; before the first pass the
 * host computes the Compute_Xbar sums once (ph_xbar_accum).  ph_loop_enable
 * switches the flag checks on / off; ph_loop_status copies {stop, iter,
 * not-optimal solves, solves, PDHG iterations (sum), PDHG iterations (max),
 * polished, cached} to host out[8] (synchronises).
 */
int ph_loop_reset(ph_batch_t b, int32_t start_iter, int32_t iter_limit,
                  double convthresh);
int ph_loop_enable(ph_batch_t b, int32_t on);
int ph_loop_set_xbar(ph_batch_t b, const double *x, const double *prob_coeff,
                     int32_t G, const int32_t *slot_k, const int32_t *slot_s0,
                     const int32_t *slot_s1, double *out_sums);
int ph_loop_conv(ph_batch_t b, const double *parts /*dev [R]*/,
                 const double *cnt /*dev [R]*/, int32_t R, double nproc,
                 double *conv_hist /*dev [iter_limit]*/);
int ph_loop_conv_local(ph_batch_t b, const double *absdiff /*dev [S]*/,
                       const int32_t *seg /*dev [R+1]*/, int32_t R,
                       const double *cnt /*dev [R]*/, double nproc,
                       double *parts /*dev [R] out*/, double *conv_hist);
/*
 * One rank: ph_update_w and ph_loop_conv_local in one launch.  wconv[s] =
 * 1 / (cnt of the reference rank holding scenario s) / nproc, so conv =
 * sum_s absdiff[s] * wconv[s] (phbase.py:254-276); same outputs as the two
 * calls (conv up to summation order), plus the stop test.
 */
int ph_loop_update_w_conv(ph_batch_t b, const double *x /*dev [n*S]*/,
                          const double *sums /*dev [2G]*/, int32_t G,
                          const int32_t *gid /*dev [K*S]*/, const double *rho,
                          const double *w_coeff /*dev [K*S] or NULL*/, double *xbar,
                          double *xsqbar, double *W, double *absdiff /*dev [S]*/,
                          const double *wconv /*dev [S]*/, double *conv_hist);
/*
 * Several ranks, one collective per iteration (what PHBase uses): the conv
 * partials of a pass travel in the NEXT pass's Compute_Xbar allreduce (one
 * buffer [2G | R]), so each pass runs
 *   [allreduce sums|parts] ph_loop_conv_lagged  ph_update_w  ph_segment_sum
 *   ph_loop_backup  ph_pdhg_solve
 * ph_loop_conv_lagged tests the pending pass's conv (conv_hist[k-1]); when
 * it is below convthresh it sets stop (1) and iter back to k, and the host
 * restores x/y from the copies ph_loop_backup saved before pass k's solve --
 * the reference's state at its break (phbase.py:1498-1553).  After the loop
 * ends at the limit (stop 2) the host flushes the last pass's partials with
 * one more allreduce + ph_loop_conv_lagged.  ph_loop_backup copies
 * x[0..nx) -> x_save, y[0..ny) -> y_save and marks the current pass pending.
 */
int ph_loop_conv_lagged(ph_batch_t b, const double *parts /*dev [R]*/,
                        const double *cnt /*dev [R]*/, int32_t R, double nproc,
                        double *conv_hist /*dev [iter_limit]*/);
int ph_loop_backup(ph_batch_t b, const double *x, double *x_save, int64_t nx,
                   const double *y, double *y_save, int64_t ny);
/*
 * With ph_loop_backup: the solve's status [S] and outer bound [S] saved
 * under the same stop check, so a convergence break restores the
 * reference's statuses and bounds too (phbase.py:1505-1510 breaks before
 * the solve; scenario_feasible and Ebound then describe the last solve run).
 */
int ph_loop_backup_status(ph_batch_t b, const int32_t *status, int32_t *status_save,
                          const double *dbound, double *dbound_save);
int ph_loop_status(ph_batch_t b, int64_t *out /*host [8]*/);

/*
 * One device-loop pass in one call (phbase.py:1498-1553, one iterk_loop
 * iteration after its Compute_Xbar allreduce): the arguments are bound once
 * per loop (ph_loop_bind_pass copies the struct; NULL unbinds), then every
 * pass is ph_loop_pass(b), so the host issues one call per PH iteration
 * (plus the collective on several ranks) instead of one per kernel.
 *   conv_part == NULL (one rank): ph_loop_update_w_conv + ph_pdhg_solve.
 *   conv_part != NULL (several ranks, the one-collective scheme above with
 *     the convergence partials pre-weighted: conv = sum over ranks of
 *     sum_s absdiff[s] * wconv[s], one slot): the lagged test of the
 *     previous pass on *conv_part (allreduced by the caller together with
 *     sums), this pass's Compute_Xbar broadcast + Update_W with its local
 *     partial written to *conv_part, ph_loop_backup + ph_loop_backup_status
 *     in one launch, ph_pdhg_solve.  After the loop the caller flushes the
 *     last partial: allreduce + ph_loop_conv_lagged(conv_part, cnt = {1},
 *     R = 1, nproc = 1).
 * Replaces: the per-iteration body of PHBase.iterk_loop (phbase.py:1498-1553).
 */
typedef struct ph_loop_pass_args {
  const double *sums;      /* dev [2G] node sums (allreduced on several ranks) */
  int32_t G;
  const int32_t *gid;      /* dev [K*S] */
  const double *rho;       /* dev [K*S] */
  const double *w_coeff;   /* dev [K*S] or NULL */
  double *xbar;            /* dev [K*S] out */
  double *xsqbar;          /* dev [K*S] out */
  double *W;               /* dev [K*S] in-out */
  double *absdiff;         /* dev [S] out */
  const double *wconv;     /* dev [S] */
  double *conv_hist;       /* dev [iter_limit] */
  double *conv_part;       /* dev [1], several ranks; NULL on one rank */
  double *x_save;          /* dev [n*S] (several ranks) */
  double *y_save;          /* dev [m*S] (several ranks) */
  int32_t *status_save;    /* dev [S] (several ranks) */
  double *dbound_save;     /* dev [S] (several ranks) */
  double w_on, prox_on;    /* the solve, as ph_pdhg_solve */
  double *x, *y, *omega;
  int32_t *status, *iters;
  double *pobj, *dbound;
  ph_solve_opts opts;
} ph_loop_pass_args;
int ph_loop_bind_pass(ph_batch_t b, const ph_loop_pass_args *args);
int ph_loop_pass(ph_batch_t b);
/*
 * Up to `iters` passes of the bound loop in one call, same results as that
 * many ph_loop_pass calls (up to the summation order of Compute_Xbar's sums
 * and of conv).  With one rank and the one-wave cached warm solve, once
 * ph_loop_status has seen a quiet stretch (no PDHG tail, at most 2e-3 cache
 * misses per scenario-pass since its previous read; PHGPU_PERSIST=1 / 0
 * forces the choice): a persistent launch runs whole passes with one grid
 * barrier each (Compute_Xbar broadcast + Update_W + the conv partial, the
 * cached map / register polish of every scenario held back in LDS, the next
 * sums; after the barrier the combined conv either drops the pass's solve --
 * the reference tests before it solves -- or commits it) while the owned
 * scenarios' data stay in LDS; a pass with a polish failure is finished by
 * the tail and post-solve kernels queued behind it (up to four such rounds
 * per call).  Otherwise
 * `iters` ph_loop_pass calls.  The caller reads ph_loop_status for how far
 * it got.  Replaces: iterk_loop's loop body (phbase.py:1498-1553) repeated.
 */
int ph_loop_run(ph_batch_t b, int32_t iters);
/* 1 when ph_loop_run takes the persistent path for the bound pass, else 0. */
int ph_loop_persistent(ph_batch_t b);
/* 1 when a ph_loop_run since the last ph_loop_reset ran the fused per-pass
 * form (two launches per pass: the cached maps, then finish_kernel: polish,
 * tail, Compute_Xbar sums and the next pass's Update_W / convergence
 * test), else 0. */
int ph_loop_fused(ph_batch_t b);
/*
 * While timing is on (ph_batch_set_timing): the persistent launches' HIP
 * events, out[3] = {loop_kernel launches, their total ms, passes they ran
 * since ph_loop_reset} (synchronises).
 */
int ph_loop_read_timing(ph_batch_t b, double *out /*host [3]*/);

/*
 * Kernel timing of ph_pdhg_solve with HIP events recorded on the batch's
 * stream around its kernels of every solve while timing is on (set_timing
 * clears the record).  read_timing synchronises and returns out[8] =
 * {solves recorded, total ms of the active-set kernel, of the polish
 * kernel, of the PDHG kernel (one-wave path: from the polish's end to the
 * solve's end; mid-size path: all phases), launches and total ms of the
 * mid-size path's PDHG phase kernel, launches and total ms of its polish
 * phase kernel}.  (Measurement support; bench.py.)
 */
int ph_batch_set_timing(ph_batch_t b, int32_t on);
int ph_batch_read_timing(ph_batch_t b, double *out /*host [8]*/);

/* Block until all work queued on the batch's stream has finished. */
int ph_batch_sync(ph_batch_t b);

/* Free the handle and the library-owned device scratch. */
void ph_batch_destroy(ph_batch_t b);

#ifdef __cplusplus
}
#endif
#endif /* PHGPU_H */
