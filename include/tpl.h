/*
 * tpl.h — C ABI of the MI355X two-pass Lanczos engine (libtpl_amd.so).
 *
 * This is the drop-in boundary for the hot path of lukefleed/two-pass-lanczos:
 * the Lanczos recurrence behind `solvers::lanczos` / `solvers::lanczos_two_pass`
 * and the low-level `algorithms::*` entry points. Every entry point below names
 * the reference item it replaces (file:line under the reference checkout).
 * The signatures are plain C (pointers + sizes, no torch / HIP types), so a
 * Rust `extern "C"` block, ctypes, or a C++ caller can bind them directly
 * (bindings: INTEGRATION.md).
 *
 * Conventions
 *   - All arithmetic is IEEE fp64 (every reference call site is f64).
 *   - Vectors `b`, `x_out`, `v_out` are host pointers when `mem == TPL_MEM_HOST`
 *     and device pointers on the operator's GPU when `mem == TPL_MEM_DEVICE`.
 *     Scalar arrays (alphas, betas, y) are always host pointers.
 *   - `v_out` matrices are column-major n x steps (leading dimension n), the
 *     layout of the reference's `Mat<f64>` V_k.
 *   - Every function returns a tpl_status; on failure tpl_last_error() returns
 *     the message, formatted exactly like the reference's `Display` strings
 *     (src/error.rs:20-58) for the Lanczos error kinds.
 *   - An operator owns one HIP stream and its device workspace; calls on one
 *     operator are not re-entrant (the reference is single-threaded, Par::Seq).
 */
#ifndef TPL_H_
#define TPL_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: mirror LanczosErrorKind (src/error.rs:20-58) ---------- */
typedef enum tpl_status {
  TPL_OK = 0,
  TPL_ERR_BREAKDOWN = 1,           /* LanczosErrorKind::Breakdown (declared, never constructed by the reference) */
  TPL_ERR_DIMENSION_MISMATCH = 2,  /* LanczosErrorKind::DimensionMismatch (reference panics instead; we report) */
  TPL_ERR_INPUT = 3,               /* LanczosErrorKind::InputError  (src/algorithms/mod.rs:268-272, lanczos_two_pass.rs:229-235) */
  TPL_ERR_PARAMETER_MISMATCH = 4,  /* LanczosErrorKind::ParameterMismatch (src/solvers.rs:78-85,158-165; lanczos_two_pass.rs:220-227) */
  TPL_ERR_EVD = 5,                 /* LanczosErrorKind::EvdError (built-in exp solver only) */
  TPL_ERR_SOLVER = 6,              /* LanczosErrorKind::SolverError (src/solvers.rs:75,156) */
  /* engine / loader errors (no reference counterpart in LanczosErrorKind) */
  TPL_ERR_INVALID_ARGUMENT = 100,
  TPL_ERR_DEVICE = 101,            /* HIP runtime failure; message carries hipGetErrorString */
  TPL_ERR_OUT_OF_MEMORY = 102,
  TPL_ERR_DATA_LOADER = 103,       /* DataLoaderError (src/utils/data_loader.rs:16-43) */
  TPL_ERR_UNSUPPORTED = 104
} tpl_status;

enum { TPL_MEM_HOST = 0, TPL_MEM_DEVICE = 1 };

typedef struct tpl_ctx_s* tpl_ctx_t; /* one GPU + one HIP stream          */
typedef struct tpl_op_s* tpl_op_t;   /* device-resident CSR operator A    */

/* Thread-local message of the last failing call ("" after success). */
const char* tpl_last_error(void);
/* The fields of the last failing call's LanczosErrorKind (src/error.rs:20-58), so a
 * binding rebuilds the variant itself instead of parsing the message:
 *   TPL_ERR_INPUT              InputError(inner)
 *   TPL_ERR_PARAMETER_MISMATCH ParameterMismatch { param_name, expected, actual }
 *                              (src/solvers.rs:78-85,158-165; lanczos_two_pass.rs:220-227)
 *   TPL_ERR_DIMENSION_MISMATCH DimensionMismatch { operator_cols, vector_rows }
 *   TPL_ERR_SOLVER             SolverError(inner) (src/solvers.rs:75,156)
 *   TPL_ERR_EVD                EvdError(inner)
 *   TPL_ERR_BREAKDOWN          Breakdown { k = breakdown_step } (never raised: a
 *                              breakdown truncates steps_taken, as in the reference)
 * status is TPL_OK after a successful call. The strings stay valid until the next
 * tpl_* call on this thread. Returns TPL_ERR_INVALID_ARGUMENT only for out == NULL.  */
typedef struct tpl_error_detail {
  int32_t status;             /* tpl_status of the last call on this thread            */
  const char* message;        /* == tpl_last_error(): the variant's Display text        */
  const char* inner;          /* InputError / SolverError / EvdError payload, else ""  */
  const char* param_name;     /* ParameterMismatch::param_name, else ""                */
  uint64_t expected, actual;  /* ParameterMismatch                                      */
  uint64_t operator_cols, vector_rows; /* DimensionMismatch                             */
  uint64_t breakdown_step;    /* Breakdown::k                                           */
} tpl_error_detail;
tpl_status tpl_last_error_detail(tpl_error_detail* out);
/* Library version string, e.g. "tpl_amd 0.1.0 gfx950". */
const char* tpl_version(void);

/* ---- context ------------------------------------------------------------- */
tpl_status tpl_ctx_create(int device, tpl_ctx_t* out);
tpl_status tpl_ctx_destroy(tpl_ctx_t ctx);
/* Synchronise the context stream (all operators created on it share it). */
tpl_status tpl_ctx_synchronize(tpl_ctx_t ctx);
/* Number of visible GPUs (0 on a host without one; never fails). */
int tpl_device_count(void);

/* ---- operator: replaces faer `LinOp<f64>` for `SparseColMatRef<usize,f64>`
 *      (used at src/algorithms/mod.rs:177, src/algorithms/lanczos_two_pass.rs:186).
 *  A must be square n x n and SYMMETRIC (the Lanczos contract; A = [[D,E^T],[E,0]]
 *  for the KKT inputs), so its CSR arrays equal the reference's CSC arrays.
 *  Host arrays are borrowed for the call only; the operator copies them to HBM.
 *  Column indices must be sorted ascending within each row, 0 <= col < n.
 *  Limits: nnz < 2^31 (int32 offsets on device).                               */
tpl_status tpl_op_create_csr(tpl_ctx_t ctx, int64_t n, int64_t nnz,
                             const int64_t* row_ptr, const int32_t* col_idx,
                             const double* vals, tpl_op_t* out);
tpl_status tpl_op_destroy(tpl_op_t op);
int64_t tpl_op_nrows(tpl_op_t op); /* LinOp::nrows / ncols */
int64_t tpl_op_nnz(tpl_op_t op);
/* Bit 0: row-partitioned operator; bit 1: passes launched eagerly (no hipGraph —
 * a host transport, or a transport that refused stream capture); bit 2: values kept
 * as int8, bit 3 / bit 4: short-row / long-row column indices kept as uint16 offsets
 * (see tpl_op_set_value_format), bit 5: the last tpl_lanczos_two_pass / tpl_lanczos
 * evaluated f(T_k) on the device (one graph, no host round trip), bit 6: rows held in the locality order
 * (tpl_op_set_reorder, tpl_op_permutation; on a replicated-long-row partition the
 * rank's own short rows are in that order and tpl_op_local_rows, not
 * tpl_op_permutation, reports it), bit 7: a replicated-long-row partition whose ranks
 * all-gather their norm partials and reduce them inside pass one's SpMV (no rank-total
 * launch). -1 if op is NULL.                                         */
int tpl_op_flags(tpl_op_t op);
/* Locality order (single-GPU operators; rebuilds the layout). mode 1: the device
 * holds P A P^T, the short rows sorted by the long rows (hub columns) they reference
 * and the long rows last, so the hub rows' gathers touch compact runs; mode 0: the
 * caller's order; mode 2 (default, auto): on up to 2^20 rows (measured gain at the
 * 500k-arc KKT, none from 1M arcs, a loss at 5M arcs: DESIGN.md §3);
 * every vector crossing the boundary (b, x, apply's x / y, V_k, the callback's view)
 * is permuted on the device, so the caller sees its own row order throughout. The
 * permutation changes the device's reduction order (summation order within rows and of
 * the partials): results are bitwise those of the oracle run on P A P^T with the same
 * schedule, and agree with the unpermuted operator to rounding. No effect when the
 * matrix has no long rows, and none on row-partitioned operators.                   */
tpl_status tpl_op_set_reorder(tpl_op_t op, int mode);
/* perm[i] = the caller's row held at internal position i (n entries; the identity
 * when the operator is not reordered). tpl_op_schedule's row lists are internal.    */
tpl_status tpl_op_permutation(tpl_op_t op, int32_t* perm);
/* Tune the locality order's group count on this device (single GPU; switches the
 * order on): rebuilds the layout for each of the `count` group counts in `groups`
 * (count 0: 12..20, 22, 24), times `iters` launches each of the pass-one and pass-two
 * SpMV kernels, keeps the fastest and reports it in *chosen (*best_us: the sum of the
 * two kernels' average launch times). The choice depends on measured times, so two
 * tuned operators of one matrix may hold different orders (each bitwise against the
 * oracle given its own permutation); untuned operators are deterministic.          */
tpl_status tpl_op_tune_order(tpl_op_t op, const int32_t* groups, int32_t count, int32_t iters,
                             int32_t* chosen, double* best_us);
/* Pin the locality order's group count (single GPU; rebuilds the layout; 0 = the
 * default 16). Deterministic: operators of one matrix with one group count hold the
 * same order on every device and process, so their results are bit-identical. The
 * bench pins the count per instance (bench.py PINNED_ORDER_GROUPS, chosen offline from
 * profiles/r02_group_sweep.txt) instead of tuning on the box.                       */
tpl_status tpl_op_set_order_groups(tpl_op_t op, int32_t groups);
/* The group count of the order the device holds (0: caller's order; -1: NULL op). */
int32_t tpl_op_order_groups(tpl_op_t op);
/* The locality order's rule alone (host only, no device): perm (n entries) as
 * tpl_op_permutation would report it for this CSR (columns ascending per row),
 * short-row threshold (<= 0: auto) and group count (<= 0: 16); *applied = 0 when the
 * order is the identity.                                                           */
tpl_status tpl_locality_order(int64_t n, const int64_t* row_ptr, const int32_t* col_idx,
                              int32_t short_row_max, int32_t groups, int32_t* perm,
                              int32_t* applied);
/* Storage format (rebuilds the layout): compress != 0 (default) keeps the values as
 * int8 when every one is an integer in [-128, 127] (not -0.0), and the column
 * indices as uint16 offsets from a per-chunk / per-bin base when the spans allow —
 * lossless, results are bit-identical; 0 keeps fp64 values and int32 columns.       */
tpl_status tpl_op_set_value_format(tpl_op_t op, int compress);

/* y = A x  — LinOp::apply (compatibility path; the solvers below keep the whole
 * recurrence on the device and never call this per step).                     */
tpl_status tpl_op_apply(tpl_op_t op, const double* x, double* y, int mem);

/* ---- f(T_k) solver callback: replaces the `f_tk_solver` closure
 *      `FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>` (src/solvers.rs:57,144).
 *  Called exactly once per solve, after pass one, with n_alphas = steps and
 *  n_betas = steps - 1. Write y' = f(T_k) e_1 into y_out (capacity y_cap = steps)
 *  and its length into *y_len. Return 0 on success; non-zero means Err(e): put
 *  e's text (NUL-terminated) into err_msg (capacity err_cap).                   */
typedef int (*tpl_ftk_fn)(const double* alphas, size_t n_alphas, const double* betas,
                          size_t n_betas, double* y_out, size_t y_cap, size_t* y_len,
                          char* err_msg, size_t err_cap, void* user);

/* Built-in f(T_k) solvers with the tpl_ftk_fn signature (user ignored):
 *  inv : y' = T_k^{-1} e_1, tridiagonal LU with partial pivoting
 *        (the harness's sp_lu / partial_piv_lu, src/bin/tradeoff.rs:245-258,
 *        tests/correctness.rs:171-179). A singular T_k yields non-finite y'
 *        exactly like an LU solve does (no error), matching the reference.
 *  exp : y' = Q exp(Lambda) Q^T e_1 via symmetric tridiagonal QL eigensolver
 *        (src/bin/stability.rs:175-193). Non-convergence -> non-zero return.
 *  sq  : y' = T_k^2 e_1 (tests/correctness.rs:287-299).                        */
int tpl_ftk_inv(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
                double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
                void* user);
int tpl_ftk_exp(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
                double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
                void* user);
int tpl_ftk_sq(const double* alphas, size_t n_alphas, const double* betas, size_t n_betas,
               double* y_out, size_t y_cap, size_t* y_len, char* err_msg, size_t err_cap,
               void* user);

/* ---- high-level API: src/solvers.rs ------------------------------------- */
/* solvers::lanczos (src/solvers.rs:46-107): standard pass (V_k kept in HBM),
 * f(T_k), x = ||b|| V_k y' (device GEMV). x_out has n entries. With a built-in f on a
 * single-GPU operator f(T_k) runs on the device by the rules of tpl_op_set_device_ftk
 * (no host round trip); any other f is called on the host.                       */
tpl_status tpl_lanczos(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                       tpl_ftk_fn f, void* f_user, double* x_out, int mem);
/* solvers::lanczos_two_pass (src/solvers.rs:133-175): pass one (scalars only),
 * f(T_k), y = y' ||b||, pass two regenerates V_k on the fly. With f == tpl_ftk_inv (or
 * tpl_ftk_exp) on a single-GPU operator the solve runs as ONE device graph: f(T_k) on the
 * GPU (inv: the host solver's exact operations, bitwise the same y), no host round trip
 * between the passes (tpl_op_set_device_ftk). Any other f is called on the host between
 * the passes.
 * On an error x_out is unspecified.                                               */
tpl_status tpl_lanczos_two_pass(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                tpl_ftk_fn f, void* f_user, double* x_out, int mem);
/* Where tpl_lanczos_two_pass evaluates the built-in f(T_k): mode 0 = host (two graphs
 * around the host call), 1 = device (the whole solve one graph), 2 = auto (default).
 *   inv: device for k <= 1365 in mode 1, k <= 500 in mode 2: the host solver's exact
 *        operations, its elimination done during pass one and its back substitution with
 *        correctly rounded (Markstein) divisions — bitwise the host result. Auto mode
 *        stops at k = 500, the largest k measured no slower than the host round trip it
 *        removes; at k = 1000-1365 the serial back substitution is slower.
 *   exp: device for k <= 1800 (modes 1 and 2): a Chebyshev expansion of exp over the
 *        Sturm-bracketed spectrum, parallel over the rows of T_k, within
 *        a small multiple of eps * exp(lambda_max) of the host QL result — the accuracy
 *        class of the reference's EVD (src/bin/stability.rs:175-193), not its bits. A
 *        T_k that is not finite or whose spectrum is too wide for the expansion is handed
 *        back to the host solver inside the same call.                              */
tpl_status tpl_op_set_device_ftk(tpl_op_t op, int mode);
/* Test / introspection: evaluate the device f(T_k) kernel alone on a given T_k (which 0:
 * inv, 1: exp; n alphas, n - 1 betas) into y_out (n host doubles, y' = f(T_k) e_1).
 * *on_device = 0 when the exp kernel handed the case back to the host (y_out then 0).  */
tpl_status tpl_op_ftk_device(tpl_op_t op, int which, const double* alphas, size_t n,
                             const double* betas, double* y_out, int* on_device);

/* ---- low-level API: src/algorithms/ -------------------------------------- */
/* Per-step callback of lanczos_standard (LanczosCallback, src/algorithms/mod.rs:82-86):
 * called after every step with k = steps so far (1-based), the DEVICE pointer of
 * V_k (column-major, ld = n, k valid columns) and the host T_k scalars
 * (k alphas, k-1 betas... exactly the reference's TridiagonalSystemView, i.e.
 * betas holds the betas pushed so far). Return non-zero to continue, 0 to stop.
 * The host polls in batches (1, 2, 4, ... up to 32 steps run ahead on the device, then
 * the callback for each of them in order): a stop at step j returns exactly the
 * j-step result (later steps never change earlier coefficients or columns), with one
 * host synchronisation per batch. Columns past k may already hold later basis
 * vectors while the callback runs; only the first k are the view.               */
typedef int (*tpl_step_cb)(size_t k, const double* v_k_device, int64_t n,
                           const double* alphas, size_t n_alphas, const double* betas,
                           size_t n_betas, void* user);

/* algorithms::lanczos::lanczos_standard (src/algorithms/lanczos.rs:55-156).
 * alphas: capacity k; betas: capacity k (k-1 used); v_out: n x k capacity or NULL.
 * On return *steps = steps_taken, *b_norm = ||b||, alphas[0..steps), betas[0..steps-1),
 * v_out columns [0, steps) filled. reorth enables full re-orthogonalisation against
 * the stored V_k (an extension with no reference counterpart): 1 = CGS2 (classical
 * Gram-Schmidt, two passes every step), 2 = selective (Kahan–Parlett "twice is
 * enough": the second pass only when the first removed more than half of ||r||^2;
 * tpl_op_reorth_second_passes reports how many ran), 0 = none.                  */
tpl_status tpl_lanczos_standard(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                double* alphas, double* betas, size_t* steps,
                                double* b_norm, double* v_out, int mem, int reorth,
                                tpl_step_cb cb, void* cb_user);

/* algorithms::lanczos_two_pass::lanczos_pass_one (src/algorithms/lanczos_two_pass.rs:65-110). */
tpl_status tpl_lanczos_pass_one(tpl_op_t op, const double* b, int64_t b_len, size_t k,
                                double* alphas, double* betas, size_t* steps,
                                double* b_norm, int mem);

/* algorithms::lanczos_two_pass::lanczos_pass_two (:128-140) and, with v_out != NULL,
 * lanczos_pass_two_with_basis (:149-166). The decomposition is passed as its
 * fields (LanczosDecomposition, src/algorithms/mod.rs:94-108); y = y_k (already
 * scaled by ||b||) with y_len entries. x_out: n entries; v_out: n x steps or NULL. */
tpl_status tpl_lanczos_pass_two(tpl_op_t op, const double* b, int64_t b_len,
                                const double* alphas, size_t n_alphas, const double* betas,
                                size_t n_betas, size_t steps, double b_norm,
                                const double* y, size_t y_len, double* x_out,
                                double* v_out, int mem);

/* ---- data loader: src/utils/data_loader.rs:211-259 (load_kkt_system) ----- */
typedef struct tpl_csr_host {
  int64_t n, nnz;
  int64_t num_nodes, num_arcs; /* KKTSystem::num_nodes / num_arcs */
  int64_t* row_ptr;            /* n + 1 */
  int32_t* col_idx;            /* nnz, ascending within each row  */
  double* vals;                /* nnz */
} tpl_csr_host;
/* Parse a DIMACS .dmx + .qfc pair with the reference's exact semantics
 * (node-index 0 rejected; .qfc read as line 1 = m, then `skip(m).take(m)`
 * one-float-per-line — so the 3-line qfcgen format yields D = empty) and
 * assemble A = [[D, E^T],[E, 0]] as CSR. Free with tpl_csr_host_free.          */
tpl_status tpl_load_kkt_system(const char* dmx_path, const char* qfc_path, tpl_csr_host* out);
void tpl_csr_host_free(tpl_csr_host* csr);
/* Synthetic KKT instance for the scale-out config (BASELINE.json configs[4]; the
 * reference's netgen stops at 1.1M arcs, data/netgen/src/netgen.h:69-70): num_arcs arcs
 * (u, v), u != v, from a splitmix64 stream seeded by `seed`, with the netgen instances'
 * degree spread: each node draws an integer out-weight in [100, 1900]
 * and in-weight in [800, 1200]; tails are drawn in proportion to out-weight, heads to
 * in-weight (total degree / mean ~0.44 .. 1.58 at 5M arcs, like netgen's 0.5 .. 1.57 at
 * 500k). Ordered by (tail, head) like netgen output, D empty (the 3-line qfc case),
 * assembled exactly as tpl_load_kkt_system assembles a parsed .dmx; the same on every
 * platform (integer arithmetic only). num_nodes for a given m follows
 * data/qcnd/pargen.c:41-50: floor((1 + sqrt(1 + 8m/0.75)) / 2).              */
tpl_status tpl_generate_kkt(int64_t num_arcs, int64_t num_nodes, uint64_t seed,
                            tpl_csr_host* out);

/* ---- introspection / measurement ---------------------------------------- */
/* SpMV layout of the operator (DESIGN.md "SpMV layout"): rows with at most
 * short_row_max nnz ("short", ascending) are stored as sliced ELL, 512 rows per
 * chunk, one workgroup each; the n_long longer rows (ascending) are cut into S column
 * slices (tpl_op_slices) handled by XCD-local workgroups and summed by the last
 * arriver.
 * G2 workgroups of E elements run the element-wise kernels (= #norm partials).
 * short_rows_out: n_short int32 or NULL; long_rows_out: n_long int32 or NULL.
 * The CPU oracle uses this to reproduce the device reduction order bit for bit.   */
tpl_status tpl_op_schedule(tpl_op_t op, int32_t* n_short, int32_t* n_long, int32_t* G2,
                           int64_t* E, int32_t* short_rows_out, int32_t* long_rows_out);
/* Layout tuning (rebuilds the layout; 0 = keep): short_row_max (> 0: explicit,
 * -1: the default auto rule T = clamp(2 * median row nnz, 4, 32)), max_g2
 * (default 1024).                                                                */
tpl_status tpl_op_set_schedule(tpl_op_t op, int32_t short_row_max, int32_t max_g2);
/* Column slices S of the long rows (1, 2, 4 or 8; part of the canonical reduction
 * order). tpl_op_set_slices rebuilds the layout with an explicit S
 * (0 = the auto rule: the fewest slices whose share of the vector fits an eighth of an L2,
 * more if a (row, slice) piece would not fit one bin).                          */
tpl_status tpl_op_slices(tpl_op_t op, int32_t* slices);
tpl_status tpl_op_set_slices(tpl_op_t op, int32_t slices);

/* Second Gram-Schmidt passes of the last re-orthogonalised tpl_lanczos_standard call
 * (steps - 1 for CGS2; the count the selective mode actually ran).                */
tpl_status tpl_op_reorth_second_passes(tpl_op_t op, int64_t* count);
/* Device memory the operator holds now, in bytes: its layout (matrix in the engine's
 * format), the ten n-vectors of the recurrence, the solver state and — once a one-pass
 * solve (tpl_lanczos / tpl_lanczos_standard) has run — the basis V_k (8 n k bytes).
 * This is the device-side counterpart of the reference's peak-memory column
 * (src/utils/perf.rs:16-31, results/scalability_*.csv rss_kb): the two-pass variant
 * never allocates V_k.                                                            */
tpl_status tpl_op_device_bytes(tpl_op_t op, uint64_t* bytes);

/* Live timing of the solver's own launches: with timing on, HIP events on the
 * operator's stream bracket pass one's graph and the graph of pass two's step
 * launches (its prologue then runs as a separate launch), so the numbers come from
 * the very launches of the last solve, inside the caller's timed region.
 * pass2_spmv_us / pass2_launches is the average duration of one pass-two step
 * launch (k_p2_spmv), launch gaps included.                                      */
tpl_status tpl_op_enable_timing(tpl_op_t op, int on);
tpl_status tpl_op_pass_timing(tpl_op_t op, double* pass1_us, double* pass2_spmv_us,
                              int64_t* pass2_launches);
/* Live in-graph durations of pass one's two kernels: with timing on, the pass-one graph
 * of a single-GPU two-pass solve with a device f (k >= 11) has workgroup 0 of the
 * k_p1_spmv and k_p1_axpy launches of 8 consecutive middle steps record its start on the
 * GPU's 100 MHz real-time clock; this returns the average start-to-start interval of each
 * kernel (its launch plus the boundary after it, like pass2_spmv_us) over those steps of
 * the last timed solve, and the number of steps.                                   */
tpl_status tpl_op_step_samples(tpl_op_t op, double* p1_spmv_us, double* p1_axpy_us,
                               int32_t* samples);

/* ---- row-partitioned operator over several GPUs ----------
 * One process per GPU. Rank r holds the rows [starts[r], starts[r+1]) of A; every
 * SpMV gathers the full vector with an in-place all-gather (RCCL over xGMI) — or only
 * its halo (tpl_dist_op_create_halo), or, with replicated long rows, their partials
 * (tpl_dist_op_create_replicated) — and alpha / beta combine the ranks' totals (each rank reduces its own partials in the
 * single-GPU canonical order; the R totals are all-gathered and reduced in rank
 * order), so all ranks hold bitwise identical alpha, beta and steps. The solver
 * entry points above take a partitioned operator unchanged; b, x_out and v_out are
 * then this rank's block of rows. All ranks must make the same calls in the same
 * order (collective semantics). Re-orthogonalisation is not supported here.      */
typedef struct tpl_dist_s* tpl_dist_t;
enum { TPL_DIST_ID_BYTES = 128 };
/* Contiguous row blocks balanced by algorithmic bytes (12 per nonzero + 40 per row);
 * host only. starts: nranks + 1 entries.                                           */
tpl_status tpl_dist_partition(int64_t n, const int64_t* row_ptr, int nranks, int64_t* starts);
/* RCCL unique id (rank 0 creates it; the caller broadcasts the bytes).            */
tpl_status tpl_dist_unique_id(uint8_t* id);
tpl_status tpl_dist_create(int device, int rank, int nranks, const uint8_t* id, tpl_dist_t* out);
/* Test transport: all-gathers go through a host callback (recv = the ranks' send
 * buffers concatenated in rank order); synchronous, no graphs.                     */
typedef int (*tpl_allgather_fn)(const void* send, void* recv, size_t bytes_per_rank, void* user);
tpl_status tpl_dist_create_host(int device, int rank, int nranks, tpl_allgather_fn fn, void* user,
                                tpl_dist_t* out);
tpl_status tpl_dist_destroy(tpl_dist_t d);
/* This rank's block: row_ptr (n_local + 1, 0-based), global column indices.
 * Every SpMV all-gathers the whole vector (8n bytes moved per SpMV).              */
tpl_status tpl_dist_op_create_csr(tpl_dist_t d, int64_t n_global, const int64_t* starts,
                                  const int64_t* row_ptr, const int32_t* col_idx,
                                  const double* vals, tpl_op_t* out);
/* Replicated-long-row partition (the structure-aware split of SURVEY.md §8(e)), from
 * the WHOLE matrix (every rank passes the same CSR): the short rows are split into
 * contiguous byte-balanced blocks; the long rows are replicated — each rank sums the
 * entries in the columns it owns, the n_long partials are all-gathered (8 n_long
 * bytes per rank per SpMV) and every rank finishes them in rank order. Needs no halo:
 * a short row may only reference its own block and the long rows (true for the KKT
 * matrices: arc rows reference node rows only), else TPL_ERR_UNSUPPORTED.
 * This rank's vector is [its short rows | all long rows] (tpl_op_local_rows).        */
tpl_status tpl_dist_op_create_replicated(tpl_dist_t d, int64_t n, const int64_t* row_ptr,
                                         const int32_t* col_idx, const double* vals,
                                         tpl_op_t* out);
/* Halo-exchange row blocks (the general form of SURVEY.md §8(e) for matrices without
 * the KKT structure), from the WHOLE matrix (every rank passes the same CSR): rank r
 * holds the rows [starts[r], starts[r+1]) (starts NULL: the tpl_dist_partition split),
 * exactly as tpl_dist_op_create_csr, but an SpMV moves only the halo — the rows of each
 * block that another rank's rows reference (B_q for rank q, H = max_q |B_q|): each
 * rank packs its B_r into its slot and the slots are all-gathered (8 H bytes per rank
 * instead of 8 n / nranks; a banded matrix of half-bandwidth w has H <= 2w). Same
 * rows, layout and reduction order as tpl_dist_op_create_csr over the same split, so
 * alpha, beta, steps and x are bitwise those of the plain row blocks.
 * Like the two partitions above, it spreads the reference's one sequential
 * operator.apply (src/algorithms/mod.rs:177) over the ranks.                          */
tpl_status tpl_dist_op_create_halo(tpl_dist_t d, int64_t n, const int64_t* starts,
                                   const int64_t* row_ptr, const int32_t* col_idx,
                                   const double* vals, tpl_op_t* out);
/* The partition every binding's "auto" takes (Python mode="auto", C++ / Rust
 * Partition::Auto), decided on the host from the WHOLE matrix for `nranks` ranks, the same
 * on every rank: TPL_PLAN_REPLICATED when the replicated-long-row split applies (no short
 * row references another rank's short rows — the KKT case), else TPL_PLAN_HALO when the
 * halo width H is at most half the widest row block (banded, mesh-like matrices), else
 * TPL_PLAN_ROWS (the whole vector all-gathered; the three hold the same bits as their
 * partition oracles, and halo and rows the same bits as each other).                */
tpl_status tpl_dist_choose_partition(int64_t n, const int64_t* row_ptr, const int32_t* col_idx,
                                     int nranks, int* mode);
/* This rank's part of the WHOLE matrix in the partition tpl_dist_choose_partition picks
 * (collective: every rank passes the same CSR); *mode (may be NULL) receives it.    */
tpl_status tpl_dist_op_create_auto(tpl_dist_t d, int64_t n, const int64_t* row_ptr,
                                   const int32_t* col_idx, const double* vals, tpl_op_t* out,
                                   int* mode);
/* Global row index of each entry of this operator's vectors (tpl_op_nrows entries). */
tpl_status tpl_op_local_rows(tpl_op_t op, int64_t* rows);

/* Identity key of a caller's compressed-sparse matrix (host only, no device call), for
 * bindings that accept the caller's own matrix per call and keep its upload (the Rust
 * shim's `HipOperand for SparseColMatRef`, integration/rust/hip.rs): key[0] hashes the
 * three arrays' addresses and lengths and n; key[1] an FNV-1a checksum of the first and
 * last 8 words of each array and `samples` evenly spaced ones. The cost is O(samples),
 * not O(nnz): a change of addresses, sizes or any sampled word is seen, a change of an
 * unsampled word is not (callers that mutate a matrix in place re-upload explicitly).
 * ptr_elem / idx_elem: 4 or 8 (bytes per index).                                      */
tpl_status tpl_operand_key(int64_t n, const void* ptr_arr, size_t ptr_len, size_t ptr_elem,
                           const void* idx_arr, size_t idx_len, size_t idx_elem,
                           const double* vals, size_t nnz, size_t samples, uint64_t* key);

/* ---- host-only plans (no GPU): the reduction order an operator would hold --------
 * The host half of tpl_op_create_csr (mode TPL_PLAN_SINGLE: auto locality order, its
 * group count pinned by order_groups > 0 as tpl_op_set_order_groups does; nranks 1,
 * rank 0), of tpl_dist_op_create_replicated (TPL_PLAN_REPLICATED) or of a row-block
 * rank with the tpl_dist_partition split (TPL_PLAN_ROWS; TPL_PLAN_HALO: of
 * tpl_dist_op_create_halo, whose tpl_kernel_algo_bytes of the exchange ids then give
 * the halo's bytes without a GPU), run by the same code: rank
 * `rank` of `nranks`, its rows, order and SpMV layout, and nothing on a device. Only
 * the host introspection calls accept the returned handle — tpl_op_nrows, tpl_op_nnz,
 * tpl_op_flags, tpl_op_schedule, tpl_op_slices, tpl_op_permutation, tpl_op_local_rows,
 * tpl_op_order_groups, tpl_kernel_algo_bytes — every other call returns
 * TPL_ERR_INVALID_ARGUMENT; free it with tpl_op_destroy. The parity fixtures use it to
 * restate a run's reduction order on a host without a GPU (tests/golden/make_parity.py). */
enum { TPL_PLAN_SINGLE = 0, TPL_PLAN_REPLICATED = 1, TPL_PLAN_ROWS = 2, TPL_PLAN_HALO = 3 };
tpl_status tpl_plan_create(int64_t n, const int64_t* row_ptr, const int32_t* col_idx,
                           const double* vals, int mode, int nranks, int rank,
                           int32_t order_groups, tpl_op_t* out);

/* Kernel ids for tpl_profile_kernel */
enum {
  TPL_KERNEL_PASS1_SPMV = 0, /* pass one: SpMV + beta-AXPY + alpha partials             */
  TPL_KERNEL_PASS1_AXPY = 1, /* pass one: alpha-AXPY + ||w||^2 partials                 */
  TPL_KERNEL_PASS2_SPMV = 2, /* pass two: SpMV + both AXPYs + scale + x += y v          */
  TPL_KERNEL_SPMV = 3,       /* plain y = A x                                           */
  /* partitioned operators only (SURVEY.md §8(e) "comm fraction"): the exchanges one
   * step issues, exactly as the pass graphs issue them (rank totals + all-gathers)  */
  TPL_KERNEL_EXCHANGE_P1 = 4, /* a pass-one step's exchanges                           */
  TPL_KERNEL_EXCHANGE_P2 = 5, /* a pass-two step's exchange                            */
  TPL_KERNEL_PASS1_STEP = 6   /* k_p1_spmv then k_p1_axpy (one pass-one step, fixed j)  */
};
/* Time `iters` back-to-back launches of one kernel on the operator's stream with
 * HIP events (a warm-up launch first). Returns the average per launch in
 * microseconds (event-to-event, so it includes the launch gap) and the
 * algorithmic bytes one launch moves ("Algorithmic bytes"). The
 * exchange ids are collective: every rank calls with the same arguments; their
 * bytes are those one rank receives.                                            */
tpl_status tpl_profile_kernel(tpl_op_t op, int kernel, int iters, double* avg_us,
                              double* algo_bytes);
/* Algorithmic bytes of one launch of `kernel` (no GPU work). */
double tpl_kernel_algo_bytes(tpl_op_t op, int kernel);

/* Blocking copy of `bytes` from device memory to host memory (used by callbacks
 * that receive device views, e.g. tpl_step_cb's V_k). */
tpl_status tpl_copy_to_host(void* dst, const void* src_device, size_t bytes);

#ifdef __cplusplus
}
#endif
#endif /* TPL_H_ */
