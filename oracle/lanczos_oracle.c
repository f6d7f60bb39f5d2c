/*
 * lanczos_oracle.c — CPU ORACLE (test infrastructure only; never shipped, never
 * on the product path). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.
 *
 * A plain-C restatement of the reference's Lanczos hot path
 * (lukefleed/two-pass-lanczos, Rust + faer 0.22.6, unbuildable here: no cargo):
 *   recurrence step   src/algorithms/mod.rs:167-212   (apply, -beta v_prev, alpha, -alpha v, ||w||)
 *   iteration state   src/algorithms/mod.rs:261-340   (v1 = b * (1/||b||), v = w * (1/beta))
 *   breakdown tol     src/algorithms/mod.rs:140-143   (1000 * f64::EPSILON, absolute)
 *   standard          src/algorithms/lanczos.rs:55-156
 *   pass one          src/algorithms/lanczos_two_pass.rs:65-110
 *   pass two          src/algorithms/lanczos_two_pass.rs:176-312
 *   reconstruction    src/solvers.rs:96-104           (x = ||b|| V_k y')
 *
 * Two reduction modes (everything else — the elementwise AXPY/scale rounding —
 * is identical in both and follows the reference op by op):
 *   FAITHFUL  (sched == NULL): CSR row-sequential ascending-column SpMV (the
 *             natural faer CSC scatter order), sequential dot and sum of
 *             squares. faer's own SIMD summation order is not pinned (its source
 *             is not vendored), so this is the "reference order" up to faer's
 *             dot/norm association — the CPU baseline of bench.py.
 *   CANONICAL (sched != NULL): reproduces the device's fixed reduction trees
 *             (two-pass-lanczos_amd/csrc/tpl_device.h) bit for bit, given the
 *             operator's layout (tpl_op_schedule).
 *
 * Build: make -C oracle (gcc, -ffp-contract=off so a*b-c stays two roundings).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define TPB 256
#define TOL 2.220446049250313080847263336181640625e-13 /* 1000 * f64::EPSILON */

enum { OR_OK = 0, OR_ZERO_B = 3, OR_BAD = 100 };

typedef struct {
  int64_t n;             /* rows */
  const int64_t* rp;
  const int32_t* ci;
  const double* v;
  int64_t ncols;         /* columns (<= 0: square); a rank's row block of a partition has
                          * n_global columns, and the long-row slices split those */
} ocsr;

static int64_t ncols_of(const ocsr* A) { return A->ncols > 0 ? A->ncols : A->n; }

typedef struct {
  int32_t n_short;
  const int32_t* srows;  /* short rows (sliced ELL), ascending */
  int32_t n_long;
  const int32_t* lrows;  /* long rows (column slices), ascending */
  int32_t G2;            /* element-wise workgroups == #norm partials */
  int64_t E;             /* elements per element-wise workgroup */
  int32_t slices;        /* column slices S of the long rows (1, 2, 4, 8) */
} osched;

#define CHUNK 512        /* short-row positions per sliced-ELL chunk (kChunkRows) */

/* ------------------------------------------------------------ trees */
static double tree64(double* a) { /* xor butterfly, offsets 1, 2, 4, 8, 16, 32 */
  /* lane 0's value after stage h only needs the lanes l = 0 mod 2h, and for those
   * l ^ h == l + h: the butterfly's lane 0 is this in-place pairwise tree (addition
   * is commutative, so a_l + a_{l^h} is the same bits for either operand order) */
  for (int h = 1; h < 64; h <<= 1)
    for (int l = 0; l < 64; l += 2 * h) a[l] = a[l] + a[l + h];
  return a[0];
}
static double tree256(const double* a) {
  double w[4], tmp[64];
  for (int q = 0; q < 4; ++q) {
    memcpy(tmp, a + 64 * q, sizeof(tmp));
    w[q] = tree64(tmp);
  }
  return (w[0] + w[1]) + (w[2] + w[3]);
}
static double reduce_partials(const double* P, int G) {
  double s[TPB];
  for (int t = 0; t < TPB; ++t) {
    s[t] = 0.0;
    for (int i = t; i < G; i += TPB) s[t] = s[t] + P[i];
  }
  return tree256(s);
}

/* ------------------------------------------------------------ SpMV */
static void spmv_faithful(const ocsr* A, const double* x, double* y) {
  #pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < A->n; ++i) {
    double s = 0.0;
    for (int64_t q = A->rp[i]; q < A->rp[i + 1]; ++q) s = s + A->v[q] * x[A->ci[q]];
    y[i] = s;
  }
}

/* long row: per slice s (columns [floor(n*s/S), floor(n*(s+1)/S))) the slice's entries
 * form a piece; a piece of at most BIG_PIECE entries: lane g (0..7) sums its entries
 * g + 8q, butterfly over the 8 lanes (xor 1, 2, 4); a longer piece: lane g (0..15) sums
 * its entries g + 16q, butterfly over 16 lanes. -> P_s; y = 0; y += P_s (s ascending). S: the
 * schedule's slice count (tpl_runtime.cpp auto_slices).
 * (device: long_bin in tpl_kernels.hip; kBigPiece in tpl_device.h) */
#define BIG_PIECE 64
static double long_row_canon(const ocsr* A, int32_t i, const double* x, int S) {
  const int64_t n = ncols_of(A);
  int64_t q = A->rp[i];
  double y = 0.0;
  for (int s = 0; s < S; ++s) {
    const int64_t bound = (s + 1 == S) ? INT64_MAX : n * (s + 1) / S;
    int64_t e = q;
    while (e < A->rp[i + 1] && A->ci[e] < bound) ++e;
    const int G = (e - q > BIG_PIECE) ? 16 : 8;
    double lane[16], nx[16];
    for (int g = 0; g < G; ++g) {
      double p = 0.0;
      for (int64_t k = q + g; k < e; k += G) p = p + A->v[k] * x[A->ci[k]];
      lane[g] = p;
    }
    for (int h = 1; h < G; h <<= 1) {
      for (int g = 0; g < G; ++g) nx[g] = lane[g] + lane[g ^ h];
      memcpy(lane, nx, (size_t)G * sizeof(double));
    }
    const double ps = lane[0];
    y = y + ps;
    q = e;
  }
  return y;
}

static void spmv_canon(const ocsr* A, const osched* S, const double* x, double* y) {
  #pragma omp parallel for schedule(static)
  for (int32_t p = 0; p < S->n_short; ++p) {
    const int32_t i = S->srows[p];
    double s = 0.0;
    for (int64_t q = A->rp[i]; q < A->rp[i + 1]; ++q) s = s + A->v[q] * x[A->ci[q]];
    y[i] = s;
  }
  #pragma omp parallel for schedule(static)
  for (int32_t r = 0; r < S->n_long; ++r) y[S->lrows[r]] = long_row_canon(A, S->lrows[r], x, S->slices);
}

static void spmv(const ocsr* A, const osched* S, const double* x, double* y) {
  if (S) spmv_canon(A, S, x, y);
  else spmv_faithful(A, x, y);
}

/* ------------------------------------------------------------ dot / norm */
/* alpha = v . w in device order: short chunk c -> partial c (thread t owns short
 * positions C*c + t + 256 q, C = CHUNK, fma accumulation, tree256); long row r ->
 * partial n_chunks + r = round(v * w); then reduce_partials over all of them. */
static double dot_canon(const osched* S, const double* v, const double* w, double* P) {
  const int32_t nch = (S->n_short + CHUNK - 1) / CHUNK;
#pragma omp parallel for schedule(static)
  for (int32_t c = 0; c < nch; ++c) {
    double acc[TPB];
    for (int t = 0; t < TPB; ++t) {
      acc[t] = 0.0;
      for (int q = 0; q < CHUNK / TPB; ++q) {
        const int32_t p = c * CHUNK + q * TPB + t;
        if (p < S->n_short) acc[t] = fma(v[S->srows[p]], w[S->srows[p]], acc[t]);
      }
    }
    P[c] = tree256(acc);
  }
  for (int32_t r = 0; r < S->n_long; ++r) P[nch + r] = v[S->lrows[r]] * w[S->lrows[r]];
  return reduce_partials(P, nch + S->n_long);
}
static double dot_faithful(int64_t n, const double* v, const double* w) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s = s + v[i] * w[i];
  return s;
}

/* ||x||^2: device order = E-partition, thread t visits pairs bE + 2t + 512q. */
static double nrm2_canon(const osched* S, int64_t n, const double* x, double* P) {
#pragma omp parallel for schedule(static)
  for (int b = 0; b < S->G2; ++b) {
    double acc[TPB];
    const int64_t beg = (int64_t)b * S->E;
    const int64_t end = beg + S->E < n ? beg + S->E : n;
    for (int t = 0; t < TPB; ++t) {
      double a = 0.0;
      for (int64_t i0 = beg + 2 * t; i0 < end; i0 += 2 * TPB) {
        a = fma(x[i0], x[i0], a);
        if (i0 + 1 < end) a = fma(x[i0 + 1], x[i0 + 1], a);
      }
      acc[t] = a;
    }
    P[b] = tree256(acc);
  }
  return reduce_partials(P, S->G2);
}
static double nrm2_faithful(int64_t n, const double* x) {
  double s = 0.0;
  for (int64_t i = 0; i < n; ++i) s = s + x[i] * x[i];
  return s;
}

/* ------------------------------------------------------------ re-orthogonalisation */
/* CGS2 of r against V[:, 0..cols) (column-major, ld = n), device order
 * (k_reorth_dot / k_reorth_reduce / k_reorth_update in tpl_kernels.hip): per pass,
 * h[c] = partials() of the G2 workgroup trees (workgroup b, thread t: acc = fma(V[c][i],
 * r[i], acc) over i = bE + t + 256q; tree256), then r[i] = r[i] - s_i with s_i = 0;
 * s_i = fma(V[c][i], h[c], s_i), c ascending. (Extension: the reference has no
 * re-orthogonalisation; pinned only against this restatement and orthonormality.) */
static double nrm2_canon(const osched* S, int64_t n, const double* x, double* P);
/* mode 1: CGS2 (two passes). mode 2: selective (Kahan–Parlett, k_reorth_decide): the
 * second pass runs only if ||r'||^2 < ||r||^2 / 2 after the first, both squared norms in
 * the canonical norm order. */
static void reorth_canon(const osched* S, int64_t n, const double* V, int cols, double* r,
                         double* P, double* h, int mode) {
  const double n0 = mode == 2 ? nrm2_canon(S, n, r, P) : 0.0;
  for (int pass = 0; pass < 2; ++pass) {
    if (mode == 2 && pass == 1 && nrm2_canon(S, n, r, P) >= 0.5 * n0) break;
    /* P[c * G2 + b]: the (column, workgroup) trees; workgroups are independent */
#pragma omp parallel for schedule(static)
    for (int b = 0; b < S->G2; ++b) {
      double acc[TPB];
      const int64_t beg = (int64_t)b * S->E;
      const int64_t end = beg + S->E < n ? beg + S->E : n;
      for (int c = 0; c < cols; ++c) {
        const double* col = V + (size_t)c * (size_t)n;
        for (int t = 0; t < TPB; ++t) {
          double a = 0.0;
          for (int64_t i = beg + t; i < end; i += TPB) a = fma(col[i], r[i], a);
          acc[t] = a;
        }
        P[(size_t)c * (size_t)S->G2 + (size_t)b] = tree256(acc);
      }
    }
    for (int c = 0; c < cols; ++c) h[c] = reduce_partials(P + (size_t)c * (size_t)S->G2, S->G2);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) {
      double sum = 0.0;
      for (int c = 0; c < cols; ++c) sum = fma(V[(size_t)c * (size_t)n + i], h[c], sum);
      r[i] = r[i] - sum;
    }
  }
}

/* ------------------------------------------------------------ drivers */
/* Standard / pass one. V (n x k, column-major) may be NULL (pass one). */
static int pass_one_impl(const ocsr* A, const osched* S, const double* b, size_t k,
                         double* alphas, double* betas, size_t* steps, double* bnorm_out,
                         double* V, int reorth) {
  const int64_t n = A->n;
  if (k == 0) return OR_BAD;
  if (reorth && (!S || !V)) return OR_BAD;
  double* h = reorth ? (double*)malloc(sizeof(double) * k) : NULL;
  const size_t np = S ? (size_t)(S->n_short + S->n_long + S->G2 + 1) : 0;
  double* P = S ? (double*)malloc(sizeof(double) * (reorth ? np + (size_t)S->G2 * k : np)) : NULL;
  double* vp = (double*)calloc((size_t)n + 1, sizeof(double));
  double* vc = (double*)malloc(sizeof(double) * ((size_t)n + 1));
  double* w = (double*)malloc(sizeof(double) * ((size_t)n + 1));
  const double bnorm = sqrt(S ? nrm2_canon(S, n, b, P) : nrm2_faithful(n, b));
  *bnorm_out = bnorm;
  *steps = 0;
  if (bnorm <= TOL) { /* src/algorithms/mod.rs:267-273 */
    free(P); free(vp); free(vc); free(w); free(h);
    return OR_ZERO_B;
  }
  const double inv0 = 1.0 / bnorm;
  #pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) vc[i] = b[i] * inv0;
  double beta_prev = 0.0;
  size_t nb = 0;
  for (size_t it = 0; it < k; ++it) {
    if (V) memcpy(V + it * (size_t)n, vc, sizeof(double) * (size_t)n);
    spmv(A, S, vc, w);                                                /* :177 */
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] - beta_prev * vp[i]; /* :184-186 */
    const double alpha = S ? dot_canon(S, vc, w, P) : dot_faithful(n, vc, w); /* :191 */
    alphas[it] = alpha;
    *steps = it + 1;
    if (it + 1 == k) break; /* beta_k is never used */
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] - alpha * vc[i];     /* :196-198 */
    if (reorth) reorth_canon(S, n, V, (int)(it + 1), w, P, h, reorth); /* extension */
    const double beta = sqrt(S ? nrm2_canon(S, n, w, P) : nrm2_faithful(n, w)); /* :202 */
    if (beta <= TOL) break;                                           /* :206-208 */
    betas[nb++] = beta;
    const double inv = 1.0 / beta;                                    /* :312-315 */
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] * inv;
    double* t = vp;
    vp = vc;
    vc = w;
    w = t;
    beta_prev = beta;
  }
  free(P); free(vp); free(vc); free(w); free(h);
  return OR_OK;
}
int oracle_pass_one(const ocsr* A, const osched* S, const double* b, size_t k, double* alphas,
                    double* betas, size_t* steps, double* bnorm_out, double* V) {
  return pass_one_impl(A, S, b, k, alphas, betas, steps, bnorm_out, V, 0);
}
/* lanczos_standard with CGS2 re-orthogonalisation (canonical order; V required). */
int oracle_pass_one_reorth(const ocsr* A, const osched* S, const double* b, size_t k,
                           double* alphas, double* betas, size_t* steps, double* bnorm_out,
                           double* V) {
  return pass_one_impl(A, S, b, k, alphas, betas, steps, bnorm_out, V, 1);
}
/* ... with the selective (Kahan–Parlett) variant. */
int oracle_pass_one_reorth_selective(const ocsr* A, const osched* S, const double* b, size_t k,
                                     double* alphas, double* betas, size_t* steps,
                                     double* bnorm_out, double* V) {
  return pass_one_impl(A, S, b, k, alphas, betas, steps, bnorm_out, V, 2);
}

/* Pass two; y already scaled by ||b||. V (n x steps) may be NULL. */
int oracle_pass_two(const ocsr* A, const osched* S, const double* b, const double* alphas,
                    const double* betas, size_t steps, double bnorm, const double* y, double* x,
                    double* V) {
  const int64_t n = A->n;
  if (bnorm <= TOL) return OR_ZERO_B; /* src/algorithms/lanczos_two_pass.rs:229-235 */
  if (steps == 0) {
    memset(x, 0, sizeof(double) * (size_t)n);
    return OR_OK;
  }
  double* vp = (double*)calloc((size_t)n + 1, sizeof(double));
  double* vc = (double*)malloc(sizeof(double) * ((size_t)n + 1));
  double* w = (double*)malloc(sizeof(double) * ((size_t)n + 1));
  const double inv0 = 1.0 / bnorm;
  #pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) vc[i] = b[i] * inv0;
  #pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) x[i] = vc[i] * y[0];
  if (V) memcpy(V, vc, sizeof(double) * (size_t)n);
  for (size_t j = 0; j + 1 < steps; ++j) {
    const double alpha = alphas[j], beta = betas[j], beta_prev = j == 0 ? 0.0 : betas[j - 1];
    spmv(A, S, vc, w);
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] - beta_prev * vp[i];
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] - alpha * vc[i];
    const double inv = 1.0 / beta;
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) w[i] = w[i] * inv;
    const double c = y[j + 1];
    #pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < n; ++i) x[i] = x[i] + c * w[i];
    double* t = vp;
    vp = vc;
    vc = w;
    w = t;
    if (V) memcpy(V + (j + 1) * (size_t)n, vc, sizeof(double) * (size_t)n);
  }
  free(vp); free(vc); free(w);
  return OR_OK;
}

/* x = ||b|| (V y'): canonical = per row fma chain over columns, then scale. */
void oracle_gemv_recon(int64_t n, size_t steps, const double* V, const double* yprime,
                       double bnorm, double* x, int canonical) {
  #pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < n; ++i) {
    double s = 0.0;
    if (canonical)
      for (size_t c = 0; c < steps; ++c) s = fma(V[c * (size_t)n + i], yprime[c], s);
    else
      for (size_t c = 0; c < steps; ++c) s = s + V[c * (size_t)n + i] * yprime[c];
    x[i] = bnorm * s;
  }
}

/* Threads of the row / block / element loops (results do not depend on it: every
 * parallel loop writes independent rows, partials or elements). bench.py's CPU
 * baseline sets 1 (the reference is single-threaded, Par::Seq). */
void oracle_set_threads(int t) {
#ifdef _OPENMP
  omp_set_num_threads(t > 0 ? t : 1);
#else
  (void)t;
#endif
}

void oracle_spmv(const ocsr* A, const osched* S, const double* x, double* y) { spmv(A, S, x, y); }

/* Building blocks of the partitioned orders (tests/partition_oracle.py composes them):
 * alpha partial total v . w of one operator's rows (device order, or sequential without
 * a schedule), sum of squares (no sqrt), partials() of an array, and the replicated long
 * rows' alpha partials (k_long_epi_p1: blocks of 256 long rows, thread t accumulates
 * fma(v, w) over rows t + 256 q, tree256). */
double oracle_dot(const osched* S, int64_t n, const double* v, const double* w) {
  if (!S) return dot_faithful(n, v, w);
  double* P = (double*)malloc(sizeof(double) * (size_t)(S->n_short + S->n_long + 1));
  const double r = dot_canon(S, v, w, P);
  free(P);
  return r;
}
double oracle_sumsq(const osched* S, int64_t n, const double* x) {
  if (!S) return nrm2_faithful(n, x);
  double* P = (double*)malloc(sizeof(double) * (size_t)(S->G2 + 1));
  const double r = nrm2_canon(S, n, x, P);
  free(P);
  return r;
}
double oracle_reduce(const double* P, int G) { return reduce_partials(P, G); }
#define LONG_EPI_ROWS 256 /* kLongEpiRows (tpl_device.h): one row per thread */
void oracle_long_alpha_blocks(int64_t nl, const double* v, const double* w, double* out) {
  const int64_t nb = (nl + LONG_EPI_ROWS - 1) / LONG_EPI_ROWS;
  for (int64_t b = 0; b < nb; ++b) {
    double acc[TPB];
    const int64_t l0 = b * LONG_EPI_ROWS;
    const int64_t l1 = l0 + LONG_EPI_ROWS < nl ? l0 + LONG_EPI_ROWS : nl;
    for (int t = 0; t < TPB; ++t) {
      double a = 0.0;
      for (int64_t l = l0 + t; l < l1; l += TPB) a = fma(v[l], w[l], a);
      acc[t] = a;
    }
    out[b] = tree256(acc);
  }
}

double oracle_nrm2(const osched* S, int64_t n, const double* x) {
  if (!S) return sqrt(nrm2_faithful(n, x));
  double* P = (double*)malloc(sizeof(double) * (size_t)(S->G2 + 1));
  const double r = sqrt(nrm2_canon(S, n, x, P));
  free(P);
  return r;
}
