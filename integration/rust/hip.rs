//! `src/hip.rs` for lukefleed/two-pass-lanczos: the Rust side of the drop-in boundary
//! (include/tpl.h). Added to the reference crate as `pub mod hip;` next to `solvers`;
//! `build.rs` gains the two lines of `integration/rust/build_rs_snippet.rs`.
//!
//! Every public item of the reference's Lanczos API has a counterpart here with the SAME
//! name, parameter names and parameter order, `stack: &mut MemStack` included, so a call
//! site compiles unchanged once its `use` line names `crate::hip` instead of
//! `crate::solvers` / `crate::algorithms::*`:
//!
//! | reference                                                           | here                                  |
//! |---------------------------------------------------------------------|---------------------------------------|
//! | `solvers::lanczos` (src/solvers.rs:46-57)                           | [`lanczos`] -> `tpl_lanczos`          |
//! | `solvers::lanczos_two_pass` (src/solvers.rs:133-144)                | [`lanczos_two_pass`] -> `tpl_lanczos_two_pass` |
//! | `lanczos::lanczos_standard` (src/algorithms/lanczos.rs:55-64)       | [`lanczos_standard`] -> `tpl_lanczos_standard` (+ `tpl_step_cb`) |
//! | `lanczos_two_pass::lanczos_pass_one` (lanczos_two_pass.rs:65-73)    | [`lanczos_pass_one`] -> `tpl_lanczos_pass_one` |
//! | `lanczos_two_pass::lanczos_pass_two` (lanczos_two_pass.rs:128-137)  | [`lanczos_pass_two`] -> `tpl_lanczos_pass_two` |
//! | `lanczos_two_pass::lanczos_pass_two_with_basis` (:149-158)          | [`lanczos_pass_two_with_basis`] -> `tpl_lanczos_pass_two` (`v_out`) |
//! | faer `LinOp<f64>` of `SparseColMatRef<usize, f64>` (mod.rs:177)     | `impl LinOp<f64> for HipCsrOp` -> `tpl_op_apply` |
//!
//! Two deliberate differences, both forced by the device:
//! * the scalar type is `f64` (the reference is generic over `T: ComplexField`, but every
//!   call site in `src/bin/*` and `tests/*` instantiates it with `f64`, and the engine is
//!   fp64 only); `T` and `T::Real` read `f64` below;
//! * `operator` is any [`HipOperand`] instead of any `LinOp<T>`: the engine's own
//!   [`HipCsrOp`] (upload once, the fast path), or the very `SparseColMatRef<usize, f64>` /
//!   `SparseColMat<usize, f64>` the call sites already pass (`&a.as_ref()` in
//!   src/bin/tradeoff.rs:268-284, src/bin/orthogonality.rs:180-197 and
//!   tests/correctness.rs:142), uploaded on first use and re-used while its operand key
//!   (include/tpl.h tpl_operand_key: the arrays' addresses and sizes plus a sampled
//!   checksum, O(4096) words per call) is unchanged; [`refresh_uploaded`] forces a new
//!   upload after an in-place change of values. [`HipCsrOp::from_csc`] once and `&op` per
//!   call is the zero-overhead form.
//!
//! `stack` is accepted and left untouched: the engine keeps its workspace in HBM
//! (faer's `apply_scratch` of [`HipCsrOp`] is empty for the same reason).
//!
//! Several GPUs (an extension: the reference is single-threaded, `Par::Seq`): one process
//! per GPU, each creates a [`HipDist`] (the RCCL communicator; rank 0's
//! [`HipDist::unique_id`] bytes reach the others by any channel the host program has —
//! MPI, a file, a socket) and then [`HipCsrOp::partitioned`] from the SAME whole matrix.
//! The functions below take the partitioned operator unchanged; `b` and the returned `x`
//! (and V_k) are then this rank's rows, [`HipCsrOp::local_rows`] — the same contract as
//! include/tpl.h's row-partitioned operators.
//!
//! Written against faer 0.22.6 (the reference's Cargo.toml). This image has no Rust
//! toolchain, so the file is UNCOMPILED here; tests/test_boundary.py type-checks every
//! `extern "C"` item, both callback types and the `#[repr(C)]` struct against
//! include/tpl.h, and every public signature against the reference's, and
//! tests/native/abi_driver.cpp / cpp_api_test.cpp make the same calls through the same
//! C ABI in the test suite.

use crate::algorithms::{
    LanczosCallback, LanczosDecomposition, LanczosOutput, LanczosPassTwoOutput,
    TridiagonalSystemView,
};
use crate::error::{LanczosError, LanczosErrorKind};
use faer::dyn_stack::{MemStack, StackReq};
use faer::matrix_free::LinOp;
use faer::sparse::{SparseColMat, SparseColMatRef};
use faer::{Mat, MatMut, MatRef, Par};
use std::cell::RefCell;
use std::ffi::{c_char, c_int, c_void, CStr};
use std::sync::{Arc, Mutex};

#[repr(C)]
pub struct TplCtx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct TplOp {
    _p: [u8; 0],
}
#[repr(C)]
pub struct TplDist {
    _p: [u8; 0],
}
/// TPL_DIST_ID_BYTES (include/tpl.h): the RCCL unique id rank 0 creates.
pub const TPL_DIST_ID_BYTES: usize = 128;
/// `tpl_ftk_fn` (include/tpl.h): the `f_tk_solver` closure behind a C callback.
type FtkFn = unsafe extern "C" fn(*const f64, usize, *const f64, usize, *mut f64, usize,
                                  *mut usize, *mut c_char, usize, *mut c_void) -> c_int;
/// `tpl_step_cb` (include/tpl.h): the `LanczosCallback` behind a C callback.
type StepCb = unsafe extern "C" fn(usize, *const f64, i64, *const f64, usize, *const f64,
                                   usize, *mut c_void) -> c_int;

const TPL_MEM_HOST: c_int = 0;

/// tpl_error_detail (include/tpl.h): the fields of the engine's LanczosErrorKind.
#[repr(C)]
struct TplErrorDetail {
    status: i32,
    message: *const c_char,
    inner: *const c_char,
    param_name: *const c_char,
    expected: u64,
    actual: u64,
    operator_cols: u64,
    vector_rows: u64,
    breakdown_step: u64,
}

extern "C" {
    fn tpl_last_error_detail(out: *mut TplErrorDetail) -> c_int;
    fn tpl_ctx_create(device: c_int, out: *mut *mut TplCtx) -> c_int;
    fn tpl_ctx_destroy(ctx: *mut TplCtx) -> c_int;
    fn tpl_op_create_csr(ctx: *mut TplCtx, n: i64, nnz: i64, row_ptr: *const i64,
                         col_idx: *const i32, vals: *const f64, out: *mut *mut TplOp) -> c_int;
    fn tpl_op_destroy(op: *mut TplOp) -> c_int;
    fn tpl_op_apply(op: *mut TplOp, x: *const f64, y: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos(op: *mut TplOp, b: *const f64, b_len: i64, k: usize, f: FtkFn,
                   f_user: *mut c_void, x_out: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_two_pass(op: *mut TplOp, b: *const f64, b_len: i64, k: usize, f: FtkFn,
                            f_user: *mut c_void, x_out: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_standard(op: *mut TplOp, b: *const f64, b_len: i64, k: usize,
                            alphas: *mut f64, betas: *mut f64, steps: *mut usize,
                            b_norm: *mut f64, v_out: *mut f64, mem: c_int, reorth: c_int,
                            cb: Option<StepCb>, cb_user: *mut c_void) -> c_int;
    fn tpl_lanczos_pass_one(op: *mut TplOp, b: *const f64, b_len: i64, k: usize,
                            alphas: *mut f64, betas: *mut f64, steps: *mut usize,
                            b_norm: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_pass_two(op: *mut TplOp, b: *const f64, b_len: i64, alphas: *const f64,
                            n_alphas: usize, betas: *const f64, n_betas: usize, steps: usize,
                            b_norm: f64, y: *const f64, y_len: usize, x_out: *mut f64,
                            v_out: *mut f64, mem: c_int) -> c_int;
    fn tpl_copy_to_host(dst: *mut c_void, src_device: *const c_void, bytes: usize) -> c_int;
    fn tpl_op_nrows(op: *mut TplOp) -> i64;
    fn tpl_op_local_rows(op: *mut TplOp, rows: *mut i64) -> c_int;
    fn tpl_dist_unique_id(id: *mut u8) -> c_int;
    fn tpl_dist_create(device: c_int, rank: c_int, nranks: c_int, id: *const u8,
                       out: *mut *mut TplDist) -> c_int;
    fn tpl_dist_destroy(d: *mut TplDist) -> c_int;
    fn tpl_dist_op_create_replicated(d: *mut TplDist, n: i64, row_ptr: *const i64,
                                     col_idx: *const i32, vals: *const f64,
                                     out: *mut *mut TplOp) -> c_int;
    fn tpl_dist_op_create_halo(d: *mut TplDist, n: i64, starts: *const i64,
                               row_ptr: *const i64, col_idx: *const i32, vals: *const f64,
                               out: *mut *mut TplOp) -> c_int;
    fn tpl_dist_op_create_auto(d: *mut TplDist, n: i64, row_ptr: *const i64,
                               col_idx: *const i32, vals: *const f64, out: *mut *mut TplOp,
                               mode: *mut c_int) -> c_int;
    fn tpl_operand_key(n: i64, ptr_arr: *const c_void, ptr_len: usize, ptr_elem: usize,
                       idx_arr: *const c_void, idx_len: usize, idx_elem: usize,
                       vals: *const f64, nnz: usize, samples: usize, key: *mut u64) -> c_int;
}

fn cstr(p: *const c_char) -> String {
    if p.is_null() {
        return String::new();
    }
    unsafe { CStr::from_ptr(p) }.to_string_lossy().into_owned()
}

/// tpl_status -> LanczosErrorKind, rebuilt from the variant's FIELDS (not by parsing the
/// message): the caller gets the reference's own variant, so `Display` and `PartialEq`
/// behave exactly as in src/error.rs:20-66.
fn check(st: c_int) -> Result<(), LanczosError> {
    if st == 0 {
        return Ok(());
    }
    let mut d = std::mem::MaybeUninit::<TplErrorDetail>::zeroed();
    let d = unsafe {
        tpl_last_error_detail(d.as_mut_ptr());
        d.assume_init()
    };
    let kind = match st {
        1 => LanczosErrorKind::Breakdown { k: d.breakdown_step as usize },
        2 => LanczosErrorKind::DimensionMismatch {
            operator_cols: d.operator_cols as usize,
            vector_rows: d.vector_rows as usize,
        },
        3 => LanczosErrorKind::InputError(cstr(d.inner)),
        4 => LanczosErrorKind::ParameterMismatch {
            param_name: cstr(d.param_name),
            expected: d.expected as usize,
            actual: d.actual as usize,
        },
        // the built-in exp's only failure is non-convergence (include/tpl.h tpl_ftk_exp)
        5 => LanczosErrorKind::EvdError(faer::linalg::evd::EvdError::NoConvergence),
        6 => LanczosErrorKind::SolverError(cstr(d.inner)),
        // Engine-only statuses (>= 100: argument, device, memory, loader) have no
        // LanczosErrorKind; they surface as SolverError with the engine's message.
        _ => LanczosErrorKind::SolverError(cstr(d.message)),
    };
    Err(LanczosError(kind))
}

/// Device-resident symmetric CSR operator (the faer `SparseColMatRef<usize, f64>` the
/// binaries build, src/utils/data_loader.rs:211-259; symmetric, so CSC == CSR).
pub struct HipCsrOp {
    ctx: *mut TplCtx,
    op: *mut TplOp,
    /// this operator's rows: all of A, or this rank's part of a partitioned A
    n: usize,
    /// One engine call at a time per operator (include/tpl.h: not re-entrant); this is
    /// what makes the operator `Sync`, as faer's `LinOp` requires. The operators of one
    /// communicator share ONE lock (their HipDist's): they share its stream and its RCCL
    /// communicator, so two of them must never capture graphs or issue collectives at once.
    lock: Arc<Mutex<()>>,
    /// partitioned: the communicator, kept alive until the operator is destroyed
    dist: Option<Arc<HipDist>>,
}

// SAFETY: the handles are only used under `lock`, and the engine's per-thread error
// text is read by `check` on the calling thread, inside the same critical section.
unsafe impl Send for HipCsrOp {}
unsafe impl Sync for HipCsrOp {}

impl core::fmt::Debug for HipCsrOp {
    fn fmt(&self, f: &mut core::fmt::Formatter<'_>) -> core::fmt::Result {
        f.debug_struct("HipCsrOp").field("n", &self.n).finish()
    }
}

/// The compact CSC arrays of `a` (faer allows non-compact storage: `col_nnz`), with the
/// engine's index types; A is symmetric, so these are also its CSR arrays.
fn compact_arrays(a: SparseColMatRef<'_, usize, f64>) -> (Vec<i64>, Vec<i32>, Vec<f64>) {
    let sym = a.symbolic();
    let mut rp = Vec::with_capacity(a.ncols() + 1);
    let mut ci = Vec::new();
    let mut v = Vec::new();
    rp.push(0i64);
    for j in 0..a.ncols() {
        ci.extend(sym.row_idx_of_col_raw(j).iter().map(|&r| r as i32));
        v.extend_from_slice(a.val_of_col(j));
        rp.push(ci.len() as i64);
    }
    (rp, ci, v)
}

impl HipCsrOp {
    /// Upload `a` once (the zero-overhead form: pass `&op` to the solvers below; no
    /// per-call host work beyond the call itself).
    pub fn from_csc(a: SparseColMatRef<'_, usize, f64>, device: i32)
                    -> Result<Self, LanczosError> {
        if a.nrows() != a.ncols() {
            return Err(LanczosError(LanczosErrorKind::DimensionMismatch {
                operator_cols: a.ncols(),
                vector_rows: a.nrows(),
            }));
        }
        let (rp, ci, v) = compact_arrays(a);
        Self::from_arrays(a.nrows(), &rp, &ci, &v, device)
    }

    fn from_arrays(n: usize, rp: &[i64], ci: &[i32], v: &[f64], device: i32)
                   -> Result<Self, LanczosError> {
        let mut ctx = std::ptr::null_mut();
        let mut op = std::ptr::null_mut();
        unsafe {
            check(tpl_ctx_create(device, &mut ctx))?;
            if let Err(e) = check(tpl_op_create_csr(ctx, n as i64, ci.len() as i64, rp.as_ptr(),
                                                    ci.as_ptr(), v.as_ptr(), &mut op)) {
                tpl_ctx_destroy(ctx);
                return Err(e);
            }
        }
        Ok(Self { ctx, op, n, lock: Arc::new(Mutex::new(())), dist: None })
    }

    /// This rank's part of the symmetric `a` over `dist`'s ranks (every rank passes the
    /// same whole matrix; collective: all ranks make the same calls in the same order).
    /// `Partition::Replicated` (the KKT form: tpl_dist_op_create_replicated, refused with
    /// a SolverError when a short row references another rank's short rows),
    /// `Partition::Halo` (any symmetric matrix: tpl_dist_op_create_halo over the
    /// byte-balanced row blocks), `Partition::Auto` (tpl_dist_op_create_auto: the rule the
    /// Python and C++ bindings share — replicated when it applies, else halo when the halo
    /// is at most half the widest block, else plain row blocks).
    pub fn partitioned(a: SparseColMatRef<'_, usize, f64>, dist: &Arc<HipDist>,
                       partition: Partition) -> Result<Self, LanczosError> {
        if a.nrows() != a.ncols() {
            return Err(LanczosError(LanczosErrorKind::DimensionMismatch {
                operator_cols: a.ncols(),
                vector_rows: a.nrows(),
            }));
        }
        let (rp, ci, v) = compact_arrays(a);
        let n = a.nrows() as i64;
        let mut op = std::ptr::null_mut();
        let _g = dist.lock.lock().unwrap();  // the communicator's stream and comm
        unsafe {
            match partition {
                Partition::Replicated => check(tpl_dist_op_create_replicated(
                    dist.d, n, rp.as_ptr(), ci.as_ptr(), v.as_ptr(), &mut op))?,
                Partition::Halo => check(tpl_dist_op_create_halo(
                    dist.d, n, std::ptr::null(), rp.as_ptr(), ci.as_ptr(), v.as_ptr(), &mut op))?,
                Partition::Auto => check(tpl_dist_op_create_auto(
                    dist.d, n, rp.as_ptr(), ci.as_ptr(), v.as_ptr(), &mut op,
                    std::ptr::null_mut()))?,
            }
            let nl = tpl_op_nrows(op) as usize;
            Ok(Self { ctx: std::ptr::null_mut(), op, n: nl, lock: dist.lock.clone(),
                      dist: Some(dist.clone()) })
        }
    }

    /// The global row of each entry of this operator's vectors (`b` and `x` of the
    /// functions below hold these rows, in this order).
    pub fn local_rows(&self) -> Result<Vec<i64>, LanczosError> {
        let mut rows = vec![0i64; self.n.max(1)];
        let _g = self.lock.lock().unwrap();
        unsafe { check(tpl_op_local_rows(self.op, rows.as_mut_ptr()))? };
        rows.truncate(self.n);
        Ok(rows)
    }

    pub fn nrows(&self) -> usize {
        self.n
    }

    /// y = A x for one host vector (the per-call compatibility path).
    pub fn apply_vec(&self, x: &[f64]) -> Result<Vec<f64>, LanczosError> {
        let mut y = vec![0.0; self.n];
        let _g = self.lock.lock().unwrap();
        unsafe { check(tpl_op_apply(self.op, x.as_ptr(), y.as_mut_ptr(), TPL_MEM_HOST))? };
        Ok(y)
    }
}

impl Drop for HipCsrOp {
    fn drop(&mut self) {
        unsafe {
            tpl_op_destroy(self.op);
            if !self.ctx.is_null() {
                tpl_ctx_destroy(self.ctx);
            }
        }
        // `dist` (the communicator) is released after the operator, when its field drops
    }
}

/// How [`HipCsrOp::partitioned`] splits the matrix over the ranks (include/tpl.h).
#[derive(Clone, Copy, Debug, PartialEq, Eq)]
pub enum Partition {
    Replicated,
    Halo,
    Auto,
}

/// One rank's RCCL communicator over xGMI (tpl_dist_create).
pub struct HipDist {
    d: *mut TplDist,
    /// Held around every engine call that touches this communicator or its stream: every
    /// operator built on it takes THIS lock as its own (HipCsrOp::lock), so two operators
    /// sharing an `Arc<HipDist>` never capture graphs or issue collectives concurrently.
    lock: Arc<Mutex<()>>,
}

// SAFETY: the handle is only used under `lock` (operator creation here, every solver call
// through the operators, which share the lock).
unsafe impl Send for HipDist {}
unsafe impl Sync for HipDist {}

impl HipDist {
    /// Rank 0: the id every rank passes to [`HipDist::new`].
    pub fn unique_id() -> Result<[u8; TPL_DIST_ID_BYTES], LanczosError> {
        let mut id = [0u8; TPL_DIST_ID_BYTES];
        unsafe { check(tpl_dist_unique_id(id.as_mut_ptr()))? };
        Ok(id)
    }

    /// This process's rank of `nranks` on GPU `device` (collective over the ranks).
    pub fn new(device: i32, rank: i32, nranks: i32, id: &[u8; TPL_DIST_ID_BYTES])
               -> Result<std::sync::Arc<Self>, LanczosError> {
        let mut d = std::ptr::null_mut();
        unsafe { check(tpl_dist_create(device, rank, nranks, id.as_ptr(), &mut d))? };
        Ok(Arc::new(Self { d, lock: Arc::new(Mutex::new(())) }))
    }
}

impl Drop for HipDist {
    fn drop(&mut self) {
        unsafe {
            tpl_dist_destroy(self.d);
        }
    }
}

/// faer's `LinOp<f64>` over `tpl_op_apply`: a compatibility path, so the reference's own
/// generic code (e.g. `solvers::lanczos` itself) can run with the product on the GPU. The
/// solvers of this module never use it — they hand the whole recurrence to the engine.
/// (For a partitioned operator it is this rank's block of rows, a collective call.)
impl LinOp<f64> for HipCsrOp {
    fn apply_scratch(&self, _rhs_ncols: usize, _par: Par) -> StackReq {
        StackReq::EMPTY // the engine's workspace lives in HBM
    }
    fn nrows(&self) -> usize {
        self.n
    }
    fn ncols(&self) -> usize {
        self.n
    }
    fn apply(&self, mut out: MatMut<'_, f64>, rhs: MatRef<'_, f64>, _par: Par,
             _stack: &mut MemStack) {
        // faer's own products panic on a shape mismatch; so does this one
        assert!(rhs.nrows() == self.n && out.nrows() == self.n && out.ncols() == rhs.ncols());
        let mut x = vec![0.0; self.n];
        for j in 0..rhs.ncols() {
            for i in 0..self.n {
                x[i] = rhs[(i, j)];
            }
            let y = self.apply_vec(&x).unwrap_or_else(|e| panic!("tpl_op_apply: {e}"));
            for i in 0..self.n {
                out[(i, j)] = y[i];
            }
        }
    }
    fn conj_apply(&self, out: MatMut<'_, f64>, rhs: MatRef<'_, f64>, par: Par,
                  stack: &mut MemStack) {
        self.apply(out, rhs, par, stack) // real: conj(A) = A
    }
}

/// What the functions below accept as `operator`.
pub trait HipOperand {
    /// Runs `g` on the device operator holding this matrix.
    fn with_hip_op<R, G: FnOnce(&HipCsrOp) -> R>(&self, g: G) -> Result<R, LanczosError>;
}

impl HipOperand for HipCsrOp {
    fn with_hip_op<R, G: FnOnce(&HipCsrOp) -> R>(&self, g: G) -> Result<R, LanczosError> {
        Ok(g(self))
    }
}

thread_local! {
    /// The last faer matrix uploaded on this thread: (operand key, operator).
    static UPLOADED: RefCell<Option<([u64; 2], HipCsrOp)>> = const { RefCell::new(None) };
}

/// Words of each array the operand key samples (include/tpl.h tpl_operand_key).
const KEY_SAMPLES: usize = 4096;

/// The identity of `a` as this thread last uploaded it (tpl_operand_key): its three
/// arrays' addresses and lengths, its dimension, and a checksum of 3 x (KEY_SAMPLES + 16)
/// words — O(KEY_SAMPLES) host work per solver call (≈10 µs), not the O(nnz) copy and
/// hash of the whole matrix (that cost sat inside the reference's own timing
/// window, src/bin/tradeoff.rs:267-286).
fn operand_key(a: SparseColMatRef<'_, usize, f64>) -> Result<[u64; 2], LanczosError> {
    let sym = a.symbolic();
    let (cp, ri, v) = (sym.col_ptr(), sym.row_idx(), a.val());
    let w = std::mem::size_of::<usize>();
    let mut key = [0u64; 2];
    unsafe {
        check(tpl_operand_key(a.nrows() as i64, cp.as_ptr() as *const c_void, cp.len(), w,
                              ri.as_ptr() as *const c_void, ri.len(), w, v.as_ptr(), v.len(),
                              KEY_SAMPLES, key.as_mut_ptr()))?
    };
    Ok(key)
}

/// Forget this thread's upload of a faer matrix: the next solver call uploads it again.
/// Needed only after changing a matrix's values IN PLACE (same arrays, same sizes) between
/// calls — the key sees new arrays, new sizes and any change in its sampled words, not a
/// change of every single word. `HipCsrOp::from_csc` (upload once, pass `&op`) has no
/// per-call host cost at all and is the form to use in new code.
pub fn refresh_uploaded() {
    UPLOADED.with(|cell| *cell.borrow_mut() = None);
}

/// The reference's call sites pass `&a.as_ref()`: upload on first use (device 0, or
/// `TPL_DEVICE`), reuse while the operand key is unchanged (per call: the key, no copy).
impl<'a> HipOperand for SparseColMatRef<'a, usize, f64> {
    fn with_hip_op<R, G: FnOnce(&HipCsrOp) -> R>(&self, g: G) -> Result<R, LanczosError> {
        if self.nrows() != self.ncols() {
            return Err(LanczosError(LanczosErrorKind::DimensionMismatch {
                operator_cols: self.ncols(),
                vector_rows: self.nrows(),
            }));
        }
        let key = operand_key(*self)?;
        UPLOADED.with(|cell| {
            let mut slot = cell.borrow_mut();
            if !matches!(&*slot, Some((k, _)) if *k == key) {
                *slot = None; // free the previous upload before the new one
                let device = std::env::var("TPL_DEVICE").ok()
                    .and_then(|s| s.parse().ok()).unwrap_or(0);
                *slot = Some((key, HipCsrOp::from_csc(*self, device)?));
            }
            Ok(g(&slot.as_ref().unwrap().1))
        })
    }
}

impl HipOperand for SparseColMat<usize, f64> {
    fn with_hip_op<R, G: FnOnce(&HipCsrOp) -> R>(&self, g: G) -> Result<R, LanczosError> {
        self.as_ref().with_hip_op(g)
    }
}

/// The FnMut closure of `solvers::lanczos*` behind the C callback (called once).
unsafe extern "C" fn ftk_trampoline<F>(a: *const f64, na: usize, b: *const f64, nb: usize,
                                       y: *mut f64, cap: usize, len: *mut usize,
                                       err: *mut c_char, ecap: usize, user: *mut c_void) -> c_int
where
    F: FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>,
{
    let f = &mut *(user as *mut F);
    let sa = if na == 0 { &[][..] } else { std::slice::from_raw_parts(a, na) };
    let sb = if nb == 0 { &[][..] } else { std::slice::from_raw_parts(b, nb) };
    match f(sa, sb) {
        Ok(m) => {
            *len = m.nrows();
            if m.ncols() != 1 || m.nrows() > cap {
                // the engine reports ParameterMismatch (src/solvers.rs:78-85,158-165)
                *len = if m.nrows() != na { m.nrows() } else { na + 1 };
                return 0;
            }
            for i in 0..m.nrows() {
                *y.add(i) = m[(i, 0)];
            }
            0
        }
        Err(e) => {
            let s = e.to_string();
            let n = s.len().min(ecap.saturating_sub(1));
            std::ptr::copy_nonoverlapping(s.as_ptr() as *const c_char, err, n);
            *err.add(n) = 0;
            1
        }
    }
}

/// `LanczosCallback` behind `tpl_step_cb`. The engine hands V_k as a DEVICE pointer; the
/// host copy grows by the new columns only (O(nk) copied over the whole run, the same
/// memory the reference's stored basis takes), and the view the callback sees is the
/// reference's: n x k, column-major, plus T_k's scalars.
struct StepState<'c> {
    cb: &'c mut LanczosCallback<f64>,
    v: Vec<f64>,
    filled: usize,
    failed: Option<LanczosError>,
}

unsafe extern "C" fn step_trampoline(k: usize, v_dev: *const f64, n: i64, al: *const f64,
                                     na: usize, be: *const f64, nb: usize,
                                     user: *mut c_void) -> c_int {
    let st = &mut *(user as *mut StepState<'_>);
    let n = n as usize;
    if k > st.filled {
        let off = st.filled * n;
        let bytes = (k - st.filled) * n * std::mem::size_of::<f64>();
        if let Err(e) = check(tpl_copy_to_host(st.v.as_mut_ptr().add(off) as *mut c_void,
                                               v_dev.add(off) as *const c_void, bytes)) {
            st.failed = Some(e);
            return 0; // stop; the error is returned after the call
        }
        st.filled = k;
    }
    let view = TridiagonalSystemView {
        alphas: if na == 0 { &[][..] } else { std::slice::from_raw_parts(al, na) },
        betas: if nb == 0 { &[][..] } else { std::slice::from_raw_parts(be, nb) },
        steps_taken: k,
    };
    let v_k = MatRef::from_column_major_slice(&st.v[..k * n], n, k);
    (st.cb)(k, v_k, &view) as c_int
}

fn column(b: MatRef<'_, f64>) -> Vec<f64> {
    (0..b.nrows()).map(|i| b[(i, 0)]).collect()
}

fn column_major(v: &[f64], n: usize, cols: usize) -> Mat<f64> {
    Mat::from_fn(n, cols, |i, j| v[i + j * n])
}

/// Drop-in for `solvers::lanczos` (src/solvers.rs:46-107): V_k stays in HBM, x = ||b|| V_k y'.
pub fn lanczos<O, F>(
    operator: &O,
    b: MatRef<'_, f64>,
    k: usize,
    stack: &mut MemStack,
    mut f_tk_solver: F,
) -> Result<Mat<f64>, LanczosError>
where
    O: HipOperand,
    F: FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>,
{
    let _ = stack;
    let bv = column(b);
    operator.with_hip_op(|op| {
        let mut x = vec![0.0; op.n];
        let _g = op.lock.lock().unwrap();
        unsafe {
            check(tpl_lanczos(op.op, bv.as_ptr(), bv.len() as i64, k, ftk_trampoline::<F>,
                              &mut f_tk_solver as *mut F as *mut c_void, x.as_mut_ptr(),
                              TPL_MEM_HOST))?;
        }
        Ok(Mat::from_fn(op.n, 1, |i, _| x[i]))
    })?
}

/// Drop-in for `solvers::lanczos_two_pass` (src/solvers.rs:133-175).
pub fn lanczos_two_pass<O, F>(
    operator: &O,
    b: MatRef<'_, f64>,
    k: usize,
    stack: &mut MemStack,
    mut f_tk_solver: F,
) -> Result<Mat<f64>, LanczosError>
where
    O: HipOperand,
    F: FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>,
{
    let _ = stack;
    let bv = column(b);
    operator.with_hip_op(|op| {
        let mut x = vec![0.0; op.n];
        let _g = op.lock.lock().unwrap();
        unsafe {
            check(tpl_lanczos_two_pass(op.op, bv.as_ptr(), bv.len() as i64, k,
                                       ftk_trampoline::<F>,
                                       &mut f_tk_solver as *mut F as *mut c_void,
                                       x.as_mut_ptr(), TPL_MEM_HOST))?;
        }
        Ok(Mat::from_fn(op.n, 1, |i, _| x[i]))
    })?
}

/// Drop-in for `algorithms::lanczos::lanczos_standard` (src/algorithms/lanczos.rs:55-156):
/// V_k is built in HBM and returned as the reference's `Mat`; the callback, when given,
/// sees exactly the reference's arguments and may stop the run early (a stop at step j
/// returns the j-step result, include/tpl.h `tpl_step_cb`).
pub fn lanczos_standard(
    operator: &impl HipOperand,
    b: MatRef<'_, f64>,
    k: usize,
    stack: &mut MemStack,
    callback: Option<&mut LanczosCallback<f64>>,
) -> Result<LanczosOutput<f64>, LanczosError> {
    let _ = stack;
    let bv = column(b);
    operator.with_hip_op(|op| {
        let n = op.n;
        let (mut al, mut be) = (vec![0.0; k.max(1)], vec![0.0; k.max(1)]);
        let (mut steps, mut bn) = (0usize, 0.0f64);
        let mut v = vec![0.0; n * k];
        let mut state = callback.map(|cb| StepState { cb, v: vec![0.0; n * k], filled: 0,
                                                      failed: None });
        let (cb, user): (Option<StepCb>, *mut c_void) = match state.as_mut() {
            Some(s) => (Some(step_trampoline as StepCb), s as *mut StepState<'_> as *mut c_void),
            None => (None, std::ptr::null_mut()),
        };
        let _g = op.lock.lock().unwrap();
        let st = unsafe {
            tpl_lanczos_standard(op.op, bv.as_ptr(), bv.len() as i64, k, al.as_mut_ptr(),
                                 be.as_mut_ptr(), &mut steps, &mut bn, v.as_mut_ptr(),
                                 TPL_MEM_HOST, 0, cb, user)
        };
        if let Some(e) = state.and_then(|s| s.failed) {
            return Err(e);
        }
        check(st)?;
        al.truncate(steps);
        be.truncate(steps.saturating_sub(1));
        Ok(LanczosOutput {
            v_k: column_major(&v, n, steps),
            decomposition: LanczosDecomposition { alphas: al, betas: be, steps_taken: steps,
                                                  b_norm: bn },
        })
    })?
}

/// Drop-in for `algorithms::lanczos_two_pass::lanczos_pass_one` (lanczos_two_pass.rs:65-110).
pub fn lanczos_pass_one(
    operator: &impl HipOperand,
    b: MatRef<'_, f64>,
    k: usize,
    stack: &mut MemStack,
) -> Result<LanczosDecomposition<f64>, LanczosError> {
    let _ = stack;
    let bv = column(b);
    operator.with_hip_op(|op| {
        let (mut al, mut be) = (vec![0.0; k.max(1)], vec![0.0; k.max(1)]);
        let (mut steps, mut bn) = (0usize, 0.0f64);
        let _g = op.lock.lock().unwrap();
        unsafe {
            check(tpl_lanczos_pass_one(op.op, bv.as_ptr(), bv.len() as i64, k, al.as_mut_ptr(),
                                       be.as_mut_ptr(), &mut steps, &mut bn, TPL_MEM_HOST))?;
        }
        al.truncate(steps);
        be.truncate(steps.saturating_sub(1));
        Ok(LanczosDecomposition { alphas: al, betas: be, steps_taken: steps, b_norm: bn })
    })?
}

/// Both pass-two entry points: `v_out` = the regenerated basis (with_basis) or none.
fn pass_two(op: &HipCsrOp, b: MatRef<'_, f64>, d: &LanczosDecomposition<f64>,
            y_k: MatRef<'_, f64>, with_basis: bool)
            -> Result<(Mat<f64>, Option<Mat<f64>>), LanczosError> {
    let bv = column(b);
    let yv = column(y_k);
    let n = op.n;
    let mut x = vec![0.0; n];
    let mut v = if with_basis { vec![0.0; n * d.steps_taken] } else { Vec::new() };
    let v_ptr = if with_basis { v.as_mut_ptr() } else { std::ptr::null_mut() };
    let _g = op.lock.lock().unwrap();
    unsafe {
        check(tpl_lanczos_pass_two(op.op, bv.as_ptr(), bv.len() as i64, d.alphas.as_ptr(),
                                   d.alphas.len(), d.betas.as_ptr(), d.betas.len(),
                                   d.steps_taken, d.b_norm, yv.as_ptr(), yv.len(),
                                   x.as_mut_ptr(), v_ptr, TPL_MEM_HOST))?;
    }
    let basis = with_basis.then(|| column_major(&v, n, d.steps_taken));
    Ok((Mat::from_fn(n, 1, |i, _| x[i]), basis))
}

/// Drop-in for `algorithms::lanczos_two_pass::lanczos_pass_two` (:128-140); y_k already
/// scaled by ||b||.
pub fn lanczos_pass_two(
    operator: &impl HipOperand,
    b: MatRef<'_, f64>,
    decomposition: &LanczosDecomposition<f64>,
    y_k: MatRef<'_, f64>,
    stack: &mut MemStack,
) -> Result<Mat<f64>, LanczosError> {
    let _ = stack;
    operator.with_hip_op(|op| pass_two(op, b, decomposition, y_k, false).map(|(x, _)| x))?
}

/// Drop-in for `algorithms::lanczos_two_pass::lanczos_pass_two_with_basis` (:149-166):
/// x_k and the regenerated basis V'_k (bitwise the one pass one / `lanczos_standard`
/// generates on the device: DESIGN.md §5 P1).
pub fn lanczos_pass_two_with_basis(
    operator: &impl HipOperand,
    b: MatRef<'_, f64>,
    decomposition: &LanczosDecomposition<f64>,
    y_k: MatRef<'_, f64>,
    stack: &mut MemStack,
) -> Result<LanczosPassTwoOutput<f64>, LanczosError> {
    let _ = stack;
    operator.with_hip_op(|op| {
        pass_two(op, b, decomposition, y_k, true)
            .map(|(x_k, v_k)| LanczosPassTwoOutput { x_k, v_k: v_k.unwrap() })
    })?
}
