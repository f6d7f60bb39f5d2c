//! `src/hip.rs` for lukefleed/two-pass-lanczos: the Rust side of the drop-in boundary
//! (include/tpl.h). Added to the reference crate as `pub mod hip;` next to `solvers`;
//! `build.rs` gains the two lines of `integration/rust/build_rs_snippet.rs`.
//!
//! Written against the reference's public API (src/solvers.rs:46-57,133-144,
//! src/algorithms/mod.rs:57-135, src/error.rs:11-58) and faer 0.22.6. This image has no
//! Rust toolchain, so the file is UNCOMPILED here; tests/native/abi_driver.cpp and
//! cpp_api_test.cpp make the same calls through the same C ABI and run in the test suite.
//!
//! The whole Lanczos loop runs on the GPU: Rust is called back only for `f_tk_solver`,
//! once per solve, exactly where src/solvers.rs:71-75 / :155-156 call it.

use crate::algorithms::LanczosDecomposition;
use crate::error::{LanczosError, LanczosErrorKind};
use faer::{Mat, MatRef};
use std::ffi::{c_char, c_int, c_void, CStr};

#[repr(C)]
pub struct TplCtx {
    _p: [u8; 0],
}
#[repr(C)]
pub struct TplOp {
    _p: [u8; 0],
}
type FtkFn = unsafe extern "C" fn(*const f64, usize, *const f64, usize, *mut f64, usize,
                                  *mut usize, *mut c_char, usize, *mut c_void) -> c_int;

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
                   user: *mut c_void, x_out: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_two_pass(op: *mut TplOp, b: *const f64, b_len: i64, k: usize, f: FtkFn,
                            user: *mut c_void, x_out: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_pass_one(op: *mut TplOp, b: *const f64, b_len: i64, k: usize,
                            alphas: *mut f64, betas: *mut f64, steps: *mut usize,
                            b_norm: *mut f64, mem: c_int) -> c_int;
    fn tpl_lanczos_pass_two(op: *mut TplOp, b: *const f64, b_len: i64, alphas: *const f64,
                            n_alphas: usize, betas: *const f64, n_betas: usize, steps: usize,
                            b_norm: f64, y: *const f64, y_len: usize, x_out: *mut f64,
                            v_out: *mut f64, mem: c_int) -> c_int;
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
        6 => LanczosErrorKind::SolverError(cstr(d.inner)),
        // 5 (EvdError) wraps faer's EvdError, which the engine cannot construct; the
        // built-in exp reports non-convergence as SolverError instead. Engine-only
        // statuses (>= 100: argument, device, memory, loader) have no LanczosErrorKind.
        _ => LanczosErrorKind::SolverError(cstr(d.message)),
    };
    Err(LanczosError(kind))
}

/// Device-resident symmetric CSR operator (the faer `SparseColMatRef<usize, f64>` the
/// binaries build, src/utils/data_loader.rs:211-259; symmetric, so CSC == CSR).
pub struct HipCsrOp {
    ctx: *mut TplCtx,
    op: *mut TplOp,
    n: usize,
}

impl HipCsrOp {
    pub fn from_csc(a: faer::sparse::SparseColMatRef<'_, usize, f64>, device: i32)
                    -> Result<Self, LanczosError> {
        let sym = a.symbolic(); // column pointers / row indices of A = A^T
        let rp: Vec<i64> = sym.col_ptr().iter().map(|&p| p as i64).collect();
        let ci: Vec<i32> = sym.row_idx().iter().map(|&r| r as i32).collect();
        let mut ctx = std::ptr::null_mut();
        let mut op = std::ptr::null_mut();
        unsafe {
            check(tpl_ctx_create(device, &mut ctx))?;
            if let Err(e) = check(tpl_op_create_csr(ctx, a.nrows() as i64, ci.len() as i64,
                                                    rp.as_ptr(), ci.as_ptr(), a.val().as_ptr(),
                                                    &mut op)) {
                tpl_ctx_destroy(ctx);
                return Err(e);
            }
        }
        Ok(Self { ctx, op, n: a.nrows() })
    }
    pub fn nrows(&self) -> usize {
        self.n
    }
    /// `LinOp::apply` (compatibility path: the solvers below never call it per step).
    pub fn apply(&self, x: &[f64]) -> Result<Vec<f64>, LanczosError> {
        let mut y = vec![0.0; self.n];
        unsafe { check(tpl_op_apply(self.op, x.as_ptr(), y.as_mut_ptr(), TPL_MEM_HOST))? };
        Ok(y)
    }
}

impl Drop for HipCsrOp {
    fn drop(&mut self) {
        unsafe {
            tpl_op_destroy(self.op);
            tpl_ctx_destroy(self.ctx);
        }
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
    let (sa, sb) = (std::slice::from_raw_parts(a, na), std::slice::from_raw_parts(b, nb));
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

fn column(b: MatRef<'_, f64>) -> Vec<f64> {
    (0..b.nrows()).map(|i| b[(i, 0)]).collect()
}

/// Drop-in for `solvers::lanczos_two_pass` (src/solvers.rs:133-175) on a HipCsrOp.
pub fn lanczos_two_pass<F>(op: &HipCsrOp, b: MatRef<'_, f64>, k: usize, mut f: F)
                           -> Result<Mat<f64>, LanczosError>
where
    F: FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>,
{
    let bv = column(b);
    let mut x = vec![0.0; op.n];
    unsafe {
        check(tpl_lanczos_two_pass(op.op, bv.as_ptr(), bv.len() as i64, k, ftk_trampoline::<F>,
                                   &mut f as *mut F as *mut c_void, x.as_mut_ptr(),
                                   TPL_MEM_HOST))?;
    }
    Ok(Mat::from_fn(op.n, 1, |i, _| x[i]))
}

/// Drop-in for `solvers::lanczos` (src/solvers.rs:46-107): V_k stays in HBM, x = ||b|| V_k y'.
pub fn lanczos<F>(op: &HipCsrOp, b: MatRef<'_, f64>, k: usize, mut f: F)
                  -> Result<Mat<f64>, LanczosError>
where
    F: FnMut(&[f64], &[f64]) -> Result<Mat<f64>, anyhow::Error>,
{
    let bv = column(b);
    let mut x = vec![0.0; op.n];
    unsafe {
        check(tpl_lanczos(op.op, bv.as_ptr(), bv.len() as i64, k, ftk_trampoline::<F>,
                          &mut f as *mut F as *mut c_void, x.as_mut_ptr(), TPL_MEM_HOST))?;
    }
    Ok(Mat::from_fn(op.n, 1, |i, _| x[i]))
}

/// `algorithms::lanczos_two_pass::lanczos_pass_one` (src/algorithms/lanczos_two_pass.rs:65-110).
pub fn lanczos_pass_one(op: &HipCsrOp, b: MatRef<'_, f64>, k: usize)
                        -> Result<LanczosDecomposition<f64>, LanczosError> {
    let bv = column(b);
    let (mut al, mut be) = (vec![0.0; k.max(1)], vec![0.0; k.max(1)]);
    let (mut steps, mut bn) = (0usize, 0.0f64);
    unsafe {
        check(tpl_lanczos_pass_one(op.op, bv.as_ptr(), bv.len() as i64, k, al.as_mut_ptr(),
                                   be.as_mut_ptr(), &mut steps, &mut bn, TPL_MEM_HOST))?;
    }
    al.truncate(steps);
    be.truncate(steps.saturating_sub(1));
    Ok(LanczosDecomposition { alphas: al, betas: be, steps_taken: steps, b_norm: bn })
}

/// `algorithms::lanczos_two_pass::lanczos_pass_two` (:128-140); y_k already scaled by ||b||.
pub fn lanczos_pass_two(op: &HipCsrOp, b: MatRef<'_, f64>, d: &LanczosDecomposition<f64>,
                        y_k: MatRef<'_, f64>) -> Result<Mat<f64>, LanczosError> {
    let bv = column(b);
    let yv = column(y_k);
    let mut x = vec![0.0; op.n];
    unsafe {
        check(tpl_lanczos_pass_two(op.op, bv.as_ptr(), bv.len() as i64, d.alphas.as_ptr(),
                                   d.alphas.len(), d.betas.as_ptr(), d.betas.len(),
                                   d.steps_taken, d.b_norm, yv.as_ptr(), yv.len(),
                                   x.as_mut_ptr(), std::ptr::null_mut(), TPL_MEM_HOST))?;
    }
    Ok(Mat::from_fn(op.n, 1, |i, _| x[i]))
}
