"""tpl_amd — MI355X-native two-pass Lanczos engine for f(A) b.

Python mirror of the reference crate's public surface (lukefleed/two-pass-lanczos,
src/lib.rs:94-101) on top of the C ABI of libtpl_amd.so (include/tpl.h):

* ``lanczos``, ``lanczos_two_pass``          — src/solvers.rs (re-exported at the root)
* ``algorithms.*``                           — src/algorithms (low-level passes)
* ``error.LanczosError``                     — src/error.rs
* ``utils.data_loader.load_kkt_system``      — src/utils/data_loader.rs
* ``HipCsrOp``                               — the device-resident operator (faer LinOp)
"""
from . import _lib
from . import algorithms, error, ftk, solvers
from .error import DataLoaderError, LanczosError, LanczosErrorKind, TplError
from .operator import HipCsrOp, HostPlan, device_count, locality_order, refresh_uploaded
from .solvers import lanczos, lanczos_two_pass

__version__ = "0.1.0"
LIB_PATH = _lib.LIB_PATH

__all__ = [
    "lanczos", "lanczos_two_pass", "algorithms", "solvers", "error", "ftk", "HipCsrOp",
    "LanczosError", "LanczosErrorKind", "TplError", "DataLoaderError", "device_count",
    "locality_order", "HostPlan", "refresh_uploaded",
]
