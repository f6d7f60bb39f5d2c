"""Host/device vector marshalling for the C ABI (numpy on the host, torch on the GPU)."""
from __future__ import annotations

import numpy as np

from . import _lib


def _is_torch_cuda(x) -> bool:
    return type(x).__module__.startswith("torch") and getattr(x, "is_cuda", False)


class Vec:
    """A column vector handed to the C ABI: pointer, length, memory kind."""

    def __init__(self, b):
        if _is_torch_cuda(b):
            import torch
            if b.dim() == 2 and b.shape[1] != 1:
                raise ValueError("b must be an n x 1 column")
            self.obj = b.reshape(-1).to(torch.float64).contiguous()
            torch.cuda.synchronize(self.obj.device)
            self.ptr = self.obj.data_ptr()
            self.mem = _lib.TPL_MEM_DEVICE
        else:
            a = np.asarray(b, dtype=np.float64)
            if a.ndim == 2 and a.shape[1] != 1:
                raise ValueError("b must be an n x 1 column")
            self.obj = np.ascontiguousarray(a.reshape(-1))
            self.ptr = self.obj.ctypes.data
            self.mem = _lib.TPL_MEM_HOST
        self.n = int(self.obj.shape[0])

    def empty(self, *shape):
        """Output buffer on the same side as b; shape in C order."""
        if self.mem == _lib.TPL_MEM_DEVICE:
            import torch
            return torch.empty(shape, dtype=torch.float64, device=self.obj.device)
        return np.empty(shape, dtype=np.float64)

    @staticmethod
    def ptr_of(a) -> int:
        return a.data_ptr() if _is_torch_cuda(a) else a.ctypes.data
