"""Panel plumbing for the host mirror: turn torch / numpy inputs into (pointer, S, T, ld).

Device path: torch CUDA(HIP) float64 tensors, (T,) for one series or (S, T) for a
panel with unit stride along time; the call runs on torch's current stream.
Host path: numpy float64 arrays; the `_host` C entry points stage them through HBM
(the JNI path).  torch is plumbing only (device memory + streams).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from .errors import raise_for_status


def is_torch(x) -> bool:
    try:
        import torch
    except ImportError:  # pragma: no cover
        return False
    return isinstance(x, torch.Tensor)


class Panel:
    """A 2-D view (S, T) of a series or panel plus its C-ABI description."""

    def __init__(self, x, name="ts"):
        self.orig = x
        self.device = is_torch(x)
        if self.device:
            import torch
            if x.dtype != torch.float64:
                raise TypeError("%s: expected float64, got %s" % (name, x.dtype))
            if x.device.type != "cuda":
                raise TypeError("%s: torch tensors must live on the GPU (there is no CPU path); "
                                "pass a numpy array for the host-staging path" % name)
            self.squeeze = x.dim() == 1
            t2 = x.unsqueeze(0) if self.squeeze else x
            if t2.dim() != 2:
                raise ValueError("%s: expected a series (T,) or a panel (S, T)" % name)
            if t2.shape[1] > 1 and t2.stride(1) != 1:
                t2 = t2.contiguous()
            self.t = t2
            self.S, self.T = int(t2.shape[0]), int(t2.shape[1])
            self.ld = int(t2.stride(0)) if self.S > 1 else self.T
            if self.ld < self.T:
                t2 = t2.contiguous()
                self.t = t2
                self.ld = self.T
            self.ptr = t2.data_ptr()
            _native.ensure_device(t2.device.index if t2.device.index is not None else torch.cuda.current_device())
        else:
            a = np.asarray(x, dtype=np.float64)
            self.squeeze = a.ndim == 1
            a2 = a.reshape(1, -1) if self.squeeze else a
            if a2.ndim != 2:
                raise ValueError("%s: expected a series (T,) or a panel (S, T)" % name)
            a2 = np.ascontiguousarray(a2)
            self.t = a2
            self.S, self.T = a2.shape
            self.ld = self.T
            self.ptr = a2.ctypes.data

    # new output of the same kind and shape
    def empty(self, S=None, T=None):
        S = self.S if S is None else S
        T = self.T if T is None else T
        if self.device:
            import torch
            return torch.empty((S, T), dtype=torch.float64, device=self.t.device)
        return np.empty((S, T), dtype=np.float64)

    def empty_i32(self, n):
        if self.device:
            import torch
            return torch.zeros((n,), dtype=torch.int32, device=self.t.device)
        return np.zeros((n,), dtype=np.int32)

    def vec(self, values, n, name):
        """per-series parameter vector (scalar broadcast) of the same kind"""
        if self.device:
            import torch
            if is_torch(values):
                v = values.to(device=self.t.device, dtype=torch.float64).reshape(-1)
            else:
                v = torch.as_tensor(np.asarray(values, dtype=np.float64).reshape(-1), device=self.t.device)
            if v.numel() == 1 and n != 1:
                v = v.expand(n)
            v = v.contiguous()
        else:
            v = np.asarray(values.cpu().numpy() if is_torch(values) else values, dtype=np.float64).reshape(-1)
            if v.size == 1 and n != 1:
                v = np.full(n, v[0])
            v = np.ascontiguousarray(v)
        if (v.numel() if self.device else v.size) != n:
            raise ValueError("%s: expected %d values, got %d" % (name, n, v.numel() if self.device else v.size))
        return v

    def out(self, y):
        """shape an output like the input (drop the series axis for a single series)"""
        return y[0] if self.squeeze else y

    @property
    def stream(self):
        if not self.device:
            return None
        import torch
        return ctypes.c_void_p(torch.cuda.current_stream(self.t.device).cuda_stream)


def ptr(x):
    if x is None:
        return None
    if is_torch(x):
        return ctypes.c_void_p(x.data_ptr())
    return ctypes.c_void_p(x.ctypes.data)


def check(status, what):
    raise_for_status(status, what)
