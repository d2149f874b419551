"""The specular term's pow on the device (rt_pow.hpp: glibc 2.35's pow,
operation for operation) equals the host's glibc pow bit for bit on the inputs
of tests/test_pow.py (lighting's domain and the algorithm's special paths)."""
import ctypes
import os

import numpy as np
import pytest

from test_pow import LIB, _libm_pow, pow_cases

pytestmark = pytest.mark.gpu


def test_device_pow_equals_glibc(rt):
    import torch
    x, y = pow_cases(200_000, seed=9)
    dx = torch.from_numpy(x).cuda()
    dy = torch.from_numpy(y).cuda()
    out = torch.empty_like(dx)
    lib = ctypes.CDLL(LIB)
    f = lib.rtamd_pow_device
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p]
    assert f(dx.data_ptr(), dy.data_ptr(), x.size, out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
    got = out.cpu().numpy()
    libm = _libm_pow()
    ref = np.array([libm(a, b) for a, b in zip(x.tolist(), y.tolist())])
    # (NaN results: the device's default NaN is positive, x86's negative; lighting never makes one)
    diff = np.flatnonzero((got.view(np.uint64) != ref.view(np.uint64)) & ~(np.isnan(got) & np.isnan(ref)))
    assert diff.size == 0, [(float.hex(x[i]), float.hex(y[i]), float.hex(ref[i]), float.hex(got[i])) for i in diff[:5]]
