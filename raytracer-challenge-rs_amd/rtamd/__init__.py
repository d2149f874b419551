"""rtamd — MI355X-native drop-in for raytracer-challenge-rs's render path.

`Camera.render(world)` (reference camera.rs:133-148) renders on the GPU through
the C-ABI in include/rt_render.h (librtamd.so, HIP kernels for gfx950). The
scene-building API mirrors the reference's Rust API (world.rs, camera.rs,
geometry/, material.rs, pattern/, transform.rs, matrix.rs).

Importing this package loads the native extension; it raises if the extension
has not been built (run `make -C raytracer-challenge-rs_amd` or
`python -c "import __graft_entry__ as g; g.build()"`). There is no CPU
fallback: rendering without a GPU raises RtError (RT_ERR_NO_DEVICE).
"""
import os as _os

_here = _os.path.dirname(_os.path.abspath(__file__))

# One HIP runtime per process: PyTorch-ROCm bundles its own libamdhip64 /
# libhsa-runtime64 (same SONAMEs as /opt/rocm's). Loading torch first makes
# librtamd.so bind to that already-loaded runtime, so device pointers and
# streams can be shared with torch (bench.py, torch.distributed). Without
# torch installed the system ROCm runtime is used.
try:  # pragma: no cover - environment dependent
    import torch as _torch  # noqa: F401
except ImportError:  # pragma: no cover
    _torch = None

try:
    from . import _rtamd  # noqa: F401
except ImportError as e:  # pragma: no cover - exercised when the build is missing
    raise ImportError(
        "rtamd native extension not built (expected rtamd/_rtamd*.so and lib/librtamd.so "
        f"under {_os.path.dirname(_here)}): {e}"
    ) from e

from ._rtamd import *  # noqa: F401,F403,E402
from ._rtamd import RtError, EPSILON  # noqa: E402

LIB_PATH = _os.path.join(_os.path.dirname(_here), "lib", "librtamd.so")
MAX_RECURSION_DEPTH = 5  # reference world.rs:16


def render_stream(dedicated_queue=False):
    """A torch stream for rendering frames concurrently (frames in flight,
    DESIGN.md §5.4), made by the library: by default a plain non-blocking
    stream (it takes one of the process's GPU_MAX_HW_QUEUES hardware queues;
    raise that variable before HIP initialises when rendering on several).
    dedicated_queue=True makes it through hipExtStreamCreateWithCUMask with
    every CU enabled, which gives it a hardware queue of its own, but every
    cross-stream event wait involving such a stream costs ~1 ms (DESIGN.md
    §5.4), so use it only for frames that never wait on another stream.
    Lives as long as the process."""
    return _torch.cuda.ExternalStream(_rtamd._stream_create(bool(dedicated_queue)))
