"""ctypes wrapper of the C oracle (oracle/rt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, as the checker / CPU baseline. The product path
(raytracer-challenge-rs_amd/) never imports this module.

Scenes come in as the C-ABI shape descriptors (bytes of rt_shape_desc), the
same bytes the product uploads; the oracle rebuilds every object through its
own restatement of the reference API (including its own Matrix::inverse).
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
BUILD = os.path.join(HERE, "_build")
LIB = os.path.join(BUILD, "liboracle.so")


class Stats(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint64) for n in (
        "rays_primary", "rays_reflect", "rays_refract", "rays_shadow",
        "sphere_tests", "plane_tests", "sphere_disc_ge0", "other_tests")] + [
        ("ms_kernel", ctypes.c_double), ("ms_total", ctypes.c_double)] + [
        # ABI 3 (include/rt_render.h): what a GPU render executed; the oracle leaves them 0
        (n, ctypes.c_uint64) for n in ("rays_shadow_traced", "sphere_tests_executed", "box_tests_executed")] + [
        ("exhaustive", ctypes.c_uint32), ("_pad", ctypes.c_uint32)]
    # the reference's work counters (what the oracle counts)
    REFERENCE = ("rays_primary", "rays_reflect", "rays_refract", "rays_shadow",
                 "sphere_tests", "plane_tests", "sphere_disc_ge0", "other_tests")

    def as_dict(self):
        return {n: getattr(self, n) for n in self.REFERENCE}


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def _load():
    if not os.path.exists(LIB):
        build()
    lib = ctypes.CDLL(LIB)
    P, D, U, I, S = ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_uint32, ctypes.c_int, ctypes.c_size_t
    lib.oracle_world_new.restype = P
    lib.oracle_world_free.argtypes = [P]
    lib.oracle_world_set_default.argtypes = [P]
    lib.oracle_world_add_desc.argtypes = [P, ctypes.c_char_p]
    lib.oracle_world_add_desc.restype = I
    lib.oracle_world_add_light.argtypes = [P, D, D]
    lib.oracle_world_add_group.argtypes = [P, ctypes.c_char_p]
    lib.oracle_world_add_group.restype = I
    lib.oracle_world_set_last_group.argtypes = [P, I]
    lib.oracle_world_set_last_group.restype = I
    lib.oracle_matrix_inverse.argtypes = [D, D]
    lib.oracle_matrix_inverse.restype = I
    lib.oracle_camera_init.argtypes = [U, U, ctypes.c_double, D, ctypes.c_char_p]
    lib.oracle_camera_init.restype = I
    lib.oracle_color_at.argtypes = [P, D, U, D, ctypes.POINTER(Stats)]
    lib.oracle_is_shadowed.argtypes = [P, D, U]
    lib.oracle_is_shadowed.restype = I
    lib.oracle_hit.argtypes = [P, D, D]
    lib.oracle_render_rows.argtypes = [P, ctypes.c_char_p, U, U, ctypes.POINTER(ctypes.c_uint32), U, U, D,
                                       ctypes.POINTER(Stats)]
    lib.oracle_render_rows.restype = I
    lib.oracle_render_pixels.argtypes = [P, ctypes.c_char_p, U, U, ctypes.POINTER(ctypes.c_uint32), U, U, D,
                                         ctypes.POINTER(Stats)]
    lib.oracle_render_pixels.restype = I
    lib.oracle_canvas_to_ppm.argtypes = [D, U, U, ctypes.c_char_p, S]
    lib.oracle_canvas_to_ppm.restype = S
    lib.oracle_nan_seen.restype = I
    for f in ("oracle_sizeof_shape_desc", "oracle_sizeof_camera_desc", "oracle_sizeof_stats"):
        getattr(lib, f).restype = S
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _dptr(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


class OracleWorld:
    """The reference `World`, rebuilt from C-ABI descriptor bytes."""

    def __init__(self, descs=b"", lights=(), default=False, groups=b"", shape_groups=None):
        """`groups`: rt_group_desc bytes (parents first), `shape_groups`: the
        innermost group of each shape (-1: none) — a World with Groups
        flattened as rt_scene_create_groups takes it (group.rs)."""
        L = lib()
        self._w = L.oracle_world_new()
        if default:
            L.oracle_world_set_default(self._w)
            return
        gsz = 56  # sizeof(rt_group_desc)
        assert len(groups) % gsz == 0, "group descriptor size mismatch"
        for i in range(0, len(groups), gsz):
            if L.oracle_world_add_group(self._w, groups[i:i + gsz]) < 0:
                raise ValueError(f"oracle rejected group {i // gsz}")
        sz = L.oracle_sizeof_shape_desc()
        assert len(descs) % sz == 0, "descriptor size mismatch"
        for i in range(0, len(descs), sz):
            rc = L.oracle_world_add_desc(self._w, descs[i:i + sz])
            if rc != 0:
                raise ValueError(f"oracle rejected shape {i // sz}: rc={rc}")
            if shape_groups is not None and shape_groups[i // sz] >= 0:
                if L.oracle_world_set_last_group(self._w, int(shape_groups[i // sz])) != 0:
                    raise ValueError(f"oracle rejected the group of shape {i // sz}")
        for pos, inten in lights:
            p = np.asarray(pos, dtype=np.float64)
            c = np.asarray(inten, dtype=np.float64)
            L.oracle_world_add_light(self._w, _dptr(p), _dptr(c))

    @classmethod
    def from_world(cls, world):
        """From an rtamd.World (host API): descriptors + lights."""
        lb = np.frombuffer(world.lights_bytes(), dtype=np.float64).reshape(-1, 6)
        return cls(world.descs_bytes(), [(r[:3], r[3:]) for r in lb], groups=world.groups_bytes(),
                   shape_groups=world.shape_groups())

    def __del__(self):
        if getattr(self, "_w", None) and _lib is not None:
            _lib.oracle_world_free(self._w)
            self._w = None

    def color_at(self, origin, direction, remaining=5):
        ray = np.array(list(origin) + list(direction), dtype=np.float64)
        out = np.zeros(3)
        st = Stats()
        lib().oracle_color_at(self._w, _dptr(ray), remaining, _dptr(out), ctypes.byref(st))
        return out, st.as_dict()

    def color_at_batch(self, rays, remaining=5):
        rays = np.ascontiguousarray(rays, dtype=np.float64)
        out = np.zeros((len(rays), 3))
        tot = {}
        for i, r in enumerate(rays):
            c, st = self.color_at(r[:3], r[3:], remaining)
            out[i] = c
            for k, v in st.items():
                tot[k] = tot.get(k, 0) + v
        return out, tot

    def is_shadowed(self, point, light=0):
        p = np.asarray(point, dtype=np.float64)
        return bool(lib().oracle_is_shadowed(self._w, _dptr(p), light))

    def hit(self, origin, direction):
        ray = np.array(list(origin) + list(direction), dtype=np.float64)
        out = np.zeros(24)
        lib().oracle_hit(self._w, _dptr(ray), _dptr(out))
        return out

    def render_rows(self, camera_desc, max_depth, rows, nthreads=1, aa_samples=1):
        """Render the given rows (list of y) with the reference algorithm:
        `Camera::render` (aa_samples 1) or `render_multithreaded` with
        AA X2..X16. Returns (rgb[len(rows), hsize, 3], stats)."""
        hsize = np.frombuffer(camera_desc[:4], dtype=np.uint32)[0]
        rows = np.ascontiguousarray(rows, dtype=np.uint32)
        out = np.zeros((len(rows), hsize, 3))
        st = Stats()
        rc = lib().oracle_render_rows(self._w, camera_desc, max_depth, aa_samples,
                                 rows.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(rows),
                                 nthreads, _dptr(out), ctypes.byref(st))
        if rc != 0:
            raise ValueError(f"oracle_render_rows rc={rc}")
        return out, st.as_dict()

    def render_pixels(self, camera_desc, max_depth, xy, nthreads=1, aa_samples=1):
        """Render the pixels xy = [(x, y), ...] with the reference algorithm
        (as render_rows). Returns (rgb[len(xy), 3], stats)."""
        pix = np.ascontiguousarray(np.asarray(xy, dtype=np.uint32).reshape(-1, 2))
        out = np.zeros((len(pix), 3))
        st = Stats()
        rc = lib().oracle_render_pixels(self._w, camera_desc, max_depth, aa_samples,
                                   pix.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), len(pix),
                                   nthreads, _dptr(out), ctypes.byref(st))
        if rc != 0:
            raise ValueError(f"oracle_render_pixels rc={rc}")
        return out, st.as_dict()

    def render(self, camera_desc, max_depth, nthreads=1, aa_samples=1):
        vsize = int(np.frombuffer(camera_desc[4:8], dtype=np.uint32)[0])
        return self.render_rows(camera_desc, max_depth, list(range(vsize)), nthreads, aa_samples)


def matrix_inverse(m16):
    a = np.ascontiguousarray(m16, dtype=np.float64)
    out = np.zeros(16)
    rc = lib().oracle_matrix_inverse(_dptr(a), _dptr(out))
    if rc != 0:
        raise ValueError("not invertible")
    return out


def camera_desc(hsize, vsize, fov, transform16):
    buf = ctypes.create_string_buffer(lib().oracle_sizeof_camera_desc())
    t = np.ascontiguousarray(transform16, dtype=np.float64)
    rc = lib().oracle_camera_init(hsize, vsize, fov, _dptr(t), buf)
    assert rc == 0
    return buf.raw


def canvas_to_ppm(rgb):
    rgb = np.ascontiguousarray(rgb, dtype=np.float64)
    h, w = rgb.shape[:2]
    n = lib().oracle_canvas_to_ppm(_dptr(rgb), w, h, None, 0)
    buf = ctypes.create_string_buffer(n)
    lib().oracle_canvas_to_ppm(_dptr(rgb), w, h, buf, n)
    return buf.raw[:n]
