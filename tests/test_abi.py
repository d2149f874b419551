"""The C-ABI boundary (include/rt_render.h) on CPU: the library loads,
exports every declared entry point, and fails loudly (no CPU fallback) when no
GPU is present. Validation that needs no device is exercised here too."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO

HEADER = os.path.join(REPO, "include", "rt_render.h")
LIB = os.path.join(PKG, "lib", "librtamd.so")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(rt_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("rt_scene_create", "rt_scene_destroy", "rt_render", "rt_render_shard_device",
                 "rt_render_multi", "rt_color_at_batch", "rt_is_shadowed_batch", "rt_hit_batch",
                 "rt_canvas_to_ppm", "rt_quantize_u8", "rt_matrix_inverse", "rt_camera_init",
                 "rt_last_error", "rt_abi_version", "rt_device_count", "rt_shard_rows", "rt_render_aa",
                 "rt_render_ex", "rt_render_shard_device_ex", "rt_color_at_batch_ex", "rt_render_ppm",
                 "rt_canvas_to_ppm_device"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(LIB)
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_abi_version_and_shard_rows():
    lib = ctypes.CDLL(LIB)
    assert lib.rt_abi_version() == 6
    f = lib.rt_shard_rows
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32] * 4
    # interleaved row blocks: every row owned exactly once
    for H, B, S in [(1080, 8, 1), (1080, 8, 2), (1080, 8, 8), (1081, 16, 3), (5, 8, 4), (0, 4, 2)]:
        assert sum(f(H, B, s, S) for s in range(S)) == H
    assert f(100, 0, 0, 1) == 0 and f(100, 4, 3, 3) == 0


def test_pattern_rows_partition():
    """rt_pattern_rows (ABI 6): a shard is the pattern (n, 1 << s); the masks of
    rtamd.distributed.block_patterns cover every row exactly once, rank 0's
    share reduced; invalid patterns own nothing."""
    import sys
    sys.path.insert(0, PKG)
    from rtamd.distributed import block_patterns, pattern_row_ids
    lib = ctypes.CDLL(LIB)
    g, s = lib.rt_pattern_rows, lib.rt_shard_rows
    g.restype = s.restype = ctypes.c_uint32
    g.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
    s.argtypes = [ctypes.c_uint32] * 4
    for H, B, S in [(1080, 8, 1), (1080, 8, 8), (1081, 16, 3), (4096, 8, 8), (5, 8, 4)]:
        for k in range(S):
            assert g(H, B, S, 1 << k) == s(H, B, k, S)
    for n, share in [(2, 0.93), (4, 0.86), (8, 0.75), (8, 0.5), (8, 1.0), (3, 0.8)]:
        period, masks = block_patterns(n, share)
        assert 1 <= period <= 64 and len(masks) == n
        assert sum(masks) == (1 << period) - 1 and all(m and not (m & o) for i, m in enumerate(masks)
                                                       for o in masks[i + 1:])
        for H, B in [(1080, 8), (4096, 8), (1081, 5)]:
            rows = [pattern_row_ids(H, B, period, m) for m in masks]
            assert sorted(y for r in rows for y in r) == list(range(H))
            assert [len(r) for r in rows] == [g(H, B, period, m) for m in masks]
        if share < 1.0:
            assert bin(masks[0]).count("1") < min(bin(m).count("1") for m in masks[1:])
    assert g(100, 4, 0, 1) == 0 and g(100, 4, 3, 8) == 0 and g(100, 4, 3, 0) == 0 and g(100, 4, 65, 1) == 0


def test_duplicate_shapes_rejected_before_any_device_work(rt):
    w = rt.World()
    w.add_object(rt.Sphere())
    w.add_object(rt.Sphere())  # structurally equal -> containers semantics ambiguous
    w.add_light(rt.PointLight(rt.Point(0, 0, -10), rt.Color(1, 1, 1)))
    with pytest.raises(rt.RtError, match="structurally equal"):
        w.upload()


def test_descriptor_layout_matches_oracle(rt, oracle):
    # the oracle and the product read the same rt_shape_desc / rt_camera_desc bytes
    L = oracle.lib()
    assert len(rt.Sphere().desc_bytes()) == L.oracle_sizeof_shape_desc() == 680
    assert len(rt.Camera(4, 3, 1.0).desc_bytes()) == L.oracle_sizeof_camera_desc() == 160
    assert L.oracle_sizeof_stats() == ctypes.sizeof(oracle.Stats) == 8 * 8 + 2 * 8 + 3 * 8 + 2 * 4


def test_cylinders_differing_only_in_bounds_are_not_duplicates(rt):
    w = rt.World()
    w.add_object(rt.Cylinder(0.0, 1.0, True))
    w.add_object(rt.Cylinder(0.0, 2.0, True))
    w.add_object(rt.Cone(-1.0, 0.0, False))
    w.add_object(rt.Cone(-1.0, 0.0, True))
    w.add_light(rt.PointLight(rt.Point(0, 0, -10), rt.Color(1, 1, 1)))
    try:
        w.upload()
    except rt.RtError as e:
        assert "structurally equal" not in str(e)
        assert "no HIP device" in str(e)


def test_duplicate_cubes_rejected(rt):
    w = rt.World()
    w.add_object(rt.Cube())
    w.add_object(rt.Cube())
    with pytest.raises(rt.RtError, match="structurally equal"):
        w.upload()


@pytest.mark.skipif(os.environ.get("RT_EXPECT_GPU") == "1", reason="GPU present")
def test_no_cpu_fallback_without_gpu(rt):
    if rt.device_count() > 0:
        pytest.skip("a GPU is visible")
    w = rt.World.default()
    c = rt.Camera(11, 11, 1.0)
    with pytest.raises(rt.RtError, match="no HIP device"):
        c.render(w)


def _host_buffer_lib():
    lib = ctypes.CDLL(LIB)
    lib.rt_host_buffer_alloc.restype = ctypes.c_void_p
    lib.rt_host_buffer_alloc.argtypes = [ctypes.c_size_t]
    lib.rt_host_buffer_free.argtypes = [ctypes.c_void_p]
    lib.rt_last_error.restype = ctypes.c_char_p
    return lib


def test_host_buffer_errors_without_crossing_the_abi():
    """rt_host_buffer_alloc reports failure as NULL + rt_last_error (zero bytes;
    no device here); rt_host_buffer_free(NULL) and of a foreign pointer are no-ops."""
    lib = _host_buffer_lib()
    assert lib.rt_host_buffer_alloc(0) is None
    assert b"zero bytes" in lib.rt_last_error()
    lib.rt_host_buffer_free(None)
    buf = ctypes.create_string_buffer(64)
    lib.rt_host_buffer_free(ctypes.addressof(buf))  # not a pool block: ignored


@pytest.mark.gpu
def test_host_buffer_pool_reuse_and_render():
    """Pinned blocks are pooled: a released block comes back for a request of
    about its size; a render canvas in pooled pinned memory equals the device frame."""
    from rtamd import scenes
    lib = _host_buffer_lib()
    p = lib.rt_host_buffer_alloc(8 << 20)
    assert p
    lib.rt_host_buffer_free(p)
    q = lib.rt_host_buffer_alloc((8 << 20) - 4096)
    assert q == p
    lib.rt_host_buffer_free(q)
    # a >= 4 MB render canvas takes pooled pinned pixels, written by DMA (rt_api.cpp copy_to_host)
    import torch
    w, cam, depth = scenes.c3(1024, 768, n_spheres=300)
    a, _ = cam.render(w, depth, want_stats=False)
    d = torch.empty((768, 1024, 3), dtype=torch.float64, device="cuda")
    cam.render_shard_device(w, depth, 8, 0, 1, d.data_ptr(), 0, False)
    torch.cuda.synchronize()
    assert a.to_numpy().tobytes() == d.cpu().numpy().tobytes()


def test_scene_create_groups_validation_without_gpu(rt):
    """rt_scene_create_groups (ABI 6) checks its group table before any device
    work: a parent must be -1 or an earlier group, a shape's group must exist;
    a valid hierarchy then fails only for want of a device (no CPU fallback)."""
    import struct
    lib = ctypes.CDLL(LIB)
    f = lib.rt_scene_create_groups
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p, ctypes.c_size_t,
                  ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]
    s1, s2 = rt.Sphere(), rt.Sphere()
    s2.set_transform(rt.translation(3, 0, 0))
    shapes = s1.desc_bytes() + s2.desc_bytes()

    def group(parent):  # rt_group_desc: min[3], max[3], parent, _pad (56 B)
        return struct.pack("<6dii", -1, -1, -1, 4, 1, 1, parent, 0)

    def create(groups, sg):
        out = ctypes.c_void_p()
        arr = (ctypes.c_int32 * len(sg))(*sg)
        rc = f(shapes, 2, arr, groups, len(groups) // 56, None, 0, 0, ctypes.byref(out))
        if rc == 0:  # (a GPU is present)
            lib.rt_scene_destroy.argtypes = [ctypes.c_void_p]
            lib.rt_scene_destroy(out)
        return rc

    assert create(group(-1) + group(5), [0, 1]) == -1  # parent after the group
    assert create(group(-1) + group(1), [0, 1]) == -1  # a group its own parent
    assert create(group(-2), [0, 0]) == -1
    assert create(group(-1), [0, 3]) == -1  # no group 3
    assert create(group(-1), [-2, 0]) == -1
    assert create(group(-1) + group(0), [1, -1]) in (0, -8)  # valid: RT_ERR_NO_DEVICE without a GPU
