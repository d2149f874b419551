"""Host side of the boundary (CPU): the C++ mirror of the reference API
(csrc/host/rt_math.hpp, rt_world.hpp) against the reference's known answers
and, bit for bit, against the oracle's independent restatement."""
import math
import struct

import numpy as np
import pytest

PI = math.pi


def test_matrix_known_answers(rt):
    # matrix.rs:569-604 (inverse_matrix1)
    a = rt.Matrix.from_rows([[-5, 2, 6, -8], [1, -5, 1, 8], [7, 7, -6, -7], [1, -3, 7, 4]])
    b = a.inverse()
    assert rt.equal(a.determinant(), 532.0)
    assert rt.equal(a.cofactor(2, 3), -160.0) and rt.equal(b[3, 2], -160.0 / 532.0)
    assert b == rt.Matrix.from_rows([[0.21805, 0.45113, 0.24060, -0.04511],
                                     [-0.80827, -1.45677, -0.44361, 0.52068],
                                     [-0.07895, -0.22368, -0.05263, 0.19737],
                                     [-0.52256, -0.81391, -0.30075, 0.30639]])
    # matrix.rs:551-565: not invertible -> error instead of panic
    singular = rt.Matrix.from_rows([[-4, 2, -2, -3], [9, 6, 2, 6], [0, -5, 1, -5], [0, 0, 0, 0]])
    assert not singular.is_invertible()
    with pytest.raises(rt.RtError):
        singular.inverse()
    # transform.rs:308-325 (arbitrary view transform)
    t = rt.view_transform(rt.Point(1, 3, 2), rt.Point(4, -2, 8), rt.Vector(1, 1, 0))
    assert t == rt.Matrix.from_rows([[-0.50709, 0.50709, 0.67612, -2.36643],
                                     [0.76772, 0.60609, 0.12122, -2.82843],
                                     [-0.35857, 0.59761, -0.71714, 0.0], [0, 0, 0, 1]])
    # matrix.rs:656-663 fluent chaining
    t = rt.Matrix.identity(4, 4).rotate_x(PI / 2.0).scale(5, 5, 5).translate(10, 5, 7)
    assert t * rt.Point(1, 0, 1) == rt.Point(15, 0, 7)


def test_camera_known_answers(rt):
    # camera.rs:287-325
    assert rt.equal(rt.Camera(200, 125, PI / 2.0).pixel_size, 0.01)
    assert rt.equal(rt.Camera(125, 200, PI / 2.0).pixel_size, 0.01)
    c = rt.Camera(201, 101, PI / 2.0)
    r = c.ray_for_pixel(0, 0)
    assert r.origin == rt.Point(0, 0, 0) and r.direction == rt.Vector(0.66519, 0.33259, -0.66851)
    c.set_transform(rt.rotation_y(PI / 4.0) * rt.translation(0, -2, 5))
    r = c.ray_for_pixel(100, 50)
    assert r.origin == rt.Point(0, 2, -5)
    assert r.direction == rt.Vector(math.sqrt(2) / 2, 0.0, -math.sqrt(2) / 2)


def _random_affine(rng):
    m = rt_mod.rotation_x(rng.uniform(-3, 3)) * rt_mod.rotation_y(rng.uniform(-3, 3))
    m = m * rt_mod.shearing(*rng.uniform(-0.5, 0.5, 6)) * rt_mod.scaling(*rng.uniform(0.1, 3.0, 3))
    return rt_mod.translation(*rng.uniform(-20, 20, 3)) * m


rt_mod = None


def test_inverse_bitwise_equal_to_oracle(rt, oracle):
    """The product's Matrix::inverse (C++) and the oracle's (C) are the same
    cofactor expansion: every bit must agree."""
    global rt_mod
    rt_mod = rt
    rng = np.random.default_rng(1234)
    for _ in range(300):
        m = _random_affine(rng)
        ours = np.array(m.inverse().to_list())
        ref = oracle.matrix_inverse(m.to_list())
        assert ours.tobytes() == ref.tobytes()
        assert np.array(rt.matrix_inverse_raw(m.to_list())).tobytes() == ref.tobytes()


def test_camera_desc_bitwise_equal_to_oracle(rt, oracle):
    for (w, h, fov) in [(11, 11, PI / 2), (200, 100, PI / 3), (125, 200, PI / 2), (1920, 1080, PI / 3), (1, 1, 1.0)]:
        c = rt.Camera(w, h, fov)
        t = rt.view_transform(rt.Point(0, 3, -12), rt.Point(0, 1, 5), rt.Vector(0, 1, 0))
        c.set_transform(t)
        assert c.desc_bytes() == oracle.camera_desc(w, h, fov, t.to_list())


def test_scene_descs_match_oracle_rebuild(rt, oracle):
    """Every shape descriptor the host produces decodes, in the oracle, to the
    same transform inverse (the oracle recomputes it independently)."""
    from rtamd import scenes
    w, _, _ = scenes.zoo()
    raw = w.descs_bytes()
    sz = oracle.lib().oracle_sizeof_shape_desc()
    for i in range(w.n_objects()):
        d = raw[i * sz:(i + 1) * sz]
        transform = np.frombuffer(d[8:8 + 128], dtype=np.float64)
        inverse = np.frombuffer(d[136:136 + 128], dtype=np.float64)
        ident = np.eye(4).ravel()
        if transform.tobytes() != ident.tobytes():
            assert oracle.matrix_inverse(transform).tobytes() == inverse.tobytes()


def test_splitmix64_known_values():
    from rtamd.scenes import SplitMix64
    g = SplitMix64(0)
    # reference values of splitmix64 seeded with 0
    assert [g.next_u64() for _ in range(3)] == [0xE220A8397B1DCDAF, 0x6E789E6AA1B965F4, 0x06C45D188009454F]
    g = SplitMix64(0x5EED0003)
    us = [g.u() for _ in range(1000)]
    assert all(0.0 <= u < 1.0 for u in us)


def test_scene_generators_deterministic(rt):
    from rtamd import scenes
    a, _, _ = scenes.c3(64, 36)
    b, _, _ = scenes.c3(64, 36)
    assert a.descs_bytes() == b.descs_bytes()
    assert a.n_objects() == 1001 and a.n_lights() == 1
    c5, cam, depth = scenes.c5(64, 64)
    assert c5.n_objects() == 10000 and c5.n_lights() == 2 and depth == 8


def test_canvas_bounds_and_pixels(rt):
    c = rt.Canvas(10, 20)
    assert c.width() == 10 and c.height() == 20
    c.set_pixel(2, 3, rt.Color(1, 0, 0))
    assert c.get_pixel(2, 3) == rt.Color(1, 0, 0)
    with pytest.raises(IndexError):
        c.get_pixel(10, 0)  # canvas.rs:78-90 should_panic -> exception
    a = c.to_numpy()
    assert a.shape == (20, 10, 3) and a[3, 2, 0] == 1.0
