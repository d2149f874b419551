"""Host-side checks of the builders in rt_bvh.cpp, compiled with g++ from the
library's own sources and run on random sphere fields of C3 and C5 sizes:
the four-wide hierarchy (wide_layout, rt_layout.hpp BvhWide)
at the leaf sizes the builder takes (exactness of the culling rests on every
slot's box holding the records below it, the LDS stack on the reported
bound), and the light buffer (build_light_buffer, threaded over faces and
cells) at the resolutions the library uses, and the line hierarchy
(build_line_bvh: leaves, and cone clusters whose test opens for every
direction taking a member's a ~ 0 branch)."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "raytracer-challenge-rs_amd", "csrc")


@pytest.fixture(scope="module")
def wide_check(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("wide") / "wide_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", CSRC, os.path.join(REPO, "tests", "cpp", "wide_check.cpp"),
                    os.path.join(CSRC, "rt_bvh.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("n,leaf,span", [(1, 1, 10), (5, 8, 4), (9, 2, 6), (1000, 2, 12), (1000, 4, 12),
                                         (3000, 1, 30), (9996, 1, 50), (9996, 2, 50)])
def test_wide_layout_invariants(wide_check, n, leaf, span):
    r = subprocess.run([wide_check, str(n), str(leaf), str(span)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.fixture(scope="module")
def lb_check(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("lb") / "lb_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-I", CSRC, os.path.join(REPO, "tests", "cpp", "lb_check.cpp"),
                    os.path.join(CSRC, "rt_bvh.cpp"), "-o", exe], check=True)
    return exe


@pytest.mark.parametrize("n,res", [(7, 3), (300, 64), (1000, 256), (9996, 512)])
def test_light_buffer_invariants(lb_check, n, res):
    r = subprocess.run([lb_check, str(n), str(res)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr


@pytest.fixture(scope="module")
def line_check(tmp_path_factory):
    if not shutil.which("g++"):
        pytest.skip("no g++")
    exe = str(tmp_path_factory.mktemp("line") / "line_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", CSRC,
                    os.path.join(REPO, "tests", "cpp", "line_check.cpp"), os.path.join(CSRC, "rt_bvh.cpp"), "-o", exe],
                   check=True)
    return exe


@pytest.mark.parametrize("n,upright", [(1, 1.0), (7, 0.5), (200, 0.5), (200, 1.0), (200, 0.0), (1500, 0.5)])
def test_line_hierarchy_gates(line_check, n, upright):
    r = subprocess.run([line_check, str(n), str(upright)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.startswith("OK"), r.stdout + r.stderr
