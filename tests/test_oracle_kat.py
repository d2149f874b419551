"""The oracle against the reference's own known-answer tests.

oracle/kat.c transcribes every #[test] on the render path (matrix.rs,
transform.rs, sphere.rs, plane.rs, intersection.rs, material.rs, pattern/,
world.rs, camera.rs, image/ppm.rs, and cube.rs / cylinder.rs / cone.rs) at
the reference tolerance (1e-5,
lib.rs:18-22). This is what pins the oracle.
"""
import os
import subprocess

import pytest

from conftest import REPO

KAT = os.path.join(REPO, "oracle", "_build", "kat")


@pytest.fixture(scope="module")
def kat_output():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    p = subprocess.run([KAT], capture_output=True, text=True, timeout=120)
    return p.returncode, p.stdout.splitlines()


EXPECTED = [
    "matrix_multiply_two_matrices", "matrix_multiply_point_vector", "matrix_determinant_4x4",
    "matrix_determinant_3x3_cofactors", "matrix_invertible_and_not", "matrix_inverse_1", "matrix_inverse_3",
    "matrix_product_by_inverse", "transform_chain", "view_transform_default_and_axes",
    "view_transform_arbitrary", "sphere_intersections", "sphere_normals", "plane_intersections_normal",
    "object_space_ray", "hit_rules", "computations_outside_inside", "computations_over_under_reflectv",
    "n1_n2_at_various_intersections", "schlick_cases", "shadow_hit_skips_no_shadow", "lighting_cases",
    "lighting_with_pattern", "stripe_pattern", "gradient_ring_checkers", "test_pattern_transforms",
    "world_intersect", "shade_intersection", "shade_intersection_inside", "color_at_miss_hit",
    "is_shadowed_cases", "shade_hit_in_shadow", "reflected_color_non_reflective",
    "reflected_color_reflective", "shade_hit_reflective", "reflected_color_max_depth",
    "mutually_reflective_terminates", "refracted_color_opaque", "refracted_color_max_depth",
    "refracted_color_total_internal_reflection", "refracted_color_with_refracted_ray",
    "shade_hit_transparent", "shade_hit_schlick", "camera_pixel_size", "camera_rays",
    "render_world_with_camera", "ppm_header_and_pixels", "ppm_color_component_scaling",
    "ppm_split_long_lines",
    # cube.rs / cylinder.rs / cone.rs and camera.rs AA offsets (row 2)
    "ray_intersects_cube", "ray_misses_cube", "normal_on_cube_surface", "cube_bounding_box",
    "ray_misses_cylinder", "ray_strikes_cylinder", "normal_vector_on_cylinder", "default_cylinder_min_max_closed",
    "intersect_constrained_cylinder", "intersect_caps_closed_cylinder", "normal_vector_on_cylinder_end_cap",
    "bounded_cylinder_bounding_box", "intersect_cone_with_ray", "intersect_cone_parallel_to_half",
    "intersect_cone_end_caps", "computing_normal_vector_cone", "bounded_cone_bounding_box",
    "rays_for_pixel_offsets", "bounding_box_intersects_cube_at_origin", "bounding_box_intersects_non_cubic",
    "group_box_gates_its_children"
]


@pytest.mark.parametrize("name", EXPECTED)
def test_reference_kat(kat_output, name):
    _, lines = kat_output
    assert f"ok {name}" in lines, [ln for ln in lines if name in ln]


def test_kat_all_pass(kat_output):
    rc, lines = kat_output
    assert rc == 0, "\n".join(ln for ln in lines if ln.startswith("FAIL"))
    assert lines[-1] == f"KAT {len(EXPECTED)}/{len(EXPECTED)}"
