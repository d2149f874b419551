"""Scene recipes for the benchmark configurations.

Built only through the public host API (the same calls the reference's demo
binaries make: Sphere()/Plane(), set_transform, material fields, add_object,
add_light, view_transform). Random scenes use splitmix64 so that any language
can regenerate them bit-for-bit.

  C1  200x100, one sphere, one light (bin/sphere_with_light.rs:34-40)
  C2  800x600, 3 spheres on a plane, Phong only, depth 1 (bin/first_scene.rs)
  C3  1920x1080, floor + 1000 random spheres, depth 5   <- headline workload
  C5  4096x4096, 4 planes + 9996 spheres, 2 lights, depth 8
  zoo a feature scene: patterns of every kind, rotated/sheared transforms,
      nested glass, a shadowless object, two lights (parity coverage)
"""
import math

from . import _rtamd as rt

PI = math.pi
MASK64 = (1 << 64) - 1


class SplitMix64:
    """splitmix64; u() = (z >> 11) * 2**-53 in [0, 1)."""

    def __init__(self, seed):
        self.state = seed & MASK64

    def next_u64(self):
        self.state = (self.state + 0x9E3779B97F4A7C15) & MASK64
        z = self.state
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK64
        return z ^ (z >> 31)

    def u(self):
        return (self.next_u64() >> 11) * (1.0 / 9007199254740992.0)


def _camera(w, h, fov, frm, to, up=(0, 1, 0)):
    c = rt.Camera(w, h, fov)
    c.set_transform(rt.view_transform(rt.Point(*frm), rt.Point(*to), rt.Vector(*up)))
    return c


def c1(width=200, height=100):
    """C1: Sphere::default() coloured (1, 0.2, 1), light (-10,10,-10)."""
    w = rt.World()
    s = rt.Sphere()
    s.material.color = rt.Color(1.0, 0.2, 1.0)
    w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    return w, _camera(width, height, PI / 3.0, (0, 0, -5), (0, 0, 0)), 5


def c2(width=800, height=600):
    """C2: floor + middle/right/left spheres, Phong only; color_at(ray, 1)."""
    w = rt.World()
    floor = rt.Plane()
    floor.material.color = rt.Color(1.0, 0.9, 0.9)
    floor.material.specular = 0.0
    w.add_object(floor)
    middle = rt.Sphere()
    middle.set_transform(rt.translation(-0.5, 1.0, 0.5))
    middle.material.color = rt.Color(0.1, 1.0, 0.5)
    middle.material.diffuse = 0.7
    middle.material.specular = 0.3
    w.add_object(middle)
    right = rt.Sphere()
    right.set_transform(rt.translation(1.5, 0.5, -0.5) * rt.scaling(0.5, 0.5, 0.5))
    right.material.color = rt.Color(0.5, 1.0, 0.1)
    right.material.diffuse = 0.7
    right.material.specular = 0.3
    w.add_object(right)
    left = rt.Sphere()
    left.set_transform(rt.translation(-1.5, 0.33, -0.75) * rt.scaling(0.33, 0.33, 0.33))
    left.material.color = rt.Color(1.0, 0.8, 0.1)
    left.material.diffuse = 0.7
    left.material.specular = 0.3
    w.add_object(left)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    return w, _camera(width, height, PI / 3.0, (0, 1.5, -5), (0, 1, 0)), 1


def _random_sphere(rng, box_lo, box_hi):
    """One C3/C5 sphere: r, centre, then a material class draw."""
    r = 0.15 + 0.35 * rng.u()
    cx = box_lo[0] + (box_hi[0] - box_lo[0]) * rng.u()
    cy = r + (box_hi[1] - box_lo[1]) * rng.u()
    cz = box_lo[2] + (box_hi[2] - box_lo[2]) * rng.u()
    s = rt.Sphere()
    s.set_transform(rt.translation(cx, cy, cz) * rt.scaling(r, r, r))
    m = s.material
    k = rng.u()
    if k < 0.5:  # diffuse
        m.color = rt.Color(0.1 + 0.9 * rng.u(), 0.1 + 0.9 * rng.u(), 0.1 + 0.9 * rng.u())
        m.ambient = 0.1
        m.diffuse = 0.9
        m.specular = 0.3
        m.shininess = 50.0
    elif k < 0.8:  # mirror
        m.reflective = 0.5 + 0.4 * rng.u()
        m.specular = 0.9
        m.shininess = 200.0
    else:  # glass
        m.color = rt.Color(0.05, 0.05, 0.05)
        m.ambient = 0.0
        m.diffuse = 0.1
        m.specular = 0.9
        m.shininess = 300.0
        m.reflective = 0.9
        m.transparency = 0.9
        m.refractive_index = 1.5
    return s


def c3(width=1920, height=1080, n_spheres=1000, seed=0x5EED0003):
    """C3 (headline): floor plane + n random spheres, 1 light, depth 5."""
    rng = SplitMix64(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.color = rt.Color(0.8, 0.8, 0.8)
    floor.material.specular = 0.0
    floor.material.reflective = 0.2
    w.add_object(floor)
    for _ in range(n_spheres):
        w.add_object(_random_sphere(rng, (-10.0, 0.0, -2.0), (10.0, 3.0, 20.0)))
    w.add_light(rt.PointLight(rt.Point(-10, 20, -10), rt.Color(1.0, 1.0, 1.0)))
    return w, _camera(width, height, PI / 3.0, (0, 3, -12), (0, 1, 5)), 5


def c3_orbit(k, n=64, width=1920, height=1080, arc=0.8):
    """Camera k of n along an arc of `arc` radians around C3's look-at point
    (0, 1, 5), at C3's distance (17) and height: the moving camera of an
    animation over the C3 scene (frame k = 0 .. n-1; the middle one is close to
    C3's own camera)."""
    a = -arc / 2.0 + arc * k / max(n - 1, 1)
    return _camera(width, height, PI / 3.0, (17.0 * math.sin(a), 3.0, 5.0 - 17.0 * math.cos(a)), (0, 1, 5))


def c5(width=4096, height=4096, n_spheres=9996, seed=0x5EED0005):
    """C5: room of 4 planes (reflect-refract.yml:55-104 style) + spheres, 2 lights, depth 8."""
    rng = SplitMix64(seed)
    w = rt.World()
    floor = rt.Plane()
    floor.material.color = rt.Color(0.8, 0.8, 0.8)
    floor.material.specular = 0.0
    floor.material.reflective = 0.2
    w.add_object(floor)
    back = rt.Plane()
    back.set_transform(rt.translation(0, 0, 30) * rt.rotation_x(PI / 2.0))
    back.material.color = rt.Color(0.6, 0.7, 0.9)
    back.material.specular = 0.0
    w.add_object(back)
    for x in (-25.0, 25.0):
        wall = rt.Plane()
        wall.set_transform(rt.translation(x, 0, 0) * rt.rotation_z(PI / 2.0))
        wall.material.color = rt.Color(0.9, 0.8, 0.7)
        wall.material.specular = 0.0
        wall.material.reflective = 0.1
        w.add_object(wall)
    for _ in range(n_spheres):
        w.add_object(_random_sphere(rng, (-25.0, 0.0, -10.0), (25.0, 30.0, 30.0)))
    w.add_light(rt.PointLight(rt.Point(-10, 25, -20), rt.Color(0.8, 0.8, 0.8)))
    w.add_light(rt.PointLight(rt.Point(15, 20, -15), rt.Color(0.4, 0.4, 0.45)))
    return w, _camera(width, height, PI / 3.0, (0, 8, -30), (0, 6, 10)), 8


def zoo(width=160, height=120):
    """Feature coverage: every pattern kind, rotated/sheared shapes, nested
    glass (n1/n2), a shadowless object, two lights, reflection + refraction."""
    w = rt.World()
    floor = rt.Plane()
    floor.material.set_pattern(rt.checkers_pattern(rt.Color(0.0, 0.5, 0.5), rt.Color(0.5, 0.0, 0.5)))
    floor.material.reflective = 0.1
    w.add_object(floor)
    left_wall = rt.Plane()
    left_wall.set_transform(rt.Matrix.identity(4, 4).rotate_x(PI / 2.0).rotate_y(-PI / 4.0).translate(0, 0, 5))
    ring = rt.ring_pattern(rt.Color(0.0, 0.0, 1.0), rt.Color(0.0, 1.0, 1.0))
    ring.set_transform(rt.scaling(0.333, 0.333, 0.333))
    left_wall.material.set_pattern(ring)
    w.add_object(left_wall)
    right_wall = rt.Plane()
    right_wall.set_transform(rt.Matrix.identity(4, 4).rotate_x(PI / 2.0).rotate_y(PI / 4.0).translate(0, 0, 5))
    stripe = rt.stripe_pattern(rt.Color.white(), rt.Color.black())
    stripe.set_transform(rt.rotation_y(0.3) * rt.scaling(0.5, 1.0, 1.0))
    right_wall.material.set_pattern(stripe)
    w.add_object(right_wall)
    middle = rt.Sphere()
    middle.set_transform(rt.translation(-0.5, 1.0, 0.5))
    middle.material.color = rt.Color(0.1, 1.0, 0.5)
    middle.material.diffuse = 0.7
    middle.material.specular = 0.3
    middle.material.reflective = 0.9
    w.add_object(middle)
    right = rt.Sphere()
    right.set_transform(rt.translation(1.5, 0.5, -0.5) * rt.scaling(0.5, 0.5, 0.5))
    right.material.set_pattern(rt.checkers_pattern(rt.Color(1.0, 0.0, 0.0), rt.Color(0.0, 1.0, 0.0)))
    w.add_object(right)
    left = rt.glass_sphere()
    left.material.color = rt.Color(0.1, 0.0, 0.0)
    left.material.diffuse = 0.05
    left.material.reflective = 0.3
    left.material.specular = 1.0
    left.material.shininess = 300.0
    left.set_transform(rt.translation(-1.5, 0.33, -0.75) * rt.scaling(0.33, 0.33, 0.33))
    w.add_object(left)
    # nested glass: outer shell with an inner air bubble and an inner denser core
    outer = rt.glass_sphere()
    outer.set_transform(rt.translation(0.6, 0.6, -1.6) * rt.scaling(0.6, 0.6, 0.6))
    outer.material.reflective = 0.5
    outer.material.color = rt.Color(0.0, 0.0, 0.1)
    outer.material.ambient = 0.0
    w.add_object(outer)
    bubble = rt.glass_sphere()
    bubble.set_transform(rt.translation(0.55, 0.6, -1.6) * rt.scaling(0.3, 0.3, 0.3))
    bubble.material.refractive_index = 1.0000034
    bubble.material.reflective = 0.2
    w.add_object(bubble)
    core = rt.glass_sphere()
    core.set_transform(rt.translation(0.75, 0.55, -1.6) * rt.scaling(0.2, 0.2, 0.2))
    core.material.refractive_index = 2.4
    w.add_object(core)
    # sheared/rotated ellipsoid with a gradient, and a shadowless test-pattern sphere
    ell = rt.Sphere()
    ell.set_transform(rt.translation(-0.3, 0.35, -2.2) * rt.shearing(0.3, 0, 0.2, 0, 0, 0.1)
                      * rt.rotation_z(0.7) * rt.scaling(0.4, 0.2, 0.3))
    grad = rt.gradient_pattern(rt.Color(1.0, 0.2, 0.1), rt.Color(0.1, 0.2, 1.0))
    grad.set_transform(rt.scaling(2.0, 1.0, 1.0) * rt.translation(1.0, 0, 0))
    ell.material.set_pattern(grad)
    w.add_object(ell)
    ghost = rt.Sphere()
    ghost.set_transform(rt.translation(1.2, 1.6, 0.3) * rt.scaling(0.25, 0.25, 0.25))
    ghost.material.set_pattern(rt.test_pattern())
    ghost.no_shadow()
    w.add_object(ghost)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    w.add_light(rt.PointLight(rt.Point(-5.0, 10.0, -6.0), rt.Color(0.33, 0.33, 0.33)))
    return w, _camera(width, height, PI / 3.0, (0.0, 1.5, -5.0), (0, 1, 0)), 5


def first_scene(width=2560, height=1440):
    """The reference demo bin/first_scene.rs:22-109 (checkered floor, ring and
    stripe walls, three spheres, a rotated cube, a closed cylinder and a closed
    cone, two lights), rendered there with render_multithreaded at X1."""
    w = rt.World()
    floor = rt.Plane()
    floor.material.set_pattern(rt.checkers_pattern(rt.Color(0.0, 0.5, 0.5), rt.Color(0.5, 0.0, 0.5)))
    left_wall = rt.Plane()
    left_wall.set_transform(rt.Matrix.identity(4, 4).rotate_x(PI / 2.0).rotate_y(-PI / 4.0).translate(0, 0, 5))
    ring = rt.ring_pattern(rt.Color(0.0, 0.0, 1.0), rt.Color(0.0, 1.0, 1.0))
    ring.set_transform(rt.scaling(0.333, 0.333, 0.333))
    left_wall.material.set_pattern(ring)
    right_wall = rt.Plane()
    right_wall.set_transform(rt.Matrix.identity(4, 4).rotate_x(PI / 2.0).rotate_y(PI / 4.0).translate(0, 0, 5))
    right_wall.material.set_pattern(rt.stripe_pattern(rt.Color.white(), rt.Color.black()))
    middle = rt.Sphere()
    middle.set_transform(rt.translation(-0.5, 1.0, 0.5))
    middle.material.color = rt.Color(0.1, 1.0, 0.5)
    middle.material.diffuse = 0.7
    middle.material.specular = 0.3
    middle.material.reflective = 0.9
    right = rt.Sphere()
    right.set_transform(rt.translation(1.5, 0.5, -0.5) * rt.scaling(0.5, 0.5, 0.5))
    right.material.set_pattern(rt.checkers_pattern(rt.Color(1.0, 0.0, 0.0), rt.Color(0.0, 1.0, 0.0)))
    left = rt.glass_sphere()
    left.material.color = rt.Color(0.1, 0.0, 0.0)
    left.material.ambient = 0.1
    left.material.diffuse = 0.05
    left.material.reflective = 0.3
    left.material.specular = 1.0
    left.material.shininess = 300.0
    left.set_transform(rt.translation(-1.5, 0.33, -0.75) * rt.scaling(0.33, 0.33, 0.33))
    cube = rt.Cube()
    cube.set_transform(rt.Matrix.identity(4, 4).rotate_y(PI / 4.0).scale(0.25, 0.25, 0.25).translate(0.0, 0.25, -1.0))
    cylinder = rt.Cylinder(0.0, 1.0, True)
    cylinder.set_transform(rt.translation(1.0, 0.0, -1.2) * rt.scaling(0.33, 0.33, 0.33))
    cone = rt.Cone(-1.0, 0.0, True)
    cone.set_transform(rt.translation(-1.0, 0.33, -1.2) * rt.scaling(0.33, 0.33, 0.33))
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    w.add_light(rt.PointLight(rt.Point(-5.0, 10.0, -6.0), rt.Color(0.33, 0.33, 0.33)))
    for o in (floor, left_wall, right_wall, middle, right, left, cube, cylinder, cone):
        w.add_object(o)
    return w, _camera(width, height, PI / 3.0, (0.0, 1.5, -5.0), (0, 1, 0)), 5


def solids(width=160, height=120):
    """Cube / Cylinder / Cone coverage: glass solids nested in each other and
    in spheres (containers with up to 4 intersections per object), open,
    closed and unbounded cylinders and cones, rotated and sheared solids,
    mirrors, patterns, a shadowless cone."""
    w = rt.World()
    floor = rt.Plane()
    floor.material.set_pattern(rt.checkers_pattern(rt.Color(0.9, 0.9, 0.9), rt.Color(0.2, 0.2, 0.3)))
    floor.material.reflective = 0.15
    w.add_object(floor)
    back = rt.Plane()
    back.set_transform(rt.translation(0, 0, 8) * rt.rotation_x(PI / 2.0))
    back.material.set_pattern(rt.stripe_pattern(rt.Color(0.8, 0.4, 0.2), rt.Color(0.2, 0.4, 0.8)))
    w.add_object(back)
    # glass cube with a glass cylinder core and an air-bubble sphere
    gcube = rt.Cube()
    gcube.set_transform(rt.translation(-1.2, 1.0, 0.0) * rt.rotation_y(0.5) * rt.rotation_x(0.3)
                        * rt.scaling(0.8, 0.8, 0.8))
    gcube.material.transparency = 0.9
    gcube.material.reflective = 0.6
    gcube.material.refractive_index = 1.5
    gcube.material.color = rt.Color(0.05, 0.1, 0.05)
    gcube.material.diffuse = 0.1
    gcube.material.specular = 1.0
    gcube.material.shininess = 300.0
    w.add_object(gcube)
    core = rt.Cylinder(-0.5, 0.5, True)
    core.set_transform(rt.translation(-1.2, 1.0, 0.0) * rt.rotation_z(0.4) * rt.scaling(0.3, 1.0, 0.3))
    core.material.transparency = 0.8
    core.material.refractive_index = 2.0
    core.material.color = rt.Color(0.2, 0.0, 0.0)
    w.add_object(core)
    bubble = rt.glass_sphere()
    bubble.set_transform(rt.translation(-1.0, 1.3, -0.3) * rt.scaling(0.2, 0.2, 0.2))
    bubble.material.refractive_index = 1.0
    w.add_object(bubble)
    # glass double-napped closed cone, and an open cone inside a glass sphere
    cone = rt.Cone(-1.0, 1.0, True)
    cone.set_transform(rt.translation(1.3, 1.0, 0.3) * rt.scaling(0.5, 1.0, 0.5))
    cone.material.transparency = 0.7
    cone.material.reflective = 0.4
    cone.material.refractive_index = 1.33
    cone.material.color = rt.Color(0.0, 0.05, 0.1)
    w.add_object(cone)
    shell = rt.glass_sphere()
    shell.set_transform(rt.translation(0.1, 0.6, -1.5) * rt.scaling(0.6, 0.6, 0.6))
    shell.material.reflective = 0.5
    w.add_object(shell)
    inner = rt.Cone(-0.5, 0.0, False)
    inner.set_transform(rt.translation(0.1, 0.8, -1.5) * rt.scaling(0.4, 0.8, 0.4))
    inner.material.color = rt.Color(1.0, 0.8, 0.1)
    w.add_object(inner)
    # opaque solids: open cylinder tube, unbounded thin cylinder (pole), sheared cube, mirror cube
    tube = rt.Cylinder(0.0, 0.7, False)
    tube.set_transform(rt.translation(-0.2, 0.0, 1.2) * rt.rotation_y(0.2) * rt.scaling(0.5, 1.0, 0.5))
    tube.material.set_pattern(rt.ring_pattern(rt.Color(1, 1, 1), rt.Color(0.1, 0.6, 0.1)))
    w.add_object(tube)
    pole = rt.Cylinder()
    pole.set_transform(rt.translation(2.4, 0.0, 2.5) * rt.scaling(0.1, 1.0, 0.1))
    pole.material.color = rt.Color(0.6, 0.6, 0.6)
    w.add_object(pole)
    shear = rt.Cube()
    shear.set_transform(rt.translation(0.9, 0.3, -2.3) * rt.shearing(0.4, 0.0, 0.0, 0.2, 0.0, 0.0)
                        * rt.scaling(0.3, 0.3, 0.3))
    shear.material.set_pattern(rt.gradient_pattern(rt.Color(1, 0, 0), rt.Color(0, 0, 1)))
    w.add_object(shear)
    mirror = rt.Cube()
    mirror.set_transform(rt.translation(-2.6, 1.0, 2.0) * rt.rotation_y(-0.6) * rt.scaling(0.05, 1.0, 1.0))
    mirror.material.reflective = 1.0
    mirror.material.color = rt.Color(0.05, 0.05, 0.05)
    w.add_object(mirror)
    ghost = rt.Cone(0.0, 0.6, True)
    ghost.set_transform(rt.translation(-0.5, 0.0, -2.5) * rt.scaling(0.3, 0.5, 0.3))
    ghost.material.set_pattern(rt.test_pattern())
    ghost.no_shadow()
    w.add_object(ghost)
    w.add_light(rt.PointLight(rt.Point(-6, 8, -8), rt.Color(1.0, 1.0, 1.0)))
    w.add_light(rt.PointLight(rt.Point(5.0, 6.0, -4.0), rt.Color(0.3, 0.3, 0.3)))
    return w, _camera(width, height, PI / 3.0, (0.0, 2.0, -5.5), (0, 0.8, 0)), 6


def _hexagon_side():
    """bin/hexagon.rs:45-69: a corner sphere and an edge cylinder in a group."""
    corner = rt.Sphere()
    corner.set_transform(rt.translation(0, 0, -1) * rt.scaling(0.25, 0.25, 0.25))
    edge = rt.Cylinder(0.0, 1.0, False)
    edge.set_transform(rt.Matrix.identity(4, 4).scale(0.25, 1.0, 0.25).rotate_z(-PI / 2.0).rotate_y(-PI / 6.0)
                       .translate(0, 0, -1))
    side = rt.Group()
    side.add_child(corner)
    side.add_child(edge)
    return side


def hexagon(width=2560, height=1440):
    """The reference demo bin/hexagon.rs:23-87: six groups (a sphere and an open
    cylinder each) rotated about y inside a hexagon group, a checkers material
    set on the whole hierarchy, the hexagon scaled by 1.5; two lights;
    Camera::render (depth 5)."""
    hexa = rt.Group()
    for n in range(6):
        side = _hexagon_side()
        side.set_transform(rt.rotation_y(n * PI / 3.0))
        hexa.add_child(side)
    m = rt.Material()
    m.set_pattern(rt.checkers_pattern(rt.Color(1.0, 0.0, 0.0), rt.Color(0.0, 1.0, 0.0)))
    hexa.set_material(m)
    hexa.set_transform(rt.scaling(1.5, 1.5, 1.5))
    w = rt.World()
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    w.add_light(rt.PointLight(rt.Point(-5.0, 10.0, -6.0), rt.Color(0.33, 0.33, 0.33)))
    w.add_object(hexa)
    return w, _camera(width, height, PI / 3.0, (0.0, 2.5, -5.0), (0, 0, 0)), 5


def groups(width=160, height=120):
    """Group coverage (group.rs, bounding_box.rs): nested groups with their own
    transforms, set_material on an inner group, a glass sphere and a glass cube
    in a group (containers across group members), a cone and a cube in a
    rotated group, a group holding a plane (a plane's box turns NaN under
    set_transform, so the group's box is its other child's and the plane is
    seen only through that box: the reference's own quirk), shapes added after
    set_transform and set_material, and ungrouped shapes beside them."""
    w = rt.World()
    floor = rt.Plane()
    floor.material.set_pattern(rt.checkers_pattern(rt.Color(0.8, 0.8, 0.8), rt.Color(0.3, 0.3, 0.4)))
    floor.material.reflective = 0.2
    w.add_object(floor)
    # outer (translated) > inner (rotated, reflective material) > glass sphere + glass cube
    inner = rt.Group()
    gs = rt.glass_sphere()
    gs.set_transform(rt.translation(0.0, 1.0, 0.0) * rt.scaling(0.7, 0.7, 0.7))
    inner.add_child(gs)
    gc = rt.Cube()
    gc.set_transform(rt.translation(0.6, 0.9, -0.4) * rt.scaling(0.35, 0.35, 0.35))
    gc.material.transparency = 0.9
    gc.material.refractive_index = 1.3
    inner.add_child(gc)
    inner.set_transform(rt.rotation_y(0.4))
    glass = rt.Material()
    glass.transparency = 0.8
    glass.reflective = 0.7
    glass.refractive_index = 1.45
    glass.color = rt.Color(0.05, 0.1, 0.1)
    glass.diffuse = 0.2
    glass.specular = 0.9
    glass.shininess = 200.0
    inner.set_material(glass)  # both members, recursively (group.rs:96-102)
    outer = rt.Group()
    outer.add_child(inner)
    cyl = rt.Cylinder(0.0, 1.5, True)
    cyl.set_transform(rt.translation(-1.6, 0.0, 0.5) * rt.scaling(0.3, 1.0, 0.3))
    cyl.material.color = rt.Color(0.9, 0.5, 0.1)
    outer.add_child(cyl)
    outer.set_transform(rt.translation(-0.8, 0.0, 0.6))  # (after its children: baked into them)
    w.add_object(outer)
    # a rotated group: cone + cube, material set on the group, then one more child
    rot = rt.Group()
    cone = rt.Cone(-1.0, 0.0, True)
    cone.set_transform(rt.translation(0.0, 1.0, 0.0) * rt.scaling(0.4, 1.0, 0.4))
    rot.add_child(cone)
    cube = rt.Cube()
    cube.set_transform(rt.translation(0.6, 0.3, 0.0) * rt.scaling(0.3, 0.3, 0.3))
    rot.add_child(cube)
    rot.set_transform(rt.translation(1.6, 0.0, -0.2) * rt.rotation_y(-0.7) * rt.rotation_z(0.2))
    mm = rt.Material()
    mm.set_pattern(rt.stripe_pattern(rt.Color(1.0, 0.9, 0.2), rt.Color(0.2, 0.4, 1.0)))
    mm.reflective = 0.3
    rot.set_material(mm)
    late = rt.Sphere()
    late.set_transform(rt.translation(0.0, 2.2, 0.0) * rt.scaling(0.3, 0.3, 0.3))
    late.material.color = rt.Color(0.9, 0.1, 0.1)
    rot.add_child(late)
    w.add_object(rot)
    # a group with a plane and a small sphere: the plane shows only inside the sphere's box
    pg = rt.Group()
    wall = rt.Plane()
    wall.set_transform(rt.translation(0.0, 0.0, 4.0) * rt.rotation_x(PI / 2.0))
    wall.material.color = rt.Color(0.2, 0.8, 0.3)
    pg.add_child(wall)
    ball = rt.Sphere()
    ball.set_transform(rt.translation(0.3, 1.6, 3.0) * rt.scaling(0.8, 0.8, 0.8))
    ball.material.reflective = 0.5
    pg.add_child(ball)
    w.add_object(pg)
    free = rt.Sphere()
    free.set_transform(rt.translation(0.2, 0.35, -1.6) * rt.scaling(0.35, 0.35, 0.35))
    free.material.color = rt.Color(0.2, 0.3, 0.9)
    free.material.reflective = 0.4
    w.add_object(free)
    w.add_light(rt.PointLight(rt.Point(-6, 8, -8), rt.Color(1.0, 1.0, 1.0)))
    w.add_light(rt.PointLight(rt.Point(4.0, 5.0, -5.0), rt.Color(0.35, 0.35, 0.35)))
    return w, _camera(width, height, PI / 3.0, (0.0, 2.2, -5.5), (0, 0.9, 0)), 6


def divided(width=128, height=72, n=5, threshold=2, seed=11):
    """Group::divide (group.rs:108-197, bounding_box.rs:138-169): an n x n x 2
    lattice of small spheres, cubes and cylinders (shuffled, random materials,
    some glass) in one group, divided with `threshold` into nested subgroups,
    then translated (the translation is baked into every level); a floor
    outside the group."""
    import random
    rnd = random.Random(seed)
    g = rt.Group()
    cells = [(i, j, k) for i in range(n) for j in range(n) for k in range(2)]
    rnd.shuffle(cells)
    for idx, (i, j, k) in enumerate(cells):
        s = (rt.Sphere, rt.Cube, lambda: rt.Cylinder(-1.0, 1.0, True))[idx % 3]()
        r = 0.22 + 0.1 * rnd.random()
        s.set_transform(rt.translation(i - (n - 1) / 2.0, 0.4 + 0.9 * k, j * 0.9) * rt.scaling(r, r, r))
        s.material.color = rt.Color(rnd.random(), rnd.random(), rnd.random())
        s.material.reflective = 0.3 * rnd.random()
        if idx % 7 == 3:
            s.material.transparency = 0.8
            s.material.refractive_index = 1.4
        g.add_child(s)
    g.divide(threshold)
    g.set_transform(rt.translation(0.0, 0.0, 0.5))
    w = rt.World()
    floor = rt.Plane()
    floor.material.set_pattern(rt.checkers_pattern(rt.Color(0.9, 0.9, 0.9), rt.Color(0.2, 0.2, 0.25)))
    w.add_object(floor)
    w.add_object(g)
    w.add_light(rt.PointLight(rt.Point(-6, 8, -8), rt.Color(1.0, 1.0, 1.0)))
    return w, _camera(width, height, PI / 3.0, (0.0, 3.5, -5.5), (0.0, 0.6, 1.5)), 5


def cones(width=320, height=240, n=600, upright=0.5, seed=23):
    """A field of cones (closed and open, finite bounds, some spanning both
    nappes) and open tubes, `upright` of the cones upright with one scale, the
    rest rotated and sheared; glass and mirrors among them, diagonal spheres, a
    reflective floor. The line hierarchy's workload (rt_bvh.cpp build_line_bvh;
    cone.rs, cylinder.rs)."""
    import random
    rnd = random.Random(seed)
    u = lambda a, b: a + (b - a) * rnd.random()  # noqa: E731
    w = rt.World()
    floor = rt.Plane()
    floor.material.reflective = 0.3
    w.add_object(floor)
    for i in range(n):
        c = (u(-8, 8), u(0.5, 3.0), u(-6, 10))
        if i % 4 == 3:
            s = rt.Cylinder(u(-1.0, 0.0), u(0.2, 1.0), False)
            tf = rt.translation(*c) * rt.rotation_z(u(-1, 1)) * rt.scaling(0.3, 0.5, 0.3)
        elif i % 8 == 6:
            s = rt.Sphere()
            tf = rt.translation(*c) * rt.scaling(0.3, 0.3, 0.3)
        else:
            lo = u(-1.0, 0.3)
            s = rt.Cone(lo, lo + u(0.3, 1.2), bool(i % 3))
            if rnd.random() < upright:
                tf = rt.translation(*c) * rt.scaling(0.4, 0.4, 0.4)
            else:
                tf = (rt.translation(*c) * rt.rotation_y(u(0, 6.3)) * rt.rotation_x(u(0, 6.3))
                      * rt.shearing(*[u(-0.2, 0.2) for _ in range(6)]) * rt.scaling(0.4, 0.5, 0.3))
        s.set_transform(tf)
        s.material.color = rt.Color(rnd.random(), rnd.random(), rnd.random())
        if i % 5 == 1:
            s.material.transparency = 0.8
            s.material.refractive_index = u(1.0, 2.0)
            s.material.reflective = 0.4
        elif i % 5 == 2:
            s.material.reflective = u(0.2, 0.9)
        w.add_object(s)
    w.add_light(rt.PointLight(rt.Point(-10, 10, -10), rt.Color(1.0, 1.0, 1.0)))
    return w, _camera(width, height, PI / 3.0, (0.0, 3.0, -12.0), (0.0, 1.0, 2.0)), 5


CONFIGS = {"c1": c1, "c2": c2, "c3": c3, "c5": c5, "zoo": zoo, "first_scene": first_scene, "solids": solids,
           "hexagon": hexagon, "groups": groups, "divided": divided, "cones": cones}


def fuzz(seed, width=64, height=48, n_spheres=None):
    """A seeded random scene for parity sweeps (tests/test_gpu_fuzz.py): one to
    three planes (one may be patterned, reflective, rotated), a cluster of
    random spheres (non-uniform scales, rotations, some shears; diffuse,
    mirror, glass with refractive indices 1.0-2.4, some nested), cubes,
    cylinders and cones (open or closed, random bounds), sometimes a group
    (transformed after its children, divided or not), patterns of every kind
    with their own transforms, shadowless objects, one to three lights, a
    random camera looking into the cluster and a depth of 1 to 6. Everything
    the fast path culls (the sphere hierarchy, the other records' and the
    lines' hierarchies, group gates, the light buffer) meets geometry it has
    not been tuned on. `n_spheres`: that many random spheres instead of 10-119
    (thousands: the scene images in global memory instead of LDS)."""
    import random
    rnd = random.Random(seed)
    u = rnd.uniform
    w = rt.World()

    def pattern():
        c1 = rt.Color(u(0, 1), u(0, 1), u(0, 1))
        c2 = rt.Color(u(0, 1), u(0, 1), u(0, 1))
        k = rnd.randrange(5)
        p = (rt.stripe_pattern, rt.gradient_pattern, rt.ring_pattern, rt.checkers_pattern)[k](c1, c2) \
            if k < 4 else rt.test_pattern()
        if rnd.random() < 0.6:
            p.set_transform(rt.rotation_y(u(-PI, PI)) * rt.scaling(u(0.2, 2.0), u(0.2, 2.0), u(0.2, 2.0)))
        return p

    def material(m, glass_p=0.25):
        r = rnd.random()
        if r < glass_p:
            m.color = rt.Color(u(0, 0.2), u(0, 0.2), u(0, 0.2))
            m.diffuse = u(0.0, 0.3)
            m.ambient = rnd.choice([0.0, 0.1])
            m.specular = u(0.5, 1.0)
            m.shininess = rnd.choice([50.0, 200.0, 300.0])
            m.reflective = u(0.0, 0.95)
            m.transparency = u(0.5, 1.0)
            m.refractive_index = rnd.choice([1.0, 1.00029, 1.333, 1.5, 1.52, 2.417])
        elif r < glass_p + 0.3:
            m.reflective = u(0.1, 1.0)
            m.specular = u(0.0, 1.0)
            m.shininess = rnd.choice([10.0, 200.0])
        else:
            if rnd.random() < 0.35:
                m.set_pattern(pattern())
            else:
                m.color = rt.Color(u(0, 1), u(0, 1), u(0, 1))
            m.ambient = u(0.0, 0.3)
            m.diffuse = u(0.3, 1.0)
            m.specular = u(0.0, 1.0)
            m.shininess = rnd.choice([1.0, 10.0, 50.0, 200.0])

    def placed(shape, scale=(0.15, 0.9), shear=0.2):
        sx, sy, sz = (u(*scale) for _ in range(3))
        if rnd.random() < 0.5:
            sy = sz = sx  # a uniform scale (the diagonal sphere records)
        m = rt.translation(u(-4, 4), u(0.0, 3.0), u(-2, 6))
        if rnd.random() < 0.4:
            m = m * rt.rotation_x(u(-PI, PI)) * rt.rotation_y(u(-PI, PI)) * rt.rotation_z(u(-PI, PI))
        if rnd.random() < shear:
            m = m * rt.shearing(u(-0.4, 0.4), 0, 0, u(-0.4, 0.4), 0, u(-0.4, 0.4))
        shape.set_transform(m * rt.scaling(sx, sy, sz))
        return shape

    floor = rt.Plane()
    material(floor.material, glass_p=0.0)
    floor.material.reflective = rnd.choice([0.0, 0.2, 0.5])
    w.add_object(floor)
    for _ in range(rnd.randrange(0, 3)):
        wall = rt.Plane()
        wall.set_transform(rt.rotation_y(u(-PI, PI)) * rt.translation(0, 0, u(6, 12)) * rt.rotation_x(PI / 2.0))
        material(wall.material, glass_p=0.05)
        w.add_object(wall)
    n_sph = rnd.randrange(10, 120)
    for _ in range(n_sph if n_spheres is None else n_spheres):
        s = placed(rt.Sphere())
        material(s.material)
        if rnd.random() < 0.05:
            s.no_shadow()
        w.add_object(s)
    for _ in range(rnd.randrange(0, 3)):  # nested glass: a shell with a core of another index inside
        shell = rt.glass_sphere()
        m = rt.translation(u(-3, 3), u(0.5, 2.5), u(-1, 5)) * rt.scaling(u(0.5, 1.2), u(0.5, 1.2), u(0.5, 1.2))
        shell.set_transform(m)
        shell.material.refractive_index = rnd.choice([1.0000034, 1.5, 2.4])
        w.add_object(shell)
        core = rt.glass_sphere()
        core.set_transform(m * rt.translation(u(-0.3, 0.3), 0.0, 0.0) * rt.scaling(0.4, 0.4, 0.4))
        core.material.refractive_index = rnd.choice([1.0, 1.33, 2.4])
        w.add_object(core)
    others = []
    for _ in range(rnd.randrange(0, 14)):
        k = rnd.randrange(3)
        if k == 0:
            o = rt.Cube()
        else:
            lo = rnd.choice([-math.inf, u(-2.0, 0.0)])
            hi = rnd.choice([math.inf, u(0.1, 2.0)])
            closed = rnd.random() < 0.5 and math.isfinite(lo) and math.isfinite(hi)
            o = rt.Cylinder(lo, hi, closed) if k == 1 else rt.Cone(lo, hi, closed)
            if not (math.isfinite(lo) and math.isfinite(hi)):
                o = rt.Cylinder(-1.0, 1.0, rnd.random() < 0.5) if k == 1 else rt.Cone(-1.0, 0.0, rnd.random() < 0.5)
        placed(o, scale=(0.1, 0.6))
        material(o.material)
        others.append(o)
    if others and rnd.random() < 0.5:  # some of them in a group, transformed after its children, maybe divided
        g = rt.Group()
        for o in others[: len(others) // 2 + 1]:
            g.add_child(o)
        if rnd.random() < 0.5:
            g.divide(rnd.choice([1, 2, 3]))
        g.set_transform(rt.translation(u(-1, 1), 0.0, u(-1, 1)) * rt.rotation_y(u(-0.5, 0.5)))
        w.add_object(g)
        others = others[len(others) // 2 + 1:]
    for o in others:
        w.add_object(o)
    for _ in range(rnd.randrange(1, 4)):
        w.add_light(rt.PointLight(rt.Point(u(-12, 12), u(3, 15), u(-12, 4)),
                                  rt.Color(u(0.2, 1.0), u(0.2, 1.0), u(0.2, 1.0))))
    frm = (u(-6, 6), u(0.5, 5), u(-10, -4))
    to = (u(-1, 1), u(0.3, 1.5), u(0, 3))
    return w, _camera(width, height, u(0.6, 1.6), frm, to), rnd.randrange(1, 7)
