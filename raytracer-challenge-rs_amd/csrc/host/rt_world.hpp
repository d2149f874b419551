// rt_world.hpp — C++ host mirror of the reference's scene API, driving the
// C-ABI (include/rt_render.h). Same names and argument meaning as
// raytracer/src/{material,light,pattern/mod,geometry/mod,world,camera,canvas}.rs,
// so a caller of `Camera::render(&World) -> Canvas` switches by changing the
// namespace. Rendering, `color_at`, `is_shadowed` and the per-hit
// `prepare_computations` all run on the GPU through the ABI; this header only
// builds and flattens the scene (host-side, like the reference's setup code).
#pragma once
#include <sys/mman.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <limits>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../../../include/rt_render.h"
#include "rt_math.hpp"

namespace rt {

struct RtError : std::runtime_error {
  int code;
  RtError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};
inline void check(int rc, const char* what) {
  if (rc != RT_OK) throw RtError(rc, std::string(what) + ": " + rt_last_error());
}

// pattern/mod.rs:17-91
struct Pattern {
  int kind = RT_PATTERN_TEST;
  Color a, b;
  Matrix transform = Matrix::identity(4, 4);
  Matrix transform_inverse = Matrix::identity(4, 4);
  void set_transform(const Matrix& t) {  // pattern/mod.rs:34-37
    transform = t;
    transform_inverse = t.inverse();
  }
};
inline Pattern test_pattern() { return Pattern{}; }
inline Pattern make_pattern(int kind, const Color& a, const Color& b) {
  Pattern p;
  p.kind = kind;
  p.a = a;
  p.b = b;
  return p;
}
inline Pattern stripe_pattern(const Color& a, const Color& b) { return make_pattern(RT_PATTERN_STRIPE, a, b); }
inline Pattern gradient_pattern(const Color& a, const Color& b) { return make_pattern(RT_PATTERN_GRADIENT, a, b); }
inline Pattern ring_pattern(const Color& a, const Color& b) { return make_pattern(RT_PATTERN_RING, a, b); }
inline Pattern checkers_pattern(const Color& a, const Color& b) { return make_pattern(RT_PATTERN_CHECKERS, a, b); }

// material.rs:10-36
struct Material {
  Color color{1.0, 1.0, 1.0};
  double ambient = 0.1, diffuse = 0.9, specular = 0.9, shininess = 200.0;
  double reflective = 0.0, transparency = 0.0, refractive_index = 1.0;
  bool has_pattern = false;
  Pattern pattern;
  void set_pattern(const Pattern& p) {
    pattern = p;
    has_pattern = true;
  }
};

// light.rs:4-24
struct PointLight {
  Point position;
  Color intensity;
  PointLight() = default;
  PointLight(const Point& p, const Color& i) : position(p), intensity(i) {}
};

// bounding_box.rs:5-93: what a Group's box is made of (Group::intersect tests
// it, group.rs:49-58). Every shape carries one, re-derived by set_transform
// (geometry/mod.rs:74-85) through the same corner products as the reference,
// infinite corners (planes, open cylinders) and their NaNs included.
struct BoundingBox {
  Point min = Point(kInf, kInf, kInf), max = Point(-kInf, -kInf, -kInf);
  static constexpr double kInf = std::numeric_limits<double>::infinity();
  BoundingBox() = default;
  BoundingBox(const Point& mn, const Point& mx) : min(mn), max(mx) {}
  void add_point(const Point& p) {  // :39-59
    if (p.x > max.x) max.x = p.x;
    if (p.y > max.y) max.y = p.y;
    if (p.z > max.z) max.z = p.z;
    if (p.x < min.x) min.x = p.x;
    if (p.y < min.y) min.y = p.y;
    if (p.z < min.z) min.z = p.z;
  }
  void add_box(const BoundingBox& b) { add_point(b.min); add_point(b.max); }  // :61-64
  bool contains_point(const Point& p) const {  // :66-70 (RangeInclusive::contains: NaN is outside)
    return min.x <= p.x && p.x <= max.x && min.y <= p.y && p.y <= max.y && min.z <= p.z && p.z <= max.z;
  }
  bool contains_box(const BoundingBox& b) const { return contains_point(b.min) && contains_point(b.max); }  // :72-74
  BoundingBox transform(const Matrix& m) const {  // :76-93
    const Point pts[8] = {min, Point(min.x, min.y, max.z), Point(min.x, max.y, min.z), Point(min.x, max.y, max.z),
                          Point(max.x, min.y, min.z), Point(max.x, min.y, max.z), Point(max.x, max.y, min.z), max};
    BoundingBox nb;
    for (const Point& p : pts) nb.add_point(m * p);
    return nb;
  }
  // :95-136, the same slab test as the device gate (rt_device.hpp bbox_intersects)
  static void check_axis(double origin, double direction, double mn, double mx, double& t0, double& t1) {
    const double n0 = mn - origin, n1 = mx - origin;
    if (std::fabs(direction) >= EPSILON) {
      t0 = n0 / direction;
      t1 = n1 / direction;
    } else {
      t0 = n0 * kInf;
      t1 = n1 * kInf;
    }
    if (t0 > t1) std::swap(t0, t1);
  }
  bool intersects(const Ray& r) const {
    double x0, x1, y0, y1, z0, z1;
    check_axis(r.origin.x, r.direction.x, min.x, max.x, x0, x1);
    check_axis(r.origin.y, r.direction.y, min.y, max.y, y0, y1);
    check_axis(r.origin.z, r.direction.z, min.z, max.z, z0, z1);
    const double tmin = std::fmax(std::fmax(x0, y0), z0);  // f64::max / f64::min ignore a NaN operand
    const double tmax = std::fmin(std::fmin(x1, y1), z1);
    return tmin <= tmax;
  }
  // :138-169: halves along the widest axis (ties to x, then y, through `equal`)
  std::pair<BoundingBox, BoundingBox> split() const {
    const double dx = std::fabs(max.x - min.x), dy = std::fabs(max.y - min.y), dz = std::fabs(max.z - min.z);
    const double greatest = std::fmax(std::fmax(dx, dy), dz);
    double x0 = min.x, y0 = min.y, z0 = min.z, x1 = max.x, y1 = max.y, z1 = max.z;
    if (equal(greatest, dx)) {
      x0 = x1 = x0 + dx / 2.0;
    } else if (equal(greatest, dy)) {
      y0 = y1 = y0 + dy / 2.0;
    } else {
      z0 = z1 = z0 + dz / 2.0;
    }
    return {BoundingBox(min, Point(x1, y1, z1)), BoundingBox(Point(x0, y0, z0), max)};
  }
};

// geometry/mod.rs:12-108 (BaseShape + the parts of `trait Shape` on the path)
struct Shape {
  int kind = RT_SHAPE_SPHERE;
  Matrix transform = Matrix::identity(4, 4);
  Matrix transform_inverse = Matrix::identity(4, 4);
  Material material;
  bool shadow = true;
  // Cylinder / Cone bounds (cylinder.rs:12-18, cone.rs:12-18)
  double minimum = -std::numeric_limits<double>::infinity();
  double maximum = std::numeric_limits<double>::infinity();
  bool closed = false;
  BoundingBox bbox = BoundingBox(Point(-1, -1, -1), Point(1, 1, 1));  // sphere.rs:20 / cube.rs:22
  void set_transform(const Matrix& t) {  // geometry/mod.rs:74-85
    bbox = bbox.transform(transform_inverse);
    const Matrix inv = t.inverse();
    transform_inverse = inv;
    transform = t;
    bbox = bbox.transform(transform);
  }
  void set_material(const Material& m) { material = m; }  // geometry/mod.rs:66-68
  BoundingBox parent_space_bounds() const { return bbox.transform(Matrix::identity(4, 4)); }  // :97-99
  void no_shadow() { shadow = false; }            // :105-107
  bool has_shadow() const { return shadow; }      // :101-103
  Matrix transform_inverse_transpose() const { return transform_inverse.transpose(); }
};
// sphere.rs:16-25, :70-77
inline Shape Sphere() { return Shape{}; }
inline Shape glass_sphere() {
  Shape s;
  s.material.transparency = 1.0;
  s.material.refractive_index = 1.5;
  return s;
}
inline Shape Plane() {  // plane.rs:19-31
  Shape s;
  s.kind = RT_SHAPE_PLANE;
  s.bbox = BoundingBox(Point(-BoundingBox::kInf, 0.0, -BoundingBox::kInf), Point(BoundingBox::kInf, 0.0, BoundingBox::kInf));
  return s;
}
inline Shape Cube() {  // cube.rs:17-26
  Shape s;
  s.kind = RT_SHAPE_CUBE;
  return s;
}
// cylinder.rs:20-40 (Cylinder::default = new(-inf, inf, false))
inline Shape Cylinder(double minimum = -std::numeric_limits<double>::infinity(),
                      double maximum = std::numeric_limits<double>::infinity(), bool closed = false) {
  Shape s;
  s.kind = RT_SHAPE_CYLINDER;
  s.minimum = minimum; s.maximum = maximum; s.closed = closed;
  s.bbox = BoundingBox(Point(-1.0, minimum, -1.0), Point(1.0, maximum, 1.0));  // cylinder.rs:30-33
  return s;
}
// cone.rs:20-46
inline Shape Cone(double minimum = -std::numeric_limits<double>::infinity(),
                  double maximum = std::numeric_limits<double>::infinity(), bool closed = false) {
  Shape s = Cylinder(minimum, maximum, closed);
  s.kind = RT_SHAPE_CONE;
  const double a = std::fabs(minimum), b = std::fabs(maximum), limit = std::fmax(a, b);  // f64::max (cone.rs:29-31)
  s.bbox = BoundingBox(Point(-limit, minimum, -limit), Point(limit, maximum, limit));
  return s;
}

// geometry/shape/group.rs:13-198: a Group holds shapes and groups in order. Its
// transform is baked into every descendant (set_transform / add_child call the
// children's set_transform with the product, group.rs:71-94,128-133), so a
// child's transform is final; its box is the union of its children's boxes.
struct Group;
struct GroupChild {  // Box<dyn Shape> of a Group: a primitive or a group
  std::shared_ptr<Shape> shape;
  std::shared_ptr<Group> group;
};
struct Group {
  Matrix transform = Matrix::identity(4, 4);
  Matrix transform_inverse = Matrix::identity(4, 4);
  Material material;
  BoundingBox bbox;  // BaseShape::default: empty
  std::vector<GroupChild> children;
  // A Group owns its children (Vec<Box<dyn Shape>>): copies are deep, so a copy
  // added to another group (add_child takes its own) or handed out (child(i))
  // never shares a shape with the original
  Group() = default;
  Group(const Group& o)
      : transform(o.transform), transform_inverse(o.transform_inverse), material(o.material), bbox(o.bbox) {
    children.reserve(o.children.size());
    for (const GroupChild& c : o.children)
      children.push_back(c.shape ? GroupChild{std::make_shared<Shape>(*c.shape), nullptr}
                                 : GroupChild{nullptr, std::make_shared<Group>(*c.group)});
  }
  Group& operator=(const Group& o) {
    if (this != &o) {
      Group t(o);
      *this = std::move(t);
    }
    return *this;
  }
  Group(Group&&) = default;
  Group& operator=(Group&&) = default;
  void set_transform(const Matrix& t);                          // group.rs:71-94
  void set_material(const Material& m);                         // group.rs:96-102
  void add_child(const Shape& s) { add(GroupChild{std::make_shared<Shape>(s), nullptr}); }  // group.rs:128-133
  void add_child(const Group& g) { add(GroupChild{nullptr, std::make_shared<Group>(g)}); }
  BoundingBox parent_space_bounds() const { return bbox.transform(Matrix::identity(4, 4)); }
  // group.rs:108-122: children whose parent-space box fits one half of this box
  // move into a new subgroup per half (partition_children :135-189,
  // make_subgroup :191-197; the subgroup is pushed without widening this box),
  // then every child group divides in turn
  void divide(size_t threshold);

 private:
  void add(GroupChild c);
};
inline const Matrix& child_transform(const GroupChild& c) { return c.shape ? c.shape->transform : c.group->transform; }
inline const BoundingBox& child_bounds(const GroupChild& c) { return c.shape ? c.shape->bbox : c.group->bbox; }
inline void child_set_transform(GroupChild& c, const Matrix& t) {
  if (c.shape) c.shape->set_transform(t);
  else c.group->set_transform(t);
}
inline void Group::set_transform(const Matrix& t) {
  const Matrix inverse_old = transform_inverse;  // remove the current transform from the children
  for (GroupChild& c : children) child_set_transform(c, inverse_old * child_transform(c));
  const Matrix inv = t.inverse();
  transform = t;
  transform_inverse = inv;
  BoundingBox nb;
  for (GroupChild& c : children) {  // apply the new one
    child_set_transform(c, transform * child_transform(c));
    nb.add_box(child_bounds(c));
  }
  bbox = nb;
}
inline void Group::set_material(const Material& m) {
  material = m;
  for (GroupChild& c : children) {
    if (c.shape) c.shape->set_material(m);
    else c.group->set_material(m);
  }
}
inline void Group::add(GroupChild c) {
  child_set_transform(c, transform * child_transform(c));
  const BoundingBox cbox = c.shape ? c.shape->parent_space_bounds() : c.group->parent_space_bounds();
  bbox.add_box(cbox);
  children.push_back(std::move(c));
}
inline void Group::divide(size_t threshold) {
  if (threshold <= children.size()) {
    const std::pair<BoundingBox, BoundingBox> halves = bbox.split();
    std::vector<GroupChild> part[2];
    for (int h = 0; h < 2; ++h) {
      const BoundingBox& hb = h ? halves.second : halves.first;
      std::vector<GroupChild> keep;
      for (GroupChild& c : children) {
        const BoundingBox cb = c.shape ? c.shape->parent_space_bounds() : c.group->parent_space_bounds();
        (hb.contains_box(cb) ? part[h] : keep).push_back(std::move(c));
      }
      children = std::move(keep);
    }
    for (int h = 0; h < 2; ++h) {
      if (part[h].empty()) continue;
      auto g = std::make_shared<Group>();
      for (GroupChild& c : part[h]) g->add(std::move(c));
      children.push_back(GroupChild{nullptr, std::move(g)});
    }
  }
  for (GroupChild& c : children)
    if (c.group) c.group->divide(threshold);
}

// canvas.rs:8-52 + image/ppm.rs
// Pixel storage of a Canvas. Frames of 2 MiB and more sit on 2-MiB aligned
// memory marked for transparent huge pages, so the first touch of a fresh
// 50-MB canvas (the device-to-host copy of `render`) takes tens of page
// faults instead of ~12 000.
// A render's output canvas (Uninit) of 4 MiB and more takes a pinned block
// from the library's pool (rt_host_buffer_alloc), which the device writes
// directly at the link rate; blocks return to the pool with the canvas.
struct PixelFree {
  bool pinned = false;
  void operator()(double* p) const noexcept {
    if (pinned) rt_host_buffer_free(p);
    else std::free(p);
  }
};
using PixelPtr = std::unique_ptr<double[], PixelFree>;
inline PixelPtr alloc_pixels(size_t n, bool pinned = false) {
  const size_t bytes = std::max<size_t>(n, 1) * sizeof(double);
  constexpr size_t kHuge = (size_t)2 << 20;
  void* p = nullptr;
  if (pinned && bytes >= 2 * kHuge) {
    if (void* q = rt_host_buffer_alloc(bytes)) return PixelPtr((double*)q, PixelFree{true});
  }
  if (bytes >= kHuge) {
    if (posix_memalign(&p, kHuge, (bytes + kHuge - 1) / kHuge * kHuge) != 0) p = nullptr;
    if (p) (void)madvise(p, (bytes + kHuge - 1) / kHuge * kHuge, MADV_HUGEPAGE);
  } else {
    p = std::malloc(bytes);
  }
  if (!p) throw std::bad_alloc();
  return PixelPtr((double*)p);
}

class Canvas {
 public:
  Canvas(size_t w, size_t h) : w_(w), h_(h), px_(alloc_pixels(w * h * 3)) {  // black (raytracer/src/canvas.rs:16)
    std::memset(px_.get(), 0, w * h * 3 * sizeof(double));
  }
  // Storage the caller overwrites entirely (a render writes every pixel): no
  // zero pass, so the pages are first touched by the copy from the device.
  struct Uninit {};
  Canvas(size_t w, size_t h, Uninit) : w_(w), h_(h), px_(alloc_pixels(w * h * 3, true)) {}
  Canvas(const Canvas& o) : w_(o.w_), h_(o.h_), px_(alloc_pixels(o.w_ * o.h_ * 3)) {
    std::memcpy(px_.get(), o.px_.get(), w_ * h_ * 3 * sizeof(double));
  }
  Canvas(Canvas&&) noexcept = default;
  Canvas& operator=(Canvas o) noexcept {
    w_ = o.w_; h_ = o.h_; px_.swap(o.px_);
    return *this;
  }
  size_t width() const { return w_; }
  size_t height() const { return h_; }
  Color get_pixel(size_t x, size_t y) const {
    const double* p = &px_[idx(x, y)];
    return Color(p[0], p[1], p[2]);
  }
  void set_pixel(size_t x, size_t y, const Color& c) {
    double* p = &px_[idx(x, y)];
    p[0] = c.red; p[1] = c.green; p[2] = c.blue;
  }
  double* data() { return px_.get(); }
  const double* data() const { return px_.get(); }
  std::string to_ppm() const {  // canvas_to_ppm (image/ppm.rs:24-51)
    size_t len = 0;  // one pass into the bound (12 bytes per pixel, a newline per row, the header)
    std::string s((size_t)12 * w_ * h_ + h_ + 32, '\0');
    check(rt_canvas_to_ppm(px_.get(), (uint32_t)w_, (uint32_t)h_, &s[0], s.size(), &len), "rt_canvas_to_ppm");
    s.resize(len);
    return s;
  }

 private:
  size_t idx(size_t x, size_t y) const {  // canvas.rs:44-48 (asserts -> exceptions)
    if (x >= w_ || y >= h_) throw std::out_of_range("Canvas: pixel out of bounds");
    return (y * w_ + x) * 3;
  }
  size_t w_, h_;
  PixelPtr px_;
};

inline rt_shape_desc to_desc(const Shape& s) {
  rt_shape_desc d;
  std::memset(&d, 0, sizeof d);
  d.kind = s.kind;
  d.casts_shadow = s.shadow ? 1 : 0;
  std::memcpy(d.transform, s.transform.data(), sizeof d.transform);
  std::memcpy(d.inverse, s.transform_inverse.data(), sizeof d.inverse);
  const Material& m = s.material;
  d.color[0] = m.color.red; d.color[1] = m.color.green; d.color[2] = m.color.blue;
  d.ambient = m.ambient; d.diffuse = m.diffuse; d.specular = m.specular; d.shininess = m.shininess;
  d.reflective = m.reflective; d.transparency = m.transparency; d.refractive_index = m.refractive_index;
  d.pattern_kind = m.has_pattern ? m.pattern.kind : RT_PATTERN_NONE;
  const Pattern& p = m.pattern;
  d.pattern_a[0] = p.a.red; d.pattern_a[1] = p.a.green; d.pattern_a[2] = p.a.blue;
  d.pattern_b[0] = p.b.red; d.pattern_b[1] = p.b.green; d.pattern_b[2] = p.b.blue;
  std::memcpy(d.pattern_transform, p.transform.data(), sizeof d.pattern_transform);
  std::memcpy(d.pattern_inverse, p.transform_inverse.data(), sizeof d.pattern_inverse);
  d.minimum = s.minimum; d.maximum = s.maximum; d.closed = s.closed ? 1 : 0;
  return d;
}

// world.rs:18-151. The flattened device copy is built lazily and dropped on
// any mutation through this API.
class World {
 public:
  World() = default;
  World(const World&) = delete;
  World& operator=(const World&) = delete;
  ~World() { drop(); }
  static std::unique_ptr<World> make_default() {  // world.rs:137-151
    auto w = std::make_unique<World>();
    w->add_light(PointLight(Point(-10, 10, -10), Color(1.0, 1.0, 1.0)));
    Shape s1 = Sphere();
    s1.material.color = Color(0.8, 1.0, 0.6);
    s1.material.diffuse = 0.7;
    s1.material.specular = 0.2;
    Shape s2 = Sphere();
    s2.set_transform(scaling(0.5, 0.5, 0.5));
    w->add_object(s1);
    w->add_object(s2);
    return w;
  }
  void add_object(const Shape& s) { drop(); objects_.push_back(GroupChild{std::make_shared<Shape>(s), nullptr}); }  // :87-89
  void add_object(const Group& g) { drop(); objects_.push_back(GroupChild{nullptr, std::make_shared<Group>(g)}); }
  void add_light(const PointLight& l) { drop(); lights_.push_back(l); }  // :83-85
  size_t n_objects() const { return objects_.size(); }
  size_t n_lights() const { return lights_.size(); }
  Shape& object(size_t i) {
    drop();
    if (!objects_.at(i).shape) throw std::invalid_argument("World::object: object is a Group");
    return *objects_[i].shape;
  }
  const Shape& object_c(size_t i) const {
    if (!objects_.at(i).shape) throw std::invalid_argument("World::object: object is a Group");
    return *objects_[i].shape;
  }
  PointLight& light(size_t i) { drop(); return lights_.at(i); }
  // The flattened World (rt_scene_create_groups): the primitives in the order
  // World::intersect's flat_map reaches them (group.rs:49-58: each group's
  // children in order), the innermost group of each (-1: none), and the groups
  // (their boxes, parents first).
  struct Flat {
    std::vector<rt_shape_desc> shapes;
    std::vector<int32_t> shape_group;
    std::vector<rt_group_desc> groups;
  };
  Flat flatten() const {
    Flat f;
    struct Walk {
      Flat& f;
      void node(const GroupChild& c, int32_t parent) {
        if (c.shape) {
          f.shapes.push_back(to_desc(*c.shape));
          f.shape_group.push_back(parent);
          return;
        }
        rt_group_desc g;
        std::memset(&g, 0, sizeof g);
        const BoundingBox& b = c.group->bbox;
        g.min[0] = b.min.x; g.min[1] = b.min.y; g.min[2] = b.min.z;
        g.max[0] = b.max.x; g.max[1] = b.max.y; g.max[2] = b.max.z;
        g.parent = parent;
        f.groups.push_back(g);
        const int32_t me = (int32_t)f.groups.size() - 1;
        for (const GroupChild& k : c.group->children) node(k, me);
      }
    } w{f};
    for (const GroupChild& c : objects_) w.node(c, -1);
    return f;
  }
  std::vector<rt_shape_desc> descs() const { return flatten().shapes; }
  std::vector<rt_light_desc> light_descs() const {
    std::vector<rt_light_desc> v(lights_.size());
    for (size_t i = 0; i < lights_.size(); ++i) {
      v[i].position[0] = lights_[i].position.x; v[i].position[1] = lights_[i].position.y;
      v[i].position[2] = lights_[i].position.z;
      v[i].intensity[0] = lights_[i].intensity.red; v[i].intensity[1] = lights_[i].intensity.green;
      v[i].intensity[2] = lights_[i].intensity.blue;
    }
    return v;
  }
  // Device-resident flattened world (uploaded on first use). `device` < 0:
  // the scene already uploaded, on whatever device it lives (device 0 when
  // none is); an explicit ordinal re-uploads when the scene lives elsewhere.
  // Every render / tuning / check path calls scene() without an ordinal, so a
  // rank that uploaded to its own GPU keeps rendering there.
  const rt_scene* scene(int device = -1) const {
    if (device < 0) device = scene_ ? scene_device_ : 0;
    if (!scene_ || scene_device_ != device) {
      const_cast<World*>(this)->drop();
      const Flat f = flatten();
      auto l = light_descs();
      rt_scene* s = nullptr;
      check(rt_scene_create_groups(f.shapes.data(), f.shapes.size(), f.shape_group.data(), f.groups.data(),
                                   f.groups.size(), l.data(), l.size(), device, &s), "rt_scene_create");
      scene_ = s;
      scene_device_ = device;
    }
    return scene_;
  }
  int scene_device() const { return scene_ ? scene_device_ : -1; }
  const void* scene_handle() const { return scene_; }
  // test hook: relabel the uploaded scene's device without moving it, so a
  // one-GPU test can check that no render path re-uploads to device 0
  void debug_relabel_device(int device) { scene_device_ = device; }
  // world.rs:70-81 on the GPU
  Color color_at(const Ray& r, unsigned remaining) const {
    double ray[6] = {r.origin.x, r.origin.y, r.origin.z, r.direction.x, r.direction.y, r.direction.z};
    double c[3];
    check(rt_color_at_batch(scene(), ray, 1, remaining, c, nullptr), "rt_color_at_batch");
    return Color(c[0], c[1], c[2]);
  }
  // world.rs:95-105 on the GPU (light given by index into `lights`)
  bool is_shadowed(const Point& p, size_t light) const {
    double pt[3] = {p.x, p.y, p.z};
    uint8_t o = 0;
    check(rt_is_shadowed_batch(scene(), pt, 1, (uint32_t)light, &o), "rt_is_shadowed_batch");
    return o != 0;
  }

 private:
  void drop() {
    if (scene_) rt_scene_destroy(scene_);
    scene_ = nullptr;
  }
  std::vector<GroupChild> objects_;
  std::vector<PointLight> lights_;
  mutable rt_scene* scene_ = nullptr;
  mutable int scene_device_ = -1;
};

// camera.rs:220-253
enum class AASamples { X1 = 1, X2 = 2, X4 = 4, X8 = 8, X16 = 16 };
struct RenderOpts {
  size_t n_threads = 1;  // CPU partitioning in the reference; no effect on the image here
  AASamples samples = AASamples::X1;
  void num_threads(size_t n) {  // camera.rs:244-247
    if (n == 0) throw std::invalid_argument("num_threads must be > 0");
    n_threads = n;
  }
  void aa_samples(AASamples s) { samples = s; }  // camera.rs:249-251
};

// camera.rs:19-253
class Camera {
 public:
  Camera(size_t hsize, size_t vsize, double field_of_view) : fov_(field_of_view) {
    check(rt_camera_init((uint32_t)hsize, (uint32_t)vsize, field_of_view, nullptr, &desc_), "rt_camera_init");
  }
  void set_transform(const Matrix& t) {  // camera.rs:128-131
    transform_ = t;
    check(rt_camera_init(desc_.hsize, desc_.vsize, fov_, t.data(), &desc_), "rt_camera_init");
  }
  size_t hsize() const { return desc_.hsize; }
  size_t vsize() const { return desc_.vsize; }
  double pixel_size() const { return desc_.pixel_size; }
  const Matrix& transform() const { return transform_; }
  double field_of_view() const { return fov_; }
  const rt_camera_desc& desc() const { return desc_; }
  Ray ray_for_pixel(size_t px, size_t py) const {  // camera.rs:57-69 (host restatement)
    const double xoffset = ((double)px + 0.5) * desc_.pixel_size;
    const double yoffset = ((double)py + 0.5) * desc_.pixel_size;
    const double world_x = desc_.half_width - xoffset;
    const double world_y = desc_.half_height - yoffset;
    const Matrix inv = Matrix::from_slice(4, 4, desc_.inverse);
    const Point pixel = inv * Point(world_x, world_y, -1.0);
    const Point origin = inv * Point::origin();
    return Ray(origin, (pixel - origin).normalize());
  }
  // camera.rs:133-148: the drop-in. `max_depth` = MAX_RECURSION_DEPTH (5).
  // `flags`: RT_RENDER_EXHAUSTIVE runs the reference's every-shape loop (exact counters).
  Canvas render(const World& world, unsigned max_depth = 5, rt_stats* stats = nullptr, uint32_t flags = 0) const {
    Canvas c(desc_.hsize, desc_.vsize, Canvas::Uninit{});
    check(rt_render_ex(world.scene(), &desc_, max_depth, 1, flags, c.data(), stats), "rt_render");
    return c;
  }
  // camera.rs:150-214: average of `rays_for_pixel` per pixel (render_opts.aa_samples).
  Canvas render_multithreaded(const World& world, unsigned max_depth = 5, rt_stats* stats = nullptr,
                              uint32_t flags = 0) const {
    Canvas c(desc_.hsize, desc_.vsize, Canvas::Uninit{});
    check(rt_render_ex(world.scene(), &desc_, max_depth, (uint32_t)render_opts.samples, flags, c.data(), stats),
          "rt_render_aa");
    return c;
  }
  // canvas_to_ppm(&self.render(world)) (camera.rs:133-148, image/ppm.rs:24-51), encoded
  // on the device; aa_samples > 1 renders as render_multithreaded does.
  std::string render_ppm(const World& world, unsigned max_depth = 5, unsigned aa_samples = 1,
                         rt_stats* stats = nullptr) const {
    std::string s;
    render_ppm_with(world, max_depth, aa_samples, stats, [&](const char* p, size_t n) { s.assign(p, n); });
    return s;
  }
  // The text in a pooled pinned block (rt_host_buffer_alloc: the device writes it at
  // the link's rate, and a frame loop reuses the same pages), handed to `take(p, n)`.
  template <typename F>
  void render_ppm_with(const World& world, unsigned max_depth, unsigned aa_samples, rt_stats* stats, F&& take) const {
    const size_t bound = 32 + (size_t)12 * desc_.hsize * desc_.vsize + desc_.vsize;
    struct Block {
      void* p;
      ~Block() { rt_host_buffer_free(p); }
    } blk{rt_host_buffer_alloc(bound)};
    std::string fallback;  // (no pinned memory to be had: a plain buffer, which the library registers)
    char* buf = (char*)blk.p;
    if (!buf) {
      fallback.resize(bound);
      buf = &fallback[0];
    }
    size_t len = 0;
    check(rt_render_ppm(world.scene(), &desc_, max_depth, aa_samples, buf, bound, &len, stats), "rt_render_ppm");
    take((const char*)buf, len);
  }
  RenderOpts render_opts;

 private:
  double fov_;
  Matrix transform_ = Matrix::identity(4, 4);
  rt_camera_desc desc_{};
};

}  // namespace rt
