// rtamd_py.cpp — pybind11 bindings of the C++ host API (host/rt_world.hpp) so
// Python tests and bench.py drive exactly the code a C++/FFI caller would.
// Nothing here computes a pixel: render / color_at / is_shadowed / hits go
// through the C-ABI into the HIP kernels.
#include <pybind11/numpy.h>
#include <pybind11/operators.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <algorithm>
#include <cstring>
#include <thread>

#include "../host/rt_world.hpp"
#include "../host/scene_parser.hpp"

namespace py = pybind11;
using namespace rt;

static py::dict stats_dict(const rt_stats& s) {
  py::dict d;
  d["rays_primary"] = s.rays_primary;
  d["rays_reflect"] = s.rays_reflect;
  d["rays_refract"] = s.rays_refract;
  d["rays_shadow"] = s.rays_shadow;
  d["sphere_tests"] = s.sphere_tests;
  d["plane_tests"] = s.plane_tests;
  // None on the fast path: only the exhaustive loop evaluates every sphere test
  if (s.sphere_disc_ge0 == RT_STATS_NOT_COUNTED) d["sphere_disc_ge0"] = py::none();
  else d["sphere_disc_ge0"] = s.sphere_disc_ge0;
  d["other_tests"] = s.other_tests;
  d["ms_kernel"] = s.ms_kernel;
  d["ms_total"] = s.ms_total;
  d["rays_shadow_traced"] = s.rays_shadow_traced;
  d["sphere_tests_executed"] = s.sphere_tests_executed;
  d["box_tests_executed"] = s.box_tests_executed;
  d["exhaustive"] = (bool)s.exhaustive;
  return d;
}

// The `exhaustive` keyword of the render bindings: None follows want_stats (the
// counted reference loop, whose counters the tests compare with the oracle's).
static uint32_t render_flags(bool want_stats, const py::object& exhaustive) {
  const bool ex = exhaustive.is_none() ? want_stats : exhaustive.cast<bool>();
  return ex ? (uint32_t)RT_RENDER_EXHAUSTIVE : 0u;
}

static py::bytes pod_bytes(const void* p, size_t n) { return py::bytes((const char*)p, n); }

static py::array_t<double> check_rays(py::array_t<double, py::array::c_style | py::array::forcecast> a,
                                      size_t width) {
  if (a.ndim() != 2 || (size_t)a.shape(1) != width)
    throw std::invalid_argument("expected an (n, " + std::to_string(width) + ") float64 array");
  return a;
}

// memcpy on up to 8 threads (large host-to-host copies out of freshly DMA'd pinned memory)
static void parallel_copy(char* dst, const char* src, size_t n) {
  const size_t kMin = (size_t)4 << 20;
  const unsigned nt = n < kMin ? 1u : (unsigned)std::min<size_t>(8, std::max(1u, std::thread::hardware_concurrency() / 2));
  if (nt <= 1) {
    std::memcpy(dst, src, n);
    return;
  }
  const size_t part = ((n + nt - 1) / nt + 4095) & ~(size_t)4095;
  std::vector<std::thread> pool;
  unsigned t = 1;
  try {
    for (; t < nt && t * part < n; ++t)
      pool.emplace_back([=] { std::memcpy(dst + t * part, src + t * part, std::min(part, n - t * part)); });
  } catch (...) {  // a thread that cannot start: copied here
  }
  for (unsigned u = t; u < nt && u * part < n; ++u) std::memcpy(dst + u * part, src + u * part, std::min(part, n - u * part));
  std::memcpy(dst, src, std::min(part, n));
  for (std::thread& th : pool) th.join();
}

extern "C" int rtamd_tuning_set(const char* key, int value);
extern "C" int rtamd_stream_create(int cu_masked, void** out);
extern "C" int rtamd_nccl_unique_id(unsigned char* out, size_t size);
extern "C" int rtamd_nccl_comm_init(int nranks, const unsigned char* id, size_t size, int rank, int device,
                                    int timeout_ms, void** comm);
extern "C" int rtamd_nccl_comm_abort(void* comm);
extern "C" int rtamd_nccl_gather_f64(const double* send, double* recv, size_t count, int root, void* comm, void* stream);
extern "C" int rtamd_nccl_comm_destroy(void* comm);
extern "C" int rtamd_wf_profile(const rt_scene* s, int enable, double out[38]);
extern "C" int rtamd_wf_gen_counts(const rt_scene* s, unsigned* out, int max);
extern "C" int rtamd_scene_tuning_set(const rt_scene* s, const char* key, int value);
extern "C" int rtamd_render_shard_host(const rt_scene* scene, const rt_camera_desc* camera, uint32_t max_depth,
                                       uint32_t aa_samples, uint32_t row_block, uint32_t shard, uint32_t n_shards,
                                       double* out_rgb, rt_stats* stats);

PYBIND11_MODULE(_rtamd, m) {
  m.doc() = "MI355X-native render path of raytracer-challenge-rs (host API over the C-ABI)";
  py::register_exception<RtError>(m, "RtError");
  m.attr("EPSILON") = EPSILON;
  m.attr("ABI_VERSION") = RT_ABI_VERSION;
  m.def("equal", &equal);
  m.def("device_count", &rt_device_count);
  m.def("abi_version", &rt_abi_version);

  py::class_<Point>(m, "Point")
      .def(py::init<double, double, double>())
      .def_static("origin", &Point::origin)
      .def_readwrite("x", &Point::x).def_readwrite("y", &Point::y).def_readwrite("z", &Point::z)
      .def("__eq__", [](const Point& a, const Point& b) { return a == b; })
      .def("__add__", [](const Point& p, const Vector& v) { return p + v; })
      .def("__sub__", [](const Point& a, const Point& b) { return a - b; })
      .def("__sub__", [](const Point& p, const Vector& v) { return p - v; })
      .def("tuple", [](const Point& p) { return py::make_tuple(p.x, p.y, p.z); })
      .def("__repr__", [](const Point& p) { return "Point(" + std::to_string(p.x) + ", " + std::to_string(p.y) + ", " + std::to_string(p.z) + ")"; });
  py::class_<Vector>(m, "Vector")
      .def(py::init<double, double, double>())
      .def_readwrite("x", &Vector::x).def_readwrite("y", &Vector::y).def_readwrite("z", &Vector::z)
      .def("magnitude", &Vector::magnitude)
      .def("normalize", &Vector::normalize)
      .def("reflect", &Vector::reflect)
      .def("__eq__", [](const Vector& a, const Vector& b) { return a == b; })
      .def("__add__", [](const Vector& a, const Vector& b) { return a + b; })
      .def("__sub__", [](const Vector& a, const Vector& b) { return a - b; })
      .def("__neg__", [](const Vector& a) { return -a; })
      .def("__mul__", [](const Vector& a, double s) { return a * s; })
      .def("tuple", [](const Vector& p) { return py::make_tuple(p.x, p.y, p.z); })
      .def("__repr__", [](const Vector& p) { return "Vector(" + std::to_string(p.x) + ", " + std::to_string(p.y) + ", " + std::to_string(p.z) + ")"; });
  m.def("dot", &dot);
  m.def("cross", &cross);
  py::class_<Color>(m, "Color")
      .def(py::init<double, double, double>())
      .def_static("black", &Color::black)
      .def_static("white", &Color::white)
      .def_readwrite("red", &Color::red).def_readwrite("green", &Color::green).def_readwrite("blue", &Color::blue)
      .def("__eq__", [](const Color& a, const Color& b) { return a == b; })
      .def("tuple", [](const Color& c) { return py::make_tuple(c.red, c.green, c.blue); })
      .def("__repr__", [](const Color& c) { return "Color(" + std::to_string(c.red) + ", " + std::to_string(c.green) + ", " + std::to_string(c.blue) + ")"; });
  py::class_<Ray>(m, "Ray")
      .def(py::init<const Point&, const Vector&>())
      .def_readwrite("origin", &Ray::origin)
      .def_readwrite("direction", &Ray::direction)
      .def("position", &Ray::position)
      .def("transform", [](const Ray& r, const Matrix& mm) { return transform(r, mm); });

  py::class_<Matrix>(m, "Matrix")
      .def(py::init<int, int>())
      .def_static("identity", &Matrix::identity)
      .def_static("from_rows", [](const std::vector<std::vector<double>>& rows) {
        int r = (int)rows.size(), c = r ? (int)rows[0].size() : 0;
        Matrix mm(r, c);
        for (int i = 0; i < r; ++i) {
          if ((int)rows[i].size() != c) throw std::invalid_argument("ragged rows");
          for (int j = 0; j < c; ++j) mm(i, j) = rows[i][j];
        }
        return mm;
      })
      .def("rows", &Matrix::rows)
      .def("columns", &Matrix::columns)
      .def("__getitem__", [](const Matrix& mm, std::pair<int, int> ij) {
        if (ij.first < 0 || ij.first >= mm.rows() || ij.second < 0 || ij.second >= mm.columns())
          throw py::index_error();
        return mm(ij.first, ij.second);
      })
      .def("__setitem__", [](Matrix& mm, std::pair<int, int> ij, double v) {
        if (ij.first < 0 || ij.first >= mm.rows() || ij.second < 0 || ij.second >= mm.columns())
          throw py::index_error();
        mm(ij.first, ij.second) = v;
      })
      .def("transpose", &Matrix::transpose)
      .def("determinant", &Matrix::determinant)
      .def("submatrix", &Matrix::submatrix)
      .def("minor", &Matrix::minor)
      .def("cofactor", &Matrix::cofactor)
      .def("is_invertible", &Matrix::is_invertible)
      .def("inverse", [](const Matrix& mm) {
        if (!mm.is_invertible()) throw RtError(RT_ERR_NOT_INVERTIBLE, "matrix is not invertible");
        return mm.inverse();
      })
      .def("translate", &Matrix::translate)
      .def("scale", &Matrix::scale)
      .def("rotate_x", &Matrix::rotate_x)
      .def("rotate_y", &Matrix::rotate_y)
      .def("rotate_z", &Matrix::rotate_z)
      .def("shear", &Matrix::shear)
      .def("__eq__", [](const Matrix& a, const Matrix& b) { return a == b; })
      .def("__mul__", [](const Matrix& a, const Matrix& b) { return a * b; })
      .def("__mul__", [](const Matrix& a, const Point& p) { return a * p; })
      .def("__mul__", [](const Matrix& a, const Vector& v) { return a * v; })
      .def("to_list", [](const Matrix& mm) {
        std::vector<double> v(mm.data(), mm.data() + mm.rows() * mm.columns());
        return v;
      });
  m.def("translation", &translation);
  m.def("scaling", &scaling);
  m.def("rotation_x", &rotation_x);
  m.def("rotation_y", &rotation_y);
  m.def("rotation_z", &rotation_z);
  m.def("shearing", &shearing);
  m.def("view_transform", &view_transform);

  py::class_<Pattern>(m, "Pattern")
      .def_readonly("kind", &Pattern::kind)
      .def_readwrite("a", &Pattern::a)
      .def_readwrite("b", &Pattern::b)
      .def_readonly("transform", &Pattern::transform)
      .def_readonly("transform_inverse", &Pattern::transform_inverse)
      .def("set_transform", &Pattern::set_transform);
  m.def("test_pattern", &test_pattern);
  m.def("stripe_pattern", &stripe_pattern);
  m.def("gradient_pattern", &gradient_pattern);
  m.def("ring_pattern", &ring_pattern);
  m.def("checkers_pattern", &checkers_pattern);

  py::class_<Material>(m, "Material")
      .def(py::init<>())
      .def_readwrite("color", &Material::color)
      .def_readwrite("ambient", &Material::ambient)
      .def_readwrite("diffuse", &Material::diffuse)
      .def_readwrite("specular", &Material::specular)
      .def_readwrite("shininess", &Material::shininess)
      .def_readwrite("reflective", &Material::reflective)
      .def_readwrite("transparency", &Material::transparency)
      .def_readwrite("refractive_index", &Material::refractive_index)
      .def_readonly("has_pattern", &Material::has_pattern)
      .def_readonly("pattern", &Material::pattern)
      .def("set_pattern", &Material::set_pattern)
      .def("copy", [](const Material& mm) { return mm; });

  py::class_<PointLight>(m, "PointLight")
      .def(py::init<const Point&, const Color&>())
      .def_readwrite("position", &PointLight::position)
      .def_readwrite("intensity", &PointLight::intensity);

  py::class_<Shape>(m, "Shape")
      .def_readonly("kind", &Shape::kind)
      .def_readwrite("material", &Shape::material)
      .def_readwrite("minimum", &Shape::minimum)
      .def_readwrite("maximum", &Shape::maximum)
      .def_readwrite("closed", &Shape::closed)
      .def_readonly("transform", &Shape::transform)
      .def_readonly("transform_inverse", &Shape::transform_inverse)
      .def("transform_inverse_transpose", &Shape::transform_inverse_transpose)
      .def("set_transform", &Shape::set_transform)
      .def("set_material", &Shape::set_material)
      .def("no_shadow", &Shape::no_shadow)
      .def("has_shadow", &Shape::has_shadow)
      .def("get_bounds", [](const Shape& s) { return s.bbox; })
      .def("parent_space_bounds", &Shape::parent_space_bounds)
      .def("desc_bytes", [](const Shape& s) { rt_shape_desc d = to_desc(s); return pod_bytes(&d, sizeof d); });
  // geometry/shape/group.rs: children by value (a copy of the shape or group is moved in, as
  // add_child takes its Box); child(i) returns a copy of child i
  py::class_<Group>(m, "Group")
      .def(py::init<>())
      .def("add_child", [](Group& g, const Shape& s) { g.add_child(s); })
      .def("add_child", [](Group& g, const Group& c) { g.add_child(c); })
      .def("set_transform", &Group::set_transform)
      .def("set_material", &Group::set_material)
      .def_readonly("transform", &Group::transform)
      .def_readonly("transform_inverse", &Group::transform_inverse)
      .def_readonly("material", &Group::material)
      .def("n_children", [](const Group& g) { return g.children.size(); })
      .def("child", [](const Group& g, size_t i) -> py::object {
        const GroupChild& c = g.children.at(i);
        if (c.shape) return py::cast(*c.shape);
        return py::cast(*c.group);
      })
      .def("get_bounds", [](const Group& g) { return g.bbox; })
      .def("parent_space_bounds", &Group::parent_space_bounds)
      .def("divide", &Group::divide, py::arg("threshold"));
  // bounding_box.rs: the box type behind Group culling
  py::class_<BoundingBox>(m, "BoundingBox")
      .def(py::init<>())
      .def(py::init<const Point&, const Point&>())
      .def_readwrite("min", &BoundingBox::min)
      .def_readwrite("max", &BoundingBox::max)
      .def("add_point", &BoundingBox::add_point)
      .def("add_bounding_box", &BoundingBox::add_box)
      .def("contains_point", &BoundingBox::contains_point)
      .def("contains_bounding_box", &BoundingBox::contains_box)
      .def("transform", &BoundingBox::transform)
      .def("intersects", &BoundingBox::intersects)
      .def("split", &BoundingBox::split);
  m.def("Sphere", &Sphere);
  m.def("glass_sphere", &glass_sphere);
  m.def("Plane", &Plane);
  m.def("Cube", &Cube);
  m.def("Cylinder", &Cylinder, py::arg("minimum") = -std::numeric_limits<double>::infinity(),
        py::arg("maximum") = std::numeric_limits<double>::infinity(), py::arg("closed") = false);
  m.def("Cone", &Cone, py::arg("minimum") = -std::numeric_limits<double>::infinity(),
        py::arg("maximum") = std::numeric_limits<double>::infinity(), py::arg("closed") = false);

  py::enum_<AASamples>(m, "AASamples")
      .value("X1", AASamples::X1).value("X2", AASamples::X2).value("X4", AASamples::X4)
      .value("X8", AASamples::X8).value("X16", AASamples::X16);
  py::class_<RenderOpts>(m, "RenderOpts")
      .def("num_threads", &RenderOpts::num_threads)
      .def("aa_samples", &RenderOpts::aa_samples)
      .def_property_readonly("samples", [](const RenderOpts& o) { return (int)o.samples; });

  py::class_<Canvas>(m, "Canvas")
      .def(py::init<size_t, size_t>())
      .def("width", &Canvas::width)
      .def("height", &Canvas::height)
      .def("get_pixel", &Canvas::get_pixel)
      .def("set_pixel", &Canvas::set_pixel)
      .def("to_ppm", [](const Canvas& c) { return py::bytes(c.to_ppm()); })
      .def("to_numpy", [](const Canvas& c) {
        py::array_t<double> a({(py::ssize_t)c.height(), (py::ssize_t)c.width(), (py::ssize_t)3});
        std::memcpy(a.mutable_data(), c.data(), c.width() * c.height() * 3 * sizeof(double));
        return a;
      });
  m.def("canvas_to_ppm", [](py::array_t<double, py::array::c_style | py::array::forcecast> rgb) {
    if (rgb.ndim() != 3 || rgb.shape(2) != 3) throw std::invalid_argument("expected (h, w, 3)");
    size_t len = 0;
    const uint32_t h = (uint32_t)rgb.shape(0), w = (uint32_t)rgb.shape(1);
    // one pass into a bytes object of the bound (12 bytes per pixel at most, + a newline per
    // row + the header), shrunk to the text afterwards: the pages past it are never touched
    const size_t bound = (size_t)12 * w * h + h + 32;
    PyObject* obj = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)bound);
    if (!obj) throw py::error_already_set();
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = rt_canvas_to_ppm(rgb.data(), w, h, PyBytes_AS_STRING(obj), bound, &len);
    }
    if (rc != RT_OK) {
      Py_DECREF(obj);
      check(rc, "rt_canvas_to_ppm");
    }
    if (_PyBytes_Resize(&obj, (Py_ssize_t)len) != 0) throw py::error_already_set();
    return py::reinterpret_steal<py::bytes>(obj);
  });
  // canvas_to_ppm of a device canvas into a device buffer (pointers as integers, e.g.
  // torch tensors' data_ptr()); returns the text's length
  m.def("canvas_to_ppm_device", [](uintptr_t d_rgb, uint32_t w, uint32_t h, uintptr_t d_out, size_t cap,
                                   uintptr_t stream) {
    size_t len = 0;
    {
      py::gil_scoped_release nogil;
      check(rt_canvas_to_ppm_device((const double*)d_rgb, w, h, (char*)d_out, cap, &len, (void*)stream),
            "rt_canvas_to_ppm_device");
    }
    return len;
  }, py::arg("d_rgb"), py::arg("width"), py::arg("height"), py::arg("d_out"), py::arg("cap"), py::arg("stream") = 0);
  m.def("quantize_u8", [](py::array_t<double, py::array::c_style | py::array::forcecast> v) {
    py::array_t<uint8_t> o(v.size());
    check(rt_quantize_u8(v.data(), (size_t)v.size(), o.mutable_data()), "rt_quantize_u8");
    return o;
  });
  m.def("matrix_inverse_raw", [](const std::vector<double>& mm) {
    if (mm.size() != 16) throw std::invalid_argument("need 16 values");
    std::vector<double> out(16);
    check(rt_matrix_inverse(mm.data(), out.data()), "rt_matrix_inverse");
    return out;
  });

  py::class_<World>(m, "World")
      .def(py::init<>())
      .def_static("default", &World::make_default)
      .def("add_object", [](World& w, const Shape& s) { w.add_object(s); })
      .def("add_object", [](World& w, const Group& g) { w.add_object(g); })
      .def("add_light", &World::add_light)
      .def("n_objects", &World::n_objects)
      .def("n_lights", &World::n_lights)
      .def("object", &World::object, py::return_value_policy::reference_internal)
      .def("light", &World::light, py::return_value_policy::reference_internal)
      .def("upload", [](const World& w, int device) { w.scene(device); }, py::arg("device") = 0)
      .def_property_readonly("scene_device", &World::scene_device)  // -1: not uploaded
      .def("_scene_handle", [](const World& w) { return (uintptr_t)w.scene_handle(); })
      .def("_debug_relabel_device", &World::debug_relabel_device)
      .def("tune", [](const World& w, const std::string& k, int v) {  // this scene's render-time knob (dev)
        check(rtamd_scene_tuning_set(w.scene(), k.c_str(), v), "tuning");
      })
      .def("check", [](const World& w) {  // rt_scene_check: every frame issued on the scene was complete
        py::gil_scoped_release nogil;
        check(rt_scene_check(w.scene()), "rt_scene_check");
      })
      .def("color_at", &World::color_at, py::arg("ray"), py::arg("remaining") = 5)
      .def("is_shadowed", &World::is_shadowed)
      .def("descs_bytes", [](const World& w) {
        auto d = w.descs();
        return pod_bytes(d.data(), d.size() * sizeof(rt_shape_desc));
      })
      .def("groups_bytes", [](const World& w) {  // rt_group_desc[], parents first
        auto f = w.flatten();
        return pod_bytes(f.groups.data(), f.groups.size() * sizeof(rt_group_desc));
      })
      .def("shape_groups", [](const World& w) { return w.flatten().shape_group; })  // innermost group per shape
      .def("lights_bytes", [](const World& w) {
        auto l = w.light_descs();
        return pod_bytes(l.data(), l.size() * sizeof(rt_light_desc));
      })
      .def("color_at_batch", [](const World& w, py::array_t<double, py::array::c_style | py::array::forcecast> rays,
                                unsigned remaining, bool want_stats, py::object exhaustive) {
        check_rays(rays, 6);
        const size_t n = (size_t)rays.shape(0);
        py::array_t<double> out({(py::ssize_t)n, (py::ssize_t)3});
        rt_stats st{};
        const uint32_t flags = render_flags(want_stats, exhaustive);
        {
          py::gil_scoped_release nogil;
          check(rt_color_at_batch_ex(w.scene(), rays.data(), n, remaining, flags, out.mutable_data(),
                                     want_stats ? &st : nullptr),
                "rt_color_at_batch");
        }
        return py::make_tuple(out, stats_dict(st));
      }, py::arg("rays"), py::arg("remaining") = 5, py::arg("want_stats") = true, py::arg("exhaustive") = py::none())
      .def("hit_batch", [](const World& w, py::array_t<double, py::array::c_style | py::array::forcecast> rays) {
        check_rays(rays, 6);
        const size_t n = (size_t)rays.shape(0);
        py::array_t<double> out({(py::ssize_t)n, (py::ssize_t)24});
        check(rt_hit_batch(w.scene(), rays.data(), n, out.mutable_data()), "rt_hit_batch");
        return out;
      })
      .def("is_shadowed_batch", [](const World& w, py::array_t<double, py::array::c_style | py::array::forcecast> pts,
                                   unsigned light) {
        check_rays(pts, 3);
        const size_t n = (size_t)pts.shape(0);
        py::array_t<uint8_t> out(n);
        check(rt_is_shadowed_batch(w.scene(), pts.data(), n, light, out.mutable_data()), "rt_is_shadowed_batch");
        return out;
      });

  py::class_<Camera>(m, "Camera")
      .def(py::init<size_t, size_t, double>())
      .def("set_transform", &Camera::set_transform)
      .def_property_readonly("hsize", &Camera::hsize)
      .def_property_readonly("vsize", &Camera::vsize)
      .def_property_readonly("pixel_size", &Camera::pixel_size)
      .def_property_readonly("transform", &Camera::transform)
      .def_property_readonly("field_of_view", &Camera::field_of_view)
      .def("ray_for_pixel", &Camera::ray_for_pixel)
      .def("desc_bytes", [](const Camera& c) { return pod_bytes(&c.desc(), sizeof(rt_camera_desc)); })
      // want_stats: return the counters. exhaustive: run the reference's every-shape loop
      // (RT_RENDER_EXHAUSTIVE: exact sphere_disc_ge0 too); None = the same as want_stats, so
      // render(w) is the counted reference loop and render(w, want_stats=False) the fast path
      .def("render", [](const Camera& c, const World& w, unsigned max_depth, bool want_stats, py::object exhaustive) {
        rt_stats st{};
        Canvas* out;
        const uint32_t flags = render_flags(want_stats, exhaustive);
        {
          py::gil_scoped_release nogil;
          out = new Canvas(c.render(w, max_depth, want_stats ? &st : nullptr, flags));
        }
        return py::make_tuple(std::unique_ptr<Canvas>(out), stats_dict(st));
      }, py::arg("world"), py::arg("max_depth") = 5, py::arg("want_stats") = true, py::arg("exhaustive") = py::none())
      .def("render_ppm", [](const Camera& c, const World& w, unsigned max_depth, unsigned aa_samples, bool want_stats) {
        rt_stats st{};
        py::object out;
        {
          py::gil_scoped_release nogil;
          // the bytes object is filled from the pinned text by a few threads: the text was
          // just written by DMA, so it is read from DRAM, which one core reads at ~25 GB/s
          c.render_ppm_with(w, max_depth, aa_samples, want_stats ? &st : nullptr, [&](const char* p, size_t n) {
            char* dst = nullptr;
            {
              py::gil_scoped_acquire gil;
              PyObject* b = PyBytes_FromStringAndSize(nullptr, (Py_ssize_t)n);
              if (!b) throw py::error_already_set();
              out = py::reinterpret_steal<py::object>(b);
              dst = PyBytes_AS_STRING(b);
            }
            parallel_copy(dst, p, n);
          });
        }
        return py::make_tuple(out, stats_dict(st));
      }, py::arg("world"), py::arg("max_depth") = 5, py::arg("aa_samples") = 1, py::arg("want_stats") = false)
      // canvas_to_ppm(&camera.render(&world)) into the caller's buffer (rt_render_ppm with a
      // reused output buffer, as a frame loop holds one): returns the text's length
      .def("render_ppm_into", [](const Camera& c, const World& w, py::buffer out, unsigned max_depth,
                                 unsigned aa_samples) {
        py::buffer_info bi = out.request(true);
        if (bi.ndim != 1 || bi.itemsize != 1) throw std::invalid_argument("expected a writable 1-D byte buffer");
        size_t len = 0;
        int rc;
        {
          py::gil_scoped_release nogil;
          rc = rt_render_ppm(w.scene(), &c.desc(), max_depth, aa_samples, (char*)bi.ptr, (size_t)bi.size, &len,
                             nullptr);
        }
        check(rc, "rt_render_ppm");
        return len;
      }, py::arg("world"), py::arg("out"), py::arg("max_depth") = 5, py::arg("aa_samples") = 1)
      .def_readwrite("render_opts", &Camera::render_opts, py::return_value_policy::reference_internal)
      .def("render_multithreaded", [](const Camera& c, const World& w, unsigned max_depth, bool want_stats,
                                      py::object exhaustive) {
        rt_stats st{};
        Canvas* out;
        const uint32_t flags = render_flags(want_stats, exhaustive);
        {
          py::gil_scoped_release nogil;
          out = new Canvas(c.render_multithreaded(w, max_depth, want_stats ? &st : nullptr, flags));
        }
        return py::make_tuple(std::unique_ptr<Canvas>(out), stats_dict(st));
      }, py::arg("world"), py::arg("max_depth") = 5, py::arg("want_stats") = true, py::arg("exhaustive") = py::none())
      .def("render_shard_device", [](const Camera& c, const World& w, unsigned max_depth, unsigned row_block,
                                     unsigned shard, unsigned n_shards, uintptr_t d_out, uintptr_t stream,
                                     bool want_stats, unsigned aa_samples, py::object exhaustive) {
        rt_stats st{};
        int rc;
        const uint32_t flags = render_flags(want_stats, exhaustive);
        {
          py::gil_scoped_release nogil;
          rc = rt_render_shard_device_ex(w.scene(), &c.desc(), max_depth, aa_samples, row_block, shard, n_shards,
                                         flags, (double*)d_out, (void*)stream, want_stats ? &st : nullptr);
        }
        check(rc, "rt_render_shard_device");
        return stats_dict(st);
      }, py::arg("world"), py::arg("max_depth"), py::arg("row_block"), py::arg("shard"), py::arg("n_shards"),
         py::arg("d_out"), py::arg("stream") = 0, py::arg("want_stats") = false, py::arg("aa_samples") = 1,
         py::arg("exhaustive") = py::none())
      .def("render_multi", [](const Camera& c, std::vector<World*> worlds, unsigned max_depth, unsigned row_block,
                              unsigned aa_samples, bool want_stats) {
        std::vector<rt_scene*> sc;
        for (size_t i = 0; i < worlds.size(); ++i) sc.push_back(const_cast<rt_scene*>(worlds[i]->scene((int)i)));
        Canvas* out = new Canvas(c.hsize(), c.vsize(), Canvas::Uninit{});  // (a pooled pinned block: every pixel is written)
        rt_stats st{};
        int rc;
        {
          py::gil_scoped_release nogil;
          rc = rt_render_multi(sc.data(), (int)sc.size(), &c.desc(), max_depth, aa_samples, row_block, out->data(),
                               want_stats ? &st : nullptr);
        }
        if (rc != RT_OK) { delete out; check(rc, "rt_render_multi"); }
        return py::make_tuple(std::unique_ptr<Canvas>(out), stats_dict(st));
      }, py::arg("worlds"), py::arg("max_depth") = 5, py::arg("row_block") = 8, py::arg("aa_samples") = 1,
         py::arg("want_stats") = true);
  m.def("shard_rows", &rt_shard_rows);
  // a pinned host buffer from the library's pool (rt_host_buffer_alloc): uint8, freed with the array
  m.def("host_buffer", [](size_t bytes) {
    void* p = rt_host_buffer_alloc(bytes);
    if (!p) throw RtError(RT_ERR_HOST, std::string("rt_host_buffer_alloc: ") + rt_last_error());
    py::capsule owner(p, [](void* q) { rt_host_buffer_free(q); });
    return py::array_t<uint8_t>({(py::ssize_t)bytes}, {(py::ssize_t)1}, (uint8_t*)p, owner);
  }, py::arg("bytes"));
  // dev/test: one device's part of rt_render_multi (shard rows straight into a full-size host canvas)
  m.def("_render_shard_host", [](const World& w, const Camera& c, unsigned max_depth, unsigned row_block,
                                 unsigned shard, unsigned n_shards,
                                 py::array_t<double, py::array::c_style> out, unsigned aa_samples, bool want_stats) {
    if (out.ndim() != 3 || (size_t)out.shape(0) != c.vsize() || (size_t)out.shape(1) != c.hsize() || out.shape(2) != 3)
      throw std::invalid_argument("expected a (vsize, hsize, 3) float64 canvas");
    double* p = out.mutable_data();
    rt_stats st{};
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = rtamd_render_shard_host(w.scene(), &c.desc(), max_depth, aa_samples, row_block, shard, n_shards, p,
                                   want_stats ? &st : nullptr);
    }
    check(rc, "rtamd_render_shard_host");
    return stats_dict(st);
  }, py::arg("world"), py::arg("camera"), py::arg("max_depth"), py::arg("row_block"), py::arg("shard"),
     py::arg("n_shards"), py::arg("out"), py::arg("aa_samples") = 1, py::arg("want_stats") = false);
  m.def("render_frames_device", [](const World& w, std::vector<const Camera*> cams, unsigned max_depth,
                                   unsigned row_block, unsigned shard, unsigned n_shards, std::vector<uintptr_t> d_outs,
                                   uintptr_t stream, bool want_stats, unsigned aa_samples) {
    if (cams.size() != d_outs.size()) throw std::invalid_argument("one device buffer per camera");
    std::vector<rt_camera_desc> descs;
    for (const Camera* c : cams) descs.push_back(c->desc());
    std::vector<double*> outs;
    for (uintptr_t p : d_outs) outs.push_back((double*)p);
    rt_stats st{};
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = rt_render_frames_device(w.scene(), descs.data(), (uint32_t)descs.size(), max_depth, aa_samples, row_block,
                                   shard, n_shards, outs.data(), (void*)stream, want_stats ? &st : nullptr);
    }
    check(rc, "rt_render_frames_device");
    return stats_dict(st);
  }, py::arg("world"), py::arg("cameras"), py::arg("max_depth"), py::arg("row_block"), py::arg("shard"),
     py::arg("n_shards"), py::arg("d_outs"), py::arg("stream") = 0, py::arg("want_stats") = false,
     py::arg("aa_samples") = 1);
  m.def("pattern_rows", &rt_pattern_rows);
  m.def("render_block_pattern_device", [](const World& w, std::vector<const Camera*> cams, unsigned max_depth,
                                          unsigned row_block, unsigned period, uint64_t mask,
                                          std::vector<uintptr_t> d_outs, uintptr_t stream, bool want_stats,
                                          unsigned aa_samples, bool exhaustive) {
    if (cams.size() != d_outs.size()) throw std::invalid_argument("one device buffer per camera");
    std::vector<rt_camera_desc> descs;
    for (const Camera* c : cams) descs.push_back(c->desc());
    std::vector<double*> outs;
    for (uintptr_t p : d_outs) outs.push_back((double*)p);
    rt_stats st{};
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = rt_render_block_pattern_device(w.scene(), descs.data(), (uint32_t)descs.size(), max_depth, aa_samples,
                                          row_block, period, mask, exhaustive ? RT_RENDER_EXHAUSTIVE : 0u,
                                          outs.data(), (void*)stream, want_stats ? &st : nullptr);
    }
    check(rc, "rt_render_block_pattern_device");
    return stats_dict(st);
  }, py::arg("world"), py::arg("cameras"), py::arg("max_depth"), py::arg("row_block"), py::arg("period"),
     py::arg("mask"), py::arg("d_outs"), py::arg("stream") = 0, py::arg("want_stats") = false,
     py::arg("aa_samples") = 1, py::arg("exhaustive") = false);

  // scene-parser/src/lib.rs: the YAML front-end (C++ restatement)
  py::register_exception<SceneParserError>(m, "SceneParserError");
  py::register_exception<yaml::ParseError>(m, "YamlError");
  py::class_<SceneParser>(m, "SceneParser")
      .def(py::init<>())
      .def("load_file", &SceneParser::load_file)
      .def("load_str", &SceneParser::load_str, py::arg("text"), py::arg("name") = "<string>")
      .def_readonly("messages", &SceneParser::messages)
      .def_property_readonly("camera", [](const SceneParser& p) -> py::object {
        if (!p.scene().camera) return py::none();
        return py::cast(*p.scene().camera);
      })
      .def_property_readonly("lights", [](const SceneParser& p) { return p.scene().lights; })
      .def_property_readonly("shapes", [](const SceneParser& p) { return p.scene().shapes; })
      .def_property_readonly("materials", [](const SceneParser& p) { return p.scene().materials; })
      .def_property_readonly("transforms", [](const SceneParser& p) { return p.scene().transforms; })
      .def("build_world", &SceneParser::build_world)
      .def("render", [](const SceneParser& p, unsigned max_depth) {
        rt_stats st{};
        Canvas* out;
        {
          py::gil_scoped_release nogil;
          out = new Canvas(p.render(max_depth, &st));
        }
        return py::make_tuple(std::unique_ptr<Canvas>(out), stats_dict(st));
      }, py::arg("max_depth") = 5)
      .def("render_to", &SceneParser::render_to, py::arg("path"), py::arg("max_depth") = 5);
  m.def("_wf_gen_counts", [](const World& w) {
    unsigned o[66] = {0};
    const int n = rtamd_wf_gen_counts(w.scene(), o, 66);
    if (n < 0) check(n, "wf_gen_counts");
    py::list l;
    for (int i = 0; i < n; ++i) l.append(o[i]);
    return l;
  }, py::arg("world"));
  m.def("_wf_profile", [](const World& w, int enable, bool read) {
    double o[38] = {0};
    check(rtamd_wf_profile(w.scene(), enable, read ? o : nullptr), "wf_profile");
    py::dict d;
    if (read) {
      const char* cls[5] = {"primary", "closest", "shadow", "prep", "combine"};
      py::dict ms, rays, disc;
      for (int i = 0; i < 5; ++i) ms[cls[i]] = o[i];
      for (int i = 0; i < 3; ++i) { rays[cls[i]] = o[5 + i]; disc[cls[i]] = o[8 + i]; }
      d["ms"] = ms; d["rays"] = rays; d["disc"] = disc;
      d["n_diag"] = o[11]; d["n_gen"] = o[12]; d["n_planes"] = o[13]; d["n_lights"] = o[14];
      d["n_quads"] = o[15];
      py::dict tests, boxes;
      for (int i = 0; i < 3; ++i) { tests[cls[i]] = o[16 + i]; boxes[cls[i]] = o[19 + i]; }
      d["tests"] = tests; d["boxes"] = boxes; d["bvh"] = (bool)o[22]; d["n_bvh_nodes"] = o[23]; d["bvh_depth"] = o[24];
      d["n_obvh_nodes"] = o[25]; d["n_other_culled"] = o[26];
      d["lb_res"] = o[27]; d["lb_items"] = o[28];
      py::dict shr, sht;
      shr["primary"] = o[29]; shr["closest"] = o[30]; sht["primary"] = o[31]; sht["closest"] = o[32];
      d["shadow_rays_in"] = shr; d["shadow_tests_in"] = sht; d["fused"] = (bool)o[33];
      d["n_bvh_wide"] = (int)o[34]; d["wide_stack"] = (int)o[35];
      d["n_lbvh_nodes"] = (int)o[36]; d["n_line_culled"] = (int)o[37];
    }
    return d;
  }, py::arg("world"), py::arg("enable") = -1, py::arg("read") = true);
  m.def("_tuning_set", [](const std::string& k, int v) { check(rtamd_tuning_set(k.c_str(), v), "tuning"); });
  m.def("_nccl_unique_id", []() {
    std::string id(128, '\0');
    check(rtamd_nccl_unique_id((unsigned char*)&id[0], id.size()), "nccl unique id");
    return py::bytes(id);
  });
  m.def("_nccl_comm_init", [](int nranks, py::bytes id, int rank, int device, int timeout_ms) {
    std::string s = id;
    void* comm = nullptr;
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = rtamd_nccl_comm_init(nranks, (const unsigned char*)s.data(), s.size(), rank, device, timeout_ms, &comm);
    }
    check(rc, "nccl comm init");
    return (uintptr_t)comm;
  }, py::arg("nranks"), py::arg("id"), py::arg("rank"), py::arg("device"), py::arg("timeout_ms") = 60000);
  m.def("_nccl_comm_abort", [](uintptr_t comm) { check(rtamd_nccl_comm_abort((void*)comm), "nccl comm abort"); });
  m.def("_nccl_gather_f64", [](uintptr_t send, uintptr_t recv, size_t count, int root, uintptr_t comm, uintptr_t stream) {
    check(rtamd_nccl_gather_f64((const double*)send, (double*)recv, count, root, (void*)comm, (void*)stream), "nccl gather");
  });
  m.def("_nccl_comm_destroy", [](uintptr_t comm) { check(rtamd_nccl_comm_destroy((void*)comm), "nccl comm destroy"); });
  m.def("_stream_create", [](bool cu_masked) {
    void* st = nullptr;
    check(rtamd_stream_create(cu_masked ? 1 : 0, &st), "stream");
    return (uintptr_t)st;
  });
}
