// scene_parser.hpp — C++ restatement of the reference's YAML scene front-end
// (scene-parser/src/lib.rs), the caller in front of `Camera::render`
// (SceneParser::render, lib.rs:267-284). Same element grammar, same order of
// evaluation and the same quirks:
//   * all `define` elements are processed first (file order), then all `add`
//     elements (lib.rs:97-117);
//   * `add` kinds: camera, light, sphere, plane, cube; any other kind is
//     skipped with a message (lib.rs:126-137);
//   * transforms compose as item * accumulated, in list order, and a string
//     item names a defined transform (lib.rs:333-373);
//   * a material is a defined name (cloned) or a hash over Material::default;
//     `extend` clones the named base and overrides the given keys
//     (lib.rs:145-187, 213-264, 286-331);
//   * patterns: `stripes` / `checkers`, anything else the default test
//     pattern; the pattern's own `transform` key is NOT read (lib.rs:450-486);
//   * numbers: Real or Integer (as f64) for floats; camera width / height
//     must be Integers and field-of-view a Real (lib.rs:403-425, 494-503).
// Errors carry the reference's SceneParserError messages (error.rs:4-25).
#pragma once
#include <fstream>
#include <map>
#include <memory>
#include <optional>
#include <sstream>
#include <string>
#include <vector>

#include "rt_world.hpp"
#include "rt_yaml.hpp"

namespace rt {

class SceneParserError : public std::runtime_error {
 public:
  explicit SceneParserError(const std::string& m) : std::runtime_error(m) {}
};

// scene-parser/src/lib.rs:49-69
struct Scene {
  std::optional<Camera> camera;
  std::vector<PointLight> lights;
  std::map<std::string, Material> materials;
  std::map<std::string, Matrix> transforms;
  std::vector<Shape> shapes;
};

class SceneParser {
 public:
  SceneParser() = default;

  // lib.rs:90-120 (from a file path)
  void load_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw SceneParserError("invalid input file `" + path + "`");
    std::stringstream ss;
    ss << f.rdbuf();
    load_str(ss.str(), path);
  }
  // the same from a string (YamlLoader::load_from_str)
  void load_str(const std::string& text, const std::string& name = "<string>") {
    const yaml::Node doc = yaml::load(text);
    if (!doc.is(yaml::Node::Array)) throw SceneParserError("invalid input file `" + name + "`");
    for (const auto& el : doc.seq)
      if (is_define_element(el)) parse_define_element(el);
    for (const auto& el : doc.seq)
      if (is_add_element(el)) parse_add_element(el);
  }

  const Scene& scene() const { return scene_; }
  Scene& scene() { return scene_; }
  std::vector<std::string> messages;  // the reference's println! diagnostics that matter

  // lib.rs:267-284: lights then shapes into a World, Camera::render.
  std::unique_ptr<World> build_world() const {
    auto w = std::make_unique<World>();
    for (const auto& l : scene_.lights) w->add_light(l);
    for (const auto& s : scene_.shapes) w->add_object(s);
    return w;
  }
  Canvas render(unsigned max_depth = 5, rt_stats* stats = nullptr) const {
    if (!scene_.camera) throw SceneParserError("missing required key `camera`");
    auto w = build_world();
    return scene_.camera->render(*w, max_depth, stats);
  }
  // lib.rs:267-284 writes a PNG; this front-end writes the PPM (image/ppm.rs)
  // (rendered and encoded on the device: rt_render_ppm; bytes = render(...).to_ppm())
  void render_to(const std::string& path, unsigned max_depth = 5) const {
    if (!scene_.camera) throw SceneParserError("missing required key `camera`");
    auto w = build_world();
    const std::string ppm = scene_.camera->hsize() <= 12288 ? scene_.camera->render_ppm(*w, max_depth)
                                                            : scene_.camera->render(*w, max_depth).to_ppm();
    std::ofstream f(path, std::ios::binary);
    if (!f) throw SceneParserError("cannot write `" + path + "`");
    f.write(ppm.data(), (std::streamsize)ppm.size());
  }

  static bool is_add_element(const yaml::Node& el) {  // lib.rs:376-382
    return el.is(yaml::Node::Hash) && el.contains("add");
  }
  static bool is_define_element(const yaml::Node& el) {  // lib.rs:384-390
    return el.is(yaml::Node::Hash) && el.contains("define");
  }

 private:
  Scene scene_;

  // lib.rs:122-140
  void parse_add_element(const yaml::Node& el) {
    const yaml::Node* kind = el.get("add");
    if (!kind || !kind->is(yaml::Node::String)) throw SceneParserError("invalid add element found");
    const std::string& k = kind->s;
    if (k == "camera") scene_.camera = parse_camera(el);
    else if (k == "light") scene_.lights.push_back(parse_light(el));
    else if (k == "sphere" || k == "plane" || k == "cube") scene_.shapes.push_back(parse_shape(k, el));
    else messages.push_back("unhandled element: " + k);
  }

  // lib.rs:142-187
  void parse_define_element(const yaml::Node& el) {
    const yaml::Node* name_el = el.get("define");
    if (!name_el || !name_el->is(yaml::Node::String)) throw SceneParserError("invalid define element found");
    const std::string name = name_el->s;
    const yaml::Node* value = el.get("value");
    if (!value) throw SceneParserError("invalid define element found");
    const yaml::Node* extend = el.get("extend");
    if (value->is(yaml::Node::Array)) {
      scene_.transforms[name] = parse_transform(*value);
    } else if (value->is(yaml::Node::Hash)) {
      if (extend) {
        if (!extend->is(yaml::Node::String)) throw SceneParserError("invalid define element found");
        auto it = scene_.materials.find(extend->s);
        if (it == scene_.materials.end()) throw SceneParserError("invalid define element found");
        scene_.materials[name] = apply_material_keys(it->second, *value);
      } else {
        scene_.materials[name] = parse_material(*value);
      }
    } else {
      throw SceneParserError("invalid define element found");  // unreachable!() in the reference
    }
  }

  // lib.rs:189-211
  Shape parse_shape(const std::string& kind, const yaml::Node& el) {
    Shape s = kind == "sphere" ? Sphere() : kind == "plane" ? Plane() : Cube();
    if (const yaml::Node* t = el.get("transform")) s.set_transform(parse_transform(*t));
    if (const yaml::Node* m = el.get("material")) s.material = parse_material(*m);
    return s;
  }

  // lib.rs:213-264 and 286-331 (identical key handling)
  Material apply_material_keys(Material m, const yaml::Node& def) const {
    if (!def.is(yaml::Node::Hash)) throw SceneParserError("failed to parse material");
    if (const yaml::Node* c = def.get("color")) {
      if (!c->is(yaml::Node::Array)) throw SceneParserError("failed to parse material");
      m.color = to_color(*c);
    }
    if (const yaml::Node* p = def.get("pattern")) m.set_pattern(parse_pattern(*p));
    if (const yaml::Node* v = def.get("ambient")) m.ambient = to_f64(*v);
    if (const yaml::Node* v = def.get("diffuse")) m.diffuse = to_f64(*v);
    if (const yaml::Node* v = def.get("specular")) m.specular = to_f64(*v);
    if (const yaml::Node* v = def.get("shininess")) m.shininess = to_f64(*v);
    if (const yaml::Node* v = def.get("reflective")) m.reflective = to_f64(*v);
    if (const yaml::Node* v = def.get("transparency")) m.transparency = to_f64(*v);
    if (const yaml::Node* v = def.get("refractive-index")) m.refractive_index = to_f64(*v);
    return m;
  }
  Material parse_material(const yaml::Node& el) const {
    if (el.is(yaml::Node::String)) {
      auto it = scene_.materials.find(el.s);
      if (it == scene_.materials.end()) throw SceneParserError("failed to parse material");
      return it->second;
    }
    if (el.is(yaml::Node::Hash)) return apply_material_keys(Material(), el);
    throw SceneParserError("failed to parse material");
  }

  // lib.rs:333-346: transform = item * transform, in list order
  Matrix parse_transform(const yaml::Node& el) const {
    if (!el.is(yaml::Node::Array)) throw SceneParserError("failed to parse transform");
    Matrix t = Matrix::identity(4, 4);
    for (const auto& item : el.seq) t = parse_transform_item(item) * t;
    return t;
  }
  // lib.rs:348-373
  Matrix parse_transform_item(const yaml::Node& el) const {
    if (el.is(yaml::Node::Array)) {
      if (el.seq.empty() || !el.seq[0].is(yaml::Node::String)) throw SceneParserError("failed to parse transform");
      const std::string& kind = el.seq[0].s;
      std::vector<double> a;
      for (size_t i = 1; i < el.seq.size(); ++i) a.push_back(to_f64(el.seq[i]));
      auto need = [&](size_t n) {
        if (a.size() < n) throw SceneParserError("failed to parse transform");  // index panic in the reference
      };
      if (kind == "scale") { need(3); return scaling(a[0], a[1], a[2]); }
      if (kind == "translate") { need(3); return translation(a[0], a[1], a[2]); }
      if (kind == "rotate-x") { need(1); return rotation_x(a[0]); }
      if (kind == "rotate-y") { need(1); return rotation_y(a[0]); }
      if (kind == "rotate-z") { need(1); return rotation_z(a[0]); }
      throw SceneParserError("failed to parse transform");
    }
    if (el.is(yaml::Node::String)) {
      auto it = scene_.transforms.find(el.s);
      if (it == scene_.transforms.end()) throw SceneParserError("failed to parse transform");
      return it->second;
    }
    throw SceneParserError("failed to parse transform");
  }

  static const yaml::Node& required(const yaml::Node& h, const std::string& key) {  // lib.rs:488-492
    const yaml::Node* v = h.get(key);
    if (!v) throw SceneParserError("missing required key `" + key + "`");
    return *v;
  }
  // lib.rs:392-427
  static Camera parse_camera(const yaml::Node& el) {
    int64_t width, height;
    double fov;
    if (!required(el, "width").as_i64(&width)) throw SceneParserError("failed to parse `width` as i64");
    if (!required(el, "height").as_i64(&height)) throw SceneParserError("failed to parse `height` as i64");
    if (!required(el, "field-of-view").as_f64(&fov))
      throw SceneParserError("failed to parse `field-of-view` as f64");
    const yaml::Node& from = required(el, "from");
    const yaml::Node& to = required(el, "to");
    const yaml::Node& up = required(el, "up");
    if (!from.is(yaml::Node::Array)) throw SceneParserError("failed to parse `from` as vec");
    if (!to.is(yaml::Node::Array)) throw SceneParserError("failed to parse `to` as vec");
    if (!up.is(yaml::Node::Array)) throw SceneParserError("failed to parse `up` as vec");
    const auto f = to3(from), t = to3(to), u = to3(up);
    if (width <= 0 || height <= 0) throw SceneParserError("failed to parse `width` as i64");
    Camera cam((size_t)width, (size_t)height, fov);
    cam.set_transform(view_transform(Point(f[0], f[1], f[2]), Point(t[0], t[1], t[2]), Vector(u[0], u[1], u[2])));
    return cam;
  }
  // lib.rs:429-448
  static PointLight parse_light(const yaml::Node& el) {
    const yaml::Node& at = required(el, "at");
    const yaml::Node& in = required(el, "intensity");
    if (!at.is(yaml::Node::Array) || !in.is(yaml::Node::Array)) throw SceneParserError("failed to parse `from` as vec");
    const auto p = to3(at);
    return PointLight(Point(p[0], p[1], p[2]), to_color(in));
  }
  // lib.rs:450-486
  static Pattern parse_pattern(const yaml::Node& el) {
    if (!el.is(yaml::Node::Hash)) throw SceneParserError("failed to parse pattern");
    const yaml::Node* kind = el.get("type");
    if (!kind || !kind->is(yaml::Node::String)) throw SceneParserError("failed to parse pattern");
    const yaml::Node* colors = el.get("colors");
    if (!colors || !colors->is(yaml::Node::Array)) throw SceneParserError("failed to parse pattern");
    std::vector<Color> cs;
    for (const auto& c : colors->seq) {
      if (!c.is(yaml::Node::Array)) throw SceneParserError("failed to parse pattern");
      cs.push_back(to_color(c));
    }
    if (kind->s == "stripes" || kind->s == "checkers") {
      if (cs.size() < 2) throw SceneParserError("failed to parse pattern");  // index panic in the reference
      return kind->s == "stripes" ? stripe_pattern(cs[0], cs[1]) : checkers_pattern(cs[0], cs[1]);
    }
    return test_pattern();  // Pattern::default()
  }
  // lib.rs:494-503
  static double to_f64(const yaml::Node& v) {
    double d;
    if (v.is(yaml::Node::Real) && v.as_f64(&d)) return d;
    if (v.is(yaml::Node::Integer)) return (double)v.i;
    throw SceneParserError("failed to parse `f` as f64");
  }
  // lib.rs:510-536 (to_point / to_vector / to_color: exactly three numbers)
  static std::vector<double> to3(const yaml::Node& v) {
    std::vector<double> n;
    for (const auto& x : v.seq) n.push_back(to_f64(x));
    if (n.size() != 3) throw SceneParserError("failed to parse `from` as vec");
    return n;
  }
  static Color to_color(const yaml::Node& v) {
    const auto n = to3(v);
    return Color(n[0], n[1], n[2]);
  }
};

}  // namespace rt
