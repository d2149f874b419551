// render_scene — the reference's scene-parser/src/bin/render_scene.rs on the
// MI355X path: `render_scene <scene-file> <output-file>` parses the YAML scene
// (csrc/host/scene_parser.hpp) and renders it with Camera::render through the
// C-ABI (GPU). The output is a P3 PPM (the reference writes a PNG).
#include <cstdio>
#include <exception>

#include "../host/scene_parser.hpp"

int main(int argc, char** argv) {
  if (argc != 3) {
    std::printf("usage: render_scene <scene-file> <output-file>\n");
    return 2;
  }
  try {
    rt::SceneParser parser;
    parser.load_file(argv[1]);
    for (const auto& m : parser.messages) std::printf("%s\n", m.c_str());
    parser.render_to(argv[2]);
    std::printf("scene saved to %s\n", argv[2]);
  } catch (const std::exception& e) {
    std::fprintf(stderr, "Error: %s\n", e.what());
    return 1;
  }
  return 0;
}
