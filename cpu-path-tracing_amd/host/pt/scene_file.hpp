// pt/scene_file.hpp -- runtime scenes for the CLI (the
// reference's main() hard-codes its scene, main.cpp:25,199-208).
//
// Text format, one item per line, '#' starts a comment:
//
//   camera <pos x y z> <look-at x y z> <up x y z> <vfov radians> <aperture> <focus distance | auto>
//   sphere <radius> <pos x y z> <emission r g b> <colour r g b> <diffuse | specular | dielectric>
//
// Exactly one camera line.  The aspect ratio is the image's w/h and "auto"
// focuses on the look-at point, |pos - look-at| (what the reference's scene
// headers do: box_scene.hpp:67-70).  Numbers are written with 17 significant
// digits, so save -> load reproduces a scene bit for bit.  ptgpu/scene.py
// (load_scene_file / save_scene_file) reads and writes the same format.
#pragma once

#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "types.hpp"

namespace pt {

namespace detail {
inline bool parse_num(std::string const &tok, double &out)
{
    char *end = nullptr;
    out = std::strtod(tok.c_str(), &end);
    return !tok.empty() && end == tok.c_str() + tok.size();
}
inline std::string fmt17(double v)
{
    char buf[40];
    std::snprintf(buf, sizeof(buf), "%.17g", v);
    return buf;
}
}  // namespace detail

// Parses `text` into `out` for a w x h image; false (and a message naming the
// line) on malformed input.
inline bool parse_scene_text(std::string const &text, int w, int h, scene &out, std::string &err)
{
    scene scn{};
    bool have_camera = false;
    std::istringstream in{text};
    std::string line;
    int lineno = 0;
    while (std::getline(in, line)) {
        ++lineno;
        auto const hash = line.find('#');
        if (hash != std::string::npos)
            line.resize(hash);
        std::istringstream ls{line};
        std::vector<std::string> tok;
        for (std::string t; ls >> t;)
            tok.push_back(t);
        if (tok.empty())
            continue;
        auto bad = [&](std::string const &why) {
            err = "line " + std::to_string(lineno) + ": " + why;
            return false;
        };
        std::vector<double> v;
        std::size_t const nnum = tok[0] == "camera" ? 11 : (tok[0] == "sphere" ? 10 : 0);  // + focus | material
        if (nnum == 0)
            return bad("unknown item '" + tok[0] + "' (camera | sphere)");
        if (tok.size() != nnum + 2)
            return bad(tok[0] + " needs " + std::to_string(nnum + 1) + " fields");
        for (std::size_t i = 1; i <= nnum; ++i) {
            double x = 0.0;
            if (!detail::parse_num(tok[i], x))
                return bad("not a number: '" + tok[i] + "'");
            v.push_back(x);
        }
        if (tok[0] == "camera") {
            if (have_camera)
                return bad("second camera");
            have_camera = true;
            auto &c = scn.camera_parameters;
            c.position = vec3{v[0], v[1], v[2]};
            c.direction = vec3{v[3], v[4], v[5]};
            c.up = vec3{v[6], v[7], v[8]};
            c.vertical_fov_radians = v[9];
            c.aperture = v[10];
            c.aspect_ratio = (w * 1.0) / (h * 1.0);
            double f = 0.0;
            if (tok[12] == "auto")
                f = (c.position - c.direction).length();
            else if (!detail::parse_num(tok[12], f))
                return bad("focus distance must be a number or 'auto'");
            c.focus_distance = f;
        } else {
            reflection_type m;
            std::string const &mat = tok[11];
            if (mat == "diffuse")
                m = reflection_type::diffuse;
            else if (mat == "specular")
                m = reflection_type::specular;
            else if (mat == "dielectric")
                m = reflection_type::dielectric;
            else
                return bad("material must be diffuse, specular or dielectric");
            if (!(v[0] > 0.0))
                return bad("radius must be positive");
            scn.spheres.push_back(sphere{v[0], {v[1], v[2], v[3]}, {v[4], v[5], v[6]}, {v[7], v[8], v[9]}, m});
        }
    }
    if (!have_camera) {
        err = "no camera line";
        return false;
    }
    out = std::move(scn);
    return true;
}

inline bool load_scene_file(std::string const &path, int w, int h, scene &out, std::string &err)
{
    std::ifstream f{path};
    if (!f) {
        err = "cannot open " + path;
        return false;
    }
    std::stringstream ss;
    ss << f.rdbuf();
    if (!parse_scene_text(ss.str(), w, h, out, err)) {
        err = path + ": " + err;
        return false;
    }
    return true;
}

inline std::string scene_text(scene const &scn)
{
    using detail::fmt17;
    auto v3 = [](vec3 const &a) { return fmt17(a.x) + " " + fmt17(a.y) + " " + fmt17(a.z); };
    static char const *const names[] = {"diffuse", "specular", "dielectric"};
    auto const &c = scn.camera_parameters;
    std::string s = "# pt-scene: camera pos look-at up vfov aperture focus; sphere radius pos emission colour material\n";
    s += "camera " + v3(c.position) + "  " + v3(c.direction) + "  " + v3(c.up) + "  " + fmt17(c.vertical_fov_radians) +
         " " + fmt17(c.aperture) + " " + fmt17(c.focus_distance) + "\n";
    for (auto const &sp : scn.spheres)
        s += "sphere " + fmt17(sp.radius) + "  " + v3(sp.position) + "  " + v3(sp.emission) + "  " + v3(sp.color) + "  " +
             names[static_cast<int>(sp.reflection)] + "\n";
    return s;
}

inline bool save_scene_file(scene const &scn, std::string const &path)
{
    std::ofstream f{path};
    f << scene_text(scn);
    return static_cast<bool>(f);
}

}  // namespace pt
