// pt_render_gpu -- the reference's main() (src/main.cpp:199-248) with the
// taskflow row loop replaced by one call into the HIP render loop, plus the
// runtime options the reference hard-codes.
//
//   pt_render_gpu [spp] [scene] [width height] [out.ppm]        (positional, as before)
//   pt_render_gpu [--spp N] [--scene NAME|FILE] [--width W] [--height H] [--seed S]
//                 [--devices 0,1,...] [--out FILE] [--format p3|p6]
//                 [--save-scene FILE] [--dump-json FILE] [--no-render] [--exact-math]
//
//   spp      total samples per pixel (main.cpp:206: divided by the 4 sub-pixels), default 4
//   scene    box_mirror (the reference binary's scene, main.cpp:25,208) | box | simple |
//            synthetic:N | a scene file (pt/scene_file.hpp)
//   devices  distinct GPUs to split the image over (ptg_render_multi): device k
//            renders the interleaved rows r = k mod N, ONE RCCL gather collects
//            them on the first device; the image is the same bit for bit for any
//            device list (default: the current device, ptg_render)
//   out      P3 (the reference's format) or P6 PPM, gamma-1/2.2 8-bit values
//            (main.cpp:240-247, utils.cpp:11-16)
//   --exact-math  the kernel's exact arithmetic (PTG_FLAG_EXACT_MATH): the image equals
//            the CPU oracle's bit for bit (default: the GPU's fast transcendentals)
//   --save-scene / --dump-json write the scene (scene file) / the scene and the
//            camera::with_config result (JSON, 17 digits) and need no GPU with --no-render
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "pt/gpu_render.hpp"
#include "pt/scene_file.hpp"
#include "pt/scenes.hpp"

namespace {

int color_to_int(double x)  // utils.cpp:11-16
{
    double const c = x < 0.0 ? 0.0 : (1.0 < x ? 1.0 : x);
    return static_cast<int>(std::round(std::pow(c, 1.0 / 2.2) * 255.0));
}

bool make_scene(std::string const &name, int w, int h, pt::scene &out, std::string &err)
{
    if (name == "box")
        out = pt::box_scene(w, h);
    else if (name == "box_mirror")
        out = pt::box_mirror_scene(w, h);
    else if (name == "simple")
        out = pt::simple_scene(w, h);
    else if (name.rfind("synthetic", 0) == 0) {
        auto const colon = name.find(':');
        int const n = colon == std::string::npos ? 10000 : std::atoi(name.c_str() + colon + 1);
        out = pt::synthetic_scene(n, w, h);
    } else
        return pt::load_scene_file(name, w, h, out, err);
    return true;
}

std::vector<int> parse_devices(std::string const &s)
{
    std::vector<int> d;
    std::size_t i = 0;
    while (i < s.size()) {
        std::size_t j = s.find(',', i);
        if (j == std::string::npos)
            j = s.size();
        d.push_back(std::atoi(s.substr(i, j - i).c_str()));
        i = j + 1;
    }
    return d;
}

void dump_json(pt::scene const &scn, pt::camera const &cam, std::string const &path)
{
    auto v3 = [](pt::vec3 const &a) {
        char b[100];
        std::snprintf(b, sizeof(b), "[%.17g, %.17g, %.17g]", a.x, a.y, a.z);
        return std::string(b);
    };
    std::ofstream f{path};
    f << "{\"spheres\": [";
    for (std::size_t i = 0; i < scn.spheres.size(); ++i) {
        auto const &s = scn.spheres[i];
        char r[40];
        std::snprintf(r, sizeof(r), "%.17g", s.radius);
        f << (i ? ", " : "") << "{\"radius\": " << r << ", \"position\": " << v3(s.position)
          << ", \"emission\": " << v3(s.emission) << ", \"color\": " << v3(s.color)
          << ", \"material\": " << static_cast<int>(s.reflection) << "}";
    }
    char lr[40];
    std::snprintf(lr, sizeof(lr), "%.17g", cam.lens_radius);
    f << "], \"camera\": {\"position\": " << v3(cam.position) << ", \"lower_left_corner\": " << v3(cam.lower_left_corner)
      << ", \"cam_x_axis\": " << v3(cam.cam_x_axis) << ", \"cam_y_axis\": " << v3(cam.cam_y_axis)
      << ", \"u\": " << v3(cam.u) << ", \"v\": " << v3(cam.v) << ", \"w\": " << v3(cam.w)
      << ", \"lens_radius\": " << lr << "}}\n";
}

}  // namespace

int main(int argc, char *argv[])
{
    constexpr int num_subpixels = 2;  // main.cpp:202
    int spp = 4, width = 1024, height = 768;
    std::string scene_name = "box_mirror", out = "image.ppm", format = "p3", save_scene, dump, devices = "-1";
    std::uint64_t seed = pt::gpu::default_seed;
    bool render = true;
    int flags = 0;
    if (argc > 1 && std::strncmp(argv[1], "--", 2) != 0) {  // the positional form
        spp = std::atoi(argv[1]);
        if (argc > 2)
            scene_name = argv[2];
        if (argc > 4) {
            width = std::atoi(argv[3]);
            height = std::atoi(argv[4]);
        }
        if (argc > 5)
            out = argv[5];
    } else {
        for (int i = 1; i < argc; ++i) {
            std::string const a = argv[i];
            auto val = [&]() -> std::string {
                if (i + 1 >= argc) {
                    std::fprintf(stderr, "%s needs a value\n", a.c_str());
                    std::exit(2);
                }
                return argv[++i];
            };
            if (a == "--spp")
                spp = std::atoi(val().c_str());
            else if (a == "--scene")
                scene_name = val();
            else if (a == "--width")
                width = std::atoi(val().c_str());
            else if (a == "--height")
                height = std::atoi(val().c_str());
            else if (a == "--seed")
                seed = std::strtoull(val().c_str(), nullptr, 0);
            else if (a == "--devices")
                devices = val();
            else if (a == "--out")
                out = val();
            else if (a == "--format")
                format = val();
            else if (a == "--save-scene")
                save_scene = val();
            else if (a == "--dump-json")
                dump = val();
            else if (a == "--no-render")
                render = false;
            else if (a == "--exact-math")
                flags |= PTG_FLAG_EXACT_MATH;
            else {
                std::fprintf(stderr, "unknown option %s\n", a.c_str());
                return 2;
            }
        }
    }
    if (width <= 0 || height <= 0 || spp < 0 || (format != "p3" && format != "p6")) {
        std::fprintf(stderr, "bad width/height/spp/format\n");
        return 2;
    }
    int const samps = spp / (num_subpixels * num_subpixels);

    pt::scene some_scene;
    std::string err;
    if (!make_scene(scene_name, width, height, some_scene, err)) {
        std::fprintf(stderr, "scene: %s\n", err.c_str());
        return 2;
    }
    auto const cam = pt::camera::with_config(some_scene.camera_parameters);
    if (!save_scene.empty() && !pt::save_scene_file(some_scene, save_scene)) {
        std::fprintf(stderr, "cannot write %s\n", save_scene.c_str());
        return 1;
    }
    if (!dump.empty())
        dump_json(some_scene, cam, dump);
    if (!render)
        return 0;

    std::vector<pt::vec3> image(static_cast<std::size_t>(width) * height, pt::vec3{0, 0, 0});
    std::vector<int> const devs = parse_devices(devices);
    int const nd = static_cast<int>(devs.size());
    auto const t0 = std::chrono::steady_clock::now();
    int rc = PTG_OK;
    if (nd == 1 && devs[0] < 0) {  // main.cpp:214-236 replaced by one call
        rc = pt::gpu::render_image(some_scene, cam, image, width, height, samps, num_subpixels, seed, -1, flags);
    } else {  // several GPUs of this process: shards + one RCCL gather
        ptg_params p{};
        p.width = width;
        p.height = height;
        p.samples = samps;
        p.num_subpixels = num_subpixels;
        p.seed = seed;
        p.band_rows = 1;
        p.shard_rank = 0;
        p.shard_count = 1;
        p.flags = flags;
        rc = ptg_render_multi(reinterpret_cast<ptg_sphere const *>(some_scene.spheres.data()), some_scene.spheres.size(),
                              reinterpret_cast<ptg_camera const *>(&cam), &p, devs.data(), nd,
                              reinterpret_cast<double *>(image.data()));
    }
    auto const t1 = std::chrono::steady_clock::now();
    if (rc != PTG_OK) {
        std::fprintf(stderr, "render failed (%d): %s\n", rc, ptg_last_error());
        return 1;
    }
    double const secs = std::chrono::duration<double>(t1 - t0).count();
    std::fprintf(stderr, "Rendered %s %dx%d at %d spp on %d device(s) in %.3f s (%.1f Msamples/s incl. setup + copies)\n",
                 scene_name.c_str(), width, height, samps * num_subpixels * num_subpixels, nd, secs,
                 double(width) * height * samps * num_subpixels * num_subpixels / secs / 1e6);

    std::ofstream g{out, std::ios::binary};
    if (format == "p6") {
        g << "P6\n" << width << ' ' << height << "\n255\n";
        for (auto const &px : image) {
            unsigned char const rgb[3] = {static_cast<unsigned char>(color_to_int(px.x)),
                                          static_cast<unsigned char>(color_to_int(px.y)),
                                          static_cast<unsigned char>(color_to_int(px.z))};
            g.write(reinterpret_cast<char const *>(rgb), 3);
        }
    } else {
        g << "P3\n" << width << ' ' << height << "\n255\n";
        for (auto const &px : image)
            g << color_to_int(px.x) << ' ' << color_to_int(px.y) << ' ' << color_to_int(px.z) << ' ';
    }
    return 0;
}
