// pt_render_gpu -- the reference's main() (src/main.cpp:199-248) with the
// taskflow row loop replaced by one call into the HIP render loop.
//
//   pt_render_gpu [spp] [scene] [width height] [out.ppm]
//     spp    total samples per pixel (main.cpp:206: divided by 4 sub-pixels), default 4
//     scene  box_mirror (the reference binary's scene, main.cpp:25,208) | box | simple | synthetic:N
//     width height  default 1024 768 (main.cpp:204-205)
//
// Writes a P3 PPM with gamma-1/2.2 8-bit values (main.cpp:240-247, utils.cpp:11-16).
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <string>
#include <vector>

#include "pt/gpu_render.hpp"
#include "pt/scenes.hpp"

namespace {

int color_to_int(double x)  // utils.cpp:11-16
{
    double const c = x < 0.0 ? 0.0 : (1.0 < x ? 1.0 : x);
    return static_cast<int>(std::round(std::pow(c, 1.0 / 2.2) * 255.0));
}

pt::scene make_scene(std::string const &name, int w, int h)
{
    if (name == "box")
        return pt::box_scene(w, h);
    if (name == "simple")
        return pt::simple_scene(w, h);
    if (name.rfind("synthetic", 0) == 0) {
        auto const colon = name.find(':');
        int const n = colon == std::string::npos ? 10000 : std::atoi(name.c_str() + colon + 1);
        return pt::synthetic_scene(n, w, h);
    }
    return pt::box_mirror_scene(w, h);
}

}  // namespace

int main(int argc, char *argv[])
{
    constexpr int num_subpixels = 2;  // main.cpp:202
    int const spp = argc > 1 ? std::atoi(argv[1]) : 4;
    std::string const scene_name = argc > 2 ? argv[2] : "box_mirror";
    int const width = argc > 4 ? std::atoi(argv[3]) : 1024;
    int const height = argc > 4 ? std::atoi(argv[4]) : 768;
    std::string const out = argc > 5 ? argv[5] : "image.ppm";
    int const samps = spp / (num_subpixels * num_subpixels);

    auto const some_scene = make_scene(scene_name, width, height);
    auto const cam = pt::camera::with_config(some_scene.camera_parameters);
    std::vector<pt::vec3> image(static_cast<std::size_t>(width) * height, pt::vec3{0, 0, 0});

    auto const t0 = std::chrono::steady_clock::now();
    int const rc = pt::gpu::render_image(some_scene, cam, image, width, height, samps, num_subpixels);
    auto const t1 = std::chrono::steady_clock::now();
    if (rc != PTG_OK) {
        std::fprintf(stderr, "render failed (%d): %s\n", rc, ptg_last_error());
        return 1;
    }
    double const secs = std::chrono::duration<double>(t1 - t0).count();
    std::fprintf(stderr, "Rendered %s %dx%d at %d spp in %.3f s (%.1f Msamples/s incl. setup + copies)\n",
                 scene_name.c_str(), width, height, samps * num_subpixels * num_subpixels, secs,
                 double(width) * height * samps * num_subpixels * num_subpixels / secs / 1e6);

    std::ofstream g{out};
    g << "P3\n" << width << ' ' << height << "\n255\n";
    for (auto const &px : image)
        g << color_to_int(px.x) << ' ' << color_to_int(px.y) << ' ' << color_to_int(px.z) << ' ';
    return 0;
}
