/* asan_check.c -- TEST INFRASTRUCTURE ONLY (tests/test_oracle_asan.py).
 *
 * Drives the oracle's Mode B through box mode's degenerate case under
 * AddressSanitizer: a scene whose only walls are a left/right pair, a camera
 * with aperture 0 looking along -z, and image column x = W/2 of a 2^19-wide
 * image with 8 sub-pixels, where the jittered camera ray has d.x == 0 exactly
 * for 1/8 of the samples (xin rounds to 2^18, s = 0.5, d.x = X.x/2 + base.x).
 * No axis the ray moves toward then has a reachable wall plane, and box mode
 * must not select a missing wall (it read the record before the
 * scene array).  Exit status 0 and "ok <count of d.x == 0 rays>" on success. */
#include <math.h>
#include <stdio.h>
#include <string.h>

#include "pt_oracle.h"

int main(void)
{
    po_sphere s[3];
    memset(s, 0, sizeof(s));
    const double big = 1e6, off = 0.4;
    s[0].radius = big; s[0].position[0] = -big - off; s[0].position[2] = -1.0;
    s[0].color[0] = 0.9; s[0].color[1] = 0.1; s[0].color[2] = 0.2;
    s[1].radius = big; s[1].position[0] = big + off; s[1].position[2] = -1.0;
    s[1].color[0] = 0.3; s[1].color[1] = 0.1; s[1].color[2] = 0.9;
    s[2].radius = 0.2; s[2].position[1] = -0.2; s[2].position[2] = -1.0;
    s[2].color[0] = s[2].color[1] = s[2].color[2] = 1.0; s[2].material = 1;
    const int W = 1 << 19, H = 1, nsub = 8;
    po_camera_config cfg;
    memset(&cfg, 0, sizeof(cfg));
    cfg.position[2] = 2.0;
    cfg.direction[2] = -1.0;
    cfg.up[1] = 1.0;
    cfg.aspect_ratio = (double)W / (double)H;
    cfg.vertical_fov_radians = 0.5;
    cfg.focal_length = 1.0;
    cfg.aperture = 0.0;
    cfg.focus_distance = 3.0;
    po_camera cam;
    po_camera_with_config(&cfg, &cam);
    int32_t axis[3], order[3];
    po_scan_layout(s, 3, &cam, axis, order);
    if (axis[0] != 3 || axis[1] != 3) {
        printf("not a wall pair: %d %d\n", axis[0], axis[1]);
        return 2;
    }
    float out[3];
    double sum = 0.0;
    for (int sy = 0; sy < nsub; ++sy)
        for (uint32_t k = 0; k < 256; ++k) {
            po_sample_f32(s, 3, &cam, W, H, nsub, 0x5EED0001ull, W / 2, 0, 0, sy, k, out);
            sum += out[0] + out[1] + out[2];
        }
    printf("ok %.6f\n", sum);
    return 0;
}
