"""Wall pairs and box mode (DESIGN.md "wall pairs", "box mode") on scenes
that probe their premise: a ray from inside the room never needs the wall
it moves away from.

ADVICE r1 (low) asked about spheres sunk into a wall.  Their sunk part lies
inside the wall, which a ray from the room reaches only through the wall's
surface -- the wall is hit there first -- so the rule holds; this is checked
against the oracle with every sphere tested in index order (BV_FULL_SCAN: no
pairs, no box mode).  What does break the premise is a path travelling
inside a wall (a dielectric wall) or a camera inside the margin band: those
walls are never paired (ptg_render.hip wall_clear, pt_oracle.c wall_clear_B).
"""
import numpy as np

import ptgpu
import pyoracle as po

SEED = 0x5EED0001


def _arrays(scn):
    cam = ptgpu.camera.with_config(scn.camera_parameters)
    return (np.ascontiguousarray(scn.to_array().view(po.SPHERE_DT)),
            np.ascontiguousarray(cam.to_array().view(po.CAMERA_DT)), cam)


def sunk_scene(W, H):
    scn = ptgpu.make_scene("box", W, H)
    glass = ptgpu.reflection_type.dielectric
    scn.spheres = scn.spheres + [ptgpu.sphere(0.15, (-0.35, 0.0, -0.8), (0, 0, 0), (1, 1, 1), glass),  # 0.1 into the left wall
                                 ptgpu.sphere(0.12, (0.3, 0.35, -0.9), (0, 0, 0), (1, 1, 1), glass)]   # into the right wall and ceiling
    return scn


def test_sunk_glass_spheres_keep_box_mode_exact():
    W, H, samps = 96, 72, 32
    sp, ca, cam = _arrays(sunk_scene(W, H))
    axis, _ = po.scan_layout(sp, ca)
    assert axis[:5] == [3, 3, 2, 4, 4]  # pairs and box mode stay on
    assert ptgpu.scene_layout(sunk_scene(W, H), cam) == po.scan_layout(sp, ca)
    b, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    with po.mode_b_variant(po.BV_FULL_SCAN):
        f, _ = po.render_xs_f32(sp, ca, W, H, samps, 2, SEED)
    a, _ = po.render_xs_f64(sp, ca, W, H, samps, 2, SEED)
    d = np.abs(b.astype(np.float64) - f)
    # the rule changes no path beyond fp32 rounding noise (measured: 1 of
    # 19,200 pixels differs at 160x120x256 spp)
    assert float(np.sqrt((d ** 2).mean())) < 1e-4 and (d.max(axis=2) > 0).mean() < 1e-3
    ra = float(np.sqrt(((b - a) ** 2).mean()))
    rf = float(np.sqrt(((f - a) ** 2).mean()))
    assert ra < 1.2 * rf + 1e-5  # as close to the double reference as without the rule


def test_dielectric_wall_and_camera_in_band_are_not_paired():
    scn = ptgpu.make_scene("box", 32, 24)
    scn.spheres[0] = ptgpu.sphere(scn.spheres[0].radius, scn.spheres[0].position, (0, 0, 0), (1, 1, 1),
                                  ptgpu.reflection_type.dielectric)  # left wall made of glass
    sp, ca, cam = _arrays(scn)
    axis, _ = po.scan_layout(sp, ca)
    assert axis[0] == 0 and axis[1] == 0 and axis[3] == 4 and axis[4] == 4  # x walls unpaired, y pair kept
    assert ptgpu.scene_layout(scn, cam) == (axis, po.scan_layout(sp, ca)[1])
    scn = ptgpu.make_scene("box", 32, 24)
    scn.camera_parameters.position = (0.39995, 0.0, 2.0)  # within 1e-4 * diagonal of the right wall's plane
    sp, ca, cam = _arrays(scn)
    axis, _ = po.scan_layout(sp, ca)
    assert axis[0] == 0 and axis[1] == 0
    assert ptgpu.scene_layout(scn, cam)[0] == axis
