"""Host-side mirror of the reference's scene types and scene builders.

Python counterparts of pt::vec3 (vec.hpp:7-32), pt::sphere (sphere.hpp:10-22),
pt::camera_config / pt::camera (camera.hpp:11-43), pt::scene (scene.hpp:12-16),
pt::reflection_type (reflection.hpp:7-12) and the three hand-built scenes
(simple_scene.hpp:14-52, box_scene.hpp:14-72, box_mirror_scene.hpp:14-72).
Arithmetic is IEEE double in the reference's evaluation order, so scenes and
cameras equal the reference's bit-for-bit (tests/test_host.py checks them
against the golden dumps of the compiled reference).

Scenes are packed into numpy structured arrays whose layout IS the C ABI's
(ptg_sphere = pt::sphere, 88 B; ptg_camera = pt::camera, 176 B).
"""
from __future__ import annotations

import enum
import math
from dataclasses import dataclass, field
from typing import List, Tuple

import numpy as np

SPHERE_DT = np.dtype([("radius", "<f8"), ("position", "<f8", 3), ("emission", "<f8", 3),
                      ("color", "<f8", 3), ("material", "<i4"), ("reserved_", "<i4")])
CAMERA_DT = np.dtype([("position", "<f8", 3), ("lower_left_corner", "<f8", 3),
                      ("cam_x_axis", "<f8", 3), ("cam_y_axis", "<f8", 3), ("u", "<f8", 3),
                      ("v", "<f8", 3), ("w", "<f8", 3), ("lens_radius", "<f8")])
assert SPHERE_DT.itemsize == 88 and CAMERA_DT.itemsize == 176


class reflection_type(enum.IntEnum):  # reflection.hpp:7-12
    diffuse = 0
    specular = 1
    dielectric = 2


Vec = Tuple[float, float, float]


def _sub(a: Vec, b: Vec) -> Vec:
    return (a[0] - b[0], a[1] - b[1], a[2] - b[2])


def _mul(a: Vec, s: float) -> Vec:
    return (a[0] * s, a[1] * s, a[2] * s)


def _norm(a: Vec) -> Vec:  # vec.cpp:35-38
    return _mul(a, 1 / math.sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]))


def _cross(a: Vec, b: Vec) -> Vec:  # vec.cpp:45-48
    return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])


def length(a: Vec) -> float:
    """vec.cpp:66-69: std::hypot(x, y, z) as libstdc++ evaluates it."""
    x, y, z = abs(a[0]), abs(a[1]), abs(a[2])
    m = (z if y < z else y) if x < y else (z if x < z else x)
    if m:
        return m * math.sqrt((x / m) * (x / m) + (y / m) * (y / m) + (z / m) * (z / m))
    return 0.0


@dataclass
class sphere:  # sphere.hpp:10-17
    radius: float = 0.0
    position: Vec = (0.0, 0.0, 0.0)
    emission: Vec = (0.0, 0.0, 0.0)
    color: Vec = (0.0, 0.0, 0.0)
    reflection: reflection_type = reflection_type.diffuse


@dataclass
class camera_config:  # camera.hpp:11-21
    position: Vec = (0.0, 0.0, 0.0)
    direction: Vec = (0.0, 0.0, 0.0)
    up: Vec = (0.0, 1.0, 0.0)
    aspect_ratio: float = 16.0 / 9.0
    vertical_fov_radians: float = 0.785398163
    focal_length: float = 1.0
    aperture: float = 0.0
    focus_distance: float = 0.0


@dataclass
class camera:  # camera.hpp:23-33
    position: Vec
    lower_left_corner: Vec
    cam_x_axis: Vec
    cam_y_axis: Vec
    u: Vec
    v: Vec
    w: Vec
    lens_radius: float

    @staticmethod
    def with_config(cfg: camera_config) -> "camera":  # camera.cpp:3-17
        vh = 2.0 * math.tan(0.5 * cfg.vertical_fov_radians)
        vw = cfg.aspect_ratio * vh
        w = _norm(_sub(cfg.position, cfg.direction))
        u = _norm(_cross(cfg.up, w))
        v = _cross(w, u)
        X = _mul(_mul(u, vw), cfg.focus_distance)
        Y = _mul(_mul(v, vh), cfg.focus_distance)
        llc = _sub(_sub(_sub(cfg.position, _mul(X, 0.5)), _mul(Y, 0.5)), _mul(w, cfg.focus_distance))
        return camera(cfg.position, llc, X, Y, u, v, w, cfg.aperture / 2.0)

    def to_array(self) -> np.ndarray:
        a = np.zeros(1, dtype=CAMERA_DT)
        for k in ("position", "lower_left_corner", "cam_x_axis", "cam_y_axis", "u", "v", "w"):
            a[0][k] = getattr(self, k)
        a[0]["lens_radius"] = self.lens_radius
        return a


@dataclass
class scene:  # scene.hpp:12-16
    spheres: List[sphere] = field(default_factory=list)
    camera_parameters: camera_config = field(default_factory=camera_config)

    def to_array(self) -> np.ndarray:
        a = np.zeros(len(self.spheres), dtype=SPHERE_DT)
        for i, s in enumerate(self.spheres):
            a[i]["radius"] = s.radius
            a[i]["position"] = s.position
            a[i]["emission"] = s.emission
            a[i]["color"] = s.color
            a[i]["material"] = int(s.reflection)
        return a


def _finish(scn: scene, w: int, h: int, fov: float, aperture: float = 0.2) -> scene:
    c = scn.camera_parameters
    c.aspect_ratio = (w * 1.0) / (h * 1.0)
    c.vertical_fov_radians = fov
    c.aperture = aperture
    c.focus_distance = length(_sub(c.position, c.direction))
    return scn


def simple_scene(w: int, h: int) -> scene:
    """simple_scene.hpp:14-52"""
    D, S, G = reflection_type.diffuse, reflection_type.specular, reflection_type.dielectric
    scn = scene([
        sphere(100.0, (0.0, -100.5, -1.0), (0.0, 0.0, 0.0), (0.8, 0.8, 0.0), D),     # ground
        sphere(0.5, (1.0, 0.0, -1.0), (0.0, 0.0, 0.0), (0.999, 0.999, 0.999), S),    # right
        sphere(0.5, (-1.0, 0.0, -1.0), (0.0, 0.0, 0.0), (0.999, 0.999, 0.999), G),   # left
        sphere(0.5, (0.0, 0.0, -1.0), (0.1, 0.1, 0.9), (0.0, 0.7, 0.1), D),          # centre light
        sphere(1.0, (1.0, 3.1, -1.0), (30.0, 30.0, 30.0), (0.0, 0.0, 0.0), D),       # top light
    ])
    scn.camera_parameters.position = (-2.0, 2.0, 1.0)
    scn.camera_parameters.direction = (0.0, 0.0, -1.0)
    return _finish(scn, w, h, 1.2)


def _box(w: int, h: int, mirror: bool) -> scene:
    big, off, y, z = 1e6, 0.4, 0.0, -1.0
    wall = reflection_type.specular if mirror else reflection_type.diffuse
    walls = [
        ((-big - off, y, z), (0.9, 0.1, 0.2)),   # left
        ((big + off, y, z), (0.3, 0.1, 0.9)),    # right
        ((0.0, 0.0, z - big), (0.1, 0.7, 0.2)),  # back
        ((0.0, big + off, z), (0.3, 0.7, 0.2)),  # top
        ((0.0, -big - off, z), (0.9, 0.9, 0.9)),  # bottom
    ]
    scn = scene([sphere(big, p, (0.0, 0.0, 0.0), c, wall) for p, c in walls])
    r = off / 2.0
    if mirror:  # box_mirror_scene.hpp:48-62
        light = (1.92, 1.91, 1.9)
        scn.spheres += [
            sphere(r, (0.0, 0.0 + off / 4.0, z + off * 1.5), light, light, reflection_type.diffuse),
            sphere(r, (off / 2.0, -off / 2.0, z + off), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0), reflection_type.specular),
            sphere(r, (-off / 2.0, -off / 2.0, z + off), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0), reflection_type.dielectric),
        ]
    else:  # box_scene.hpp:48-62
        scn.spheres += [
            sphere(r, (0.0, 0.0 + off / 4.0, z - off / 2.5), (9.0, 9.0, 9.0), (1.8, 1.8, 1.8), reflection_type.diffuse),
            sphere(r, (off / 2.0, -off / 2.0, z + off * 1.5), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0), reflection_type.specular),
            sphere(r, (-off / 2.0, -off / 2.0, z + off * 1.5), (0.0, 0.0, 0.0), (1.0, 1.0, 1.0), reflection_type.dielectric),
        ]
    scn.camera_parameters.position = (0.0, 0.0, 2.0)
    scn.camera_parameters.direction = (0.0, 0.0, z + off * 1.5)
    return _finish(scn, w, h, 0.75 if mirror else 0.5)


def box_scene(w: int, h: int) -> scene:
    """box_scene.hpp:14-72 (diffuse walls)"""
    return _box(w, h, mirror=False)


def box_mirror_scene(w: int, h: int) -> scene:
    """box_mirror_scene.hpp:14-72 (the scene the shipped binary renders, main.cpp:25,208)"""
    return _box(w, h, mirror=True)


def _canonical(raw: np.ndarray) -> np.ndarray:
    """generate_canonical<double,53> over pairs of mt19937 words (random.tcc:3348-3380)."""
    g = raw.astype(np.float64).reshape(-1, 2)
    r = (g[:, 0] + g[:, 1] * 4294967296.0) / 18446744073709551616.0
    return np.where(r >= 1.0, np.nextafter(1.0, 0.0), r)


def synthetic_scene(n: int, w: int, h: int, gen_seed: int = 42) -> scene:
    """BASELINE.json configs[4]: a ground sphere (R 1e3), one emitter, n-2 small
    random spheres (materials 80/15/5 % diffuse/specular/dielectric).  The
    reference has no such generator; this one is defined in DESIGN.md and
    mirrored by the oracle's po_scene_synthetic."""
    if n < 2:
        raise ValueError("synthetic scene needs n >= 2")
    bg = np.random.MT19937()
    bg._legacy_seeding(gen_seed)  # == std::mt19937(gen_seed)
    u = _canonical(bg.random_raw(2 * 7 * (n - 2))).reshape(-1, 7) if n > 2 else np.zeros((0, 7))
    D = reflection_type.diffuse
    scn = scene([sphere(1000.0, (0.0, -1000.0, 0.0), (0.0, 0.0, 0.0), (0.5, 0.5, 0.5), D),
                 sphere(2.0, (0.0, 8.0, 0.0), (8.0, 8.0, 8.0), (0.8, 0.8, 0.8), D)])
    for row in u:
        r = 0.05 + 0.1 * row[0]
        x = -10.0 + 20.0 * row[1]
        z = -10.0 + 20.0 * row[2]
        m = row[3]
        col = (0.2 + 0.75 * row[4], 0.2 + 0.75 * row[5], 0.2 + 0.75 * row[6])
        mat = D if m < 0.80 else (reflection_type.specular if m < 0.95 else reflection_type.dielectric)
        scn.spheres.append(sphere(float(r), (float(x), float(r), float(z)), (0.0, 0.0, 0.0),
                                  tuple(float(c) for c in col), mat))
    c = scn.camera_parameters
    c.position = (0.0, 2.0, 12.0)
    c.direction = (0.0, 0.0, 0.0)
    return _finish(scn, w, h, 0.8, aperture=0.0)


SCENES = {"simple": simple_scene, "box": box_scene, "box_mirror": box_mirror_scene}

# ---- scene files (the reference hard-codes its scene,
# main.cpp:25,199-208).  Same format as host/pt/scene_file.hpp:
#   camera <pos x y z> <look-at x y z> <up x y z> <vfov radians> <aperture> <focus | auto>
#   sphere <radius> <pos x y z> <emission r g b> <colour r g b> <diffuse|specular|dielectric>
# '#' starts a comment; aspect ratio = w/h; "auto" focus = |pos - look-at|.
# Numbers are written with 17 significant digits: save -> load is exact.

_MATERIALS = {"diffuse": reflection_type.diffuse, "specular": reflection_type.specular,
              "dielectric": reflection_type.dielectric}


class SceneFileError(ValueError):
    pass


def parse_scene_text(text: str, w: int, h: int) -> scene:
    scn = scene()
    have_camera = False
    for lineno, raw in enumerate(text.splitlines(), 1):
        tok = raw.split("#", 1)[0].split()
        if not tok:
            continue

        def bad(why):
            return SceneFileError(f"line {lineno}: {why}")

        nnum = {"camera": 11, "sphere": 10}.get(tok[0])
        if nnum is None:
            raise bad(f"unknown item '{tok[0]}' (camera | sphere)")
        if len(tok) != nnum + 2:
            raise bad(f"{tok[0]} needs {nnum + 1} fields")
        try:
            v = [float(t) for t in tok[1:nnum + 1]]
        except ValueError as e:
            raise bad(f"not a number: {e}") from None
        if tok[0] == "camera":
            if have_camera:
                raise bad("second camera")
            have_camera = True
            c = scn.camera_parameters
            c.position, c.direction, c.up = tuple(v[0:3]), tuple(v[3:6]), tuple(v[6:9])
            c.vertical_fov_radians, c.aperture = v[9], v[10]
            c.aspect_ratio = (w * 1.0) / (h * 1.0)
            if tok[12] == "auto":
                c.focus_distance = length(_sub(c.position, c.direction))
            else:
                try:
                    c.focus_distance = float(tok[12])
                except ValueError:
                    raise bad("focus distance must be a number or 'auto'") from None
        else:
            if tok[11] not in _MATERIALS:
                raise bad("material must be diffuse, specular or dielectric")
            if not v[0] > 0.0:
                raise bad("radius must be positive")
            scn.spheres.append(sphere(v[0], tuple(v[1:4]), tuple(v[4:7]), tuple(v[7:10]), _MATERIALS[tok[11]]))
    if not have_camera:
        raise SceneFileError("no camera line")
    return scn


def load_scene_file(path: str, w: int, h: int) -> scene:
    with open(path) as f:
        return parse_scene_text(f.read(), w, h)


def scene_text(scn: scene) -> str:
    f = lambda x: "%.17g" % x  # noqa: E731
    v3 = lambda a: " ".join(f(x) for x in a)  # noqa: E731
    names = {0: "diffuse", 1: "specular", 2: "dielectric"}
    c = scn.camera_parameters
    out = ["# pt-scene: camera pos look-at up vfov aperture focus; sphere radius pos emission colour material",
           f"camera {v3(c.position)}  {v3(c.direction)}  {v3(c.up)}  {f(c.vertical_fov_radians)} "
           f"{f(c.aperture)} {f(c.focus_distance)}"]
    for s in scn.spheres:
        out.append(f"sphere {f(s.radius)}  {v3(s.position)}  {v3(s.emission)}  {v3(s.color)}  "
                   f"{names[int(s.reflection)]}")
    return "\n".join(out) + "\n"


def save_scene_file(scn: scene, path: str) -> None:
    with open(path, "w") as f:
        f.write(scene_text(scn))


def make_scene(name: str, w: int, h: int) -> scene:
    """A built-in scene (simple, box, box_mirror, synthetic[:N]) or a scene file."""
    if name.startswith("synthetic"):
        n = int(name.split(":")[1]) if ":" in name else 10000
        return synthetic_scene(n, w, h)
    if name in SCENES:
        return SCENES[name](w, h)
    return load_scene_file(name, w, h)
