"""Synthetic scenes, cameras and configs for the BASELINE.json configurations.

Host-side data generation only (no rendering).  Scene recipe conventions follow the reference demo
(src/main.ts:341-431): unit root octree at the origin, an enclosing matte BoxEntity added LAST
with max_in_depth 1 (src/main.ts:393,396), camera at (0.5,0.5,0.5) with init_h = pi/6
(src/main.ts:366), SkySphere(SolidTexture(0.2,0.2,0.7)) (src/main.ts:378).  Randomness is the
build's own splitmix64 stream (seeded), so every backend sees bit-identical inputs.
"""
import math
from dataclasses import dataclass, field

import numpy as np

from . import abi

SUBSTANCES = np.array([1.0, 1.333, 1.5])          # AIR, WATER, GLASS (src/substance.ts:9-11)
SUB_AIR = 0
SKY_RGB = (0.2, 0.2, 0.7)

# --- splitmix64 ---------------------------------------------------------------------------------
_GOLD = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64_uniform(seed, n, offset=0):
    """n uniforms in [0,1): the (offset+1)..(offset+n)-th outputs of splitmix64(seed), 53-bit."""
    with np.errstate(over="ignore"):
        k = np.arange(offset + 1, offset + n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * _GOLD
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


class Stream:
    def __init__(self, seed):
        self.seed, self.off = seed, 0

    def take(self, n):
        u = splitmix64_uniform(self.seed, n, self.off)
        self.off += n
        return u


# --- scene container ----------------------------------------------------------------------------
@dataclass
class SceneSpec:
    name: str
    entities: np.ndarray                     # abi.ENTITY_DTYPE, in add_entity_to_octree call order
    shades: np.ndarray                       # abi.SHADE_DTYPE
    substances: np.ndarray = field(default_factory=lambda: SUBSTANCES.copy())
    root_pos: tuple = (0.0, 0.0, 0.0)
    root_size: float = 1.0
    images: list = field(default_factory=list)   # ImageTextures, [H, W, 3] uint8 (rt_shade.image = k + 1)


def _shade(response=abi.RT_RESP_REFLECTION, light=0, mirror=0, rgb=(1, 1, 1), roughness=0.0):
    s = np.zeros(1, abi.SHADE_DTYPE)
    s["response"], s["light"], s["mirror"], s["roughness"] = response, light, mirror, roughness
    s["rgb"][0] = rgb
    return s


def _entities(n):
    e = np.zeros(n, abi.ENTITY_DTYPE)
    e["substance"] = SUB_AIR
    return e


def room_box():
    """scene_box: BoxEntity(pos (0.5,0.5,0.5), size 1), matte-terminal grey, added last with
    max_in_depth 1, max_out_depth 0 (src/main.ts:393,396)."""
    e = _entities(1)
    e["type"] = abi.RT_ENT_BOX
    e["geom"][0, :4] = (0.5, 0.5, 0.5, 1.0)
    e["max_in_depth"], e["max_out_depth"] = 1, 0
    return e, _shade(rgb=(0.5, 0.5, 0.5))


def _concat(parts_e, parts_s):
    """Concatenate entity/shade groups, re-basing shade indices."""
    ents, shades, base = [], [], 0
    for e, s in zip(parts_e, parts_s):
        e = e.copy()
        e["shade"] += base
        ents.append(e)
        shades.append(s)
        base += len(s)
    return np.concatenate(ents), np.concatenate(shades)


def _materials(st, n, p_mirror, p_light):
    """Per-entity (material, texture) shades: matte albedo U[0.2,1]^3, mirror tint U[0.5,1]^3,
    light = normalised random colour x 5 (get_random_color_with_intensity, src/main.ts:62-66)."""
    u = st.take(n * 4).reshape(n, 4)
    kind = np.where(u[:, 0] < p_light, 2, np.where(u[:, 0] < p_light + p_mirror, 1, 0))
    s = np.zeros(n, abi.SHADE_DTYPE)
    s["response"] = abi.RT_RESP_REFLECTION
    s["mirror"] = (kind == 1).astype(np.int32)
    s["light"] = (kind == 2).astype(np.int32)
    rgb = np.empty((n, 3))
    matte = 0.2 + 0.8 * u[:, 1:4]
    tint = 0.5 + 0.5 * u[:, 1:4]
    lc = u[:, 1:4] + 1e-3
    lc = lc / np.sqrt((lc * lc).sum(1, keepdims=True)) * 5.0
    rgb[kind == 0] = matte[kind == 0]
    rgb[kind == 1] = tint[kind == 1]
    rgb[kind == 2] = lc[kind == 2]
    s["rgb"] = rgb
    return s


def config1_spheres():
    """Config 1: 8 spheres at the octant centres (0.25/0.75)^3, diameter 0.3, materials cycling
    matte/mirror/light, max_in_depth 3 + the room box."""
    e = _entities(8)
    s = np.zeros(8, abi.SHADE_DTYPE)
    for k in range(8):
        c = [0.25 + 0.5 * ((k >> i) & 1) for i in range(3)]
        e[k]["type"] = abi.RT_ENT_SPHERE
        e[k]["geom"][:4] = (*c, 0.3)
        e[k]["max_in_depth"], e[k]["max_out_depth"] = 3, 0
        e[k]["shade"] = k
        kind = k % 3
        s[k] = _shade(mirror=int(kind == 1), light=int(kind == 2),
                      rgb=[(0.9, 0.3, 0.2), (0.8, 0.9, 1.0), (5.0, 4.0, 3.0)][kind])[0]
    rb, rs = room_box()
    ents, shades = _concat([e, rb], [s, rs])
    return SceneSpec("config1_8spheres", ents, shades)


def roughen(spec, values=(0.05, 0.3, 0.8)):
    """Copy of `spec` with roughness_index > 0 on every mirror shade, cycling through `values`
    (rough mirrors: Ray.scatter_ray, src/raytracer.ts:121-133,233-235)."""
    sh = spec.shades.copy()
    idx = np.nonzero(sh["mirror"])[0]
    for k, i in enumerate(idx):
        sh["roughness"][i] = values[k % len(values)]
    return SceneSpec(spec.name + "_rough", spec.entities, sh, spec.substances, spec.root_pos, spec.root_size,
                     list(spec.images))


def test_image(w, h, seed):
    """A deterministic RGB image with sharp texel edges: a checkerboard over smooth gradients."""
    u = Stream(seed).take(3)
    y, x = np.mgrid[0:h, 0:w]
    chk = ((x // max(1, w // 8) + y // max(1, h // 6)) & 1) * 96
    img = np.stack([(x * 255 // max(1, w - 1) + chk) % 256, (y * 255 // max(1, h - 1) + 64 * u[0]) % 256,
                    (chk + 128 * u[1] + 37 * x * y) % 256], axis=-1)
    return img.astype(np.uint8)


def texture(spec, images, every=2, sky=False):
    """Copy of `spec` with ImageTextures: every `every`-th shade (lights excluded) samples one of
    `images` instead of its SolidTexture colour (ImageTexture.get_color at entity.map_uv)."""
    sh = spec.shades.copy()
    imgs = list(spec.images) + list(images)
    base = len(spec.images)
    for i in range(len(sh)):
        if i % every == 0 and not sh["light"][i]:
            sh["image"][i] = base + 1 + (i // every) % len(images)
    return SceneSpec(spec.name + "_tex", spec.entities, sh, spec.substances, spec.root_pos, spec.root_size, imgs)


def random_triangles(st, n, half_extent, lo=0.02, hi=0.98, max_in_depth=6):
    c = lo + (hi - lo) * st.take(n * 3).reshape(n, 3)
    off = (st.take(n * 9).reshape(n, 3, 3) * 2 - 1) * half_extent
    v = c[:, None, :] + off
    e = _entities(n)
    e["type"] = abi.RT_ENT_FACE
    e["geom"] = v.reshape(n, 9)
    e["max_in_depth"], e["max_out_depth"] = max_in_depth, 0
    return e


def random_spheres(st, n, dmin, dmax, lo=0.02, hi=0.98, max_in_depth=6):
    c = lo + (hi - lo) * st.take(n * 3).reshape(n, 3)
    d = dmin + (dmax - dmin) * st.take(n)
    e = _entities(n)
    e["type"] = abi.RT_ENT_SPHERE
    e["geom"][:, :3] = c
    e["geom"][:, 3] = d
    e["max_in_depth"], e["max_out_depth"] = max_in_depth, 0
    return e


def tri_scene(n_tri, half_extent, max_in_depth, n_sph=0, p_mirror=0.0, p_light=0.0, seed=42, name=None):
    st = Stream(seed)
    tri = random_triangles(st, n_tri, half_extent, max_in_depth=max_in_depth)
    parts_e, parts_s = [tri], []
    if n_sph:
        parts_e.append(random_spheres(st, n_sph, 0.002, 0.01, max_in_depth=max_in_depth))
    ents = np.concatenate(parts_e)
    ents["shade"] = np.arange(len(ents))
    shades = _materials(st, len(ents), p_mirror, p_light)
    rb, rs = room_box()
    ents, shades = _concat([ents, rb], [shades, rs])
    return SceneSpec(name or "tri%d" % n_tri, ents, shades)


def config2():
    """Config 2: 10k random triangles (centre U[0.02,0.98]^3, vertices +U[-0.003,0.003]^3), depth 6."""
    return tri_scene(10_000, 0.003, 6, p_mirror=0.25, p_light=0.05, name="config2_10k_tri")


def config3():
    """Config 3 (north star): 100k triangles (half-extent 0.001) + 1k spheres (d U[0.002,0.01]),
    depth 8, materials ~70% matte / 25% mirror / 5% light."""
    return tri_scene(100_000, 0.001, 8, n_sph=1000, p_mirror=0.25, p_light=0.05, name="config3_100k_tri_1k_sph")


def small_random(seed, n_tri=200, n_sph=40, n_box=10, depth=5, p_mirror=0.3, p_light=0.1, half=0.02):
    """Small mixed scenes for parity sweeps (all three primitive kinds, mirrors, lights)."""
    st = Stream(seed)
    # a triangle's cubic AABB is [min corner, min corner + max extent]: keep centre + 3*half inside
    tri = random_triangles(st, n_tri, half, lo=half + 0.01, hi=1 - 3 * half - 0.01, max_in_depth=depth)
    sph = random_spheres(st, n_sph, 0.01, 0.12, lo=0.15, hi=0.85, max_in_depth=depth)
    box = _entities(n_box)
    box["type"] = abi.RT_ENT_BOX
    box["geom"][:, :3] = 0.1 + 0.8 * st.take(n_box * 3).reshape(n_box, 3)
    box["geom"][:, 3] = 0.02 + 0.1 * st.take(n_box)
    box["max_in_depth"] = depth
    ents = np.concatenate([tri, sph, box])
    perm = np.argsort(st.take(len(ents)), kind="stable")       # interleave kinds in set order
    ents = ents[perm]
    ents["shade"] = np.arange(len(ents))
    shades = _materials(st, len(ents), p_mirror, p_light)
    rb, rs = room_box()
    ents, shades = _concat([ents, rb], [shades, rs])
    return SceneSpec("small%d" % seed, ents, shades)


def config5(n_tri=1_000_000, n_sph=2000, seed=42):
    """Config 5: 1M triangles (half-extent 0.0003) + spheres (d U[0.002,0.01]) + 16 large spheres
    (8 glass, 8 mirrors; d U[0.08,0.2]), depth 10, refmax 5.
    Materials ~70% matte / 25% mirror / 5% light; every third small sphere and 8 large ones are GLASS
    with a TRANSMISSION material (refract_ray + entity_at_pos, src/raytracer.ts:135-150,238-249;
    src/octree_entity.ts:191-202).  "Shadow rays" in BASELINE's wording have no counterpart in the
    reference's Ray.trace (src/raytracer.ts:168-277 never samples lights): they are a build
    extension, off unless lights are set (rt_set_lights; bench.py --lights K)."""
    st = Stream(seed)
    tri = random_triangles(st, n_tri, 0.0003, max_in_depth=10)
    sph = random_spheres(st, n_sph, 0.002, 0.01, max_in_depth=10)
    big = random_spheres(st, 16, 0.08, 0.2, lo=0.15, hi=0.85, max_in_depth=10)   # multi-bounce paths
    ents = np.concatenate([tri, sph, big])
    ents["shade"] = np.arange(len(ents))
    shades = _materials(st, len(ents), 0.25, 0.05)
    nb = n_tri + n_sph
    shades["mirror"][nb + 8:], shades["light"][nb + 8:] = 1, 0
    shades["rgb"][nb + 8:] = 0.9
    glass = np.concatenate([n_tri + np.arange(0, n_sph, 3), nb + np.arange(8)])
    shades["response"][glass] = abi.RT_RESP_TRANSMISSION
    shades["mirror"][glass] = 0
    shades["light"][glass] = 0
    shades["rgb"][glass] = 0.9 + 0.1 * st.take(len(glass) * 3).reshape(-1, 3)
    ents["substance"][glass] = 2                                 # GLASS (src/substance.ts:11)
    rb, rs = room_box()
    ents, shades = _concat([ents, rb], [shades, rs])
    return SceneSpec("config5_1m_tri_%d_sph_glass" % n_sph, ents, shades)


SCENES = {"config1": config1_spheres, "config2": config2, "config3": config3, "config5": config5}


# --- camera (src/view/camera.ts:61-145) ----------------------------------------------------------
def _rot_pair(bx, by, rot):
    c, s = rot
    return ([bx[i] * c + by[i] * s for i in range(3)], [bx[i] * -s + by[i] * c for i in range(3)])


def make_camera(width, height, pos=(0.5, 0.5, 0.5), init_v=0.0, init_h=math.pi / 6,
                fov_h=math.pi / 2, fov_v=None, vertical_locked=True):
    """Camera(conf, init_pos, init_v_angle, init_h_angle) state → rt_camera_desc."""
    if fov_v is None:
        fov_v = math.pi / 2 * height / width
    fr, lf, up = [1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]
    scan_h = (math.cos(fov_h / width), math.sin(fov_h / width))
    scan_v = (math.cos(fov_v / height), math.sin(fov_v / height))
    if init_h is not None:                                   # rotate_h → rotate_h_v (:121-130)
        v = (math.cos(init_h), math.sin(init_h))

        def rot2(a):
            o = (-a[1], a[0])                                 # vector.ortho
            return [a[0] * v[0] + o[0] * v[1], a[1] * v[0] + o[1] * v[1]]
        f2, l2 = rot2(fr[:2]), rot2(lf[:2])
        fr, lf = [f2[0], f2[1], fr[2]], [l2[0], l2[1], lf[2]]
        up = [fr[1] * lf[2] - fr[2] * lf[1], fr[2] * lf[0] - fr[0] * lf[2], fr[0] * lf[1] - fr[1] * lf[0]]
    if init_v is not None:                                   # rotate_v → rotate_v_v (:134-145)
        v = (math.cos(init_v), math.sin(init_v))
        cmp_sign = 1 if v[1] < 0 else -1
        nfr, nup = _rot_pair(fr, up, v)
        dz = nfr[2] - fr[2]
        sgn = (dz > 0) - (dz < 0)
        if not (vertical_locked and sgn == cmp_sign):
            fr, up = nfr, nup
    cam = abi.rt_camera_desc()
    cam.width, cam.height = int(width), int(height)
    cam.pos[:] = [float(x) for x in pos]
    cam.fr[:], cam.lf[:], cam.up[:] = fr, lf, up
    cam.scan_h[:], cam.scan_v[:] = scan_h, scan_v
    return cam


def make_config(refmax, sky=SKY_RGB, atten=1.0, default_substance=SUB_AIR, col_weight=1.0, scatter_seed=None,
                sky_image=0):
    """scatter_seed: None = RT_SCATTER_REJECT (rough mirrors unsupported), else RT_SCATTER_COUNTER.
    sky_image: 0 = SkySphere(SolidTexture(sky)), k = SkySphere of the scene's image k-1."""
    c = abi.rt_config_desc()
    c.refmax = int(refmax)
    c.default_substance = int(default_substance)
    c.sky_rgb[:] = [float(x) for x in sky]
    c.distance_attenuation_factor = float(atten)
    c.col_weight = float(col_weight)
    c.scatter_mode = abi.RT_SCATTER_REJECT if scatter_seed is None else abi.RT_SCATTER_COUNTER
    c.scatter_seed = 0 if scatter_seed is None else int(scatter_seed) & (2 ** 64 - 1)
    c.sky_image = int(sky_image)
    return c


def reseat_throw_scene(textured=False, width=64, height=48):
    """A light whose hit point makes the post-light re-seat throw (src/raytracer.ts:276).

    Non-dyadic root [-2, 1)^3 (size 3).  The light is a box in the root's Set whose +x face is at
    x = 1 - 2^-53; the camera sits outside the root at (1.5, 0.5, 0.5) looking down -x, so the walker
    returns only the root (src/octree_space.ts:254-277, 283-286) and rays hit the light's +x face.
    There node_at_pos computes (x + 2)·(2/3) = 2 (rounded) and y, z in the upper halves: Octree.get(8)
    throws.  The centre ray misses the light and hits a matte sphere, so the scan's first throw comes
    after some pixels are final.  Returns (spec, camera)."""
    e = _entities(2)
    e["type"] = (abi.RT_ENT_BOX, abi.RT_ENT_SPHERE)
    e["geom"][0, :4] = (0.8999999999999998, 0.8, 0.5, 0.2)
    e["geom"][1, :4] = (0.2, 0.2, 0.6, 0.3)
    e["shade"] = 0, 1
    e["max_in_depth"], e["max_out_depth"] = 0, 0
    sh = np.concatenate([_shade(light=1, rgb=(5, 4, 3)), _shade(rgb=(0.3, 0.6, 0.9))])
    images = []
    if textured:
        sh["image"][0] = 1
        images = [test_image(5, 3, 11)]
    spec = SceneSpec("reseat_throw" + ("_tex" if textured else ""), e, sh, root_pos=(-2.0, -2.0, -2.0),
                     root_size=3.0, images=images)
    cam = make_camera(width, height, pos=(1.5, 0.5, 0.5), init_h=None, init_v=None)
    cam.fr[:], cam.lf[:], cam.up[:] = [-1.0, 0.0, 0.0], [0.0, -1.0, 0.0], [0.0, 0.0, 1.0]
    return spec, cam


# Workloads named in BASELINE.json configs: (scene factory, width, height, refmax)
WORKLOADS = {
    "config1": (config1_spheres, 256, 256, 2),
    "config2": (config2, 1920, 1080, 1),
    "config3": (config3, 1920, 1080, 2),
    "config4": (config3, 3840, 2160, 2),      # the 8-GPU tile-split configuration (any N runs it)
    "config5": (config5, 3840, 2160, 5),
}
