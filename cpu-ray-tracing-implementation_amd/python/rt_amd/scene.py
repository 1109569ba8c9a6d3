"""Python-side scene assembly onto the C ABI's rt_scene_desc.

Mirrors the constructors of the reference's hittables/materials/textures
(sphere.h, quad.h, triangle.h, hittable.h, hittable_list.h, bvh_node.h,
volumne.h, material.h, texture.h) so tests can build arbitrary scenes. The
production caller is the C++ plugin surface in ../../rt/ (camera::render).
"""
import ctypes
import math

import numpy as np

from . import abi


class SceneBuilder:
    def __init__(self, rand=None):
        """rand: the uniform [0,1) source procedural textures draw their tables from (the
        reference's random_double, utility.h:20); default: glibc rand(), as the reference."""
        self.objects, self.children, self.materials, self.textures = [], [], [], []
        self.tex_data = []
        if rand is None:
            import ctypes
            libc = ctypes.CDLL(None)
            libc.rand.restype = ctypes.c_int
            rand = lambda: libc.rand() / (2147483647 + 1.0)
        self._rand = rand

    # textures (texture.h:12-63)
    def solid(self, color):
        t = abi.rt_texture(kind=abi.RT_TEX_SOLID)
        t.color[:] = [float(c) for c in color]
        self.textures.append(t)
        return len(self.textures) - 1

    def checker(self, odd, even, scale):
        t = abi.rt_texture(kind=abi.RT_TEX_CHECKER, scale=float(scale))
        t.odd[:] = [float(c) for c in odd]
        t.even[:] = [float(c) for c in even]
        self.textures.append(t)
        return len(self.textures) - 1

    # procedural textures (texture.h:80-119, noise.h): tables drawn as the constructors draw them
    def _emit_data(self, values):
        off = len(self.tex_data)
        self.tex_data.extend(float(v) for v in values)
        return off

    def perlin(self, scale):
        rd = self._rand
        offsets = []
        for _ in range(256):  # unit_vector(random_vec(-1, 1)): GCC evaluates vec3(...) right to left
            z, y, x = (-1 + 2 * rd() for _ in range(3))
            n = math.sqrt(x * x + y * y + z * z)
            offsets += [x / n, y / n, z / n]
        perms = []
        for _ in range(3):  # perm_x, perm_y, perm_z: Fisher-Yates with random_int(0, i) (noise.h:82-97)
            p = list(range(256))
            for i in range(255, 0, -1):
                t = int(0 + (i - 0) * rd())
                p[i], p[t] = p[t], p[i]
            perms += p
        t = abi.rt_texture(kind=abi.RT_TEX_PERLIN, scale=float(scale), data=self._emit_data(offsets + perms))
        self.textures.append(t)
        return len(self.textures) - 1

    def value(self, resolution):
        rd = self._rand
        vals = [float(np.float32(rd())) for _ in range(resolution ** 3)]  # std::vector<float> (noise.h:135)
        t = abi.rt_texture(kind=abi.RT_TEX_VALUE, scale=float(resolution), data=self._emit_data(vals))
        self.textures.append(t)
        return len(self.textures) - 1

    def image(self, linear_rgb):
        """picture_texture (texture.h:65-78) over linear RGB floats (H, W, 3), row 0 at the top,
        stored as bytes with image.h's float_to_byte. An empty array samples as magenta."""
        a = np.asarray(linear_rgb, dtype=np.float32)
        h, w = (a.shape[0], a.shape[1]) if a.size else (0, 0)
        b = np.where(a <= 0, 0, np.where(a >= 1, 255, np.floor(256.0 * a.astype(np.float64)))).astype(np.uint8)
        off = len(getattr(self, "image_data", b""))
        self.image_data = getattr(self, "image_data", b"") + b.tobytes()
        t = abi.rt_texture(kind=abi.RT_TEX_IMAGE, data=off)
        t.color[0], t.color[1] = float(w), float(h)
        self.textures.append(t)
        return len(self.textures) - 1

    def worley(self):
        self.textures.append(abi.rt_texture(kind=abi.RT_TEX_WORLEY))
        return len(self.textures) - 1

    def voronoi(self):
        self.textures.append(abi.rt_texture(kind=abi.RT_TEX_VORONOI))
        return len(self.textures) - 1

    # materials (material.h)
    def _mat(self, kind, tex, fuzz=0.0, refraction=1.0, smoothness=0.0, specular_prob=0.0):
        self.materials.append(abi.rt_material(kind=kind, texture=tex, fuzz=fuzz, refraction=refraction,
                                              smoothness=smoothness, specular_prob=specular_prob))
        return len(self.materials) - 1

    def lambertian(self, tex):
        return self._mat(abi.RT_MAT_LAMBERTIAN, tex)

    def metal(self, tex, fuzz=0.0):  # fuzz clamped to [0,1] (material.h:80-82)
        return self._mat(abi.RT_MAT_METAL, tex, fuzz=min(1.0, max(0.0, fuzz)))

    def dielectric(self, tex, refraction):
        return self._mat(abi.RT_MAT_DIELECTRIC, tex, refraction=refraction)

    def isotropic(self, tex):
        return self._mat(abi.RT_MAT_ISOTROPIC, tex)

    def diffuse_light(self, tex):
        return self._mat(abi.RT_MAT_DIFFUSE_LIGHT, tex)

    def gloss(self, tex, smoothness, specular_prob):  # material.h:145-155 (smoothness clamped on compile)
        return self._mat(abi.RT_MAT_GLOSS, tex, smoothness=smoothness, specular_prob=specular_prob)

    # hittables
    def _obj(self, **kw):
        o = abi.rt_object(material=-1, child=-1, first_child=0, child_count=0)
        for k, v in kw.items():
            if k in ("a", "b", "c"):
                getattr(o, k)[:] = [float(x) for x in v]
            else:
                setattr(o, k, v)
        self.objects.append(o)
        return len(self.objects) - 1

    def sphere(self, center, radius, mat):
        return self._obj(kind=abi.RT_OBJ_SPHERE, a=center, s0=float(radius), material=mat)

    def moving_sphere(self, c1, c2, radius, mat):
        return self._obj(kind=abi.RT_OBJ_SPHERE, a=c1, b=c2, s0=float(radius), material=mat, moving=1)

    def quad(self, q, u, v, mat):
        return self._obj(kind=abi.RT_OBJ_QUAD, a=q, b=u, c=v, material=mat)

    def triangle(self, p0, p1, p2, mat):
        return self._obj(kind=abi.RT_OBJ_TRIANGLE, a=p0, b=p1, c=p2, material=mat)

    def _group(self, kind, members):
        first = len(self.children)
        self.children.extend(members)
        return self._obj(kind=kind, first_child=first, child_count=len(members))

    def hlist(self, members):
        return self._group(abi.RT_OBJ_LIST, list(members))

    def bvh(self, members):
        return self._group(abi.RT_OBJ_BVH, list(members))

    def translate(self, obj, offset):
        return self._obj(kind=abi.RT_OBJ_TRANSLATE, child=obj, a=offset)

    def rotate(self, axis, obj, degrees):  # hittable.h:95-98 sin/cos of degrees_to_radians
        rad = degrees * math.pi / 180.0
        kind = {0: abi.RT_OBJ_ROTATE_X, 1: abi.RT_OBJ_ROTATE_Y, 2: abi.RT_OBJ_ROTATE_Z}[axis]
        return self._obj(kind=kind, child=obj, s0=math.sin(rad), s1=math.cos(rad))

    def volume(self, boundary, density, tex):  # volumne.h:11-15 makes an isotropic phase function
        return self._obj(kind=abi.RT_OBJ_VOLUME, child=boundary, s0=float(density), material=self.isotropic(tex))

    def box_members(self, a, b, mat):  # quad.h:91-112
        mn = [min(a[i], b[i]) for i in range(3)]
        mx = [max(a[i], b[i]) for i in range(3)]
        dx, dy, dz = (mx[0] - mn[0], 0, 0), (0, mx[1] - mn[1], 0), (0, 0, mx[2] - mn[2])
        neg = lambda v: tuple(-x for x in v)
        return [self.quad((mn[0], mn[1], mx[2]), dy, dx, mat), self.quad((mx[0], mn[1], mx[2]), dy, neg(dz), mat),
                self.quad((mx[0], mn[1], mn[2]), dy, neg(dx), mat), self.quad((mn[0], mn[1], mn[2]), dy, dz, mat),
                self.quad((mn[0], mx[1], mx[2]), neg(dz), dx, mat), self.quad((mn[0], mn[1], mn[2]), dz, dx, mat)]

    def box(self, a, b, mat):
        return self.hlist(self.box_members(a, b, mat))

    def desc(self, world, light=-1, background=-1):
        """The rt_scene_desc; the returned object keeps the arrays alive."""
        d = abi.rt_scene_desc()
        self._keep = (
            (abi.rt_object * max(1, len(self.objects)))(*self.objects),
            (abi.c_int32 * max(1, len(self.children)))(*self.children),
            (abi.rt_material * max(1, len(self.materials)))(*self.materials),
            (abi.rt_texture * max(1, len(self.textures)))(*self.textures),
            (abi.c_double * max(1, len(self.tex_data)))(*self.tex_data),
            (ctypes.c_uint8 * max(1, len(getattr(self, "image_data", b""))))(*getattr(self, "image_data", b"")),
        )
        d.objects, d.children, d.materials, d.textures, d.tex_data, d.image_data = self._keep
        d.num_tex_data = len(self.tex_data)
        d.num_image_data = len(getattr(self, "image_data", b""))
        d.num_objects, d.num_children = len(self.objects), len(self.children)
        d.num_materials, d.num_textures = len(self.materials), len(self.textures)
        d.world, d.light, d.background = world, light, background
        d._owner = self
        return d


def perspective(image_width, aspect, pos, lookat, focal_length=1.0, fovy_degree=90.0):
    """camera::initialize_perspective (camera.h:21-50), including its float-typed fovy/theta/focal."""
    pos, lookat = np.asarray(pos, float), np.asarray(lookat, float)
    unit = lambda v: v / math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    cross = lambda a, b: np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])
    d = unit(lookat - pos)
    right = unit(cross(d, np.array([0.0, 1.0, 0.0])))
    up = cross(right, d)
    focal = float(np.float32(focal_length))
    h = max(1, int(image_width / aspect))
    theta = float(np.float32(float(np.float32(fovy_degree)) * math.pi / 180.0))
    vh = 2.0 * math.tan(theta / 2.0) * focal
    vw = vh * (float(image_width) / h)
    c = abi.rt_camera_desc(mode=abi.RT_CAM_PERSPECTIVE, image_width=image_width, image_height=h,
                           viewport_width=vw, viewport_height=vh, focal_length=focal, focus_dist=3.4)
    c.pos[:], c.dir[:], c.right[:], c.up[:] = list(pos), list(d), list(right), list(up)
    return c


def _frame(pos, lookat):
    """camera.h:23-28: dir, right, up from pos and lookat with world up (0, 1, 0)."""
    pos, lookat = np.asarray(pos, float), np.asarray(lookat, float)
    unit = lambda v: v / math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    cross = lambda a, b: np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]])
    d = unit(lookat - pos)
    right = unit(cross(d, np.array([0.0, 1.0, 0.0])))
    return pos, d, right, cross(right, d)


def _desc(mode, image_width, h, pos, d, right, up, vw, vh, focal=1.0, focus=3.4, du=(0, 0, 0), dv=(0, 0, 0)):
    c = abi.rt_camera_desc(mode=mode, image_width=image_width, image_height=h, viewport_width=vw,
                           viewport_height=vh, focal_length=focal, focus_dist=focus)
    c.pos[:], c.dir[:], c.right[:], c.up[:] = list(pos), list(d), list(right), list(up)
    c.defocus_u[:], c.defocus_v[:] = list(du), list(dv)
    return c


def orthonormal(image_width, aspect, viewport_height, pos, lookat):
    """camera::initialize_orthnormal (camera.h:52-72)."""
    pos, d, right, up = _frame(pos, lookat)
    h = max(1, int(image_width / aspect))
    return _desc(abi.RT_CAM_ORTHONORMAL, image_width, h, pos, d, right, up,
                 viewport_height * (float(image_width) / h), viewport_height)


def fisheye(image_width, aspect, pos, lookat, focal_length=1.0, fovy_degree=90.0):
    """camera::initialize_fisheye (camera.h:74-100): the perspective frame, fisheye ray mapping."""
    c = perspective(image_width, aspect, pos, lookat, focal_length, fovy_degree)
    c.mode = abi.RT_CAM_FISHEYE
    return c


def lens(image_width, aspect, pos, lookat, defocus_angle, focus_dist=1.0, fovy_degree=90.0):
    """camera::initialize_lens (camera.h:102-132): float aspect ratio, float angles and focus distance."""
    pos, d, right, up = _frame(pos, lookat)
    f32 = np.float32
    h = max(1, int(f32(image_width) / f32(aspect)))  # int / float is a float division
    focus = float(f32(focus_dist))
    theta = float(f32(float(f32(fovy_degree)) * math.pi / 180.0))
    vh = 2.0 * math.tan(theta / 2.0) * focus
    vw = vh * (float(image_width) / h)
    r = focus * math.tan(float(f32(defocus_angle) / f32(2)) * math.pi / 180.0)
    return _desc(abi.RT_CAM_LENS, image_width, h, pos, d, right, up, vw, vh, 1.0, focus, right * r, up * r)
