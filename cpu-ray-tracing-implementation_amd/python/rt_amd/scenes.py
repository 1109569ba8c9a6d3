"""The reference's main.cc scenes used by the BASELINE configs, built on SceneBuilder.

Random draws use glibc rand() (utility.h:20) in the order GCC evaluates the
reference's expressions; scenes that draw call srand(1) first, as the
reference's main() implicitly does.
"""
import ctypes
import math

from .scene import SceneBuilder, fisheye, lens, orthonormal, perspective

_libc = ctypes.CDLL(None)
_libc.rand.restype = ctypes.c_int


def _rnd():
    return _libc.rand() / (2147483647 + 1.0)


def cornell_box(width=600, aspect=1.0):  # main.cc:198-225
    s = SceneBuilder()
    red = s.lambertian(s.solid((.65, .05, .05)))
    white = s.lambertian(s.solid((0.73, 0.73, 0.73)))
    green = s.lambertian(s.solid((.12, .45, .15)))
    light = s.diffuse_light(s.solid((15, 15, 15)))
    w = [s.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green), s.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red),
         s.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white),
         s.quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white),
         s.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white)]
    w.append(s.translate(s.box((0, 0, 0), (165, 330, 165), white), (100, 0, 200)))
    w.append(s.translate(s.box((0, 0, 0), (165, 165, 165), white), (50, 0, 100)))
    lq = s.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light)
    w.append(lq)
    world = s.bvh(w)
    cam = perspective(width, aspect, (278, 278, -800), (278, 278, 0), 1, 40.0)
    return s.desc(world, light=lq, background=s.solid((0, 0, 0))), cam, 40, 4


def cornell_triangles(width=600, aspect=1.0):
    """cornell_box with every wall/box quad split into triangles (q, q+u, q+v), (q+u+v, q+v, q+u):
    exercises triangle.h on the main.cc Cornell scene (the oracle builds the same)."""
    s = SceneBuilder()
    red = s.lambertian(s.solid((.65, .05, .05)))
    white = s.lambertian(s.solid((0.73, 0.73, 0.73)))
    green = s.lambertian(s.solid((.12, .45, .15)))
    light = s.diffuse_light(s.solid((15, 15, 15)))
    add = lambda v, w: tuple(a + b for a, b in zip(v, w))

    def tris(q, u, v, m):
        return [s.triangle(q, add(q, u), add(q, v), m), s.triangle(add(add(q, u), v), add(q, v), add(q, u), m)]

    def box(a, b, m):
        dx, dy, dz = (b[0] - a[0], 0, 0), (0, b[1] - a[1], 0), (0, 0, b[2] - a[2])
        neg = lambda v: tuple(-x for x in v)
        out = []
        for q, u, v in [((a[0], a[1], b[2]), dy, dx), ((b[0], a[1], b[2]), dy, neg(dz)), ((b[0], a[1], a[2]), dy, neg(dx)),
                        ((a[0], a[1], a[2]), dy, dz), ((a[0], b[1], b[2]), neg(dz), dx), ((a[0], a[1], a[2]), dz, dx)]:
            out += tris(q, u, v, m)
        return s.hlist(out)

    w = (tris((555, 0, 0), (0, 555, 0), (0, 0, 555), green) + tris((0, 0, 0), (0, 555, 0), (0, 0, 555), red) +
         tris((0, 0, 0), (555, 0, 0), (0, 0, 555), white) + tris((555, 555, 555), (-555, 0, 0), (0, 0, -555), white) +
         tris((0, 0, 555), (555, 0, 0), (0, 555, 0), white))
    w.append(s.translate(box((0, 0, 0), (165, 330, 165), white), (100, 0, 200)))
    w.append(s.translate(box((0, 0, 0), (165, 165, 165), white), (50, 0, 100)))
    lq = s.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light)  # the light stays a quad (importance-sampled)
    w.append(lq)
    world = s.bvh(w)
    cam = perspective(width, aspect, (278, 278, -800), (278, 278, 0), 1, 40.0)
    return s.desc(world, light=lq, background=s.solid((0, 0, 0))), cam, 40, 4


def cornell_box_with_volume(width=600, aspect=1.0):  # main.cc:227-253
    s = SceneBuilder()
    red = s.lambertian(s.solid((.65, .05, .05)))
    white = s.lambertian(s.solid((.73, .73, .73)))
    green = s.lambertian(s.solid((.12, .45, .15)))
    light = s.diffuse_light(s.solid((7, 7, 7)))
    w = [s.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green), s.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red),
         s.quad((0, 555, 0), (555, 0, 0), (0, 0, 555), white), s.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white),
         s.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white)]
    b1 = s.translate(s.rotate(1, s.box((0, 0, 0), (150, 280, 150), white), 45), (265, 0, 285))
    b2 = s.translate(s.rotate(1, s.box((0, 0, 0), (140, 140, 140), white), -15), (130, 0, 65))
    w.append(s.volume(b1, 0.02, s.solid((0, 0, 0))))
    w.append(s.volume(b2, 0.02, s.solid((1, 1, 1))))
    lq = s.quad((113, 554, 127), (330, 0, 0), (0, 0, 305), light)
    w.append(lq)
    world = s.hlist(w)
    cam = perspective(width, aspect, (278, 278, -800), (278, 278, 0), 1, 40)
    return s.desc(world, light=lq, background=s.solid((0, 0, 0))), cam, 100, 5


def rtow(width=1280, aspect=16.0 / 9.0, moving=False):  # main.cc:105-153
    _libc.srand(1)
    s = SceneBuilder()
    ground = s.lambertian(s.checker((1.0, 1.0, 1.0), (0.6, 0.6, 0.2), 1.0))
    w = [s.sphere((0, -1000, 0), 1000, ground)]
    for a in range(-11, 11):
        for b in range(-11, 11):
            choose = _rnd()
            rz = _rnd()  # center1(a + .7*rd(), .2, b + .7*rd()): GCC evaluates z first
            rx = _rnd()
            c1 = (a + 0.7 * rx, 0.2, b + 0.7 * rz)
            c2 = (c1[0], c1[1] + (0 + (.15 - 0) * _rnd()), c1[2])
            if math.sqrt((c1[0] - 4) ** 2 + (c1[1] - 0.2) ** 2 + c1[2] ** 2) <= 0.9 or choose < 0.3:
                continue
            if choose < 0.8:
                bz, by, bx = _rnd(), _rnd(), _rnd()
                az, ay, ax = _rnd(), _rnd(), _rnd()
                m = s.lambertian(s.solid((ax * bx, ay * by, az * bz)))
            elif choose < 0.95:
                z, y, x = (0.5 + (1 - 0.5) * _rnd() for _ in range(3))
                m = s.metal(s.solid((x, y, z)), 0.0)
            else:
                m = s.dielectric(s.solid((1, 1, 1)), 1.5)
            w.append(s.moving_sphere(c1, c2, 0.2, m) if moving else s.sphere(c1, 0.2, m))
    glass = s.dielectric(s.solid((1, 1, 1)), 1.5)
    matte = s.lambertian(s.solid((0.4, 0.2, 0.1)))
    w += [s.sphere((0, 1, 0), 1.0, glass), s.sphere((-4, 1, 0), 1.0, matte), s.sphere((4, 1, 0), 1.0, glass)]
    world = s.bvh(w)
    cam = perspective(width, aspect, (13, 2, 3), (0, 0, 0), 1, 20)
    return s.desc(world, background=s.solid((0.7, 0.8, 1.0))), cam, 20, 50


def three_material_ball(width=1280, aspect=16.0 / 9.0):  # main.cc:67-84
    s = SceneBuilder()
    ground = s.lambertian(s.checker((1.0, 1.0, 1.0), (0.6, 0.6, 0.2), 1.0))
    glass = s.dielectric(s.solid((1.0, 1.0, 1.0)), 1.5)
    matte = s.lambertian(s.solid((0.4, 0.2, 0.1)))
    metal = s.metal(s.solid((0.7, 0.6, 0.5)), 0.0)
    world = s.hlist([s.sphere((0, -1000, 0), 1000, ground), s.sphere((0, 1, 0), 1.0, glass),
                     s.sphere((-4, 1, 0), 1.0, matte), s.sphere((4, 1, 0), 1.0, metal)])
    cam = perspective(width, aspect, (13, 2, 3), (0, 0, 0), 1, 20.0)
    return s.desc(world, background=s.solid((0.7, 0.8, 1.0))), cam, 100, 5


def three_material_ball_with_defocus_blur(width=1280, aspect=16.0 / 9.0):  # main.cc:87-103
    desc, _, spp, depth = three_material_ball(width, aspect)
    cam = lens(width, aspect, (13, 2, 3), (1, 1, 1), 2.0, 15, 20.0)
    return desc, cam, 1000, 5


def cornell_glossy(width=600, aspect=1.0):
    """Cornell box with four gloss spheres of rising specular probability, the materials of
    cornell_box_with_glossy_ball (main.cc:309-343) with solid colours instead of the earth image."""
    s = SceneBuilder()
    red, white = s.lambertian(s.solid((.65, .05, .05))), s.lambertian(s.solid((.73, .73, .73)))
    green, light = s.lambertian(s.solid((.12, .45, .15))), s.diffuse_light(s.solid((15, 15, 15)))
    walls = [s.quad((555, 0, 0), (0, 555, 0), (0, 0, 555), green), s.quad((0, 0, 0), (0, 555, 0), (0, 0, 555), red),
             s.quad((0, 0, 0), (555, 0, 0), (0, 0, 555), white),
             s.quad((555, 555, 555), (-555, 0, 0), (0, 0, -555), white),
             s.quad((0, 0, 555), (555, 0, 0), (0, 555, 0), white)]
    lq = s.quad((343, 554, 332), (-130, 0, 0), (0, 0, -105), light)
    tex = s.solid((0.2, 0.4, 0.8))
    balls = [s.sphere((110 + 110 * k, 90, 250), 80, s.gloss(tex, sm, sp))
             for k, (sm, sp) in enumerate([(1.0, 1.0), (1.0, 0.4), (0.6, 0.15), (1.5, 0.02)])]
    world = s.hlist(walls + balls + [lq])
    cam = perspective(width, aspect, (278, 278, -800), (278, 278, 0), 1, 40.0)
    return s.desc(world, light=lq), cam, 100, 8


SCENES = {"cornell_box": cornell_box, "cornell_triangles": cornell_triangles, "cornell_box_with_volume": cornell_box_with_volume,
          "rtow": rtow, "rtow_motion": lambda **kw: rtow(moving=True, **kw),
          "three_material_ball": three_material_ball,
          "three_material_ball_with_defocus_blur": three_material_ball_with_defocus_blur,
          "cornell_glossy": cornell_glossy}
