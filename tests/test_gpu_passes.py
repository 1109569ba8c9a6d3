"""Renders whose item partial sums exceed the memory budget come in chunk passes (rt_kernels.hip render(),
k_resolve): every pass is one launch over a range of each pixel's chunks, and its resolve adds them to the
running per-pixel sums in chunk order -- the additions camera.h:163-170's per-pixel loop makes, in the same
order as one pass. So the image must be bit-identical whatever the budget, and a call past 2^31 items (which
the item counter cannot hold in one launch) must render. Rounds 1-4 refused it (RT_ERR_INVALID_ARGUMENT) and
let C5 fp64 allocate ~38 GB of partial sums."""
import numpy as np
import pytest

import rt_amd
from rt_amd import abi, scenes

pytestmark = pytest.mark.gpu

F32, F64 = abi.RT_PREC_F32, abi.RT_PREC_F64


@pytest.fixture(scope="module")
def ctx():
    c = rt_amd.Context(0)
    yield c
    c.close()


def _render(ctx, cam, spp, depth, prec, **kw):
    ctx.reset_counters()
    img = ctx.render(cam, spp, depth, seed=7, precision=prec, **kw)
    st = ctx.stats()
    return img, st.passes, st.partial_bytes


@pytest.mark.parametrize("scene,width,spp,depth", [("cornell_box", 64, 256, 8),               # flat program
                                                   ("cornell_box_with_volume", 48, 128, 5),   # volume program
                                                   ("rtow", 48, 64, 50)],                     # wide BVH in LDS
                         ids=["flat", "volume", "wide"])
@pytest.mark.parametrize("prec", [F32, F64], ids=["f32", "f64"])
def test_passes_give_the_one_pass_image(ctx, monkeypatch, scene, width, spp, depth, prec):
    desc, cam, _, _ = scenes.SCENES[scene](width=width)
    ctx.upload(desc)
    one, p1, b1 = _render(ctx, cam, spp, depth, prec)
    wf1, _, _ = _render(ctx, cam, spp, depth, prec, segments_per_launch=4)
    assert p1 == 1
    npix = cam.image_width * cam.image_height
    item_bytes = 3 * (8 if prec == F64 else 4)
    monkeypatch.setenv("RT_PARTIAL_BUDGET", str(3 * item_bytes * npix))  # three chunks per pass
    many, pn, bn = _render(ctx, cam, spp, depth, prec)
    assert pn > 2 and bn == 3 * item_bytes * npix < b1
    assert np.array_equal(one, many), int((one != many).any(-1).sum())
    # the launch-per-K wavefront schedule goes through the same passes (its kernels may differ from the
    # persistent ones -- RTOW takes the binary BVH there -- so it is compared with its own one-pass image)
    wf, pw, _ = _render(ctx, cam, spp, depth, prec, segments_per_launch=4)
    assert pw == pn
    assert np.array_equal(wf1, wf), int((wf1 != wf).any(-1).sum())


def test_call_past_2_pow_31_items_matches_row_renders(ctx):
    # 1024 x 1024 pixels x 2100 items of one sample = 2.2 G items: more than one launch's 32-bit item space
    desc, cam, _, _ = scenes.cornell_box(width=1024)
    ctx.upload(desc)
    assert cam.image_width * cam.image_height * 2100 > 2**31
    full, passes, nbytes = _render(ctx, cam, 2100, 2, F32, samples_per_item=1)
    assert passes >= 2 and nbytes <= 2 << 30
    assert np.isfinite(full).all() and full.mean() > 0.01
    for y in (0, 517, 1023):
        row = ctx.render(cam, 2100, 2, seed=7, precision=F32, samples_per_item=1, tiles=[(0, y, 1024, 1)])
        assert np.array_equal(row, full[y]), (y, int((row != full[y]).any(-1).sum()))
