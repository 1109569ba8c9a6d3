"""The multi-GPU tile plan of rt_multi_plan (include/rt_hip.h; camera.h:154-172's row
parallelism lifted to tiles over GPUs) on the host: for 1, 2, 4 and 8
devices it equals bench.py's torch.distributed plan (rt_amd.tiling) and covers every pixel
exactly once, so the gathered image is the whole framebuffer."""
import numpy as np
import pytest

from rt_amd import multi_plan
from rt_amd.tiling import pixel_index, plan


@pytest.mark.parametrize("W,H", [(800, 800), (1200, 800), (1920, 1080), (97, 33), (31, 5)])
@pytest.mark.parametrize("n", [1, 2, 4, 8])
def test_plan_matches_tiling_and_covers_the_image(W, H, n):
    tiles, counts, maxpix = plan(W, H, n, ts=32)
    seen = np.zeros(W * H, dtype=np.int64)
    for r in range(n):
        mine = multi_plan(W, H, n, r, 32)
        assert mine == [tuple(t) for t in tiles[r]]
        idx = pixel_index(mine, W)
        assert len(idx) == counts[r] <= maxpix
        seen[idx] += 1
    assert (seen == 1).all()


def test_plan_balances_ranks():
    # C2 at 8 GPUs: 32x32 tiles leave the ranks within 1.3 % of each other in pixels
    counts = [sum(t[2] * t[3] for t in multi_plan(800, 800, 8, r)) for r in range(8)]
    assert max(counts) / min(counts) < 1.02


def test_plan_rejects_bad_arguments():
    with pytest.raises(ValueError):
        multi_plan(0, 10, 2, 0)
    with pytest.raises(ValueError):
        multi_plan(10, 10, 2, 2)
