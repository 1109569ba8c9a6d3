"""Regenerates the committed fixtures in tests/golden/ (run from the repo root:
`python tests/golden/make_golden.py`). survey_pins.json is not generated: it
records outputs of the reference itself that SURVEY.md measured (see there)."""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(REPO, "oracle"), os.path.join(REPO, "cpu-ray-tracing-implementation_amd", "python")]
import oracle  # noqa: E402

# counter-RNG vectors: (seed, pixel, sample, dim) -> u32, edge values included
cases = []
for seed in (0, 1, 7, 0xFFFFFFFF, 0x123456789ABCDEF0, 2 ** 64 - 1):
    for pixel in (0, 1, 639999, 2 ** 32 - 1):
        for sample in (0, 1, 1023, 2 ** 32 - 1):
            for dim in (0, 2, 3, 18, 802, 2 ** 32 - 1):
                cases.append([seed, pixel, sample, dim, oracle.rng_u32(seed, pixel, sample, dim)])
with open(os.path.join(HERE, "rng_vectors.json"), "w") as f:
    json.dump({"generator": "oracle/oracle.cpp orc_rng_u32", "cases": cases}, f)

# oracle regression hashes (counter RNG): guards the restatement against drift
regress = []
for name, w, a, spp, d, seed in [("cornell_box", 32, 0, 4, 8, 1), ("cornell_box_with_volume", 32, 0, 4, 5, 2),
                                 ("rtow", 36, 1.5, 4, 50, 3), ("three_material_ball", 32, 0, 4, 5, 4),
                                 ("cornell_triangles", 32, 0, 4, 8, 5)]:
    sc, cam, _, _ = oracle.builtin(name, w, a)
    img, segs = oracle.render(sc, cam, spp, d, seed=seed, threads=1)
    regress.append({"scene": name, "width": w, "aspect": a, "spp": spp, "depth": d, "seed": seed,
                    "sha256_f64": hashlib.sha256(img.tobytes()).hexdigest(), "segments": segs,
                    "mean_rgb": img.reshape(-1, 3).mean(0).tolist()})
with open(os.path.join(HERE, "oracle_regression.json"), "w") as f:
    json.dump(regress, f, indent=1)
print(f"{len(cases)} rng vectors, {len(regress)} regression images")
