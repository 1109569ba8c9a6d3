"""Generates tests/golden/ref_geom.json, the reference-computed fixtures of tests/test_oracle_refpins.py
(run in the container that has /root/reference).

The reference's own geometry and sampling code -- sphere.h, triangle.h, aabb.h, hittable_list.h,
bvh_node.h, onb.h, pdf.h, noise.h and utility.h, compiled where they lie (oracle/Makefile `ref` ->
oracle/_ref/ref_geom, source oracle/ref_geom.cpp) -- evaluated on fixed generated cases. The
fixture is its output verbatim: inputs and the reference's results, doubles with 17 digits.

    make -C oracle ref && python tests/golden/make_ref_geom_golden.py
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
EXE = os.path.join(REPO, "oracle", "_ref", "ref_geom")


def main():
    text = subprocess.run([EXE], check=True, capture_output=True, text=True).stdout
    data = json.loads(text)  # validates the document
    with open(os.path.join(HERE, "ref_geom.json"), "w") as f:
        f.write(text)
    print({k: len(v) for k, v in data.items()})


if __name__ == "__main__":
    main()
