#!/usr/bin/env python3
"""Static VALU opcode mix of one kernel of librt_hip.so (its gfx950 code object, llvm-objdump), split into
the classes the SQ_INSTS_VALU_* counters count -- fp64 add/mul/fma, fp64 transcendental, conversions,
64-bit integer -- and the rest, with the rest broken down further (fp64 compares / min / max and other
fp64 opcodes the counters do not single out, fp32, moves and selects, 32-bit integer).

  python scripts/valu_static_mix.py <lib.so> <kernel substring> [--out file.json]

Used for bench.py's fp64 roofline: the counters give the dynamic counts of their classes;
this gives the share of the uncounted fp64 opcodes inside the remainder."""
import argparse
import collections
import json
import os
import re
import subprocess
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def classify(op):
    if re.match(r"v_(add|mul|fma|fmac)_f64", op):
        return "f64_addmulfma"
    if re.match(r"v_(rcp|rsq|sqrt|sin|cos|log|exp)_f64", op):
        return "f64_trans"
    if op.startswith("v_cvt"):
        return "cvt"
    if re.search(r"_[iu]64", op) or re.match(r"v_(lshl|lshr|ashr)rev_b64|v_lshl_add_u64|v_mad_u64|v_mad_i64", op):
        return "int64"
    if "f64" in op:
        if op.startswith("v_cmp"):
            return "f64_cmp"
        if re.match(r"v_(min|max)_f64", op):
            return "f64_minmax"
        return "f64_other"
    if re.match(r"v_(rcp|rsq|sqrt|sin|cos|log|exp)_f32", op):
        return "f32_trans"
    if op.startswith(("v_mov", "v_cndmask", "v_readlane", "v_readfirstlane", "v_writelane", "v_mbcnt")):
        return "move_select"
    if "f32" in op or "f16" in op:
        return "f32"
    return "int32_other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib")
    ap.add_argument("kernel")
    ap.add_argument("--out")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        so = os.path.join(td, "lib.so")
        subprocess.run(["cp", a.lib, so], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={so}"], capture_output=True)
        subprocess.run([f"{LLVM}/llvm-objdump", "--offloading", so], cwd=td, capture_output=True, check=True)
        objs = [f for f in os.listdir(td) if "gfx950" in f]
        text = ""
        for o in objs:
            text += subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", "-C", os.path.join(td, o)],
                                   capture_output=True, text=True).stdout
    counts, name, on = collections.Counter(), None, False
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.*)>:$", line)
        if m:
            name = m.group(1)
            on = a.kernel in name
            continue
        if on:
            m = re.match(r"^\s+(v_[a-z0-9_]+)", line)
            if m:
                counts[m.group(1)] += 1
    cls = collections.Counter()
    for op, n in counts.items():
        cls[classify(op)] += n
    total = sum(cls.values())
    res = {"kernel": a.kernel, "lib": os.path.basename(a.lib), "static_valu": total,
           "classes": dict(cls.most_common()), "opcodes": dict(counts.most_common())}
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps({"static_valu": total, "classes": res["classes"]}))


if __name__ == "__main__":
    main()
