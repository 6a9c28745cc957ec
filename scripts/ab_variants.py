"""Builds timing variants of one kernel source (development only): each
variant is the work-tree file with literal (old -> new) replacements, compiled
and linked with the other objects of build/ into
trik-media-sensors-dsp_amd/ab/NAME/libtrik_hsv.so (scripts/kbench times them
side by side).  The shipped sources carry no A/B switches.

usage: python scripts/ab_variants.py VARIANTS.py [name ...]
VARIANTS.py defines FILE (a csrc/ file name) and VARIANTS = {name: [(old, new), ...]};
a name with REV=<git rev> as its first entry takes the file at that revision.
"""
import os
import runpy
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "trik-media-sensors-dsp_amd")
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-result"]


def build(name, file, subs):
    out = os.path.join(PKG, "ab", name)
    os.makedirs(out, exist_ok=True)
    if subs and isinstance(subs[0], str) and subs[0].startswith("REV="):
        src = subprocess.run(["git", "show", f"{subs[0][4:]}:trik-media-sensors-dsp_amd/csrc/{file}"], cwd=ROOT,
                             check=True, capture_output=True, text=True).stdout
        subs = subs[1:]
    else:
        src = open(os.path.join(PKG, "csrc", file)).read()
    for old, new in subs:
        n = src.count(old)
        if n != 1:
            raise SystemExit(f"{name}: pattern found {n} times: {old[:80]!r}")
        src = src.replace(old, new)
    path = os.path.join(out, file)
    with open(path, "w") as f:
        f.write(src)
    obj = os.path.join(out, "var.o")
    subprocess.run([HIPCC, *FLAGS, "-I", os.path.join(PKG, "csrc"), "-c", "-o", obj, path], check=True)
    objs = sorted(os.path.join(PKG, "build", o) for o in os.listdir(os.path.join(PKG, "build"))
                  if o.endswith(".o") and o != file + ".o")
    subprocess.run([HIPCC, "-shared", "-fPIC", "--offload-arch=gfx950", "-o", os.path.join(out, "libtrik_hsv.so"),
                    obj, *objs, "-ldl", "-lpthread"], check=True)
    return name


def main():
    spec = runpy.run_path(sys.argv[1])
    names = sys.argv[2:] or list(spec["VARIANTS"])
    subprocess.run(["make", "-s", "-C", os.path.join(PKG, "csrc")], check=True)
    with ThreadPoolExecutor(max_workers=4) as ex:
        for n in ex.map(lambda n: build(n, spec["FILE"], spec["VARIANTS"][n]), names):
            print("built ab/" + n, flush=True)


if __name__ == "__main__":
    main()
