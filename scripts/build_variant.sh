#!/bin/bash
# Builds a timing variant of one source file (development only): a copy of
# csrc/FILE with Python regex substitutions applied, linked with the other
# objects of build/ -> trik-media-sensors-dsp_amd/ab/NAME/libtrik_hsv.so.
#   bash scripts/build_variant.sh NAME FILE 'pattern=>replacement' ...
# (the shipped sources carry no attribution switches; the variants live here)
# REV=<git rev> takes csrc/FILE as of that revision instead of the work tree.
set -eu
cd "$(dirname "$0")/../trik-media-sensors-dsp_amd"
make -s -C csrc >/dev/null
N="$1"; F="$2"; shift 2
mkdir -p "ab/$N"
SRC="csrc/$F"
if [ -n "${REV:-}" ]; then git show "$REV:trik-media-sensors-dsp_amd/csrc/$F" > "ab/$N/$F.rev"; SRC="ab/$N/$F.rev"; fi
python3 - "$SRC" "ab/$N/$F" "$@" <<'PY'
import re, sys
src, dst, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
s = open(src).read()
for sub in subs:
    pat, rep = sub.split("=>", 1)
    s, n = re.subn(pat, rep, s)
    if n == 0:
        sys.exit(f"no match: {pat}")
open(dst, "w").write(s)
PY
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-result -Icsrc \
    -c -o "ab/$N/var.o" "ab/$N/$F"
base="${F%.*}"
objs=$(ls build/*.o | grep -v "/$F.o")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "ab/$N/libtrik_hsv.so" "ab/$N/var.o" $objs -ldl -lpthread
echo "built ab/$N ($base)"
