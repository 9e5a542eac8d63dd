#!/bin/bash
# A/B variant of the library from an edited copy of posecell.hip (the product source
# stays untouched): abtmp/<name>.so, with each "old=>new" argument applied as a
# literal substitution (python str.replace, must match) to the copy.
# usage: tools/build_pc_edit.sh <name> 'old=>new' ['old=>new' ...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p abtmp tools/ab
python3 - "$name" "$@" <<'PY'
import sys
name, edits = sys.argv[1], sys.argv[2:]
s = open('pyratslam_amd/csrc/posecell.hip').read()
for e in edits:
    old, new = e.split('=>', 1)
    assert old in s, 'no match: ' + old
    s = s.replace(old, new)
open('abtmp/%s.hip' % name, 'w').write(s)
PY
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Ipyratslam_amd/csrc -x hip \
   -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=9 -c abtmp/$name.hip -o tools/ab/$name.pc.o
$H --offload-arch=gfx950 -shared -fPIC -o abtmp/$name.so pyratslam_amd/build/rs_common.o \
   tools/ab/$name.pc.o pyratslam_amd/build/view_templates.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo abtmp/$name.so
