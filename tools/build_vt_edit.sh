#!/bin/bash
# A/B variant of the library from an edited copy of view_templates.hip (the product
# source stays untouched): abtmp/<name>.so, each "old=>new" argument a literal
# substitution (must match).   usage: tools/build_vt_edit.sh <name> ['old=>new' ...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p abtmp tools/ab
python3 - "$name" "$@" <<'PY'
import sys
name, edits = sys.argv[1], sys.argv[2:]
s = open('pyratslam_amd/csrc/view_templates.hip').read()
for e in edits:
    old, new = e.split('=>', 1)
    assert old in s, 'no match: ' + old
    s = s.replace(old, new)
open('abtmp/%s_vt.hip' % name, 'w').write(s)
PY
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ipyratslam_amd/csrc -x hip \
   -mllvm -amdgpu-atomic-optimizer-strategy=None -c abtmp/${name}_vt.hip -o tools/ab/$name.vt.o
$H --offload-arch=gfx950 -shared -fPIC -o abtmp/$name.so pyratslam_amd/build/rs_common.o \
   pyratslam_amd/build/posecell.o tools/ab/$name.vt.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo abtmp/$name.so
