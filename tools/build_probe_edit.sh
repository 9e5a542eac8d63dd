#!/bin/bash
# tools/pc_probe.hip built against an edited copy of posecell.hip (the product source
# stays untouched): abtmp/<name>_probe, each "old=>new" argument a literal
# substitution (must match).   usage: tools/build_probe_edit.sh <name> ['old=>new' ...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p abtmp/$name
python3 - "$name" "$@" <<'PY'
import sys
name, edits = sys.argv[1], sys.argv[2:]
s = open('pyratslam_amd/csrc/posecell.hip').read()
for e in edits:
    old, new = e.split('=>', 1)
    assert old in s, 'no match: ' + old
    s = s.replace(old, new)
open('abtmp/%s/posecell.hip' % name, 'w').write(s)
PY
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Iabtmp/$name -Ipyratslam_amd/csrc -x hip \
   -fno-slp-vectorize -mllvm -amdgpu-kernarg-preload-count=9 tools/pc_probe.hip pyratslam_amd/csrc/rs_common.cpp -o abtmp/${name}_probe
echo abtmp/${name}_probe
