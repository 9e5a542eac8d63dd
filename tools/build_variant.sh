#!/bin/bash
# Build an A/B variant of the library: tools/ab/<name>.so from view_templates.hip
# (or a given source file) plus the current pose-cell objects.
# usage: tools/build_variant.sh <name> [vt_source.hip] [extra hipcc flags...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; src=${2:-pyratslam_amd/csrc/view_templates.hip}; shift; shift || true
mkdir -p tools/ab
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Iinclude -Ipyratslam_amd/csrc -x hip \
   -mllvm -amdgpu-atomic-optimizer-strategy=None "$@" -c "$src" -o tools/ab/$name.vt.o
$H --offload-arch=gfx950 -shared -fPIC -o tools/ab/$name.so pyratslam_amd/build/rs_common.o \
   pyratslam_amd/build/posecell.o tools/ab/$name.vt.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo tools/ab/$name.so
