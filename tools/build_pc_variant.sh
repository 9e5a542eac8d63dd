#!/bin/bash
# Build an A/B variant of the library: tools/ab/<name>.so from posecell.hip
# compiled with extra hipcc flags (e.g. -DPC_CO_YREG=1) plus the current
# view-template objects.
# usage: tools/build_pc_variant.sh <name> [extra hipcc flags...]
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p tools/ab abtmp
H=/opt/rocm/bin/hipcc
$H --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Iinclude -Ipyratslam_amd/csrc -x hip \
   -fno-slp-vectorize "$@" -c pyratslam_amd/csrc/posecell.hip -o tools/ab/$name.pc.o
$H --offload-arch=gfx950 -shared -fPIC -o abtmp/$name.so pyratslam_amd/build/rs_common.o \
   tools/ab/$name.pc.o pyratslam_amd/build/view_templates.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
echo abtmp/$name.so
