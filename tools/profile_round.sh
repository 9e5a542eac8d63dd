#!/bin/bash
# Collect the profiles judged under profiles/ (run on the GPU box from the repo root):
#   kernel trace + stats of the default bench, two separate PMC passes
#   (FETCH_SIZE, WRITE_SIZE: they do not fit one TCC pass) of a shorter bench, and
#   one SQ pass (VALU instructions, wave cycles, stalls, GRBM clock).
# usage: tools/profile_round.sh <tag>     -> gpurun_out/prof_<tag>, pmc_{fetch,write,sq}_<tag>
set -euo pipefail
tag=${1:?tag}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
A="--library-total 0 --no-cpu-baseline --no-replay --steps 5 --warmup 1 --pc-steps 200 --pc-warmup 20 --pc-calls 20 --pc-stress-steps 100"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$tag -o run -- python bench.py --no-cpu-baseline --library-total 0 > gpurun_out/prof_$tag.log 2>&1
# configs[2] (100k-template library) in its own trace, so the headline scan's average stays its own
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_lib_$tag -o run -- python bench.py --no-cpu-baseline --no-replay --no-pc-stress --steps 2 --warmup 1 --pc-steps 20 --pc-warmup 5 --pc-calls 5 > gpurun_out/prof_lib_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_$tag -o run -- python bench.py $A > gpurun_out/pmc_fetch_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_$tag -o run -- python bench.py $A > gpurun_out/pmc_write_$tag.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc_sq_$tag -o run -- python bench.py $A > gpurun_out/pmc_sq_$tag.log 2>&1
echo "profiles collected: $tag"
