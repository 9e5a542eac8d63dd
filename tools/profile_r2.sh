#!/bin/bash
# Profiles judged under profiles/ (run on the GPU box from the repo root):
#   tools/profile_r2.sh <tag> [configs...]   -> gpurun_out/prof_<tag>/
# Per configuration (tools/scan_profile.py: one kernel configuration per process,
# so every dispatch of a kernel belongs to it): a kernel trace + stats, and three
# PMC passes -- FETCH_SIZE, WRITE_SIZE (they do not fit one TCC pass) and the SQ
# set (VALU instructions, wave-cycle split, GRBM clock).  Plus the kernel trace +
# stats of the default bench command itself (the bench's live timings must agree
# with it).  Summarised by tools/pmc_collect.py.
tag=${1:?tag}
shift
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-.}" || exit 1
out=gpurun_out/prof_$tag
mkdir -p "$out"
declare -A CMD=(
  [headline]="scan --templates 1000 --queries 10240 --launches 60"
  [stress]="scan --templates 10000 --queries 5120 --launches 16"
  [library]="scan --templates 100000 --queries 2048 --launches 6"
  [pc64]="pc --shape 64,64,36 --steps 400"
  [pc128]="pc --shape 128,128,72 --steps 300"
)
configs=("$@")
[ ${#configs[@]} -eq 0 ] && configs=(headline stress library pc64 pc128 bench)
SQ="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
for c in "${configs[@]}"; do
  if [ "$c" = bench ]; then
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/bench_trace" -o run \
        -- python bench.py > "$out/bench.json" 2> "$out/bench.err" || { echo "bench trace failed: $?"; exit 1; }
    continue
  fi
  args=${CMD[$c]}
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/${c}_trace" -o run \
      -- python tools/scan_profile.py $args > "$out/${c}_trace.log" 2>&1 || { echo "$c trace failed: $?"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/${c}_fetch" -o run \
      -- python tools/scan_profile.py $args > "$out/${c}_fetch.log" 2>&1 || { echo "$c fetch failed: $?"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/${c}_write" -o run \
      -- python tools/scan_profile.py $args > "$out/${c}_write.log" 2>&1 || { echo "$c write failed: $?"; exit 1; }
  timeout -s KILL 240 rocprofv3 --pmc $SQ --output-format csv -d "$out/${c}_sq" -o run \
      -- python tools/scan_profile.py $args > "$out/${c}_sq.log" 2>&1 || { echo "$c sq failed: $?"; exit 1; }
  echo "profiled $c"
done
echo "profiles collected: $tag"
