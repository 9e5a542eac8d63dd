set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r4_v4.log 2>&1 || { tail -40 gpurun_out/gputest_r4_v4.log; exit 1; }
tail -2 gpurun_out/gputest_r4_v4.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 1000 bash tools/profile_r2.sh r4_v2 pc64 pc128 headline stress library bench > gpurun_out/prof_r4_v2.log 2>&1 || { tail -20 gpurun_out/prof_r4_v2.log; exit 1; }
tail -2 gpurun_out/prof_r4_v2.log
