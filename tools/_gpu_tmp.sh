set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r4_v1.log 2>&1 || { tail -40 gpurun_out/gputest_r4_v1.log; exit 1; }
tail -3 gpurun_out/gputest_r4_v1.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
