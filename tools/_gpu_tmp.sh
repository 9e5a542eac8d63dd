set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/gputest_final.log 2>&1 || { tail -30 gpurun_out/gputest_final.log; exit 1; }
tail -2 gpurun_out/gputest_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2
