set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_view_templates_gpu.py -k "zero_sized or small_batches" -m gpu > gpurun_out/gputest_zero.log 2>&1; rc=$?; tail -8 gpurun_out/gputest_zero.log; exit $rc
