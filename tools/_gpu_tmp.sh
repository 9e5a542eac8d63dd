set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_posecell_gpu.py -k "reference_attributes or golden_trajectory" -m gpu > gpurun_out/gputest_attr.log 2>&1; rc=$?; tail -5 gpurun_out/gputest_attr.log; exit $rc
