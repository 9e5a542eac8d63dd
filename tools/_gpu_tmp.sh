set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_halo_gpu.py > gpurun_out/halo_t.log 2>&1 || { tail -40 gpurun_out/halo_t.log; exit 1; }
tail -2 gpurun_out/halo_t.log
