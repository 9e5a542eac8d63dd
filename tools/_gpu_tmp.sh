cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u tools/flake_check.py 40 > gpurun_out/flake.log 2>&1
rc=$?; tail -8 gpurun_out/flake.log; if fatal $rc; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; exit $rc
