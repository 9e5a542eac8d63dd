cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_posecell_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pc_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pc_tests.log; exit $rc
