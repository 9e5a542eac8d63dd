cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_posecell_gpu.py > gpurun_out/pc_t.log 2>&1 || { echo "tests failed $?"; tail -5 gpurun_out/pc_t.log; exit 1; }
tail -1 gpurun_out/pc_t.log
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms cols stream cols --steps 3000 || exit 1
