cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_posecell_gpu.py tests/test_replay_gpu.py tests/test_host_control.py > gpurun_out/pc_t.log 2>&1 || { echo "tests failed $?"; tail -5 gpurun_out/pc_t.log; exit 1; }
tail -1 gpurun_out/pc_t.log
timeout -k 10 300 python tools/pc_sweep.py --shape 64,64,36 --forms rows rows --steps 5000 || exit 1
timeout -k 10 300 python tools/pc_sweep.py --shape 21,21,36 --forms rows --steps 5000 || exit 1
timeout -k 10 300 python tools/pc_call_cost.py 2>&1 | tail -1
