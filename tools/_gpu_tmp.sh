cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_posecell_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "persistent" > gpurun_out/pc_persist.log 2>&1; rc=$?
tail -3 gpurun_out/pc_persist.log
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 200 python tools/pc_sweep.py --shape 64,64,36 --steps 2000 --check-steps 20 --forms rows persist:1 persist:2 persist:4 persist:8 rows persist:2 2>&1 | grep "{"
