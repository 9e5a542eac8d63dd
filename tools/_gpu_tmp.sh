cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_posecell_gpu.py > gpurun_out/pc_chunk_test.log 2>&1 || { echo "tests failed $?"; grep -E "FAIL|Error|assert" gpurun_out/pc_chunk_test.log | head -20; tail -5 gpurun_out/pc_chunk_test.log; exit 1; }
tail -1 gpurun_out/pc_chunk_test.log
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms cols cols:36 cols:24 cols:18 stream --steps 3000 || exit 1
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms cols cols:36 --steps 3000 || exit 1
