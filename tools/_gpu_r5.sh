set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_halo_gpu.py tests/test_posecell_gpu.py tests/test_threading_gpu.py -m gpu > gpurun_out/gputest_r5_v2.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v2.log; exit 1; }
tail -3 gpurun_out/gputest_r5_v2.log
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' @RS_PC_HALO_REC=device @RS_PC_HALO_SETTLE=1 rows --calls 3000 > gpurun_out/anat5.log 2>&1
cat gpurun_out/anat5.log
