set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_posecell_gpu.py tests/test_halo_gpu.py tests/test_replay_gpu.py -m gpu > gpurun_out/gputest_run1.log 2>&1 || { tail -30 gpurun_out/gputest_run1.log; exit 1; }
tail -2 gpurun_out/gputest_run1.log
timeout -k 10 200 python -u tools/replay_anatomy.py > gpurun_out/replay_anat5.log 2>&1 && tail -1 gpurun_out/replay_anat5.log | cut -c1-300
