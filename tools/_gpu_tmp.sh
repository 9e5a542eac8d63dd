set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_zc2.log 2>&1 || { tail -60 gpurun_out/gputest_zc2.log; exit 1; }
tail -3 gpurun_out/gputest_zc2.log
timeout -k 10 200 python -u tools/replay_anatomy.py > gpurun_out/replay_anat3.log 2>&1 && cat gpurun_out/replay_anat3.log
RS_VT_ZC=0 timeout -k 10 200 python -u tools/replay_anatomy.py > gpurun_out/replay_anat3_nozc.log 2>&1 && cat gpurun_out/replay_anat3_nozc.log
timeout -k 10 200 python -u tools/vt_call_anatomy.py > gpurun_out/vt_anat3.log 2>&1 && cat gpurun_out/vt_anat3.log
