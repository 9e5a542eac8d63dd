set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_halo_gpu.py tests/test_posecell_gpu.py tests/test_replay_gpu.py tests/test_threading_gpu.py -m gpu > gpurun_out/gputest_r5_v6.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v6.log; exit 1; }
tail -2 gpurun_out/gputest_r5_v6.log
for sh in 21,21,36 64,64,36; do timeout -k 10 200 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so abtmp/xpold.so --shape $sh --mode node --steps 3000 --rounds 4 > gpurun_out/ab_xp_$sh.log 2>&1; tail -2 gpurun_out/ab_xp_$sh.log; done
