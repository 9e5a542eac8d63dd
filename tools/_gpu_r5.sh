set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_r5_v5.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v5.log; exit 1; }
tail -3 gpurun_out/gputest_r5_v5.log
for sh in 21,21,36 64,64,36; do timeout -k 10 200 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_FLAGS=0 --shape $sh --mode node --steps 3000 --rounds 4 > gpurun_out/ab_flags_$sh.log 2>&1; tail -2 gpurun_out/ab_flags_$sh.log; done
