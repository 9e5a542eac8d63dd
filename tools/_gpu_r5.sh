set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_r5_v1.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v1.log; exit 1; }
tail -3 gpurun_out/gputest_r5_v1.log
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' @RS_PC_HALO_SETTLE=1 rows --calls 2000 > gpurun_out/anat4.log 2>&1
cat gpurun_out/anat4.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_SETTLE=1 --shape 64,64,36 --steps 4000 --rounds 3 > gpurun_out/ab_halo_lazy.log 2>&1
tail -3 gpurun_out/ab_halo_lazy.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_SETTLE=1 --shape 64,64,36 --mode update --steps 3000 --rounds 3 > gpurun_out/ab_halo_lazy_upd.log 2>&1
tail -3 gpurun_out/ab_halo_lazy_upd.log
