set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_r5_v4.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v4.log; exit 1; }
tail -3 gpurun_out/gputest_r5_v4.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_POLL=0 --shape 64,64,36 --mode update --steps 5000 --rounds 4 > gpurun_out/ab_poll2.log 2>&1
tail -2 gpurun_out/ab_poll2.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=rows "pyratslam_amd/libratslam_hip.so@RS_PC_FORM=rows;RS_PC_HALO_POLL=0" --shape 64,64,36 --mode update --steps 5000 --rounds 3 > gpurun_out/ab_poll_rows.log 2>&1
tail -2 gpurun_out/ab_poll_rows.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_POLL=0 --shape 128,128,72 --mode update --steps 2000 --rounds 3 > gpurun_out/ab_poll_cols.log 2>&1
tail -2 gpurun_out/ab_poll_cols.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_POLL=0 --shape 64,64,36 --steps 4000 --rounds 3 > gpurun_out/ab_poll_run.log 2>&1
tail -2 gpurun_out/ab_poll_run.log
