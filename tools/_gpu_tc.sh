set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tc_gpu.py -m gpu > gpurun_out/tc_test3.log 2>&1 || { tail -40 gpurun_out/tc_test3.log; exit 1; }
tail -3 gpurun_out/tc_test3.log
for f in tc:36,4,1 tc:36,8,1 tc:24,4,1; do RS_PC_FORM=$f timeout -k 10 60 ./tools/pc_probe 128 128 72 1.5 > gpurun_out/probe3_$f.log 2>&1; echo "probe $f rc=$?"; cat gpurun_out/probe3_$f.log; done
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=cols pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,8 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,8,1 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,4,1 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,4,1 --shape 128,128,72 --steps 2000 --rounds 3 > gpurun_out/tc_ab3.log 2>&1
tail -6 gpurun_out/tc_ab3.log
