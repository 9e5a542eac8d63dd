set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tc_gpu.py -m gpu > gpurun_out/tc_test1.log 2>&1 || { tail -40 gpurun_out/tc_test1.log; exit 1; }
tail -3 gpurun_out/tc_test1.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=cols pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:12,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,8 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,8 --shape 128,128,72 --steps 2000 --rounds 3 > gpurun_out/tc_ab1.log 2>&1
tail -20 gpurun_out/tc_ab1.log
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' rows tc:12,4 --calls 2000 > gpurun_out/anat1.log 2>&1
tail -5 gpurun_out/anat1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/anat_halo -o run -- python3 tools/pc_call_anatomy.py --child --mode calls --calls 2000 > gpurun_out/anat_halo.log 2>&1
echo rocprof rc=$?
