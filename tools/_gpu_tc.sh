set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tc_gpu.py tests/test_halo_gpu.py -m gpu > gpurun_out/tc_test2.log 2>&1 || { tail -40 gpurun_out/tc_test2.log; exit 1; }
tail -3 gpurun_out/tc_test2.log
for f in cols tc:12,4 tc:24,4 tc:24,8 tc:36,8; do RS_PC_FORM=$f timeout -k 10 60 ./tools/pc_probe 128 128 72 1.5 > gpurun_out/probe2_$f.log 2>&1; echo "probe $f rc=$?"; done
grep -h "excite alone\|excite + path\|grid\|phase\|first start" gpurun_out/probe2_*.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=cols pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:12,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,8 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,8 --shape 128,128,72 --steps 2000 --rounds 3 > gpurun_out/tc_ab2.log 2>&1
tail -6 gpurun_out/tc_ab2.log
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' @RS_PC_HALO_FENCE=1 @RS_PC_HALO_EXPORT=kernel rows --calls 2000 > gpurun_out/anat2.log 2>&1
cat gpurun_out/anat2.log
