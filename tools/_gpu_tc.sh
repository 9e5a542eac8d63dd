set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_tc_gpu.py -m gpu > gpurun_out/tc_test1.log 2>&1 || { tail -40 gpurun_out/tc_test1.log; exit 1; }
tail -3 gpurun_out/tc_test1.log
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=cols pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:12,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,4 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:24,8 pyratslam_amd/libratslam_hip.so@RS_PC_FORM=tc:36,8 --shape 128,128,72 --steps 2000 --rounds 3 > gpurun_out/tc_ab1.log 2>&1
tail -20 gpurun_out/tc_ab1.log
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' rows tc:12,4 @ROC_ACTIVE_WAIT_TIMEOUT=0 @ROC_ACTIVE_WAIT_TIMEOUT=50 @ROC_ACTIVE_WAIT_TIMEOUT=200 rows@ROC_ACTIVE_WAIT_TIMEOUT=200 --calls 2000 > gpurun_out/anat1.log 2>&1
cat gpurun_out/anat1.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --hip-runtime-trace --kernel-trace --stats -d gpurun_out/anat_halo -o run -- python3 tools/pc_call_anatomy.py --child --mode calls --calls 2000 > gpurun_out/anat_halo.log 2>&1
echo rocprof rc=$?
for f in cols tc:12,4 tc:24,4 tc:24,8 tc:36,8; do RS_PC_FORM=$f timeout -k 10 60 ./tools/pc_probe 128 128 72 1.5 > gpurun_out/probe_$f.log 2>&1; echo "probe $f rc=$?"; done
cat gpurun_out/probe_tc:24,4.log
for sh in 32,32,18 50,50,10; do timeout -k 10 120 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so --shape $sh --steps 2000 --rounds 2 > gpurun_out/ab_small_$sh.log 2>&1; tail -2 gpurun_out/ab_small_$sh.log; done
