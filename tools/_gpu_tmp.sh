set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_halo_gpu.py > gpurun_out/halo_t2.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ]; then tail -60 gpurun_out/halo_t2.log; exit $rc; fi
for vt in 0 1.5 3; do
  RS_PC_FORM=halo timeout -k 10 60 ./tools/pc_probe 64 64 36 $vt > gpurun_out/probe2_halo_$vt.log 2>&1 || exit 1
done
cat gpurun_out/probe2_halo_*.log
timeout -k 10 300 python tools/pc_ab.py pyratslam_amd/libratslam_hip.so@RS_PC_FORM=rows pyratslam_amd/libratslam_hip.so@RS_PC_FORM=halo --shape 64,64,36 --rounds 3 --steps 3000 > gpurun_out/halo_ab2.log 2>&1
rc=$?
cat gpurun_out/halo_ab2.log
exit $rc
