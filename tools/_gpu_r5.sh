set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for sh in 64,64,36 21,21,36; do timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so abtmp/hf12.so --shape $sh --steps 4000 --rounds 4 > gpurun_out/ab_hf12_$sh.log 2>&1; tail -3 gpurun_out/ab_hf12_$sh.log; done
timeout -k 10 60 ./tools/pc_probe 64 64 36 1.5 > gpurun_out/probe_hf9.log 2>&1; grep -v "^$" gpurun_out/probe_hf9.log | head -20
timeout -k 10 60 ./abtmp/pc_probe12 64 64 36 1.5 > gpurun_out/probe_hf12.log 2>&1; grep -v "^$" gpurun_out/probe_hf12.log | head -20
