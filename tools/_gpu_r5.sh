set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/profile_r2.sh r5_v1 > gpurun_out/profile_r5_v1.log 2>&1 || { tail -20 gpurun_out/profile_r5_v1.log; exit 1; }
tail -3 gpurun_out/profile_r5_v1.log
