set -o pipefail
cd $GRAFT_REPO_ROOT
L=pyratslam_amd/libratslam_hip.so
ls $L > /dev/null || exit 1
for m in run update node; do
  echo "== mode $m 64"
  timeout -k 10 200 python -u tools/pc_ab.py $L@RS_PC_FORM=rows $L@RS_PC_FORM=halo --shape 64,64,36 --rounds 3 --steps 3000 --mode $m > gpurun_out/ab_$m.log 2>&1 || { tail -20 gpurun_out/ab_$m.log; exit 1; }
  tail -4 gpurun_out/ab_$m.log
done
echo "== 21"
timeout -k 10 200 python -u tools/pc_ab.py $L@RS_PC_FORM=rows $L@RS_PC_FORM=halo --shape 21,21,36 --rounds 3 --steps 3000 > gpurun_out/ab_21.log 2>&1 || { tail -20 gpurun_out/ab_21.log; exit 1; }
tail -4 gpurun_out/ab_21.log
