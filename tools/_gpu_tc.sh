set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for vt in 0 1.5 3; do for f in cols tc:36,8,1 tc:36,8; do echo "== $f vt=$vt"; RS_PC_FORM=$f timeout -k 10 60 ./tools/pc_probe 128 128 72 $vt > gpurun_out/probe4.log 2>&1 || exit 1; grep -v "^   phase" gpurun_out/probe4.log; grep "phase" gpurun_out/probe4.log | tr '\n' ' '; echo; done; done
