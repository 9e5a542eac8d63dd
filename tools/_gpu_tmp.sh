cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 500 python -u tools/pc_ab.py abtmp/final.so abtmp/fs4.so abtmp/fc4.so abtmp/fs1.so abtmp/fr1.so --rounds 3 > gpurun_out/pc_ab19.log 2>&1
rc=$?; tail -5 gpurun_out/pc_ab19.log; exit $rc
