cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 60 abtmp/pc_probe_tvwt 128 128 72 > gpurun_out/probe128_tvwt.log 2>&1
rc=$?; cat gpurun_out/probe128_tvwt.log; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u tools/pc_ab.py abtmp/base.so abtmp/tvec.so abtmp/tvwt.so abtmp/base.so@RS_PC_CTL=inline abtmp/tvwt.so@RS_PC_CTL=inline --rounds 3 > gpurun_out/pc_ab3.log 2>&1
rc=$?; cat gpurun_out/pc_ab3.log; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u tools/pc_ab.py abtmp/base.so abtmp/tvec.so abtmp/tvwt.so --shape 64,64,36 --rounds 2 > gpurun_out/pc_ab3_64.log 2>&1
rc=$?; cat gpurun_out/pc_ab3_64.log; exit $rc
