cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 400 python -u tools/pc_ab.py abtmp/new.so abtmp/ctl1.so --shape 64,64,36 --rounds 4 > gpurun_out/pc_ab6_64.log 2>&1
rc=$?; cat gpurun_out/pc_ab6_64.log; if fatal $rc; then exit $rc; fi
timeout -k 10 1000 bash tools/profile_r2.sh r2_v6 > gpurun_out/prof_r2_v6.log 2>&1
rc=$?; tail -5 gpurun_out/prof_r2_v6.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; tail -c 300 gpurun_out/bench.log; exit $rc
