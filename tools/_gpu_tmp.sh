cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -u -m pytest tests/test_posecell_gpu.py tests/test_replay_gpu.py -x -q --timeout 180 --timeout-method thread > gpurun_out/pc_tests.log 2>&1
rc=$?; tail -15 gpurun_out/pc_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 60 tools/pc_probe 64 64 36 > gpurun_out/probe64.log 2>&1
rc=$?; cat gpurun_out/probe64.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u tools/pc_ab.py abtmp/thf4.so abtmp/rsh.so --shape 64,64,36 --rounds 4 > gpurun_out/pc_ab14.log 2>&1
rc=$?; tail -3 gpurun_out/pc_ab14.log; exit $rc
