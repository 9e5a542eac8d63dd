cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 60 tools/pc_probe 128 128 72 > gpurun_out/probe128.log 2>&1
rc=$?; cat gpurun_out/probe128.log; if fatal $rc; then exit $rc; fi
timeout -k 10 60 tools/pc_probe 64 64 36 > gpurun_out/probe64.log 2>&1
rc=$?; cat gpurun_out/probe64.log; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u tools/pc_ab.py abtmp/base.so abtmp/new.so abtmp/new.so@RS_PC_CTL=ring --rounds 2 > gpurun_out/pc_ab4.log 2>&1
rc=$?; cat gpurun_out/pc_ab4.log; if fatal $rc; then exit $rc; fi
timeout -k 10 400 python -u tools/pc_ab.py abtmp/base.so abtmp/new.so abtmp/new.so@RS_PC_CTL=inline --shape 64,64,36 --rounds 2 > gpurun_out/pc_ab4_64.log 2>&1
rc=$?; cat gpurun_out/pc_ab4_64.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; tail -c 300 gpurun_out/bench.log; exit $rc
