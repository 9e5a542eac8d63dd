cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log; if fatal $rc; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; if fatal $rc; then exit $rc; fi
timeout -k 10 60 tools/pc_probe 64 64 36 > gpurun_out/probe64.log 2>&1
rc=$?; cat gpurun_out/probe64.log; if fatal $rc; then exit $rc; fi
timeout -k 10 1000 bash tools/profile_r2.sh r2_v9 pc64 pc128 bench > gpurun_out/prof_r2_v9.log 2>&1
rc=$?; tail -3 gpurun_out/prof_r2_v9.log; if fatal $rc; then exit $rc; fi
timeout -k 10 300 python -u bench.py > gpurun_out/bench.log 2> gpurun_out/bench.err
rc=$?; tail -c 200 gpurun_out/bench.log; exit $rc
