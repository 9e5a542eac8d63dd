cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_view_templates_gpu.py tests/test_configs_gpu.py > gpurun_out/vt_onebar_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/vt_onebar_test.log; exit 1; }
tail -1 gpurun_out/vt_onebar_test.log
timeout -k 10 300 python tools/scan_ab.py abtmp/twobar.so abtmp/onebar.so --templates 1000 --queries 10240 --reps 20 || exit 1
timeout -k 10 300 python tools/scan_ab.py abtmp/twobar.so abtmp/onebar.so --templates 10000 --queries 5120 --reps 6 || exit 1
timeout -k 10 300 python tools/scan_ab.py abtmp/twobar.so abtmp/onebar.so --templates 1000 --queries 1024 --reps 30 || exit 1
