set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_posecell_gpu.py > gpurun_out/pc_t.log 2>&1 || { tail -40 gpurun_out/pc_t.log; exit 1; }
tail -2 gpurun_out/pc_t.log
timeout -k 10 400 python -u tools/pc_ab.py abtmp/pre.so abtmp/cols.so --shape 128,128,72 --rounds 4 --steps 1500 > gpurun_out/ab_cols.log 2>&1 || { tail -20 gpurun_out/ab_cols.log; exit 1; }
tail -2 gpurun_out/ab_cols.log; grep max_abs gpurun_out/ab_cols.log | cut -c1-60,150-230
