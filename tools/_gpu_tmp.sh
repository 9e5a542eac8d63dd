cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_posecell_gpu.py > gpurun_out/pc_cols_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/pc_cols_test.log; exit 1; }
tail -1 gpurun_out/pc_cols_test.log
B="/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Ipyratslam_amd/csrc tools/pc_probe.hip pyratslam_amd/csrc/rs_common.cpp"
V=("9" "12")
for v in "${V[@]}"; do $B -DPC_CO_NW=$v -o /tmp/pcp_$v & done; wait
for v in "${V[@]}"; do echo "== NW=$v"; RS_PC_FORM=cols timeout -k 10 60 /tmp/pcp_$v 128 128 72 | grep -E "phase|alone|first" || exit 1; done
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms stream cols --steps 3000 || exit 1
