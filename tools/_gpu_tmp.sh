cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_posecell_gpu.py -k "forms or default_form" > gpurun_out/pc_cols_test.log 2>&1 || { echo "tests failed $?"; tail -30 gpurun_out/pc_cols_test.log; exit 1; }
tail -4 gpurun_out/pc_cols_test.log
for v in "9 8" "12 8" "8 8" "16 8" "9 16"; do
  set -- $v
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -DPC_CO_NW=$1 -DPC_CO_TX=$2 -Iinclude -Ipyratslam_amd/csrc tools/pc_probe.hip pyratslam_amd/csrc/rs_common.cpp -o /tmp/pc_probe_$1_$2 || exit 1
done
for v in "9 8" "12 8" "8 8" "16 8" "9 16"; do
  set -- $v
  echo "== NW=$1 TX=$2"
  RS_PC_FORM=cols timeout -k 10 120 /tmp/pc_probe_$1_$2 128 128 72 || exit 1
done
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms stream cols --steps 2000
