set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_view_templates_gpu.py -m gpu -k "stream" > gpurun_out/vt_stream.log 2>&1 || { tail -30 gpurun_out/vt_stream.log; exit 1; }
tail -2 gpurun_out/vt_stream.log
for g in 0 1 2 5 10; do RS_VT_UP_GROUP=$g timeout -k 10 300 python -u bench.py --library-total 0 --no-pc-stress --no-replay --no-cpu-baseline --pc-calls 3000 --node-calls 500 > gpurun_out/bq_$g.json 2>/dev/null || exit 1; python3 -c "import json;d=json.loads(open('gpurun_out/bq_$g.json').read().strip().splitlines()[-1]);t=d['template_scan'];p=d['pose_cell'];print('group $g', round(d['value']/1e9,3), round(t['pcie_inclusive_compares_per_s']/1e9,3), round(t['pcie_inclusive_per_batch_compares_per_s']/1e9,3), 'upd', round(1e6/p['update_calls_per_s'],2), 'ties', p.get('update_near_tie_calls'))"; done
for sh in 21,21,36 64,64,36; do timeout -k 10 200 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_EXPORT=last --shape $sh --mode node --steps 2000 --rounds 3 > gpurun_out/ab_node_$sh.log 2>&1; tail -2 gpurun_out/ab_node_$sh.log; done
timeout -k 10 300 python -u tools/pc_call_anatomy.py '' --calls 10000 > gpurun_out/anat6.log 2>&1
cat gpurun_out/anat6.log
