set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/gputest_r5_v7.log 2>&1 || { tail -60 gpurun_out/gputest_r5_v7.log; exit 1; }
tail -2 gpurun_out/gputest_r5_v7.log
for p in 1 0 1 0; do RS_VT_POLL=$p timeout -k 10 300 python -u bench.py --library-total 0 --no-pc-stress --no-cpu-baseline --pc-calls 2000 --node-calls 300 --steps 5 > gpurun_out/bvp_$p.json 2>/dev/null || exit 1; python3 -c "import json;d=json.loads(open('gpurun_out/bvp_$p.json').read().strip().splitlines()[-1]);r=d['replay'];print('poll $p', round(d['value']/1e9,3), {k: round(v) for k,v in r.items() if k.endswith('per_s')}, r.get('publish',{}).get('messages_per_s'))"; done
timeout -k 10 300 python -u tools/pc_ab.py pyratslam_amd/libratslam_hip.so pyratslam_amd/libratslam_hip.so@RS_PC_HALO_POLL=0 --shape 64,64,36 --mode update --steps 5000 --rounds 4 > gpurun_out/ab_poll3.log 2>&1
tail -2 gpurun_out/ab_poll3.log
