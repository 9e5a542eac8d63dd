set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest_r4_v6.log 2>&1 || { tail -40 gpurun_out/gputest_r4_v6.log; exit 1; }
tail -2 gpurun_out/gputest_r4_v6.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r4_v6.json 2> gpurun_out/bench_r4_v6.err || { tail -30 gpurun_out/bench_r4_v6.err; exit 1; }
python - <<'PY'
import json
d=json.loads(open('gpurun_out/bench_r4_v6.json').read().strip().splitlines()[-1])
pc=d['pose_cell']
print('value', d['value'], 'frac', d['roofline']['frac'], 'steps/s', pc['steps_per_s'], 'us', pc['us_per_step'], 'dev', pc['device_us_per_step'], 'update/s', pc['update_calls_per_s'])
for k,v in pc['node_step'].items():
    if isinstance(v, dict): print(k, v['update_us'], v['update_plus_read_us'], v['update_plus_read_eager_us'])
s=d.get('pose_cell_stress') or {}
print('stress', s.get('us_per_step'), s.get('roofline',{}).get('frac'))
PY
timeout -k 10 1000 bash tools/profile_r2.sh r4_v6 pc64 pc128 headline stress library bench > gpurun_out/prof_r4_v6.log 2>&1 || { tail -20 gpurun_out/prof_r4_v6.log; exit 1; }
tail -1 gpurun_out/prof_r4_v6.log
