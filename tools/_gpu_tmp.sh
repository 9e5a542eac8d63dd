set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_view_templates_gpu.py -k "stream" -m gpu > gpurun_out/gputest_sched.log 2>&1 || { tail -30 gpurun_out/gputest_sched.log; exit 1; }
RS_VT_UP_SCHED=tail1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_view_templates_gpu.py -k "stream" -m gpu >> gpurun_out/gputest_sched.log 2>&1 || { tail -30 gpurun_out/gputest_sched.log; exit 1; }
grep passed gpurun_out/gputest_sched.log
A="--no-pc-stress --no-replay --library-total 0 --no-cpu-baseline --pc-steps 200 --pc-calls 200 --node-calls 100"
for r in 1 2 3; do
for cfg in "default 0" "tail1 0" "tail1 3" "default 3"; do
set -- $cfg
RS_VT_UP_SCHED=$1 RS_VT_UP_GROUP=$2 timeout -k 10 200 python -u bench.py $A > gpurun_out/bench_sched_$1_$2.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/bench_sched_$1_$2.json').read().strip().splitlines()[-1]); t=d['template_scan']; print('$1 g$2', round(d['value']/1e9,3), round(t['pcie_inclusive_compares_per_s']/1e9,3))"
done
done
