cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py --gpus 2 --same-device --steps 3 --warmup 1 --no-cpu-baseline --no-pc-stress --no-replay > gpurun_out/bench_2same.json 2> gpurun_out/bench_2same.err; echo "rc=$?"
tail -c 1500 gpurun_out/bench_2same.json; tail -5 gpurun_out/bench_2same.err
