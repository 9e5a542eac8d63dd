set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocprofv3 --list-avail > gpurun_out/pmc_avail.txt 2>&1 || true
grep -i -E "ICACHE|IFETCH|SQC_" gpurun_out/pmc_avail.txt | head -40
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/icache -o run -- python tools/scan_profile.py pc --shape 64,64,36 --steps 400 > gpurun_out/icache.log 2>&1; echo rc=$?
tail -3 gpurun_out/icache.log
