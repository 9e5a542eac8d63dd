#!/bin/bash
# GPU-box run of the test suite and the default bench (run from the repo root):
#   tools/gpu_check.sh <tag> [pytest selection...]
# Steps run under their own time limits; a step that times out, aborts or
# faults (124/134/137/139) ends the script, a step that merely fails does not.
tag=${1:?tag}
shift
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
mkdir -p gpurun_out
fatal() { case $1 in 124|134|137|139) return 0;; *) return 1;; esac; }
sel=("$@")
[ ${#sel[@]} -eq 0 ] && sel=(tests)
timeout -k 10 900 python -u -m pytest "${sel[@]}" -m gpu -v --timeout 300 --timeout-method thread \
    > gpurun_out/gputest_$tag.log 2>&1
rc=$?
tail -5 gpurun_out/gputest_$tag.log
if fatal $rc; then echo "tests ended with $rc: stopping"; exit $rc; fi
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
brc=$?
tail -c 600 gpurun_out/bench_$tag.json
echo "pytest rc=$rc bench rc=$brc"
exit $(( rc != 0 ? rc : brc ))
