cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for t in 1000 10000; do
timeout -k 10 300 python tools/scan_ab.py tools/ab/old.so tools/ab/nh2.so tools/ab/nh1.so --templates $t --reps 20 || exit $?
done
timeout -k 10 300 python tools/scan_ab.py tools/ab/old.so tools/ab/nh1.so --templates 100000 --reps 3 || exit $?
