cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms cols --steps 3000 || exit 1
RS_PC_INLINE=1 timeout -k 10 300 python tools/pc_sweep.py --shape 128,128,72 --forms cols --steps 3000 || exit 1
timeout -k 10 300 python tools/pc_sweep.py --shape 64,64,36 --forms rows --steps 5000 || exit 1
RS_PC_INLINE=1 timeout -k 10 300 python tools/pc_sweep.py --shape 64,64,36 --forms rows --steps 5000 || exit 1
