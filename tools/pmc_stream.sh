set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
A="python tools/pc_sweep.py --shape 128,128,72 --forms stream --steps 30 --check-steps 2"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d gpurun_out/pmcA -o run -- $A > gpurun_out/pmcA.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_WAIT_ANY --output-format csv -d gpurun_out/pmcB -o run -- $A > gpurun_out/pmcB.log 2>&1
echo done
