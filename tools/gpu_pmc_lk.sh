cd /tmp && export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
MB="python tools/microbench.py lk --points 128000 --reps 2"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d gpurun_out/pmc1 -o run --output-format csv -- $MB > gpurun_out/pmc.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_MISC -d gpurun_out/pmc2 -o run --output-format csv -- $MB >> gpurun_out/pmc.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmc3 -o run --output-format csv -- $MB >> gpurun_out/pmc.log 2>&1
echo rc $?
