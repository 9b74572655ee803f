source scripts/r4_call.sh
export TMPDIR=/tmp
step dpp 60 gpurun_out/dpp_rate.txt ./scripts/dpp_rate_probe
step list 60 gpurun_out/counters_list.txt rocprofv3 -L
A="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
B="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_MISC"
step pmc3 400 gpurun_out/pmc3.log bash scripts/pmc_pass.sh gpurun_out/pmc_cfg3 cfg3 "$A" "$B"
step pmc4 400 gpurun_out/pmc4.log bash scripts/pmc_pass.sh gpurun_out/pmc_cfg4 cfg4 "$A" "$B"
step prof 600 gpurun_out/prof.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 64
