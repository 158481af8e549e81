#!/bin/bash
# SQ counters of the random-pattern decode table kernel: issue mix and stalls
set -o pipefail
cd $GRAFT_REPO_ROOT
MODE=decode PAT=dec_stage_kernel BENCH_ARGS="--pattern random --sdk-chunks 0" bash scripts/gpu_pmc_mode.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD"
bash scripts/gpu_splitb_pmc.sh
