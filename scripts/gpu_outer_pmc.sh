#!/bin/bash
# SQ counters of the OuterCoder matrix kernel (LDS array busy, bank conflicts, issue stalls)
set -o pipefail
cd $GRAFT_REPO_ROOT
MODE=outer PAT=rs16_matrix BENCH_ARGS="--sdk-chunks 0" bash scripts/gpu_pmc_mode.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE" \
  "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_SMEM"
