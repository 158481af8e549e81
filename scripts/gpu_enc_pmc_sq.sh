#!/bin/bash
# SQ counters of the encode kernel (issue mix, waits, LDS) on the default 1024-object step
set -o pipefail
cd $GRAFT_REPO_ROOT
MODE=encode PAT=enc_dma BENCH_ARGS="--sdk-chunks 0" bash scripts/gpu_pmc_mode.sh \
  "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE" \
  "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
