#!/bin/bash
# SQ counter passes over k_nse_system for the assembly variants in VARS.
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmcasm; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for v in ${VARS:-base}; do
  for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_SALU"; do
    i=$((i+1)); rm -rf /tmp/pmc
    VAR=$v timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --kernel-include-regex "k_nse_system" --output-format csv -d /tmp/pmc -o pmc -- python3 $GRAFT_REPO_ROOT/tools/asm_sq.py > $OUT/probe_${v}_$i.log 2>&1 || exit $?
    find /tmp/pmc -name "*counter_collection*.csv" -exec cp {} $OUT/${v}_g$i.csv \;
  done
done
