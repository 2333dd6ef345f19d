#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, as the guide prescribes) over a python command.
#   tools/pmc_probe.sh <outdir> python3 tools/lin_sweep.py
# Summarise with: python tools/pmc_table.py <outdir>
set -e
out=$1; shift
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
  "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i + 1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d "$out/p$i" -o run --output-format csv -- "$@" > "$out/p$i.log" 2>&1
done
