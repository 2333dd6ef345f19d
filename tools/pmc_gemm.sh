set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
export S3OD_GEMM_CFG=${CFG:-5}
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM" ; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $R/gpurun_out/pmc/p$i -o out --output-format csv -- python3 $R/tools/gemm_probe.py $SHAPE 10 > $R/gpurun_out/pmc/log$i.txt 2>&1
done
