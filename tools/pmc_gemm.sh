# rocprofv3 counter passes over one GEMM-engine op (tools/gemm_probe.py), one pass per counter group, plus a kernel
# trace; results under gpurun_out/pmc_<TAG>/ (dev tool, run on the GPU box):
#   TAG=upfwd OP=gelu SHAPE="65536 3072 768" bash tools/pmc_gemm.sh
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
D=$R/gpurun_out/pmc_${TAG:-x}
mkdir -p $D
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $D/trace -o out --output-format csv -- python3 $R/tools/gemm_probe.py $OP $SHAPE 10 > $D/log0.txt 2>&1
i=0
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $C -d $D/p$i -o out --output-format csv -- python3 $R/tools/gemm_probe.py $OP $SHAPE 10 > $D/log$i.txt 2>&1
done
