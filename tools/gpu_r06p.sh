# Round-6 counter evidence (dev, GPU box): the up-projection GEMM (GELU pair) before / after the round-6 epilogue
# (before_lib = the build at 1901edc), the attention forward at both shapes, the register-weight decoder convs.
# One --pmc pass per counter group (tools/pmc_gemm.sh / tools/pmc_cmd.sh); tables by tools/pmc_table.py.
set -e
R=$GRAFT_REPO_ROOT
cd $R
S3OD_HIP_LIB=$R/before_lib/libs3od_hip.so TAG=r06_up_before OP=gelu SHAPE="65536 3072 768" bash tools/pmc_gemm.sh
cd $R && python3 tools/pmc_table.py gpurun_out/pmc_r06_up_before > gpurun_out/pmc_r06_up_before/table.txt
TAG=r06_up_after OP=gelu SHAPE="65536 3072 768" bash tools/pmc_gemm.sh
cd $R && python3 tools/pmc_table.py gpurun_out/pmc_r06_up_after > gpurun_out/pmc_r06_up_after/table.txt
cd $R && AB_ROUNDS=1 bash tools/pmc_cmd.sh r06_afwd attn_fwd tools/attn_ab.py S3OD_NONE 0
cd $R && ARMS=CONV_RW=1 bash tools/pmc_cmd.sh r06_rw "c64_rw|convT4s2_rw|conv4s2_rw" tools/conv64_bench.py
