# Builds the C-ABI library libs3od_hip.so for gfx950 (MI355X) in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := s3od_amd/csrc
SRCS := $(wildcard $(CSRC)/*.hip)
OBJS := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.hpp)
FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1

all: s3od_amd/libs3od_hip.so

# attention: no SLP vectorisation -- hipcc packs the P*dP / P*V products into v_pk_mul_f32 on
# register pairs that do not match the bf16 packing, then repairs them with v_mov / v_alignbit /
# v_perm (dK/dV loop: 185 -> 145 VALU per 64 MFMA without it; attention backward 3144 -> 3019 us at
# bs 16, N 4101, same box); packed f32 VALU beside MFMAs
# is an anti-lever on CDNA4 anyway
ATTN_FLAGS := -fno-slp-vectorize

build/attention.o: $(CSRC)/attention.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(FLAGS) $(ATTN_FLAGS) -c $< -o $@

# the LDS-DMA 3x3 weight gradient and the 4-wave 256x256 GEMM keep their MFMA accumulators in AGPRs (no VGPR
# form; see the file headers)
build/gemm_q.o: $(CSRC)/gemm_q.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(filter-out -mllvm -amdgpu-mfma-vgpr-form=1,$(FLAGS)) -c $< -o $@

build/wgrad_dma.o: $(CSRC)/wgrad_dma.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(filter-out -mllvm -amdgpu-mfma-vgpr-form=1,$(FLAGS)) -c $< -o $@

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

s3od_amd/libs3od_hip.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -lhipblaslt -o $@

# dev: the ping-pong kernels of gemm_ops.hip with the block timeline compiled in (tools/pp_timeline.py)
timeline: $(OBJS)
	@mkdir -p build_tl tl_lib
	$(HIPCC) $(FLAGS) -DS3OD_TIMELINE -c $(CSRC)/gemm_ops.hip -o build_tl/gemm_ops.o
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(filter-out build/gemm_ops.o,$(OBJS)) build_tl/gemm_ops.o -lhipblaslt -o tl_lib/libs3od_hip.so

clean:
	rm -rf build s3od_amd/libs3od_hip.so

.PHONY: all clean timeline
