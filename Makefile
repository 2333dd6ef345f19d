# Builds the C-ABI library libs3od_hip.so for gfx950 (MI355X) in-tree.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := s3od_amd/csrc
SRCS := $(wildcard $(CSRC)/*.hip)
OBJS := $(patsubst $(CSRC)/%.hip,build/%.o,$(SRCS))
HDRS := $(wildcard $(CSRC)/*.hpp)
FLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -munsafe-fp-atomics -mllvm -amdgpu-mfma-vgpr-form=1

all: s3od_amd/libs3od_hip.so

build/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p build
	$(HIPCC) $(FLAGS) -c $< -o $@

s3od_amd/libs3od_hip.so: $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC $(OBJS) -o $@

clean:
	rm -rf build s3od_amd/libs3od_hip.so

.PHONY: all clean
