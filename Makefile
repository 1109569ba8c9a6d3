# Top-level build. Everything lands in-tree (git-ignored, travels to the GPU box).
#   make            librt_hip.so (HIP, gfx950) + the oracle (test infrastructure)
PKG      := cpu-ray-tracing-implementation_amd
BUILD    := $(PKG)/build
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall --offload-arch=$(ARCH)

LIB_SRCS := $(PKG)/csrc/rt_kernels.hip $(PKG)/csrc/scene_compile.cpp
LIB_HDRS := $(PKG)/csrc/rt_device.h $(PKG)/csrc/rt_scene.h $(PKG)/csrc/scene_compile.h include/rt_hip.h

all: $(BUILD)/librt_hip.so oracle

$(BUILD)/librt_hip.so: $(LIB_SRCS) $(LIB_HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(LIB_SRCS)

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean
