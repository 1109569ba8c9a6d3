# Top-level build. Everything lands in-tree (git-ignored, travels to the GPU box).
#   make            librt_hip.so (HIP, gfx950) + the oracle (test infrastructure)
PKG      := cpu-ray-tracing-implementation_amd
BUILD    := $(PKG)/build
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
# -ffp-contract=on: contraction decided per source expression, so the persistent and the
# launch-per-K kernels (same shade code, different inlining) produce bit-identical images.
# -fno-slp-vectorize: the SLP vectoriser paired fp32 values into packed-math operands ((x, -x) pairs
# for v_pk_mul_f32 / v_pk_fma_f32), which hold two registers and issue in 4 cycles for 2 lanes' worth --
# no faster than two plain fp32 ops on gfx950 (tools/valu_rates) -- and those pairs were what spilled:
# off, the fp32 wide and volume kernels have no scratch, and C2 fp32 21.2 -> 20.4 ms/frame, C3 fp32
# 51.0 -> 49.7, C5 fp32 1,249 -> 1,179 (r04f)
HIPFLAGS ?= -O3 -std=c++17 -fPIC -Wall -ffp-contract=on -fno-slp-vectorize --offload-arch=$(ARCH)

LIB_SRCS := $(PKG)/csrc/rt_kernels.hip $(PKG)/csrc/rt_multi.hip $(PKG)/csrc/scene_compile.cpp
LIB_HDRS := $(PKG)/csrc/rt_device.h $(PKG)/csrc/rt_sin.h $(PKG)/csrc/rt_scene.h $(PKG)/csrc/scene_compile.h include/rt_hip.h

CXX      ?= g++
CXXFLAGS ?= -O2 -std=c++17 -fPIC -Wall -Wextra -Wno-unused-parameter
RT_HDRS  := $(wildcard $(PKG)/rt/*.h) include/rt_hip.h

all: $(BUILD)/librt_hip.so $(BUILD)/librt_scenes.so $(BUILD)/rt_main tools/valu_rates tools/l1_rates oracle

# one object per source, so a host-only change does not recompile the kernels
LIB_OBJS := $(BUILD)/obj/rt_kernels.o $(BUILD)/obj/rt_multi.o $(BUILD)/obj/scene_compile.o
$(BUILD)/obj/%.o: $(PKG)/csrc/%.hip $(LIB_HDRS)
	@mkdir -p $(BUILD)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(BUILD)/obj/%.o: $(PKG)/csrc/%.cpp $(LIB_HDRS)
	@mkdir -p $(BUILD)/obj
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<
$(BUILD)/librt_hip.so: $(LIB_OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(LIB_OBJS) -ldl

# development build with correctly rounded fp32 math (scripts/dev_divergence.py --lib)
precise: $(BUILD)/librt_hip_precise.so
$(BUILD)/librt_hip_precise.so: $(LIB_SRCS) $(LIB_HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DRT_PRECISE_F32 -shared -o $@ $(LIB_SRCS)

# development build printing every traced segment (scripts/dev_sample_trace.py)
trace: $(BUILD)/librt_hip_trace.so
$(BUILD)/librt_hip_trace.so: $(LIB_SRCS) $(LIB_HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DRT_DEBUG_TRACE -shared -o $@ $(LIB_SRCS)

# development build with per-section shader clocks (scripts/dev_sections.py)
sections: $(BUILD)/librt_hip_sections.so
$(BUILD)/librt_hip_sections.so: $(LIB_SRCS) $(LIB_HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -DRT_SECTION_CLOCKS -shared -o $@ $(LIB_SRCS)

# the reference's config scenes written against the drop-in plugin surface (+ rtsc_* C ABI for tests)
$(BUILD)/librt_scenes.so: $(PKG)/scenes/config_scenes.cpp $(PKG)/scenes/config_scenes.h $(RT_HDRS) $(BUILD)/librt_hip.so
	$(CXX) $(CXXFLAGS) -shared -o $@ $(PKG)/scenes/config_scenes.cpp -L$(BUILD) -lrt_hip -Wl,-rpath,'$$ORIGIN'

# the reference's main.cc driver on the plugin surface
$(BUILD)/rt_main: examples/main.cc $(PKG)/scenes/config_scenes.cpp $(PKG)/scenes/config_scenes.h $(RT_HDRS) $(BUILD)/librt_hip.so
	$(CXX) $(CXXFLAGS) -o $@ examples/main.cc $(PKG)/scenes/config_scenes.cpp -L$(BUILD) -lrt_hip -Wl,-rpath,'$$ORIGIN'

# measurement tool: issue cost of single VALU opcodes (scripts/valu_rates.sh, bench.py's fp64 roofline)
tools/valu_rates: tools/valu_rates.hip
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<
# measurement tool: L1 (TA/TD) cost of a vector load by width, active lanes and address pattern
tools/l1_rates: tools/l1_rates.hip
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -o $@ $<

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf $(BUILD)
	$(MAKE) -C oracle clean

.PHONY: all oracle clean precise trace sections
