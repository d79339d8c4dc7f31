# Builds libdeltareplay.so (HIP for gfx950 + host C++) in-tree, and the CPU oracle baseline.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
CSRC := delta_amd/csrc
LIB := delta_amd/libdeltareplay.so
HIP_SRCS := $(CSRC)/engine.hip $(CSRC)/k_json.hip $(CSRC)/k_parquet.hip $(CSRC)/k_snappy.hip $(CSRC)/k_replay.hip $(CSRC)/k_util.hip $(CSRC)/k_shard.hip $(CSRC)/k_filter.hip $(CSRC)/k_index.hip $(CSRC)/k_encode.hip
CXX_SRCS := $(CSRC)/parquet_meta.cpp $(CSRC)/log_segment.cpp $(CSRC)/json_host.cpp $(CSRC)/snappy_host.cpp
OBJDIR := build/obj
HIP_OBJS := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRCS))
CXX_OBJS := $(patsubst $(CSRC)/%.cpp,$(OBJDIR)/%.o,$(CXX_SRCS))
HDRS := $(wildcard $(CSRC)/*.h) include/deltareplay.h
HIPFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Wno-unused-variable
CXXFLAGS := -O2 -std=c++17 -fPIC -Wall

JL_HOST := build/libjsonlane_host.so
# the same library with the tape kernels' LDS index checks (k_json.hip -DDR_BOUNDS_CHECK;
# tests/test_gpu_bounds.py loads it through DR_LIB)
LIB_BOUNDS := delta_amd/libdeltareplay_bounds.so
BOUNDS_OBJS := $(filter-out $(OBJDIR)/k_json.o,$(HIP_OBJS)) $(OBJDIR)/k_json_bounds.o

all: $(LIB) $(LIB_BOUNDS) oracle $(JL_HOST)

# host build of the K1 line walker, fuzzed against Python json by tests/test_json_lane.py
$(JL_HOST): tests/native/json_lane_host.cpp $(CSRC)/json_lane.h
	@mkdir -p build
	g++ -O2 -std=c++17 -fPIC -shared -Wall -o $@ $<


$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.cpp $(HDRS)
	@mkdir -p $(OBJDIR)
	g++ $(CXXFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS) $(CXX_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

$(OBJDIR)/k_json_bounds.o: $(CSRC)/k_json.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DDR_BOUNDS_CHECK -c $< -o $@

$(LIB_BOUNDS): $(BOUNDS_OBJS) $(CXX_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $^

oracle:
	$(MAKE) -C oracle

clean:
	rm -rf build $(LIB) $(LIB_BOUNDS)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle
