# libnemohip: gfx950 kernels + C ABI (include/nemohip.h).  Cross-compiles here
# (no GPU needed); the .so travels to the GPU box with the gpurun snapshot.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result -Wno-unused-value
BUILD := build
SRCS := $(wildcard nemo_amd/csrc/*.hip)
HOST_SRCS := $(wildcard nemo_amd/csrc/*.cpp)
OBJS := $(patsubst nemo_amd/csrc/%.hip,$(BUILD)/%.o,$(SRCS)) $(patsubst nemo_amd/csrc/%.cpp,$(BUILD)/%.host.o,$(HOST_SRCS))
CXX_HOST ?= g++
HOSTFLAGS ?= -O3 -std=c++17 -fPIC -pthread -Wall
HDRS := $(wildcard nemo_amd/csrc/*.h) include/nemohip.h
LIB := nemo_amd/libnemohip.so

all: $(LIB) oracle tools

$(BUILD)/%.o: nemo_amd/csrc/%.hip $(HDRS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

# host-only parts of the library (native Molly ingest)
$(BUILD)/%.host.o: nemo_amd/csrc/%.cpp $(HDRS)
	@mkdir -p $(BUILD)
	$(CXX_HOST) $(HOSTFLAGS) -c -o $@ $<

$(LIB): $(OBJS)
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(OBJS) -pthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

# diagnostic build with in-kernel phase stamps (never shipped as libnemohip.so)
stamps: $(SRCS) $(HDRS)
	@mkdir -p $(BUILD)/stamps
	for f in $(SRCS); do $(HIPCC) $(HIPFLAGS) -DNEMO_STAMPS -c -o $(BUILD)/stamps/$$(basename $$f .hip).o $$f || exit 1; done
	$(HIPCC) $(HIPFLAGS) -shared -o nemo_amd/libnemohip_stamps.so $(BUILD)/stamps/*.o -pthread -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib

oracle:
	$(MAKE) -s -C oracle

tools:
	$(MAKE) -s -C tools

clean:
	rm -rf $(BUILD) $(LIB)
	$(MAKE) -s -C oracle clean
	$(MAKE) -s -C tools clean

.PHONY: all oracle tools clean stamps
