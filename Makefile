# Builds the HIP extension in-tree: conv-tasnet_amd/libctn_hip.so (gfx950 only).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := conv-tasnet_amd
SRC      := $(wildcard $(PKG)/csrc/*.hip)
OBJ      := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRC))
HDR      := $(wildcard $(PKG)/csrc/*.h) include/ctn.h
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude
LIB      := $(PKG)/libctn_hip.so

all: $(LIB)

build/%.o: $(PKG)/csrc/%.hip $(HDR)
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean
