# Builds the HIP extension in-tree: conv-tasnet_amd/libctn_hip.so (gfx950 only).
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
PKG      := conv-tasnet_amd
SRC      := $(wildcard $(PKG)/csrc/*.hip)
OBJ      := $(patsubst $(PKG)/csrc/%.hip,build/%.o,$(SRC))
HDR      := $(wildcard $(PKG)/csrc/*.h) include/ctn.h
# device codegen: MFMA accumulators in VGPRs (no accvgpr copies around the MFMAs;
# gemm_cols 83 -> 55 us).  IEEE mode stays on: turning it off measured neutral
# everywhere except the NORM_BWD WS GEMM, which it slowed by 9%.
DEVFLAGS := -mllvm -amdgpu-mfma-vgpr-form
CXXFLAGS := -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function -Iinclude $(DEVFLAGS)
LIB      := $(PKG)/libctn_hip.so

all: $(LIB)

build/%.o: $(PKG)/csrc/%.hip $(HDR) Makefile
	@mkdir -p build
	$(HIPCC) $(CXXFLAGS) -c $< -o $@

$(LIB): $(OBJ)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJ)

clean:
	rm -rf build $(LIB)

.PHONY: all clean

# bound-finding microbenchmarks (not part of the library): build/ws_bench_<bits>
MB_EXPS := 0 1 2 3 4 8 12
microbench: $(patsubst %,build/ws_bench_%,$(MB_EXPS))
build/ws_bench_%: tools/microbench/ws_bench.hip $(PKG)/csrc/ctn_gemm_ws.hip $(HDR)
	@mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -Iinclude $(DEVFLAGS) -DCTN_WS_EXP=$* $< -o $@

.PHONY: microbench

# dual-GEMM bound-finding microbenchmarks: build/dual_bench_<bits>
DU_EXPS := 0 12 13 14 28 76 92 94 222
dualbench: $(patsubst %,build/dual_bench_%,$(DU_EXPS))
build/dual_bench_%: tools/microbench/dual_bench.hip $(PKG)/csrc/ctn_gemm_dual.hip $(HDR)
	@mkdir -p build
	$(HIPCC) -O3 -std=c++17 --offload-arch=$(ARCH) -Iinclude $(DEVFLAGS) -DCTN_DU_EXP=$* $< -o $@

.PHONY: dualbench
