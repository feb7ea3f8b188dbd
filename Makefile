# Builds (for gfx950):
#   hartallo_amd/libhartallo_amd.so  the product: HIP kernels + host writer + C ABI
#   tests/emu/libhl_emu.so           test-only host build of the kernel logic
#   tests/gpu_unit/libhl_unit.so     test-only GPU unit kernels (coop pipeline vs scalar primitives)
#   oracle/...                       test-only CPU oracle and reference build (oracle/Makefile)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CSRC    := hartallo_amd/csrc
HDRS    := $(wildcard $(CSRC)/*.h) include/hartallo_amd.h
# -ffp-contract=off: the RDO costs are IEEE double and must round exactly like the reference
CXXFLAGS := -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable

.PHONY: all product emu unit oracle profile clean
all: product emu unit oracle

product: hartallo_amd/libhartallo_amd.so
emu: tests/emu/libhl_emu.so
unit: tests/gpu_unit/libhl_unit.so

hartallo_amd/libhartallo_amd.so: $(CSRC)/hl_encoder.hip $(CSRC)/hl_writer.cpp $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ $(CSRC)/hl_encoder.hip $(CSRC)/hl_writer.cpp

tests/emu/libhl_emu.so: tests/emu/hl_emu.hip $(CSRC)/hl_writer.cpp $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -O2 -shared -o $@ tests/emu/hl_emu.hip $(CSRC)/hl_writer.cpp

tests/gpu_unit/libhl_unit.so: tests/gpu_unit/hl_unit.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ tests/gpu_unit/hl_unit.hip

# profiling build: same library with per-phase clock64 counters (tools/phase_profile.py)
profile: build/prof/hartallo_amd/libhartallo_amd.so
build/prof/hartallo_amd/libhartallo_amd.so: $(CSRC)/hl_encoder.hip $(CSRC)/hl_writer.cpp $(HDRS)
	mkdir -p build/prof/hartallo_amd
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -DHL_PROFILE=1 -shared -o $@ $(CSRC)/hl_encoder.hip $(CSRC)/hl_writer.cpp

oracle:
	$(MAKE) -C oracle

clean:
	rm -f hartallo_amd/libhartallo_amd.so tests/emu/libhl_emu.so tests/gpu_unit/libhl_unit.so
	$(MAKE) -C oracle clean
