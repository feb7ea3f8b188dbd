# Builds (for gfx950):
#   hartallo_amd/libhartallo_amd.so  the product: HIP kernels + host writer + C ABI
#   tests/emu/libhl_emu.so           test-only host build of the kernel logic
#   tests/gpu_unit/libhl_unit.so     test-only GPU unit kernels (coop pipeline vs scalar primitives)
#   oracle/...                       test-only CPU oracle and reference build (oracle/Makefile)
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
CSRC    := hartallo_amd/csrc
HDRS    := $(wildcard $(CSRC)/*.h) include/hartallo_amd.h
HOSTSRC := $(CSRC)/hl_writer.cpp $(CSRC)/hl_rc.cpp
# the product kernels, and k_pipeline again with the 8x8-family helpers (runs of one picture)
KSRC    := $(CSRC)/hl_encoder.hip $(CSRC)/hl_encoder_fam3.hip
# -ffp-contract=off: the RDO costs are IEEE double and must round exactly like the reference
CXXFLAGS := -std=c++17 -O3 -fPIC -ffp-contract=off -Wall -Wno-unused-function -Wno-unused-variable
# device code scheduling of the product: the ILP-iterative strategy shortens
# the latency-bound macroblock decision (1088p bench +1.5 %, bit-exact;
# profiles/r02_sched_strategy_ab.log)
DEVFLAGS := -mllvm -amdgpu-sched-strategy=iterative-ilp

.PHONY: all product emu unit oracle profile poison variant clean
all: product emu unit oracle

product: hartallo_amd/libhartallo_amd.so
emu: tests/emu/libhl_emu.so
unit: tests/gpu_unit/libhl_unit.so

hartallo_amd/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) -shared -o $@ $(KSRC) $(HOSTSRC)

tests/emu/libhl_emu.so: tests/emu/hl_emu.hip $(HOSTSRC) $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -O2 -DHL_FAM3=1 -shared -o $@ tests/emu/hl_emu.hip $(HOSTSRC)

tests/gpu_unit/libhl_unit.so: tests/gpu_unit/hl_unit.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ tests/gpu_unit/hl_unit.hip

# profiling build: same library (same device scheduling flags) with per-phase
# clock64 counters (tools/phase_profile.py)
profile: build/prof/hartallo_amd/libhartallo_amd.so
build/prof/hartallo_amd/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	mkdir -p build/prof/hartallo_amd
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) -DHL_PROFILE=1 -shared -o $@ $(KSRC) $(HOSTSRC)

# debug builds: LDS poisoned before every macroblock with two different salts
# (tools/gpu_diag.sh); any output difference names a read of uninitialised LDS
poison: build/poison1/libhartallo_amd.so build/poison2/libhartallo_amd.so
build/poison%/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	mkdir -p build/poison$*
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) -DHL_POISON_LDS=$* -shared -o $@ $(KSRC) $(HOSTSRC)

# memory-scope variants of the pipelined run's fences (diagnostics)
scopes: build/acqsys/libhartallo_amd.so build/relacqsys/libhartallo_amd.so
build/acqsys/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	mkdir -p build/acqsys
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) '-DHL_ACQ_SCOPE=""' -shared -o $@ $(KSRC) $(HOSTSRC)
build/relacqsys/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	mkdir -p build/relacqsys
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) '-DHL_ACQ_SCOPE=""' '-DHL_REL_SCOPE=""' -shared -o $@ $(KSRC) $(HOSTSRC)

# variants of the product for A/B runs: make variant V=<name> VDEFS="-D..."
variant: build/$(V)/libhartallo_amd.so
build/$(V)/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	mkdir -p build/$(V)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) $(VDEFS) -shared -o $@ $(KSRC) $(HOSTSRC)

oracle: product  # oracle/_ref/drop_in_enc links the product library
	$(MAKE) -C oracle

clean:
	rm -f hartallo_amd/libhartallo_amd.so tests/emu/libhl_emu.so tests/gpu_unit/libhl_unit.so
	$(MAKE) -C oracle clean
