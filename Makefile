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

.PHONY: all product emu unit oracle profile poison variant sanitize ubsan clean
all: product emu unit oracle sanitize

product: hartallo_amd/libhartallo_amd.so
emu: tests/emu/libhl_emu.so
unit: tests/gpu_unit/libhl_unit.so

hartallo_amd/libhartallo_amd.so: $(KSRC) $(HOSTSRC) $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) $(DEVFLAGS) -shared -o $@ $(KSRC) $(HOSTSRC)

tests/emu/libhl_emu.so: tests/emu/hl_emu.hip $(HOSTSRC) $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -O2 -DHL_FAM3=1 -shared -o $@ tests/emu/hl_emu.hip $(HOSTSRC)

tests/gpu_unit/libhl_unit.so: tests/gpu_unit/hl_unit.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(CXXFLAGS) -shared -o $@ tests/gpu_unit/hl_unit.hip

# sanitizer builds of the host code (tests/test_sanitizers.py, CPU):
#   tests/sanitize/libhl_emu_asan.so  the emulator (the kernel logic on the
#       host) under AddressSanitizer, the product's host writer (hl_writer.cpp)
#       and rate controller (hl_rc.cpp) under AddressSanitizer +
#       UndefinedBehaviorSanitizer; run with the clang ASan runtime preloaded
#   tests/sanitize/rowgate_tsan  the pipelined run's row-gated slice writers
#       (hl_writer.h RowGate) under ThreadSanitizer
# (hipcc: every -fsanitize= directly after -Xarch_host, host code only)
SANFLAGS := -std=c++17 -O1 -g -fno-omit-frame-pointer -fPIC -ffp-contract=off -Wno-unused-function -Wno-unused-variable
ASAN := -Xarch_host -fsanitize=address
UBSAN := -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined
sanitize: tests/sanitize/libhl_emu_asan.so tests/sanitize/rowgate_tsan
tests/sanitize/hl_writer_asan.o: $(CSRC)/hl_writer.cpp $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(SANFLAGS) $(ASAN) $(UBSAN) -c -o $@ $<
tests/sanitize/hl_rc_asan.o: $(CSRC)/hl_rc.cpp $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(SANFLAGS) $(ASAN) $(UBSAN) -c -o $@ $<
tests/sanitize/hl_emu_asan.o: tests/emu/hl_emu.hip $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(SANFLAGS) -DHL_FAM3=1 $(ASAN) -c -o $@ $<
tests/sanitize/libhl_emu_asan.so: tests/sanitize/hl_emu_asan.o tests/sanitize/hl_writer_asan.o tests/sanitize/hl_rc_asan.o
	$(HIPCC) --offload-arch=$(ARCH) $(ASAN) $(UBSAN) -shared-libsan -shared -o $@ $^
tests/sanitize/rowgate_tsan: tests/sanitize/rowgate_tsan.cpp $(CSRC)/hl_writer.cpp $(HDRS)
	$(HIPCC) $(SANFLAGS) -Xarch_host -fsanitize=thread -o $@ tests/sanitize/rowgate_tsan.cpp $(CSRC)/hl_writer.cpp -lpthread
# the emulator under UndefinedBehaviorSanitizer too: a 16-minute compile of
# the kernel logic, run once per change of the shift / overflow idioms
# (DESIGN.md §2); tests/test_sanitizers.py uses it when it is present
ubsan: tests/sanitize/libhl_emu_ubsan.so
tests/sanitize/libhl_emu_ubsan.so: tests/emu/hl_emu.hip $(HOSTSRC) $(HDRS)
	$(HIPCC) --offload-arch=$(ARCH) $(SANFLAGS) -DHL_FAM3=1 $(ASAN) $(UBSAN) -shared-libsan -shared -o $@ tests/emu/hl_emu.hip $(HOSTSRC)

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
	rm -f hartallo_amd/libhartallo_amd.so tests/emu/libhl_emu.so tests/gpu_unit/libhl_unit.so tests/sanitize/*.so tests/sanitize/*.o tests/sanitize/rowgate_tsan
	$(MAKE) -C oracle clean
