# Top-level build: the gfx950 product library, the oracle, the reference build.
#   make            libmtcp_gpu.so + oracle/libmtcp_oracle.so
#   make ref        oracle/_ref (needs /root/reference; this container only)
#   make golden     regenerate tests/golden from the reference
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -fPIC -std=c++17 -Wall -Wno-unused-result
LIB      := mtcp_amd/lib/libmtcp_gpu.so
SRCS     := mtcp_amd/csrc/mtcp_gpu.hip mtcp_amd/csrc/pktgen.hip mtcp_amd/csrc/rxq.hip
DEPS     := $(SRCS) mtcp_amd/csrc/dispatch.hpp mtcp_amd/csrc/rx_kernels.hpp mtcp_amd/csrc/rx_wave.hpp mtcp_amd/csrc/rx_span.hpp mtcp_amd/csrc/host_copy.hpp mtcp_amd/csrc/park.hpp mtcp_amd/csrc/wait.hpp mtcp_amd/csrc/ctx_internal.hpp mtcp_amd/csrc/flow_kernels.hpp include/mtcp_gpu.h include/mtcp_gpu_pktgen.h include/mtcp_gpu_rxq.h

.PHONY: all lib oracle ref golden examples clean tools

all: lib oracle

lib: $(LIB)

$(LIB): $(DEPS)
	mkdir -p mtcp_amd/lib
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $(SRCS)

oracle:
	$(MAKE) -C oracle

ref:
	$(MAKE) -C oracle ref

golden:
	$(MAKE) -C oracle golden

clean:
	rm -f $(LIB) tests/c/libmtcp_gpu_testing.so tests/c/rxloop tests/c/admit_test tests/c/park_test tests/c/asan_host tools/libstream_ceiling.so
	$(MAKE) -C oracle clean

# the probe tools instantiate rx_kernel's profiling / timing-probe variants
# (ABL, STAMP, XSKIP), which only a -DMTCP_GPU_TESTING build allows
TOOLFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -w -DMTCP_GPU_TESTING

tools/rx_variants: tools/rx_variants.hip mtcp_amd/csrc/rx_kernels.hpp $(LIB)
	$(HIPCC) $(TOOLFLAGS) -o $@ $< -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../mtcp_amd/lib'

tools/hbm_ceiling: tools/hbm_ceiling.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -w -o $@ $<

tools/store_probe: tools/store_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -w -o $@ $<

tools/pcie_probe: tools/pcie_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -w -o $@ $<

tools: tools/rx_variants tools/hbm_ceiling tools/store_probe tools/pcie_probe tools/wave_probe

# The test-only library: mtcp_gpu_debug_stall (tests/c/mtcp_gpu_testing.h),
# fault injection kept out of the product library
TESTLIB := tests/c/libmtcp_gpu_testing.so
$(TESTLIB): tests/c/gpu_testing.hip tests/c/mtcp_gpu_testing.h include/mtcp_gpu.h $(LIB)
	$(HIPCC) $(HIPFLAGS) -Iinclude -shared -o $@ $< -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../../mtcp_amd/lib'

# gpu_module.c driven by the RunMainLoop rx harness; the
# mTCP types come from the test doubles in tests/c/mtcp_double.  A test
# build (-DMTCP_GPU_TESTING): the fault-injection variables are read.
tests/c/rxloop: tests/c/rxloop.c mtcp_amd/io_module/gpu_module.c mtcp_amd/io_module/gpu_topo.h include/mtcp_gpu_rxq.h oracle/mtcp_oracle.c $(LIB) $(TESTLIB)
	gcc -std=gnu99 -O3 -Wall -pthread -DMTCP_GPU_TESTING -Itests/c/mtcp_double -Itests/c -Iinclude -o $@ tests/c/rxloop.c \
	    mtcp_amd/io_module/gpu_module.c oracle/mtcp_oracle.c -Lmtcp_amd/lib -Ltests/c -lmtcp_gpu -lmtcp_gpu_testing -ldl \
	    -Wl,-rpath,'$$ORIGIN/../../mtcp_amd/lib' -Wl,-rpath,'$$ORIGIN'

# park.hpp's best fit and caps, run on the GPU box (tests/test_gpu_bounded.py)
tests/c/park_test: tests/c/park_test.hip mtcp_amd/csrc/park.hpp
	$(HIPCC) --offload-arch=$(ARCH) -O2 -std=c++17 -Wall -o $@ $<

# the C ABI's host code under AddressSanitizer (host side only: the pool has
# no GPU ASan), run on the GPU box by tests/test_gpu_bounded.py
ASAN_SRCS := tests/c/asan_host.hip mtcp_amd/csrc/mtcp_gpu.hip mtcp_amd/csrc/rxq.hip mtcp_amd/csrc/pktgen.hip
tests/c/asan_host: $(ASAN_SRCS) $(DEPS)
	$(HIPCC) --offload-arch=$(ARCH) -O2 -g -std=c++17 -Wall -Wno-unused-result -Xarch_host -fsanitize=address \
	    -Xarch_host -fno-omit-frame-pointer -o $@ $(ASAN_SRCS)

# the admission / limit logic of gpu_module.c, unit-tested on the CPU
tests/c/admit_test: tests/c/admit_test.c mtcp_amd/io_module/gpu_module.c $(LIB)
	gcc -std=gnu99 -O1 -Wall -pthread -Itests/c/mtcp_double -Iinclude -o $@ tests/c/admit_test.c \
	    oracle/mtcp_oracle.c -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../../mtcp_amd/lib'

tools/wave_probe: tools/wave_probe.hip mtcp_amd/csrc/rx_span.hpp mtcp_amd/csrc/rx_wave.hpp mtcp_amd/csrc/rx_kernels.hpp $(LIB)
	$(HIPCC) $(TOOLFLAGS) -o $@ $< -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../mtcp_amd/lib'

tools/occ_probe: tools/occ_probe.hip mtcp_amd/csrc/rx_kernels.hpp $(LIB)
	$(HIPCC) $(TOOLFLAGS) -o $@ $< -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../mtcp_amd/lib'

tools/tx_probe: tools/tx_probe.hip mtcp_amd/csrc/rx_kernels.hpp $(LIB)
	$(HIPCC) $(TOOLFLAGS) -o $@ $< -Lmtcp_amd/lib -lmtcp_gpu -Wl,-rpath,'$$ORIGIN/../mtcp_amd/lib'

# bench.py's read-ceiling leg (measurement only, not the product)
tools/libstream_ceiling.so: tools/stream_ceiling.hip
	$(HIPCC) $(HIPFLAGS) -shared -o $@ $<

tools/sector_probe: tools/sector_probe.hip
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -w -o $@ $<
