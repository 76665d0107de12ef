# Builds the gfx950 HIP hot path (smcdet_amd/libsmcdet_hip.so) and the C oracle.
HIPCC ?= /opt/rocm/bin/hipcc
ARCH ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-result
CSRC := smcdet_amd/csrc
SRCS := $(CSRC)/common.hip $(CSRC)/model_kernels.hip $(CSRC)/mh_kernel.hip $(CSRC)/mala_kernel.hip $(CSRC)/chain_kernel.hip $(CSRC)/smc_kernels.hip $(CSRC)/agg_kernel.hip
HDRS := $(CSRC)/device.h $(CSRC)/render.h $(CSRC)/mcmc.h $(CSRC)/tile.h include/smcdet_hip.h
OBJS := $(SRCS:.hip=.o)
LIB := smcdet_amd/libsmcdet_hip.so
DIAG_DIR := build/diag
DIAG_LIB := smcdet_amd/libsmcdet_hip_diag.so
DIAG_OBJS := $(patsubst $(CSRC)/%.hip,$(DIAG_DIR)/%.o,$(SRCS))
# build provenance: sha1 of the sources in this order (smcdet_amd/_hip.py
# SOURCES recomputes it and refuses a library built from other sources)
SRC_HASH := $(shell cat $(SRCS) $(HDRS) | sha1sum | cut -c1-40)

all: $(LIB) $(DIAG_LIB) oracle

$(CSRC)/%.o: $(CSRC)/%.hip $(HDRS)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

# the hash is compiled into common.o, so it depends on every source
$(CSRC)/common.o: $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DSMCDET_SRC_HASH=\"$(SRC_HASH)\" -c $(CSRC)/common.hip -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJS)

oracle:
	$(MAKE) -C oracle

# diagnostic build: the product's kernels plus the A/B and timing-only
# variants (radial PSF table, scalar slots, ablations, no 1/v cache), which the
# product library refuses; tests reach it through
# smcdet_amd._hip.diag_library()
diag: $(DIAG_LIB)
$(DIAG_DIR)/%.o: $(CSRC)/%.hip $(HDRS)
	mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -DSMCDET_DIAG -c $< -o $@
$(DIAG_DIR)/common.o: $(SRCS) $(HDRS)
	mkdir -p $(DIAG_DIR)
	$(HIPCC) $(HIPFLAGS) -DSMCDET_DIAG -DSMCDET_SRC_HASH=\"$(SRC_HASH)\" -c $(CSRC)/common.hip -o $@
$(DIAG_LIB): $(DIAG_OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(DIAG_OBJS)

# profiling build with in-kernel phase timestamps (scripts/trace_phases.py)
TRACE_LIB := smcdet_amd/libsmcdet_hip_trace.so
trace: $(TRACE_LIB)
$(TRACE_LIB): $(SRCS) $(HDRS)
	$(HIPCC) $(HIPFLAGS) -DSMCDET_TRACE -shared -o $@ $(SRCS)

clean:
	rm -f $(OBJS) $(LIB) $(TRACE_LIB) $(DIAG_LIB) $(DIAG_OBJS)
	$(MAKE) -C oracle clean

.PHONY: all clean oracle trace diag

# host sanitizer builds: the C oracle and the library's host side
# (-Xarch_host -fsanitize=..., device code not compiled: nothing is launched)
# with drivers that run without a GPU (tests/test_sanitizers.py)
ASAN_DIR := build/asan
ASAN_FLAGS := -fsanitize=address,undefined -fno-omit-frame-pointer -g -O1
asan: $(ASAN_DIR)/oracle_driver $(ASAN_DIR)/capi_driver

$(ASAN_DIR)/oracle_driver: scripts/asan/oracle_driver.c oracle/mh_oracle.c
	mkdir -p $(ASAN_DIR)
	gcc $(ASAN_FLAGS) -fopenmp -std=c11 -o $@ scripts/asan/oracle_driver.c -lm

ASAN_HIP := $(HIPCC) -std=c++17 -O1 -g --offload-arch=$(ARCH) -Xarch_host -fsanitize=address \
  -Xarch_host -fsanitize=undefined -Xarch_host -fno-omit-frame-pointer
ASAN_OBJS := $(patsubst $(CSRC)/%.hip,$(ASAN_DIR)/%.o,$(SRCS))
$(ASAN_DIR)/%.o: $(CSRC)/%.hip $(HDRS)
	mkdir -p $(ASAN_DIR)
	$(ASAN_HIP) -c $< -o $@
$(ASAN_DIR)/capi_driver.o: scripts/asan/capi_driver.cpp include/smcdet_hip.h
	mkdir -p $(ASAN_DIR)
	$(ASAN_HIP) -c $< -o $@
$(ASAN_DIR)/capi_driver: $(ASAN_DIR)/capi_driver.o $(ASAN_OBJS)
	$(ASAN_HIP) -o $@ $^

.PHONY: asan
