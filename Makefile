# Builds (in-tree, so the .so files travel to the GPU box with the snapshot):
#   cause_amd/libcauseweave.so      product: gfx950 HIP kernels + C-ABI (include/causeweave.h)
#   cause_amd/libcauseweave_gen.so  synthetic workload generator (bench/tests input only)
#   oracle/liboracle.so             CPU restatement of the reference (test checker only)
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC -shared --offload-arch=$(ARCH) -Wall -Wno-unused-function
CC       ?= gcc
CXX      ?= g++

LIB     := cause_amd/libcauseweave.so
GENLIB  := cause_amd/libcauseweave_gen.so
ORACLE  := oracle/liboracle.so

HIP_SRC := cause_amd/csrc/causeweave.hip
HIP_HDR := include/causeweave.h cause_amd/csrc/cw_internal.h cause_amd/csrc/exact.hip cause_amd/csrc/k128.hip cause_amd/csrc/mappack.hip cause_amd/csrc/dist.hip cause_amd/csrc/onesweep.hip

all: $(LIB) $(GENLIB) $(ORACLE)

# build id = hash of every source of the product library: profiles/pmc_traffic.json
# records the id it was measured on, and bench.py reports traffic only for that build
BUILD_ID = $(shell cat $(HIP_SRC) $(HIP_HDR) Makefile | sha1sum | cut -c1-16)

$(LIB): $(HIP_SRC) $(HIP_HDR) Makefile
	$(HIPCC) $(HIPFLAGS) -DCW_BUILD_ID='"$(BUILD_ID)"' -Iinclude -Icause_amd/csrc $(HIP_SRC) -o $@

$(GENLIB): cause_amd/csrc/gen.cpp cause_amd/csrc/gen.h
	$(CXX) -O3 -march=x86-64-v2 -std=c++17 -fPIC -shared -Wall -pthread $< -o $@

$(ORACLE): oracle/weave_oracle.c oracle/weave_oracle.h
	$(CC) -O3 -march=x86-64-v2 -std=c11 -fPIC -shared -Wall -pthread $< -o $@

oracle: $(ORACLE)

clean:
	rm -f $(LIB) $(GENLIB) $(ORACLE)

.PHONY: all clean oracle
