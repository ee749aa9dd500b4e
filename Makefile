# Build libgachain (HIP/gfx950 kernels + C ABI + C host core), the drop-in
# CLI tools, and the test-only oracle.  In-tree outputs (git-ignored, but they
# travel to the GPU box with gpurun snapshots).
#
#   make            product: lib + tools
#   make oracle     oracle/_build/libgacoracle.so (CPU restatement, tests only)
#   make ref        oracle/_ref/* from /root/reference (needs the reference tree)

HIPCC    ?= /opt/rocm/bin/hipcc
CC       ?= gcc
PKG      := genomealignmenttools_amd
CSRC     := $(PKG)/csrc
LIBDIR   := $(PKG)/lib
BINDIR   := $(PKG)/bin
OBJDIR   := build/obj

ARCH     := gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off \
            -Iinclude -I$(CSRC) -Wall -Wno-unused-result -Wno-unused-value $(HIPEXTRA)
CFLAGS   := -O2 -mpopcnt -std=gnu11 -fPIC -Wall -ffp-contract=off -Iinclude -I$(CSRC)

HOST_SRC := $(wildcard $(CSRC)/host/*.c)
HOST_OBJ := $(patsubst $(CSRC)/host/%.c,$(OBJDIR)/host/%.o,$(HOST_SRC))
HIP_SRC  := $(CSRC)/gac_kernels.hip $(CSRC)/gac_dp.hip $(CSRC)/gac_dptree.hip $(CSRC)/gac_device.hip $(CSRC)/gac_comm.hip
HIP_OBJ  := $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(HIP_SRC))
HDRS     := include/gachain.h $(CSRC)/gac_kernels.h $(CSRC)/gac_dp.h $(wildcard $(CSRC)/host/*.h)

EXECDIR  := $(PKG)/libexec
# GPU tools: the binary lives in libexec/, bin/<tool> is a 2-line sh launcher
# that turns on transparent huge pages for malloc (glibc.malloc.hugetlb=1:
# fewer page faults on the GB-scale chain/net arrays) and host->device copies
# by blit kernels instead of the SDMA engines (HSA_ENABLE_SDMA=0: 20 vs 13
# GB/s for the genome uploads on the box, profiles/r02f_*), and execs it --
# before anything touches the GPU.  Either can be overridden from outside.
# NetFilterNonNested.perl, chainSort and chainMergeSort are host-only: in bin/.
GPU_TOOLS := scoreChain chainNet chainCleaner axtChain
HOST_TOOLS := NetFilterNonNested.perl chainSort chainMergeSort
TOOLS    := $(addprefix $(EXECDIR)/,$(GPU_TOOLS)) $(addprefix $(BINDIR)/,$(GPU_TOOLS)) \
            $(addprefix $(BINDIR)/,$(HOST_TOOLS))
TOOL_LIB_SRC := $(wildcard $(CSRC)/tools/lib/*.c)
TOOL_LIB_OBJ := $(patsubst $(CSRC)/tools/lib/%.c,$(OBJDIR)/tools/lib/%.o,$(TOOL_LIB_SRC))

all: $(LIBDIR)/libgachain.so $(LIBDIR)/libgachain_kent.so $(TOOLS)

$(OBJDIR)/host/%.o: $(CSRC)/host/%.c $(HDRS)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -c $< -o $@

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIBDIR)/libgachain.so: $(HIP_OBJ) $(HOST_OBJ)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $^ -Wl,-soname,libgachain.so -ldl

# kent-signature shims over the batch ABI (include/gachain_kent.h)
$(LIBDIR)/libgachain_kent.so: $(CSRC)/kent/gac_kent.c include/gachain_kent.h $(LIBDIR)/libgachain.so
	$(CC) $(CFLAGS) -shared $< -o $@ -L$(LIBDIR) -lgachain -Wl,-rpath,'$$ORIGIN' \
	    -Wl,-soname,libgachain_kent.so

$(OBJDIR)/tools/lib/%.o: $(CSRC)/tools/lib/%.c $(HDRS) $(wildcard $(CSRC)/tools/lib/*.h)
	@mkdir -p $(dir $@)
	$(CC) $(CFLAGS) -I$(CSRC)/tools/lib -c $< -o $@

$(EXECDIR)/%: $(CSRC)/tools/%.c $(TOOL_LIB_OBJ) $(LIBDIR)/libgachain.so $(HDRS)
	@mkdir -p $(EXECDIR)
	$(CC) $(CFLAGS) -I$(CSRC)/tools/lib $< $(TOOL_LIB_OBJ) -o $@ -L$(LIBDIR) -lgachain \
	    -Wl,-rpath,'$$ORIGIN/../lib' -lz -lm -lpthread

# host-only tools (no device): built straight into bin/
$(BINDIR)/NetFilterNonNested.perl: $(CSRC)/tools/NetFilterNonNested.perl.c $(TOOL_LIB_OBJ) $(LIBDIR)/libgachain.so $(HDRS)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -I$(CSRC)/tools/lib $< $(TOOL_LIB_OBJ) -o $@ -L$(LIBDIR) -lgachain \
	    -Wl,-rpath,'$$ORIGIN/../lib' -lz -lm -lpthread

$(BINDIR)/chainSort $(BINDIR)/chainMergeSort: $(BINDIR)/%: $(CSRC)/tools/%.c $(TOOL_LIB_OBJ) $(LIBDIR)/libgachain.so $(HDRS)
	@mkdir -p $(BINDIR)
	$(CC) $(CFLAGS) -I$(CSRC)/tools/lib $< $(TOOL_LIB_OBJ) -o $@ -L$(LIBDIR) -lgachain \
	    -Wl,-rpath,'$$ORIGIN/../lib' -lz -lm -lpthread

$(BINDIR)/%: $(EXECDIR)/%
	@mkdir -p $(BINDIR)
	printf '#!/bin/sh\np=$$(readlink -f "$$0")\nHSA_ENABLE_SDMA=$${HSA_ENABLE_SDMA:-0} GLIBC_TUNABLES="glibc.malloc.hugetlb=1$${GLIBC_TUNABLES:+:$$GLIBC_TUNABLES}" exec "$${p%%/*}/../libexec/%s" "$$@"\n' $* > $@
	chmod +x $@

oracle: oracle/_build/libgacoracle.so

# bench/test infrastructure: the whole-genome synthetic set generator (C5,
# C4) and the random-line gather ceiling probe bench.py reports k_tile against
synth: $(EXECDIR)/gac_synth $(EXECDIR)/gac_gather_ceiling

$(EXECDIR)/gac_gather_ceiling: scripts/probes/gather_ceiling.hip
	@mkdir -p $(EXECDIR)
	$(HIPCC) --offload-arch=$(ARCH) -O3 -std=c++17 -Wno-unused-result -Wno-unused-value $< -o $@

$(EXECDIR)/gac_synth: $(CSRC)/synth/gac_synth.c
	@mkdir -p $(EXECDIR)
	$(CC) -O2 -std=gnu11 -Wall $< -o $@ -lm -lpthread

oracle/_build/libgacoracle.so: oracle/gac_oracle.c
	@mkdir -p oracle/_build
	$(CC) -O2 -std=gnu11 -fPIC -shared -Wall $< -o $@ -lm

ref:
	$(MAKE) -f oracle/ref.mk -j8

clean:
	rm -rf build $(LIBDIR) $(BINDIR) $(EXECDIR) oracle/_build

.PHONY: all oracle synth ref clean

# TEST INFRASTRUCTURE: axtChain's host half (front end + kd-tree DP) on a CPU
# stand-in of the device ABI, for profiling in GPU-less containers.  Not part
# of `all`; never shipped (oracle/cpu_gac_stub.c).
cpu-axtchain: oracle/_build/axtChain_cpu

oracle/_build/axtChain_cpu: $(CSRC)/tools/axtChain.c $(CSRC)/host/gac_axtchain.c \
		$(CSRC)/host/gac_host.c oracle/cpu_gac_stub.c $(TOOL_LIB_SRC)
	@mkdir -p oracle/_build
	$(CC) -O2 -g -mpopcnt -std=gnu11 -Wall -ffp-contract=off -Iinclude -I$(CSRC) -I$(CSRC)/host -I$(CSRC)/tools/lib $^ \
	    -o $@ -lz -lm -lpthread $(CPU_EXTRA)

# chainNet -rescore on the same stand-in: the sparse genome upload's word
# runs are checked on CPU (the stand-in poisons every word outside them)
cpu-chainnet: oracle/_build/chainNet_cpu

oracle/_build/chainNet_cpu: $(CSRC)/tools/chainNet.c $(CSRC)/host/gac_net.c \
		$(CSRC)/host/gac_host.c oracle/cpu_gac_stub.c $(TOOL_LIB_SRC)
	@mkdir -p oracle/_build
	$(CC) -O2 -g -mpopcnt -std=gnu11 -Wall -ffp-contract=off -Iinclude -I$(CSRC) -I$(CSRC)/host -I$(CSRC)/tools/lib $^ \
	    -o $@ -lz -lm -lpthread $(CPU_EXTRA)

.PHONY: cpu-axtchain cpu-chainnet

# A/B probe builds of libgachain with extra compile flags (loaded by the
# Python binding under GAC_LIB_VARIANT=NAME): make variant NAME=mb7 VFLAGS=-DGAC_TILE_MINB=7
# (VSRC=DIR: the .hip sources and kernel headers from DIR instead, e.g. an
# earlier commit's, extracted with git show)
VSRC ?= $(CSRC)
variant: $(HOST_OBJ)
	@mkdir -p build/variants/$(NAME) $(LIBDIR)/variants/$(NAME)
	for f in $(notdir $(HIP_SRC)); do $(HIPCC) -I$(VSRC) $(HIPFLAGS) $(VFLAGS) -c $(VSRC)/$$f -o build/variants/$(NAME)/$$(basename $$f .hip).o || exit 1; done
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $(LIBDIR)/variants/$(NAME)/libgachain.so \
	    build/variants/$(NAME)/*.o $(HOST_OBJ) -Wl,-soname,libgachain.so
.PHONY: variant

# chainCleaner on the same stand-in (CPU profiling of its host loop)
cpu-chaincleaner: oracle/_build/chainCleaner_cpu

oracle/_build/chainCleaner_cpu: $(CSRC)/tools/chainCleaner.c $(CSRC)/host/gac_net.c \
		$(CSRC)/host/gac_host.c oracle/cpu_gac_stub.c $(TOOL_LIB_SRC)
	@mkdir -p oracle/_build
	$(CC) -O2 -g -mpopcnt -std=gnu11 -Wall -ffp-contract=off -Iinclude -I$(CSRC) -I$(CSRC)/host -I$(CSRC)/tools/lib $^ \
	    -o $@ -lz -lm -lpthread $(CPU_EXTRA)

.PHONY: cpu-chaincleaner
