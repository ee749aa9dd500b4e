# oracle/ref.mk -- compile the REFERENCE tools from the read-only sources under
# /root/reference into oracle/_ref/ (test infrastructure only: used to pin the
# CPU restatement in oracle/gac_oracle.c, to generate the golden fixtures in
# tests/golden/, and as bench.py's cpu_baseline leg).
#
# This is our own short recipe: it compiles the reference's C files directly
# with gcc; it does NOT run the reference's build system and writes nothing
# under /root/reference.  No reference source is copied into the repo.
#
#   make -f oracle/ref.mk            (from the repo root)
#
# Notes
#  * kent/src/lib/linefile.c #includes "htslib/tbx.h" (header present in the
#    reference tree) and references the tabix/hts reader (lineFileOnTabix...).
#    Building htslib would need its generated version.h, so htslib is NOT
#    built; the ten hts_*/tbx_* symbols stay unresolved at link time
#    (--warn-unresolved-symbols).  They are only reachable for tabix-indexed
#    URLs, never on the chain-scoring path.
#  * -fcommon: kent has tentative definitions in headers (GCC>=10 default is
#    -fno-common).  No -march / -ffp-contract: same FP as the reference build
#    (x86-64 SSE2, no FMA).
#  * COPT matches kent's common.mk default (-O -g); tools get -O2.

REF      ?= /root/reference
K        := $(REF)/kent/src
OUT      ?= oracle/_ref
OBJ      := $(OUT)/obj
CC       ?= gcc
DEFS     := -D_FILE_OFFSET_BITS=64 -D_LARGEFILE_SOURCE -D_GNU_SOURCE -DMACHTYPE_x86_64
KCFLAGS  := -O -g -fcommon -fPIC $(DEFS) -I$(K)/inc -I$(K)/hg/inc -I$(K)/htslib -w
TCFLAGS  := -O2 -fcommon $(DEFS) -I$(K)/inc -I$(K)/hg/inc -w
LIBS     := -lm -lz -lssl -lcrypto -pthread -Wl,--warn-unresolved-symbols

# kent/src/lib files that do not compile here (no png/uuid headers) or are
# not on any tool's path (need htslib internals / windows).
SKIP     := bamFile knetUdc oswin9x pngwrite uuid vcf
LIBSRC   := $(filter-out $(addprefix $(K)/lib/,$(addsuffix .c,$(SKIP))),$(wildcard $(K)/lib/*.c))
LIBOBJ   := $(patsubst $(K)/lib/%.c,$(OBJ)/lib/%.o,$(LIBSRC))
HGOBJ    := $(OBJ)/hg/chainNet.o

TOOLS    := $(OUT)/scoreChain $(OUT)/chainNet $(OUT)/chainCleaner \
            $(OUT)/axtChain $(OUT)/chainSort $(OUT)/chainMergeSort $(OUT)/netSyntenic

all: $(TOOLS) $(OUT)/kentref

$(OBJ)/lib/%.o: $(K)/lib/%.c
	@mkdir -p $(dir $@)
	$(CC) $(KCFLAGS) -c $< -o $@

$(OBJ)/hg/chainNet.o: $(K)/hg/lib/chainNet.c
	@mkdir -p $(dir $@)
	$(CC) $(KCFLAGS) -c $< -o $@

$(OUT)/jkweb.a: $(LIBOBJ)
	rm -f $@ && ar rcs $@ $^

$(OUT)/scoreChain: $(REF)/src/scoreChain/scoreChain.c $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(OUT)/jkweb.a $(LIBS) 2>/dev/null

$(OUT)/chainNet: $(REF)/src/chainNet/chainNet.c $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(OUT)/jkweb.a $(LIBS) 2>/dev/null

$(OUT)/chainCleaner: $(REF)/src/chainCleaner/chainCleaner.c $(HGOBJ) $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(HGOBJ) $(OUT)/jkweb.a $(LIBS) 2>/dev/null

$(OUT)/axtChain: $(K)/hg/mouseStuff/axtChain/axtChain.c $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(OUT)/jkweb.a $(LIBS) 2>/dev/null

$(OUT)/chainSort: $(K)/hg/mouseStuff/chainSort/chainSort.c $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(OUT)/jkweb.a $(LIBS) 2>/dev/null

$(OUT)/chainMergeSort: $(K)/hg/mouseStuff/chainMergeSort/chainMergeSort.c $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(OUT)/jkweb.a $(LIBS) 2>/dev/null

# netSyntenic: adds the type/qFar/qDup fields NetFilterNonNested's synteny
# modes read (goldens for those modes; not on the hot path)
$(OUT)/netSyntenic: $(K)/hg/mouseStuff/netSyntenic/netSyntenic.c $(HGOBJ) $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) $< -o $@ $(HGOBJ) $(OUT)/jkweb.a $(LIBS) 2>/dev/null

# The reference's kent objects driven by our harness (the reference's own
# chainSubsetOnT + chainCalcScore, scoreChain's local-score loop restated) --
# golden generation and the cpu_baseline "reference" leg.
$(OUT)/kentref: oracle/ref_harness.c oracle/kentapi_workload.inc $(OUT)/jkweb.a
	$(CC) $(TCFLAGS) -std=gnu99 -I$(K)/inc -Ioracle $< -o $@ $(OUT)/jkweb.a $(LIBS)

clean:
	rm -rf $(OUT)

.PHONY: all clean
