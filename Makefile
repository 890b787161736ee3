# Build recipe for the MI355X FEC engine.
#   make            -> quic_amd/libquic_fec.so (gfx950) + oracle (and oracle/_ref when
#                      /root/reference is present)
#   make lib        -> the product library only
# hipcc cross-compiles gfx950 code objects without a GPU.

ROOT    := $(dir $(abspath $(lastword $(MAKEFILE_LIST))))
CSRC    := $(ROOT)quic_amd/csrc
LIB     := $(ROOT)quic_amd/libquic_fec.so
TABLES  := $(ROOT)quic_amd/data/cauchy_256_tables.bin
HIPCC   ?= /opt/rocm/bin/hipcc
ARCH    ?= gfx950
HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -fvisibility=hidden \
            -mllvm -structurizecfg-skip-uniform-regions=true \
            -DQFEC_BUILD -DQFEC_TABLES_PATH='"$(TABLES)"' -Wall -Wno-unused-function \
            -MMD -MP -I$(ROOT)build/gen -I$(CSRC)

# config D kernel instantiations, one per object (each compiles for minutes; -j builds them
# in parallel)
DCOLK := e63 e83 d62 d82
# preset syndrome-decode instantiations, one object per code (gf_psyn.h)
PSYNK := 1010 1015 1020 1515 55
SRCS := $(CSRC)/fec_kernels.hip $(CSRC)/xor_dma.hip $(CSRC)/gf_stream.hip $(CSRC)/gf_bsyn.hip $(CSRC)/gf_psyn.hip $(PSYNK:%=$(CSRC)/gf_psyn_%.hip) $(CSRC)/gf_dcol.hip $(DCOLK:%=$(CSRC)/gf_dcol_%.hip) $(CSRC)/pp_null.hip $(CSRC)/fec_api.cpp $(CSRC)/fec_group.cpp $(CSRC)/fec_wire.cpp
# the headers every object depends on; the rest (include/*.h, pp_null.h, ...) are tracked per
# object by -MMD below, so a public-header edit rebuilds only the host files that include it
HDRS := $(CSRC)/fec_kernels.h $(CSRC)/gf256.h $(CSRC)/gf_bitslice.h
OBJS := $(ROOT)build/fec_kernels.o $(ROOT)build/xor_dma.o $(ROOT)build/gf_stream.o $(ROOT)build/gf_bsyn.o $(ROOT)build/gf_psyn.o $(PSYNK:%=$(ROOT)build/gf_psyn_%.o) $(ROOT)build/gf_dcol.o $(DCOLK:%=$(ROOT)build/gf_dcol_%.o) $(ROOT)build/pp_null.o $(ROOT)build/fec_api.o $(ROOT)build/fec_group.o $(ROOT)build/fec_wire.o

# Build guard (tools/check_stubs.py): every kernel stub a host pass registers has device code
# in the same object.  Run after each HIP compile (the object is deleted on a mismatch) and on
# all objects before the link (the library is deleted on a mismatch), so a partial build can
# never ship.
STUBCHECK := python3 $(ROOT)tools/check_stubs.py

TOOL := $(ROOT)quic_amd/bin/fec_loopback
LAT  := $(ROOT)quic_amd/bin/dropin_latency
GRPX := $(ROOT)quic_amd/bin/group_roundtrip

.PHONY: all lib oracle tools clean
all: lib oracle tools

tools: $(TOOL) $(LAT) $(GRPX)

# the QuicFecGroup C++ class (include/quic_fec_group.hpp) exercised like the reference's callers
$(GRPX): $(ROOT)tools/group_cxx/group_roundtrip.cpp $(LIB) $(ROOT)include/quic_fec_group.hpp $(ROOT)include/quic_fec_group.h
	@mkdir -p $(ROOT)quic_amd/bin
	g++ -O2 -std=c++17 -Wall -I$(ROOT)include -o $@ $< -L$(ROOT)quic_amd -lquic_fec \
	    -Wl,-rpath,'$$ORIGIN/..' -ldl

$(LAT): $(ROOT)tools/latency/dropin_latency.cpp $(LIB) $(ROOT)include/quic_fec.h
	@mkdir -p $(ROOT)quic_amd/bin
	g++ -O2 -std=c++17 -Wall -I$(ROOT)include -o $@ $< -L$(ROOT)quic_amd -lquic_fec \
	    -Wl,-rpath,'$$ORIGIN/..' -ldl

$(TOOL): $(ROOT)tools/loopback/fec_loopback.cpp $(LIB) $(ROOT)include/quic_fec_group.h
	@mkdir -p $(ROOT)quic_amd/bin
	g++ -O2 -std=c++17 -Wall -I$(ROOT)include -o $@ $< -L$(ROOT)quic_amd -lquic_fec \
	    -Wl,-rpath,'$$ORIGIN/..' -ldl -lpthread

lib: $(LIB)

$(ROOT)build/fec_kernels.o: $(CSRC)/fec_kernels.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/xor_dma.o: $(CSRC)/xor_dma.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

GEN := $(ROOT)build/gen/cauchy_const.h
# the counted-vmcnt kernels keep their device assembly (build/<name>-hip-amdgcn-amd-amdhsa-
# gfx950.s, the text the object is assembled from): tests/test_isa.py reads it instead of
# compiling the files a second time
SAVE_ASM := -save-temps=obj
$(GEN): $(TABLES) $(ROOT)tools/gen_cauchy_const.py
	python3 $(ROOT)tools/gen_cauchy_const.py && touch $@

# the 256-leaf jump table of the run-time windowed product (gf_winjump.h)
WJGEN := $(ROOT)build/gen/win_jump.h
# (the generator rewrites the header only when its text changes; the touch marks it newer
# than a changed generator)
$(WJGEN): $(ROOT)tools/gen_win_jump.py
	python3 $(ROOT)tools/gen_win_jump.py && touch $@

$(ROOT)build/gf_stream.o: $(CSRC)/gf_stream.hip $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/gf_bsyn.o: $(CSRC)/gf_bsyn.hip $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

# gf_psyn indexes its accumulator arrays through uniform branch trees; SimplifyCFG would sink
# the branches' identical loads into one load with a computed index, which leaves the
# arrays in scratch memory (VMEM outside the counted waits)
PSYNFLAGS := -mllvm -simplifycfg-sink-common=false
$(ROOT)build/gf_psyn.o: $(CSRC)/gf_psyn.hip $(CSRC)/gf_psyn.h $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(PSYNFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/gf_psyn_%.o: $(CSRC)/gf_psyn_%.hip $(CSRC)/gf_psyn.h $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(PSYNFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/gf_dcol.o: $(CSRC)/gf_dcol.hip $(CSRC)/gf_dcol.h $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/gf_dcol_%.o: $(CSRC)/gf_dcol_%.hip $(CSRC)/gf_dcol.h $(CSRC)/gf_winjump.h $(HDRS) $(GEN) $(WJGEN)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) $(SAVE_ASM) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/pp_null.o: $(CSRC)/pp_null.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/fec_api.o: $(CSRC)/fec_api.cpp $(HDRS) $(TABLES)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/fec_group.o: $(CSRC)/fec_group.cpp $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(ROOT)build/fec_wire.o: $(CSRC)/fec_wire.cpp $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@
	@$(STUBCHECK) $@ || { rm -f $@; exit 1; }

$(LIB): $(OBJS)
	@$(STUBCHECK) $(OBJS) || { rm -f $@; exit 1; }
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@.tmp $(OBJS)
	@mv -f $@.tmp $@

oracle:
	$(MAKE) -s -C $(ROOT)oracle

# header dependencies generated by -MMD (every header a source includes, transitively)
-include $(OBJS:.o=.d)

clean:
	rm -rf $(ROOT)build $(LIB) $(TOOL) $(LAT)
	$(MAKE) -s -C $(ROOT)oracle clean
