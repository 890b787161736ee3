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
            -DQFEC_BUILD -DQFEC_TABLES_PATH='"$(TABLES)"' -Wall -Wno-unused-function

SRCS := $(CSRC)/fec_kernels.hip $(CSRC)/xor_dma.hip $(CSRC)/gf_group.hip $(CSRC)/gf_stream.hip $(CSRC)/fec_api.cpp $(CSRC)/fec_group.cpp $(CSRC)/fec_wire.cpp
HDRS := $(CSRC)/fec_kernels.h $(CSRC)/gf256.h $(CSRC)/gf_bitslice.h $(ROOT)include/quic_fec.h \
        $(ROOT)include/quic_fec_group.h $(ROOT)Makefile
OBJS := $(ROOT)build/fec_kernels.o $(ROOT)build/xor_dma.o $(ROOT)build/gf_group.o $(ROOT)build/gf_stream.o $(ROOT)build/fec_api.o $(ROOT)build/fec_group.o $(ROOT)build/fec_wire.o

TOOL := $(ROOT)quic_amd/bin/fec_loopback

.PHONY: all lib oracle tools clean
all: lib oracle tools

tools: $(TOOL)

$(TOOL): $(ROOT)tools/loopback/fec_loopback.cpp $(LIB) $(ROOT)include/quic_fec_group.h
	@mkdir -p $(ROOT)quic_amd/bin
	g++ -O2 -std=c++17 -Wall -I$(ROOT)include -o $@ $< -L$(ROOT)quic_amd -lquic_fec \
	    -Wl,-rpath,'$$ORIGIN/..' -ldl -lpthread

lib: $(LIB)

$(ROOT)build/fec_kernels.o: $(CSRC)/fec_kernels.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ROOT)build/xor_dma.o: $(CSRC)/xor_dma.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ROOT)build/gf_group.o: $(CSRC)/gf_group.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ROOT)build/gf_stream.o: $(CSRC)/gf_stream.hip $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(ROOT)build/fec_api.o: $(CSRC)/fec_api.cpp $(HDRS) $(TABLES)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(ROOT)build/fec_group.o: $(CSRC)/fec_group.cpp $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(ROOT)build/fec_wire.o: $(CSRC)/fec_wire.cpp $(HDRS)
	@mkdir -p $(ROOT)build
	$(HIPCC) $(HIPFLAGS) -x hip -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

oracle:
	$(MAKE) -s -C $(ROOT)oracle

clean:
	rm -rf $(ROOT)build $(LIB) $(TOOL)
	$(MAKE) -s -C $(ROOT)oracle clean
