# Build: the product library (HIP for gfx950 + C++ host C-ABI) and the CPU oracle (test infra).
#   make            -> both
#   make lib        -> ssnt-tts-rust_amd/lib/libssnt_tts_c.so
#   make oracle     -> oracle/build/libssnt_oracle.so
ROCM      ?= /opt/rocm
HIPCC     ?= $(ROCM)/bin/hipcc
PKG       := ssnt-tts-rust_amd
CSRC      := $(PKG)/csrc
LIBDIR    := $(PKG)/lib
LIB       := $(LIBDIR)/libssnt_tts_c.so
ORACLE    := oracle/build/libssnt_oracle.so

# -ffp-contract=off: the fwd-bwd arithmetic is specified op-by-op (no a*b+c contraction) so
# the CPU oracle reproduces it bit for bit. Correctly rounded f32 division is HIP's default.
HIPFLAGS  := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fvisibility=hidden -Wall \
             -Wno-unused-function -I include -I $(CSRC)
HIP_SRCS  := $(CSRC)/fwd_bwd.hip $(CSRC)/fwd_bwd_stream.hip $(CSRC)/fwd_bwd_wide.hip $(CSRC)/v2_fwd_bwd.hip \
             $(CSRC)/decode.hip \
             $(CSRC)/fused_decode.hip $(CSRC)/capi.hip
# the A/B and diagnostic builds compile the same sources with their own macros
AB_SRCS   := $(HIP_SRCS)
HIP_HDRS  := $(wildcard $(CSRC)/*.h) include/ssnt_tts_c.h
HIP_OBJS  := $(patsubst $(CSRC)/%.hip,$(LIBDIR)/obj/%.o,$(HIP_SRCS))

all: lib lib-ab lib-diag lib-diag-fault oracle

lib: $(LIB)
oracle: $(ORACLE)

# A/B build (tests and tools only; include/ssnt_tts_c_ab.h): the product plus process-wide kernel
# / staging / sync knobs and the selection decode ordering. Own soname, so a
# process can load it beside the product library.
ABDIR     := $(LIBDIR)/ab
AB_OBJS   := $(patsubst $(CSRC)/%.hip,$(ABDIR)/obj/%.o,$(AB_SRCS))
lib-ab: $(ABDIR)/libssnt_tts_c_ab.so
$(ABDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_AB -c $< -o $@
$(ABDIR)/libssnt_tts_c_ab.so: $(AB_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(AB_OBJS) -Wl,-soname,libssnt_tts_c_ab.so

$(LIBDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(HIP_OBJS) -Wl,-soname,libssnt_tts_c.so

# diagnostic build with in-kernel s_memtime totals (tools/diag_fwd_bwd.py); never the product
DIAGDIR   := $(LIBDIR)/diag
DIAG_OBJS := $(patsubst $(CSRC)/%.hip,$(DIAGDIR)/obj/%.o,$(AB_SRCS))
lib-diag: $(DIAGDIR)/libssnt_tts_c.so
$(DIAGDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_AB -DSSNT_DIAG -c $< -o $@
$(DIAGDIR)/libssnt_tts_c.so: $(DIAG_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(DIAG_OBJS) -Wl,-soname,libssnt_tts_c.so

# negative control of the diagnostic ring tags: converters label every slot with a wrong row
# (tests/test_gpu_fwd_bwd.py::test_ring_tags_diag_build expects kStatusRingTag from it)
DFDIR     := $(LIBDIR)/diagfault
DF_OBJS   := $(patsubst $(CSRC)/%.hip,$(DFDIR)/obj/%.o,$(AB_SRCS))
lib-diag-fault: $(DFDIR)/libssnt_tts_c.so
$(DFDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_AB -DSSNT_DIAG -DSSNT_DIAG_TAG_FAULT=1 -c $< -o $@
$(DFDIR)/libssnt_tts_c.so: $(DF_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(DF_OBJS) -Wl,-soname,libssnt_tts_c.so

$(ORACLE): oracle/ssnt_oracle.c
	@mkdir -p $(dir $@)
	gcc -O3 -std=c11 -fopenmp -ffp-contract=off -fPIC -shared -Wall -o $@ $< -lm

clean:
	rm -rf $(LIBDIR) oracle/build

.PHONY: all lib lib-ab lib-diag lib-diag-fault oracle clean
