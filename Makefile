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
HIPFLAGS  := --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall \
             -Wno-unused-function -I include -I $(CSRC)
HIP_SRCS  := $(CSRC)/fwd_bwd.hip $(CSRC)/fwd_bwd_stream.hip $(CSRC)/fwd_bwd_pair.hip $(CSRC)/fwd_bwd_wide.hip $(CSRC)/v2_fwd_bwd.hip \
             $(CSRC)/decode.hip \
             $(CSRC)/fused_decode.hip $(CSRC)/capi.hip
HIP_HDRS  := $(wildcard $(CSRC)/*.h) include/ssnt_tts_c.h
HIP_OBJS  := $(patsubst $(CSRC)/%.hip,$(LIBDIR)/obj/%.o,$(HIP_SRCS))

all: lib oracle

lib: $(LIB)
oracle: $(ORACLE)

$(LIBDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(LIB): $(HIP_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(HIP_OBJS) -Wl,-soname,libssnt_tts_c.so

# diagnostic build with in-kernel s_memtime totals (tools/diag_fwd_bwd.py); never the product
DIAGDIR   := $(LIBDIR)/diag
DIAG_OBJS := $(patsubst $(CSRC)/%.hip,$(DIAGDIR)/obj/%.o,$(HIP_SRCS))
lib-diag: $(DIAGDIR)/libssnt_tts_c.so
$(DIAGDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_DIAG -c $< -o $@
$(DIAGDIR)/libssnt_tts_c.so: $(DIAG_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(DIAG_OBJS) -Wl,-soname,libssnt_tts_c.so

# experiment build: one kernel instance (K=2, no log_obs), diag stamps, SSNT_EXP env knobs
EXPDIR    := $(LIBDIR)/exp
EXP_OBJS  := $(patsubst $(CSRC)/%.hip,$(EXPDIR)/obj/%.o,$(HIP_SRCS))
lib-exp: $(EXPDIR)/libssnt_tts_c.so
$(EXPDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_DIAG -DSSNT_EXP -c $< -o $@
# experiment build without the diagnostic stamps (kernel time of SSNT_EXP masks, tools/ab_exp.py)
EXPNDIR   := $(LIBDIR)/expnd
EXPN_OBJS := $(patsubst $(CSRC)/%.hip,$(EXPNDIR)/obj/%.o,$(HIP_SRCS))
lib-expnd: $(EXPNDIR)/libssnt_tts_c.so
$(EXPNDIR)/obj/%.o: $(CSRC)/%.hip $(HIP_HDRS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -DSSNT_EXP -c $< -o $@
$(EXPNDIR)/libssnt_tts_c.so: $(EXPN_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(EXPN_OBJS) -Wl,-soname,libssnt_tts_c.so

$(EXPDIR)/libssnt_tts_c.so: $(EXP_OBJS)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(EXP_OBJS) -Wl,-soname,libssnt_tts_c.so

$(ORACLE): oracle/ssnt_oracle.c
	@mkdir -p $(dir $@)
	gcc -O3 -std=c11 -fopenmp -ffp-contract=off -fPIC -shared -Wall -o $@ $< -lm

clean:
	rm -rf $(LIBDIR) oracle/build

.PHONY: all lib lib-diag lib-exp lib-expnd oracle clean
