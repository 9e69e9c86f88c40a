# Builds libdpac.so (gfx950) in-tree.  The oracle (oracle/) is Python (torch-CPU float64)
# and needs no build.
#   make -j8        -> deeppde_actorcritic_amd/libdpac.so
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
PKG       := deeppde_actorcritic_amd
CSRC      := $(PKG)/csrc
OBJDIR    := build/obj
# state dimensions with compiled kernels (every shipped reference config: 4, 5, 10, 20)
DIMS      ?= 4,5,10,20
DIMS_EVEN ?= 4,10,20
HIPFLAGS  := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) \
             -DDPAC_DIMS=$(DIMS) -DDPAC_DIMS_EVEN=$(DIMS_EVEN) -Wno-pass-failed \
             -ffp-contract=off
EQNS      := lqr lqrvar ekn vdp
HDRS      := $(wildcard $(CSRC)/*.h) include/dpac.h
OBJS      := $(OBJDIR)/dpac_abi.o $(OBJDIR)/dpac_mlp.o $(OBJDIR)/dpac_params.o \
             $(foreach e,$(EQNS),$(OBJDIR)/dpac_eqn_$(e)_f32.o $(OBJDIR)/dpac_eqn_$(e)_f64.o)
LIB       := $(PKG)/libdpac.so

.PHONY: all lib clean
all: lib
lib: $(LIB)

$(OBJDIR)/dpac_abi.o: $(CSRC)/dpac_abi.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/dpac_mlp.o: $(CSRC)/dpac_mlp.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/dpac_params.o: $(CSRC)/dpac_params.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(OBJDIR)/dpac_eqn_%_f32.o: $(CSRC)/dpac_eqn_%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DDPAC_TU_DOUBLE=0 -c $< -o $@

$(OBJDIR)/dpac_eqn_%_f64.o: $(CSRC)/dpac_eqn_%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -DDPAC_TU_DOUBLE=1 -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

clean:
	rm -rf build $(LIB)
