# Builds libdpac.so (gfx950) in-tree.  The oracle (oracle/) is Python (torch-CPU float64)
# and needs no build.
#   make -j8        -> deeppde_actorcritic_amd/libdpac.so
# Each equation family's kernels are compiled once per dtype AND state dimension (one object
# each, registered at load time: Registrar in dpac_kernels.h), so the heavy template
# instantiations build in parallel.
HIPCC     ?= /opt/rocm/bin/hipcc
ARCH      ?= gfx950
PKG       := deeppde_actorcritic_amd
CSRC      := $(PKG)/csrc
OBJDIR    := build/obj
# state dimensions with compiled kernels (every shipped reference config: 4, 5, 10, 20);
# VDP needs an even dimension
DIMS      ?= 4,5,10,20
DIMS_EVEN ?= 4,10,20
comma     := ,
DIM_LIST  := $(subst $(comma), ,$(DIMS))
EVEN_LIST := $(subst $(comma), ,$(DIMS_EVEN))
BASEFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -Iinclude -I$(CSRC) -Wno-pass-failed \
             -ffp-contract=off -MMD -MP
HIPFLAGS  := $(BASEFLAGS) -DDPAC_DIMS=$(DIMS) -DDPAC_DIMS_EVEN=$(DIMS_EVEN)
EQNS      := lqr lqrvar ekn vdp
# header dependencies: generated per object (-MMD); a build without .d files rebuilds all
HDRS      :=
eqn_dims   = $(if $(filter vdp,$(1)),$(EVEN_LIST),$(DIM_LIST))
EQN_OBJS  := $(foreach e,$(EQNS),$(foreach d,$(call eqn_dims,$(e)),$(foreach t,f32 f64,$(OBJDIR)/dpac_eqn_$(e)_$(t)_d$(d).o)))
OBJS      := $(OBJDIR)/dpac_abi.o $(OBJDIR)/dpac_mlp.o $(OBJDIR)/dpac_params.o $(EQN_OBJS)
LIB       := $(PKG)/libdpac.so

.PHONY: all lib ext plugins bounds clean
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

# $(1) equation, $(2) f32 | f64, $(3) dimension
define EQN_RULE
$(OBJDIR)/dpac_eqn_$(1)_$(2)_d$(3).o: $(CSRC)/dpac_eqn_$(1).hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(BASEFLAGS) -DDPAC_DIMS=$(3) -DDPAC_DIMS_EVEN=$(3) -DDPAC_TU_DOUBLE=$(if $(filter f64,$(2)),1,0) -c $$< -o $$@
endef
$(foreach e,$(EQNS),$(foreach d,$(call eqn_dims,$(e)),$(foreach t,f32 f64,$(eval $(call EQN_RULE,$(e),$(t),$(d))))))

-include $(OBJS:.o=.d)

$(LIB): $(OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(OBJS)

# Dimension plugins: the equation kernels for state dimensions outside DIMS, one shared
# object per dimension, $(PKG)/libdpac_d<D>.so, linked against libdpac.so; _lib.load() loads
# every plugin beside libdpac.so, and its instantiations register into the same dispatch table
# (Registrar, dpac_kernels.h).  VDP needs an even dimension (d = 2c).
#   make ext EXT_DIMS=7,12
EXT_DIMS  ?= 7
EXT_LIST  := $(subst $(comma), ,$(EXT_DIMS))
EXTDIR    := build/ext
ext_eqns   = lqr lqrvar ekn $(if $(filter 0,$(shell echo $$(($(1) % 2)))),vdp,)
ext_objs   = $(foreach e,$(call ext_eqns,$(1)),$(foreach t,f32 f64,$(EXTDIR)/dpac_eqn_$(e)_$(t)_d$(1).o))
define EXT_RULE
$(EXTDIR)/dpac_eqn_$(1)_$(2)_d$(3).o: $(CSRC)/dpac_eqn_$(1).hip
	@mkdir -p $(EXTDIR)
	$(HIPCC) $(BASEFLAGS) -DDPAC_DIMS=$(3) -DDPAC_DIMS_EVEN=$(3) -DDPAC_TU_DOUBLE=$(if $(filter f64,$(2)),1,0) -c $$< -o $$@
endef
$(foreach d,$(EXT_LIST),$(foreach e,$(call ext_eqns,$(d)),$(foreach t,f32 f64,$(eval $(call EXT_RULE,$(e),$(t),$(d))))))
define EXT_LIB
$(PKG)/libdpac_d$(1).so: $(call ext_objs,$(1))
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $$@ $(call ext_objs,$(1)) -L$(PKG) -ldpac -Wl,-rpath,'$$$$ORIGIN'
endef
$(foreach d,$(EXT_LIST),$(eval $(call EXT_LIB,$(d))))
-include $(wildcard $(EXTDIR)/*.d)
ext: lib $(foreach d,$(EXT_LIST),$(PKG)/libdpac_d$(d).so)
# the plugins alone, against the libdpac.so in place (never rebuilt here): _lib.ensure_dim's
# on-demand build, which must not relink a library the calling process has loaded
plugins: $(foreach d,$(EXT_LIST),$(PKG)/libdpac_d$(d).so)

clean:
	rm -rf build $(LIB) $(PKG)/libdpac_d*.so

# Host-side sanitizer run of the C-ABI validation layer (no GPU needed): every TU with
# AddressSanitizer + UndefinedBehaviorSanitizer on the host side only (device code is
# unchanged), d = 20 kernels, linked into build/asan/libdpac_asan.so, driven by
# tests/abi_sanitize.c.   make sanitize   (log: build/asan/abi_sanitize.log)
ASAN_DIR  := build/asan
ASAN_HOST := -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
             -Xarch_host -fno-omit-frame-pointer -Xarch_host -fno-sanitize-recover=undefined
ASAN_FLAGS := $(filter-out -DDPAC_DIMS=% -DDPAC_DIMS_EVEN=%,$(HIPFLAGS)) -DDPAC_DIMS=20 -DDPAC_DIMS_EVEN=20 -O1 $(ASAN_HOST)
ASAN_OBJS := $(ASAN_DIR)/dpac_abi.o $(ASAN_DIR)/dpac_mlp.o $(ASAN_DIR)/dpac_params.o \
             $(foreach e,$(EQNS),$(ASAN_DIR)/dpac_eqn_$(e)_f32.o $(ASAN_DIR)/dpac_eqn_$(e)_f64.o)
CLANG     ?= /opt/rocm/llvm/bin/clang
SANRT     := $(dir $(firstword $(wildcard /opt/rocm/llvm/lib/clang/*/lib/linux/libclang_rt.asan-x86_64.so)))

.PHONY: sanitize
$(ASAN_DIR)/dpac_%.o: $(CSRC)/dpac_%.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(ASAN_FLAGS) -c $< -o $@
$(ASAN_DIR)/dpac_eqn_%_f32.o: $(CSRC)/dpac_eqn_%.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(ASAN_FLAGS) -DDPAC_TU_DOUBLE=0 -c $< -o $@
$(ASAN_DIR)/dpac_eqn_%_f64.o: $(CSRC)/dpac_eqn_%.hip $(HDRS)
	@mkdir -p $(ASAN_DIR)
	$(HIPCC) $(ASAN_FLAGS) -DDPAC_TU_DOUBLE=1 -c $< -o $@
$(ASAN_DIR)/libdpac_asan.so: $(ASAN_OBJS)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -fsanitize=address,undefined -shared-libsan -o $@ $(ASAN_OBJS)
$(ASAN_DIR)/abi_sanitize: tests/abi_sanitize.c $(ASAN_DIR)/libdpac_asan.so include/dpac.h
	$(CLANG) -g -O1 -fsanitize=address,undefined -shared-libsan -fno-omit-frame-pointer -Iinclude $< \
	  -L$(ASAN_DIR) -ldpac_asan -Wl,-rpath,$(abspath $(ASAN_DIR)) -Wl,-rpath,$(SANRT) -o $@
sanitize: $(ASAN_DIR)/abi_sanitize
	ASAN_OPTIONS=detect_leaks=0:halt_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
	  $(ASAN_DIR)/abi_sanitize > $(ASAN_DIR)/abi_sanitize.log 2>&1; rc=$$?; tail -3 $(ASAN_DIR)/abi_sanitize.log; exit $$rc

# The DPAC_CHECK_BOUNDS test build (dpac_device.h): the row kernels' object (dpac_mlp.hip) rebuilt
# with every row-indexed TD-operand / prologue load checking that its row is live, linked with the
# main build's other objects -> tools/variants/libdpac_bounds.so (DPAC_LIB=...;
# tests/test_gpu_td_fused.py runs tests/bounds_check.py under it).
BOUNDS_LIB := tools/variants/libdpac_bounds.so
bounds: $(BOUNDS_LIB)
build/bounds/dpac_mlp.o: $(CSRC)/dpac_mlp.hip $(OBJDIR)/dpac_mlp.o
	@mkdir -p build/bounds
	$(HIPCC) $(HIPFLAGS) -DDPAC_CHECK_BOUNDS=1 -c $< -o $@
$(BOUNDS_LIB): build/bounds/dpac_mlp.o $(OBJS)
	@mkdir -p tools/variants
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -o $@ $(filter-out $(OBJDIR)/dpac_mlp.o,$(OBJS)) build/bounds/dpac_mlp.o
