# Builds libffmp (gfx950) in-tree.  `make` == __graft_entry__.build() (one object per source, so an
# edit of one .hip recompiles only that file).
HIPCC ?= /opt/rocm/bin/hipcc
HIPFLAGS = --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -Iinclude
LIB = flow_field_based_motion_planner_amd/lib/libffmp.so
CSRC = flow_field_based_motion_planner_amd/csrc
SRC = $(CSRC)/ffmp_kernels.hip $(CSRC)/ffmp_ring.hip $(CSRC)/ffmp_conv.hip
HDRS = $(CSRC)/ffmp_device.h include/ffmp.h
OBJDIR = build/obj
OBJ = $(patsubst $(CSRC)/%.hip,$(OBJDIR)/%.o,$(SRC))

all: $(LIB)

$(OBJDIR)/%.o: $(CSRC)/%.hip $(HDRS)
	@mkdir -p $(OBJDIR)
	$(HIPCC) $(HIPFLAGS) -c -o $@ $<

$(LIB): $(OBJ)
	@mkdir -p $(dir $@)
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o $@ $(OBJ)

# a probe variant of the library: make probe V=name DEFS="-DFFMP_...=..." -> tools/_probe/libffmp_name.so
# (FFMP_LIB=... selects it; tools/_probe/ travels to the GPU box: delete a variant once measured)
probe: $(SRC) $(HDRS)
	@mkdir -p tools/_probe
	$(HIPCC) $(HIPFLAGS) $(DEFS) -shared -o tools/_probe/libffmp_$(V).so $(SRC)

# the same with only the convolutions rebuilt (the other objects as `make` built them)
probe-conv: $(OBJDIR)/ffmp_kernels.o $(OBJDIR)/ffmp_ring.o $(CSRC)/ffmp_conv.hip $(HDRS)
	@mkdir -p tools/_probe
	$(HIPCC) $(HIPFLAGS) $(DEFS) -c -o build/conv_$(V).o $(CSRC)/ffmp_conv.hip
	$(HIPCC) --offload-arch=gfx950 -shared -fPIC -o tools/_probe/libffmp_$(V).so $(OBJDIR)/ffmp_kernels.o $(OBJDIR)/ffmp_ring.o build/conv_$(V).o

asm: $(SRC) $(HDRS)
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -S --cuda-device-only -o /tmp/ffmp_kernels.s $(CSRC)/ffmp_kernels.hip

clean:
	rm -f $(LIB) $(OBJ)

.PHONY: all probe probe-conv asm clean
