# Builds libffmp (gfx950) in-tree.  `make` == __graft_entry__.build().
HIPCC ?= /opt/rocm/bin/hipcc
HIPFLAGS = --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -fPIC -shared -Iinclude
LIB = flow_field_based_motion_planner_amd/lib/libffmp.so
SRC = flow_field_based_motion_planner_amd/csrc/ffmp_kernels.hip flow_field_based_motion_planner_amd/csrc/ffmp_ring.hip flow_field_based_motion_planner_amd/csrc/ffmp_conv.hip
DEPS = $(SRC) flow_field_based_motion_planner_amd/csrc/ffmp_device.h include/ffmp.h

all: $(LIB)

$(LIB): $(DEPS)
	@mkdir -p $(dir $@)
	$(HIPCC) $(HIPFLAGS) -o $@ $(SRC)

asm: $(DEPS)
	$(HIPCC) --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -S --cuda-device-only -o /tmp/ffmp_kernels.s flow_field_based_motion_planner_amd/csrc/ffmp_kernels.hip

clean:
	rm -f $(LIB)

.PHONY: all asm clean
