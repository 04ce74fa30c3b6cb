#!/bin/bash
# Builds the host-sanitized libffmp and the two C drivers of tools/gpu_sanitize.sh into tools/_build
# (CPU; hipcc cross-compiles the device code, which is not sanitized).
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/tools/_build
mkdir -p $B
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O1 -g -std=c++17 -ffp-contract=off -fPIC -shared -I$R/include \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined \
  -o $B/libffmp_san.so $R/flow_field_based_motion_planner_amd/csrc/ffmp_kernels.hip $R/flow_field_based_motion_planner_amd/csrc/ffmp_ring.hip
for prog in ring_sanitize c_abi_consumer; do
  /opt/rocm/llvm/bin/clang -g -O1 -fsanitize=address,undefined -fno-sanitize=function -fno-sanitize-recover=undefined \
    -D__HIP_PLATFORM_AMD__ -I$R/include -I/opt/rocm/include $R/tests/$prog.c -L$B -lffmp_san \
    -L/opt/rocm/lib -lamdhip64 -lm -Wl,-rpath,'$ORIGIN' -Wl,-rpath,/opt/rocm/lib -o $B/${prog}_san
done
