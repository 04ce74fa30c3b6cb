#!/bin/bash
# Host-code sanitizers on the GPU box: libffmp with ASan + UBSan on its HOST code only
# (tools/_build/libffmp_san.so, built by tools/build_sanitize.sh) driven by two plain-C programs
# built with -fsanitize=address,undefined: the seamless ring's host code (tests/ring_sanitize.c)
# and a 512-env reset + 25-step run (tests/c_abi_consumer.c).  GPU code is not sanitized.
# LeakSanitizer off: ring pieces are never freed by design (ffmp_ring.hip "never unmap").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export ASAN_OPTIONS=protect_shadow_gap=0:detect_leaks=0
export UBSAN_OPTIONS=print_stacktrace=1
timeout -k 10 180 $R/tools/_build/ring_sanitize_san || exit 1
timeout -k 10 300 $R/tools/_build/c_abi_consumer_san || exit 1
