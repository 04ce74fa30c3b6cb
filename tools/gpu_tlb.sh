#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
mkdir -p $R/gpurun_out/tlb
cd /tmp && export TMPDIR=/tmp
for r in 1 2 3 4 5 6; do
  timeout -k 10 300 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum --kernel-include-regex raster_kernel --output-format csv -d $R/gpurun_out/tlb/a$r -o run -- python3 $R/tools/tlb_probe.py > /dev/null 2>&1 || exit 1
done
for r in 1 2 3 4; do
  timeout -k 10 300 rocprofv3 --pmc TCC_EA0_WRREQ_STALL_sum TCP_UTCL1_STALL_MULTI_MISS_sum --kernel-include-regex raster_kernel --output-format csv -d $R/gpurun_out/tlb/b$r -o run -- python3 $R/tools/tlb_probe.py > /dev/null 2>&1 || exit 1
done
cd $R && python3 tools/summarize_pmc_runs.py gpurun_out/tlb
