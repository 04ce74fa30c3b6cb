#!/bin/bash
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/counters.txt 2>&1
grep -ioE '(UTCL[0-9A-Z_]*|TCP_UTCL[0-9A-Z_]*|TC[AP]_TLB[0-9A-Z_]*|[A-Z_]*TRANSLATION[A-Z_]*|[A-Z0-9_]*TLB[A-Z0-9_]*|TCC_EA0_WR[A-Z0-9_]*|TCC_EA0_WRREQ[A-Z0-9_]*|TCC_WRITE[A-Z0-9_]*)' $GRAFT_REPO_ROOT/gpurun_out/counters.txt | sort -u | head -80
wc -l $GRAFT_REPO_ROOT/gpurun_out/counters.txt
