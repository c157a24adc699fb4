#!/bin/bash
cd /tmp && export TMPDIR=/tmp
mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r5h
timeout -s KILL 60 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/r5h/counters.txt 2>&1
grep -o -E "\b(TA|TD|TCP|TCC|SQ|GRBM|SPI)_[A-Z0-9_]+" $GRAFT_REPO_ROOT/gpurun_out/r5h/counters.txt | sort -u > $GRAFT_REPO_ROOT/gpurun_out/r5h/names.txt
wc -l $GRAFT_REPO_ROOT/gpurun_out/r5h/names.txt
