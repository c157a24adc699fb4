#!/bin/bash
# Evidence that decode steps are hipGraph launches: rocprofv3 HIP-API trace +
# kernel trace of a short bench run (no PMC counters in the same run).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_graph" -o run -- python3 "$R/bench.py" --batch 256 --steps 1 --warmup 1 > "$R/gpurun_out/prof_graph.log" 2>&1
rc=$?; tail -3 "$R/gpurun_out/prof_graph.log"; echo "prof rc=$rc"; exit $rc
