#!/bin/bash
# Round 5 (after the combine / retune / norm changes): the whole GPU suite, smoke() and the headline bench on the current tree.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${R5_OUT:-r5ac}; mkdir -p $O
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread \
    -p no:cacheprovider > $O/gpu_suite.log 2>&1
rc=$?; tail -5 $O/gpu_suite.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python -u bench.py --steps 8 --warmup 2 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cut -c1-300 $O/bench.json
if [ -n "${R5_70B:-}" ]; then
  timeout -k 10 600 python -u bench.py --model llama-3-70b --workload ask --batch 256 --steps 3 --warmup 1 \
      > $O/b70_256.json 2> $O/b70_256.err || { tail -5 $O/b70_256.err; exit 1; }
  cut -c1-400 $O/b70_256.json
fi
