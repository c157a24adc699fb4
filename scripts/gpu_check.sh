#!/bin/bash
# GPU-box validation: build, GPU tests, smoke(), 1-GPU bench, rocprofv3 kernel stats
# (SKIP_TESTS / SKIP_BENCH / SKIP_PROF=1 skip a step; PYTEST_ARGS / BENCH_ARGS / PROF_ARGS).
# Each GPU step has its own time limit; a crash/timeout/abort ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
fatal() { case "$1" in 124|137|134|139|-6|-11) return 0;; *) return 1;; esac; }

python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -30 gpurun_out/build.log; exit 1; }
echo "build ok"

if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  tail -25 gpurun_out/pytest_gpu.log
  if fatal $rc; then echo "pytest fatal rc=$rc"; exit $rc; fi
  echo "pytest rc=$rc"
fi

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; tail -2 gpurun_out/smoke.log; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc

if [ "${SKIP_BENCH:-0}" != "1" ]; then
  timeout -k 10 900 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?
  tail -5 gpurun_out/bench.err; cat gpurun_out/bench.json
  if [ $rc -ne 0 ]; then echo "bench rc=$rc"; exit $rc; fi
fi

if [ "${SKIP_PROF:-0}" != "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 ${PROF_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
  rc=$?
  tail -3 "$GRAFT_REPO_ROOT/gpurun_out/prof.log"
  echo "prof rc=$rc"
fi
