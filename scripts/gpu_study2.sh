#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -6 gpurun_out/pytest_gpu.log; echo "pytest rc=$rc"
case $rc in 0|1) ;; *) exit $rc;; esac
for B in 512 1024; do
  timeout -k 10 600 python bench.py --batch $B --steps 3 --warmup 1 > gpurun_out/bench_b$B.json 2> gpurun_out/bench_b$B.err; rc=$?
  echo "bench B=$B rc=$rc"; cat gpurun_out/bench_b$B.json; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof512" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 1 --warmup 1 --batch 512 > "$GRAFT_REPO_ROOT/gpurun_out/prof512.log" 2>&1
echo "prof rc=$?"
