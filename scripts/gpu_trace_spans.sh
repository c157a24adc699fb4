set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
DRTC_TIME_DECODE=1 timeout -k 10 600 python bench.py --steps 2 --warmup 1 --trace gpurun_out/trace_b1024.json > gpurun_out/bench_trace.json 2> gpurun_out/bench_trace.err
rc=$?; tail -2 gpurun_out/bench_trace.err; cut -c1-300 gpurun_out/bench_trace.json; exit $rc
