set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 300 python scripts/small_kernels_bench.py > gpurun_out/small_kernels.log 2>&1
rc=$?; cat gpurun_out/small_kernels.log; exit $rc
