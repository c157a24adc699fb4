set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 400 python -m pytest tests/test_custom_allreduce_gpu.py -x -q > gpurun_out/pytest_ar.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_ar.log; echo "ar rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_gpu.log; echo "gpu rc=$rc"; exit $rc
