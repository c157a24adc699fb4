set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_kernels_gpu.py -x -q -k "decode" > gpurun_out/pytest_decode.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_decode.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/decode_attn_bench.py > gpurun_out/decode_attn_sweep2.log 2>&1
rc=$?; grep -E "^B|\*" gpurun_out/decode_attn_sweep2.log; exit $rc
