#!/bin/bash
# Round 5: mixed steps launched behind the in-flight decode step (no drain before a served
# engine's admission): engine / model GPU tests, the headline bench, and two direct-service runs
# plus one with DRTC_MIXED_PIPELINE=0 on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5ah; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_model_gpu.py tests/test_service_gpu.py tests/test_model_real_shapes_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
echo "engine $(python3 -c "import json;print(json.load(open('$O/engine.json'))['value'])")"
for r in 1 2 off; do
  if [ $r = off ]; then export DRTC_MIXED_PIPELINE=0; fi
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
    --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc_$r.json 2> $O/svc_$r.err || { tail -5 $O/svc_$r.err; exit 1; }
  echo "svc $r $(python3 -c "import json;d=json.load(open('$O/svc_$r.json'));print(d['gen_tokens_per_s'],d['steady_gen_tokens_per_s'],d['p50_latency_ms'],d['replica_delta'])")"
done
