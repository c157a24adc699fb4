#!/bin/bash
# Round 5: kernel-trace anatomy of the headline on the current tree (per-phase busy/wall and the
# idle-gap attribution), then the engine bench and two gated direct-service runs on the same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/r5s; mkdir -p $O
bash scripts/gpu_prof_model.sh r5s --steps 2 --warmup 1 > $O/prof.out 2>&1
rc=$?; tail -3 $O/prof.out; [ $rc -eq 0 ] || exit $rc
mv gpurun_out/r5s_* gpurun_out/r5s.json $O/ 2>/dev/null
python scripts/trace_gaps.py $O/r5s_kernel_trace.csv.gz > $O/gaps.txt 2>&1 || true
head -3 $O/r5s_summary_full.md
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
echo "engine $(python3 -c "import json;d=json.load(open('$O/engine.json'));print(d['value'])")"
for r in 1 2; do
  timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend pool --client-procs 8 --mode direct \
    --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc_direct_$r.json 2> $O/svc_direct_$r.err || { tail -5 $O/svc_direct_$r.err; exit 1; }
  echo "svc direct $r $(python3 -c "import json;d=json.load(open('$O/svc_direct_$r.json'));print(d['gen_tokens_per_s'],d['steady_gen_tokens_per_s'],d['p50_latency_ms'],d['replica_delta'])")"
done
