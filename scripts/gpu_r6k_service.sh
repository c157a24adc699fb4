#!/bin/bash
# Round 6: the direct service path with ONE closed-loop client per engine
# slot (1,024) against the headline engine on the same box - front-end / backend / admission
# variants, one run each:  R6K_ARMS="tag:frontend:backend:ENV=VAL,..." (space-separated).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/${R6K_OUT:-r6k}; mkdir -p $O
# heartbeat file under gpurun_out/ (the service runs print only when they end)
( while sleep 50; do date +%s >> $O/heartbeat; done ) & HB=$!
trap "kill $HB 2>/dev/null" EXIT
# the T = 1024 MoE layer (Mixtral decode at batch 1024): kernel trace of the variant-3 / 4 arms
if [ "${R6K_MOE_TRACE:-1}" = 1 ]; then
  R=$PWD; cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof -o run -- python3 $R/scripts/moe_prefill_anatomy.py 1024 > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
  cd $R
  S=$(find $O/prof -name '*kernel_stats.csv' | head -1); cp "$S" $O/kernel_stats_moe1024.csv; rm -rf $O/prof
  grep "^T=" $O/prof.log
  python3 - "$O/kernel_stats_moe1024.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:12]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms  calls {r["Calls"]:>5}  avg {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
fi
timeout -k 10 400 python -u bench.py --steps 6 --warmup 2 > $O/engine.json 2> $O/engine.err || { tail -5 $O/engine.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/engine.json'));print('engine', d['value'])"
for arm in ${R6K_ARMS:-threads_pool:threads:pool: aio_pool:aio:pool: threads_engine:threads:engine:}; do
  IFS=: read tag fe be envs <<< "$arm"
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 400 python scripts/service_bench.py --model llama-3-8b --backend $be --frontend $fe \
    --client-procs 8 --mode direct --requests 20480 --concurrency 1024 --max-batch 1024 > $O/svc_$tag.json 2> $O/svc_$tag.err || { tail -5 $O/svc_$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/svc_$tag.json'));e=json.load(open('$O/engine.json'))['value'];print('svc $tag', d['gen_tokens_per_s'], round(100*d['gen_tokens_per_s']/e,1), '%', 'steady', d['steady_gen_tokens_per_s'], 'p50', d['p50_latency_ms'], 'errors', d['errors'])"
done
