"""bench.py's driver contract on CPU (gloo): one JSON line from rank 0 with the
whole-job value, max-over-ranks timing and DP global batch."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARGS = ["--steps", "1", "--warmup", "0", "--model", "tiny-llama", "--batch", "4",
        "--max-new-tokens", "4", "--max-model-len", "1024"]


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _json_line(out: str) -> dict:
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def _check(r: dict, n: int) -> None:
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r, k
    assert r["n_gpus"] == n and r["steps"] == 1 and r["warmup"] == 0
    # self-verification of the multi-rank run: one device entry per rank, the collective
    # backend and the communicator size as the process group reports them
    assert len(r["devices"]) == n and r["rccl_world"] == n
    assert r["backend"] == ("gloo" if n > 1 else "none")
    # seq_len = average prompt + generated tokens per sequence
    assert r["config"]["seq_len"] == round(r["config"]["avg_prompt_tokens"] + 4)
    assert r["value"] > 0 and r["higher_is_better"] is True and r["scaling"] == "weak"
    assert r["config"]["global_batch"] == 4 * n
    assert r["config"]["parallelism"] == f"dp{n}"
    # value is the whole-job aggregate: generated tokens of every rank / max time
    assert abs(r["value"] - 4 * n * 4 / (r["ms_per_step"] / 1000)) / r["value"] < 0.05


def test_bench_single_process():
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *ARGS], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_json_line(p.stdout), 1)


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_json_line(p.stdout), 2)


def test_bench_open_loop_poisson():
    """--arrival-rate: Poisson arrivals, latency from the scheduled arrival,
    p50/p99 latency / TTFT / TPOT; mixed prefill+decode steps happen."""
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    args = ["--steps", "1", "--warmup", "0", "--model", "tiny-llama", "--batch", "8",
            "--max-new-tokens", "6", "--max-model-len", "1024", "--arrival-rate", "200",
            "--requests", "24", "--mixed-tokens", "512"]
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = _json_line(p.stdout)
    assert r["mode"] == "open-loop" and r["requests_per_replica"] == 24
    for k in ("p50_latency_ms", "p99_latency_ms", "p50_ttft_ms", "p99_ttft_ms",
              "p50_tpot_ms", "p99_tpot_ms"):
        assert r[k] > 0, k
    assert r["p99_latency_ms"] >= r["p50_latency_ms"]
    assert r["engine_stats"]["mixed_steps"] > 0
    assert r["steady_req_per_s"] >= 0 and r["steady_gen_tokens_per_s"] >= 0


def test_service_bench_open_loop_scripted():
    """scripts/service_bench.py --arrival-rate: open-loop Poisson RPCs against
    the LLM gRPC service (scripted backend), latency from the scheduled send."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "service_bench.py"),
                        "--backend", "scripted", "--requests", "40", "--arrival-rate", "150"],
                       cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    r = _json_line(p.stdout)
    assert r["load"].startswith("open-loop") and r["requests"] == 40 and r["errors"] == 0
    assert r["p99_latency_ms"] >= r["p50_latency_ms"] > 0


def test_bench_self_launch_two_ranks():
    """`python bench.py --gpus 2` with no torchrun: the script starts its two rank
    processes itself (gloo here, RCCL on GPUs) and reports the whole-job value."""
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    _check(_json_line(p.stdout), 2)


def test_bench_world_size_mismatch_is_an_error():
    env = dict(os.environ, RANK="0", WORLD_SIZE="1", LOCAL_RANK="0")
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", *ARGS],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0 and not [ln for ln in p.stdout.splitlines() if ln.startswith("{")]


def _self_launch(n: int, extra: list[str]) -> dict:
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), *extra],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    return _json_line(p.stdout)


def test_bench_self_launch_tensor_parallel():
    """`bench.py --gpus 2 --tp 2`: one TP group over both ranks (all-reduce after o / down),
    the same requests on every rank: global batch = one replica's, scaling strong."""
    r = _self_launch(2, ["--tp", "2", *ARGS])
    assert r["config"]["parallelism"] == "tp2" and r["config"]["global_batch"] == 4
    assert r["scaling"] == "strong" and r["n_gpus"] == 2 and r["rccl_world"] == 2
    assert r["backend"] == "gloo" and len(r["devices"]) == 2
    assert abs(r["value"] - 4 * 4 / (r["ms_per_step"] / 1000)) / r["value"] < 0.05


def test_bench_self_launch_tp_ep_mixtral():
    """Mixtral-shaped MoE over a 4-rank TP group with expert parallelism (the experts split
    over the ranks, tokens exchanged by all-to-all): the path of the Mixtral EP=8 config."""
    args = ["--steps", "1", "--warmup", "0", "--model", "tiny-mixtral", "--batch", "4",
            "--max-new-tokens", "4", "--max-model-len", "1024", "--workload", "suggest"]
    r = _self_launch(4, ["--tp", "4", *args])
    assert r["config"]["parallelism"] == "tp4" and r["config"]["model"] == "tiny-mixtral"
    assert r["rccl_world"] == 4 and len(r["devices"]) == 4
    assert r["engine_stats"]["decode_tokens"] >= 4 * 3
