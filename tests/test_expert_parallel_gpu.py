"""Expert all-to-all (parallel/expert_parallel.py) with the fused HIP expert kernel:
2 and 4 ranks as separate processes on the box's GPU, exact-split and
static-capacity forms vs the single-process fp32-accumulated MoE reference."""
import os
import subprocess
import sys

import pytest

from drtc_amd.utils.cluster import free_port

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 4])
def test_ep_all_to_all_fused_experts_multiprocess(hipk, world):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "ep_worker.py")],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                                      text=True))
    outs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=240)
            outs.append((p.returncode, out))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, (rc, out) in enumerate(outs):
        assert rc == 0, f"rank {r} rc={rc}\n{out[-3000:]}"
        assert f"rank {r}: OK" in out
