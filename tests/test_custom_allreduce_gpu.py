"""Custom one-/two-shot IPC all-reduce (csrc/kernels/allreduce.hip) with 2, 3
and 4 ranks as separate processes sharing the box's GPU: exact (bitwise) sums
vs a fixed-order fp32 reference, staging double-buffer reuse across both
kernels, hipGraph replay."""
import os
import subprocess
import sys

import pytest

from drtc_amd.utils.cluster import free_port

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_custom_allreduce_multiprocess(hipk, world):
    port = free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "ar_worker.py")],
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
