"""Data-parallel equivalence on the GPU: 2 ranks (gloo, both on the one GPU of
the test box) with local batch b against one replica with batch 2b on the same samples, through
the staged backward + bucketed all-reduce of mmt_dist. The N-GPU RCCL run is bench.py's."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dp_two_ranks_match_single_replica():
    env = dict(os.environ)
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_port()}", os.path.join(HERE, "workers", "dp_equivalence.py")]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=100)
    print(r.stdout[-3000:])
    print(r.stderr[-3000:])
    assert r.returncode == 0
    assert "rank 0 ok" in r.stdout and "rank 1 ok" in r.stdout
