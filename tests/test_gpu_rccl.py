"""Partitioned GO through the RCCL transport: two processes (torch.distributed.run), one engine
each, checked against a single engine (tools/rccl_probe.py).  On a one-GPU box both ranks share
device 0 and RCCL carries the exchange over its socket transport (distinct NCCL_HOSTID); on a
multi-GPU node the same calls run over xGMI."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_partitioned_two_processes():
    """Parity, then failures forced on ONE rank (a duplicated-hub start list over one rank's 2^32
    edge limit; injected allocation failures in GO and FIND PATH): both processes must return
    the same code and keep answering.  NBG_COMM_TIMEOUT_S bounds any wait on a peer."""
    env = dict(os.environ, NBG_COMM_TIMEOUT_S="60")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", "29517", os.path.join(ROOT, "tools", "rccl_probe.py"),
           "--same-device"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=150, env=env)
    assert p.returncode == 0 and "RCCL partitioned probe: PASS" in p.stdout, p.stdout[-3000:] + p.stderr[-3000:]
