"""The native communicator between PROCESSES on the GPU box (verdict r03
missing #4): two ranks, each its own process on device 0 under
torch.distributed.run, each with Comm.init_host(ProcessGroupChannel()) — the
comm.hip protocol (payload packing, failed-rank word, root fold, status and
hit gathers, staging-fault handling) with a real process boundary, as
bench.py --gpus N rehearses it.  (RCCL itself takes one rank per GPU, so two
RCCL ranks need two GPUs: tests/test_gpu_multidev.py on the 8-GPU node.)"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_processes_native_protocol(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", "29571", "tests/mp_comm_worker.py",
                        str(tmp_path)], cwd=ROOT, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    res = [json.load(open(tmp_path / f"rank{k}.json")) for k in range(2)]
    for d in res:
        bad = {k: v for k, v in d.items() if k not in ("rank", "world", "fault_decode_rc") and v is not True}
        assert not bad, (d["rank"], bad, d.get("fault_decode_rc"))
