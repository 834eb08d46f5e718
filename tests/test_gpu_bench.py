"""bench.py end to end on the GPU: the JSON contract, and the sharded N-rank
path (contiguous shards + one sum-reduce) giving the same folded power sums
as one rank over the same global stream, and as the CPU oracle."""
import json
import os
import subprocess
import sys

import pytest

from oracle import coracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(cmd, timeout=600):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0])


def test_bench_contract_and_sharded_parity():
    n_total, seed, t = 40_000_000, 0x5EED0002, 32
    one = run([sys.executable, "bench.py", "--steps", "3", "--warmup", "1", "--ids-per-gpu", str(n_total),
               "--cpu-sample", "2e6"])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in one
    assert one["n_gpus"] == 1 and one["steps"] == 3 and one["value"] > 0
    rf = one["roofline"]
    assert rf["bound"] == "hbm" and rf["unit"] == "GB/s" and abs(rf["frac"] - rf["achieved"] / rf["peak"]) < 1e-9
    v = rf["valu"]                        # the integer-issue roofline (tools/issue_model.py)
    assert v["bound"] == "valu-issue" and 0 < v["frac"] < 1.5 and abs(v["frac"] - v["peak"] / v["achieved"]) < 1e-9
    assert 1.0 < one["clock_ghz"] < 3.0 and v["clock_ghz"] == one["clock_ghz"]   # this run's shader clock
    assert v["anchor"]["ops_per_id"] == {"lazy_modmuls": 9, "macs": 24, "row0_adds": 8}
    cb = one["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["parity_with_gpu"] is True
    # the crate's own unit: TSC ticks around the insert loop, the TSC rate from the same region
    assert cb["tsc_cycles_per_id"] > 0 and 0.5 < cb["tsc_ghz"] < 6 and cb["published_crate_tsc_cycles_per_id"] > 0
    assert abs(cb["tsc_cycles_per_id"] - cb["ns_per_id"] * cb["tsc_ghz"]) < 1e-6 * cb["tsc_cycles_per_id"] + 1e-3
    want = coracle.encode_u32_seed(seed, n_total, t)
    assert one["result"]["power_sums_head"] == want[:4] and one["result"]["count"] == n_total

    two = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", "29561", "bench.py", "--gpus", "2", "--steps", "3",
               "--warmup", "1", "--ids-per-gpu", str(n_total // 2), "--dist-backend", "host"])
    assert two["n_gpus"] == 2 and two["cpu_baseline"] is None
    assert two["config"]["collectives"] == "host" and "rehearsal" in two["config"]["workload"]
    assert two["result"]["digest"] == one["result"]["digest"]
    assert two["result"]["count"] == n_total
    # the untimed strong-scaling pass: the N = 1 stream of --ids-per-gpu ids in 2 shards through the
    # same communicator equals rank 0's single-GPU encode of it
    p = two["parity"]
    assert p["equals_n1"] is True and p["last_value_equal"] is True
    import hashlib
    want2 = coracle.encode_u32_seed(seed, n_total // 2, t)
    assert p["digest"] == hashlib.sha256((",".join(map(str, want2)) + f"|{n_total // 2}").encode()).hexdigest()[:16]
    assert len(two["ranks"]) == 2 and [r["rank"] for r in two["ranks"]] == [0, 1]
    # the untimed sharded decode (configs[4]'s protocol on a log of --ids-per-gpu ids): the broadcast and
    # all-gathers give rank 0's single-GPU hit list, every drop among the hits
    dp = two["decode_parity"]
    assert dp["equals_single_gpu"] is True and dp["drops_recovered"] is True and dp["d"] == 32 and dp["hits"] >= 32
    assert "rccl" not in two                   # host channel: no RCCL communicator to report


def test_bench_native_comm_world1_matches():
    """bench.py's native multi-GPU step (encode + one ncclReduce through
    qk_comm, comm.hip) at world 1: same folded result as the plain step."""
    n_total = 20_000_000
    a = run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--ids-per-gpu", str(n_total),
             "--cpu-sample", "0"])
    b = run([sys.executable, "bench.py", "--steps", "2", "--warmup", "1", "--ids-per-gpu", str(n_total),
             "--cpu-sample", "0", "--comm"])
    assert a["result"]["digest"] == b["result"]["digest"] and b["result"]["count"] == n_total
    assert b["roofline"]["kernel_avg_ms"] > 0
