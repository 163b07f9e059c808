"""The multi-rank bench path on real engines (the world > 1 path had run only
over gloo with stubbed engine calls, tests/test_shard_gloo.py).

bench.py under torch.distributed.run with two ranks on the GPU box's one device
(GSDR_BENCH_SHARED_DEVICE=1: both ranks on device 0, the rank collectives over gloo,
since RCCL refuses two ranks on one device): process-group init, each rank's block span
and channel set (gsdr.shard), the barriers around the timed region and the
max-over-ranks time, with every rank running the real acquisition grids and tracking
pool on its share of the stream.  Rank 0's line must carry n_gpus 2, the rehearsal
label (never a scaling number), its share of the visible satellites acquired and its
channels converged (the bench's own check).  The 8-GPU RCCL run is the driver's."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks_one_device():
    env = dict(os.environ)
    env["GSDR_BENCH_SHARED_DEVICE"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONUNBUFFERED"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps",
           "3", "--warmup", "1", "--no-cpu-baseline"]
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = lines[0]
    print("two-rank line:", json.dumps({k: d[k] for k in ("value", "ms_per_step", "n_gpus", "rehearsal")}))
    assert d["n_gpus"] == 2 and "rehearsal" in d
    assert d["value"] > 0 and d["scaling"] == "weak"
    # rank 0: blocks [0, 64) of the 128-block stream and channels 0, 2, 4, 6
    assert "acquisition blocks [0,64)" in d["config"]["parallelism"]
    assert "channels [0, 2, 4, 6]" in d["config"]["parallelism"]
    chk = d["check"]
    assert chk["acquired_block0"] >= 1
    assert chk["channels_within_25hz"] == 4, chk
