"""bench.py's multi-rank path end to end on CPU: ``--gpus 2`` with no
torchrun environment makes bench.py start ``torch.distributed.run`` itself as a
child process; the two ranks (gloo) run the ChunkPipeline baton ring on a toy
model and rank 0 prints the one JSON line, with n_gpus = 2 and outputs equal to
the one-rank run (the driver's N = 1, 2, 4, 8 scaling command takes this path;
run_model.py:472 is the reference's DDP launch)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "selftest", "--steps", "2",
                        "--warmup", "1", "--seq-frames", "44", "--frames", "6", "--overlap", "2", *argv],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    return lines[0]


def test_bench_launches_ranks_itself():
    one = _bench("--gpus", "1")
    two = _bench("--gpus", "2")
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["value"] > 0 and two["steps"] == 2
    for k, v in one["checksum"].items():
        assert abs(two["checksum"][k] - v) <= 1e-6 * max(1.0, abs(v)), (k, v, two["checksum"][k])
