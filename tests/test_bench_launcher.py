"""bench.py --gpus N starts N ranks itself (torch.distributed.run, 127.0.0.1) when no
launcher did; --dry-run stops after the rendezvous (gloo, no GPU) and rank 0 reports the
world size the process group actually holds."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_launches_its_own_ranks():
    env = dict(os.environ, GS_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                         env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
    assert json.loads(line)["n_gpus"] == 2
