"""bench.py contract under the multi-rank launcher (gloo on CPU, tiny GPT-2): the driver runs
``torch.distributed.run --nproc-per-node N bench.py --gpus N`` and parses ONE JSON line from rank 0."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("n", [2, 4])
def test_bench_multirank_json_line(n):
    env = dict(os.environ, CUDA_VISIBLE_DEVICES="", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "2", "--warmup", "1",
           "--model", "gpt2-tiny", "--seq-len", "32", "--batch-per-gpu", "4"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["steps"] == 2 and d["warmup"] == 1
    assert d["config"]["global_batch"] == 4 * n and d["config"]["parallelism"] == f"pp{n}"
    assert d["value"] > 0 and d["higher_is_better"] is True and d["scaling"] == "weak"
    assert d["config"]["last_loss"] is not None
