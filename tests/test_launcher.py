"""bench.py --gpus N runs N ranks or fails loudly (evoxmi/parallel/launch.py).

The reference's distributed workflow spans every visible device
(/root/reference/src/evox/workflows/std_workflow.py:329-345); the benchmark entry point
must never report a one-GPU number for an N-GPU request.  Here the launcher is driven
with gloo ranks on the host (``--device cpu``, a tiny CMA-ES config).
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TINY = ["--pop", "32", "--dim", "12", "--steps", "2", "--warmup", "1", "--phase-steps", "0"]


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          timeout=timeout, env=e, cwd=ROOT)


def _line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out  # rank 0 alone prints
    return json.loads(lines[0])


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_spawns_n_gloo_ranks(n):
    r = _run(["--device", "cpu", "--gpus", str(n)] + TINY)
    assert r.returncode == 0, r.stderr[-2000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == n
    assert d["dist_backend"] == ("gloo" if n > 1 else None)
    assert d["rccl_world"] == 0  # gloo, not RCCL
    assert d["config"]["parallelism"] == f"pop-shard{n if n > 1 else 1}"
    assert d["gemm_precision"].startswith("bf16x6") or d["gemm_precision"] == "f32 MFMA"


def test_bench_refuses_more_gpus_than_visible():
    import torch

    have = torch.cuda.device_count()
    r = _run(["--gpus", str(max(have + 1, 2))] + TINY, timeout=120)
    assert r.returncode != 0
    assert "GPU(s) are visible" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_bench_refuses_world_size_mismatch():
    r = _run(["--device", "cpu", "--gpus", "2"] + TINY, env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"}, timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr


def test_spawn_ranks_reports_first_failure(tmp_path):
    from evoxmi.parallel.launch import spawn_ranks

    script = tmp_path / "r.py"
    script.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert spawn_ranks(3, [str(script)], device="cpu") == 3


def test_spawn_ranks_stops_ranks_blocked_on_a_dead_peer(tmp_path):
    """Rank 1 exits non-zero after rendezvous while rank 0 waits in a barrier: the launcher
    returns rank 1's status promptly and terminates rank 0 (no hang, no orphan)."""
    import time

    from evoxmi.parallel.launch import spawn_ranks

    pidfile = tmp_path / "pid0"
    script = tmp_path / "r.py"
    script.write_text(
        "import os, sys, datetime\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo', timeout=datetime.timedelta(seconds=600))\n"
        "if dist.get_rank() == 1:\n"
        "    sys.exit(5)\n"
        f"open({str(pidfile)!r}, 'w').write(str(os.getpid()))\n"
        "dist.barrier()\n"
    )
    t0 = time.monotonic()
    assert spawn_ranks(2, [str(script)], device="cpu", timeout=300) == 5
    assert time.monotonic() - t0 < 120
    if pidfile.exists():
        pid = int(pidfile.read_text())
        with pytest.raises(ProcessLookupError):
            os.kill(pid, 0)  # reaped: no process left behind


def test_spawn_ranks_timeout_kills_every_rank(tmp_path):
    from evoxmi.parallel.launch import spawn_ranks

    script = tmp_path / "r.py"
    script.write_text("import time\ntime.sleep(600)\n")
    assert spawn_ranks(2, [str(script)], device="cpu", timeout=2) == 124
