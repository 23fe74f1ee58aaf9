"""examples/ run on the CPU, and the reference's published config-1 result is pinned.

The reference's pso_ackley.ipynb (cells 6-7) prints best fitness 0.0 at
x = (-4.0062014e-07, 5.2837186e-07) after 100 generations of PSO (pop 100, bounds ±32) on
Ackley d = 2 with key 42.  At such an x the f32 Ackley is one rounding step above zero (≈9.5e-7:
20 − 20·exp(−0.2·|x|/√2) − e + e^{cos…} loses its last bits), so the pin is best ≤ 1e-6 and
|x|∞ ≤ 1e-6 — parity within f32 rounding (the streams differ: Philox here, threefry there)."""
import importlib.util
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "examples", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_pso_ackley_matches_the_reference_notebook():
    best, x = _load("pso_ackley").run("cpu", generations=100, seed=42)
    assert best <= 1e-6, best
    assert float(x.abs().max()) <= 1e-6, x


def test_custom_algorithm_and_problem():
    trace, sol = _load("custom_algorithm_and_problem").run("cpu", generations=40)
    assert trace == sorted(trace)  # best-so-far never decreases (maximisation)
    assert trace[-1] >= 95 and int(sol.sum()) == int(trace[-1])


def test_coevolution_example():
    assert _load("coevolution").run("cpu", generations=200) < 0.5


def test_neuroevolution_cartpole_example():
    best = _load("neuroevolution_cartpole").run("cpu", generations=20)
    assert best[-1] >= 150 and best[-1] >= best[0]


def test_distributed_cmaes_example_two_gloo_ranks(tmp_path):
    ck = str(tmp_path / "ck.safetensors")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "distributed_cmaes.py"), "--gpus", "2", "--device", "cpu",
                        "--generations", "10", "--checkpoint", ck], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "ranks 2: best fitness" in r.stdout and os.path.exists(ck)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "examples", "distributed_cmaes.py"), "--device", "cpu",
                        "--generations", "5", "--checkpoint", ck, "--resume"], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "after 15 generations" in r.stdout


def test_knob_table_is_current():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "knob_table.py")], capture_output=True, text=True, timeout=120)
    with open(os.path.join(ROOT, "docs", "knobs.md")) as f:
        assert r.stdout == f.read(), "regenerate docs/knobs.md: python tools/knob_table.py > docs/knobs.md"
