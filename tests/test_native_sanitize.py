"""Host-code sanitizers: the framework's header-only host algorithms are
compiled alone with AddressSanitizer + UndefinedBehaviorSanitizer (``-fsanitize=address,
undefined``, host code only — GPU sanitizers are not available on the MI355X pool) and
checked against a Python transcription on random inputs, including the n = 0 / 1 edge
cases.  Any sanitizer report makes the harness exit non-zero."""
import os
import shutil
import subprocess

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _sr_reference(a, b, u, pc):
    n = len(a)
    r = list(range(n))
    swapped, it = True, 0
    while it < (n + 1) // 2 and swapped:
        swapped = False
        for j in range(n - 1):
            key = a if u[j] < pc else b
            if key[r[j]] < key[r[j + 1]]:
                r[j], r[j + 1] = r[j + 1], r[j]
                swapped = True
        it += 1
    return r


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    cxx = shutil.which("g++") or shutil.which("clang++")
    if cxx is None:
        pytest.skip("no host C++ compiler")
    exe = str(tmp_path_factory.mktemp("native") / "host_sanitize")
    src = os.path.join(ROOT, "tests", "native", "host_sanitize.cpp")
    subprocess.run([cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
                    "-fno-sanitize-recover=all", src, "-o", exe], check=True)
    return exe


def test_stochastic_ranking_under_asan_ubsan(harness):
    g = torch.Generator().manual_seed(0)
    lines, refs = [], []
    for n in [0, 1, 2, 7, 64, 301]:
        a, b, u = torch.rand(n, generator=g), torch.rand(n, generator=g), torch.rand(max(n - 1, 0), generator=g)
        a[: n // 4] = 0.5  # ties
        vals = lambda t: " ".join(f"{float(x):.9g}" for x in t)
        lines.append(f"sr {n} 0.45 {vals(a)} {vals(b)} {vals(u)}")
        fl = lambda t: [float(f"{float(x):.9g}") for x in t]
        refs.append(_sr_reference(fl(a), fl(b), fl(u), 0.45))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([harness], input="\n".join(lines) + "\n", capture_output=True, text=True, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-2000:]
    got = [list(map(int, l.split())) for l in out.stdout.splitlines()]
    assert got == refs


def _tile_reference(M, N, mode, ov):
    if ov:
        t = 4 if (ov == 8 and mode != 0) else ov
    elif mode == 0 and M >= 2048 and N >= 64:
        t = 8
    else:
        t, best = 4, float("inf")
        for c in (4, 3, 2):
            b = 16 * c
            tm, tn = -(-M // b), -(-N // b)
            tiles = tm * tn if mode == 0 else tm * (tm + 1) // 2
            cost = ((tiles + 255) // 256) * float(b * b)
            if cost < best * 0.999:
                best, t = cost, c
    bm, bn = 16 * t, (64 if t == 8 else 16 * t)
    tm, tn = -(-M // bm), -(-N // bn)
    return t, (tm * tn if mode == 0 else tm * (tm + 1) // 2), tn


def test_gemm_tile_selection_under_asan_ubsan(harness):
    """The GEMM launch geometry (tile code, workgroups, column tiles — the latter two size the
    stats / row-terms partial buffers) for edge and flagship shapes, incl. 64-bit grids."""
    cases = [(1, 1, 0, 0), (16, 16, 1, 0), (1000, 1000, 1, 0), (1000, 1000, 2, 0), (10000, 1000, 0, 0), (5000, 1000, 0, 0),
             (2047, 64, 0, 0), (2048, 63, 0, 0), (300, 20, 0, 0), (257, 64, 0, 0), (1000, 1000, 0, 8), (1000, 1000, 1, 8),
             (123, 4567, 0, 3), (3_000_000, 100_000, 0, 0), (70_000, 70_000, 1, 0)]
    lines = [f"tile {M} {N} {mode} {ov}" for M, N, mode, ov in cases]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    out = subprocess.run([harness], input="\n".join(lines) + "\n", capture_output=True, text=True, env=env)
    assert out.returncode == 0, out.stderr[-2000:]
    assert "runtime error" not in out.stderr and "AddressSanitizer" not in out.stderr, out.stderr[-2000:]
    got = [tuple(map(int, l.split())) for l in out.stdout.splitlines()]
    assert got == [_tile_reference(*c) for c in cases]
