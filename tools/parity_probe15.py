"""Per-seed trajectories behind tests/test_eigh_sbr.py::test_cmaes_trajectories_sbr_vs_library_eigh
for seeds 7-21 and every correction precision (torch = rocSOLVER reference), written as JSON lines
so that the test's statistics can be recomputed for any seed subset offline.

    python tools/parity_probe15.py OUT.jsonl
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from parity_probe import traj  # noqa: E402


def main():
    out = sys.argv[1]
    with open(out, "w") as fh:
        for impl, prec in (("torch", "x6"), ("sbr", "x3"), ("sbr", "x3all"), ("sbr", "x6")):
            for s in range(7, 22):
                f = traj(impl, s, prec)
                fh.write(json.dumps({"impl": impl, "prec": prec, "seed": s, "f": f}) + "\n")
                fh.flush()
                print(impl, prec, s, f[10], f[99], flush=True)


if __name__ == "__main__":
    main()
