"""Run bench.py with module constants overridden (A/B of tuned constants that are not knobs).

    python tools/bench_ab.py evoxmi.ops.sbr_device.ORDER2_THR=0 -- --steps 20 --warmup 5
"""
import ast
import importlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    argv = sys.argv[1:]
    cut = argv.index("--") if "--" in argv else len(argv)
    for item in argv[:cut]:
        name, val = item.split("=", 1)
        mod, attr = name.rsplit(".", 1)
        setattr(importlib.import_module(mod), attr, ast.literal_eval(val))
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv[cut + 1 :]
    import runpy

    runpy.run_path(os.path.join(ROOT, "bench.py"), run_name="__main__")


if __name__ == "__main__":
    main()
