"""Time-budgeted DE harness on CEC2022 (parity with the reference fork's ``run/run_de.py``).

For every function of the suite and every independent run, the optimiser runs until
``--max-time`` seconds have elapsed; after each generation the elapsed fraction is
injected into the algorithm state as ``progress`` (and the step count as ``iter``),
which drives the L-SHADE-family schedules (reference ``run/run_de.py:74-94``).
Results are appended to ``<out>/result_de.txt`` (best fitness of runs 2..R and the
FE count) and ``<out>/result_de_history.txt`` (best-so-far history of the median run,
``--samples`` points).

MI355X-specific: with ``--graph`` (default on a GPU) each generation is one hipGraph
replay; the best-so-far value is read back only every ``--sync-every`` generations so
the host never stalls the queue for the time check.  ``--concurrent K`` runs K
independent runs at once, each on its own HIP stream (a pop-100, d-20 generation
occupies a handful of CUs, so K graphs replayed on K streams overlap on the 256 CUs);
every run still gets its own ``--max-time`` wall-clock budget.

``--batched`` runs ALL ``--runs`` independent runs as one vmapped computation
(:class:`evoxmi.algorithms.BatchedRuns`): one (runs·pop, d) evaluation and one launch
sequence (one hipGraph replay) per generation advance every run, sharing the wall-clock
budget.  Run ``r`` uses the same per-run key in both modes (``split(fold_in(key_f, 1),
runs)[r]``), so with ``--progress steps`` (progress = step / --max-steps, no clock)
the batched and sequential harnesses compute the same runs.

Example: ``python run/run_de.py --algo LSHADE --dim 20 --pop 100 --runs 4 --max-time 5``
"""
from __future__ import annotations

import argparse
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402


class _nullcontext:
    def __enter__(self):
        return None

    def __exit__(self, *a):
        return False


def sample_history(num_samples, hist):
    if not hist:
        return []
    n = len(hist)
    idx = [int(i * (n - 1) / max(num_samples - 1, 1)) for i in range(num_samples)]
    return [hist[i] for i in idx]


def main(argv=None):
    from evoxmi import random as rnd
    from evoxmi.algorithms import de_variants
    from evoxmi.monitors import EvalMonitor
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", default="EVDE", choices=de_variants.__all__)
    ap.add_argument("--funcs", default="1-12")
    ap.add_argument("--dim", type=int, default=20)
    ap.add_argument("--pop", type=int, default=100)
    ap.add_argument("--runs", type=int, default=32)
    ap.add_argument("--max-time", type=float, default=60.0)
    ap.add_argument("--max-steps", type=int, default=9999999)
    ap.add_argument("--samples", type=int, default=100)
    ap.add_argument("--sync-every", type=int, default=10)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--out", default="run")
    ap.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--concurrent", type=int, default=1, help="independent runs executed at once on separate HIP streams")
    ap.add_argument("--batched", action="store_true", help="all runs as one vmapped computation (BatchedRuns)")
    ap.add_argument("--progress", choices=("time", "steps"), default="time",
                    help="progress injected into the state: elapsed/--max-time (reference) or step/--max-steps")
    ap.add_argument("--json", default=None, help="write a per-function summary (aggregate gens/s, best values)")
    args = ap.parse_args(argv)

    a, _, b = args.funcs.partition("-")
    funcs = list(range(int(a), int(b or a) + 1))
    dev = torch.device(args.device)
    graph = dev.type == "cuda" and not args.no_graph
    D = args.dim
    lb, ub = torch.full((D,), -100.0, device=dev), torch.full((D,), 100.0, device=dev)
    os.makedirs(args.out, exist_ok=True)
    res_path, hist_path = os.path.join(args.out, "result_de.txt"), os.path.join(args.out, "result_de_history.txt")
    header = f"Problem_Dim: {D}, Time: {args.max_time}, Optimizer: {args.algo}, Popsize: {args.pop}, Iters: {args.max_steps}\n\n"
    for pth in (res_path, hist_path):
        with open(pth, "w") as f:
            f.write(header)
    key = rnd.PRNGKey(args.seed, device=dev)
    summary = {}
    for fn in funcs:
        problem = CEC2022TestSuit.create(fn)
        name = type(problem).__name__
        print(name, flush=True)
        with open(res_path, "a") as f:
            f.write(f"{name}  ")
        with open(hist_path, "a") as f:
            f.write(f"{name}  ")
        best_all, hist_all = [], []
        steps = 0
        K = max(1, args.concurrent)
        fkey = rnd.fold_in(key, fn)
        run_keys = rnd.split(rnd.fold_in(fkey, 1), args.runs)
        if args.batched:
            best_all, hist_all, steps, gps = _run_batched(args, problem, lb, ub, fkey, graph, dev)
            summary[name] = {"gens_per_s_aggregate": gps, "steps": steps, "best": best_all}
            with open(res_path, "a") as f:
                f.write(" ".join(str(b) for b in best_all) + f" {steps * args.pop}\n")
            order = sorted(range(len(best_all)), key=lambda k: best_all[k])
            with open(hist_path, "a") as f:
                f.write(f"{hist_all[order[len(order) // 2]]}\n")
            continue
        t_fn = time.time()
        gens_total = 0
        for run0 in range(0, args.runs, K):
            batch = list(range(run0, min(args.runs, run0 + K)))
            jobs = []
            for run in batch:
                algo = getattr(de_variants, args.algo)(lb=lb, ub=ub, pop_size=args.pop)
                mon = EvalMonitor(full_fit_history=False)
                wf = StdWorkflow(algo, problem, monitors=[mon], graph=graph)
                st0 = _with_algorithm_key(wf.init(fkey), algo, run_keys[run])
                stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" and K > 1 else None
                jobs.append({"run": run, "wf": wf, "mon": mon, "state": st0, "hist": [], "stream": stream, "steps": 0, "done": False})
            t0 = time.time()
            for i in range(args.max_steps):
                active = [j for j in jobs if not j["done"]]
                if not active:
                    break
                for j in active:
                    with torch.cuda.stream(j["stream"]) if j["stream"] is not None else _nullcontext():
                        state = j["wf"].step(j["state"])
                        j["steps"] = i
                        if i % args.sync_every == 0 or i == args.max_steps - 1:
                            j["hist"].append(float(j["mon"].get_best_fitness()))
                        elapsed = time.time() - t0
                        alg = state.get_child_state("algorithm")
                        upd = {}
                        if "progress" in alg.keys():
                            upd["progress"] = elapsed / args.max_time if args.progress == "time" else (i + 1) / args.max_steps
                        if "iter" in alg.keys() and not isinstance(alg.iter, torch.Tensor):
                            upd["iter"] = i
                        if upd:
                            state = state.update_child("algorithm", alg.update(**upd))
                        j["state"] = state
                        if elapsed >= args.max_time or (args.progress == "steps" and i + 1 >= args.max_steps):
                            j["done"] = True
            if dev.type == "cuda":
                torch.cuda.synchronize()
            for j in jobs:
                run, steps = j["run"], j["steps"]
                gens_total += steps + 1
                best = float(j["mon"].get_best_fitness())
                j["hist"].append(best)
                print(f"min fitness: {best}\nSteps: {steps} Runs: {run}\nTime: {time.time() - t0:.3f} s\n", flush=True)
                if run >= 1 or args.runs == 1:
                    best_all.append(best)
                    hist_all.append(sample_history(args.samples, j["hist"]))
                    with open(res_path, "a") as f:
                        f.write(f"{best} ")
        with open(res_path, "a") as f:
            f.write(f"{steps * args.pop}\n")
        summary[name] = {"gens_per_s_aggregate": gens_total / (time.time() - t_fn), "steps": steps, "best": best_all}
        order = sorted(range(len(best_all)), key=lambda k: best_all[k])
        med = order[len(order) // 2]
        with open(hist_path, "a") as f:
            f.write(f"{hist_all[med]}\n")
    if args.json:
        import json

        with open(args.json, "w") as f:
            json.dump({"algo": args.algo, "dim": D, "pop": args.pop, "runs": args.runs, "batched": args.batched,
                       "functions": summary}, f)
    return summary


def _with_algorithm_key(state, algo, key):
    """Re-initialise the algorithm's sub-state from ``key`` (keeping its node id)."""
    st, _ = algo._recursive_init(key, algo._node_id, algo._module_name, False)
    return state.update_child("algorithm", st)


def _run_batched(args, problem, lb, ub, fkey, graph, dev):
    """All runs of one function as one vmapped computation; returns (best of runs
    2..R (all if R == 1), sampled median history, steps, aggregate generations/s)."""
    from evoxmi import random as rnd
    from evoxmi.algorithms import de_variants
    from evoxmi.algorithms.containers.batched import BatchedRuns
    from evoxmi.workflows import StdWorkflow

    algo = BatchedRuns(getattr(de_variants, args.algo)(lb=lb, ub=ub, pop_size=args.pop), args.runs)
    wf = StdWorkflow(algo, problem, graph=graph)
    # the runs' keys are split(fold_in(fkey, 1), R) exactly as in the sequential harness
    state = _with_algorithm_key(wf.init(fkey), algo, rnd.fold_in(fkey, 1))
    has_progress = "progress" in state.get_child_state("algorithm").runs.keys()
    hist = []
    t0 = time.time()
    i = 0
    while i < args.max_steps:
        state = wf.step(state)
        elapsed = time.time() - t0
        alg = state.get_child_state("algorithm")
        if i % args.sync_every == 0:
            hist.append(algo.best_fitness(alg).tolist())
        if has_progress:
            prog = elapsed / args.max_time if args.progress == "time" else (i + 1) / args.max_steps
            state = state.update_child("algorithm", algo.set_field(alg, progress=prog))
        i += 1
        if elapsed >= args.max_time:
            break
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.time() - t0
    best = algo.best_fitness(state.get_child_state("algorithm")).tolist()
    hist.append(best)
    keep = list(range(1, args.runs)) if args.runs > 1 else [0]
    steps = i - 1
    print(f"batched {args.runs} runs: {i} generations in {dt:.3f} s "
          f"({i * args.runs / dt:.0f} aggregate gens/s); best {min(best)}", flush=True)
    bests = [best[r] for r in keep]
    order = sorted(keep, key=lambda r: best[r])
    med = order[len(order) // 2]
    return bests, sample_history(args.samples, [h[med] for h in hist]), steps, i * args.runs / dt


if __name__ == "__main__":
    main()
