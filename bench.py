"""Flagship benchmark: CMA-ES pop=10 000 on CEC'22 (F1, shifted-rotated Zakharov), d=1000.

Metric (BASELINE.json): generations/s and evaluations/s of one full generation
(ask → evaluate → tell incl. the per-generation eigendecomposition).  ``value`` is
the whole-job evaluations/s (λ × generations/s); N GPUs share one population of
λ = 10 000 (population-sharded SPMD over RCCL ⇒ strong scaling).

Data: synthetic CEC'22 F1 instance at d = 1000 (seeded shift vector and
Haar-random rotation — the reference ships CEC data only for D ∈ {2, 10, 20}),
random initial mean; fp32 compute (the reference runs CMA-ES in float32).

Usage: ``python bench.py [--gpus N] [--steps K] [--warmup W]``; with N > 1 the
driver launches it under ``torch.distributed.run`` (one rank per GPU).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pop", type=int, default=10000)
    ap.add_argument("--dim", type=int, default=1000)
    ap.add_argument("--func", type=int, default=1)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--profile-phases", action="store_true")
    ap.add_argument("--force-dist", action="store_true", help="run the distributed (sharded + RCCL) path even on one rank")
    ap.add_argument("--phase-steps", type=int, default=3, help="eager generations timed per phase after the timed loop (0: off)")
    ap.add_argument("--simulate-rank", type=int, default=None,
                    help="time rank R's share of a --world N step on this one GPU (collectives replaced by same-size local ops)")
    ap.add_argument("--world", type=int, default=8, help="world size simulated by --simulate-rank")
    ap.add_argument("--link-gbps", type=float, default=None, help="--simulate-rank wire model: GB/s per xGMI link and direction")
    ap.add_argument("--latency-us", type=float, default=None, help="--simulate-rank wire model: latency per collective (µs)")
    ap.add_argument("--monitor", nargs="?", const="host", default=None, choices=["host", "device", "best"],
                    help="attach an EvalMonitor in the timed loop: full fitness history copied to the host "
                         "asynchronously (host), kept on the device (device), or best-so-far only (best)")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: gloo ranks on the host (tests of the launcher only; not a benchmark)")
    args = ap.parse_args()

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    # --gpus N without torchrun: spawn N rank processes here, before this process makes any
    # HIP call, or fail loudly when fewer than N GPUs are visible (evoxmi/parallel/launch.py)
    from evoxmi.parallel.launch import LaunchError, ensure_ranks

    if args.simulate_rank is None:
        try:
            ensure_ranks(args.gpus, device=args.device)
        except LaunchError as e:
            print(f"bench.py: {e}", file=sys.stderr, flush=True)
            sys.exit(2)
    from evoxmi import config
    from evoxmi import random as rnd
    from evoxmi.algorithms import CMAES
    from evoxmi.parallel import init_distributed
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow
    import torch.distributed as dist

    sim = args.simulate_rank is not None
    if sim:
        rank, world, device = 0, 1, torch.device("cuda", 0)
        torch.cuda.set_device(device)
    else:
        rank, world, device = init_distributed(backend="gloo" if args.device == "cpu" else None, force=args.force_dist)
        if world != args.gpus:
            print(f"bench.py: --gpus {args.gpus} but the job has {world} rank(s)", file=sys.stderr, flush=True)
            sys.exit(2)
    if device.type != "cuda" and args.device == "cuda":
        print("bench.py: no HIP device visible", file=sys.stderr, flush=True)
        sys.exit(2)
    torch.manual_seed(0)
    key = rnd.PRNGKey(2024, device=device)
    center = (torch.rand(args.dim, generator=torch.Generator().manual_seed(1)) * 160 - 80).to(device)
    algo = CMAES(center_init=center, init_stdev=20.0, pop_size=args.pop)
    prob = CEC2022TestSuit.create(args.func)
    use_graph = (not args.no_graph) and device.type == "cuda"
    monitors = []
    if args.monitor:
        from evoxmi.monitors import EvalMonitor

        monitors = [EvalMonitor(full_fit_history=args.monitor != "best", history_to_host=args.monitor == "host")]
    # "auto": a step that cannot be captured (e.g. a collective the communicator refuses to
    # record) runs eagerly instead of ending the run; the JSON reports which one was timed
    wf = StdWorkflow(algo, prob, graph="auto" if use_graph else False, monitors=monitors)
    state = wf.init(key)
    dist_on = (world > 1 or args.force_dist) and not sim
    if dist_on:
        state = wf.enable_distributed(state)
    sim_ctx = None
    if sim:
        from evoxmi.parallel.context import SimulatedDistContext

        sim_ctx = SimulatedDistContext(args.simulate_rank, args.world, algorithm=algo)
        if args.link_gbps:
            sim_ctx.wire.link_gbps = args.link_gbps
        if args.latency_us is not None:
            sim_ctx.wire.latency_us = args.latency_us
        state = wf.enable_distributed(state, context=sim_ctx)

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)
        if dist_on:
            dist.barrier()

    from evoxmi.ops import eigh as eigh_mod

    from evoxmi.ops import sbr_device

    for _ in range(args.warmup):
        state = wf.step(state)
    if use_graph and hasattr(wf, "prepare_graphs"):
        # every graph variant the timed generations replay is captured here, not inside the timing
        state = wf.prepare_graphs(state, args.steps + 1)
    sync()
    eigh_mod.HISTORY.clear()
    dev_counts = sbr_device.snapshot_counts()  # device-mode solves: per-solve ring read after timing
    if sim_ctx is not None:
        sim_ctx.counters.reset()  # wire accounting of the timed generations only
    t0 = time.perf_counter()
    for _ in range(args.steps):
        state = wf.step(state)
    sync()
    elapsed = time.perf_counter() - t0
    wire = sim_ctx.counters.summary(args.steps, sim_ctx.wire, args.world, graph=use_graph) if sim_ctx is not None else None
    # per-phase breakdown (outside the timed region): a few eager generations with
    # stream-ordered hipEvent timers; "tell" includes "eigh" (and "all_reduce" when sharded)
    hist = list(eigh_mod.HISTORY)  # decompositions of the timed generations only (host mode)
    dev_hist = sbr_device.histories_since(dev_counts)  # [off_rel, 0, iterations, fallback] (device mode)
    phases = None
    if args.phase_steps > 0:
        from evoxmi.utils.profiling import PhaseTimer

        timer = PhaseTimer(device)
        wf.phase_timer = timer
        graph_on, wf.graph = wf.graph, False
        for _ in range(args.phase_steps):
            state = wf.step(state)
        sync()
        wf.graph, wf.phase_timer = graph_on, None
        phases = {k: round(v["mean_ms"], 4) for k, v in timer.summary().items()}
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if dist_on:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    ms = elapsed / args.steps * 1e3
    gens_per_s = args.steps / elapsed
    evals_per_s = gens_per_s * args.pop
    backend = dist.get_backend() if dist_on else None
    if rank == 0:
        out = {
            "metric": "generations/sec + evaluations/sec, CMA-ES pop=10k on CEC'22 at 1/2/4/8 MI355X",
            "value": round(evals_per_s, 1),
            "unit": "evals/s (evaluations/sec; generations/sec in generations_per_sec)",
            "n_gpus": dist.get_world_size() if dist_on else 1,
            # ranks of the process group that ran the step (0: no group, one process)
            "rccl_world": dist.get_world_size() if backend == "nccl" else 0,
            "dist_backend": backend,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "fp32",
            # the framework GEMMs' arithmetic: square products on gemm_ks.hip (an exact 3-way bf16
            # split with six bf16 MFMA products), the tall 10 000-row products on gemm_blk.hip (per-row
            # scaled f16 pairs, three f16 MFMA products); both f32-accurate (tests/test_gemm_ks.py,
            # tests/test_gemm_blk.py: the 2e-6·Σ|ab| bound)
            "gemm_precision": ({"x6": "bf16x6", "x6w": "bf16x6 32x32", "f32": "f32 MFMA"}.get(config.get("gemm_prec"), config.get("gemm_prec"))
                               + (" square / f16x3 tall" if config.get("gemm_tall") == "h3" else "") + " (f32-accurate)"
                               + {"x3all": "; eigensolver corrections (exp(αX) − I terms, basis update, Newton–Schulz) bf16x3",
                                  "x3late": "; eigensolver exp(αX) − I terms bf16x3, settled solves' basis corrections bf16x3",
                                  "x3": "; eigensolver exp(αX) − I terms bf16x3"}.get(config.get("sbr_corr_prec"), "")),
            "data": f"synthetic (seeded CEC'22 F{args.func} shift + Haar rotation at d={args.dim}; random init mean)",
            "generations_per_sec": round(gens_per_s, 3),
            "config": {
                "model": "CMA-ES on CEC2022 F1 (shifted-rotated Zakharov)" if args.func == 1 else f"CMA-ES on CEC2022 F{args.func}",
                "global_batch": args.pop,
                "seq_len": args.dim,
                "parallelism": f"pop-shard{world}" if not sim else f"simulated-rank{args.simulate_rank}-of-{args.world}",
                "pop_size": args.pop,
                "dim": args.dim,
                "hipgraph": bool(use_graph and not getattr(wf, "_graph_failed", False)),
                "eigh": config.get("eigh") + ("-" + config.get("sbr_mode") if config.get("eigh") == "sbr" else ""),
            },
        }
        if phases:
            out["phases_ms_eager"] = phases
        if args.monitor:
            hist = monitors[0].get_history()
            out["monitor"] = {"type": "EvalMonitor", "mode": args.monitor, "generations_recorded": len(hist),
                              "host_side": bool(hist) and not hist[-1].is_cuda,
                              "best_fitness": float(monitors[0].get_best_fitness())}
        if sim:
            # one rank's share of an N-GPU step (the driver's --gpus 1 headline never sets this)
            out["simulated"] = {
                "rank": args.simulate_rank,
                "world": args.world,
                "rows_per_rank": -(-args.pop // args.world),
                "collectives": "replaced by same-size local ops; wire time modelled below (parallel/wire.py)",
                "wire_model": sim_ctx.wire.describe(),
                **{k: round(v, 4) for k, v in wire.items()},
                "projected_ms_with_wire": round(ms + wire["wire_ms_per_gen"], 4),
            }
            if phases:
                rep = phases.get("eigh", 0.0)
                out["simulated"]["replicated_ms_eager"] = rep
                out["simulated"]["sharded_ms_eager"] = round(phases.get("ask", 0.0) + phases.get("evaluate", 0.0) +
                                                             phases.get("tell", 0.0) - rep, 4)
        if dev_hist.shape[0]:
            # every timed generation's decomposition (device-controlled schedule, read back
            # once after the timed loop): relative off-norm ‖offdiag(BᵀCB)‖/‖diag‖
            out["eigh_stats"] = {
                "generations": int(dev_hist.shape[0]),
                "max_off_rel": float(dev_hist[:, 0].max()),
                "tol": config.get("eigh_tol"),
                "mode": "device",
                "schedule_iters": config.get("sbr_device_iters"),
                "mean_refine_iters": float(dev_hist[:, 2].mean()),
                "max_refine_iters": int(dev_hist[:, 2].max()),
                "fallbacks": int(dev_hist[:, 3].sum()),
                # status bits of each solve (eigh_sbr_dev.hip): 1 capped (not converged),
                # 2 recovered from a divergence, 4 stopped by the lean-slot guard
                "capped": int((dev_hist[:, 1].long() & 1).sum()),
                "recovered": int(((dev_hist[:, 1].long() & 2) != 0).sum()),
                "lean_guard_stops": int(((dev_hist[:, 1].long() & 4) != 0).sum()),
                "schedule_escalations": int(getattr(algo, "schedule_escalations", 0)),
                # eigensolver schedule each timed generation replayed (L late / W warm / C cold),
                # chosen from the measured convergence of the solve two generations back
                "schedule_per_gen": algo.schedule_levels(args.steps) if hasattr(algo, "schedule_levels") else None,
                # refinement iterations of each timed generation, in order
                "iters_per_gen": "".join(str(min(int(v), 9)) if v < 10 else "+" for v in dev_hist[:, 2].tolist()),
            }
        elif hist:
            # every timed generation's decomposition: relative off-norm ‖offdiag(BᵀCB)‖/‖diag‖
            out["eigh_stats"] = {
                "generations": len(hist),
                "max_off_rel": max(h.off_rel for h in hist),
                "tol": config.get("eigh_tol"),
                "mean_jacobi_sweeps": sum(h.jacobi_sweeps for h in hist) / len(hist),
                "mean_refine_iters": sum(h.refine_iters for h in hist) / len(hist),
                "fallbacks": sum(h.fallback for h in hist),
            }
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
