"""Multi-objective north-star throughput (BASELINE.json configs 3 and 5).

  nsga2 : NSGA-II pop=4096 on DTLZ2 (m=3, d=500)           — 1×MI355X
  moead : MOEA/D pop=16384 on LSMOP1 (m=3, d=10000), Tchebycheff aggregation

python tools/bench_mo.py --algo nsga2|moead [--gens 20] [--warmup 3] [--no-graph]
torchrun --nproc-per-node 8 --master-addr 127.0.0.1 tools/bench_mo.py --algo moead

Prints one JSON line (rank 0): generations/s and evaluations/s of full generations
(ask → evaluate → tell), random-init populations, fp32.  Under torchrun (or with
--force-dist) the workflow is population-sharded: MOEA/D ranks own contiguous slot
ranges, generate/evaluate only their offspring, all-gather the (N, m) objectives; in the
owner-computes mode (default) each rank keeps only its halo current and reads the halo's
winning rows from their generating rank over xGMI (IPC peer buffers), in the replica
mode it regenerates every winner locally.  The line reports the halo fractions at
2/4/8 ranks and the cross-shard winner fraction.  ``--simulate-rank R --world N`` times
rank R's share of an N-GPU step on one GPU (collectives → same-size local operations).
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def build(args, dev):
    from evoxmi.algorithms import MOEAD, NSGA2
    from evoxmi.problems.numerical import DTLZ2, LSMOP1

    m = 3
    if args.algo == "nsga2":
        d = args.dim or 500
        lb, ub = torch.zeros(d, device=dev), torch.ones(d, device=dev)
        return NSGA2(lb, ub, m, args.pop or 4096), DTLZ2(d=d, m=m)
    d = args.dim or 10000
    lb = torch.zeros(d, device=dev)
    ub = torch.cat([torch.ones(m - 1, device=dev), 10 * torch.ones(d - m + 1, device=dev)])
    return MOEAD(lb, ub, m, args.pop or 16384, func_name="tchebycheff"), LSMOP1(d=d, m=m)


def main():
    from evoxmi import random as rnd
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--algo", choices=["nsga2", "moead"], default="nsga2")
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); spawned here unless torchrun started them")
    ap.add_argument("--pop", type=int, default=0)
    ap.add_argument("--dim", type=int, default=0)
    ap.add_argument("--gens", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true")
    ap.add_argument("--force-dist", action="store_true", help="sharded protocol even on one rank")
    ap.add_argument("--simulate-rank", type=int, default=None,  # -1 (MOEA/D): the rank with the largest halo
                    help="time rank R's share of a --world N sharded step on this one GPU (collectives → same-size local ops)")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--shard", choices=["auto", "owner", "replica"], default="auto", help="MOEA/D sharded mode")
    ap.add_argument("--link-gbps", type=float, default=None, help="--simulate-rank wire model: GB/s per xGMI link and direction")
    args = ap.parse_args()
    import torch.distributed as dist
    from evoxmi.parallel import init_distributed
    from evoxmi.parallel.launch import LaunchError, ensure_ranks

    if args.simulate_rank is None:
        try:
            ensure_ranks(args.gpus, device="cpu" if args.cpu else "cuda")
        except LaunchError as e:
            print(f"bench_mo.py: {e}", file=sys.stderr, flush=True)
            sys.exit(2)

    sim = args.simulate_rank is not None
    if sim:
        rank, world, dev = 0, 1, torch.device("cpu" if args.cpu else "cuda")
    else:
        rank, world, dev = init_distributed(force=args.force_dist, backend="gloo" if args.cpu else None)
        if world != args.gpus:
            print(f"bench_mo.py: --gpus {args.gpus} but the job has {world} rank(s)", file=sys.stderr, flush=True)
            sys.exit(2)
    if args.cpu:
        dev = torch.device("cpu")
    algo, prob = build(args, dev)
    if hasattr(algo, "shard"):
        algo.shard = args.shard
    dist_on = (world > 1 or args.force_dist) and not sim

    def sync():
        if dev.type == "cuda":
            torch.cuda.synchronize()
        if dist_on:
            dist.barrier()

    wf = StdWorkflow(algo, prob, graph=not (args.no_graph or args.cpu))
    st = wf.init(rnd.PRNGKey(7, device=dev))
    if dist_on:
        st = wf.enable_distributed(st)
    if sim:
        from evoxmi.parallel.context import SimulatedDistContext

        if args.simulate_rank < 0 and args.algo == "moead":
            # the rank with the largest owner-computes halo: the one that sets the step time
            a0 = st.get_child_state("algorithm")
            fr = [algo.halo_fraction(a0, r, args.world) for r in range(args.world)]
            args.simulate_rank = max(range(args.world), key=lambda r: fr[r])
        args.simulate_rank = max(args.simulate_rank, 0)
        sim_ctx = SimulatedDistContext(args.simulate_rank, args.world, algorithm=algo)
        if args.link_gbps:
            sim_ctx.wire.link_gbps = args.link_gbps
        st = wf.enable_distributed(st, context=sim_ctx)
    for _ in range(1 + args.warmup):
        st = wf.step(st)
    sync()
    if sim:
        sim_ctx.counters.reset()
    t = time.perf_counter()
    for _ in range(args.gens):
        st = wf.step(st)
    sync()
    dt = torch.tensor([(time.perf_counter() - t) / args.gens], dtype=torch.float64, device=dev)
    if dist_on:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt)
    a = st.get_child_state("algorithm")
    fit = a.fitness
    pop = algo.pop_size
    out = {
        "config": args.algo, "pop": pop, "dim": algo.dim, "n_objs": 3, "graph": not (args.no_graph or args.cpu), "n_gpus": dist.get_world_size() if dist.is_initialized() else 1,
        "parallelism": (f"simulated-rank{args.simulate_rank}-of-{args.world}" if sim else (f"pop-shard{world}" if dist_on else "single")),
        "ms_per_gen": round(dt * 1e3, 3), "gens_per_sec": round(1 / dt, 2), "evals_per_sec": round(pop / dt, 1),
        "fitness_finite": bool(torch.isfinite(fit).all()), "mean_obj": [round(float(v), 4) for v in fit.mean(0)],
    }
    if sim:
        w = sim_ctx.counters.summary(args.gens, sim_ctx.wire, args.world, graph=not (args.no_graph or args.cpu))
        out["wire_model"] = sim_ctx.wire.describe()
        out.update({k: round(v, 4) for k, v in w.items()})
        out["projected_ms_with_wire"] = round(dt * 1e3 + w["wire_ms_per_gen"], 4)
    if args.algo == "moead":
        from evoxmi.algorithms.mo.moead import cross_shard_winner_fraction

        frac, cross = cross_shard_winner_fraction(a.win, max(world, 2) if not dist_on else world)
        out["winner_fraction"] = round(frac, 4)
        out["cross_shard_winner_fraction"] = round(cross, 4)
        out["cross_shard_fraction_world"] = world if dist_on else 2
        # owner-computes: the share of the population each rank keeps current (its halo)
        for w in (2, 4, 8):
            fr = [algo.halo_fraction(a, r, w) for r in range(w)]
            out[f"halo_fraction_world{w}"] = {"mean": round(sum(fr) / w, 4), "max": round(max(fr), 4)}
        if wf._dist is not None:
            out["shard_mode"] = "owner" if algo._owner_mode(a, wf._dist) else "replica"
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
