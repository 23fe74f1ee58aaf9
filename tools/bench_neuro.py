"""OpenES + Brax-style Ant throughput (north-star config 4: pop 8192, MLP 27-64-64-8).

python tools/bench_neuro.py [--pop 8192] [--cap 1000] [--gens 5]
torchrun --nproc-per-node N tools/bench_neuro.py ...   (population sharded over N GPUs:
each rank rolls out its slice, OpenES all-reduces the partial gradient over RCCL)
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402


def main():
    from evoxmi import random as rnd
    from evoxmi.algorithms import OpenES
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector, rank_based_fitness
    from evoxmi.workflows import StdWorkflow

    ap = argparse.ArgumentParser()
    ap.add_argument("--pop", type=int, default=8192)
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one per GPU); spawned here unless torchrun started them")
    ap.add_argument("--cap", type=int, default=1000)
    ap.add_argument("--gens", type=int, default=5)
    ap.add_argument("--hidden", type=int, default=64)
    ap.add_argument("--wscale", type=float, default=0.1)
    ap.add_argument("--kernel-only", action="store_true", help="time the fused rollout alone on random policies")
    ap.add_argument("--force-dist", action="store_true", help="distributed path even on one rank")
    ap.add_argument("--graph", action="store_true", help="capture the generation in a hipGraph")
    ap.add_argument("--per-gen", action="store_true", help="print each generation's wall time and episode lengths")
    ap.add_argument("--dump-pop", default=None, help="save the last generation's population (rollout-probe input)")
    args = ap.parse_args()
    if args.kernel_only:
        return kernel_only(args)
    from evoxmi.parallel import init_distributed
    from evoxmi.parallel.launch import LaunchError, ensure_ranks
    import torch.distributed as dist

    try:
        ensure_ranks(args.gpus)
    except LaunchError as e:
        print(f"bench_neuro.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    rank, world, dev = init_distributed(force=args.force_dist)
    if world != args.gpus:
        print(f"bench_neuro.py: --gpus {args.gpus} but the job has {world} rank(s)", file=sys.stderr, flush=True)
        sys.exit(2)
    dist_on = world > 1 or args.force_dist
    policy = MLPPolicy([27, args.hidden, args.hidden, 8])
    params = policy.init(rnd.PRNGKey(0), device=dev)
    tv = TreeAndVector(params)
    algo = OpenES(tv.to_vector(params), args.pop, learning_rate=0.01, noise_stdev=0.05, optimizer="adam")
    prob = Brax(policy, "ant", args.cap)
    wf = StdWorkflow(algo, prob, sol_transforms=[tv.batched_to_tree], fit_transforms=[rank_based_fitness],
                     opt_direction="max", graph=args.graph)
    st = wf.init(rnd.PRNGKey(1, device=dev))
    if dist_on:
        st = wf.enable_distributed(st)

    def sync():
        torch.cuda.synchronize()
        if dist_on:
            dist.barrier()

    st = wf.step(st)
    sync()
    t = time.perf_counter()
    env_steps = torch.zeros((), dtype=torch.int64, device=dev)
    for gi in range(args.gens):
        if args.per_gen:
            sync()
            tg = time.perf_counter()
        st = wf.step(st)
        env_steps += prob.last_episode_lengths.sum()
        if args.per_gen:
            sync()
            L = prob.last_episode_lengths
            if rank == 0:
                print(json.dumps({"gen": gi, "ms": round((time.perf_counter() - tg) * 1e3, 3), "max_len": int(L.max()),
                                  "mean_len": round(float(L.float().mean()), 1)}), flush=True)
    sync()
    dt = torch.tensor([(time.perf_counter() - t) / args.gens], dtype=torch.float64, device=dev)
    if args.dump_pop:
        torch.save(st.get_child_state("algorithm").population.cpu(), args.dump_pop)
        # the last population's rollout timed in this process: workflow init state vs the probe's
        from evoxmi.ops import neuro
        from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

        Wf = policy.flat(tv.batched_to_tree(st.get_child_state("algorithm").population))
        s_wf = prob._initial_state(st.get_child_state("problem").key, Wf.device)
        s_pr = get_environment("ant").reset(rnd.PRNGKey(0), 1)[0][0].to(Wf.device)
        print("init states equal:", bool(torch.equal(s_wf, s_pr)), flush=True)
        for name, s0 in (("workflow_init", s_wf), ("probe_init", s_pr)):
            for _ in range(2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                _, L = neuro.ant_rollout(Wf, args.hidden, args.hidden, s0, args.cap)
                e1.record()
                torch.cuda.synchronize()
                print(name, round(e0.elapsed_time(e1), 3), "ms mean_len", round(float(L.float().mean()), 1), flush=True)
    if dist_on:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        dist.all_reduce(env_steps)
    dt, env_steps = float(dt), int(env_steps)
    out = {"pop": args.pop, "n_gpus": dist.get_world_size() if dist.is_initialized() else 1, "cap_episode": args.cap, "params": policy.num_params, "ms_per_gen": round(dt * 1e3, 2),
           "gens_per_sec": round(1 / dt, 3), "env_steps_per_sec": round(env_steps / args.gens / dt, 1),
           "mean_episode_len": round(env_steps / args.gens / args.pop, 1), "graph": args.graph}
    if rank == 0:
        print(json.dumps(out))
    if dist_on:
        dist.destroy_process_group()


def kernel_only(args):
    """Rollout throughput without the ES loop: random-init policies (+ a large
    perturbation so some survive long), counted in env steps actually simulated."""
    from evoxmi import random as rnd
    from evoxmi.ops import neuro
    from evoxmi.problems.neuroevolution.reinforcement_learning.envs import get_environment

    h = args.hidden
    P = neuro.ant_param_count(h, h)
    g = torch.Generator(device="cuda").manual_seed(0)
    W = args.wscale * torch.randn(args.pop, P, device="cuda", generator=g)
    s0, _ = get_environment("ant").reset(rnd.PRNGKey(0), 1)
    init = s0[0].cuda()
    neuro.ant_rollout(W, h, h, init, args.cap)
    torch.cuda.synchronize()
    t = time.perf_counter()
    steps = 0
    for _ in range(args.gens):
        _, st = neuro.ant_rollout(W, h, h, init, args.cap)
        steps += st.sum()
    torch.cuda.synchronize()
    max_len = int(st.max())
    dt = (time.perf_counter() - t) / args.gens
    steps = int(steps) / args.gens
    print(json.dumps({"mode": "kernel_only", "pop": args.pop, "hidden": h, "cap": args.cap, "ms_per_rollout": round(dt * 1e3, 3),
                      "mean_episode_len": round(steps / args.pop, 1), "max_episode_len": max_len,
                      "us_per_step_of_longest": round(dt * 1e6 / max(max_len, 1), 3), "env_steps_per_sec": round(steps / dt, 1)}))


if __name__ == "__main__":
    main()
