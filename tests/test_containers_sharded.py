"""Cooperative co-evolution mapped onto ranks: 2 gloo ranks, each owning
half of the sub-populations, reproduce the single-process VectorizedCoevolution run bit
for bit (CPU)."""
import os
import socket

import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make():
    from evoxmi.algorithms import CSO, VectorizedCoevolution
    from evoxmi.problems.numerical import Ackley
    from evoxmi.workflows import StdWorkflow

    subs = [CSO(lb=torch.full((10,), -32.0), ub=torch.full((10,), 32.0), pop_size=20) for _ in range(4)]
    return StdWorkflow(VectorizedCoevolution(subs, dim=40, num_subpops=4, random_subpop=True), Ackley())


def _run(wf, gens, dist=False):
    from evoxmi import random as rnd

    st = wf.init(rnd.PRNGKey(11))
    if dist:
        st = wf.enable_distributed(st)
    for _ in range(gens):
        st = wf.step(st)
    a = st.get_child_state("algorithm")
    return a.best_dec.clone(), a.best_fit.clone()


def _worker(rank, world, port, gens, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    out[rank] = _run(_make(), gens, dist=True)
    destroy()


def test_vectorized_coevolution_two_ranks_bit_identical():
    gens = 12
    ref_dec, ref_fit = _run(_make(), gens)
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), gens, out), nprocs=2, join=True)
    for r in range(2):
        dec, fit = out[r]
        assert torch.equal(dec, ref_dec) and torch.equal(fit, ref_fit), f"rank {r} differs from the single process"
    assert float(ref_fit.min()) < float(ref_fit.max()) + 1  # sanity: finite
