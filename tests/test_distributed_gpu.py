"""Multi-process SPMD paths with the HIP kernels in the loop (MI355X, marked gpu).

The pool's boxes have one GPU, and RCCL refuses two ranks on one device, so these
tests run 2 ranks on ``cuda:0`` with the gloo backend (gloo stages CUDA tensors through
the host).  They exercise exactly the sharded code that the 8-GPU RCCL runs use —
rank-local Philox rows, the fused kernels, the all-gathers / all-reduces — and compare
with the single-process result.  The RCCL collectives themselves, captured in the
hipGraph, are covered by ``bench.py --force-dist`` under torchrun on one GPU.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _make(kind):
    from evoxmi.algorithms import CMAES, OpenES
    from evoxmi.problems.numerical import CEC2022TestSuit, Sphere
    from evoxmi.workflows import StdWorkflow

    if kind == "cmaes":
        d = 64
        alg = CMAES(torch.linspace(-3, 3, d, device="cuda"), init_stdev=2.0, pop_size=512)
        return StdWorkflow(alg, CEC2022TestSuit.create(1))
    alg = OpenES(torch.full((40,), 1.0, device="cuda"), 256, learning_rate=0.05, noise_stdev=0.2, optimizer="adam")
    return StdWorkflow(alg, Sphere())


def _field(kind):
    return "mean" if kind == "cmaes" else "center"


def _worker(rank, world, port, kind, gens, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK="0")
    from evoxmi import random as rnd
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    torch.cuda.set_device(0)
    wf = _make(kind)
    st = wf.init(rnd.PRNGKey(3, device="cuda"))
    st = wf.enable_distributed(st)
    for _ in range(gens):
        st = wf.step(st)
    torch.cuda.synchronize()
    out[rank] = st.get_child_state("algorithm")[_field(kind)].cpu()
    destroy()


# CMA-ES: one generation (afterwards the Jacobi eigenbasis of the clustered spectrum
# amplifies rounding-level differences of the all-reduced statistics into different
# — equally valid — sample rotations, so longer runs are compared replica-to-replica only)
@pytest.mark.parametrize("kind,gens", [("cmaes", 1), ("cmaes", 5), ("openes", 8)])
def test_sharded_two_ranks_on_gpu_match_single_process(kind, gens):
    from evoxmi import random as rnd

    wf = _make(kind)
    st = wf.init(rnd.PRNGKey(3, device="cuda"))
    for _ in range(gens):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")[_field(kind)].cpu()
    mgr = mp.get_context("spawn").Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), kind, gens, out), nprocs=2, join=True)
    assert torch.equal(out[0], out[1])  # replicas stay bit-identical
    if kind == "cmaes" and gens > 1:
        return
    # reduction order differs from the single process (rank partial sums + all-reduce)
    assert torch.allclose(out[0], ref, rtol=1e-3, atol=1e-3)
