"""Neighbourhood topologies for PSO (reference ``pso_variants/topology_utils.py:15-251``).

Adjacency matrices (N×N, 1 = neighbour, self-loops included) and the padded
adjacency-list form used by FIPS / SwmmPSO.  ``get_square_neighbour`` builds the von
Neumann grid with wrap-around; the reference indexes the column with the row
counter (``:98``) and prints the matrices — here the grid is correct and silent.
"""
from __future__ import annotations

import math

import torch

from ....ops import random as rnd
from .utils import get_distance_matrix, row_argsort, select_from_mask


def get_full_neighbour(population):
    N = population.shape[0]
    return torch.ones((N, N), dtype=torch.int32, device=population.device)


def get_ring_neighbour(population, K: int):
    N = population.shape[0]
    i = torch.arange(N, device=population.device)
    d = (i[:, None] - i[None, :]).abs()
    d = torch.minimum(d, N - d)
    return (d <= K).to(torch.int32)


def get_square_neighbour(population):
    N = population.shape[0]
    col = math.floor(math.sqrt(N))
    while col > 1 and N % col != 0:
        col -= 1
    row = N // col
    grid = torch.arange(N).reshape(col, row)
    adj = torch.zeros((N, N), dtype=torch.int32)
    for i in range(col):
        for j in range(row):
            x = grid[i, j]
            for di, dj in ((0, 1), (1, 0), (0, -1), (-1, 0)):
                adj[x, grid[(i + di) % col, (j + dj) % row]] = 1
    return adj.to(population.device)


def build_adjacancy_matrix_by_K_nearest_neighbour(distance_ranking, K: int):
    N = distance_ranking.shape[0]
    idx = distance_ranking[:, : K + 1]
    A = torch.zeros((N, N), dtype=torch.int32, device=distance_ranking.device)
    rows = torch.arange(N, device=A.device)[:, None].expand(N, K + 1)
    A[rows.reshape(-1), idx.reshape(-1)] = 1
    A[idx.reshape(-1), rows.reshape(-1)] = 1
    return A


def mutate_shortcut(key, adjacancy_matrix, num_shortcut: int):
    """Rewire ``num_shortcut`` random edges: one endpoint of each moves to a random node."""
    N = adjacancy_matrix.shape[0]
    if num_shortcut <= 0:
        return adjacancy_matrix
    k1, k2, k3 = rnd.split(key, 3)
    dev = adjacancy_matrix.device
    eye = torch.eye(N, dtype=adjacancy_matrix.dtype, device=dev)
    flat = torch.triu(adjacancy_matrix - eye).reshape(-1)
    rows = torch.arange(N, device=dev).repeat_interleave(N)
    cols = torch.arange(N, device=dev).repeat(N)
    mask = select_from_mask(k1, flat, num_shortcut).bool()
    mrow = rnd.randint(k2, (N * N,), 0, 2).to(dev).bool()
    nodes = rnd.randint(k3, (N * N,), 0, N).to(dev)
    rows = torch.where(mask & mrow, nodes, rows)
    cols = torch.where(mask & ~mrow, nodes, cols)
    out = torch.zeros(N * N, dtype=adjacancy_matrix.dtype, device=dev).index_add_(0, rows * N + cols, flat).reshape(N, N)
    return torch.clamp(out + out.T + eye, 0, 1)


def get_circles_neighbour(random_key, population, K: int, shortcut: int):
    adj = build_adjacancy_matrix_by_K_nearest_neighbour(row_argsort(get_distance_matrix(population)), K)
    return mutate_shortcut(random_key, adj, shortcut)


def build_adjacancy_list_from_matrix(adjacancy_matrix, keep_self_loop=True):
    """Padded neighbour lists (N, N): row i holds its neighbours first (ascending), the
    padding repeats i; the mask marks real entries (reference ``:143-171``)."""
    N = adjacancy_matrix.shape[0]
    dev = adjacancy_matrix.device
    nz = adjacancy_matrix != 0
    key = (~nz).to(torch.int64) * N + torch.arange(N, device=dev)[None, :]
    lst = torch.argsort(key, dim=1)
    valid = torch.gather(nz, 1, lst)
    ident = torch.arange(N, device=dev)[:, None].expand(N, N)
    mask = valid.to(adjacancy_matrix.dtype)
    if not keep_self_loop:
        mask = torch.where(lst == ident, torch.zeros_like(mask), mask)
    return torch.where(valid, lst, ident).to(torch.int64), mask


def get_neighbour_best_fitness(fitness, adjacancy_list):
    f = fitness[adjacancy_list]
    j = torch.argmin(f, dim=1)
    idx = adjacancy_list.gather(1, j[:, None])[:, 0]
    return fitness[idx], idx
