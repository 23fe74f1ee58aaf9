"""The block pairing the Jacobi kernels compute in registers (``round_blk``,
csrc/kernels/eigh_jacobi.hip) must equal the host schedule table row by row: the
fused apply+solve path still reads the table, and the GPU bit-identity test
(test_jacobi_fused_apply_solve_is_bit_identical) relies on both giving the same rounds."""
import pytest

from evoxmi.ops import jacobi


@pytest.mark.parametrize("nb", [2, 4, 8, 14, 64, 256])
def test_closed_form_pairing_matches_table(nb):
    tab = jacobi._schedule_cpu(nb).tolist()
    for t in range(nb):
        assert jacobi.round_pairing(t, nb) == tab[t]


@pytest.mark.parametrize("nb", [4, 16, 64])
def test_each_sweep_pairs_every_block_pair_once(nb):
    seen = set()
    for t in range(1, nb):
        row = jacobi.round_pairing(t, nb)
        assert sorted(row) == list(range(nb))  # a perfect matching per round
        seen |= {tuple(sorted(row[2 * p: 2 * p + 2])) for p in range(nb // 2)}
    assert len(seen) == nb * (nb - 1) // 2
