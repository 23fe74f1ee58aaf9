"""Philox4x32-10 key API: bit-exactness against an independent numpy uint64
implementation, distribution sanity, and key algebra."""
import numpy as np
import pytest
import torch

from evoxmi import random as rnd


def np_philox(ctr, key, rounds=10):
    M0, M1, W0, W1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57), 0x9E3779B9, 0xBB67AE85
    c = [np.uint64(x) for x in ctr]
    k0, k1 = key
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(rounds):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        c = [(p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0), p1 & mask, (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1), p0 & mask]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return [int(x) for x in c]


def test_philox_matches_numpy_reference():
    key = rnd.PRNGKey(0x1234567890AB)
    k = [int(x) for x in key.tolist()]
    w = rnd.bits(key, (40,)).tolist()
    for b in range(10):
        ref = np_philox([b, 0, 0, 0], k)
        assert w[4 * b : 4 * b + 4] == ref


def test_known_answer_vector():
    # Random123 known-answer test for philox4x32-10 with zero counter and key
    ref = np_philox([0, 0, 0, 0], [0, 0])
    assert ref == [0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8]


def test_split_fold_distinct():
    key = rnd.PRNGKey(42)
    ks = rnd.split(key, 8)
    assert ks.shape == (8, 2)
    assert len({tuple(k.tolist()) for k in ks}) == 8
    assert not torch.equal(rnd.fold_in(key, 1), rnd.fold_in(key, 2))


def test_distributions():
    key = rnd.PRNGKey(7)
    u = rnd.uniform(key, (100000,))
    assert 0 < u.min() and u.max() < 1 and abs(u.mean().item() - 0.5) < 0.01
    z = rnd.normal(key, (100000,))
    assert abs(z.mean().item()) < 0.02 and abs(z.std().item() - 1) < 0.02
    r = rnd.randint(key, (10000,), 3, 9)
    assert r.min() == 3 and r.max() == 8
    p = rnd.permutation(key, 50)
    assert sorted(p.tolist()) == list(range(50))
    c = rnd.choice(key, 10, (5,), replace=False)
    assert len(set(c.tolist())) == 5


def test_offset_sharding_consistency():
    key = rnd.PRNGKey(3)
    full = rnd.normal(key, (8, 6))
    part = rnd.normal(key, (4, 6), offset=4 * 6)
    assert torch.allclose(full[4:], part)


@pytest.mark.gpu
def test_gpu_philox_bit_exact():
    key = rnd.PRNGKey(99)
    cpu = rnd.uniform(key, (10000,))
    gpu = rnd.uniform(key.cuda(), (10000,)).cpu()
    assert torch.equal(cpu, gpu)
    zc = rnd.normal(key, (4096 * 3,))
    zg = rnd.normal(key.cuda(), (4096 * 3,)).cpu()
    assert torch.allclose(zc, zg, atol=1e-5, rtol=1e-5)
    part = rnd.normal(key.cuda(), (4096,), offset=4096).cpu()
    assert torch.allclose(zc[4096:8192], part, atol=1e-5, rtol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize("num", [1, 2, 5, 300])
def test_split_on_the_device_matches_the_host(num):
    """rnd.split on a GPU key writes the (num, 2) keys from one launch (philox_words, 2 words
    per block): bitwise the host keys; fold_in and the bits of a split key agree too."""
    for seed in (0, 7, 2**40 + 3):
        kc = rnd.PRNGKey(seed)
        kg = kc.cuda()
        sc, sg = rnd.split(kc, num), rnd.split(kg, num)
        assert sg.shape == (num, 2) and sg.is_contiguous()
        assert torch.equal(sc, sg.cpu())
        assert torch.equal(rnd.bits(sc[-1], (37,)), rnd.bits(sg[-1], (37,)).cpu())
