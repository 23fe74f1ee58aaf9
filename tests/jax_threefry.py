"""numpy re-implementation of JAX's classic threefry2x32 PRNG (``jax.random.PRNGKey``,
``split``, ``uniform``) — only used to regenerate the random inputs the reference's
golden tests were computed on (``tests/test_lsmop.py``, ``tests/test_maf.py``).  No JAX
is available here; this follows the published Threefry-2x32 (20 rounds) algorithm and
JAX's original (non-partitionable) bit layout: counts = iota(n) split into halves.
"""
import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def _rotl(x, r):
    return ((x << np.uint64(r)) | (x >> np.uint64(32 - r))) & M32


def threefry2x32(key, x0, x1):
    k0, k1 = np.uint64(key[0]), np.uint64(key[1])
    k2 = k0 ^ k1 ^ np.uint64(0x1BD11BDA)
    ks = [k0, k1, k2]
    x0 = (x0.astype(np.uint64) + ks[0]) & M32
    x1 = (x1.astype(np.uint64) + ks[1]) & M32
    rot = [[13, 15, 26, 6], [17, 29, 16, 24]]
    for i in range(5):
        for r in rot[i % 2]:
            x0 = (x0 + x1) & M32
            x1 = _rotl(x1, r)
            x1 = x1 ^ x0
        x0 = (x0 + ks[(i + 1) % 3]) & M32
        x1 = (x1 + ks[(i + 2) % 3] + np.uint64(i + 1)) & M32
    return x0.astype(np.uint32), x1.astype(np.uint32)


def PRNGKey(seed):
    seed = int(seed)
    return np.array([(seed >> 32) & 0xFFFFFFFF, seed & 0xFFFFFFFF], dtype=np.uint32)


def random_bits(key, n):
    count = np.arange(n, dtype=np.uint32)
    odd = n % 2
    if odd:
        count = np.concatenate([count, np.zeros(1, np.uint32)])
    half = count.shape[0] // 2
    a, b = threefry2x32(key, count[:half], count[half:])
    return np.concatenate([a, b])[:n]


def split(key, num=2):
    bits = random_bits(key, 2 * num)
    return bits.reshape(num, 2)


def uniform(key, shape, minval=0.0, maxval=1.0):
    n = int(np.prod(shape))
    bits = random_bits(key, n)
    f = ((bits >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)
    f = f.reshape(shape)
    minval = np.asarray(minval, np.float32)
    maxval = np.asarray(maxval, np.float32)
    return np.maximum(minval, f * (maxval - minval) + minval).astype(np.float32)


def normal(key, shape):
    """jax.random.normal: √2·erfinv(U(nextafter(−1, 0), 1)) in float32."""
    from scipy.special import erfinv

    lo = np.nextafter(np.float32(-1.0), np.float32(0.0))
    u = uniform(key, shape, lo, np.float32(1.0))
    return (np.sqrt(np.float32(2.0)) * erfinv(u.astype(np.float64))).astype(np.float32)
