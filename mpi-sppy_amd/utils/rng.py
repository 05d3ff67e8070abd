"""Many scenarios' ``numpy.random.RandomState(seed).rand()`` streams at once.

The reference's scenario creators seed one legacy RandomState per scenario
(``farmer.py:159-183``: ``RandomState(scennum + seedoffset)`` then ``rand()``
per crop).  Constructing and seeding a RandomState costs ~0.1 ms, which is
most of building a million-scenario batch.  This module reproduces the first
few ``rand()`` draws of many seeds with vectorised integer arithmetic over the
seeds, bit for bit:

* legacy seeding (numpy ``mt19937_seed``): key[0] = seed,
  key[i] = 1812433253 * (key[i-1] ^ (key[i-1] >> 30)) + i  (mod 2**32);
* the first twist of MT19937 for the output words needed (new key[i] depends on
  key[i], key[i+1] and key[i+397]), then the standard tempering;
* ``rand()`` = (a >> 5) * 2**26 + (b >> 6), scaled by 2**-53, from two words.

Only ``rand()`` is reproduced; draws of other distributions (``normal()``)
fall back to RandomState in the callers.
"""
import numpy as np

_N, _M = 624, 397
_CHUNK = 32768          # seeds per pass (the key rows of a chunk stay in cache)


def _temper(y):
    y = y ^ (y >> np.uint32(11))
    y = y ^ ((y << np.uint32(7)) & np.uint32(0x9D2C5680))
    y = y ^ ((y << np.uint32(15)) & np.uint32(0xEFC60000))
    return y ^ (y >> np.uint32(18))


def _words_chunk(v, k, out):
    need = _M + k                                  # key[0 .. M + k - 1]
    key = np.empty((need, v.size), dtype=np.uint32)
    mult = np.uint32(1812433253)
    with np.errstate(over="ignore"):               # uint32 arithmetic wraps mod 2**32, as in C
        for pos in range(need):
            key[pos] = v
            v = mult * (v ^ (v >> np.uint32(30))) + np.uint32(pos + 1)
    one = np.uint32(1)
    upper, lower, mat = np.uint32(0x80000000), np.uint32(0x7FFFFFFF), np.uint32(0x9908B0DF)
    for i in range(k):
        y = (key[i] & upper) | (key[i + 1] & lower)
        w = key[i + _M] ^ (y >> one) ^ ((np.uint32(0) - (y & one)) & mat)
        out[:, i] = _temper(w)


def first_words(seeds, k):
    """(len(seeds), k) uint32: the first k 32-bit outputs of RandomState(seed)
    for each seed (k <= 227: all come from the first half of the first twist)."""
    if not 0 < k <= _N - _M:
        raise ValueError("first_words: 1 <= k <= %d" % (_N - _M))
    s = np.asarray(seeds, dtype=np.int64).ravel()
    if s.size and (s.min() < 0 or s.max() > 0xFFFFFFFF):
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    out = np.empty((s.size, k), dtype=np.uint32)
    for a in range(0, s.size, _CHUNK):
        _words_chunk(s[a:a + _CHUNK].astype(np.uint32), k, out[a:a + _CHUNK])
    return out


def first_rands(seeds, k):
    """(len(seeds), k) float64: the first k ``RandomState(seed).rand()`` draws."""
    w = first_words(seeds, 2 * k)
    a = (w[:, 0::2] >> np.uint32(5)).astype(np.float64)
    b = (w[:, 1::2] >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0
