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
  key[i], key[i+1] and key[i+397]), then the standard tempering; past the first
  227 words (key[i+397] wraps onto words the same twist already replaced) and
  past 624 words (further twists) the whole 624-word state is carried;
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


def _words_chunk_full(v, k, out):
    """Any k: the full MT19937 state, twisted in place (numpy's mt19937_gen
    order: words 0..226 from the old state, 227..622 from words this twist
    already replaced, 623 from the new word 0), as many twists as k needs."""
    key = np.empty((_N, v.size), dtype=np.uint32)
    mult = np.uint32(1812433253)
    with np.errstate(over="ignore"):
        for pos in range(_N):
            key[pos] = v
            v = mult * (v ^ (v >> np.uint32(30))) + np.uint32(pos + 1)
    one = np.uint32(1)
    upper, lower, mat = np.uint32(0x80000000), np.uint32(0x7FFFFFFF), np.uint32(0x9908B0DF)
    done = 0
    while done < k:
        for i in range(_N):
            y = (key[i] & upper) | (key[(i + 1) % _N] & lower)
            key[i] = key[(i + _M) % _N] ^ (y >> one) ^ ((np.uint32(0) - (y & one)) & mat)
        take = min(_N, k - done)
        out[:, done:done + take] = _temper(key[:take]).T
        done += take


def first_words(seeds, k):
    """(len(seeds), k) uint32: the first k 32-bit outputs of RandomState(seed)
    for each seed (k <= 227: all from the first half of the first twist, the
    short path; larger k: the full state, _words_chunk_full)."""
    if k < 1:
        raise ValueError("first_words: k >= 1")
    s = np.asarray(seeds, dtype=np.int64).ravel()
    if s.size and (s.min() < 0 or s.max() > 0xFFFFFFFF):
        raise ValueError("Seed must be between 0 and 2**32 - 1")
    out = np.empty((s.size, k), dtype=np.uint32)
    fill = _words_chunk if k <= _N - _M else _words_chunk_full
    for a in range(0, s.size, _CHUNK):
        fill(s[a:a + _CHUNK].astype(np.uint32), k, out[a:a + _CHUNK])
    return out


def first_rands(seeds, k):
    """(len(seeds), k) float64: the first k ``RandomState(seed).rand()`` draws."""
    w = first_words(seeds, 2 * k)
    a = (w[:, 0::2] >> np.uint32(5)).astype(np.float64)
    b = (w[:, 1::2] >> np.uint32(6)).astype(np.float64)
    return (a * 67108864.0 + b) / 9007199254740992.0
