"""CPU check of the identity the round-6 selection kernels rely on
(csrc/lfm_entropy.hip: ent_next / ent_link / ent_rows): the bigram histogram of
bwt_GPU's stably key-sorted pair array L (klb_imageIO.cpp:2030-2093,
lfm_Predictors.cu:2883-2914, restated by oracle/lfm_oracle.c
lfmo_entropy_chunk) equals the histogram of (c[i-1], partner[i]) over the
positions, where partner[i] is the val of the next occurrence of byte c[i],
the last occurrence of a byte takes the first val of the next non-empty byte
(byte 0's the sentinel's val c[S-1], the sentinel the first val of the next
non-empty byte >= 1), and the last element of L has no bigram.  The model
below is written from that rule alone, position by position, and compared
with the sort definition on skewed, one-byte, absent-byte and random chunks."""
import numpy as np
import pytest


def hist_by_sort(c):
    """h[(L[j] << 8) | L[j+1]], j < S, with L the stable key sort of (c[i],
    c[i-1]) plus the sentinel (0, c[S-1]) (the oracle's definition)."""
    keys = np.concatenate([c, [0]])
    vals = np.concatenate([[0], c[:-1], [c[-1]]])
    L = vals[np.argsort(keys, kind="stable")]
    return np.bincount((L[:-1] << 8) | L[1:], minlength=65536)


def hist_by_partner(c):
    S = len(c)
    val = np.concatenate([[0], c[:-1]])
    partner = np.full(S, -1, np.int64)
    first = {}  # first val of each byte among the positions after i
    for i in range(S - 1, -1, -1):
        partner[i] = first.get(int(c[i]), -1)
        first[int(c[i])] = int(val[i])
    last = {int(b): int(i) for i, b in enumerate(c)}  # last occurrence of each byte
    nxt, nf = {}, -1  # first val of the next non-empty byte above k
    for k in range(255, -1, -1):
        nxt[k] = nf
        if k in first:
            nf = first[k]
    skip = -1
    for k, i in last.items():
        p = int(c[-1]) if k == 0 else nxt[k]
        if p < 0:
            skip = i  # the end of L: no bigram
        else:
            partner[i] = p
    keep = np.arange(S) != skip
    h = np.bincount((val[keep] << 8) | partner[keep], minlength=65536)
    if nxt[0] >= 0:  # the sentinel's bigram
        h[(int(c[-1]) << 8) | nxt[0]] += 1
    return h


@pytest.mark.parametrize("kind", ["skewed", "uniform", "two_bytes", "zeros", "no_zero", "runs"])
def test_partner_histogram_equals_sorted_pairs(kind):
    rng = np.random.default_rng(sum(map(ord, kind)))  # (fixed per case)
    for S in (1, 2, 3, 17, 64, 65, 200, 999):
        if kind == "skewed":
            c = np.minimum(np.abs(rng.normal(0, 6, S)).astype(np.int64), 255)
        elif kind == "uniform":
            c = rng.integers(0, 256, S)
        elif kind == "two_bytes":
            c = rng.choice([7, 200], S)
        elif kind == "zeros":
            c = np.zeros(S, np.int64)
        elif kind == "no_zero":
            c = rng.integers(1, 4, S)
        else:
            c = np.repeat(rng.integers(0, 5, S // 8 + 1), 8)[:S]
        c = c.astype(np.int64)
        assert np.array_equal(hist_by_sort(c), hist_by_partner(c)), (kind, S)
