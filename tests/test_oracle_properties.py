"""Size-independent properties of the oracle (tests/ infrastructure), drawn by
hypothesis: the code is linear over GF(2) (parity of a XOR b = parity of a XOR
parity of b), systematic (data shards untouched), and any k present shards of a
codeword rebuild the rest (the crate's reconstruct rule, first k present in
index order, reference src/vfs/block.rs:556-565).  The C and numpy
restatements agree on every drawn case.  The GPU parity suites check the HIP
path against this oracle; these properties check the oracle itself beyond the
published vectors it is pinned to.
"""
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

from oracle import c_oracle
from oracle import rs_oracle as O

codes = st.tuples(st.integers(1, 12), st.integers(1, 6))
lengths = st.integers(1, 300)


def _encode(k, p, data):
    sh = [d.copy() for d in data] + [np.zeros(len(data[0]), np.uint8) for _ in range(p)]
    c_oracle.encode(k, p, sh)
    return sh


@settings(max_examples=60, deadline=None)
@given(codes, lengths, st.integers(0, 2**32 - 1))
def test_linear_and_systematic(kp, L, seed):
    k, p = kp
    rng = np.random.default_rng(seed)
    a = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    b = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    ea, eb = _encode(k, p, a), _encode(k, p, b)
    eab = _encode(k, p, [x ^ y for x, y in zip(a, b)])
    for i in range(k):
        assert np.array_equal(ea[i], a[i])                       # systematic
    for r in range(k, k + p):
        assert np.array_equal(eab[r], ea[r] ^ eb[r])            # linear over GF(2)


@settings(max_examples=60, deadline=None)
@given(codes, lengths, st.integers(0, 2**32 - 1), st.data())
def test_any_k_present_rebuild_the_codeword(kp, L, seed, data):
    k, p = kp
    rng = np.random.default_rng(seed)
    cw = _encode(k, p, [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)])
    t = k + p
    lost = data.draw(st.sets(st.integers(0, t - 1), min_size=0, max_size=p))
    shards = [None if i in lost else cw[i].copy() for i in range(t)]
    out = c_oracle.reconstruct(k, p, shards, L)
    for i in range(t):
        assert np.array_equal(out[i], cw[i]), (k, p, sorted(lost), i)


@settings(max_examples=40, deadline=None)
@given(codes, st.integers(1, 64), st.integers(0, 2**32 - 1))
def test_numpy_and_c_restatements_agree(kp, L, seed):
    k, p = kp
    rng = np.random.default_rng(seed)
    data = [rng.integers(0, 256, L, dtype=np.uint8) for _ in range(k)]
    c = _encode(k, p, data)
    rs = O.ReedSolomon(k, p)
    n = [d.copy() for d in data] + [np.zeros(L, np.uint8) for _ in range(p)]
    rs.encode(n)
    for i in range(k + p):
        assert np.array_equal(np.asarray(n[i]), c[i])
