"""CPU tests of the parallel host sampler (libncf_sampler.so): MT19937 jump-ahead,
the parallel word generator, and the parallel ng_sample pass against the
sequential pass and the oracle's C restatement of datasets.py:53-69 -- bit-exact
negatives and the same NumPy global state afterwards."""
import ctypes
import os

import numpy as np
import pytest
import scipy.sparse as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _lib():
    import ncf_amd._lib as L
    return L.sampler_lib()


def _seeded(seed):
    key = np.empty(624, np.uint32)
    pos = np.empty(1, np.int32)
    _lib().ncf_mt_seed(seed, key.ctypes.data, pos.ctypes.data)
    return key, pos


@pytest.mark.parametrize("k", [1, 2, 7, 33, 160, 1000, 4097])
def test_mt_jump_lands_on_the_generators_array(k):
    """ncf_mt_jump(key, 624 k) == the key[624] array numpy holds after 624 k draws."""
    key, pos = _seeded(1234 + k)
    seq_key, seq_pos = key.copy(), pos.copy()
    _lib().ncf_mt_words(seq_key.ctypes.data, seq_pos.ctypes.data, 624 * k, None)
    assert int(seq_pos[0]) == 624
    jk = key.copy()
    assert _lib().ncf_mt_jump(jk.ctypes.data, 624 * k) == 0
    assert np.array_equal(jk, seq_key)
    # and numpy continues identically from it
    np.random.set_state(("MT19937", jk, 624, 0, 0.0))
    a = np.random.randint(1 << 30, size=50)
    np.random.set_state(("MT19937", seq_key, 624, 0, 0.0))
    assert np.array_equal(a, np.random.randint(1 << 30, size=50))


def test_mt_jump_arbitrary_distance_matches_window_shift():
    """A jump of J words that is not a multiple of 624 is the stream shifted by J:
    the window jumped by J from the seeded array, consumed from its start, gives
    words J+624.. of the seeded stream (the seeded array itself is words 0..623
    of the untempered stream; the first draw regenerates)."""
    key, pos = _seeded(99)
    n = 40000
    words = np.empty(n, np.uint32)
    k2, p2 = key.copy(), pos.copy()
    _lib().ncf_mt_words(k2.ctypes.data, p2.ctypes.data, n, words.ctypes.data)
    for J in (1, 5, 623, 625, 1300, 19937, 20001):
        jk = key.copy()
        _lib().ncf_mt_jump(jk.ctypes.data, J)
        out = np.empty(1000, np.uint32)
        pj = np.array([0], np.int32)  # next draw = temper(window[0]) = word J of the untempered stream
        _lib().ncf_mt_words(jk.ctypes.data, pj.ctypes.data, 1000, out.ctypes.data)
        # out[i] = temper(x_{J+i}) and words[i] = temper(x_{624+i})
        if J >= 624:
            assert np.array_equal(out, words[J - 624: J - 624 + 1000])
        else:  # x_J .. x_623 are the seeded array itself, then the stream
            assert np.array_equal(out[624 - J:], words[: 1000 - (624 - J)])


@pytest.mark.parametrize("threads", [1, 2, 3, 8])
@pytest.mark.parametrize("n,start", [(1, 624), (623, 624), (5000, 17), (700_001, 624), (2_000_000, 0),
                                     (1_234_567, 300)])
def test_parallel_words_match_sequential(threads, n, start):
    L = _lib()
    key, pos = _seeded(7 + n)
    pos[0] = start
    if start < 624:  # any valid mid-block state: advance a seeded generator
        key, pos = _seeded(7 + n)
        L.ncf_mt_words(key.ctypes.data, pos.ctypes.data, 624 + start, None)
    a_key, a_pos = key.copy(), pos.copy()
    a = np.empty(n, np.uint32)
    L.ncf_mt_words(a_key.ctypes.data, a_pos.ctypes.data, n, a.ctypes.data)
    h = L.ncf_words_create(threads)
    try:
        b_key, b_pos = key.copy(), pos.copy()
        b = np.zeros(n, np.uint32)
        assert L.ncf_words_fill(h, b_key.ctypes.data, b_pos.ctypes.data, n, b.ctypes.data) == 0
    finally:
        L.ncf_words_destroy(h)
    assert np.array_equal(a, b)
    assert np.array_equal(a_key, b_key) and int(a_pos[0]) == int(b_pos[0])


def _ml1m_like(seed, U=6041, I=3707, hi=330):
    rng = np.random.default_rng(seed)
    counts = rng.integers(1, hi, U)
    pu = np.repeat(np.arange(U), counts)
    pi = rng.integers(0, I, len(pu))
    return pu, pi, U, I


def _passes(pu, pi, U, I, ng, seed, threads, n_pass, num_item=None, mem=None):
    from ncf_amd.data import HostSampler
    num_item = I if num_item is None else num_item
    s = HostSampler(pu, pi, U, I, *(mem or (None, None)), threads=threads)
    np.random.seed(seed)
    outs = [s.sample(num_item, ng).copy() for _ in range(n_pass)]
    after = np.random.get_state()
    return outs, after, s.stats()


@pytest.mark.parametrize("threads", [2, 8])
@pytest.mark.parametrize("ng,seed", [(4, 21), (1, 3)])
def test_parallel_pass_matches_sequential_and_oracle(threads, ng, seed):
    from oracle import ncf_oracle as O
    pu, pi, U, I = _ml1m_like(seed)
    seq, st_seq, _ = _passes(pu, pi, U, I, ng, seed, 1, 3)
    par, st_par, stats = _passes(pu, pi, U, I, ng, seed, threads, 3)
    assert stats["parallel"] == 3 and stats["epoch_fallbacks"] == 0 and stats["sequential"] == 0
    for a, b in zip(seq, par):
        assert np.array_equal(a, b)
    assert np.array_equal(st_seq[1], st_par[1]) and st_seq[2] == st_par[2]
    assert np.array_equal(par[0], O.ng_sample(pu, pi, I, ng, seed))


def test_parallel_pass_edge_shapes():
    """Heavy users (a user owning ~95% of the items: long redraw runs), positives
    not grouped by user (alternating runs), num_item larger than the membership
    universe, a single run, and far more threads than blocks."""
    from oracle import ncf_oracle as O
    rng = np.random.default_rng(5)
    I = 2000
    heavy = np.stack([np.zeros(1900, np.int64), rng.permutation(I)[:1900]], 1)
    light = np.stack([rng.integers(1, 300, 20000), rng.integers(0, I, 20000)], 1)
    pos = np.concatenate([light[:7000], heavy, light[7000:]])
    pu, pi = pos[:, 0], pos[:, 1]
    seq, st_seq, _ = _passes(pu, pi, 300, I, 4, 11, 1, 2)
    par, st_par, stats = _passes(pu, pi, 300, I, 4, 11, 8, 2)
    assert stats["parallel"] == 2 and stats["epoch_fallbacks"] == 0
    assert all(np.array_equal(a, b) for a, b in zip(seq, par))
    assert np.array_equal(st_seq[1], st_par[1]) and st_seq[2] == st_par[2]
    assert np.array_equal(par[0], O.ng_sample(pu, pi, I, 4, 11))
    # num_item beyond the membership universe (candidates >= n_items are never members)
    seq, st_seq, _ = _passes(pu, pi, 300, I, 3, 12, 1, 1, num_item=I + 777)
    par, st_par, _ = _passes(pu, pi, 300, I, 3, 12, 6, 1, num_item=I + 777)
    assert np.array_equal(seq[0], par[0]) and st_seq[2] == st_par[2]
    assert np.array_equal(par[0], O.ng_sample(pu, pi, I + 777, 3, 12))
    # one user, one run
    pu1 = np.zeros(500, np.int64)
    pi1 = rng.permutation(I)[:500]
    seq, st_seq, _ = _passes(pu1, pi1, 1, I, 4, 13, 1, 2)
    par, st_par, _ = _passes(pu1, pi1, 1, I, 4, 13, 16, 2)
    assert all(np.array_equal(a, b) for a, b in zip(seq, par)) and np.array_equal(st_seq[1], st_par[1])


def test_user_owning_every_item_refuses():
    from ncf_amd.data import HostSampler
    pu = np.array([0] * 10 + [1, 1])
    pi = np.array(list(range(10)) + [3, 4])
    s = HostSampler(pu, pi, 2, 10, threads=4)
    np.random.seed(0)
    with pytest.raises(RuntimeError, match="every item"):
        s.sample(10, 4)
    s1 = HostSampler(pu, pi, 2, 10, threads=1)
    with pytest.raises(RuntimeError, match="every item"):
        s1.sample(10, 4)


def test_train_mat_membership_and_duplicates_like_reference():
    """NCFData with a dok train_mat holding pairs beyond the positives and with
    duplicate positives: the redraw test is `(u, j) in train_mat` (datasets.py:61)."""
    from ncf_amd.data import NCFData
    rng = np.random.default_rng(2)
    U, I = 40, 60
    pos = np.stack([np.repeat(np.arange(U), 6), rng.integers(0, I, U * 6)], 1)
    pos = np.concatenate([pos, pos[:10]])  # duplicates
    pos = pos[np.argsort(pos[:, 0], kind="stable")]
    extra = np.stack([rng.integers(0, U, 300), rng.integers(0, I, 300)], 1)
    mat = sp.dok_matrix((U, I), dtype=np.float32)
    for u, i in np.concatenate([pos, extra]).tolist():
        mat[u, i] = 1.0
    for threads in (1, 4):
        np.random.seed(17)
        d = NCFData(pos.tolist(), I, mat, 3, True)
        d._get_sampler().set_threads(threads)
        d.ng_sample()
        got = d._ng_i.astype(np.int64)
        np.random.seed(17)
        exp = []
        for u in pos[:, 0].tolist():
            for _ in range(3):
                j = np.random.randint(I)
                while (u, j) in mat:
                    j = np.random.randint(I)
                exp.append(j)
        assert np.array_equal(got, np.asarray(exp))


def test_cached_gaussian_survives_ng_sample():
    """randint draws leave the legacy state's cached Gaussian alone (the reference's
    ng_sample only calls randint)."""
    from ncf_amd.data import NCFData
    pos = np.stack([np.repeat(np.arange(20), 5), np.tile(np.arange(5), 20)], 1)
    np.random.seed(3)
    np.random.standard_normal()  # caches the second Gaussian of the pair
    st = np.random.get_state()
    assert st[3] == 1
    d = NCFData(pos.tolist(), 30, None, 2, True)
    d.ng_sample()
    st2 = np.random.get_state()
    assert st2[3] == 1 and st2[4] == st[4]


def _ml20m_like(seed=0):
    """ml-20m-shaped positives (138,493 users x 26,744 items, lognormal activity,
    Zipf(0.8) popularity; duplicates allowed) -- fast, not the bench's generator."""
    rng = np.random.default_rng(seed)
    U, I = 138_494, 26_745
    w = rng.lognormal(0.0, 1.0, U - 1)
    counts = 20 + np.floor(w / w.sum() * (19_861_770 - 20 * (U - 1))).astype(np.int64)
    counts = np.minimum(counts, I // 2)
    p = np.arange(1, I, dtype=np.float64) ** -0.8
    p /= p.sum()
    pu = np.repeat(np.arange(1, U, dtype=np.int32), counts)
    pi = (rng.choice(I - 1, size=len(pu), p=p) + 1).astype(np.int32)
    return pu, pi, U, I


def test_ml20m_shape_all_negatives_bit_exact_vs_oracle():
    """Every one of the ~79M negatives of an ml-20m-shaped epoch, parallel pass vs the
    oracle's C restatement, then a second pass vs the sequential pass."""
    from oracle import ncf_oracle as O
    pu, pi, U, I = _ml20m_like()
    par, st_par, stats = _passes(pu, pi, U, I, 4, 0, 8, 2)
    assert stats["parallel"] == 2 and stats["epoch_fallbacks"] == 0
    exp = O.ng_sample(pu, pi, I, 4, 0)
    assert len(exp) == 4 * len(pu) > 70_000_000
    assert np.array_equal(par[0], exp)
    del exp
    seq, st_seq, _ = _passes(pu, pi, U, I, 4, 0, 1, 2)
    assert np.array_equal(seq[1], par[1])
    assert np.array_equal(st_seq[1], st_par[1]) and st_seq[2] == st_par[2]
