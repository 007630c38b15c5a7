"""The covariance k-NN's sorted-list updates (perception_amd/csrc/pcore_cov.h), restated in Python and held to the
counting insertion of the oracle's knn_self (oracle/pcore_oracle.cpp) on lists with many ties.

Round 6 rewrote two updates without changing their results:
  * the threshold step's running k smallest: t[q] <- med3(t[q-1], t[q], d), t[0] <- min(t[0], d), where the kernel
    had t[q-1] > d ? t[q-1] : (t[q] > d ? d : t[q]);
  * the collected candidates' insertion from a +inf-filled list: values by the same medians, indices by the shared
    compares g[q] = nd[q] > d, where the kernel had the counting insertion (start at pos = min(len, k - 1), move past
    the entries strictly greater than d).
The GPU tests check the kernels bit for bit against the oracle; this checks the algebra on the CPU.
"""
import math
import random

K = 10


def med3(a, b, c):
    return max(min(a, b), min(max(a, b), c))


def running_select(ds):
    t = [math.inf] * K
    for d in ds:
        for q in range(K - 1, 0, -1):
            t[q] = t[q - 1] if t[q - 1] > d else (d if t[q] > d else t[q])
        t[0] = d if t[0] > d else t[0]
    return t


def running_med3(ds):
    t = [math.inf] * K
    for d in ds:
        for q in range(K - 1, 0, -1):
            t[q] = med3(t[q - 1], t[q], d)
        t[0] = min(t[0], d)
    return t


def counting_insert(cands):
    """orc knn_self / the kernel's round-5 insertion: (d, j) in increasing j."""
    nd, nb = [0.0] * K, [0] * K
    n = 0
    for d, j in cands:
        if n < K:
            pos = n
        elif d < nd[K - 1]:
            pos = K - 1
        else:
            continue
        g = sum(1 for q in range(pos) if nd[q] > d)
        fin = pos - g
        for q in range(pos, fin, -1):
            nd[q], nb[q] = nd[q - 1], nb[q - 1]
        nd[fin], nb[fin] = d, j
        n = min(n + 1, K)
    return nd[:n], nb[:n]


def sentinel_insert(cands):
    """pcore_cov.h cov_knn_round_thr step 3 (round 6)."""
    nd, nb = [math.inf] * K, [0] * K
    n = 0
    for d, j in cands:
        if not d < nd[K - 1]:
            continue
        g = [nd[q] > d for q in range(K)]
        for q in range(K - 1, 0, -1):
            nd[q] = med3(nd[q - 1], nd[q], d)
            nb[q] = nb[q - 1] if g[q - 1] else (j if g[q] else nb[q])
        nd[0] = min(nd[0], d)
        nb[0] = j if g[0] else nb[0]
        n = min(n + 1, K)
    return nd[:n], nb[:n]


def _draws(rng, n, levels):
    # few distinct values: ties everywhere, including with the list's entries and +0.0
    return [rng.randrange(levels) * 0.125 for _ in range(n)]


def test_running_minima_median_form_equals_selects():
    rng = random.Random(7)
    for trial in range(3000):
        ds = _draws(rng, rng.randrange(0, 60), rng.choice([2, 5, 40, 10 ** 6]))
        assert running_med3(ds) == running_select(ds), trial


def test_median_is_the_select_on_sorted_pairs():
    rng = random.Random(11)
    for _ in range(20000):
        a, b = sorted(_draws(rng, 2, 6) + [])
        d = rng.randrange(6) * 0.125
        assert med3(a, b, d) == (a if a > d else (d if b > d else b))
        assert med3(a, math.inf, d) == (a if a > d else d)


def test_sentinel_insertion_equals_counting_insertion():
    rng = random.Random(3)
    for trial in range(4000):
        m = rng.randrange(0, 40)
        ds = _draws(rng, m, rng.choice([1, 3, 8, 50, 10 ** 6]))
        cands = list(zip(ds, sorted(rng.sample(range(10 * m + 1), m))))  # increasing indices, as collected
        assert sentinel_insert(cands) == counting_insert(cands), trial
