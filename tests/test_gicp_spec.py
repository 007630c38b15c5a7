"""CPU tests of the GICP spec against independent restatements.

The GPU kernels and the oracle's bit-exact GICP share pcore_gicp_math.h; these tests hold that shared arithmetic
to references that share nothing with it:
  - the double sin / cos of pcore_dmath.h against numpy (1 ulp);
  - se3_exp against scipy's matrix exponential of the twist;
  - the damped pivoted LDLT against numpy.linalg.solve;
  - the per-point linearisation (H, b, e^T M e) against the oracle's long-double 4x4 textbook form (1e-9 relative);
  - the whole LM iteration against tests/gicp_reference.py (numpy + scipy, fast_gicp's published step_lm);
  - the three-FMA correspondence key against the exact float squared-distance argmin.
Fast_gicp itself is not vendored: parity against the reference binary stays unpinned.
"""
from __future__ import annotations

import numpy as np
import pytest
import scipy.linalg as sla

import oracle
from tests import gicp_reference as gref
from tests.helpers import SceneCase

C3_NAMES = ("003_cracker_box", "004_sugar_box", "005_tomato_soup_can", "006_mustard_bottle", "010_potted_meat_can")


@pytest.fixture(scope="module")
def c3_pairs():
    """(rendered cloud, its covariances, label segment, segment covariances) of C3-style candidate poses: five
    objects, stride 8, 640x480, candidates around the ground truth (oracle raster + unprojection)."""
    case = SceneCase(names=C3_NAMES, n_poses=5, seed=7)
    sc = case.scene
    depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses, case.pose_model, case.pose_label,
                                sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    seg_cov = {}
    out = []
    for i in range(len(case.poses)):
        xyz = oracle.depth_to_cloud(depth[i], 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        lab = int(case.pose_label[i])
        tgt = case.obs_xyz[case.label_start[lab]:case.label_end[lab]]
        if len(xyz) == 0 or len(tgt) == 0:
            continue
        if lab not in seg_cov:
            seg_cov[lab] = oracle.covariances(tgt)
        out.append((xyz, oracle.covariances(xyz), tgt, seg_cov[lab]))
    assert len(out) >= 20
    return out


def test_sin_cos_within_one_ulp():
    rng = np.random.default_rng(1)
    xs = np.concatenate([rng.uniform(-4, 4, 4000), rng.uniform(-1e3, 1e3, 2000), rng.uniform(-1e6, 1e6, 500),
                         np.geomspace(1e-300, 1.0, 200), -np.geomspace(1e-12, 1.0, 50),
                         np.arange(-40, 41) * (np.pi / 4)])
    for f, ref in ((oracle.sin_d, np.sin), (oracle.cos_d, np.cos)):
        got = np.array([f(x) for x in xs])
        want = ref(xs)
        ulp = np.spacing(np.maximum(np.abs(want), 1e-300)) * np.where(np.abs(xs) < 1e4, 1.0, 2.0)
        # near a zero of the function the absolute error is the reduction's (three-part pi/2)
        err = np.abs(got - want)
        assert np.all((err <= ulp) | (err <= 1e-29 * np.maximum(1.0, np.abs(xs)))), f
    assert np.isnan(oracle.sin_d(np.inf)) and np.isnan(oracle.cos_d(np.nan))
    assert oracle.sin_d(0.0) == 0.0 and oracle.cos_d(0.0) == 1.0


@pytest.mark.parametrize("scale", [0.0, 1e-12, 3e-6, 1e-3, 0.2, 1.5, 3.0])
def test_se3_exp_matches_matrix_exponential(scale):
    """se3_exp (fast_gicp so3.hpp: exact so3_exp quaternion + V rho) = expm of the twist; the Taylor branches below
    theta^2 = 1e-10 and theta = 1e-10 included (below theta = 1e-10 fast_gicp takes V = R instead of I + Omega / 2
    + ..., off by theta |rho| / 2; above it, (1 - cos theta) / theta^2 and (theta - sin theta) / theta^3 as published
    cancel to ~eps / theta relative, so V rho is good to ~eps |rho| / theta)."""
    rng = np.random.default_rng(int(scale * 1e6) + 3)
    for _ in range(20):
        w = rng.normal(size=3)
        w = w / np.linalg.norm(w) * scale
        d = np.concatenate([w, rng.normal(size=3) * 0.05])
        T = oracle.gicp_se3_exp(d)
        ref = gref.se3_exp(d)
        rho = np.abs(d[3:]).max()
        tol = 5e-15 + (scale * rho if scale < 1e-10 else 1e-15 * rho / scale)
        assert np.abs(T - ref).max() < tol
        R = T[:3, :3]
        assert np.abs(R @ R.T - np.eye(3)).max() < 4e-15


def test_lm_solve_matches_dense_solve():
    """The damped solve (pcore_gicp_math.h lm_solve_schur: 3x3 block elimination of the translation block with
    adjugates) against numpy's dense solve of H + lambda I, -b: random SPD systems with column scales over four
    decades, half of them with the largest diagonal last; the error is bounded by cond(H + lambda I) times a few ulps.
    A zero system gives a zero step (as Eigen's LDLT of the zero matrix does)."""
    rng = np.random.default_rng(5)
    for trial in range(200):
        A = rng.normal(size=(6, 6)) * rng.uniform(0.01, 100, 6)
        H = A @ A.T
        if trial % 2:
            H = H[::-1, ::-1].copy()
        b = rng.normal(size=6)
        lam = [0.0, 1e-9, 1e-3][trial % 3] * np.abs(np.diag(H)).max()
        d = oracle.gicp_lm_solve(H, b, lam)
        ref = np.linalg.solve(H + lam * np.eye(6), -b)
        cond = np.linalg.cond(H + lam * np.eye(6))
        assert np.abs(d - ref).max() <= 1e-14 * cond * np.abs(ref).max(), (trial, cond)
    assert np.all(oracle.gicp_lm_solve(np.zeros((6, 6)), np.ones(6), 0.0) == 0.0)


def test_lm_solve_on_gicp_systems_matches_dense_solve(c3_pairs):
    """On the normal equations GICP actually forms (C3 candidates at the identity, at a perturbed pose and at the
    converged one, damped by the first iteration's lambda; condition numbers up to ~2e5): the block solve within
    1e-15 cond(H + lambda I) relative of numpy's (measured: <= 1e-16 cond)."""
    rng = np.random.default_rng(9)
    for src, scov, tgt, tcov in c3_pairs:
        T_conv, _ = oracle.gicp(src, scov, tgt, tcov)
        pert = gref.se3_exp(np.concatenate([rng.normal(size=3) * 0.05, rng.normal(size=3) * 0.01]))
        for T in (np.eye(4), pert, T_conv):
            _, H, b, _ = oracle.gicp_linearize(src, scov, tgt, tcov, T)
            lam = 1e-9 * np.abs(np.diag(H)).max()
            d = oracle.gicp_lm_solve(H, b, lam)
            ref = np.linalg.solve(H + lam * np.eye(6), -b)
            cond = np.linalg.cond(H + lam * np.eye(6))
            assert np.abs(d - ref).max() <= 1e-15 * cond * np.abs(ref).max()


def _rel(a, b):
    return np.abs(np.asarray(a) - np.asarray(b)).max() / max(np.abs(np.asarray(b)).max(), 1e-300)


def test_linearize_matches_textbook(c3_pairs):
    """The shared per-point step (upper J^T M J, J^T M e, e^T M e; adjugate inverse, structural zeros skipped) equals
    fast_gicp's 4x4 homogeneous form evaluated independently in long double, to 1e-9 relative, at the identity, at a
    perturbed transform and at the converged one."""
    rng = np.random.default_rng(11)
    for src, scov, tgt, tcov in c3_pairs[::2]:
        T_conv, _ = oracle.gicp(src, scov, tgt, tcov)
        pert = gref.se3_exp(np.concatenate([rng.normal(size=3) * 0.05, rng.normal(size=3) * 0.01]))
        for T in (np.eye(4), pert, T_conv):
            c0, H0, b0, y0 = oracle.gicp_linearize(src, scov, tgt, tcov, T, textbook=False)
            c1, H1, b1, y1 = oracle.gicp_linearize(src, scov, tgt, tcov, T, textbook=True)
            assert np.array_equal(c0, c1)
            assert _rel(H0, H1) < 1e-9
            assert _rel(b0, b1) < 1e-9 or np.abs(b0 - b1).max() < 1e-9 * np.abs(H1).max()
            assert abs(y0 - y1) <= 1e-9 * max(abs(y1), 1e-12)


def test_gicp_matches_independent_numpy_lm(c3_pairs):
    """The oracle's GICP (the GPU's arithmetic) and the independent numpy / scipy restatement of fast_gicp's LM
    (tests/gicp_reference.py) run the same number of iterations and land within 1e-9 of each other -- including
    the poses that run all 150 iterations (wrong candidates whose correspondences flip between two sets every
    iteration, a limit cycle the published step_lm accepts)."""
    iters = []
    for src, scov, tgt, tcov in c3_pairs:
        T1, it1 = oracle.gicp(src, scov, tgt, tcov, cycle_window=0)
        T2, it2 = gref.gicp(src, scov, tgt, tcov)
        assert it1 == it2
        assert np.abs(T1 - T2).max() < 1e-9
        iters.append(it1)
    assert min(iters) >= 1 and max(iters) <= 150


def _key_gap(q, tgt):
    j = oracle.gicp_nn(q, tgt)
    d = ((q[:, None, :] - tgt[None, :, :]) ** 2).sum(-1, dtype=np.float32)  # float squared distances
    ok = j >= 0
    got = d[np.arange(len(q))[ok], j[ok]]
    return got - d[ok].min(1), ok


@pytest.mark.parametrize("n_tgt", [57, 180, 2048, 2049])
def test_key_nearest_is_the_nearest(c3_pairs, n_tgt):
    """The correspondence key |q'-t'|^2 - |q'|^2 (three FMAs about the segment's origin) picks a target whose float
    squared distance is within 1e-9 m^2 of the true nearest one -- queries on the object, a centimetre off it, a
    decimetre off and a metre away; segments of 2048 targets (the largest key scan) and 2049 (the plain distance of
    the grid-search path, exact)."""
    rng = np.random.default_rng(n_tgt)
    pool = np.concatenate([p[2] for p in c3_pairs] + [p[0] for p in c3_pairs])
    tgt = pool[rng.choice(len(pool), min(n_tgt, len(pool)), replace=False)]
    if len(tgt) < n_tgt:  # whole-scene style segment: jittered copies
        extra = tgt[rng.choice(len(tgt), n_tgt - len(tgt))] + rng.normal(scale=0.003, size=(n_tgt - len(tgt), 3))
        tgt = np.concatenate([tgt, extra]).astype(np.float32)
    base = tgt[rng.choice(len(tgt), 300)]
    for off in (0.0, 0.01, 0.1, 1.0):
        q = (base + rng.normal(scale=off, size=base.shape)).astype(np.float32) if off else base.copy()
        gap, ok = _key_gap(q, tgt)
        assert ok.all()
        if n_tgt > 2048:
            assert np.all(gap == 0.0)
        else:
            assert np.all(gap <= 1e-9 + 1e-6 * off * off), (off, gap.max())


def test_key_nearest_ties_and_tiny_keys():
    """Exact duplicates: the first index wins (strict <); queries at a target give keys near -|q'|^2 and denormal
    differences without losing the nearest."""
    t = np.array([[0.1, 0.2, 0.8], [0.1, 0.2, 0.8], [0.1, 0.2, 0.80000001], [0.3, 0.2, 0.8]], np.float32)
    j = oracle.gicp_nn(t[[0, 2, 3]], t)
    assert list(j) == [0, 0, 3] or list(j) == [0, 2, 3]
    assert j[0] == 0
    q = np.array([[0.2, 0.2, 0.8], [1e-30, 0.0, 0.0]], np.float32)
    assert list(oracle.gicp_nn(q, t)) == [0, 0]


def test_max_iteration_poses_are_two_cycles(c3_pairs):
    """Why ~40 % of C3's candidates run all 150 iterations: step_lm scores a trial with the
    iteration's own correspondences, which every Gauss-Newton step improves, so it is accepted; re-correspondence at
    the new pose then restores the previous set.  The trace of such a pose alternates between two states: x_{k+1}
    returns to within 1e-9 of x_{k-1} while moving > 1e-5 from x_k -- but never bit-exactly (periods 1..8 checked),
    so no exact shortcut exists and the spec runs the iterations out."""
    n_cycles = 0
    for src, scov, tgt, tcov in c3_pairs:
        T, it, tr = oracle.gicp_trace(src, scov, tgt, tcov)
        assert np.array_equal(T[:3, :3], tr[-1, :9].reshape(3, 3)) and np.array_equal(T[:3, 3], tr[-1, 9:12])
        if it < 150:
            continue
        X = tr[:, :12]
        tail = range(130, 150)
        back = max(np.abs(X[k] - X[k - 2]).max() for k in tail)
        step = min(np.abs(X[k] - X[k - 1]).max() for k in tail)
        if back < 1e-9 and step > 1e-5:
            n_cycles += 1
            for P in range(1, 9):
                assert not any(np.array_equal(X[k].view(np.uint64), X[k - P].view(np.uint64)) for k in range(P, 150))
    assert n_cycles >= 2


def test_cube_rn_is_correctly_rounded():
    """step_lm's (2 rho - 1)^3 (fast_gicp: std::pow(.., 3)) is computed as one correctly rounded cube
    (pcore_gicp_math.h cube_rn), checked against exact rationals; the two-rounding (u u) u it replaced differs from
    the exact cube on ~1 in 4 inputs, glibc's pow on ~1 in 1000.  lm_gain = max(1/3, 1 - cube)."""
    from fractions import Fraction

    rng = np.random.default_rng(12)
    us = np.concatenate([rng.uniform(-1, 1, 6000), rng.uniform(-3, 3, 1000), np.geomspace(1e-200, 1, 200),
                         -np.geomspace(1e-12, 1, 100), [0.0, -0.0, 1.0, -1.0, 0.5, 2.0 ** -30]])
    naive = 0
    for u in us:
        exact = float(Fraction(float(u)) ** 3)
        assert oracle.cube_rn(u) == exact, u
        naive += ((u * u) * u) != exact
    assert naive > len(us) // 20  # the rounding mattered
    for rho in (-5.0, -0.3, 0.0, 0.25, 0.5, 0.75, 0.9, 1.0, 1.7, 3.0):
        u = Fraction(2.0 * rho - 1.0)  # 2 rho - 1 as the double the code forms
        assert oracle.lm_gain(rho) == max(1.0 / 3.0, 1.0 - float(u ** 3)), rho


@pytest.fixture(scope="module")
def c3_pairs_120():
    """120 C3-style candidates (24 per object around the ground truth), their clouds, and BOTH covariance sets: the
    oracle's and tests/gicp_reference.py's numpy ones (lexsort k-NN, eigh normal)."""
    case = SceneCase(names=C3_NAMES, n_poses=24, seed=7)
    sc = case.scene
    depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, case.poses, case.pose_model, case.pose_label,
                                sc.width, sc.height, sc.proj, sc.src_depth_cm, sc.mask, 1.0)
    seg = {}
    out = []
    for i in range(len(case.poses)):
        xyz = oracle.depth_to_cloud(depth[i], 8, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        lab = int(case.pose_label[i])
        tgt = case.obs_xyz[case.label_start[lab]:case.label_end[lab]]
        if len(xyz) == 0 or len(tgt) == 0:
            continue
        if lab not in seg:
            seg[lab] = (oracle.covariances(tgt), gref.covariances(tgt))
        out.append((xyz, oracle.covariances(xyz), gref.covariances(xyz), tgt) + seg[lab])
    return out


def test_gicp_independent_chain_120_c3_poses(c3_pairs_120):
    """>= 100 C3 candidates, the capped (150-iteration) ones included, through a chain that
    shares nothing with the product's GICP header -- numpy covariances on both clouds, numpy / scipy LM -- against the
    oracle (the GPU's arithmetic, bit-exact with the kernels): equal iteration counts, transforms within 1e-9."""
    iters = []
    for src, scov_o, scov_g, tgt, tcov_o, tcov_g in c3_pairs_120:
        assert np.abs(scov_o - scov_g).max() < 1e-12
        T1, it1 = oracle.gicp(src, scov_o, tgt, tcov_o, cycle_window=0)
        T2, it2 = gref.gicp(src, scov_g, tgt, tcov_g)
        assert it1 == it2
        assert np.abs(T1 - T2).max() < 1e-9
        iters.append(it1)
    iters = np.array(iters)
    assert len(iters) >= 100 and (iters >= 150).sum() >= 20 and (iters < 150).sum() >= 20


def _float_T(T):
    return np.concatenate([T[:3, :3].reshape(-1), T[:3, 3]]).astype(np.float32)


def test_cycle_exit_against_full_length_chains(c3_pairs_120):
    """The spec's cycle exit (pcore_gicp_math.h cycle_update, W = 8) against running every
    iteration out, on the 120 C3 candidates: the same reported iteration counts; the float transform (what
    concatenate_transforms composes) bit-identical on >= 99 % of the candidates and within 1e-6 on the rest; and the
    exit's result against the independent numpy chain run to 150 iterations (tests/gicp_reference.py): equal
    iterations, within 1e-6.  The exits happen (the capped candidates are LM cycles) and save iterations."""
    same = exits = run_on = run_off = 0
    worst = 0.0
    for src, scov_o, scov_g, tgt, tcov_o, tcov_g in c3_pairs_120:
        T0, it0, tr0 = oracle.gicp_trace(src, scov_o, tgt, tcov_o, cycle_window=0)
        T1, it1, tr1 = oracle.gicp_trace(src, scov_o, tgt, tcov_o, cycle_window=oracle.GICP_CYCLE_WINDOW)
        T2, it2 = oracle.gicp(src, scov_o, tgt, tcov_o)  # the default is the spec's window
        assert np.array_equal(T1, T2) and it1 == it2
        assert it0 == it1
        exits += len(tr1) < len(tr0)
        run_on += len(tr1)
        run_off += len(tr0)
        f0, f1 = _float_T(T0), _float_T(T1)
        same += np.array_equal(f0.view(np.uint32), f1.view(np.uint32))
        worst = max(worst, float(np.abs(f0 - f1).max()))
        Tg, itg = gref.gicp(src, scov_g, tgt, tcov_g)
        assert itg == it1 and np.abs(_float_T(Tg) - f1).max() <= 1e-6
    n = len(c3_pairs_120)
    assert same >= 0.99 * n and worst <= 1e-6
    assert exits >= 20 and run_on < 0.75 * run_off


def test_schur_and_ldlt_chains_take_the_same_decisions(c3_pairs_120):
    """the spec's damped solve (3x3 block elimination) against fast_gicp's own (Eigen's pivoted LDLT,
    restated in the oracle as a test reference) over whole GICP chains on the 120 C3 candidates, every iteration run
    out: every iteration's LM decision (trials, status) is the same, so the iteration counts are; the transforms
    agree to 1e-9.  And the two solves agree on the lm_solve_cases systems within 1e-14 cond relative."""
    worst = 0.0
    for src, scov_o, _, tgt, tcov_o, _ in c3_pairs_120:
        T1, it1, tr1 = oracle.gicp_trace(src, scov_o, tgt, tcov_o, solver="schur")
        T2, it2, tr2 = oracle.gicp_trace(src, scov_o, tgt, tcov_o, solver="ldlt")
        assert it1 == it2
        assert np.array_equal(tr1[:, 13], tr2[:, 13]) and np.array_equal(tr1[:, 15], tr2[:, 15])
        worst = max(worst, float(np.abs(T1 - T2).max()))
    assert worst < 1e-9
    for sysv, lam in lm_solve_cases()[:1500]:
        if not np.isfinite(sysv).all():
            continue
        H = np.zeros((6, 6))
        H[np.triu_indices(6)] = sysv[:21]
        Hs = H + np.triu(H, 1).T + lam * np.eye(6)
        if not (np.all(np.linalg.eigvalsh(Hs) > 1e-12 * np.abs(Hs).max()) and np.linalg.cond(Hs) < 1e10):
            continue
        d1, d2 = oracle.gicp_lm_solve_sys(sysv, lam), oracle.gicp_lm_solve_ldlt_sys(sysv, lam)
        assert np.abs(d1 - d2).max() <= 1e-14 * np.linalg.cond(Hs) * np.abs(d2).max() + 1e-300


def test_cycle_window_constants_agree():
    """The spec's window is one number in the oracle, the Python host and include/pcore.h."""
    import re
    from pathlib import Path

    from perception_amd import _native
    h = (Path(__file__).resolve().parents[1] / "include" / "pcore.h").read_text()
    assert int(re.search(r"#define PCORE_GICP_CYCLE_WINDOW (\d+)", h).group(1)) == 8
    assert oracle.GICP_CYCLE_WINDOW == _native.ICP_CYCLE_WINDOW == 8


def test_gicp_whole_scene_targets_independent_chain():
    """C1's 3-DoF table-top GICP against the WHOLE observed cloud (19.2 k targets at stride 4:
    the segments above 2,048 targets that gicp_wide_kernel's exact grid shell search serves, and the plain float
    distance rule), the two 150-iteration poses that GICP walks away from the scene included: oracle vs the numpy
    chain with numpy covariances, equal iterations, transforms within 1e-9."""
    from perception_amd import workloads
    from tests.helpers import oracle_render_fn

    c1 = workloads.c1_tabletop(oracle_render_fn)
    sc = c1.scene
    obs, _ = oracle.depth_to_cloud_bounded(sc.depth_raw, 4, sc.cx, sc.cy, sc.fx, sc.fy, sc.depth_factor)
    assert len(obs) > 2048 * 4
    tcov_o, tcov_g = oracle.covariances(obs), gref.covariances(obs)
    assert np.abs(tcov_o - tcov_g).max() < 1e-12
    idx = np.array([c1.gt_index, 90, 66, 3], np.int64)  # 90: 150 iterations, 66: 47 (oracle, this scene)
    depth = oracle.render_depth(sc.bank.tris, sc.bank.tris_model_count, c1.poses[idx], np.zeros(len(idx), np.int32),
                                None, sc.width, sc.height, sc.proj, c1.src_depth_cm, None, 1.0)
    iters = []
    for i in range(len(idx)):
        src = oracle.depth_to_cloud(depth[i], 4, sc.cx, sc.cy, sc.fx, sc.fy, 100.0)[0]
        T1, it1 = oracle.gicp(src, oracle.covariances(src), obs, tcov_o, cycle_window=0)
        T2, it2 = gref.gicp(src, gref.covariances(src), obs, tcov_g)
        assert it1 == it2, (idx[i], it1, it2)
        assert np.abs(T1 - T2).max() < 1e-9
        iters.append(it1)
    assert max(iters) == 150


def lm_solve_cases():
    """Random SPD and indefinite 28-term systems, tied and zero diagonals, a zero system, huge / tiny scales and
    non-finite entries, with their damping: (sys, lambda) pairs (also the GPU solve's test cases)."""
    rng = np.random.default_rng(31)
    iu = np.triu_indices(6)
    cases = []
    for t in range(4000):
        A = rng.normal(size=(6, 6)) * rng.choice([1e-6, 1.0, 1e3, 1e12])
        H = A @ A.T if t % 3 else A + A.T  # SPD or indefinite
        if t % 7 == 0:  # ties in the diagonal magnitudes
            v = H[0, 0]
            for i in rng.choice(6, 3, replace=False):
                H[i, i] = v if rng.random() < 0.5 else -v
        if t % 11 == 0:
            H[rng.integers(6), :] = 0.0
            H = (H + H.T) * 0.5
        b = rng.normal(size=6)
        cases.append((np.concatenate([H[iu], b, [0.0]]), float(rng.choice([0.0, 1e-9, 1e-3, 10.0]))))
    cases.append((np.zeros(28), 0.0))
    cases.append((np.zeros(28), 1e-9))
    z = np.zeros(28)
    z[[0, 6, 11]] = 5.0
    cases.append((z.copy(), 0.0))
    for bad in (np.nan, np.inf, -np.inf):
        for pos in (0, 3, 6, 20, 22):
            sysb = cases[5][0].copy()
            sysb[pos] = bad
            cases.append((sysb, 1e-9))
    return cases


def test_lm_solve_degenerate_systems():
    """The block solve's edge cases over the systems the GPU test also runs (tests/test_gpu_gicp_solve.py): the zero
    system gives d = 0 with or without damping; a non-finite entry gives a non-finite step (lm_iteration's guard then
    stops the pose); a finite SPD system a finite step."""
    for sysv, lam in lm_solve_cases():
        d = oracle.gicp_lm_solve_sys(sysv, lam)
        H = np.zeros((6, 6))
        H[np.triu_indices(6)] = sysv[:21]
        if not np.isfinite(sysv).all():
            assert not np.isfinite(d).all()
        elif not np.any(np.diag(H) + lam):
            assert np.all(d == 0.0)
        else:
            Hs = H + np.triu(H, 1).T + lam * np.eye(6)
            if np.all(np.linalg.eigvalsh(Hs) > 1e-12 * np.abs(Hs).max()) and np.linalg.cond(Hs) < 1e10:
                ref = np.linalg.solve(Hs, -sysv[21:27])
                assert np.abs(d - ref).max() <= 1e-14 * np.linalg.cond(Hs) * np.abs(ref).max() + 1e-300


def test_se3_exp_series_and_quotients_meet_at_the_switch():
    """se3_exp switches from the power series of imag / real / c1 / c2 (theta^2 < 1/4) to the published quotients of
    sin / cos: on both sides of the switch the result is within a few ulps of scipy's expm of the twist, and small steps
    (theta ~ 1e-3, where the published (theta - sin theta) / theta^3 loses ~1e-10 relative to cancellation) match expm
    to 1e-15."""
    rng = np.random.default_rng(17)
    for theta in (0.5 * (1 - 1e-12), 0.5, 0.5 * (1 + 1e-12), 1e-3, 3e-5):
        for _ in range(10):
            w = rng.normal(size=3)
            w = w / np.linalg.norm(w) * theta
            d = np.concatenate([w, rng.normal(size=3) * 0.05])
            assert np.abs(oracle.gicp_se3_exp(d) - gref.se3_exp(d)).max() < 3e-16 * 8
