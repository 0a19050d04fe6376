"""The sqrt-free sphere decisions (rg_kernels.hip sphere_clear_side / sphere_shadow_quick /
sphere_behind) against the reference's tail (bodies.rs:105-119 + rendering.rs:152-155), on CPU.

numpy's float64 add/mul/sqrt are IEEE round-to-nearest without contraction, so the restatement
below computes exactly what the kernel computes (-ffp-contract=off).  Whenever the quick test
decides (shadow: 1 occluded / 0 not; closest: "behind"), the reference's answer must agree; the
test also checks that the quick test does decide the cases it is for (rays leaving a sphere's
surface, spheres behind or in front of the origin), so it cannot pass vacuously.
"""
import numpy as np

K = 1.0 + 2.0 ** -49
TINY = 2.0 ** -900


def geometry(c, r, o, d):
    hx, hy, hz = c[:, 0] - o[:, 0], c[:, 1] - o[:, 1], c[:, 2] - o[:, 2]   # bodies.rs:92
    adj = (hx * d[:, 0] + hy * d[:, 1]) + hz * d[:, 2]                    # :93
    opp = ((hx * hx + hy * hy) + hz * hz) - adj * adj                     # :95
    return r * r, opp, adj


def tail(r2, opp, adj):
    """sphere_tail: (hit, t) -- bodies.rs:105-119."""
    with np.errstate(invalid="ignore"):
        th = np.sqrt(r2 - opp)
    d0, d1 = adj - th, adj + th
    hit = ~((d0 < 0.0) & (d1 < 0.0))
    t = np.where(d0 < 0.0, d1, np.where(d1 < 0.0, d0, np.fmin(d0, d1)))
    return hit, t


def clear_side(r2, opp, adj):
    x = r2 - opp
    p = adj * adj
    with np.errstate(invalid="ignore"):
        return (p >= TINY) & (p > x * K)


def shadow_quick(r2, opp, adj, ld):
    cs = clear_side(r2, opp, adj)
    return np.where(~cs, -1, np.where(adj < 0.0, 0, np.where(adj <= ld, 1, -1)))


def behind(r2, opp, adj):
    return (adj < 0.0) & clear_side(r2, opp, adj)


def _unit(v):
    return v / np.sqrt((v * v).sum(axis=1))[:, None]


def _cases(rng, n):
    """Rays from sphere surfaces (the shadow bias 1e-13 outward and inward), from random points
    inside, near and far outside, grazing the silhouette, with lights at random distances."""
    c = rng.uniform(-50, 50, (n, 3))
    r = rng.choice([1e-3, 0.5, 1.0, 5.0, 40.0], n) * rng.uniform(0.5, 2.0, n)
    nrm = _unit(rng.normal(size=(n, 3)))
    kind = rng.integers(0, 6, n)
    off = np.select([kind == 0, kind == 1, kind == 2, kind == 3, kind == 4],
                    [1e-13, -1e-13, rng.uniform(-1, 1, n) * r, rng.uniform(1, 30, n) * r, 0.0],
                    rng.uniform(1e-9, 1e-6, n) * r)
    o = c + nrm * (r + off)[:, None]
    d = _unit(rng.normal(size=(n, 3)))
    # a third aimed at grazing the sphere: direction to a point on the silhouette ring (+- 1e-12)
    g = rng.random(n) < 0.35
    tgt = c + _unit(np.cross(nrm, rng.normal(size=(n, 3)))) * (r * (1 + rng.normal(size=n) * 1e-12))[:, None]
    d[g] = _unit(tgt[g] - o[g])
    ld = np.select([rng.random(n) < 0.3, rng.random(n) < 0.5], [np.inf, rng.uniform(0, 3, n) * r],
                   rng.uniform(0, 200, n))
    return c, r, o, d, ld


def test_shadow_and_closest_quick_decisions_agree_with_the_tail():
    rng = np.random.default_rng(20261018)
    decided_s = decided_c = cand_total = 0
    for _ in range(20):
        c, r, o, d, ld = _cases(rng, 200_000)
        r2, opp, adj = geometry(c, r, o, d)
        cand = ~(opp > r2)                                                   # bodies.rs:97-101
        r2, opp, adj, ld = r2[cand], opp[cand], adj[cand], ld[cand]
        cand_total += len(r2)
        hit, t = tail(r2, opp, adj)
        occl = hit & ~(t > ld)
        q = shadow_quick(r2, opp, adj, ld)
        dec = q >= 0
        assert np.array_equal(q[dec] == 1, occl[dec]), "a quick shadow decision differs from the tail"
        b = behind(r2, opp, adj)
        assert not hit[b].any(), "a sphere declared behind is hit by the tail"
        decided_s += int(dec.sum())
        decided_c += int(b.sum())
        # negative control: without the light-distance bound a "sphere in front" is not an occluder
        wrong = np.where(~clear_side(r2, opp, adj), -1, np.where(adj < 0.0, 0, 1))
        assert not np.array_equal(wrong[wrong >= 0] == 1, occl[wrong >= 0])
    # not vacuous: most candidates are decided (rays leaving a surface, spheres behind / in front)
    assert decided_s > 0.5 * cand_total and decided_c > 0.1 * cand_total, (decided_s, decided_c, cand_total)


def test_quick_decisions_on_edge_values():
    """Zero, tiny, huge, infinite and NaN operands: the quick test never decides against the tail."""
    vals = np.array([0.0, -0.0, 5e-324, -5e-324, 2.0 ** -1022, 2.0 ** -900, 2.0 ** -450, 1e-300, 1e-20, 1e-8,
                     0.5, 1.0, 3.0, 1e8, 1e150, 1e154, 1e160, 1e300, np.inf, -np.inf, np.nan])
    vals = np.concatenate([vals, -vals[1:]])
    r2, opp, adj, ld = (a.ravel() for a in np.meshgrid(np.abs(vals), vals, vals, np.abs(vals), indexing="ij"))
    cand = ~(opp > r2)
    r2, opp, adj, ld = r2[cand], opp[cand], adj[cand], ld[cand]
    with np.errstate(all="ignore"):
        hit, t = tail(r2, opp, adj)
        occl = hit & ~(t > ld)
        q = shadow_quick(r2, opp, adj, ld)
        b = behind(r2, opp, adj)
    dec = q >= 0
    assert np.array_equal(q[dec] == 1, occl[dec])
    assert not hit[b].any()


def plane_quick(num, den, ld):
    """plane_shadow_quick (rg_kernels.hip): 1 hit, 0 no hit, -1 divide."""
    with np.errstate(all="ignore"):
        q = ld * den
        ok = (np.abs(num) >= TINY) & (den <= 2.0 ** 100)
        okq = (ld >= TINY) & (q <= 2.0 ** 1000)
        r = np.full(num.shape, -1)
        r = np.where(ok & ~(num < 0.0) & okq & (num >= q * (1.0 + 2.0 ** -50)), 0, r)
        r = np.where(ok & ~(num < 0.0) & okq & (num <= q * (1.0 - 2.0 ** -50)), 1, r)
        r = np.where(ok & (num < 0.0), 0, r)
    return r


def test_plane_shadow_quick_agrees_with_the_division():
    rng = np.random.default_rng(7)
    decided = total = 0
    for _ in range(10):
        n = 500_000
        den = np.exp(rng.uniform(np.log(1.0001e-6), np.log(10.0), n))
        ld = np.exp(rng.uniform(np.log(1e-6), np.log(1e6), n))
        # quotients around the light distance: within a few ulps, within 1e-12, and anywhere
        k = rng.integers(0, 3, n)
        target = ld * np.select([k == 0, k == 1], [1 + rng.integers(-8, 9, n) * 2.0 ** -52,
                                                   1 + rng.normal(size=n) * 1e-12], rng.uniform(-2, 3, n))
        num = target * den
        num = np.where(rng.random(n) < 0.05, -num, num)
        dist = num / den
        hit = (dist >= 0.0) & ~(dist > ld)
        q = plane_quick(num, den, ld)
        dec = q >= 0
        assert np.array_equal(q[dec] == 1, hit[dec])
        decided += int(dec.sum())
        total += n
    assert decided > 0.6 * total
    # edge values never decide against the division
    vals = np.array([0.0, -0.0, 5e-324, 2.0 ** -1022, 2.0 ** -900, 1e-300, 1e-7, 1.0000001e-6, 0.5, 1.0, 3.0, 1e30,
                     2.0 ** 100, 1e200, 1e308, np.inf, np.nan])
    vals = np.concatenate([vals, -vals[1:]])
    num, den, ld = (a.ravel() for a in np.meshgrid(vals, vals[vals > 1e-6], np.abs(vals), indexing="ij"))
    with np.errstate(all="ignore"):
        dist = num / den
        hit = (dist >= 0.0) & ~(dist > ld)
    q = plane_quick(num, den, ld)
    dec = q >= 0
    assert np.array_equal(q[dec] == 1, hit[dec])
