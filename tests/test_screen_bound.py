"""CPU check of the screened scan's distance bound (screen.hip).

The screen computes approx = |a|^2 + |b|^2 - 2 <a', b'> (L2; a = q - c, b = x - c, primes =
bf16 rounding) from fp32 norms and an f32 accumulation of exact bf16 products, and prunes a
pair only when approx - delta exceeds a threshold. Exactness rests on |d_ref - approx| <= delta
for the reference's own fp32 distance d_ref (ivf_flat_index.cpp:352-362: diff = q - x rounded,
diff * diff rounded, acc + term rounded, d = 0..D-1). This test restates the kernel's arithmetic
in numpy float32 (bf16 round-to-nearest-even with subnormals flushed, norms from float64 sums
rounded as the kernel rounds them, the accumulation in two different orders) and checks the
bound on random and adversarial data: iid Gaussian, tight clusters far from the origin, mixed
magnitudes, vectors right at the centroid, and IP.
"""
import numpy as np
import pytest

U = 2.0 ** -24


def bf16(x):
    """Nearest bf16 (ties to even), +0 for |x| < 2^-126, as screen.hip's bf16_bits."""
    x = np.asarray(x, np.float32)
    b = x.view(np.uint32).astype(np.uint64)
    ex = b & 0x7F800000
    r = ((b + 0x7FFF + ((b >> 16) & 1)) >> 16) << 16
    r = np.where(ex == 0, 0, r)
    return r.astype(np.uint32).view(np.float32)


def ru(v):
    """float(v) rounded up, v >= 0 (the kernel's __double2float_ru(sqrt(..) * (1 + 2^-30)))."""
    v = np.asarray(v, np.float64) * (1.0 + 2.0 ** -30)
    f = v.astype(np.float32)
    return np.where(f.astype(np.float64) < v, np.nextafter(f, np.float32(np.inf)), f)


def ref_dist(q, x, metric):
    """The reference's sequential fp32 sum (one row of x per query q)."""
    q = q.astype(np.float32)
    x = x.astype(np.float32)
    if metric == 0:
        t = (q[None, :] - x) ** 2          # each op rounds in float32
    else:
        t = q[None, :] * x
    s = np.cumsum(t, axis=1, dtype=np.float32)[:, -1]
    return s if metric == 0 else -s


def f32_dot(a, b, order):
    """f32 accumulation of exact bf16 products (sequential or pairwise order)."""
    p = (a.astype(np.float64) * b.astype(np.float64)).astype(np.float32)  # exact in f32
    if order == "seq":
        return np.cumsum(p, axis=-1, dtype=np.float32)[..., -1]
    while p.shape[-1] > 1:
        if p.shape[-1] % 2:
            p = np.concatenate([p, np.zeros(p.shape[:-1] + (1,), np.float32)], axis=-1)
        p = (p[..., 0::2] + p[..., 1::2]).astype(np.float32)
    return p[..., 0]


def screen_bound(q, c, X, metric, order):
    dp = q.shape[0]
    cm = np.float32((4 * dp + 16) * float.fromhex("0x1.02p-24"))
    cr = np.float32((dp + 2) * float.fromhex("0x1.02p-24"))
    cu = np.float32(float.fromhex("0x1.02p-23"))
    # per vector (ivf_screen_build): b = x - c in double, b' = bf16(float(b))
    bd = X.astype(np.float64) - c.astype(np.float64)
    bq = bf16(bd.astype(np.float32))
    B2 = (bd * bd).sum(1).astype(np.float32)
    Bn = ru(np.sqrt((bd * bd).sum(1)))
    E = ru(np.sqrt(((bd - bq.astype(np.float64)) ** 2).sum(1)))
    Xn = ru(np.sqrt((X.astype(np.float64) ** 2).sum(1)))
    # per pair (ivf_screen_pairs): L2 a = q - c, IP a = q
    ad = q.astype(np.float64) - (c.astype(np.float64) if metric == 0 else 0.0)
    aq = bf16(ad.astype(np.float32))
    A2 = np.float32((ad * ad).sum())
    An = ru(np.sqrt((ad * ad).sum()))
    F = ru(np.sqrt(((ad - aq.astype(np.float64)) ** 2).sum()))
    qc = np.float32((q.astype(np.float64) * c.astype(np.float64)).sum())
    Cn = ru(np.sqrt((c.astype(np.float64) ** 2).sum()))
    dot = f32_dot(np.broadcast_to(aq, bq.shape), bq, order)
    an, bn = np.float32(An + F), (Bn + E).astype(np.float32)
    cs = (an * E + F * bn + F * E).astype(np.float32)
    if metric == 0:
        approx = ((A2 + B2).astype(np.float32) - np.float32(2) * dot).astype(np.float32)
        rest = (np.float32(2) * (cs + cm * (an * bn)) + cu * (A2 + B2 + np.abs(approx))).astype(np.float32)
        dl = (rest + cr * (np.abs(approx) + rest)).astype(np.float32)
    else:
        qn = np.float32(An)  # (IP: An = |q|)
        approx = (-(qc + dot)).astype(np.float32)
        dl = (cs + cm * (an * bn) + cr * (qn * Xn) + cu * (qn * Cn + an * bn + np.abs(approx))).astype(np.float32)
    dl = (dl * np.float32(1.001) + np.float32(1e-30)).astype(np.float32)
    return approx, dl


CASES = {
    "iid": lambda r, d: (r.standard_normal(d), 0.2 * r.standard_normal(d), r.standard_normal((400, d))),
    "clustered": lambda r, d: (
        (c := 30.0 * np.ones(d) / np.sqrt(d) + r.standard_normal(d)) + 0.05 * r.standard_normal(d),
        c, c + 0.05 * r.standard_normal((400, d))),
    "far_ball_centroid_at_origin": lambda r, d: (
        (c := 100.0 * np.ones(d) / np.sqrt(d)) + 0.01 * r.standard_normal(d), 0.0 * c,
        c + 0.01 * r.standard_normal((400, d))),
    "mixed_scales": lambda r, d: (
        r.standard_normal(d) * np.exp(r.uniform(-20, 20, d)), r.standard_normal(d),
        r.standard_normal((400, d)) * np.exp(r.uniform(-20, 20, (400, d)))),
    "at_centroid": lambda r, d: ((c := r.standard_normal(d)), c, np.repeat(c[None], 400, 0)),
    "tiny": lambda r, d: (1e-20 * r.standard_normal(d), 1e-20 * r.standard_normal(d),
                          1e-20 * r.standard_normal((400, d))),
}


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("case", sorted(CASES))
@pytest.mark.parametrize("dim", [64, 768])
def test_screen_bound_holds(metric, case, dim):
    r = np.random.default_rng(dim + 7 * metric + sum(map(ord, case)))
    for _ in range(3):
        q, c, X = (np.asarray(v, np.float32) for v in CASES[case](r, dim))
        d = ref_dist(q, X, metric)
        for order in ("seq", "pairwise"):
            approx, dl = screen_bound(q, c, X, metric, order)
            lo = (approx - dl).astype(np.float32)
            hi = (approx + dl).astype(np.float32)
            bad = ~((lo <= d) & (d <= hi))
            assert not bad.any(), (case, order, float(d[bad][0]), float(approx[bad][0]), float(dl[bad][0]))


def test_screen_bound_is_tight_on_iid_768():
    """The bound is a small fraction of the distance spread on the headline's data (the
    reason the screen prunes): iid N(0,1), |a|, |b| ~ 28, distances spread by ~68."""
    r = np.random.default_rng(5)
    q, c, X = (np.asarray(v, np.float32) for v in CASES["iid"](r, 768))
    d = ref_dist(q, X, 0)
    approx, dl = screen_bound(q, c, X, 0, "seq")
    assert float(np.max(dl)) < 0.15 * float(np.std(d))
    assert float(np.max(np.abs(approx - d))) < float(np.min(dl))
