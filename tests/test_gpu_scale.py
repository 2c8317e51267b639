"""Full-size parity (BASELINE.json configs[1-4] sizes) through properties that
do not need the CPU oracle to redo the whole job:

* NTT / INTT at 2^24 (configs[2]), plain and coset: round trip is the
  identity; linearity NTT(a + b) = NTT(a) + NTT(b); and exact values at
  sampled output indices for a sparse input, evaluated directly
  (sum_j a_j omega^{jk}, omega = 5^((r-1)/2^28) ^ (2^28 / n), coset:
  a_j -> a_j g^j) — the arkworks Radix2EvaluationDomain definition.
* G1 MSM at 2^24 with the fixed-base table (configs[4]'s per-GPU scale at
  N=4) and at 2^26 (configs[4]'s global size, c = 22 / 12-copy table):
  linearity MSM(a) + MSM(b) = MSM(a + b); and a sparse-scalar MSM equal to
  the oracle's sum over its non-zero terms.
"""
import numpy as np
import pytest

import oracle_ctypes as O

pytestmark = pytest.mark.gpu
R = O.R
RL = np.array([R >> (64 * i) & 0xFFFFFFFFFFFFFFFF for i in range(4)], np.uint64)


@pytest.fixture(scope="module")
def ctx():
    from zelana_amd.gpu import Context
    c = Context(0)
    yield c
    c.close()


def add_mod_r(a, b):
    """(n, 4) u64 canonical + (n, 4) -> mod r, vectorised with explicit carries."""
    out = np.zeros_like(a)
    carry = np.zeros(a.shape[0], np.uint64)
    for i in range(4):
        s = a[:, i] + b[:, i]
        c1 = (s < a[:, i]).astype(np.uint64)
        s2 = s + carry
        c2 = (s2 < s).astype(np.uint64)
        out[:, i] = s2
        carry = c1 | c2
    # subtract r where out >= r (sums < 2r < 2^255: no carry out of limb 3)
    ge = np.ones(a.shape[0], bool)
    decided = np.zeros(a.shape[0], bool)
    for i in (3, 2, 1, 0):
        gt = (out[:, i] > RL[i]) & ~decided
        lt = (out[:, i] < RL[i]) & ~decided
        ge[lt] = False
        decided |= gt | lt
    borrow = np.zeros(a.shape[0], np.uint64)
    sub = out.copy()
    for i in range(4):
        d = sub[:, i] - RL[i]
        b1 = (sub[:, i] < RL[i]).astype(np.uint64)
        d2 = d - borrow
        b2 = (d < borrow).astype(np.uint64)
        sub[:, i] = d2
        borrow = b1 | b2
    out[ge] = sub[ge]
    return out


def to_int(row):
    return sum(int(v) << (64 * i) for i, v in enumerate(row))


def omega(log_n):
    w = pow(5, (R - 1) >> 28, R)
    return pow(w, 1 << (28 - log_n), R)


@pytest.mark.parametrize("coset", [False, True])
def test_ntt_2pow24_roundtrip_and_linearity(ctx, coset):
    from zelana_amd.gpu import DeviceBuffer
    log_n = 24
    n = 1 << log_n
    a = ctx.scalars_generate(seed=240 + coset, n=n)
    b = ctx.scalars_generate(seed=250 + coset, n=n)
    ha, hb = np.zeros((n, 4), np.uint64), np.zeros((n, 4), np.uint64)
    a.download(ha)
    b.download(hb)
    hs = add_mod_r(ha, hb)
    s = DeviceBuffer(ctx, n * 32)
    s.upload(hs)
    for buf in (a, b, s):
        ctx.ntt_device(buf, log_n, False, coset)
    fa, fb, fs = (np.zeros((n, 4), np.uint64) for _ in range(3))
    a.download(fa)
    b.download(fb)
    s.download(fs)
    assert np.array_equal(add_mod_r(fa, fb), fs)
    assert not np.array_equal(fa, ha)
    ctx.ntt_device(a, log_n, True, coset)
    back = np.zeros((n, 4), np.uint64)
    a.download(back)
    assert np.array_equal(back, ha)


@pytest.mark.parametrize("inverse,coset", [(False, False), (True, False), (False, True), (True, True)])
def test_ntt_2pow24_sparse_exact(ctx, inverse, coset):
    log_n = 24
    n = 1 << log_n
    rng = np.random.default_rng(24 + 2 * inverse + coset)
    idx = rng.choice(n, 40, replace=False)
    vals = [int.from_bytes(rng.bytes(32), "little") % R for _ in idx]
    data = np.zeros((n, 4), np.uint64)
    for j, v in zip(idx, vals):
        data[j] = [(v >> (64 * i)) & 0xFFFFFFFFFFFFFFFF for i in range(4)]
    out = ctx.ntt(data, log_n, inverse, coset)
    w = omega(log_n)
    if inverse:
        w = pow(w, R - 2, R)
    ninv = pow(n, R - 2, R)
    g = 5
    for k in rng.choice(n, 12, replace=False):
        acc = sum(v * pow(w, int(j) * int(k), R) for j, v in zip(idx, vals)) % R
        if not inverse:
            if coset:  # coset FFT: evaluations of a(g X)
                acc = sum(v * pow(g, int(j), R) * pow(w, int(j) * int(k), R) for j, v in zip(idx, vals)) % R
        else:
            acc = acc * ninv % R
            if coset:  # coset IFFT: coefficients scaled by g^-k
                acc = acc * pow(pow(g, R - 2, R), int(k), R) % R
        assert to_int(out[k]) == acc, (k, inverse, coset)


@pytest.mark.parametrize("log_n", [24, 26])
def test_msm_table_linearity_and_sparse(ctx, log_n):
    from zelana_amd.gpu import DeviceBuffer, g1_add
    n = 1 << log_n
    bases = ctx.bases_generate(seed=1000 + log_n, n=n)
    info = bases.precompute()
    if log_n == 26:
        assert info[1:] == (22, 12, 1), info  # the config-5 plan
    a = ctx.scalars_generate(seed=31, n=n)
    b = ctx.scalars_generate(seed=32, n=n)
    ha, hb = np.zeros((n, 4), np.uint64), np.zeros((n, 4), np.uint64)
    a.download(ha)
    b.download(hb)
    s = DeviceBuffer(ctx, n * 32)
    s.upload(add_mod_r(ha, hb))
    ma, mb, ms = ctx.msm(bases, a), ctx.msm(bases, b), ctx.msm(bases, s)
    assert np.array_equal(g1_add(ma, mb), ms)
    # sparse scalars: the full-size run against the oracle over its non-zero terms
    rng = np.random.default_rng(7)
    idx = np.sort(rng.choice(n, 300, replace=False))
    sp = np.zeros((n, 4), np.uint64)
    sp[idx] = ha[idx]
    d = DeviceBuffer(ctx, n * 32)
    d.upload(sp)
    got = ctx.msm(bases, d)
    pts = bases.export()[idx]
    assert np.array_equal(got, O.msm_g1(np.ascontiguousarray(pts), np.ascontiguousarray(ha[idx])))
    # and the same sparse MSM with the table's window pinned off (plain Pippenger)
    ctx.set_window(16)
    assert np.array_equal(ctx.msm(bases, d), got)
    ctx.set_window(0)


def test_msm_2pow20_table_plan_matches_oracle(ctx):
    """Config 2 at its own size and plan: 2^20 uniform
    scalars over the c = 20, 13-copy full table (one window of 13 x 2^20
    entries, one lane per bucket), against the oracle's full 2^20 MSM
    (ark-ec msm_bigint_wnaf restated) over the exported bases; also through
    three lanes in flight, as the bench times it."""
    import os
    n = 1 << 20
    bases = ctx.bases_generate(seed=1020, n=n)
    info = bases.precompute()
    assert info[1:] == (20, 13, 1), info  # the bench's headline plan
    d = ctx.scalars_generate(seed=20, n=n)
    hs = np.zeros((n, 4), np.uint64)
    d.download(hs)
    want = O.msm_g1(bases.export(), hs, threads=min(16, os.cpu_count() or 1))
    assert np.array_equal(ctx.msm(bases, d), want)
    ctx.set_lanes(3)
    try:
        jobs = [ctx.msm_submit(bases, d, n) for _ in range(3)]
        for j in jobs:
            assert np.array_equal(ctx.msm_wait(j), want)
    finally:
        ctx.set_lanes(2)


def test_msm_lanes_distinct_inputs_in_flight(ctx):
    """Table MSMs with different scalars in flight on three lanes, whose
    accumulations are chained across lanes (msm.hip msm_acc_phase), each
    equal the same MSM run alone: no lane reads another lane's sort, items or
    buckets.  Two base sets alternate so consecutive lanes also switch
    tables; c = 20 puts them on the one-lane-per-bucket (chained) path."""
    n = 1 << 18
    sets = [ctx.bases_generate(seed=1020 + k, n=n) for k in range(2)]
    for b in sets:
        assert b.precompute(c=20)[1] == 20
    scal = [ctx.scalars_generate(seed=40 + i, n=n) for i in range(6)]
    ctx.set_lanes(1)
    alone = [ctx.msm(sets[i % 2], scal[i]) for i in range(6)]
    ctx.set_lanes(3)
    try:
        jobs = [ctx.msm_submit(sets[i % 2], scal[i], n) for i in range(6)]
        for i, j in enumerate(jobs):
            assert np.array_equal(ctx.msm_wait(j), alone[i]), i
    finally:
        ctx.set_lanes(2)
    assert not np.array_equal(alone[0], alone[1])


def test_msm_2pow26_table_plan_matches_oracle(ctx):
    """Config 5 at its full size: one 2^26 MSM over the
    c = 22, 12-copy table, as one GPU runs it (bench.py extra.msm_global_2_26,
    and every rank's shard plan at N = 1), equals the oracle's full 2^26 MSM
    (ark-ec msm_bigint_wnaf restated, pthreads over windows; ~40 s on 16
    cores) over the exported bases.  Also the 2-lane pipelined form."""
    import os
    import time
    n = 1 << 26
    bases = ctx.bases_generate(seed=1026, n=n)
    info = bases.precompute()
    assert info[1:] == (22, 12, 1), info
    d = ctx.scalars_generate(seed=26, n=n)
    got = ctx.msm(bases, d)
    ctx.set_lanes(2)
    try:
        jobs = [ctx.msm_submit(bases, d, n) for _ in range(2)]
        piped = [ctx.msm_wait(j) for j in jobs]
    finally:
        ctx.set_lanes(2)
    hs = np.zeros((n, 4), np.uint64)
    d.download(hs)
    pts = bases.export()
    del bases
    t0 = time.perf_counter()
    want = O.msm_g1(pts, hs, threads=min(16, os.cpu_count() or 1))
    print(f"oracle 2^26 MSM: {time.perf_counter() - t0:.1f} s", flush=True)
    assert np.array_equal(got, want)
    for p in piped:
        assert np.array_equal(p, want)
