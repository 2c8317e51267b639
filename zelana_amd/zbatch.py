"""zelana_batch front-end: the config-4 circuit as an R1CS + its witness.

Restates forge/circuits/zelana_batch/src/main.nr (the Noir circuit the
reference proves with sunspot/gnark) on top of
zelana_lib (forge/circuits/zelana_lib/src/poseidon.nr, merkle.nr, account.nr,
nullifier.nr).  The reference compiles it with nargo to ACIR and sunspot to a
gnark R1CS; neither exists here, so this module is its own arithmetization of
the same statement, built to feed libzkmi's Groth16 prover:

  * MiMC (poseidon.nr:15-56, host restatement prover-worker/src/mimc.rs:52-122):
    91 rounds of t = x + k + c_i, x <- t^7 (t^2, t^4, t^6, t^7: 4 constraints),
    c_i = (i+1)^3 + (i+1); sponge state <- permute(state + input, 0);
    hash_k(x_1..x_k) = sponge([k, x_1, ..., x_k]).  Permutations of constants
    are folded (no constraints), as the Noir compiler folds them: every
    hash_k costs k permutations.
  * Merkle path (merkle.nr:29-52): per level d = idx * (sibling - cur),
    (left, right) = (cur + d, sibling - d), cur = hash_2(left, right); path
    indices are boolean.
  * `if slot.is_valid { ... }` (main.nr:143-214, 221-270, 276-338): both branches
    are constrained; asserts are predicated on the flag, state updates are
    selects.  The `as u64` casts (main.nr:165-166, 231-232) become 64-bit range
    checks of flag*balance, flag*amount and their difference (exact for values
    below 2^64, which the u64 casts of honest witnesses are); `signature != 0`
    is an inverse witness.
  * Final asserts (main.nr:352-356) are unpredicated equalities with the
    public inputs: pre/post state root, pre/post shielded root, withdrawal
    root, batch hash, batch id (7 instance variables after One).

Note the reference's own inconsistency (recorded, not fixed): the circuit's
nullifier is hash_4(3, sk, cm, pos) (nullifier.nr:26-33) while the host
mimc.rs:140-144 uses hash_3(3, sk, hash_2(cm, pos)); the circuit is followed.

Pinned by: the batch-58 batch-hash KAT (mimc.rs:386-450) and Prover.toml of
batch 70 (5 transfers): recomputed post_state_root, withdrawal_root and
batch_hash equal its public inputs (tests/test_zbatch.py).
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

from .r1cs import R1CS, R

MIMC_ROUNDS = 91
RC = [((i + 1) ** 3 + (i + 1)) % R for i in range(MIMC_ROUNDS)]
TREE_DEPTH = 32
MAX_TRANSFERS, MAX_WITHDRAWALS, MAX_SHIELDED = 8, 4, 4  # main.nr:28-30
PUBLIC = ("pre_state_root", "post_state_root", "pre_shielded_root", "post_shielded_root", "withdrawal_root",
          "batch_hash", "batch_id")


# ----------------------------------------------------------------- host MiMC
def _native_mimc():
    """libzelana_prover.so's MiMC (zelana_amd/host/mimc.cpp), or None when the
    host library is not built (or ZKMI_ZBATCH_PY=1): the Python below is then
    the witness path, with identical values (tests/test_zbatch.py)."""
    global _NATIVE
    if _NATIVE is False:
        _NATIVE = None
        path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libzelana_prover.so")
        if os.path.exists(path) and os.environ.get("ZKMI_ZBATCH_PY") != "1":
            L = ctypes.CDLL(path)
            L.zp_mimc_permute.argtypes = [ctypes.c_void_p] * 3
            L.zp_mimc_trace.argtypes = [ctypes.c_void_p] * 2
            assert L.zp_mimc_rounds() == MIMC_ROUNDS
            _NATIVE = L
    return _NATIVE


_NATIVE = False


def _limbs(x: int) -> np.ndarray:
    return np.frombuffer(x.to_bytes(32, "little"), np.uint64)


def _int(a: np.ndarray) -> int:
    return int.from_bytes(a.tobytes(), "little")


def mimc_permute(x: int, k: int = 0) -> int:
    L = _native_mimc()
    if L is not None:
        xa, ka, y = _limbs(x % R), _limbs(k % R), np.empty(4, np.uint64)
        L.zp_mimc_permute(xa.ctypes.data, ka.ctypes.data, y.ctypes.data)
        return _int(y)
    for c in RC:
        t = (x + k + c) % R
        t2 = t * t % R
        t4 = t2 * t2 % R
        x = t4 * t2 % R * t % R
    return (x + k) % R


def mimc_hash(*xs: int) -> int:
    state = 0
    for v in (len(xs),) + xs:
        state = mimc_permute((state + v) % R)
    return state


def account_leaf(pubkey: int, balance: int, nonce: int) -> int:
    return mimc_hash(1, pubkey, balance, nonce)  # account.nr:85-88


def merkle_root(leaf: int, path, idx) -> int:
    cur = leaf
    for s, b in zip(path, idx):
        cur = mimc_hash(s, cur) if b == 1 else mimc_hash(cur, s)
    return cur


def batch_hash_host(batch_id: int, transfers=(), withdrawals=(), shielded=()) -> int:
    """prover-worker/src/mimc.rs:176-214 (compute_batch_hash)."""
    acc = mimc_hash(4, batch_id)
    for (spk, rpk, amount, nonce) in transfers:
        acc = mimc_hash(acc, mimc_hash(spk, rpk, amount, nonce), amount)
    for (spk, l1, amount) in withdrawals:
        acc = mimc_hash(acc, mimc_hash(l1, amount, spk), amount)
    for (nul, cm) in shielded:
        acc = mimc_hash(acc, nul, cm)
    return mimc_hash(acc, len(transfers), len(withdrawals), len(shielded))


# ------------------------------------------------------------ circuit builder
class LC:
    """Linear combination over variables (0 = One) with its value."""
    __slots__ = ("t", "v")

    def __init__(self, terms, value):
        self.t = terms  # list of (var, coeff)
        self.v = value % R

    def is_const(self):
        return all(var == 0 for var, _ in self.t)

    def __add__(self, o):
        o = o if isinstance(o, LC) else const(o)
        return LC(_merge(self.t, o.t, 1), self.v + o.v)

    def __sub__(self, o):
        o = o if isinstance(o, LC) else const(o)
        return LC(_merge(self.t, o.t, R - 1), self.v - o.v)


def _merge(a, b, s):
    d = {}
    for var, c in a:
        d[var] = (d.get(var, 0) + c) % R
    for var, c in b:
        d[var] = (d.get(var, 0) + s * c) % R
    return [(var, c) for var, c in d.items() if c]


def const(c: int) -> LC:
    c %= R
    return LC([(0, c)] if c else [], c)


class Builder:
    """Allocates variables in order (One, instance, witness) and collects
    constraints: MiMC permutations in bulk (identical 364-row shape), the rest
    as explicit rows."""

    def __init__(self, record: bool = False):
        # values in variable order: lists of ints, and (4*91, 4) u64 arrays
        # for native MiMC traces; `vals` is the open int list
        self.vals = [1]
        self.parts = [self.vals]
        self.nv = 1
        self.num_instance = 1
        self.rows = {"a": [], "b": [], "c": []}
        self.perms = []  # (first variable, input terms)
        # witness program (record=True): the free inputs (variables the batch
        # supplies) and every derived witness as an op over linear
        # combinations, in allocation order (zelana_amd/wprog.py)
        self.record = record
        self.input_vars = [0]  # z[0] = One is input 0
        self.input_vals = [1]
        self.ops = []  # (kind, out, a_terms, b_terms)

    # variables
    def instance(self, value: int) -> LC:
        assert self.nv == self.num_instance, "instance variables come first"
        self.num_instance += 1
        return self.input(value)

    def input(self, value: int) -> LC:
        """A free input of the witness (a Prover.toml value), in order."""
        if self.record:
            self.input_vars.append(self.nv)
            self.input_vals.append(value % R)
        return self.witness(value)

    def witness(self, value: int) -> LC:
        self.vals.append(value % R)
        self.nv += 1
        return LC([(self.nv - 1, 1)], value)

    def set_value(self, var: int, value: int):
        """Overwrite an int-held value (instance variables: public_from_witness)."""
        base = 0
        for part in self.parts:
            if var < base + len(part):
                assert isinstance(part, list), "variable belongs to a MiMC trace"
                part[var - base] = value % R
                return
            base += len(part)
        raise IndexError(var)

    def enforce(self, a: LC, b: LC, c: LC):
        self.rows["a"].append(a.t)
        self.rows["b"].append(b.t)
        self.rows["c"].append(c.t)

    # gadgets
    def mul(self, a: LC, b: LC) -> LC:
        if a.is_const() or b.is_const():  # scaling: no constraint
            k, x = (a, b) if a.is_const() else (b, a)
            return LC([(var, c * k.v % R) for var, c in x.t if c * k.v % R], x.v * k.v)
        w = self.witness(a.v * b.v)
        if self.record:
            self.ops.append(("mul", w.t[0][0], a.t, b.t))
        self.enforce(a, b, w)
        return w

    def boolean(self, x: LC):
        self.enforce(x, x - 1, const(0))

    def assert_eq(self, a: LC, b: LC):
        self.enforce(a - b, const(1), const(0))

    def assert_zero_if(self, pred: LC, x: LC):
        self.enforce(pred, x, const(0))

    def nonzero_if(self, pred: LC, x: LC):
        s = self.mul(pred, x)
        inv = self.witness(pow(s.v, R - 2, R) if s.v else 0)
        if self.record:
            self.ops.append(("inv", inv.t[0][0], s.t, []))
        self.enforce(s, inv, pred)

    def select(self, cond: LC, a: LC, b: LC) -> LC:
        return b + self.mul(cond, a - b)

    def range64(self, x: LC):
        bits = [self.witness((x.v >> i) & 1) for i in range(64)]
        if self.record:
            self.ops.append(("bits64", bits[0].t[0][0], x.t, []))
        for bt in bits:
            self.boolean(bt)
        s = LC([(bt.t[0][0], 1 << i) for i, bt in enumerate(bits)], x.v)
        self.assert_eq(s, x)

    def permute(self, x: LC) -> LC:
        if x.is_const():
            return const(mimc_permute(x.v))
        v0 = self.nv
        if self.record:
            self.ops.append(("perm", v0, x.t, []))
        L = _native_mimc()
        if L is not None:
            tr = np.empty((4 * MIMC_ROUNDS, 4), np.uint64)
            xa = _limbs(x.v)  # held: ctypes.data does not keep the array alive
            L.zp_mimc_trace(xa.ctypes.data, tr.ctypes.data)
            self.vals = []
            self.parts += [tr, self.vals]
            self.nv += 4 * MIMC_ROUNDS
            self.perms.append((v0, x.t))
            return LC([(v0 + 4 * MIMC_ROUNDS - 1, 1)], _int(tr[-1]))
        t = x.v
        vals = self.vals
        self.nv += 4 * MIMC_ROUNDS
        for c in RC:
            t = (t + c) % R
            t2 = t * t % R
            t4 = t2 * t2 % R
            t6 = t4 * t2 % R
            t7 = t6 * t % R
            vals.extend((t2, t4, t6, t7))
            t = t7
        self.perms.append((v0, x.t))
        return LC([(v0 + 4 * MIMC_ROUNDS - 1, 1)], t)

    def hash(self, *xs: LC) -> LC:
        state = const(0)
        for v in (const(len(xs)),) + xs:
            state = self.permute(state + v)
        return state

    def merkle_root(self, leaf: LC, path, idx) -> LC:
        cur = leaf
        for s, b in zip(path, idx):
            d = self.mul(b, s - cur)
            cur = self.hash(cur + d, s - d)
        return cur

    # assembly
    def to_r1cs(self) -> tuple[R1CS, np.ndarray]:
        nv = self.nv
        cs = R1CS(self.num_instance, nv - self.num_instance)
        P = len(self.perms)
        ng = len(self.rows["a"])
        m = P * 4 * MIMC_ROUNDS + ng
        coeffs = {}  # distinct coefficient -> id

        def cid(c):
            i = coeffs.get(c)
            if i is None:
                i = coeffs[c] = len(coeffs)
            return i

        rc_id = np.array([cid(c) for c in RC], np.int64)
        one_id = cid(1)
        for name in ("a", "b", "c"):
            cols, cids, counts = [], [], []
            # permutations: rows r*4 + k of perm p
            if P:
                v0 = np.array([p[0] for p in self.perms], np.int64)
                # round 0 "t" terms: input terms + c_0
                t0 = []
                for _, terms in self.perms:
                    d = dict(terms)
                    d[0] = (d.get(0, 0) + RC[0]) % R
                    t0.append([(var, c) for var, c in d.items() if c])
                pc, pi, pn = _perm_rows(name, v0, t0, rc_id, one_id, cid)
                cols.append(pc)
                cids.append(pi)
                counts.append(pn)
            rows = self.rows[name]
            gn = np.array([len(r) for r in rows], np.int64)
            gc = np.array([var for r in rows for var, _ in r], np.int64)
            gi = np.array([cid(c) for r in rows for _, c in r], np.int64)
            cols.append(gc)
            cids.append(gi)
            counts.append(gn)
            col = np.concatenate(cols).astype(np.uint64)
            ci = np.concatenate(cids)
            cnt = np.concatenate(counts)
            rp = np.zeros(m + 1, np.uint64)
            np.cumsum(cnt, out=rp[1:])
            table = np.array([[(c >> (64 * k)) & 0xFFFFFFFFFFFFFFFF for k in range(4)] for c in coeffs], np.uint64)
            val = table[ci] if len(ci) else np.zeros((1, 4), np.uint64)
            if not len(col):
                col = np.zeros(1, np.uint64)
            cs.set_csr(name, rp, col, val)
        cs._m = m
        return cs, self.assignment()

    def assignment(self) -> np.ndarray:
        """z as (num_variables, 4) canonical u64 limbs."""
        nv = self.nv
        z = np.concatenate([p if isinstance(p, np.ndarray) else
                            np.frombuffer(b"".join(v.to_bytes(32, "little") for v in p), np.uint64).reshape(-1, 4)
                            for p in self.parts if len(p)])
        assert z.shape == (nv, 4)
        return z


def _perm_rows(name, v0, t0, rc_id, one_id, cid):
    """CSR pieces (cols, coeff ids, per-row counts) of all MiMC permutations,
    rows ordered (perm, round, k).  Variables of round r of a permutation at
    v0: t2 = v0+4r, t4 = +1, t6 = +2, t7 = +3; t_r = t7_{r-1} + c_r (round 0:
    the input terms + c_0).  Rows: t^2 = t2, t2*t2 = t4, t4*t2 = t6, t6*t = t7."""
    P, Rn = len(v0), MIMC_ROUNDS
    base = v0[:, None] + 4 * np.arange(Rn)[None, :]  # (P, R) t2 index
    # term lists per (p, r, k): built as fixed-width arrays with a count
    W = 2
    col = np.zeros((P, Rn, 4, W), np.int64)
    cix = np.zeros((P, Rn, 4, W), np.int64)
    cnt = np.zeros((P, Rn, 4), np.int64)
    prev_t7 = base - 1  # t7 of round r-1 (round 0 overwritten below)
    tcol = np.stack([prev_t7, np.zeros_like(prev_t7)], -1)
    tcid = np.stack([np.full_like(prev_t7, one_id), np.broadcast_to(rc_id[None, :], prev_t7.shape)], -1)
    if name == "a":
        col[:, :, 0], cix[:, :, 0], cnt[:, :, 0] = tcol, tcid, 2
        col[:, :, 1, 0], cnt[:, :, 1] = base, 1
        col[:, :, 2, 0], cnt[:, :, 2] = base + 1, 1
        col[:, :, 3, 0], cnt[:, :, 3] = base + 2, 1
    elif name == "b":
        col[:, :, 0], cix[:, :, 0], cnt[:, :, 0] = tcol, tcid, 2
        col[:, :, 1, 0], cnt[:, :, 1] = base, 1
        col[:, :, 2, 0], cnt[:, :, 2] = base, 1
        col[:, :, 3], cix[:, :, 3], cnt[:, :, 3] = tcol, tcid, 2
    else:
        for k in range(4):
            col[:, :, k, 0], cnt[:, :, k] = base + k, 1
    if name in ("a", "b"):
        cix[:, :, 1:, 0] = np.where(cnt[:, :, 1:] > 0, one_id, 0)
    else:
        cix[:, :, :, 0] = one_id
    # flatten rounds 1.. as fixed arrays; round 0 rows with the input terms
    out_c, out_i, out_n = [], [], []
    k_t = (0, 3) if name == "b" else ((0,) if name == "a" else ())
    for p in range(P):
        for k in range(4):
            if k in k_t:
                terms = t0[p]
                out_c.append(np.array([v for v, _ in terms], np.int64))
                out_i.append(np.array([cid(c) for _, c in terms], np.int64))
                out_n.append(len(terms))
            else:
                n = int(cnt[p, 0, k])
                out_c.append(col[p, 0, k, :n])
                out_i.append(cix[p, 0, k, :n])
                out_n.append(n)
        n_rest = cnt[p, 1:].reshape(-1)
        mask = (np.arange(W)[None, :] < n_rest[:, None])
        out_c.append(col[p, 1:].reshape(-1, W)[mask])
        out_i.append(cix[p, 1:].reshape(-1, W)[mask])
        out_n.append(None)
        out_n[-1] = n_rest
    counts = np.concatenate([np.atleast_1d(np.asarray(x, np.int64)) for x in out_n])
    return np.concatenate(out_c), np.concatenate(out_i), counts


# ---------------------------------------------------------------- the circuit
def _f(x) -> int:
    if isinstance(x, bool):
        return int(x)
    return int(x) % R


def build(prover: dict, max_transfers=MAX_TRANSFERS, max_withdrawals=MAX_WITHDRAWALS, max_shielded=MAX_SHIELDED,
          public_from_witness: bool = False, depth: int = TREE_DEPTH, witness_only: bool = False,
          builder: Builder | None = None):
    """R1CS + full assignment z for a Prover.toml-shaped dict (main.nr:112-357).

    public_from_witness: set the 7 public inputs to the values the witness
    computes (for reduced circuits); otherwise they are taken from `prover`
    and the final asserts only hold if the witness reproduces them.
    Returns (cs, z, computed) with computed = the 7 recomputed public values.
    witness_only: skip the matrices (cs is None) — per-batch proving, where the
    circuit's R1CS (and its key) are fixed."""
    b = builder if builder is not None else Builder()
    pub = {k: b.instance(_f(prover.get(k, 0))) for k in PUBLIC}
    batch_id = pub["batch_id"]
    cur_root = pub["pre_state_root"]
    cur_sh = pub["pre_shielded_root"]
    batch_acc = b.hash(const(4), batch_id)
    wd_acc = b.hash(const(5), batch_id)

    def w(x):
        return b.input(_f(x))

    def path_vars(s, pre):
        path = [w(x) for x in list(s[pre + "_path"])[:depth]]
        idx = [w(x) for x in list(s[pre + "_path_indices"])[:depth]]
        for i in idx:
            b.boolean(i)
        return path, idx

    def leaf(pk, bal, nonce):
        return b.hash(const(1), pk, bal, nonce)

    def u64_ge(valid, bal, amt):
        bp, ap = b.mul(valid, bal), b.mul(valid, amt)
        b.range64(bp)
        b.range64(ap)
        b.range64(bp - ap)

    def update_root(valid, old_leaf, new_leaf, path, idx, old_root):
        b.assert_zero_if(valid, b.merkle_root(old_leaf, path, idx) - old_root)  # merkle.nr:87-96
        return b.merkle_root(new_leaf, path, idx)

    empty_t = {"sender_path": [0] * depth, "sender_path_indices": [0] * depth,
               "receiver_path": [0] * depth, "receiver_path_indices": [0] * depth}
    transfers = list(prover.get("transfers", []))[:max_transfers]
    for i in range(max_transfers):  # main.nr:143-214
        t = transfers[i] if i < len(transfers) else empty_t
        valid = w(t.get("is_valid", False))
        b.boolean(valid)
        spk, sbal, snonce = w(t.get("sender_pubkey", 0)), w(t.get("sender_balance", 0)), w(t.get("sender_nonce", 0))
        spath, sidx = path_vars(t, "sender")
        rpk, rbal, rnonce = (w(t.get("receiver_pubkey", 0)), w(t.get("receiver_balance", 0)),
                             w(t.get("receiver_nonce", 0)))
        rpath, ridx = path_vars(t, "receiver")
        amount, sig = w(t.get("amount", 0)), w(t.get("signature", 0))
        s_leaf = leaf(spk, sbal, snonce)
        b.assert_zero_if(valid, b.merkle_root(s_leaf, spath, sidx) - cur_root)
        u64_ge(valid, sbal, amount)
        tx_hash = b.hash(spk, rpk, amount, snonce)
        b.nonzero_if(valid, sig)
        new_s_leaf = leaf(spk, sbal - amount, snonce + 1)
        root1 = b.select(valid, update_root(valid, s_leaf, new_s_leaf, spath, sidx, cur_root), cur_root)
        r_leaf = leaf(rpk, rbal, rnonce)
        new_r_leaf = leaf(rpk, rbal + amount, rnonce)
        cur_root = b.select(valid, update_root(valid, r_leaf, new_r_leaf, rpath, ridx, root1), root1)
        batch_acc = b.select(valid, b.hash(batch_acc, tx_hash, amount), batch_acc)

    empty_w = {"sender_path": [0] * depth, "sender_path_indices": [0] * depth}
    withdrawals = list(prover.get("withdrawals", []))[:max_withdrawals]
    for i in range(max_withdrawals):  # main.nr:221-270
        t = withdrawals[i] if i < len(withdrawals) else empty_w
        valid = w(t.get("is_valid", False))
        b.boolean(valid)
        spk, sbal, snonce = w(t.get("sender_pubkey", 0)), w(t.get("sender_balance", 0)), w(t.get("sender_nonce", 0))
        spath, sidx = path_vars(t, "sender")
        l1, amount, sig = w(t.get("l1_recipient", 0)), w(t.get("amount", 0)), w(t.get("signature", 0))
        s_leaf = leaf(spk, sbal, snonce)
        b.assert_zero_if(valid, b.merkle_root(s_leaf, spath, sidx) - cur_root)
        u64_ge(valid, sbal, amount)
        b.nonzero_if(valid, sig)
        new_s_leaf = leaf(spk, sbal - amount, snonce + 1)
        cur_root = b.select(valid, update_root(valid, s_leaf, new_s_leaf, spath, sidx, cur_root), cur_root)
        wd_hash = b.hash(l1, amount, spk)
        wd_acc = b.select(valid, b.hash(wd_acc, wd_hash), wd_acc)
        batch_acc = b.select(valid, b.hash(batch_acc, wd_hash, amount), batch_acc)

    empty_s = {"input_path": [0] * depth, "input_path_indices": [0] * depth}
    shielded = list(prover.get("shielded", []))[:max_shielded]
    for i in range(max_shielded):  # main.nr:276-338
        t = shielded[i] if i < len(shielded) else empty_s
        valid = w(t.get("is_valid", False))
        skip = w(t.get("skip_verification", False))
        b.boolean(valid)
        b.boolean(skip)
        vs = b.mul(valid, skip)  # valid and skip
        vf = valid - vs          # valid and not skip
        owner, value, blind = w(t.get("input_owner", 0)), w(t.get("input_value", 0)), w(t.get("input_blinding", 0))
        pos = w(t.get("input_position", 0))
        ipath, iidx = path_vars(t, "input")
        sk = w(t.get("spending_key", 0))
        oowner, ovalue, oblind = (w(t.get("output_owner", 0)), w(t.get("output_value", 0)),
                                  w(t.get("output_blinding", 0)))
        ocm_given, nul = w(t.get("output_commitment", 0)), w(t.get("nullifier", 0))
        # pass-through branch (main.nr:280-290)
        root_a = b.hash(cur_sh, ocm_given)
        acc_a = b.hash(batch_acc, nul, ocm_given)
        # full verification branch (main.nr:291-336)
        in_cm = b.hash(owner, value, blind)
        b.assert_zero_if(vf, b.merkle_root(in_cm, ipath, iidx) - cur_sh)
        b.assert_zero_if(vf, b.hash(const(3), sk, in_cm, pos) - nul)  # nullifier.nr:26-33
        b.assert_zero_if(vf, value - ovalue)
        out_cm = b.hash(oowner, ovalue, oblind)
        root_b = b.hash(cur_sh, out_cm)
        acc_b = b.hash(batch_acc, nul, out_cm)
        cur_sh = b.select(vs, root_a, b.select(vf, root_b, cur_sh))
        batch_acc = b.select(vs, acc_a, b.select(vf, acc_b, batch_acc))

    nt, nw, ns = w(prover.get("num_transfers", 0)), w(prover.get("num_withdrawals", 0)), w(prover.get("num_shielded", 0))
    final_batch = b.hash(batch_acc, nt, nw, ns)  # main.nr:343-348
    final_wd = b.hash(wd_acc, nw)
    computed = {"pre_state_root": pub["pre_state_root"].v, "post_state_root": cur_root.v,
                "pre_shielded_root": pub["pre_shielded_root"].v, "post_shielded_root": cur_sh.v,
                "withdrawal_root": final_wd.v, "batch_hash": final_batch.v, "batch_id": batch_id.v}
    if public_from_witness:
        for k, lc in pub.items():
            b.set_value(lc.t[0][0], computed[k])
            lc.v = computed[k]
    b.assert_eq(cur_root, pub["post_state_root"])  # main.nr:353-356
    b.assert_eq(cur_sh, pub["post_shielded_root"])
    b.assert_eq(final_wd, pub["withdrawal_root"])
    b.assert_eq(final_batch, pub["batch_hash"])
    if witness_only:
        return None, b.assignment(), computed
    cs, z = b.to_r1cs()
    return cs, z, computed


def batch_inputs(prover: dict, max_transfers=MAX_TRANSFERS, max_withdrawals=MAX_WITHDRAWALS,
                 max_shielded=MAX_SHIELDED, depth: int = TREE_DEPTH) -> np.ndarray:
    """The free inputs of build()'s witness in allocation order (One, the 7
    public inputs, then every w(...) of main.nr's slots): what a batch hands
    the GPU witness program (zelana_amd/wprog.py) instead of the 1.4M-entry z.
    Must follow build()'s order exactly (tests/test_zbatch.py checks it
    against the recording Builder).  Returns (n_inputs, 4) canonical u64."""
    vals = [1] + [_f(prover.get(k, 0)) for k in PUBLIC]

    def path(s, pre):
        vals.extend(_f(x) for x in list(s.get(pre + "_path", [0] * depth))[:depth])
        vals.extend(_f(x) for x in list(s.get(pre + "_path_indices", [0] * depth))[:depth])

    transfers = list(prover.get("transfers", []))[:max_transfers]
    for i in range(max_transfers):
        t = transfers[i] if i < len(transfers) else {}
        vals += [_f(t.get("is_valid", False)), _f(t.get("sender_pubkey", 0)), _f(t.get("sender_balance", 0)),
                 _f(t.get("sender_nonce", 0))]
        path(t, "sender")
        vals += [_f(t.get("receiver_pubkey", 0)), _f(t.get("receiver_balance", 0)), _f(t.get("receiver_nonce", 0))]
        path(t, "receiver")
        vals += [_f(t.get("amount", 0)), _f(t.get("signature", 0))]
    withdrawals = list(prover.get("withdrawals", []))[:max_withdrawals]
    for i in range(max_withdrawals):
        t = withdrawals[i] if i < len(withdrawals) else {}
        vals += [_f(t.get("is_valid", False)), _f(t.get("sender_pubkey", 0)), _f(t.get("sender_balance", 0)),
                 _f(t.get("sender_nonce", 0))]
        path(t, "sender")
        vals += [_f(t.get("l1_recipient", 0)), _f(t.get("amount", 0)), _f(t.get("signature", 0))]
    shielded = list(prover.get("shielded", []))[:max_shielded]
    for i in range(max_shielded):
        t = shielded[i] if i < len(shielded) else {}
        vals += [_f(t.get(k, False if k in ("is_valid", "skip_verification") else 0))
                 for k in ("is_valid", "skip_verification", "input_owner", "input_value", "input_blinding",
                           "input_position")]
        path(t, "input")
        vals += [_f(t.get(k, 0)) for k in ("spending_key", "output_owner", "output_value", "output_blinding",
                                           "output_commitment", "nullifier")]
    vals += [_f(prover.get(k, 0)) for k in ("num_transfers", "num_withdrawals", "num_shielded")]
    raw = b"".join(v.to_bytes(32, "little") for v in vals)
    return np.frombuffer(raw, np.uint64).reshape(-1, 4).copy()


def load_prover_toml(path: str) -> dict:
    import tomli
    with open(path, "rb") as f:
        return tomli.load(f)


# ------------------------------------------------------- synthetic batches
class SparseTree:
    """Sparse MiMC Merkle tree (merkle.nr layout: level-0 siblings first;
    empty subtrees hash up from 0 leaves)."""

    def __init__(self, depth: int):
        self.depth = depth
        self.leaves: dict[int, int] = {}
        self.zero = [0]
        for _ in range(depth):
            self.zero.append(mimc_hash(self.zero[-1], self.zero[-1]))
        self._nodes: dict[tuple[int, int], int] = {}

    def _node(self, level: int, index: int) -> int:
        if level == 0:
            return self.leaves.get(index, 0)
        key = (level, index)
        v = self._nodes.get(key)
        if v is None:
            v = mimc_hash(self._node(level - 1, 2 * index), self._node(level - 1, 2 * index + 1))
            self._nodes[key] = v
        return v

    def root(self) -> int:
        return self._node(self.depth, 0)

    def set(self, index: int, leaf: int):
        self.leaves[index] = leaf
        for lv in range(1, self.depth + 1):
            self._nodes.pop((lv, index >> lv), None)

    def path(self, index: int):
        sib, idx = [], []
        for lv in range(self.depth):
            i = index >> lv
            sib.append(self._node(lv, i ^ 1))
            idx.append(i & 1)
        return sib, idx


def synthetic_batch(depth: int, n_transfers: int, seed: int = 0, n_accounts: int = 6,
                    max_transfers: int = MAX_TRANSFERS) -> dict:
    """A Prover.toml-shaped batch over a depth-`depth` tree: n_transfers valid
    transfers between random accounts, sender then receiver paths taken
    against the running root (as main.nr consumes them)."""
    import random
    rnd = random.Random(seed)
    n_accounts = max(2, min(n_accounts, 1 << depth))
    tree = SparseTree(depth)
    accts = {}
    for a in range(n_accounts):
        pk = rnd.randrange(1, R)
        bal, nonce = rnd.randrange(10 ** 9, 10 ** 10), rnd.randrange(0, 100)
        slot = rnd.randrange(0, 1 << depth)
        while slot in tree.leaves:
            slot = rnd.randrange(0, 1 << depth)
        accts[a] = [pk, bal, nonce, slot]
        tree.set(slot, account_leaf(pk, bal, nonce))
    pre = tree.root()
    transfers, tx_data = [], []
    for _ in range(n_transfers):
        s, r = rnd.sample(range(n_accounts), 2)
        spk, sbal, snonce, sslot = accts[s]
        amount = rnd.randrange(1, sbal // 4)
        spath, sidx = tree.path(sslot)
        tree.set(sslot, account_leaf(spk, sbal - amount, snonce + 1))
        accts[s][1:3] = [sbal - amount, snonce + 1]
        rpk, rbal, rnonce, rslot = accts[r]
        rpath, ridx = tree.path(rslot)
        tree.set(rslot, account_leaf(rpk, rbal + amount, rnonce))
        accts[r][1] = rbal + amount
        transfers.append({"sender_pubkey": spk, "sender_balance": sbal, "sender_nonce": snonce,
                          "sender_path": spath, "sender_path_indices": sidx,
                          "receiver_pubkey": rpk, "receiver_balance": rbal, "receiver_nonce": rnonce,
                          "receiver_path": rpath, "receiver_path_indices": ridx,
                          "amount": amount, "signature": rnd.randrange(1, R), "is_valid": True})
        tx_data.append((spk, rpk, amount, snonce))
    batch_id = rnd.randrange(1, 1000)
    empty_root = mimc_hash(0, 0)
    return {"pre_state_root": pre, "post_state_root": tree.root(), "pre_shielded_root": empty_root,
            "post_shielded_root": empty_root,
            "withdrawal_root": mimc_hash(mimc_hash(5, batch_id), 0),
            "batch_hash": batch_hash_host(batch_id, transfers=tx_data), "batch_id": batch_id,
            "num_transfers": n_transfers, "num_withdrawals": 0, "num_shielded": 0,
            "transfers": transfers[:max_transfers]}
