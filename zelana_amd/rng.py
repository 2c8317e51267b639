"""rand 0.8 StdRng (= rand_chacha 0.3.1 ChaCha12Rng) seeded via rand_core
0.6.4 SeedableRng::seed_from_u64, and ark-ff 0.5 Fp::rand — the host-side
plumbing that Groth16Prover::prove uses to draw r, s
(core/src/sequencer/settlement/prover.rs:354: StdRng::seed_from_u64(batch_id);
ark-groth16 create_random_proof: r = Fr::rand, then s = Fr::rand).

Only a few blocks are ever drawn per proof, so plain Python is enough.
"""
from __future__ import annotations

R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_MASK32 = 0xFFFFFFFF
_R_MONT_INV = pow(1 << 256, -1, R)


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & _MASK32


def _qr(s, a, b, c, d):
    s[a] = (s[a] + s[b]) & _MASK32; s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & _MASK32; s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & _MASK32; s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & _MASK32; s[b] = _rotl(s[b] ^ s[c], 7)


class StdRng:
    def __init__(self, key_words: list[int]):
        self.key = key_words
        self.counter = 0
        self.buf: list[int] = []

    @classmethod
    def seed_from_u64(cls, state: int) -> "StdRng":
        mul, inc = 6364136223846793005, 11634580027462260723
        words = []
        for _ in range(8):
            state = (state * mul + inc) & 0xFFFFFFFFFFFFFFFF
            xs = (((state >> 18) ^ state) >> 27) & _MASK32
            rot = state >> 59
            words.append(((xs >> rot) | (xs << ((32 - rot) & 31))) & _MASK32)
        return cls(words)

    def _block(self):
        inp = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574] + self.key + [
            self.counter & _MASK32, self.counter >> 32, 0, 0]
        x = list(inp)
        for _ in range(6):  # 12 rounds
            _qr(x, 0, 4, 8, 12); _qr(x, 1, 5, 9, 13); _qr(x, 2, 6, 10, 14); _qr(x, 3, 7, 11, 15)
            _qr(x, 0, 5, 10, 15); _qr(x, 1, 6, 11, 12); _qr(x, 2, 7, 8, 13); _qr(x, 3, 4, 9, 14)
        self.counter += 1
        self.buf = [(a + b) & _MASK32 for a, b in zip(x, inp)]

    def next_u32(self) -> int:
        if not self.buf:
            self._block()
        return self.buf.pop(0)

    def next_u64(self) -> int:
        lo = self.next_u32()
        return lo | (self.next_u32() << 32)

    def fr_rand(self) -> int:
        """ark-ff Fp::rand: 4 limbs, top masked to 254 bits, reject >= r; the
        limbs are the Montgomery form, so the value is limbs * 2^-256 mod r."""
        while True:
            limbs = [self.next_u64() for _ in range(4)]
            limbs[3] &= (1 << 62) - 1
            v = sum(l << (64 * i) for i, l in enumerate(limbs))
            if v < R:
                return v * _R_MONT_INV % R
