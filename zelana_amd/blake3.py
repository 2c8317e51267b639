"""BLAKE3 (hash mode, 32-byte output) for Groth16Prover::compute_vk_hash
(core/src/sequencer/settlement/prover.rs:289-294: blake3(compressed vk)) and
compute_batch_hash (:525-558).  The blake3 crate is a third-party dependency
absent here; this restates the published algorithm.  Inputs are small (a VK is
a few hundred bytes), so a plain-Python implementation suffices."""
from __future__ import annotations

import struct

IV = [0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A, 0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19]
PERM = [2, 6, 3, 10, 7, 0, 4, 13, 1, 11, 12, 5, 9, 14, 15, 8]
CHUNK_START, CHUNK_END, PARENT, ROOT = 1, 2, 4, 8
M32 = 0xFFFFFFFF


def _g(s, a, b, c, d, x, y):
    s[a] = (s[a] + s[b] + x) & M32
    s[d] = ((s[d] ^ s[a]) >> 16 | (s[d] ^ s[a]) << 16) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 12 | (s[b] ^ s[c]) << 20) & M32
    s[a] = (s[a] + s[b] + y) & M32
    s[d] = ((s[d] ^ s[a]) >> 8 | (s[d] ^ s[a]) << 24) & M32
    s[c] = (s[c] + s[d]) & M32
    s[b] = ((s[b] ^ s[c]) >> 7 | (s[b] ^ s[c]) << 25) & M32


def _compress(cv, block_words, counter, block_len, flags):
    s = list(cv) + IV[:4] + [counter & M32, (counter >> 32) & M32, block_len, flags]
    m = list(block_words)
    for r in range(7):
        _g(s, 0, 4, 8, 12, m[0], m[1]); _g(s, 1, 5, 9, 13, m[2], m[3])
        _g(s, 2, 6, 10, 14, m[4], m[5]); _g(s, 3, 7, 11, 15, m[6], m[7])
        _g(s, 0, 5, 10, 15, m[8], m[9]); _g(s, 1, 6, 11, 12, m[10], m[11])
        _g(s, 2, 7, 8, 13, m[12], m[13]); _g(s, 3, 4, 9, 14, m[14], m[15])
        if r < 6:
            m = [m[p] for p in PERM]
    return [s[i] ^ s[i + 8] for i in range(8)] + [s[i + 8] ^ cv[i] for i in range(8)]


def _words(block: bytes):
    return list(struct.unpack("<16I", block.ljust(64, b"\0")))


def _chunk_cv(chunk: bytes, counter: int, is_root: bool):
    cv = IV
    blocks = [chunk[i:i + 64] for i in range(0, max(len(chunk), 1), 64)] or [b""]
    for i, b in enumerate(blocks):
        flags = (CHUNK_START if i == 0 else 0) | (CHUNK_END if i == len(blocks) - 1 else 0)
        if is_root and i == len(blocks) - 1:
            flags |= ROOT
        cv = _compress(cv, _words(b), counter, len(b), flags)[:8]
    return cv


def blake3(data: bytes) -> bytes:
    chunks = [data[i:i + 1024] for i in range(0, len(data), 1024)] or [b""]
    if len(chunks) == 1:
        return struct.pack("<8I", *_chunk_cv(chunks[0], 0, True))
    cvs = [_chunk_cv(c, i, False) for i, c in enumerate(chunks)]
    # merge like the reference tree: left subtree = largest power of two < n chunks
    def merge(lo, hi, root):
        n = hi - lo
        if n == 1:
            return cvs[lo]
        left = 1 << ((n - 1).bit_length() - 1)
        lcv, rcv = merge(lo, lo + left, False), merge(lo + left, hi, False)
        return _compress(IV, lcv + rcv, 0, 64, PARENT | (ROOT if root else 0))[:8]
    return struct.pack("<8I", *merge(0, len(cvs), True))
