"""The forge prover-worker output contract (zelana_amd/batch_worker.py) on CPU:
the public witness of batch 70 (tests/golden/zelana_batch_70_Prover.toml,
a copy of forge/circuits/zelana_batch/Prover.toml) in the layout the worker's
`parse_public_witness` reads (forge/crates/prover-worker/src/prover.rs:575-596),
read back by an independent restatement of that function."""
import os
import struct

import pytest

from zelana_amd import batch_worker as BW
from zelana_amd import zbatch as Z

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _reference_parse(bytes_):
    """prover.rs:575-596, line for line: < 12 bytes -> empty; count from the
    first 4 bytes (big-endian); inputs start at byte 12, 32 bytes each, hex
    with a 0x prefix; a short tail is skipped."""
    if len(bytes_) < 12:
        return []
    count = int.from_bytes(bytes_[0:4], "big")
    data_start = 12
    inputs = []
    for i in range(count):
        offset = data_start + i * 32
        if offset + 32 <= len(bytes_):
            inputs.append("0x" + bytes_[offset:offset + 32].hex())
    return inputs


def _batch70():
    return Z.load_prover_toml(os.path.join(GOLD, "zelana_batch_70_Prover.toml"))


def test_batch70_public_witness_layout():
    d = _batch70()
    pw = BW.public_witness_bytes(BW.public_values(d))
    assert len(pw) == 236  # 4-B count + 8 B + 7 x 32 B
    assert struct.unpack(">III", pw[:12]) == (7, 0, 7)
    parsed = _reference_parse(pw)
    assert parsed == BW.parse_public_witness(pw)
    assert len(parsed) == 7
    # the worker's public_inputs are the circuit's pub parameters in main.nr:114-120 order
    for name, hx in zip(Z.PUBLIC, parsed):
        assert int(hx, 16) == int(d[name]) % Z.R, name
        assert len(hx) == 66
    assert int(parsed[-1], 16) == 70


def test_public_witness_edges():
    assert _reference_parse(b"") == [] == BW.parse_public_witness(b"")
    assert BW.parse_public_witness(bytes(11)) == []
    pw = BW.public_witness_bytes([1, Z.R - 1])
    assert BW.parse_public_witness(pw) == _reference_parse(pw) == ["0x" + "00" * 31 + "01", "0x" + (Z.R - 1).to_bytes(32, "big").hex()]
    # a truncated tail is skipped, as the reference does
    assert BW.parse_public_witness(pw[:-1]) == _reference_parse(pw[:-1]) == ["0x" + "00" * 31 + "01"]
    with pytest.raises(ValueError):
        BW.public_witness_bytes([Z.R])
