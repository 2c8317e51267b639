"""CPU: the sharded MSM's host epilogue (msm_host.cpp msm_host_assemble_combine,
run by msm_wait on every rank's exchanged payload).  Window shards placed at
their global windows and point shards summed term by term give the one-rank
result (G1 / G2, uneven splits, an empty rank, several segments per term)
-- the host side of the N > 1 path, which the one-GPU pool cannot run on
hardware (tests/host/assemble_check.cpp)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_sharded_epilogue_window_and_point_shards(tmp_path):
    exe = tmp_path / "assemble_check"
    src = os.path.join(HERE, "..", "zelana_amd", "csrc", "msm_host.cpp")
    subprocess.run(["g++", "-O2", "-std=c++17", "-mbmi2", "-madx", "-o", str(exe),
                    os.path.join(HERE, "host", "assemble_check.cpp"), src], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("ok ")
