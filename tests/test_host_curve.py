"""Host build of the device field / curve code (ff.h, ec.h compile for the CPU
too): the lazy-reduction G1 mixed addition used by the MSM accumulation loop
must produce the same group elements as the plain formula (chains with
repeated bases, cancellations, negated bases, doubling and infinity)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_madd_g1_lazy_matches_plain(tmp_path):
    exe = tmp_path / "madd_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-o", str(exe), os.path.join(HERE, "host", "madd_check.cpp")],
                   check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("ok ")
