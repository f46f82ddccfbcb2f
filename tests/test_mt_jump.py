"""CPU check of the MT19937 jump-ahead mathematics the SecAgg mask expansion uses on the device
(fedml_amd/csrc/mt_poly.h): Berlekamp-Massey finds a degree-19937 characteristic polynomial phi that
annihilates numpy's word sequence, the correlation of the sequence with x^J mod phi reproduces the
sequentially generated window J words ahead (many J and seeds), and both carry-less products agree.
Built with g++ from tools/mt_jump_check.cpp (host C++ only)."""
from __future__ import annotations

import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_mt_jump_polynomials(tmp_path):
    exe = str(tmp_path / "mt_jump_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "fedml_amd", "csrc"),
                    os.path.join(ROOT, "tools", "mt_jump_check.cpp"), "-o", exe, "-pthread"], check=True)
    out = subprocess.run([exe, "4"], check=True, capture_output=True, text=True, timeout=120).stdout
    res = json.loads(out.strip().splitlines()[-1])
    assert res["ok"] and res["phi_weight"] == 135  # MT19937's characteristic polynomial has 135 terms
