"""Host unit test of the bitsliced AES core (tools/mb/aes_bitsliced.h, the VALU-only AES evaluated against the
T-table rounds in DESIGN.md §5) against the oracle's AES: compiled with g++ and run on the CPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("gcc") is None, reason="no host compiler")
def test_bitsliced_aes_matches_oracle(tmp_path):
    obj = tmp_path / "gcm_ref.o"
    exe = tmp_path / "test_bitsliced"
    subprocess.run(["gcc", "-O2", "-c", os.path.join(ROOT, "oracle", "gcm_ref.c"), "-o", str(obj)], check=True)
    subprocess.run(["g++", "-O2", "-std=c++17", os.path.join(ROOT, "tests", "c", "test_bitsliced.cpp"), str(obj), "-o",
                    str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok (0 mismatches)" in r.stdout


def test_sbox_circuit_generator_is_current():
    # the committed .inc is what the generator emits from the verified circuit
    gen = os.path.join(ROOT, "tools", "gen", "gen_bs_sbox.py")
    inc = os.path.join(ROOT, "tools", "mb", "aes_bs_sbox.inc")
    before = open(inc).read()
    subprocess.run(["python3", gen], check=True, capture_output=True)
    assert open(inc).read() == before
