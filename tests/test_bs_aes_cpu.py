"""Host checks of the bitsliced AES engine (tools/bs_aes.h, the VALU
half of the hybrid expand kernel): the 82-gate bitop3 S-box on all 256 inputs,
the plane transposes, the MMO hash with run-time and compile-time key masks
against the T-table AES of aes_core.h (pinned by the reference KAT in
test_oracle.py).  bitop3 / v_perm / v_alignbit are emulated on the host."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bs_aes_host(tmp_path):
    exe = tmp_path / "bs_aes_test"
    subprocess.run(["g++", "-O1", "-std=c++17", os.path.join(ROOT, "tests", "cpp", "bs_aes_test.cc"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
